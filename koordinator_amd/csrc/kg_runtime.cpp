// kg_runtime.cpp — host runtime behind the C ABI of include/koordgpu.h.
//
// Owns the device-resident node snapshot (one record per node, see kg_layout.h), the pod batches
// and their result buffers, the launch sequencing on one HIP stream per context, the event-based
// timing of the dominant kernel, and the RCCL communicator of the node-sharded multi-GPU mode.
// Host-side derivations done once per node row at upload (never per evaluation):
//   * LoadAware usage-threshold cut-offs: the largest estimated usage e with
//     int64(math.Round(float64(e)/float64(total)*100)) <= threshold (load_aware.go:326), found by
//     bisection on the exact float64 expression (it is monotone in e);
//   * per-profile LoadAware filter modes (thresholds empty / NodeMetric missing / expired / nil,
//     load_aware.go:175-210) and the Score's zero cases (:265-279);
//   * reciprocals of the static divisors (allocatable, zone totals) for the corrected quotient;
//   * extension.Amplify of the node's cpuset-allocated milli-cpu (node_resource_amplification.go:170).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>
#include <tuple>
#include <string>
#include <vector>

#include "../../include/koordgpu.h"
#include "kg_kernels.h"
#include "kg_layout.h"

using namespace kg;

struct kg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    std::mutex mu;  // serialises calls on one context (Unreserve may arrive from binding goroutines)
    bool profiling = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_live;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_free;
    double prof_ms = 0.0;
    uint64_t prof_launches = 0;
    ncclComm_t comm = nullptr;
    int rank = 0, world = 1;
    // config-5 select: the plain pods' k_select1 runs on `side` while `stream` builds DevSum and pass 1
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    // a second side lane: config 5's class-1 kernels beside the general ones (forked and joined inside a launcher)
    hipStream_t side2 = nullptr;
    hipEvent_t fork2 = nullptr, join2 = nullptr;
};

struct kg_snap {
    kg_ctx* ctx = nullptr;
    kg_config cfg{};
    KCfg kcfg{};
    uint32_t n = 0, base = 0;
    NodeRec* d_nodes = nullptr;
    ZoneRec* d_zones = nullptr;
    uint32_t* d_big = nullptr;  // [0] = count, [1..] = list of F_BIG records (k_big_scan)
    int8_t* d_zsel = nullptr;   // replay: NUMA zone each record chose for the current pod
    uint32_t* d_pos = nullptr;  // snapshot index -> record position (block replay)
    // Records are stored grouped by storage class (node_class: 0 = no per-zone scoring, 1 = NUMA
    // SingleNUMANode), each group in ascending snapshot index; the high half of v[N_FLAGS] holds the snapshot index.
    std::vector<NodeRec> h_nodes;  // device order
    std::vector<ZoneRec> h_zones;
    std::vector<uint32_t> pos;     // snapshot index -> record position
    uint32_t n0 = 0;               // records of class 0 (positions [0, n0))
    uint32_t n_topo = 0;           // Restricted / BestEffort records (need the general NUMA topology manager)
    uint32_t n_big_est = 0;        // F_BIG records at the last upload / row update (grid sizing of k_big_sel)
    bool uploaded = false;
    bool weights_small = false;  // per-resource weights <= 2^12: float64 fast path allowed
    // config-5 tables (KG_PLUGIN_DEV / RSV / QUOTA)
    DevRec* d_dev = nullptr;       // [record]
    std::vector<DevRec> h_dev;     // device order
    QuotaLim* d_qlim = nullptr;
    QuotaState* d_qstate = nullptr;  // [2][n_quotas]
    uint32_t n_quotas = 0;
    RsvView* d_views = nullptr;
    uint32_t* d_vfirst = nullptr;  // ExtDev::vfirst / vmap
    uint32_t* d_vmap = nullptr;
    RsvInfo* d_infos = nullptr;
    uint32_t* d_cls_begin = nullptr;  // [RSV_MAX_CLASSES + 1]
    DevRec* d_rdev = nullptr;         // kg_rsv_dev tables
    uint32_t* d_rdev_rec = nullptr;   // record (position) of the node each kg_rsv_dev table belongs to
    uint32_t n_rdev = 0;
    uint32_t* d_special = nullptr;    // [0] = count, [1..]: records the fast-base ext kernels leave to PART 2
    uint32_t n_view_nodes = 0;        // nodes holding a reservation view
    // PART 2 grid: the class-1 records and the largest reservation class's views (F_BIG records come on top)
    uint32_t special_est() const { return std::max(n - n0, max_cls_views); }
    uint32_t n_views = 0;
    uint32_t max_cls_views = 0;  // views of the largest reservation class
    std::vector<kg_rsv_view> h_views;  // as uploaded (local snapshot indices; kg_snapshot_update_views / record moves)
    std::vector<kg_rsv_info> h_infos;
    std::vector<uint64_t> cls_mask;  // per snapshot index: classes with a view on the node
    // A Reserve / Unreserve / row update on a node that holds views changes what its views restore
    // (absolute restored Requested etc.): the caller recomputes the restore (the reference reruns the
    // Reservation transformer every cycle) and re-uploads; until then selects on the snapshot refuse.
    bool views_stale = false;
    // the uploaded reservation views in ABI form (by node index: they survive record moves), for per-node updates;
    // stale[i]: node i holds views and changed since they were computed
    std::vector<kg_rsv_dev> h_rdevs;
    std::vector<uint8_t> stale;
    uint32_t n_stale = 0;
    // Reservation.Reserve on the device (kg_replay / kg_assume_ext) updates the views in place while no reservation
    // holds GPUs (rsv_gpu false); views_on_device: the host copies trail the device ones (read back before use)
    bool rsv_gpu = false, views_on_device = false;
    // DeviceShare restore inputs of the GPU-holding reservations (kg_snapshot_upload_rsv_gpu): with them the Reserves
    // follow those reservations on the device (gpu_restore_apply); an upload / update of the views drops them
    int32_t* d_graw = nullptr;       // [record] GpuRawNode index, -1 = none
    GpuRawNode* d_gnodes = nullptr;
    GpuRawRsv* d_grsv = nullptr;
    uint32_t n_gnodes = 0, n_grsv = 0;
    bool gpu_raw = false;
    // a Reserve can follow every reservation of the snapshot on the device (none holds GPUs, or their inputs are here)
    bool rsv_follow() const { return !rsv_gpu || gpu_raw; }
    std::vector<uint32_t> view_order;  // device view t -> h_views index
    int32_t* d_nsel = nullptr;         // replay: nominated reservation of each record's pair (2 x n, like d_zsel)
    RsvStep* d_rstep = nullptr;        // replay with views: [3] per-step Reservation normalisation and winner
    uint64_t* d_rlist = nullptr;       // replay with views: [3][n] pairs with a Reservation score term (2 x u64)
    // Generation: bumped by every call that changes what the snapshot holds (upload, row update, Assume /
    // Forget, replay, quota / reservation upload); kg_snapshot_generation reads it.
    uint64_t gen = 0;
    // batched row updates: staged records (NodeRec, ZoneRec[, DevRec] per row) and their positions
    uint8_t* d_stage = nullptr;
    uint32_t* d_stage_pos = nullptr;
    size_t stage_cap = 0;  // rows
    std::vector<uint8_t> h_stage;
    // Saved Reserve state: `ck` for kg_snapshot_checkpoint / rollback (planners), `bk` for the cleanup of a
    // failed kg_batch_schedule. Invalidated by anything that may move records or replace tables.
    struct Saved {
        NodeRec* nodes = nullptr;
        ZoneRec* zones = nullptr;
        DevRec* dev = nullptr;
        kg_cpu_alloc* cpu = nullptr;
        QuotaState* q = nullptr;
        uint32_t nq = 0;
        RsvView* views = nullptr;  // the views and reservations Reservation.Reserve changes on the device
        RsvInfo* infos = nullptr;
        uint32_t nv = 0, ni = 0;
        DevRec* rdev = nullptr;  // GPU restore tables and their raw inputs (GPU-holding reservations)
        GpuRawNode* gnodes = nullptr;
        GpuRawRsv* grsv = nullptr;
        uint32_t nrd = 0, ngn = 0, ngr = 0;
        bool views_on_device = false;
        bool valid = false, views_stale = false;
        std::vector<uint8_t> stale;
        uint32_t n_stale = 0;
    } ck, bk;
    void invalidate_saved() { ck.valid = bk.valid = false; }
    // cpuset binding: CPU topology table, per-record allocations (device order, like h_dev)
    kg_cpu_topo* d_cpu_topos = nullptr;
    uint32_t n_cpu_topos = 0;
    kg_cpu_alloc* d_cpu_alloc = nullptr;
    std::vector<kg_cpu_alloc> h_cpu_alloc;
    bool has_cpu = false;   // the snapshot carries CPU topologies
    bool node_bind = false; // some node has a CPU bind policy (every pod with a cpu request binds there)
    // GPU partition tables (kg_node_columns.gpu_parts): entries and per (table, GPU count) ranges
    kg_gpu_partition* d_parts = nullptr;
    uint32_t* d_part_rng = nullptr;  // [KG_GPU_MAX_TABLES * 9]
    int64_t* d_binpack = nullptr;    // [KG_GPU_MAX_TABLES][3][256]
    uint32_t n_gpu_tables = 0, n_gpu_parts = 0;
    bool ext() const { return (cfg.plugins & KG_PLUGIN_EXT) != 0; }
    ExtDev ext_dev() const {
        ExtDev e{};
        e.parts = n_gpu_tables ? d_parts : nullptr;
        e.n_parts = n_gpu_tables ? n_gpu_parts : 0u;
        e.part_rng = d_part_rng;
        e.binpack = d_binpack;
        e.dev = d_dev;
        e.qlim = d_qlim;
        e.qstate = d_qstate;
        e.n_quotas = n_quotas;
        e.views = d_views;
        e.infos = d_infos;
        e.cls_begin = d_cls_begin;
        e.vfirst = d_vfirst;
        e.vmap = d_vmap;
        e.rdev = d_rdev;
        e.graw = gpu_raw ? d_graw : nullptr;
        e.gnodes = d_gnodes;
        e.grsv = d_grsv;
        return e;
    }
};

struct kg_pods {
    kg_ctx* ctx = nullptr;
    uint32_t cap = 0, n = 0;
    // Inputs of the batch: one device blob filled from pinned staging by one copy per upload, regions in
    // pod_layout(n) order; the PodsDev and list pointers below point into it for the current batch.
    uint8_t* d_in = nullptr;
    uint8_t* h_in = nullptr;  // pinned host staging of the same size
    hipEvent_t in_copied = nullptr;  // the last upload's copy out of h_in (the next upload rewrites h_in after it)
    bool in_pending = false;
    uint32_t defaults_n = 0;  // the config-5 regions hold the absent-column defaults for a batch of this size (0: no)
    size_t in_bytes = 0;
    PodsDev dev{};
    uint32_t* d_order = nullptr;  // lanes of the base select: fast pods grouped by wave kind, then integer-path pods
    uint32_t n_fast = 0;          // pods in the float64 fast domain (the leading d_order entries)
    uint32_t* d_pmap = nullptr;   // config-5 "plain" pods (batch positions) grouped by wave kind
    uint32_t* d_xlist = nullptr;  // config-5 pods through k_ext_select (batch positions)
    uint32_t* d_xpos = nullptr;   // per pod its lane in d_xlist (~0 = a plain pod): the stored pairs' column
    uint32_t* d_stat_list = nullptr;  // pods carrying a GPU request or a reservation class
    int64_t* d_dev_req = nullptr;     // [n][KG_DEV_R]
    uint32_t* d_xcols = nullptr;      // dev_count, dev_keys, quota (int32), quota_keys, rsv_class (int32), dev_flags, dev_tmpl: 7 x n
    uint8_t* d_dcls = nullptr;        // GPU request class per pod (DevSum nibble), DEV_CLASSES = none
    DevClass* d_dclass = nullptr;
    uint32_t n_dclass = 0;
    uint32_t n_stat = 0;
    uint32_t n_stat_cls = 0;          // leading d_stat_list entries without a GPU request (class views only)
    uint32_t n_plain = 0, n_x = 0;
    // select results
    uint64_t* d_partial = nullptr;
    uint64_t* d_ipairs = nullptr;       // pruned integer lanes: surviving (lane, record) pairs (LaunchSelect.ipairs)
    uint32_t* d_ipair_count = nullptr;
    size_t ipairs_cap = 0;
    size_t partial_cap = 0;  // entries
    uint64_t* d_keys = nullptr;
    uint32_t k_last = 0, kk_last = 0;
    uint64_t* h_keys = nullptr;    // pinned download staging of the keys [cap][KG_TOPK_MAX]
    uint32_t* d_pstat = nullptr;   // per pod: KG_ST_UNSUPPORTED / KG_ST_QUOTA of the last select (kg_result_status)
    uint32_t* d_reason = nullptr;  // replay: per pod OR of the filter status bits (kg_replay out_reason)
    DevSum* d_devsum = nullptr;    // per record DevSum of the last config-5 select
    size_t devsum_cap = 0;
    uint64_t* d_gz = nullptr;      // gpu_zone_sum per (class-1 record, GPU request class) of the last config-5 select
    size_t gz_cap = 0;
    uint8_t* d_rcode = nullptr;    // [kg_rsv_dev table][DEV_CLASSES]: GPU allocator outcome on the restore tables
    size_t rcode_cap = 0;
    // one-pass fast-base select of the GPU pods (ExtDev.cls_max / fb_max / rows): [cap] fast-base maxima, [cap] rows
    // to re-run, [DEV_CLASSES] per-class bounds, row count
    uint32_t* d_spec = nullptr;
    int64_t* d_split = nullptr;  // kg_assume_numa / kg_forget_numa: per-zone amounts of a NUMA allocation
    // replay / shard scratch
    uint64_t* d_winners = nullptr;
    uint32_t* d_step = nullptr;
    uint64_t* d_gather = nullptr;
    size_t gather_cap = 0;
    bool fast_ok = false;  // every pod in the fast domain (no value >= 2^44, no pod NUMA policy, no cpuset binding)
    bool pod_policy = false;  // some pod carries its own NUMA policy
    bool any_cpu_bind = false;  // some pod binds cpusets (KG_POD_CPU_BIND)
    bool dev_unclassed = false; // some GPU pod has no GPU request class (more than DEV_CLASSES)
    std::vector<uint32_t> h_flags;  // host copies for argument checks (kg_forget of a cpuset pod)
    std::vector<int64_t> h_req_cpu;
    // config-5 scratch
    uint32_t* d_qst = nullptr;        // ElasticQuota PreFilter status per pod
    uint32_t* d_dev_max = nullptr;    // [cap] pass-1 NormalizeScore maxima
    uint32_t* d_rsv_max = nullptr;
    uint64_t* d_pref = nullptr;
    uint32_t* d_minors = nullptr;     // replay: GPU minors chosen per pod
    uint64_t* d_buckets = nullptr;    // replay: [3][128] per-score best keys (REPLAY_BUCKET_STRIDE apart)
    uint32_t* d_done = nullptr;       // config-5 replay: workgroups done in the current step launch (last one picks)
    uint64_t* d_xpairs = nullptr;     // fast-base config-5 select: stored general pairs (ExtDev::xpairs)
    size_t xpairs_cap = 0;            // entries
    uint32_t xT = 0;                  // row length of the pairs the last ext_stats_local stored (0 = none)
    int32_t* d_aout = nullptr;        // kg_assume_ext outputs
    uint64_t* d_rec = nullptr;        // kg_reserve / kg_unreserve: cpuset CPUs [4] + NUMA zone amounts [8]
    uint32_t* d_batch = nullptr;      // kg_batch_schedule: groups + per-pod outputs (7 x cap + 1 words)
    hipGraphExec_t xexec = nullptr;   // ext replay graph
    std::vector<uint8_t> xkey;
    uint64_t* d_tkeys = nullptr;  // [KG_TOPK_MAX][cap] config-5 sub-batch keys before the scatter
    // replay graph (G steps) cached for the (snapshot buffers, batch size, configuration) it captured
    hipGraphExec_t rexec = nullptr;
    std::vector<uint8_t> rkey;
    // block replay: per-window chunk lists and merged lists, graph of RB_R windows
    uint64_t* d_rbpart = nullptr;
    size_t rbpart_cap = 0;  // entries
    uint64_t* d_rbtops = nullptr;
    hipGraphExec_t bexec = nullptr;
    std::vector<uint8_t> bkey;
    LaunchRb rb_args{};
};

// ------------------------------------------------------------------------------------------------
namespace {

kg_status fail(kg_ctx* ctx, kg_status s, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (ctx) ctx->err = buf;
    return s;
}

#define HIP_TRY(ctx, expr)                                                                                     \
    do {                                                                                                       \
        hipError_t e_ = (expr);                                                                                \
        if (e_ != hipSuccess)                                                                                  \
            return fail((ctx), e_ == hipErrorOutOfMemory ? KG_OOM : KG_DEVICE_ERROR, "%s: %s (%s:%d)", #expr, \
                        hipGetErrorString(e_), __FILE__, __LINE__);                                            \
    } while (0)

#define NCCL_TRY(ctx, expr)                                                                                    \
    do {                                                                                                       \
        ncclResult_t r_ = (expr);                                                                              \
        if (r_ != ncclSuccess)                                                                                 \
            return fail((ctx), KG_DEVICE_ERROR, "%s: %s", #expr, ncclGetErrorString(r_));                     \
    } while (0)

constexpr int64_t I64_MAX = std::numeric_limits<int64_t>::max();

int64_t amplify(int64_t origin, double ratio) {
    if (ratio <= 1) return origin;
    return (int64_t)std::ceil((double)origin * ratio);
}

// usage-percent predicate of filterNodeUsage, evaluated in float64 exactly as Go does
bool usage_ok(int64_t e, int64_t total, int64_t thr) {
    volatile double q = (double)e / (double)total;  // volatile: keep the two roundings separate
    volatile double p = q * 100.0;
    double r = std::round(p);
    return r <= (double)thr;
}

// largest e with usage_ok(e) (cut-off), I64_MAX when no check applies
int64_t la_cut(int64_t thr, int64_t total) {
    if (thr == 0 || total == 0) return I64_MAX;
    if (!usage_ok(0, total, thr)) return -1;
    const int64_t top = (int64_t)1 << 53;
    if (usage_ok(top, total, thr)) return I64_MAX;
    int64_t lo = 0, hi = top;  // usage_ok(lo) && !usage_ok(hi)
    while (hi - lo > 1) {
        int64_t mid = lo + (hi - lo) / 2;
        if (usage_ok(mid, total, thr))
            lo = mid;
        else
            hi = mid;
    }
    return lo;
}

// 1/x rounded toward +inf (0 for x == 0): with it, trunc((F*100 - r*100) * rcp) is the exact
// truncating quotient of the fast path (kg_eval.h lr100)
double rcp_up(int64_t x) {
    if (x == 0) return 0.0;
    const double d = (double)x;
    double r = 1.0 / d;
    if (std::fma(r, d, -1.0) < 0.0) r = std::nextafter(r, std::numeric_limits<double>::infinity());
    return r;
}

int64_t rcp_bits(int64_t x) {
    const double r = rcp_up(x);
    int64_t b;
    std::memcpy(&b, &r, 8);
    return b;
}

// 0.5 / w as float (0 for w == 0): the fast path's weighted quotient is trunc((2 sum + 1) * this)
float half_rcp(int64_t w) { return w > 0 ? 0.5f * (1.0f / (float)w) : 0.0f; }

uint64_t pack32(int64_t lo, int64_t hi) { return (uint64_t)(uint32_t)lo | ((uint64_t)(uint32_t)hi << 32); }

uint64_t pack_f32(float lo, float hi) {
    uint32_t a, b;
    std::memcpy(&a, &lo, 4);
    std::memcpy(&b, &hi, 4);
    return (uint64_t)a | ((uint64_t)b << 32);
}

bool valid_weight(int64_t w) { return w >= 0 && w <= (1 << 20); }

kg_status build_kcfg(kg_ctx* ctx, const kg_config* c, KCfg* k) {
    std::memset(k, 0, sizeof(*k));
    const int64_t ws[] = {c->weight_nrf, c->weight_la, c->weight_numa, c->nrf_w_cpu, c->nrf_w_mem, c->nrf_w_sc[0],
                          c->nrf_w_sc[1], c->la_w[0], c->la_w[1], c->la_dominant_w, c->numa_w_cpu, c->numa_w_mem,
                          c->numa_hint_w_cpu, c->numa_hint_w_mem};
    for (int64_t w : ws)
        if (!valid_weight(w)) return fail(ctx, KG_INVALID_ARG, "weight %lld outside [0, 2^20]", (long long)w);
    if (c->plugins & ~(KG_PLUGIN_NRF | KG_PLUGIN_LA | KG_PLUGIN_NUMA | KG_PLUGIN_EXT))
        return fail(ctx, KG_UNSUPPORTED, "plugins mask 0x%x", c->plugins);
    if (c->plugins & KG_PLUGIN_EXT) {
        const int64_t xs[] = {c->weight_dev, c->weight_rsv, c->dev_w[0], c->dev_w[1], c->dev_w[2]};
        for (int64_t w : xs)
            if (!valid_weight(w)) return fail(ctx, KG_INVALID_ARG, "weight %lld outside [0, 2^20]", (long long)w);
        // totals must stay below 2^31 for the packed selection key: Σ weight x 100 per plugin
        const int64_t wsum = c->weight_nrf + c->weight_la + c->weight_numa + c->weight_dev + c->weight_rsv;
        if (wsum * 100 >= (1ll << 31)) return fail(ctx, KG_INVALID_ARG, "score weights too large for the packed key");
        k->w_dev = (c->plugins & KG_PLUGIN_DEV) ? (int32_t)c->weight_dev : 0;
        k->w_rsv = (c->plugins & KG_PLUGIN_RSV) ? (int32_t)c->weight_rsv : 0;
        for (int r = 0; r < DEV_R; r++) k->dev_w[r] = (int32_t)c->dev_w[r];
    }
    k->plugins = c->plugins;
    k->la_score_enabled = c->la_score_enabled;
    k->la_score_prod = c->la_score_prod;
    k->w_nrf = c->weight_nrf;
    k->w_la = c->weight_la;
    k->w_numa = c->weight_numa;
    k->nrf_w[0] = c->nrf_w_cpu;
    k->nrf_w[1] = c->nrf_w_mem;
    k->nrf_w[2] = c->nrf_w_sc[0];
    k->nrf_w[3] = c->nrf_w_sc[1];
    k->la_w[0] = c->la_w[0];
    k->la_w[1] = c->la_w[1];
    k->la_dom_w = c->la_dominant_w;
    k->la_wsum = c->la_dominant_w + c->la_w[0] + c->la_w[1];
    k->numa_w_cpu = c->numa_w_cpu;
    k->numa_w_mem = c->numa_w_mem;
    k->numa_hint_w_cpu = c->numa_hint_w_cpu;
    k->numa_hint_w_mem = c->numa_hint_w_mem;
    k->la_hw = half_rcp(k->la_wsum);
    k->most = (c->numa_most_allocated ? MOST_NUMA : 0u) | (c->numa_hint_most_allocated ? MOST_NUMA_HINT : 0u) |
              (c->dev_most_allocated ? MOST_DEV : 0u);
    if (c->nrf_most_allocated & ~0xFu) return fail(ctx, KG_INVALID_ARG, "nrf_most_allocated 0x%x", c->nrf_most_allocated);
    k->nrf_most = c->nrf_most_allocated;
    if ((c->nrf_ignored_scalars | c->rsv_ignored_scalars) & ~3u) return fail(ctx, KG_INVALID_ARG, "ignored scalar mask");
    k->nrf_ign = c->nrf_ignored_scalars;
    k->rsv_ign = c->rsv_ignored_scalars;
    return KG_OK;
}

uint32_t la_fmode(const kg_config& c, uint32_t la_flags, const int64_t* thr) {
    bool empty = true;
    for (int r = 0; r < KG_LA_R; r++)
        if (thr[r] != 0) empty = false;
    if (empty) return FMODE_PASS;
    if (!(la_flags & KG_LA_HAS_METRIC)) return FMODE_PASS;
    if (c.la_filter_expired && (la_flags & KG_LA_EXPIRED)) return c.la_schedule_expired ? FMODE_PASS : FMODE_FAIL_EXPIRED;
    if (la_flags & KG_LA_NM_NIL) return FMODE_PASS;
    return FMODE_CHECK;
}

#define COL(p, i) ((p) ? (p)[i] : 0)

kg_status build_row(kg_ctx* ctx, const kg_config& c, const kg_node_columns* s, uint32_t i, NodeRec* rec, ZoneRec* zr) {
    std::memset(rec, 0, sizeof(*rec));
    std::memset(zr, 0, sizeof(*zr));
    int64_t* v = rec->v;
    v[N_ALLOC_CPU] = COL(s->alloc_cpu, i);
    v[N_ALLOC_MEM] = COL(s->alloc_mem, i);
    v[N_ALLOC_EPH] = COL(s->alloc_eph, i);
    v[N_ALLOC_PODS] = COL(s->alloc_pods, i);
    v[N_REQ_CPU] = COL(s->req_cpu, i);
    v[N_REQ_MEM] = COL(s->req_mem, i);
    v[N_REQ_EPH] = COL(s->req_eph, i);
    v[N_NUM_PODS] = COL(s->num_pods, i);
    v[N_NZ_CPU] = COL(s->nz_cpu, i);
    v[N_NZ_MEM] = COL(s->nz_mem, i);
    v[N_SC_ALLOC0] = COL(s->sc_alloc[0], i);
    v[N_SC_ALLOC1] = COL(s->sc_alloc[1], i);
    v[N_SC_REQ0] = COL(s->sc_req[0], i);
    v[N_SC_REQ1] = COL(s->sc_req[1], i);
    for (int64_t x : {v[N_ALLOC_CPU], v[N_ALLOC_MEM], v[N_SC_ALLOC0], v[N_SC_ALLOC1]})
        if (x < 0) return fail(ctx, KG_INVALID_ARG, "node %u: negative allocatable", i);
    const uint32_t laf = COL(s->la_flags, i);
    int64_t thr_u[KG_LA_R], thr_p[KG_LA_R], thr_a[KG_LA_R], la_alloc[KG_LA_R];
    for (int r = 0; r < KG_LA_R; r++) {
        la_alloc[r] = COL(s->la_alloc[r], i);
        if (la_alloc[r] < 0) return fail(ctx, KG_INVALID_ARG, "node %u: negative LoadAware allocatable", i);
        thr_u[r] = COL(s->la_thr_usage[r], i);
        thr_p[r] = COL(s->la_thr_prod[r], i);
        thr_a[r] = COL(s->la_thr_agg[r], i);
    }
    const int64_t* thr_np = (laf & KG_LA_AGG_THR) ? thr_a : thr_u;
    v[N_LA_ALLOC0] = la_alloc[0];
    v[N_LA_ALLOC1] = la_alloc[1];
    v[N_LA_FCUT_NP0] = la_cut(thr_np[0], la_alloc[0]);
    v[N_LA_FCUT_NP1] = la_cut(thr_np[1], la_alloc[1]);
    v[N_LA_FCUT_PROD0] = la_cut(thr_p[0], la_alloc[0]);
    v[N_LA_FCUT_PROD1] = la_cut(thr_p[1], la_alloc[1]);
    v[N_LA_FBASE_NP0] = COL(s->la_fbase_np[0], i);
    v[N_LA_FBASE_NP1] = COL(s->la_fbase_np[1], i);
    v[N_LA_FBASE_PROD0] = COL(s->la_fbase_prod[0], i);
    v[N_LA_FBASE_PROD1] = COL(s->la_fbase_prod[1], i);
    v[N_LA_SBASE_NP0] = COL(s->la_sbase_np[0], i);
    v[N_LA_SBASE_NP1] = COL(s->la_sbase_np[1], i);
    v[N_LA_SBASE_PROD0] = COL(s->la_sbase_prod[0], i);
    v[N_LA_SBASE_PROD1] = COL(s->la_sbase_prod[1], i);
    uint32_t f = 0;
    f |= la_fmode(c, laf, thr_np) << F_LA_FMODE_NP_SHIFT;
    f |= la_fmode(c, laf, thr_p) << F_LA_FMODE_PROD_SHIFT;
    if (laf & KG_LA_AGG_THR) f |= F_LA_NP_AGG;
    if (laf & KG_LA_PROD_THR) f |= F_LA_PROD_THR;
    if (!(laf & KG_LA_HAS_METRIC) || (laf & KG_LA_EXPIRED) || (laf & KG_LA_NM_NIL)) f |= F_LA_SCORE_ZERO;
    if (laf & KG_LA_HAS_METRIC) f |= F_LA_HAS_METRIC;
    const uint32_t pol = COL(s->numa_policy, i);
    const uint32_t Z = COL(s->numa_zones, i);
    if (pol > KG_NUMA_SINGLE_NODE) return fail(ctx, KG_INVALID_ARG, "node %u: NUMA policy %u", i, pol);
    if (Z > KG_MAX_ZONES) return fail(ctx, KG_UNSUPPORTED, "node %u: %u NUMA zones > %d", i, Z, KG_MAX_ZONES);
    f |= pol << F_NUMA_POLICY_SHIFT;
    f |= Z << F_NUMA_ZONES_SHIFT;
    if (pol == KG_NUMA_BEST_EFFORT) f |= F_TOPO;  // the Reserve runs the topology manager (window replay: integer path)
    if (s->rsv_numa && s->rsv_numa[i]) f |= F_RSV_NUMA;
    const double ratio = s->cpu_amp_ratio ? s->cpu_amp_ratio[i] : 0.0;
    if (ratio > 1) f |= F_AMP;
    v[N_FLAGS] = f;
    v[N_RSV_CLASSES] = 0;  // set by kg_snapshot_upload_reservations
    v[N_DEV_MINORS] = s->dev_minors ? (int64_t)s->dev_minors[i] : -1;
    if (v[N_DEV_MINORS] > DEV_MINORS) return fail(ctx, KG_UNSUPPORTED, "node %u: %lld GPU minors > %d", i, (long long)v[N_DEV_MINORS], DEV_MINORS);
    v[N_CPUSET] = COL(s->cpuset_alloc_milli, i);
    v[N_AMP_CPUSET] = amplify(v[N_CPUSET], ratio);
    v[N_RCP_CPU] = rcp_bits(v[N_ALLOC_CPU]);
    v[N_RCP_MEM] = rcp_bits(v[N_ALLOC_MEM]);
    v[N_RCP_SC0] = rcp_bits(v[N_SC_ALLOC0]);
    v[N_RCP_SC1] = rcp_bits(v[N_SC_ALLOC1]);
    // LoadAware Score is 0 on this node (no / expired / nil NodeMetric): the fast path's leastUsed
    // terms vanish with a zero reciprocal (the integer path checks F_LA_SCORE_ZERO itself)
    const bool la_zero = (f & F_LA_SCORE_ZERO) != 0;
    v[N_RCP_LA0] = la_zero ? 0 : rcp_bits(la_alloc[0]);
    v[N_RCP_LA1] = la_zero ? 0 : rcp_bits(la_alloc[1]);
    // weights masked by "capacity != 0" (the LeastAllocated loops skip such resources), doubled
    auto on = [](int64_t w, int64_t cap) { return (w != 0 && cap != 0) ? 2 * w : 0; };
    {
        const int64_t w0 = on(c.nrf_w_cpu, v[N_ALLOC_CPU]), w1 = on(c.nrf_w_mem, v[N_ALLOC_MEM]);
        v[N_W_NRF01] = (int64_t)pack32(w0, w1);
        // scalar weights as 16-bit halves (the fast path requires weights <= 4096) and 1 / max(Σ 2w, 2) over
        // all four resources, the reciprocal of pods requesting both scalars
        const int64_t w2 = on(c.nrf_w_sc[0], v[N_SC_ALLOC0]), w3 = on(c.nrf_w_sc[1], v[N_SC_ALLOC1]);
        uint32_t hb4;
        const float h4 = 1.0f / (float)std::max<int64_t>(w0 + w1 + w2 + w3, 2);
        std::memcpy(&hb4, &h4, 4);
        v[N_W_NRF23] = (int64_t)pack32((w2 & 0xFFFF) | ((w3 & 0xFFFF) << 16), hb4);
        const int64_t wc = on(c.numa_w_cpu, v[N_ALLOC_CPU]), wm = on(c.numa_w_mem, v[N_ALLOC_MEM]);
        v[N_W_NUMA] = (int64_t)pack32(wc, wm);
        // NUMA score 0.5 / (w_cpu + w_mem); LeastAllocated 1 / max(Σ 2w, 2) over cpu / memory (correctly
        // rounded: within the weighted-mean error bound of kg_eval.h, so pods without scalar requests
        // need no reciprocal in the select loop)
        v[N_W_AUX] = (int64_t)pack_f32(half_rcp((wc + wm) / 2), 1.0f / (float)std::max<int64_t>(w0 + w1, 2));
    }
    for (int z = 0; z < KG_MAX_ZONES; z++) {
        zr->cpu[z] = COL(s->zone_cpu[z], i);
        zr->mem[z] = COL(s->zone_mem[z], i);
        zr->cpu_used[z] = COL(s->zone_cpu_used[z], i);
        zr->mem_used[z] = COL(s->zone_mem_used[z], i);
        if (zr->cpu[z] < 0 || zr->mem[z] < 0) return fail(ctx, KG_INVALID_ARG, "node %u: negative zone total", i);
        zr->rcp_cpu[z] = rcp_up(zr->cpu[z]);
        zr->rcp_mem[z] = rcp_up(zr->mem[z]);
        ZoneFast& zf = zr->zf[z];
        zf.rcp_cpu = zr->rcp_cpu[z];
        zf.rcp_mem = zr->rcp_mem[z];
        const int64_t hc = on(c.numa_hint_w_cpu, zr->cpu[z]), hm = on(c.numa_hint_w_mem, zr->mem[z]);
        const int64_t fc = on(c.numa_w_cpu, zr->cpu[z]), fm = on(c.numa_w_mem, zr->mem[z]);
        zf.w_hint = pack32(hc, hm);
        zf.w_score = pack32(fc, fm);
        zf.hpack = pack_f32(half_rcp((hc + hm) / 2), half_rcp((fc + fm) / 2));
    }
    zr->status = COL(s->numa_zone_status, i);
    // the cpuset pods behind the statuses (a Release takes its pod out of them): given, or one per non-idle status
    for (int z = 0; z < MAX_ZONES; z++) {
        if (s->numa_zone_pods) {
            zr->cz_single[z] = (uint8_t)(s->numa_zone_pods[i] >> (8 * z));
            zr->cz_shared[z] = (uint8_t)(s->numa_zone_pods[i] >> (8 * (MAX_ZONES + z)));
        } else {
            const uint32_t st = (zr->status >> (2 * z)) & 3u;
            zr->cz_single[z] = st == 1u ? 1 : 0;
            zr->cz_shared[z] = st >= 2u ? 1 : 0;
        }
    }
    if (s->numa_zone_pods) zr->status = zone_status_of_counts(*zr);
    zr->amp_ratio = ratio > 1 ? ratio : 1.0;
    zr->cpu_topo = -1;
    zr->cpu_meta = 1u;
    if (s->cpu_topo && s->cpu_topos) {
        const int32_t ti = s->cpu_topo[i];
        const uint32_t mr = s->cpu_max_ref ? std::max<uint32_t>(1u, s->cpu_max_ref[i]) : 1u;
        const uint32_t nb = s->cpu_bind_policy ? s->cpu_bind_policy[i] : 0u;
        const uint32_t sg = s->cpu_strategy ? s->cpu_strategy[i] : 0u;
        if (ti >= (int32_t)s->n_cpu_topos || nb > 2 || sg > 1 || mr > 255)
            return fail(ctx, KG_INVALID_ARG, "node %u: CPU topology %d / bind policy %u / strategy %u", i, ti, nb, sg);
        uint32_t cpc = 0;
        if (ti >= 0) {
            const kg_cpu_topo& t = s->cpu_topos[ti];
            if (t.n_sockets && t.n_nodes && t.n_cores && t.n_cpus) {  // CPUTopology.IsValid
                zr->cpu_topo = ti;
                cpc = t.n_cpus / t.n_cores;
                cpu_counts(t, s->cpu_alloc ? &s->cpu_alloc[i] : nullptr, (int)mr, *zr);
            }
        }
        zr->cpu_meta = mr | nb << CPU_META_BIND_SHIFT | sg << CPU_META_STRATEGY_SHIFT | cpc << CPU_META_CPC_SHIFT;
        if (zr->cpu_topo >= 0 && v[N_CPUSET] != 1000 * (int64_t)zr->cpu_allocated)
            return fail(ctx, KG_INVALID_ARG, "node %u: cpuset_alloc_milli %lld != 1000 x %d allocated CPUs", i,
                        (long long)v[N_CPUSET], zr->cpu_allocated);
    }
    if (zr->status >> (KG_ZONE_RECORD_SHIFT + KG_MAX_ZONES))  // 2 bits per zone, then the record bits
        return fail(ctx, KG_INVALID_ARG, "node %u: zone status 0x%x", i, zr->status);
    // GPU topology tree / partition table (static)
    zr->dev_topo = s->dev_topo ? s->dev_topo[i] : ~0ull;
    zr->dev_part = s->dev_part ? s->dev_part[i] : 0u;
    if ((zr->dev_part & ~(0xFFu | KG_GPU_HONOR | KG_GPU_TREE | (15u << KG_GPU_TMPL_SHIFT))) || (zr->dev_part & 0xFFu) > KG_GPU_MAX_TABLES)
        return fail(ctx, KG_INVALID_ARG, "node %u: dev_part 0x%x", i, zr->dev_part);
    // GPU NUMA node ids: each a zone id (< KG_MAX_ZONES), KG_GPU_NUMA_ANY or KG_GPU_NUMA_NONE
    zr->dev_numa = s->dev_numa ? s->dev_numa[i] : 0xFFFFFFFFu;
    for (int m = 0; m < KG_DEV_MINORS; m++) {
        const uint32_t q = (zr->dev_numa >> (4 * m)) & 0xFu;
        if (q >= (uint32_t)KG_MAX_ZONES && q != KG_GPU_NUMA_ANY && q != KG_GPU_NUMA_NONE)
            return fail(ctx, KG_UNSUPPORTED, "node %u: GPU minor %d on NUMA node %u (>= %d zones)", i, m, q, KG_MAX_ZONES);
    }
    derive_node(*rec, *zr);
    return KG_OK;
}

void build_dev(const kg_node_columns* s, uint32_t i, DevRec* d) {
    std::memset(d, 0, sizeof(*d));
    if (!s->dev_total || !s->dev_free) return;
    for (int r = 0; r < DEV_R; r++)
        for (int m = 0; m < DEV_MINORS; m++) {
            const size_t x = ((size_t)i * DEV_R + r) * DEV_MINORS + m;
            d->total[r][m] = s->dev_total[x];
            d->free_[r][m] = s->dev_free[x];
        }
}

bool force_exact() {
    static int v = -1;
    if (v < 0) {
        const char* e = std::getenv("KG_FORCE_EXACT");
        v = (e && e[0] == '1') ? 1 : 0;
    }
    return v == 1;
}

// KG_REPLAY_STEP=1: replay one pod per launch (k_replay) instead of by windows (k_rb_*)
bool force_step_replay() {
    const char* e = std::getenv("KG_REPLAY_STEP");  // read per call: tests switch it per case
    return e && e[0] == '1';
}

// KG_REPLAY_NOGRAPH=1: window replay by direct launches (kernel tracers that cannot follow graphs)
bool replay_no_graph() {
    const char* e = std::getenv("KG_REPLAY_NOGRAPH");
    return e && e[0] == '1';
}

// KG_SELECT_INT=1: select kernel on the integer path only (A/B and parity checks of the fast path)
// KG_EXT_SPLIT=0: every config-5 pod through k_ext_select (A/B aid for the plain-pod split)
bool ext_split_off() {
    static int v = -1;
    if (v < 0) {
        const char* e = std::getenv("KG_EXT_SPLIT");
        v = (e && e[0] == '0') ? 1 : 0;
    }
    return v == 1;
}

// KG_SELECT_UNFUSED=1: k == 1 selects through per-chunk partials + merge (A/B aid for the fused top-1)
bool unfused() {
    static int v = -1;
    if (v < 0) {
        const char* e = std::getenv("KG_SELECT_UNFUSED");
        v = (e && e[0] == '1') ? 1 : 0;
    }
    return v == 1;
}

bool force_int() {
    static int v = -1;
    if (v < 0) {
        const char* e = std::getenv("KG_SELECT_INT");
        v = (e && e[0] == '1') ? 1 : 0;
    }
    return v == 1;
}

// Node chunk of the select kernel: enough (pod-block, chunk) workgroups to fill 256 CUs several
// times over, while each wave still walks a long run of nodes.
// KG_SELECT_BLOCKS: workgroup target of the base select launches (tuning aid; default 8192)
uint32_t select_blocks() {
    static uint32_t v = 0;
    if (v == 0) {
        const char* e = std::getenv("KG_SELECT_BLOCKS");
        const long x = e ? std::strtol(e, nullptr, 10) : 0;
        v = (x >= 64 && x <= 65536) ? (uint32_t)x : 8192u;
    }
    return v;
}

uint32_t select_chunk(uint32_t n_nodes, uint32_t n_pods, uint32_t target_blocks = 0) {
    if (target_blocks == 0) target_blocks = select_blocks();
    const uint32_t pod_blocks = (n_pods + 255) / 256;
    uint32_t n_chunks = std::max<uint32_t>(1, (target_blocks + pod_blocks - 1) / pod_blocks);
    uint32_t chunk = (n_nodes + n_chunks - 1) / n_chunks;
    chunk = std::max<uint32_t>(chunk, 32);
    return std::max<uint32_t>(1, std::min<uint32_t>(chunk, std::max<uint32_t>(n_nodes, 1)));
}

void set_node_index(NodeRec& r, uint32_t i) {
    r.v[N_FLAGS] = (int64_t)(((uint64_t)r.v[N_FLAGS] & 0xFFFFFFFFull) | ((uint64_t)i << 32));
}

uint32_t rec_numa_policy(const NodeRec& r) { return ((uint32_t)r.v[N_FLAGS] >> F_NUMA_POLICY_SHIFT) & 15u; }

void count_topo(kg_snap* s) {
    uint32_t t = 0, b = 0;
    for (uint32_t p = 0; p < s->n; p++) {
        const uint32_t pol = rec_numa_policy(s->h_nodes[p]);
        // SingleNUMANode nodes with a node CPU bind policy bind every pod's cpus: the general topology manager too
        const bool node_bind = p < s->h_zones.size() && ((s->h_zones[p].cpu_meta >> CPU_META_BIND_SHIFT) & 3u) != 0u;
        t += pol == KG_NUMA_BEST_EFFORT || pol == KG_NUMA_RESTRICTED || (pol == KG_NUMA_SINGLE_NODE && node_bind);
        b += ((uint32_t)s->h_nodes[p].v[N_FLAGS] & F_BIG) != 0;
    }
    s->n_topo = t;
    s->n_big_est = b;
}

// Select-mode ext kernels may drop the general topology manager when nothing in the pair set needs it
// (a cpuset-binding pod on a SingleNUMANode node runs the general topology manager: its CPUs join every hint)
bool need_topo(const kg_snap* s, const kg_pods* p) {
    return s->n_topo != 0 || p->pod_policy || (p->any_cpu_bind && s->n > s->n0);
}

kg_status check_views(kg_snap* s) {
    if ((s->cfg.plugins & KG_PLUGIN_RSV) && s->n_views && s->views_stale)
        return fail(s->ctx, KG_UNSUPPORTED,
                    "reservation views are stale after a state change on %u node(s) holding them: update them "
                    "(kg_snapshot_update_views) or re-upload them (kg_snapshot_upload_reservations)", s->n_stale);
    return KG_OK;
}

void touch_views(kg_snap* s, uint32_t node) {
    if (node < s->cls_mask.size() && s->cls_mask[node]) {
        if (node < s->stale.size() && !s->stale[node]) {
            s->stale[node] = 1;
            s->n_stale++;
        }
        s->views_stale = true;
    }
}


// Place records (indexed by snapshot index) in device order: class 0 then class 1, each ascending.
void place_records(kg_snap* s, std::vector<NodeRec>& recs, std::vector<ZoneRec>& zrs, std::vector<DevRec>* devs = nullptr,
                   std::vector<kg_cpu_alloc>* cpus = nullptr) {
    const uint32_t n = s->n;
    s->pos.resize(n);
    if (devs) s->h_dev.resize(n);
    if (cpus) s->h_cpu_alloc.resize(n);
    uint32_t n0 = 0;
    for (uint32_t i = 0; i < n; i++) n0 += node_class(recs[i]) == 0;
    uint32_t a = 0, b = n0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t p = node_class(recs[i]) == 0 ? a++ : b++;
        s->pos[i] = p;
        s->h_nodes[p] = recs[i];
        s->h_zones[p] = zrs[i];
        if (devs) s->h_dev[p] = (*devs)[i];
        if (cpus) s->h_cpu_alloc[p] = (*cpus)[i];
    }
    s->n0 = n0;
    count_topo(s);
}

kg_status record_begin(kg_ctx* ctx, hipEvent_t* a, hipEvent_t* b) {
    *a = *b = nullptr;
    if (!ctx->profiling) return KG_OK;
    if (!ctx->ev_free.empty()) {
        *a = ctx->ev_free.back().first;
        *b = ctx->ev_free.back().second;
        ctx->ev_free.pop_back();
    } else {
        HIP_TRY(ctx, hipEventCreate(a));
        HIP_TRY(ctx, hipEventCreate(b));
    }
    HIP_TRY(ctx, hipEventRecord(*a, ctx->stream));
    return KG_OK;
}

kg_status record_end(kg_ctx* ctx, hipEvent_t a, hipEvent_t b) {
    if (!a) return KG_OK;
    HIP_TRY(ctx, hipEventRecord(b, ctx->stream));
    ctx->ev_live.emplace_back(a, b);
    return KG_OK;
}

}  // namespace

// ------------------------------------------------------------------------------------------------
extern "C" {  // defined with the reservation entry points
static kg_status upload_views(kg_snap* s, const kg_rsv_view* views, uint32_t nv, const kg_rsv_info* infos, uint32_t ni,
                              const kg_rsv_dev* devs, uint32_t nd);
static kg_status sync_views_from_device(kg_snap* s);
}

extern "C" {

int kg_abi_version(void) { return KG_ABI_VERSION; }

const char* kg_status_string(kg_status s) {
    switch (s) {
        case KG_OK: return "ok";
        case KG_INVALID_ARG: return "invalid argument";
        case KG_DEVICE_ERROR: return "device error";
        case KG_OOM: return "out of device memory";
        case KG_UNSUPPORTED: return "unsupported on the device path";
        case KG_NO_DEVICE: return "no device";
        case KG_RESERVE_FAILED: return "reserve failed";
    }
    return "unknown";
}

int kg_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

kg_status kg_open(int device, kg_ctx** out) {
    if (!out) return KG_INVALID_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return KG_NO_DEVICE;
    if (device < 0 || device >= n) return KG_INVALID_ARG;
    kg_ctx* ctx = new kg_ctx();
    ctx->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return KG_DEVICE_ERROR;
    }
    *out = ctx;
    return KG_OK;
}

kg_status kg_close(kg_ctx* ctx) {
    if (!ctx) return KG_INVALID_ARG;
    hipSetDevice(ctx->device);
    hipStreamSynchronize(ctx->stream);
    if (ctx->comm) ncclCommDestroy(ctx->comm);
    for (auto& e : ctx->ev_live) {
        hipEventDestroy(e.first);
        hipEventDestroy(e.second);
    }
    for (auto& e : ctx->ev_free) {
        hipEventDestroy(e.first);
        hipEventDestroy(e.second);
    }
    if (ctx->side) hipStreamDestroy(ctx->side);
    if (ctx->fork) hipEventDestroy(ctx->fork);
    if (ctx->join) hipEventDestroy(ctx->join);
    if (ctx->side2) hipStreamDestroy(ctx->side2);
    if (ctx->fork2) hipEventDestroy(ctx->fork2);
    if (ctx->join2) hipEventDestroy(ctx->join2);
    hipStreamDestroy(ctx->stream);
    delete ctx;
    return KG_OK;
}

const char* kg_last_error(const kg_ctx* ctx) { return ctx ? ctx->err.c_str() : ""; }

kg_status kg_sync(kg_ctx* ctx) {
    if (!ctx) return KG_INVALID_ARG;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return KG_OK;
}

kg_status kg_snapshot_create(kg_ctx* ctx, const kg_config* cfg, uint32_t n_nodes, uint32_t index_base, kg_snap** out) {
    if (!ctx || !cfg || !out) return KG_INVALID_ARG;
    std::lock_guard<std::mutex> g(ctx->mu);
    *out = nullptr;
    if ((uint64_t)index_base + n_nodes > 0x7FFFFFFFull)
        return fail(ctx, KG_INVALID_ARG, "node index range exceeds 2^31");
    kg_snap* s = new kg_snap();
    s->ctx = ctx;
    s->cfg = *cfg;
    kg_status st = build_kcfg(ctx, cfg, &s->kcfg);
    if (st != KG_OK) {
        delete s;
        return st;
    }
    {
        const int64_t rw[] = {cfg->nrf_w_cpu, cfg->nrf_w_mem, cfg->nrf_w_sc[0], cfg->nrf_w_sc[1], cfg->la_w[0],
                              cfg->la_w[1], cfg->la_dominant_w, cfg->numa_w_cpu, cfg->numa_w_mem,
                              cfg->numa_hint_w_cpu, cfg->numa_hint_w_mem};
        s->weights_small = true;
        for (int64_t w : rw) s->weights_small &= (w >= 0 && w <= 4096);
        s->weights_small &= (cfg->la_w[0] + cfg->la_w[1] + cfg->la_dominant_w) <= 4096;
        s->weights_small &= !cfg->numa_most_allocated && !cfg->numa_hint_most_allocated &&
                            !cfg->nrf_most_allocated &&  // fast path: LeastAllocated
                            !cfg->nrf_ignored_scalars;     // fast path: every requested scalar is checked
    }
    s->n = n_nodes;
    s->base = index_base;
    s->h_nodes.resize(n_nodes);
    s->h_zones.resize(n_nodes);
    hipSetDevice(ctx->device);
    const size_t nb = sizeof(NodeRec) * std::max<uint32_t>(n_nodes, 1), zb = sizeof(ZoneRec) * std::max<uint32_t>(n_nodes, 1);
    if (hipMalloc(&s->d_nodes, nb) != hipSuccess || hipMalloc(&s->d_zones, zb) != hipSuccess ||
        hipMalloc(&s->d_big, sizeof(uint32_t) * ((size_t)n_nodes + 1)) != hipSuccess ||
        hipMalloc(&s->d_zsel, 2 * (size_t)std::max<uint32_t>(n_nodes, 1)) != hipSuccess ||
        hipMalloc(&s->d_nsel, sizeof(int32_t) * 2 * (size_t)std::max<uint32_t>(n_nodes, 1)) != hipSuccess ||
        hipMalloc(&s->d_pos, sizeof(uint32_t) * std::max<uint32_t>(n_nodes, 1)) != hipSuccess ||
        hipMemset(s->d_big, 0, sizeof(uint32_t)) != hipSuccess) {
        hipFree(s->d_nodes);
        hipFree(s->d_zones);
        delete s;
        return fail(ctx, KG_OOM, "snapshot of %u nodes", n_nodes);
    }
    if ((cfg->plugins & KG_PLUGIN_DEV) && hipMalloc(&s->d_dev, sizeof(DevRec) * std::max<uint32_t>(n_nodes, 1)) != hipSuccess) {
        hipFree(s->d_nodes);
        hipFree(s->d_zones);
        delete s;
        return fail(ctx, KG_OOM, "device tables of %u nodes", n_nodes);
    }
    s->cls_mask.assign(n_nodes, 0);
    *out = s;
    return KG_OK;
}

static const char* cpu_topo_problem(const kg_cpu_topo& t);

// Replace the GPU partition tables (kg_node_columns.gpu_parts; GetGPUPartitionIndexer order) on the device.
static kg_status upload_gpu_parts(kg_snap* s, const kg_node_columns* cols) {
    kg_ctx* ctx = s->ctx;
    const uint32_t n = cols->gpu_parts ? cols->n_gpu_parts : 0u;
    if (n > KG_GPU_MAX_PARTS) return fail(ctx, KG_UNSUPPORTED, "%u GPU partitions > %d", n, KG_GPU_MAX_PARTS);
    std::vector<uint32_t> rng(KG_GPU_MAX_TABLES * 9, 0u);
    uint32_t tables = 0;
    for (uint32_t t = 0; t < n; t++) {
        const kg_gpu_partition& q = cols->gpu_parts[t];
        if (q.table >= KG_GPU_MAX_TABLES || q.n_gpus < 1 || q.n_gpus > 8)
            return fail(ctx, KG_INVALID_ARG, "GPU partition %u: table %u, %u GPUs", t, q.table, q.n_gpus);
        const uint32_t key = q.table * 9u + q.n_gpus;
        if (t > 0) {
            const kg_gpu_partition& pq = cols->gpu_parts[t - 1];
            const uint32_t pkey = pq.table * 9u + pq.n_gpus;
            if (pkey > key || (pkey == key && pq.alloc_score > q.alloc_score))
                return fail(ctx, KG_INVALID_ARG, "GPU partition %u: not grouped by table / GPU count / score", t);
            if (pkey != key && (rng[key] >> 16) != 0) return fail(ctx, KG_INVALID_ARG, "GPU partition %u: group split", t);
        }
        if ((rng[key] >> 16) == 0) rng[key] = t;
        rng[key] = (rng[key] & 0xFFFFu) | ((t + 1u) << 16);
        tables = std::max(tables, (uint32_t)q.table + 1u);
    }
    // selectPartitionByBinPack's per-size sums for every allocated-minor mask (allocator_gpu.go:270-285): the
    // partitions of the lowest AllocationScore group of (table, 8 / 4 / 2 GPUs) disjoint from the mask
    std::vector<int64_t> bp((size_t)KG_GPU_MAX_TABLES * 3 * 256, 0);
    const uint32_t sizes[3] = {8, 4, 2};
    for (uint32_t tb = 0; tb < tables; tb++)
        for (int k = 0; k < 3; k++) {
            const uint32_t r = rng[tb * 9 + sizes[k]], b = r & 0xFFFFu, en = r >> 16;
            for (uint32_t mask = 0; mask < 256; mask++) {
                int64_t sum = 0;
                for (uint32_t u = b; u < en && cols->gpu_parts[u].alloc_score == cols->gpu_parts[b].alloc_score; u++)
                    if (!(cols->gpu_parts[u].minors & mask)) sum += cols->gpu_parts[u].alloc_score;
                bp[((size_t)tb * 3 + k) * 256 + mask] = sum;
            }
        }
    if (!s->d_part_rng) HIP_TRY(ctx, hipMalloc(&s->d_part_rng, sizeof(uint32_t) * KG_GPU_MAX_TABLES * 9));
    if (!s->d_binpack) HIP_TRY(ctx, hipMalloc(&s->d_binpack, sizeof(int64_t) * bp.size()));
    HIP_TRY(ctx, hipMemcpyAsync(s->d_part_rng, rng.data(), sizeof(uint32_t) * rng.size(), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(s->d_binpack, bp.data(), sizeof(int64_t) * bp.size(), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // the staging vectors go out of scope
    // fixed capacity, so the pointer a captured replay graph holds never changes (only the contents do)
    if (!s->d_parts) HIP_TRY(ctx, hipMalloc(&s->d_parts, sizeof(kg_gpu_partition) * KG_GPU_MAX_PARTS));
    if (n) {
        HIP_TRY(ctx, hipMemcpyAsync(s->d_parts, cols->gpu_parts, sizeof(kg_gpu_partition) * n, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    s->n_gpu_tables = tables;
    if (n) s->n_gpu_parts = n;
    return KG_OK;
}

// Node rows name partition tables that exist.
static kg_status check_gpu_tables(kg_ctx* ctx, const kg_node_columns* cols, uint32_t n_rows, uint32_t tables) {
    for (uint32_t i = 0; cols->dev_part && i < n_rows; i++)
        if ((cols->dev_part[i] & 0xFFu) > tables)
            return fail(ctx, KG_INVALID_ARG, "node row %u: GPU partition table %u of %u", i, cols->dev_part[i] & 0xFFu, tables);
    return KG_OK;
}

// Replace the CPU topology table (kg_node_columns.cpu_topos) on the device.
static kg_status upload_cpu_topos(kg_snap* s, const kg_node_columns* cols, uint32_t n_rows) {
    kg_ctx* ctx = s->ctx;
    for (uint32_t t = 0; t < cols->n_cpu_topos; t++)
        if (const char* why = cpu_topo_problem(cols->cpu_topos[t])) return fail(ctx, KG_UNSUPPORTED, "CPU topology %u: %s", t, why);
    if (cols->n_cpu_topos > s->n_cpu_topos || !s->d_cpu_topos) {
        hipFree(s->d_cpu_topos);
        s->d_cpu_topos = nullptr;
        HIP_TRY(ctx, hipMalloc(&s->d_cpu_topos, sizeof(kg_cpu_topo) * std::max<uint32_t>(cols->n_cpu_topos, 1)));
    }
    if (cols->n_cpu_topos)
        HIP_TRY(ctx, hipMemcpyAsync(s->d_cpu_topos, cols->cpu_topos, sizeof(kg_cpu_topo) * cols->n_cpu_topos,
                                    hipMemcpyHostToDevice, ctx->stream));
    s->n_cpu_topos = std::max(s->n_cpu_topos, cols->n_cpu_topos);
    if (!s->d_cpu_alloc) HIP_TRY(ctx, hipMalloc(&s->d_cpu_alloc, sizeof(kg_cpu_alloc) * std::max<uint32_t>(s->n, 1)));
    s->has_cpu = true;
    for (uint32_t i = 0; cols->cpu_bind_policy && i < n_rows; i++) s->node_bind |= cols->cpu_bind_policy[i] != 0;
    return KG_OK;
}

kg_status kg_snapshot_upload(kg_snap* s, const kg_node_columns* cols) {
    if (!s || !cols) return KG_INVALID_ARG;
    kg_ctx* ctx = s->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    std::vector<NodeRec> recs(s->n);
    std::vector<ZoneRec> zrs(s->n);
    const bool dev = s->d_dev != nullptr;
    std::vector<DevRec> devs(dev ? s->n : 0);
    for (uint32_t i = 0; i < s->n; i++) {
        kg_status st = build_row(ctx, s->cfg, cols, i, &recs[i], &zrs[i]);
        if (st != KG_OK) return st;
        set_node_index(recs[i], i);
        recs[i].v[N_RSV_CLASSES] = (int64_t)s->cls_mask[i];
        if (dev) build_dev(cols, i, &devs[i]);
    }
    const bool cpu = cols->cpu_topo && cols->cpu_topos;
    std::vector<kg_cpu_alloc> cpus(cpu ? s->n : 0);
    for (uint32_t i = 0; cpu && i < s->n; i++) {
        if (cols->cpu_alloc) cpus[i] = cols->cpu_alloc[i];
        else std::memset(&cpus[i], 0, sizeof(kg_cpu_alloc));
    }
    {
        uint32_t tables = 0;
        for (uint32_t t = 0; cols->gpu_parts && t < cols->n_gpu_parts; t++)
            tables = std::max(tables, (uint32_t)cols->gpu_parts[t].table + 1u);
        kg_status st = check_gpu_tables(ctx, cols, s->n, tables);
        if (st != KG_OK) return st;
    }
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    s->node_bind = false;
    if (cpu) {
        kg_status st = upload_cpu_topos(s, cols, s->n);
        if (st != KG_OK) return st;
    } else {
        s->has_cpu = false;
    }
    if (dev) {
        kg_status st = upload_gpu_parts(s, cols);
        if (st != KG_OK) return st;
    }
    place_records(s, recs, zrs, dev ? &devs : nullptr, cpu ? &cpus : nullptr);
    HIP_TRY(ctx, hipMemcpyAsync(s->d_pos, s->pos.data(), sizeof(uint32_t) * s->n, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(s->d_nodes, s->h_nodes.data(), sizeof(NodeRec) * s->n, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(s->d_zones, s->h_zones.data(), sizeof(ZoneRec) * s->n, hipMemcpyHostToDevice, ctx->stream));
    if (dev) HIP_TRY(ctx, hipMemcpyAsync(s->d_dev, s->h_dev.data(), sizeof(DevRec) * s->n, hipMemcpyHostToDevice, ctx->stream));
    if (cpu)
        HIP_TRY(ctx, hipMemcpyAsync(s->d_cpu_alloc, s->h_cpu_alloc.data(), sizeof(kg_cpu_alloc) * s->n, hipMemcpyHostToDevice,
                                    ctx->stream));
    HIP_TRY(ctx, launch_big_scan(s->d_nodes, s->n, s->d_big + 1, s->d_big, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    s->uploaded = true;
    s->gen++;
    s->invalidate_saved();
    return KG_OK;
}

kg_status kg_snapshot_update_rows(kg_snap* s, const uint32_t* rows, uint32_t n, const kg_node_columns* cols) {
    if (!s || (!rows && n) || !cols) return KG_INVALID_ARG;
    kg_ctx* ctx = s->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (!s->uploaded) return fail(ctx, KG_INVALID_ARG, "snapshot not uploaded");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    std::vector<NodeRec> recs(n);
    std::vector<ZoneRec> zrs(n);
    const bool dev = s->d_dev != nullptr;
    std::vector<DevRec> devs(dev ? n : 0);
    bool moved = false;  // a row changes storage class: the record groups are rebuilt
    for (uint32_t k = 0; k < n; k++) {
        if (rows[k] >= s->n) return fail(ctx, KG_INVALID_ARG, "row %u >= %u", rows[k], s->n);
        touch_views(s, rows[k]);
        kg_status st = build_row(ctx, s->cfg, cols, k, &recs[k], &zrs[k]);
        if (st != KG_OK) return st;
        set_node_index(recs[k], rows[k]);
        recs[k].v[N_RSV_CLASSES] = (int64_t)s->cls_mask[rows[k]];
        if (dev) build_dev(cols, k, &devs[k]);
        moved |= node_class(recs[k]) != (s->pos[rows[k]] < s->n0 ? 0u : 1u);
    }
    {
        kg_status st = check_gpu_tables(ctx, cols, n, s->n_gpu_tables);  // rows name the uploaded tables
        if (st != KG_OK) return st;
    }
    const bool cpu = s->has_cpu;
    if (cpu && !(cols->cpu_topo && cols->cpu_topos))
        return fail(ctx, KG_INVALID_ARG, "the snapshot carries CPU topologies: row updates must carry them too");
    std::vector<kg_cpu_alloc> cpus(cpu ? n : 0);
    for (uint32_t k = 0; cpu && k < n; k++) {
        if (cols->cpu_alloc) cpus[k] = cols->cpu_alloc[k];
        else std::memset(&cpus[k], 0, sizeof(kg_cpu_alloc));
    }
    if (cpu) {
        kg_status st = upload_cpu_topos(s, cols, n);
        if (st != KG_OK) return st;
    }
    if (moved) {
        // device records carry Assume state: read them back, replace the rows, regroup, re-upload
        HIP_TRY(ctx, hipMemcpyAsync(s->h_nodes.data(), s->d_nodes, sizeof(NodeRec) * s->n, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(s->h_zones.data(), s->d_zones, sizeof(ZoneRec) * s->n, hipMemcpyDeviceToHost, ctx->stream));
        if (dev) HIP_TRY(ctx, hipMemcpyAsync(s->h_dev.data(), s->d_dev, sizeof(DevRec) * s->n, hipMemcpyDeviceToHost, ctx->stream));
        if (cpu) {
            s->h_cpu_alloc.resize(s->n);
            HIP_TRY(ctx, hipMemcpyAsync(s->h_cpu_alloc.data(), s->d_cpu_alloc, sizeof(kg_cpu_alloc) * s->n,
                                        hipMemcpyDeviceToHost, ctx->stream));
        }
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        std::vector<NodeRec> all(s->n);
        std::vector<ZoneRec> allz(s->n);
        std::vector<DevRec> alld(dev ? s->n : 0);
        std::vector<kg_cpu_alloc> allc(cpu ? s->n : 0);
        for (uint32_t p = 0; p < s->n; p++) {
            const uint32_t i = node_index(s->h_nodes[p]);
            all[i] = s->h_nodes[p];
            allz[i] = s->h_zones[p];
            if (dev) alld[i] = s->h_dev[p];
            if (cpu) allc[i] = s->h_cpu_alloc[p];
        }
        for (uint32_t k = 0; k < n; k++) {
            all[rows[k]] = recs[k];
            allz[rows[k]] = zrs[k];
            if (dev) alld[rows[k]] = devs[k];
            if (cpu) allc[rows[k]] = cpus[k];
        }
        place_records(s, all, allz, dev ? &alld : nullptr, cpu ? &allc : nullptr);
        if (cpu)
            HIP_TRY(ctx, hipMemcpyAsync(s->d_cpu_alloc, s->h_cpu_alloc.data(), sizeof(kg_cpu_alloc) * s->n,
                                        hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(s->d_pos, s->pos.data(), sizeof(uint32_t) * s->n, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(s->d_nodes, s->h_nodes.data(), sizeof(NodeRec) * s->n, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(s->d_zones, s->h_zones.data(), sizeof(ZoneRec) * s->n, hipMemcpyHostToDevice, ctx->stream));
        if (dev) HIP_TRY(ctx, hipMemcpyAsync(s->d_dev, s->h_dev.data(), sizeof(DevRec) * s->n, hipMemcpyHostToDevice, ctx->stream));
        if (s->n_views) {  // the views name records by position: re-place them (their staleness stays as it is)
            kg_status sst = sync_views_from_device(s);
            if (sst != KG_OK) return sst;
            const std::vector<uint8_t> keep = s->stale;
            const uint32_t keep_n = s->n_stale;
            const std::vector<kg_rsv_view> v = s->h_views;
            const std::vector<kg_rsv_info> in = s->h_infos;
            const std::vector<kg_rsv_dev> d = s->h_rdevs;
            kg_status st = upload_views(s, v.data(), (uint32_t)v.size(), in.data(), (uint32_t)in.size(), d.data(),
                                        (uint32_t)d.size());
            if (st != KG_OK) return st;
            s->stale = keep;
            s->n_stale = keep_n;
            s->views_stale = keep_n != 0;
        }
    } else if (n) {
        // one staged copy of every changed record, then one scatter launch to their positions
        const size_t rb = sizeof(NodeRec) + sizeof(ZoneRec) + (dev ? sizeof(DevRec) : 0);
        if (n > s->stage_cap) {
            hipFree(s->d_stage);
            hipFree(s->d_stage_pos);
            s->d_stage = nullptr;
            s->d_stage_pos = nullptr;
            s->stage_cap = 0;
            const size_t cap = std::max<size_t>(n, 256);
            if (hipMalloc(&s->d_stage, (sizeof(NodeRec) + sizeof(ZoneRec) + sizeof(DevRec)) * cap) != hipSuccess ||
                hipMalloc(&s->d_stage_pos, sizeof(uint32_t) * cap) != hipSuccess)
                return fail(ctx, KG_OOM, "row-update staging for %u rows", n);
            s->stage_cap = cap;
        }
        s->h_stage.resize(rb * n + sizeof(uint32_t) * n);
        uint8_t* h = s->h_stage.data();
        uint32_t* hpos = reinterpret_cast<uint32_t*>(h + rb * n);
        for (uint32_t k = 0; k < n; k++) {
            const uint32_t p = s->pos[rows[k]];
            s->h_nodes[p] = recs[k];
            s->h_zones[p] = zrs[k];
            uint8_t* o = h + rb * k;
            std::memcpy(o, &recs[k], sizeof(NodeRec));
            std::memcpy(o + sizeof(NodeRec), &zrs[k], sizeof(ZoneRec));
            if (dev) {
                s->h_dev[p] = devs[k];
                std::memcpy(o + sizeof(NodeRec) + sizeof(ZoneRec), &devs[k], sizeof(DevRec));
            }
            hpos[k] = p;
            if (cpu) {
                s->h_cpu_alloc[p] = cpus[k];
                HIP_TRY(ctx, hipMemcpyAsync(s->d_cpu_alloc + p, &s->h_cpu_alloc[p], sizeof(kg_cpu_alloc),
                                            hipMemcpyHostToDevice, ctx->stream));
            }
        }
        HIP_TRY(ctx, hipMemcpyAsync(s->d_stage, h, rb * n, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(s->d_stage_pos, hpos, sizeof(uint32_t) * n, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(ctx, launch_scatter_rows(s->d_stage, s->d_stage_pos, n, dev, s->d_nodes, s->d_zones, s->d_dev, ctx->stream));
        count_topo(s);
    }
    HIP_TRY(ctx, launch_big_scan(s->d_nodes, s->n, s->d_big + 1, s->d_big, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    s->gen++;
    s->invalidate_saved();
    return KG_OK;
}

kg_status kg_snapshot_generation(kg_snap* s, uint64_t* out) {
    if (!s || !out) return KG_INVALID_ARG;
    std::lock_guard<std::mutex> g(s->ctx->mu);
    *out = s->gen;
    return KG_OK;
}

kg_status kg_snapshot_read_state(kg_snap* s, kg_node_state* o) {
    if (!s || !o) return KG_INVALID_ARG;
    kg_ctx* ctx = s->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    std::vector<NodeRec> h(s->n);
    std::vector<ZoneRec> z(s->n);
    std::vector<DevRec> dv(s->d_dev ? s->n : 0);
    std::vector<kg_cpu_alloc> ca(s->d_cpu_alloc && s->has_cpu ? s->n : 0);
    if (!ca.empty())
        HIP_TRY(ctx, hipMemcpyAsync(ca.data(), s->d_cpu_alloc, sizeof(kg_cpu_alloc) * s->n, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(h.data(), s->d_nodes, sizeof(NodeRec) * s->n, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(z.data(), s->d_zones, sizeof(ZoneRec) * s->n, hipMemcpyDeviceToHost, ctx->stream));
    if (s->d_dev) HIP_TRY(ctx, hipMemcpyAsync(dv.data(), s->d_dev, sizeof(DevRec) * s->n, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    for (uint32_t pp = 0; pp < s->n; pp++) {
        const int64_t* v = h[pp].v;
        const ZoneRec& zr = z[pp];
        const uint32_t i = node_index(h[pp]);
        if (o->req_cpu) o->req_cpu[i] = v[N_REQ_CPU];
        if (o->req_mem) o->req_mem[i] = v[N_REQ_MEM];
        if (o->req_eph) o->req_eph[i] = v[N_REQ_EPH];
        if (o->num_pods) o->num_pods[i] = v[N_NUM_PODS];
        if (o->nz_cpu) o->nz_cpu[i] = v[N_NZ_CPU];
        if (o->nz_mem) o->nz_mem[i] = v[N_NZ_MEM];
        if (o->sc_req[0]) o->sc_req[0][i] = v[N_SC_REQ0];
        if (o->sc_req[1]) o->sc_req[1][i] = v[N_SC_REQ1];
        const int fb_np[2] = {N_LA_FBASE_NP0, N_LA_FBASE_NP1}, fb_p[2] = {N_LA_FBASE_PROD0, N_LA_FBASE_PROD1};
        const int sb_np[2] = {N_LA_SBASE_NP0, N_LA_SBASE_NP1}, sb_p[2] = {N_LA_SBASE_PROD0, N_LA_SBASE_PROD1};
        for (int r = 0; r < KG_LA_R; r++) {
            if (o->la_fbase_np[r]) o->la_fbase_np[r][i] = v[fb_np[r]];
            if (o->la_fbase_prod[r]) o->la_fbase_prod[r][i] = v[fb_p[r]];
            if (o->la_sbase_np[r]) o->la_sbase_np[r][i] = v[sb_np[r]];
            if (o->la_sbase_prod[r]) o->la_sbase_prod[r][i] = v[sb_p[r]];
        }
        for (int zz = 0; zz < KG_MAX_ZONES; zz++) {
            if (o->zone_cpu_used[zz]) o->zone_cpu_used[zz][i] = zr.cpu_used[zz];
            if (o->zone_mem_used[zz]) o->zone_mem_used[zz][i] = zr.mem_used[zz];
        }
        if (o->cpuset_alloc_milli) o->cpuset_alloc_milli[i] = v[N_CPUSET];
        if (o->numa_zone_status) o->numa_zone_status[i] = zr.status;
        if (o->numa_zone_pods) {
            uint64_t w = 0;
            for (int zz = 0; zz < MAX_ZONES; zz++)
                w |= (uint64_t)zr.cz_single[zz] << (8 * zz) | (uint64_t)zr.cz_shared[zz] << (8 * (MAX_ZONES + zz));
            o->numa_zone_pods[i] = w;
        }
        if (o->cpu_alloc) {
            if (!ca.empty()) o->cpu_alloc[i] = ca[pp];
            else std::memset(&o->cpu_alloc[i], 0, sizeof(kg_cpu_alloc));
        }
        if (o->dev_free && s->d_dev)
            for (int r = 0; r < DEV_R; r++)
                for (int m = 0; m < DEV_MINORS; m++) o->dev_free[((size_t)i * DEV_R + r) * DEV_MINORS + m] = dv[pp].free_[r][m];
    }
    return KG_OK;
}

kg_status kg_snapshot_destroy(kg_snap* s) {
    if (!s) return KG_INVALID_ARG;
    hipSetDevice(s->ctx->device);
    hipStreamSynchronize(s->ctx->stream);
    hipFree(s->d_nodes);
    hipFree(s->d_zones);
    hipFree(s->d_big);
    hipFree(s->d_zsel);
    hipFree(s->d_nsel);
    hipFree(s->d_rstep);
    hipFree(s->d_rlist);
    hipFree(s->d_pos);
    hipFree(s->d_dev);
    hipFree(s->d_parts);
    hipFree(s->d_part_rng);
    hipFree(s->d_rdev_rec);
    hipFree(s->d_binpack);
    hipFree(s->d_qlim);
    hipFree(s->d_qstate);
    hipFree(s->d_views);
    hipFree(s->d_vfirst);
    hipFree(s->d_vmap);
    hipFree(s->d_infos);
    hipFree(s->d_cls_begin);
    hipFree(s->d_rdev);
    hipFree(s->d_special);
    hipFree(s->d_stage);
    hipFree(s->d_stage_pos);
    for (kg_snap::Saved* k : {&s->ck, &s->bk}) {
        hipFree(k->nodes);
        hipFree(k->zones);
        hipFree(k->dev);
        hipFree(k->cpu);
        hipFree(k->q);
        hipFree(k->views);
        hipFree(k->infos);
        hipFree(k->rdev);
        hipFree(k->gnodes);
        hipFree(k->grsv);
    }
    hipFree(s->d_graw);
    hipFree(s->d_gnodes);
    hipFree(s->d_grsv);
    hipFree(s->d_cpu_topos);
    hipFree(s->d_cpu_alloc);
    delete s;
    return KG_OK;
}

}  // extern "C"

namespace {

// Regions of a pod batch's input blob for n pods (256-byte aligned). The regions every select reads come
// first; the config-5 regions after `ext` are copied only when the batch carries config-5 data (else they
// are set on the device). The layout depends on n only, so cached replay graphs keyed on n stay valid.
struct PodLayout {
    size_t cols, flags, order, pmap, ext, xlist, xpos, stat, dev_req, dev_bw, xcols, dclass, dcls, total;
};

PodLayout pod_layout(uint32_t n) {
    PodLayout L{};
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o = (o + bytes + 255) & ~(size_t)255;
        return at;
    };
    L.cols = take(sizeof(int64_t) * 9 * (size_t)n);
    L.flags = take(sizeof(uint32_t) * (size_t)n);
    L.order = take(sizeof(uint32_t) * (size_t)n);
    L.pmap = take(sizeof(uint32_t) * (size_t)n);
    L.ext = o;
    L.xlist = take(sizeof(uint32_t) * (size_t)n);
    L.xpos = take(sizeof(uint32_t) * (size_t)n);
    L.stat = take(sizeof(uint32_t) * (size_t)n);
    L.dev_req = take(sizeof(int64_t) * DEV_R * (size_t)n);
    L.dev_bw = take(sizeof(int64_t) * (size_t)n);
    L.xcols = take(sizeof(uint32_t) * 7 * (size_t)n);
    L.dclass = take(sizeof(DevClass) * DEV_CLASSES);
    L.dcls = take((size_t)n);
    L.total = o;
    return L;
}

// Point the batch's device views at the regions of pod_layout(n).
void pod_views(kg_pods* p, uint32_t n) {
    const PodLayout L = pod_layout(n);
    uint8_t* d = p->d_in;
    int64_t* c = reinterpret_cast<int64_t*>(d + L.cols);
    PodsDev& v = p->dev;
    v.req_cpu = c + 0 * (size_t)n;
    v.req_mem = c + 1 * (size_t)n;
    v.req_eph = c + 2 * (size_t)n;
    v.sc_req0 = c + 3 * (size_t)n;
    v.sc_req1 = c + 4 * (size_t)n;
    v.nz_cpu = c + 5 * (size_t)n;
    v.nz_mem = c + 6 * (size_t)n;
    v.la_est0 = c + 7 * (size_t)n;
    v.la_est1 = c + 8 * (size_t)n;
    v.flags = reinterpret_cast<uint32_t*>(d + L.flags);
    p->d_order = reinterpret_cast<uint32_t*>(d + L.order);
    p->d_pmap = reinterpret_cast<uint32_t*>(d + L.pmap);
    p->d_xlist = reinterpret_cast<uint32_t*>(d + L.xlist);
    p->d_xpos = reinterpret_cast<uint32_t*>(d + L.xpos);
    p->d_stat_list = reinterpret_cast<uint32_t*>(d + L.stat);
    p->d_dev_req = reinterpret_cast<int64_t*>(d + L.dev_req);
    p->d_xcols = reinterpret_cast<uint32_t*>(d + L.xcols);
    p->d_dclass = reinterpret_cast<DevClass*>(d + L.dclass);
    p->d_dcls = d + L.dcls;
    v.dev_req = p->d_dev_req;
    v.dev_count = p->d_xcols;
    v.dev_keys = p->d_xcols + (size_t)n;
    v.quota = reinterpret_cast<const int32_t*>(p->d_xcols + 2 * (size_t)n);
    v.quota_keys = p->d_xcols + 3 * (size_t)n;
    v.rsv_class = reinterpret_cast<const int32_t*>(p->d_xcols + 4 * (size_t)n);
    v.dev_flags = p->d_xcols + 5 * (size_t)n;
    v.dev_tmpl = p->d_xcols + 6 * (size_t)n;
    v.dev_bw = reinterpret_cast<const int64_t*>(d + L.dev_bw);
    v.dev_cls = p->d_dcls;
}

}  // namespace

extern "C" {

kg_status kg_pods_create(kg_ctx* ctx, uint32_t capacity, kg_pods** out) {
    if (!ctx || !out || capacity == 0) return KG_INVALID_ARG;
    std::lock_guard<std::mutex> g(ctx->mu);
    *out = nullptr;
    kg_pods* p = new kg_pods();
    p->ctx = ctx;
    p->cap = capacity;
    p->in_bytes = pod_layout(capacity).total;
    hipSetDevice(ctx->device);
    bool ok = hipMalloc(&p->d_in, p->in_bytes) == hipSuccess &&
              hipHostMalloc(&p->h_in, p->in_bytes, hipHostMallocDefault) == hipSuccess &&
              hipMalloc(&p->d_keys, sizeof(uint64_t) * KG_TOPK_MAX * capacity) == hipSuccess &&
              hipHostMalloc(&p->h_keys, sizeof(uint64_t) * KG_TOPK_MAX * capacity, hipHostMallocDefault) == hipSuccess &&
              hipMalloc(&p->d_winners, sizeof(uint64_t) * (capacity + 1)) == hipSuccess &&
              hipMalloc(&p->d_step, sizeof(uint32_t) * 64) == hipSuccess &&
              hipMalloc(&p->d_qst, sizeof(uint32_t) * capacity) == hipSuccess &&
              hipMalloc(&p->d_dev_max, sizeof(uint32_t) * capacity) == hipSuccess &&
              hipMalloc(&p->d_rsv_max, sizeof(uint32_t) * capacity) == hipSuccess &&
              hipMalloc(&p->d_pref, sizeof(uint64_t) * capacity) == hipSuccess &&
              hipMalloc(&p->d_minors, sizeof(uint32_t) * (capacity + 1)) == hipSuccess &&
              hipMalloc(&p->d_buckets, sizeof(uint64_t) * REPLAY_BUCKET_WORDS) == hipSuccess &&
              hipMalloc(&p->d_aout, sizeof(int32_t) * 4) == hipSuccess &&
              hipMalloc(&p->d_tkeys, sizeof(uint64_t) * KG_TOPK_MAX * capacity) == hipSuccess &&
              hipMalloc(&p->d_spec, sizeof(uint32_t) * (2 * (size_t)capacity + DEV_CLASSES + 1)) == hipSuccess &&
              hipMalloc(&p->d_pstat, sizeof(uint32_t) * capacity) == hipSuccess &&
              hipMalloc(&p->d_reason, sizeof(uint32_t) * (capacity + 1)) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&p->in_copied, hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        if (p->in_copied) hipEventDestroy(p->in_copied);
        for (void* b : {(void*)p->d_in, (void*)p->d_keys, (void*)p->d_winners, (void*)p->d_step, (void*)p->d_qst,
                        (void*)p->d_dev_max, (void*)p->d_rsv_max, (void*)p->d_pref, (void*)p->d_minors, (void*)p->d_buckets,
                        (void*)p->d_aout, (void*)p->d_tkeys, (void*)p->d_spec, (void*)p->d_pstat, (void*)p->d_reason})
            hipFree(b);
        hipHostFree(p->h_in);
        hipHostFree(p->h_keys);
        delete p;
        return fail(ctx, KG_OOM, "pod batch of %u", capacity);
    }
    pod_views(p, 0);
    *out = p;
    return KG_OK;
}

kg_status kg_pods_upload(kg_pods* p, const kg_pod_columns* cols, uint32_t n) {
    if (!p || !cols) return KG_INVALID_ARG;
    kg_ctx* ctx = p->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (n > p->cap) return fail(ctx, KG_INVALID_ARG, "%u pods > capacity %u", n, p->cap);
    // ---- validation: nothing of the batch object changes before every check has passed
    for (uint32_t j = 0; j < n; j++) {
        const uint32_t pol = cols->numa_policy ? cols->numa_policy[j] : 0;
        if (pol > KG_NUMA_SINGLE_NODE) return fail(ctx, KG_INVALID_ARG, "pod %u: NUMA policy %u", j, pol);
        for (int r = 0; cols->dev_req && r < DEV_R; r++)
            if (cols->dev_req[(size_t)j * DEV_R + r] < 0) return fail(ctx, KG_INVALID_ARG, "pod %u: negative GPU request", j);
        const int32_t cls = cols->rsv_class ? cols->rsv_class[j] : -1;
        if (cls >= RSV_MAX_CLASSES) return fail(ctx, KG_UNSUPPORTED, "pod %u: reservation class %d >= %d", j, cls, RSV_MAX_CLASSES);
        const uint32_t df = cols->dev_flags ? cols->dev_flags[j] : 0u;
        if ((df & ~0x17Fu) || ((df >> KG_GPU_POD_SCOPE_SHIFT) & 7u) > 5u)
            return fail(ctx, KG_INVALID_ARG, "pod %u: GPU requirement flags 0x%x", j, df);
        if ((df & KG_GPU_POD_RING_BW) && !cols->dev_ring_bw)
            return fail(ctx, KG_INVALID_ARG, "pod %u: KG_GPU_POD_RING_BW without dev_ring_bw", j);
        if ((df & KG_GPU_POD_TEMPLATE) && (!cols->dev_tmpl || (cols->dev_tmpl[j] >> (2 * KG_GPU_TMPL_NONE))))
            return fail(ctx, KG_INVALID_ARG, "pod %u: KG_GPU_POD_TEMPLATE without a dev_tmpl entry", j);
    }
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    // the side stream's plain-pod select of the previous batch reads d_in: it has to finish before the copy
    if (ctx->side) HIP_TRY(ctx, hipStreamSynchronize(ctx->side));
    if (ctx->side2) HIP_TRY(ctx, hipStreamSynchronize(ctx->side2));
    // the previous upload's copy out of the pinned staging has completed before it is rewritten (the upload itself
    // returns without waiting for its copy: the launches that read the batch follow it on the same stream)
    if (p->in_pending) {
        HIP_TRY(ctx, hipEventSynchronize(p->in_copied));
        p->in_pending = false;
    }
    const PodLayout L = pod_layout(n);
    uint8_t* h = p->h_in;
    int64_t* hc = reinterpret_cast<int64_t*>(h + L.cols);
    const int64_t* src[9] = {cols->req_cpu, cols->req_mem, cols->req_eph, cols->sc_req[0], cols->sc_req[1],
                             cols->nz_cpu, cols->nz_mem, cols->la_est[0], cols->la_est[1]};
    // per pod: outside the fast domain (a value < 0 or >= 2^44: one unsigned compare)
    std::vector<uint8_t> slow(std::max<uint32_t>(n, 1), 0);
    for (int c = 0; c < 9; c++) {
        int64_t* dst = hc + (size_t)c * n;
        if (!src[c]) {
            std::memset(dst, 0, sizeof(int64_t) * n);
            continue;
        }
        std::memcpy(dst, src[c], sizeof(int64_t) * n);
        for (uint32_t j = 0; j < n; j++) slow[j] |= (uint64_t)src[c][j] >= (uint64_t)FAST_LIMIT;
    }
    uint32_t* f = reinterpret_cast<uint32_t*>(h + L.flags);
    bool any_pol = false, any_bind = false, any_rsv_req = false;
    for (uint32_t j = 0; j < n; j++) {
        const uint32_t pol = cols->numa_policy ? cols->numa_policy[j] : 0;
        f[j] = (cols->flags ? (cols->flags[j] & 0xFFFFu) : 0u) | (pol << 16);
        any_pol |= pol != KG_NUMA_NONE;
        any_bind |= (f[j] & KG_POD_CPU_BIND) != 0;
        any_rsv_req |= (f[j] & KG_POD_RSV_REQUIRED) != 0;
        // values inside the fast domain: the pruned integer lanes may bound the pod with the fast path (POD_FASTV)
        if (!slow[j]) f[j] |= POD_FASTV;
        // the fast block has no CPU counts and no pod-level NUMA policy: such pods take the integer path
        slow[j] |= pol != KG_NUMA_NONE || (f[j] & KG_POD_CPU_BIND) != 0;
    }
    // fast select lanes: the fast pods grouped by wave kind (fast_kind_match in kg_eval.h; keys are written
    // per pod, so the order changes no result), then the integer-path pods in batch order
    auto wave_kind = [&](uint32_t j) {
        const uint32_t fl = f[j];
        const int64_t cpu = hc[j], mem = hc[(size_t)n + j], sc0 = hc[3 * (size_t)n + j], sc1 = hc[4 * (size_t)n + j];
        const uint32_t excl = KG_POD_DAEMONSET | KG_POD_NUMA_SKIP | KG_POD_CPU_BIND;
        if ((fl & (KG_POD_PROD | excl)) == KG_POD_PROD && (fl & (KG_POD_HAS_CPU | KG_POD_HAS_MEM)) && sc0 == 0 && sc1 == 0)
            return 0;
        if ((fl & (KG_POD_PROD | excl | KG_POD_HAS_CPU | KG_POD_HAS_MEM)) == 0 && cpu == 0 && mem == 0 && sc0 != 0 && sc1 != 0)
            return 1;
        return 2;
    };
    std::vector<uint8_t> wk(std::max<uint32_t>(n, 1));
    uint32_t cnt[4] = {0, 0, 0, 0};
    for (uint32_t j = 0; j < n; j++) {
        wk[j] = slow[j] ? 3 : (uint8_t)wave_kind(j);
        cnt[wk[j]]++;
    }
    uint32_t* order = reinterpret_cast<uint32_t*>(h + L.order);
    {
        uint32_t at[4] = {0, cnt[0], cnt[0] + cnt[1], cnt[0] + cnt[1] + cnt[2]};
        for (uint32_t j = 0; j < n; j++) order[at[wk[j]]++] = j;
    }
    const uint32_t n_fast = cnt[0] + cnt[1] + cnt[2];
    // config-5 columns (absent columns: no GPU request, no quota, no reservation class)
    const bool ext_cols = cols->dev_req || cols->dev_count || cols->dev_keys || cols->quota || cols->quota_keys ||
                          cols->rsv_class || cols->dev_flags || cols->dev_tmpl;
    uint32_t* xc = reinterpret_cast<uint32_t*>(h + L.xcols);
    uint32_t* pmap = reinterpret_cast<uint32_t*>(h + L.pmap);
    uint32_t* xlist = reinterpret_cast<uint32_t*>(h + L.xlist);
    uint32_t* stat = reinterpret_cast<uint32_t*>(h + L.stat);
    uint32_t np = 0, nx = 0, ns = 0;
    std::vector<DevClass> classes;
    bool unclassed = false;
    if (!ext_cols && !any_rsv_req) {
        // every pod is "plain": the plain lanes are the wave-kind order of every pod
        std::memcpy(pmap, order, sizeof(uint32_t) * n);
        np = n;
    } else {
        int64_t* dreq = reinterpret_cast<int64_t*>(h + L.dev_req);
        int64_t* dbw = reinterpret_cast<int64_t*>(h + L.dev_bw);
        uint8_t* dcls = h + L.dcls;
        for (uint32_t j = 0; j < n; j++) {
            const uint32_t cntj = cols->dev_count ? cols->dev_count[j] : 0u;
            const uint32_t keys = cols->dev_keys ? cols->dev_keys[j] : 0u;
            const uint32_t dfl = cols->dev_flags ? cols->dev_flags[j] : 0u;
            const uint32_t tmpl = (dfl & KG_GPU_POD_TEMPLATE) ? cols->dev_tmpl[j] : 0u;
            for (int r = 0; r < DEV_R; r++) dreq[(size_t)j * DEV_R + r] = cols->dev_req ? cols->dev_req[(size_t)j * DEV_R + r] : 0;
            dbw[j] = (dfl & KG_GPU_POD_RING_BW) ? cols->dev_ring_bw[j] : 0;
            dcls[j] = (uint8_t)DEV_CLASSES;
            if (cntj > 0) {  // GPU request class: everything the allocator and the Score read
                DevClass c{};
                c.dkeys = keys & 7u;
                c.dcount = cntj;
                c.dflags = dfl;
                c.dtmpl = tmpl;
                c.dbw = dbw[j];
                for (int r = 0; r < DEV_R; r++) c.dreq[r] = dreq[(size_t)j * DEV_R + r];
                size_t k = 0;
                while (k < classes.size() && !(classes[k].dkeys == c.dkeys && classes[k].dreq[0] == c.dreq[0] &&
                                               classes[k].dreq[1] == c.dreq[1] && classes[k].dreq[2] == c.dreq[2] &&
                                               classes[k].dcount == c.dcount && classes[k].dflags == c.dflags &&
                                               classes[k].dtmpl == c.dtmpl && classes[k].dbw == c.dbw))
                    k++;
                if (k == classes.size() && classes.size() < (size_t)DEV_CLASSES) classes.push_back(c);
                if (k < classes.size()) dcls[j] = (uint8_t)k;
            }
            unclassed |= cntj > 0 && dcls[j] == (uint8_t)DEV_CLASSES;
            const int32_t q = cols->quota ? cols->quota[j] : -1;
            const int32_t cls = cols->rsv_class ? cols->rsv_class[j] : -1;
            xc[j] = cntj;
            xc[(size_t)n + j] = keys;
            xc[2 * (size_t)n + j] = (uint32_t)q;
            xc[3 * (size_t)n + j] = cols->quota_keys ? cols->quota_keys[j] : 0u;
            xc[4 * (size_t)n + j] = (uint32_t)cls;
            xc[5 * (size_t)n + j] = dfl;
            xc[6 * (size_t)n + j] = tmpl;
            if (cntj > 0 || cls >= 0) stat[ns++] = j;
            if (cntj == 0 && cls < 0 && !(f[j] & KG_POD_RSV_REQUIRED)) pmap[np++] = j;
            else xlist[nx++] = j;
        }
        // wave-uniform work in the config-5 kernels: pods without a GPU request first (n_stat_cls, pairs_row0 rely
        // on it), then within each part by reservation class (the general-record kernels walk the class's views per
        // lane), then by GPU request; rows are scattered back by list, so the order does not change any result
        auto kind = [&](uint32_t j) {
            const uint32_t c = xc[j];
            const uint64_t gpu = c > 0 ? ((uint64_t)(0u - c) << 8) | (xc[(size_t)n + j] & 0xFFu) : 0u;  // count, request keys
            const int32_t cls = (int32_t)xc[4 * (size_t)n + j];
            return std::make_tuple(c > 0, cls, (f[j] & KG_POD_RSV_REQUIRED) != 0, gpu);
        };
        auto by_kind = [&](uint32_t a, uint32_t b) { return kind(a) < kind(b); };
        std::stable_sort(stat, stat + ns, by_kind);
        std::stable_sort(xlist, xlist + nx, by_kind);
        uint32_t* xpos = reinterpret_cast<uint32_t*>(h + L.xpos);
        std::memset(xpos, 0xFF, sizeof(uint32_t) * n);
        for (uint32_t k = 0; k < nx; k++) xpos[xlist[k]] = k;
        // plain lanes grouped by wave kind (stable buckets)
        std::vector<uint32_t> by;
        by.reserve(np);
        for (uint8_t k = 0; k < 4; k++)
            for (uint32_t t = 0; t < np; t++)
                if (wk[pmap[t]] == k) by.push_back(pmap[t]);
        std::memcpy(pmap, by.data(), sizeof(uint32_t) * np);
        if (!classes.empty()) std::memcpy(h + L.dclass, classes.data(), sizeof(DevClass) * classes.size());
    }
    uint32_t n_stat_cls = 0;
    while (n_stat_cls < ns && xc[stat[n_stat_cls]] == 0) n_stat_cls++;
    // ---- one copy of the regions this batch needs; absent config-5 columns set on the device
    pod_views(p, n);
    const bool ext_copy = ext_cols || any_rsv_req;
    const size_t bytes = n ? (ext_copy ? L.total : L.ext) : 0;
    if (bytes) HIP_TRY(ctx, hipMemcpyAsync(p->d_in, h, bytes, hipMemcpyHostToDevice, ctx->stream));
    // absent config-5 columns: their defaults, unless the previous batch of the same size left them there (nothing else
    // writes those regions)
    if (n && !ext_copy && p->defaults_n != n) {
        HIP_TRY(ctx, hipMemsetAsync(p->d_dev_req, 0, sizeof(int64_t) * DEV_R * n, ctx->stream));
        HIP_TRY(ctx, hipMemsetAsync(const_cast<int64_t*>(p->dev.dev_bw), 0, sizeof(int64_t) * n, ctx->stream));
        const int xdef[7] = {0, 0, 0xFF, 0, 0xFF, 0, 0};  // -1 quota / class
        for (int c = 0; c < 7; c++)
            HIP_TRY(ctx, hipMemsetAsync(p->d_xcols + (size_t)c * n, xdef[c], sizeof(uint32_t) * n, ctx->stream));
        HIP_TRY(ctx, hipMemsetAsync(p->d_dcls, DEV_CLASSES, n, ctx->stream));
    }
    p->defaults_n = ext_copy ? 0u : n;
    if (bytes) {
        HIP_TRY(ctx, hipEventRecord(p->in_copied, ctx->stream));
        p->in_pending = true;
    }
    // ---- commit
    p->n = n;
    p->n_fast = n_fast;
    p->fast_ok = n_fast == n;
    p->pod_policy = any_pol;
    p->any_cpu_bind = any_bind;
    p->h_flags.assign(f, f + n);
    p->h_req_cpu.assign(hc, hc + n);
    p->n_stat = ns;
    p->n_stat_cls = n_stat_cls;
    p->n_plain = np;
    p->n_x = nx;
    p->n_dclass = (uint32_t)classes.size();
    p->dev_unclassed = unclassed;
    return KG_OK;
}

kg_status kg_pods_destroy(kg_pods* p) {
    if (!p) return KG_INVALID_ARG;
    hipSetDevice(p->ctx->device);
    hipStreamSynchronize(p->ctx->stream);
    if (p->ctx->side) hipStreamSynchronize(p->ctx->side);  // a plain-pod select may still read the batch there
    if (p->ctx->side2) hipStreamSynchronize(p->ctx->side2);  // and a class-1 lane of the config-5 kernels
    for (void* b : {(void*)p->d_ipairs, (void*)p->d_ipair_count})
        hipFree(b);
    for (void* b : {(void*)p->d_in, (void*)p->d_keys, (void*)p->d_winners, (void*)p->d_step, (void*)p->d_partial,
                    (void*)p->d_gather, (void*)p->d_qst, (void*)p->d_dev_max, (void*)p->d_rsv_max, (void*)p->d_pref,
                    (void*)p->d_minors, (void*)p->d_buckets, (void*)p->d_aout, (void*)p->d_tkeys, (void*)p->d_pstat,
                    (void*)p->d_reason, (void*)p->d_devsum, (void*)p->d_gz, (void*)p->d_spec, (void*)p->d_split, (void*)p->d_batch, (void*)p->d_rcode, (void*)p->d_done, (void*)p->d_rec, (void*)p->d_xpairs})
        hipFree(b);
    hipHostFree(p->h_in);
    hipHostFree(p->h_keys);
    if (p->in_copied) hipEventDestroy(p->in_copied);
    hipFree(p->d_rbpart);
    hipFree(p->d_rbtops);
    if (p->rexec) hipGraphExecDestroy(p->rexec);
    if (p->xexec) hipGraphExecDestroy(p->xexec);
    if (p->bexec) hipGraphExecDestroy(p->bexec);
    delete p;
    return KG_OK;
}

static kg_status check_pair(kg_snap* s, kg_pods* p) {
    if (!s || !p) return KG_INVALID_ARG;
    if (s->ctx != p->ctx) return fail(s->ctx, KG_INVALID_ARG, "snapshot and pods belong to different contexts");
    if (!s->uploaded) return fail(s->ctx, KG_INVALID_ARG, "snapshot not uploaded");
    return KG_OK;
}

static kg_status check_ext(kg_snap* s) {
    kg_ctx* ctx = s->ctx;
    if ((s->cfg.plugins & KG_PLUGIN_QUOTA) && s->n_quotas == 0 && !s->d_qstate)
        return fail(ctx, KG_INVALID_ARG, "KG_PLUGIN_QUOTA without kg_snapshot_upload_quotas");
    return KG_OK;
}

static kg_status ext_verify(kg_snap* s, kg_pods* p, kg_verify_out* out) {
    kg_ctx* ctx = s->ctx;
    kg_status st0 = check_ext(s);
    if (st0 != KG_OK) return st0;
    const size_t pairs = (size_t)p->n * s->n;
    if (pairs == 0) return KG_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    ExtVerifyDev d{};
    void* buf = nullptr;
    HIP_TRY(ctx, hipMalloc(&buf, pairs * (4 + 8 * 7 + 1)));
    char* b = (char*)buf;
    d.s_nrf = (int64_t*)b;
    d.s_la = d.s_nrf + pairs;
    d.s_numa = d.s_la + pairs;
    d.s_dev = d.s_numa + pairs;
    d.s_rsv = d.s_dev + pairs;
    d.order = d.s_rsv + pairs;
    d.total = d.order + pairs;
    d.status = (uint32_t*)(d.total + pairs);
    d.zone = (int8_t*)(d.status + pairs);
    const ExtDev e = s->ext_dev();
    hipError_t err = launch_ext_gate(p->dev, p->n, e, s->cfg.plugins, p->d_qst, nullptr, ctx->stream);
    if (err == hipSuccess)
        err = launch_ext_verify(s->d_nodes, s->d_zones, e, p->dev, p->n, s->n, s->base, s->kcfg, force_exact(), p->d_qst,
                                d, ctx->stream);
    if (err == hipSuccess) {
        struct {
            void* dst;
            const void* src;
            size_t sz;
        } cp[] = {{out->status, d.status, 4},     {out->score_nrf, d.s_nrf, 8}, {out->score_la, d.s_la, 8},
                  {out->score_numa, d.s_numa, 8}, {out->total, d.total, 8},     {out->numa_zone, d.zone, 1},
                  {out->score_dev, d.s_dev, 8},   {out->score_rsv, d.s_rsv, 8}};
        for (auto& c : cp)
            if (c.dst && err == hipSuccess) err = hipMemcpyAsync(c.dst, c.src, c.sz * pairs, hipMemcpyDeviceToHost, ctx->stream);
        if (err == hipSuccess) err = hipStreamSynchronize(ctx->stream);
    }
    hipFree(buf);
    HIP_TRY(ctx, err);
    return KG_OK;
}

kg_status kg_eval_verify(kg_snap* s, kg_pods* p, kg_verify_out* out) {
    kg_status st = check_pair(s, p);
    if (st != KG_OK) return st;
    if (!out) return KG_INVALID_ARG;
    kg_ctx* ctx = s->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    st = check_views(s);
    if (st != KG_OK) return st;
    if (s->ext()) return ext_verify(s, p, out);
    const size_t pairs = (size_t)p->n * s->n;
    if (pairs == 0) return KG_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    VerifyDev d{};
    void* buf = nullptr;
    const size_t bytes = pairs * (4 + 8 * 4 + 1);
    HIP_TRY(ctx, hipMalloc(&buf, bytes));
    char* b = (char*)buf;
    d.s_nrf = (int64_t*)b;
    d.s_la = d.s_nrf + pairs;
    d.s_numa = d.s_la + pairs;
    d.total = d.s_numa + pairs;
    d.status = (uint32_t*)(d.total + pairs);
    d.zone = (int8_t*)(d.status + pairs);
    hipError_t e = launch_verify(s->d_nodes, s->d_zones, p->dev, p->n, s->n, s->kcfg, force_exact(), d, ctx->stream);
    if (e == hipSuccess) {
        struct {
            void* dst;
            const void* src;
            size_t sz;
        } cp[] = {{out->status, d.status, 4}, {out->score_nrf, d.s_nrf, 8}, {out->score_la, d.s_la, 8},
                  {out->score_numa, d.s_numa, 8}, {out->total, d.total, 8}, {out->numa_zone, d.zone, 1}};
        for (auto& c : cp)
            if (c.dst && e == hipSuccess) e = hipMemcpyAsync(c.dst, c.src, c.sz * pairs, hipMemcpyDeviceToHost, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    }
    if (e == hipSuccess && out->score_dev) std::memset(out->score_dev, 0, 8 * pairs);
    if (e == hipSuccess && out->score_rsv) std::memset(out->score_rsv, 0, 8 * pairs);
    hipFree(buf);
    HIP_TRY(ctx, e);
    return KG_OK;
}

static kg_status ensure_partial(kg_pods* p, size_t need) {
    kg_ctx* ctx = p->ctx;
    if (need <= p->partial_cap) return KG_OK;
    if (p->d_partial) {
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        HIP_TRY(ctx, hipFree(p->d_partial));
        p->d_partial = nullptr;
    }
    HIP_TRY(ctx, hipMalloc(&p->d_partial, sizeof(uint64_t) * need));
    p->partial_cap = need;
    return KG_OK;
}

// config-5 pass 1 / pass 2 take the base plugins from the fast block where the fast path is valid:
// same conditions as the plain-pod split, plus all three base plugins enabled (eval_fast_key<7>)
static bool ext_fast_base(const kg_snap* s, const kg_pods* p) {
    // the fast-base kernels read the DeviceShare outcome from DevSum by class: every GPU pod needs one
    return !ext_split_off() && !force_exact() && !force_int() && s->weights_small && p->fast_ok && !need_topo(s, p) &&
           (s->kcfg.plugins & 7u) == 7u && !p->dev_unclassed;
}

// Regions of kg_pods::d_spec (one-pass fast-base select of the GPU pods).
static uint32_t* spec_fb_max(kg_pods* p) { return p->d_spec; }
static uint32_t* spec_rows(kg_pods* p) { return p->d_spec + p->cap; }
static uint32_t* spec_cls_max(kg_pods* p) { return p->d_spec + 2 * (size_t)p->cap; }
static uint32_t* spec_n_rows(kg_pods* p) { return p->d_spec + 2 * (size_t)p->cap + DEV_CLASSES; }

// config-5 matrix mode, pass 1: quota gate + per-pod NormalizeScore inputs of this shard
// The fast-base kernels take the SingleNUMANode (class-1) records' DeviceShare hints from a per-class table.
static bool gpu_zone_active(const kg_snap* s, const kg_pods* p) {
    return s->n > s->n0 && (s->kcfg.plugins & KG_PLUGIN_DEV) && (s->kcfg.plugins & KG_PLUGIN_NUMA) && p->n_dclass != 0 &&
           !std::getenv("KG_NO_GZ");
}
static bool gz_active(const kg_snap* s, const kg_pods* p) { return s->d_dev && ext_fast_base(s, p) && gpu_zone_active(s, p); }

// Fast-base batch whose storage-class-1 records (not F_BIG) run the light eval_c1 kernels off k_special_scan's second
// list: DeviceShare's hints are tabulated (e.gz), or no pod of the batch requests GPUs.
static bool c1_split(const kg_snap* s, const kg_pods* p) {
    return ext_fast_base(s, p) && s->n > s->n0 &&
           (gz_active(s, p) || p->n_dclass == 0 || !(s->kcfg.plugins & KG_PLUGIN_DEV));
}
static const uint32_t* c1_list(const kg_snap* s, const kg_pods* p) {
    return c1_split(s, p) ? s->d_special + s->n + 1 : nullptr;
}
// grid sizing of the general-record kernels: F_BIG records (plus class 1 unless split) or the largest class's views
static uint32_t special_est(const kg_snap* s, const kg_pods* p) {
    return c1_split(s, p) ? std::max(s->n_big_est, s->max_cls_views) : s->special_est();
}

// grid sizing of k_ext_select_sp: with the general pairs stored it evaluates the special list's pairs of the class pods
// (and the pairs of the rare lanes the statistics pass flagged), else every general pair
static uint32_t live_est(const kg_snap* s, const kg_pods* p) {
    return p->xT ? std::max<uint32_t>(c1_split(s, p) ? s->n_big_est : s->n - s->n0 + s->n_big_est, 1u) : special_est(s, p);
}

// room for the batch's DevSum table over this snapshot's records
static kg_status devsum_reserve(kg_snap* s, kg_pods* p) {
    kg_ctx* ctx = s->ctx;
    if (p->devsum_cap >= s->n) return KG_OK;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipFree(p->d_devsum));
    p->d_devsum = nullptr;
    p->devsum_cap = 0;
    HIP_TRY(ctx, hipMalloc(&p->d_devsum, sizeof(DevSum) * std::max<uint32_t>(s->n, 1)));
    p->devsum_cap = s->n;
    return KG_OK;
}

// room for the batch's e.gz table (gpu_zone_sum per SingleNUMANode record and GPU request class)
static kg_status gz_reserve(kg_snap* s, kg_pods* p) {
    kg_ctx* ctx = s->ctx;
    const size_t need = (size_t)(s->n - s->n0) * DEV_CLASSES;
    if (p->gz_cap >= need) return KG_OK;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipFree(p->d_gz));
    p->d_gz = nullptr;
    p->gz_cap = 0;
    HIP_TRY(ctx, hipMalloc(&p->d_gz, sizeof(uint64_t) * std::max<size_t>(need, 1)));
    p->gz_cap = need;
    return KG_OK;
}

// The replay reads DeviceShare off reservation views from the batch's DevSum table (built at its start, the winner's
// entry refreshed by each step after a Reserve that changed its minors): every GPU request class fits the table.
static bool replay_dsum(const kg_snap* s, const kg_pods* p) {
    return s->d_dev && (s->kcfg.plugins & KG_PLUGIN_DEV) && p->n_dclass != 0 && s->n != 0;
}

// Fast-base replay (k_ext_replay<false, true>): the pairs on fast-base records run the fast-base select's arithmetic
// (fast block, DevSum, e.gz on SingleNUMANode records); not with FitError reasons (the fast pairs carry no filter bits).
static bool replay_fb(const kg_snap* s, const kg_pods* p, bool exact, bool reasons) {
    if (exact || reasons || !ext_fast_base(s, p)) return false;
    return !((s->kcfg.plugins & KG_PLUGIN_DEV) && p->n_dclass != 0) || replay_dsum(s, p);
}
static bool replay_gz(const kg_snap* s, const kg_pods* p, bool exact, bool reasons) {
    return replay_fb(s, p, exact, reasons) && s->d_dev && gpu_zone_active(s, p);
}
// The batch's DevSum table over this snapshot's records (fast-base config-5 select with DeviceShare).
static const SideLane* side_lane2(kg_ctx* ctx, SideLane& l);

// *lane_open: k_gpu_zone_sum went to the second side lane and is not joined yet (only the class-1 kernels read its
// table: they run on that lane after it; the caller joins the lane into the main stream before the select)
static kg_status ext_dev_sum(kg_snap* s, kg_pods* p, ExtDev& e, bool* lane_open) {
    kg_ctx* ctx = s->ctx;
    e.dsum = nullptr;
    if (!s->d_dev || !ext_fast_base(s, p)) return KG_OK;
    const kg_status st = devsum_reserve(s, p);
    if (st != KG_OK) return st;
    const bool gz = gz_active(s, p);
    if (gz) {  // (may synchronise: before the fork)
        const kg_status gst = gz_reserve(s, p);
        if (gst != KG_OK) return gst;
    }
    const bool codes = s->n_rdev && s->d_rdev && p->n_dclass;
    if (codes && p->rcode_cap < (size_t)s->n_rdev * DEV_CLASSES) {
        const size_t need = (size_t)s->n_rdev * DEV_CLASSES;
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        HIP_TRY(ctx, hipFree(p->d_rcode));
        p->d_rcode = nullptr;
        p->rcode_cap = 0;
        HIP_TRY(ctx, hipMalloc(&p->d_rcode, need));
        p->rcode_cap = need;
    }
    // DeviceShare's NUMA hints of the SingleNUMANode records (per class) on the second side lane beside DevSum and
    // the restore tables' codes: the three tables are independent. DevSum is submitted first (the accumulators and its
    // cls_max were zeroed before the quota gate, ext_gate_local): the statistics wait for it.
    SideLane lane{};
    const SideLane* l2 = gz ? side_lane2(ctx, lane) : nullptr;
    if (l2) HIP_TRY(ctx, hipEventRecord(l2->fork, ctx->stream));
    auto drain = [&]() {
        if (l2) hipStreamSynchronize(l2->s);
    };
    if (launch_dev_sum(s->d_nodes, s->d_zones, s->d_dev, s->n, s->n0, p->d_dclass, p->n_dclass, s->kcfg, s->ext_dev(),
                       p->d_devsum, spec_cls_max(p), ctx->stream, false) != hipSuccess)
        return fail(ctx, KG_DEVICE_ERROR, "dev sum launch failed");
    e.gz = nullptr;
    if (gz) {
        if ((l2 && hipStreamWaitEvent(l2->s, l2->fork, 0) != hipSuccess) ||
            launch_gpu_zone_sum(s->d_nodes, s->d_zones, s->d_dev, s->n, s->n0, p->d_dclass, p->n_dclass, s->kcfg,
                                s->ext_dev(), p->d_gz, l2 ? l2->s : ctx->stream) != hipSuccess ||
            (l2 && hipEventRecord(l2->join, l2->s) != hipSuccess)) {
            drain();
            return fail(ctx, KG_DEVICE_ERROR, "gpu zone sum launch failed");
        }
        e.gz = p->d_gz;
    }
    e.dsum = p->d_devsum;
    e.rcode = nullptr;
    if (codes) {  // the GPU restore tables of the reservation views, per class
        if (launch_rdev_codes(s->d_nodes, s->d_zones, s->d_dev, s->d_rdev, s->d_rdev_rec, s->n_rdev, p->d_dclass,
                              p->n_dclass, s->kcfg, s->ext_dev(), p->d_rcode, ctx->stream) != hipSuccess) {
            drain();
            return fail(ctx, KG_DEVICE_ERROR, "restore codes launch failed");
        }
        e.rcode = p->d_rcode;
    }
    *lane_open = l2 != nullptr;
    return KG_OK;
}

// Quota gate (writes every pod's status first) and the pass-1 accumulators of the batch.
// (the accumulators are zeroed before the gate kernel: the plain pods' select forks right behind it, and k_dev_sum is
// then the main stream's next dispatch — behind a fill it lost the race for the CUs to the select's ~8k workgroups,
// 0.21 -> 0.96 ms)
static kg_status ext_gate_local(kg_snap* s, kg_pods* p) {
    kg_ctx* ctx = s->ctx;
    HIP_TRY(ctx, hipMemsetAsync(p->d_dev_max, 0, sizeof(uint32_t) * p->n, ctx->stream));
    HIP_TRY(ctx, hipMemsetAsync(p->d_rsv_max, 0, sizeof(uint32_t) * p->n, ctx->stream));
    HIP_TRY(ctx, hipMemsetAsync(p->d_pref, 0xFF, sizeof(uint64_t) * p->n, ctx->stream));
    HIP_TRY(ctx, hipMemsetAsync(spec_fb_max(p), 0, sizeof(uint32_t) * p->n, ctx->stream));
    HIP_TRY(ctx, hipMemsetAsync(spec_cls_max(p), 0, sizeof(uint32_t) * DEV_CLASSES, ctx->stream));  // k_dev_sum's
    HIP_TRY(ctx, launch_ext_gate(p->dev, p->n, s->ext_dev(), s->cfg.plugins, p->d_qst, p->d_pstat, ctx->stream));
    return KG_OK;
}

// the second side lane (nullptr when KG_NO_SIDE_STREAM is set or it cannot be created: one stream then)
static const SideLane* side_lane2(kg_ctx* ctx, SideLane& l) {
    if (std::getenv("KG_NO_SIDE_STREAM")) return nullptr;
    if (!ctx->side2) {
        if (hipStreamCreateWithFlags(&ctx->side2, hipStreamNonBlocking) != hipSuccess) return nullptr;
        if (hipEventCreateWithFlags(&ctx->fork2, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&ctx->join2, hipEventDisableTiming) != hipSuccess)
            return nullptr;
    }
    l.s = ctx->side2;
    l.fork = ctx->fork2;
    l.join = ctx->join2;
    return (l.s && l.fork && l.join) ? &l : nullptr;
}

// config-5 select: plain pods (no GPU request, no reservation class or affinity) take the base select by lane list
// and the others k_ext_select by d_xlist (ext_select_local)
static bool ext_split(const kg_snap* s, const kg_pods* p) {
    return !ext_split_off() && !force_exact() && !force_int() && s->weights_small && p->fast_ok && !need_topo(s, p);
}

static kg_status ext_stats_local(kg_snap* s, kg_pods* p, bool gated = false) {
    kg_ctx* ctx = s->ctx;
    ExtDev e = s->ext_dev();
    SideLane lane{};
    kg_status dst = gated ? KG_OK : ext_gate_local(s, p);
    if (dst != KG_OK) return dst;
    bool zone_lane = false;
    dst = ext_dev_sum(s, p, e, &zone_lane);
    if (dst != KG_OK) return dst;
    if (ext_fast_base(s, p)) {  // records for the PART 2 kernels (pass 1 and pass 2 of this batch)
        if (!s->d_special) HIP_TRY(ctx, hipMalloc(&s->d_special, sizeof(uint32_t) * 2 * ((size_t)s->n + 1)));
        HIP_TRY(ctx, launch_special_scan(s->d_nodes, s->n, s->n0, s->d_special, const_cast<uint32_t*>(c1_list(s, p)),
                                         ctx->stream));
    }
    p->xT = 0;
    if (ext_fast_base(s, p) && (s->cfg.plugins & (KG_PLUGIN_DEV | KG_PLUGIN_RSV)) && !std::getenv("KG_NO_XPAIRS")) {
        // the general pairs' selection inputs, stored for the select pass: [special list + largest class's views][the
        // select pass's lane], then a flag row (a lane with a pair the select pass evaluates again)
        uint32_t T = special_est(s, p) + s->max_cls_views + 64;
        if (const char* cap = std::getenv("KG_XPAIRS_T"))  // tests: fewer positions, so that lanes get flagged
            T = std::max(1u, std::min<uint32_t>(T, (uint32_t)std::strtoul(cap, nullptr, 10)));
        const bool split = ext_split(s, p);
        const uint32_t xn = split ? p->n_x : p->n;
        const size_t need = (size_t)xn * (T + 1);
        if (need * sizeof(uint64_t) <= ((size_t)4 << 30)) {
            if (p->xpairs_cap < need) {
                HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
                HIP_TRY(ctx, hipFree(p->d_xpairs));
                p->d_xpairs = nullptr;
                p->xpairs_cap = 0;
                // the stored pairs are a speed-up only: without the memory the select evaluates those pairs again
                if (hipMalloc(&p->d_xpairs, sizeof(uint64_t) * std::max<size_t>(need, 1)) != hipSuccess) {
                    (void)hipGetLastError();
                    p->d_xpairs = nullptr;
                } else {
                    p->xpairs_cap = need;
                }
            }
            if (p->d_xpairs) {
                HIP_TRY(ctx, hipMemsetAsync(p->d_xpairs + (size_t)T * xn, 0, sizeof(uint64_t) * xn, ctx->stream));
                p->xT = T;
                e.xpairs = p->d_xpairs;
                e.xT = T;
                e.xn = xn;
                e.xpos = split ? p->d_xpos : nullptr;
                e.xsp = s->d_special;
            }
        }
    }
    if (s->cfg.plugins & (KG_PLUGIN_DEV | KG_PLUGIN_RSV)) {
        // pods without a GPU request only get statistics from the nodes holding a view of their
        // reservation class (elsewhere s_dev = s_rsv = order = 0): one lane per pod over those views
        const uint32_t nc = p->n_stat_cls, ng = p->n_stat - nc;
        const bool views = nc && (s->cfg.plugins & KG_PLUGIN_RSV) && s->n_views;
        // the class pods' views on the second side lane, ahead of the class-1 statistics launch_ext_stats puts there:
        // both beside the GPU pods' general records on the main stream (disjoint pods)
        const SideLane* l2 = (views && ng) ? side_lane2(ctx, lane) : nullptr;
        if (l2) {
            HIP_TRY(ctx, hipEventRecord(l2->fork, ctx->stream));
            HIP_TRY(ctx, hipStreamWaitEvent(l2->s, l2->fork, 0));
        }
        if (views) {
            const hipError_t err = launch_ext_stats_views(s->d_nodes, s->d_zones, e, p->dev, p->d_stat_list, nc,
                                                          s->max_cls_views, s->base, s->kcfg, force_exact(), need_topo(s, p),
                                                          p->d_qst, p->d_dev_max, p->d_rsv_max, p->d_pref,
                                                          l2 ? l2->s : ctx->stream);
            if (err != hipSuccess) {
                if (l2) hipStreamSynchronize(l2->s);
                return fail(ctx, KG_DEVICE_ERROR, "view statistics launch failed: %s", hipGetErrorString(err));
            }
        }
        // config-5 waves cost unequal amounts (GPU count, views): more, smaller chunks shorten the tail
        const uint32_t chunk = select_chunk(s->n, std::max<uint32_t>(ng, 1), 8192);
        const hipError_t err = launch_ext_stats(s->d_nodes, s->d_zones, e, p->dev, p->d_stat_list + nc, ng, s->n, s->n0, chunk,
                                                s->base, s->kcfg, force_exact(), need_topo(s, p), ext_fast_base(s, p),
                                                p->d_qst, p->d_dev_max, p->d_rsv_max, p->d_pref, s->d_special,
                                                special_est(s, p), c1_list(s, p), s->n - s->n0, ctx->stream,
                                                side_lane2(ctx, lane));
        if (err != hipSuccess) {
            if (l2) hipStreamSynchronize(l2->s);
            return fail(ctx, KG_DEVICE_ERROR, "statistics launch failed: %s", hipGetErrorString(err));
        }
        if (l2) {  // (launch_ext_stats joins the lane only when it used it)
            HIP_TRY(ctx, hipEventRecord(l2->join, l2->s));
            HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, l2->join, 0));
            zone_lane = false;
        }
    }
    if (zone_lane) {  // the GPU zone hints' lane, not joined by the statistics
        SideLane z{};
        const SideLane* l2 = side_lane2(ctx, z);
        if (l2) {
            HIP_TRY(ctx, hipEventRecord(l2->join, l2->s));
            HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, l2->join, 0));
        }
    }
    return KG_OK;
}

// Launch description of a matrix-mode select of n_lanes pods (order: the n_fast fast lanes, then the
// integer-path lanes) whose keys go to out[row][kk] for rows (pod positions) [0, n_rows); *parts = the
// partial rows it needs (row stride n_rows). F_BIG records are spread over big_y chunks sized for ~2048
// workgroups from the snapshot's F_BIG count at its last upload (the device list may have grown since:
// the chunks then just get longer).
static LaunchSelect make_select(const kg_snap* s, const PodsDev& pods, const uint32_t* order, uint32_t n_lanes,
                                uint32_t n_fast, uint32_t n_rows, uint32_t kk, bool fast, uint64_t* out,
                                const uint32_t* pmap, uint32_t* pstat, uint32_t* parts) {
    LaunchSelect a{};
    a.nodes = s->d_nodes;
    a.zones = s->d_zones;
    a.pods = pods;
    a.n_pods = n_lanes;
    a.n_rows = n_rows;
    a.index_base = s->base;
    a.k = kk;
    a.exact = force_exact();
    a.fast = fast && !a.exact && !force_int() && s->weights_small;
    a.n_fast = a.fast ? n_fast : 0;
    a.cfg = s->kcfg;
    a.pmap = pmap;
    a.pstat = pstat;
    a.out = out;
    a.order = order;
    a.big_list = s->d_big + 1;
    a.big_count = s->d_big;
    a.fused = a.fast && kk == 1 && !unfused();
    a.fused_k = kk > 1 && !unfused();
    uint32_t np = 0;
    if (a.n_fast) {
        const uint32_t bounds[3] = {0, s->n0, s->n};
        for (int c = 0; c < 2; c++) {
            SelectRange& r = a.range[c];
            r.begin = bounds[c];
            r.end = bounds[c + 1];
            r.chunk = select_chunk(r.end - r.begin, a.n_fast);  // each class launch fills the chip on its own
            r.n_chunks = (r.end - r.begin + r.chunk - 1) / r.chunk;
            r.part0 = np;
            if (!a.fused && !a.fused_k) np += r.n_chunks;
        }
        const uint32_t pod_blocks = (a.n_fast + 255) / 256;
        const uint32_t want = std::max<uint32_t>(1, (2048 + pod_blocks - 1) / pod_blocks);
        a.big_y = std::max<uint32_t>(1, std::min<uint32_t>(want, (s->n_big_est + 7) / 8));
        a.big_part0 = np;
        if (!a.fused && !a.fused_k) np += a.big_y;
    }
    const uint32_t n_int = n_lanes - a.n_fast;
    if (n_int && s->n) {
        SelectRange& r = a.irange;
        r.begin = 0;
        r.end = s->n;
        r.chunk = select_chunk(s->n, n_int);
        r.n_chunks = (s->n + r.chunk - 1) / r.chunk;
        r.part0 = np;
        if (kk > 1 && !a.fused_k) np += r.n_chunks;  // top-1 / fused top-K of the integer lanes: atomics into out
    }
    *parts = np;
    return a;
}

// The plain pods' select can run beside the config-5 kernels when it is the fused top-1 (no partials shared
// with the x lanes' merge).
static bool plain_side_ok(const kg_snap* s, const kg_pods* p, uint32_t kk) {
    const bool split = !ext_split_off() && !force_exact() && !force_int() && s->weights_small && p->fast_ok &&
                       !need_topo(s, p);
    return split && kk == 1 && p->n_plain != 0 && !unfused();
}

static kg_status ensure_side(kg_ctx* ctx) {
    if (!ctx->side) {
        HIP_TRY(ctx, hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
        HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->fork, hipEventDisableTiming));
        HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->join, hipEventDisableTiming));
    }
    return KG_OK;
}

static kg_status launch_plain_side(kg_snap* s, kg_pods* p, uint32_t kk, uint64_t* d_out) {
    kg_ctx* ctx = s->ctx;
    kg_status sst = ensure_side(ctx);
    if (sst != KG_OK) return sst;
    uint32_t fparts = 0;
    LaunchSelect a = make_select(s, p->dev, p->d_pmap, p->n_plain, p->n_plain, p->n, kk, true, d_out, nullptr, p->d_pstat,
                                 &fparts);
    if (fparts) return fail(ctx, KG_DEVICE_ERROR, "side-stream select needs %u partial rows", fparts);
    a.partial = nullptr;
    HIP_TRY(ctx, hipEventRecord(ctx->fork, ctx->stream));
    HIP_TRY(ctx, hipStreamWaitEvent(ctx->side, ctx->fork, 0));
    HIP_TRY(ctx, launch_select(a, ctx->side));
    HIP_TRY(ctx, hipEventRecord(ctx->join, ctx->side));
    return KG_OK;
}

// config-5 matrix mode, pass 2: totals with the normalised terms -> per-pod top-k in d_out.
// Split: a plain pod's DeviceShare / Reservation terms are 0 and it passes their filters on every node
// (eval_pair_ext with dcount == 0, no view, no required affinity), so its keys are exactly the base
// select's; those pods run the fast select through their lane list (d_pmap) straight into d_out, the
// others k_ext_select by list. ElasticQuota rejections are applied by the scatters.
// Fast-base batches: k_ext_select<FB> over the fast-base records with the guessed DeviceShare maxima (plus their
// real ones), [all-reduce of those over the shards,] k_ext_fix_rows + re-run of the wrong guesses, then the general
// records with the final maxima; top-1 is fused (atomicMax into the row's key, no partials / merge).
static kg_status ext_select_local(kg_snap* s, kg_pods* p, uint32_t kk, uint64_t* d_out, bool global = false,
                                  bool plain_on_side = false) {
    kg_ctx* ctx = s->ctx;
    SideLane lane2{};
    const bool split = ext_split(s, p);
    const uint32_t n_x = split ? p->n_x : p->n;
    const uint32_t* xl = split ? p->d_xlist : nullptr;
    const uint32_t chunk = select_chunk(s->n, std::max<uint32_t>(n_x, 1), 8192);
    const bool fb = n_x && ext_fast_base(s, p);
    const bool fused = fb && kk == 1;
    const uint32_t lest = live_est(s, p);  // (before p->xT is consumed below)
    // a fast-base launch writes the fast-record kernel's chunks, then the special-record kernel's
    uint32_t xparts = n_x ? (s->n + chunk - 1) / chunk : 0;
    if (fb) {  // k_ext_select_xs's and k_ext_select_sp's rows
        uint32_t c2, y2, c5, y5;
        ext_part2_grid(special_est(s, p), (n_x + 255) / 256, &c2, &y2);
        ext_part2_grid(lest, (n_x + 255) / 256, &c5, &y5);
        xparts += y2 + y5;
        if (c1_split(s, p)) {
            ext_part2_grid(s->n - s->n0, (n_x + 255) / 256, &c2, &y2);
            xparts += y2;
        }
    }
    if (fused) xparts = 0;
    const uint32_t n_plain = split ? p->n_plain : 0;
    uint32_t fparts = 0;
    LaunchSelect a = make_select(s, p->dev, p->d_pmap, n_plain, n_plain, p->n, kk, true, d_out, nullptr, p->d_pstat, &fparts);
    const size_t xneed = (size_t)xparts * n_x * kk;
    kg_status st = ensure_partial(p, std::max<size_t>(xneed + (size_t)fparts * p->n * kk, 1));
    if (st != KG_OK) return st;
    a.partial = p->d_partial + xneed;
    uint64_t* xkeys = split ? p->d_tkeys : d_out;            // the x rows' merged keys
    uint64_t* xpart = fused ? xkeys : p->d_partial;          // where the x kernels write
    if (fused) HIP_TRY(ctx, hipMemsetAsync(xkeys, 0, sizeof(uint64_t) * n_x, ctx->stream));
    ExtDev xe = s->ext_dev();
    xe.dsum = (s->d_dev && ext_fast_base(s, p)) ? p->d_devsum : nullptr;  // ext_stats_local built it for this batch
    if (fb && p->xT) {  // the general pairs ext_stats_local stored for this batch
        xe.xpairs = p->d_xpairs;
        xe.xT = p->xT;
        xe.xn = n_x;
        xe.xpos = xl ? p->d_xpos : nullptr;
        xe.xsp = s->d_special;
    }
    p->xT = 0;
    xe.rcode = (xe.dsum && s->n_rdev && p->n_dclass) ? p->d_rcode : nullptr;   // and the restore tables' codes
    xe.gz = (xe.dsum && gz_active(s, p)) ? p->d_gz : nullptr;                 // and the class-1 records' GPU hints
    const bool guess = fb && xe.dsum && (s->cfg.plugins & KG_PLUGIN_DEV) && p->n_stat > p->n_stat_cls;
    if (guess) {
        xe.cls_max = spec_cls_max(p);
        xe.fb_max = spec_fb_max(p);
    }
    if (global && !guess) {  // the shards that guessed hold fast-base maxima this one's kernels must see first
        NCCL_TRY(ctx, ncclAllReduce(spec_fb_max(p), spec_fb_max(p), p->n, ncclUint32, ncclMax, ctx->comm, ctx->stream));
        HIP_TRY(ctx, launch_max_fold(p->d_dev_max, spec_fb_max(p), p->n, ctx->stream));
    }
    if (n_plain && !plain_on_side)
        HIP_TRY(ctx, launch_select(a, ctx->stream));  // zeroes d_out first at k = 1: before the x scatter
    // top-1 one-pass select with a class-1 list: the class-1 kernel runs on the second side lane beside the one-pass
    // select with the same guessed maxima (instead of after the re-run, at the end of the step), joins before
    // k_ext_fix_rows (which zeroes the wrong rows' keys) and re-runs on the wrong rows after it
    const uint32_t* c1l = fb ? c1_list(s, p) : nullptr;
    const SideLane* l2 = (fused && guess && c1l && n_x) ? side_lane2(ctx, lane2) : nullptr;
    if (l2) {
        HIP_TRY(ctx, hipEventRecord(l2->fork, ctx->stream));
        HIP_TRY(ctx, hipStreamWaitEvent(l2->s, l2->fork, 0));
        if (launch_ext_select_c1_top1(s->d_nodes, s->d_zones, xe, p->dev, xl, n_x, s->n0, s->base, s->kcfg, p->d_qst,
                                      p->d_dev_max, p->d_pref, xpart, c1l, s->n - s->n0, l2->s) != hipSuccess ||
            hipEventRecord(l2->join, l2->s) != hipSuccess) {
            hipStreamSynchronize(l2->s);
            return fail(ctx, KG_DEVICE_ERROR, "class-1 select launch failed");
        }
    }
    if (n_x) {
        const hipError_t err = launch_ext_select(s->d_nodes, s->d_zones, xe, p->dev, xl, n_x, s->n, s->n0, chunk, kk, s->base,
                                                 s->kcfg, force_exact(), need_topo(s, p), fb, p->d_qst, p->d_dev_max,
                                                 p->d_rsv_max, p->d_pref, xpart, p->d_pstat, ctx->stream);
        if (err != hipSuccess) {
            if (l2) hipStreamSynchronize(l2->s);
            return fail(ctx, KG_DEVICE_ERROR, "one-pass select launch failed: %s", hipGetErrorString(err));
        }
    }
    if (l2) HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, l2->join, 0));
    if (guess) {
        if (global) NCCL_TRY(ctx, ncclAllReduce(xe.fb_max, xe.fb_max, p->n, ncclUint32, ncclMax, ctx->comm, ctx->stream));
        HIP_TRY(ctx, launch_ext_fix(s->d_nodes, s->d_zones, xe, p->dev, xl, n_x, s->n, s->n0, chunk, kk, s->base, s->kcfg,
                                    p->d_qst, p->d_dev_max, p->d_rsv_max, p->d_pref, xpart, p->d_pstat, spec_rows(p),
                                    spec_n_rows(p), ctx->stream));
        if (l2) {  // the class-1 pairs of the re-run rows with their final maxima
            ExtDev f = xe;
            f.cls_max = nullptr;
            f.rows = spec_rows(p);
            f.n_rows = spec_n_rows(p);
            HIP_TRY(ctx, launch_ext_select_c1_top1(s->d_nodes, s->d_zones, f, p->dev, xl, n_x, s->n0, s->base, s->kcfg,
                                                   p->d_qst, p->d_dev_max, p->d_pref, xpart, c1l, s->n - s->n0, ctx->stream));
        }
        if (std::getenv("KG_TRACE_FIX")) {  // diagnostics: how many rows the guess missed
            uint32_t nr = 0;
            HIP_TRY(ctx, hipMemcpyAsync(&nr, spec_n_rows(p), sizeof(nr), hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            std::fprintf(stderr, "kg: one-pass select re-ran %u of %u rows\n", nr, n_x);
        }
    }
    if (fb && std::getenv("KG_TRACE_SP")) {  // diagnostics: the general records' work of this batch
        uint32_t nsp = 0, nc1 = 0;
        std::vector<uint64_t> flag(xe.xpairs ? n_x : 0);
        HIP_TRY(ctx, hipMemcpyAsync(&nsp, s->d_special, sizeof(nsp), hipMemcpyDeviceToHost, ctx->stream));
        if (c1_list(s, p))
            HIP_TRY(ctx, hipMemcpyAsync(&nc1, c1_list(s, p), sizeof(nc1), hipMemcpyDeviceToHost, ctx->stream));
        if (!flag.empty())
            HIP_TRY(ctx, hipMemcpyAsync(flag.data(), xe.xpairs + (size_t)xe.xT * xe.xn, sizeof(uint64_t) * n_x,
                                        hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        size_t nf = 0;
        for (uint64_t f : flag) nf += f != 0;
        std::fprintf(stderr, "kg: general records: special %u, class-1 %u, largest class %u views, n_x %u (stat %u, class-only %u), "
                     "xT %u, flagged lanes %zu\n", nsp, nc1, s->max_cls_views, n_x, p->n_stat, p->n_stat_cls, xe.xT, nf);
    }
    if (fb) {
        xe.cls_max = nullptr;
        HIP_TRY(ctx, launch_ext_select_sp(s->d_nodes, s->d_zones, xe, p->dev, xl, n_x, s->n, s->n0, chunk, kk, s->base, s->kcfg,
                                          p->d_qst, p->d_dev_max, p->d_rsv_max, p->d_pref, xpart, p->d_pstat, s->d_special,
                                          special_est(s, p), l2 ? nullptr : c1l, s->n - s->n0, lest, c1_split(s, p),
                                          ctx->stream, side_lane2(ctx, lane2)));
    }
    if (plain_on_side) HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->join, 0));  // d_out zeroed + plain keys in
    if (!split) {
        if (!fused) HIP_TRY(ctx, launch_merge(p->d_partial, xparts, p->n, kk, d_out, ctx->stream));
        return KG_OK;
    }
    if (n_x) {
        if (!fused) HIP_TRY(ctx, launch_merge(p->d_partial, xparts, n_x, kk, p->d_tkeys, ctx->stream));
        HIP_TRY(ctx, launch_scatter_keys(p->d_tkeys, p->d_xlist, n_x, kk, false, nullptr, d_out, nullptr, ctx->stream));
    }
    if (n_plain)  // the plain keys are in place: apply the ElasticQuota rejections
        HIP_TRY(ctx, launch_scatter_keys(d_out, p->d_pmap, n_plain, kk, true, p->d_qst, d_out, p->d_pstat, ctx->stream));
    return KG_OK;
}

static kg_status select_local(kg_snap* s, kg_pods* p, uint32_t k, uint64_t* d_out) {
    kg_ctx* ctx = s->ctx;
    if (k == 0 || k > (uint32_t)KG_TOPK_MAX) return fail(ctx, KG_INVALID_ARG, "k=%u outside [1, %d]", k, KG_TOPK_MAX);
    const uint32_t kk = k == 1 ? 1 : KG_TOPK_MAX;
    if (s->ext()) {
        kg_status st0 = check_ext(s);
        if (st0 != KG_OK) return st0;
        HIP_TRY(ctx, hipSetDevice(ctx->device));
        p->k_last = k;
        p->kk_last = kk;
        if (p->n == 0) return KG_OK;
        if (s->n == 0) {
            HIP_TRY(ctx, hipMemsetAsync(d_out, 0, sizeof(uint64_t) * kk * p->n, ctx->stream));
            HIP_TRY(ctx, hipMemsetAsync(p->d_pstat, 0, sizeof(uint32_t) * p->n, ctx->stream));
            return KG_OK;
        }
        // kernel-time bracket (kg_profile_read): the whole config-5 step, DevSum / pass 1 included
        hipEvent_t e0, e1;
        st0 = record_begin(ctx, &e0, &e1);
        if (st0 != KG_OK) return st0;
        // the plain pods' fused select depends on nothing the config-5 kernels build: it runs on the side stream
        // from the fork (after the quota gate has written every pod's status) and joins before the scatters
        const bool side = plain_side_ok(s, p, kk) && !std::getenv("KG_NO_SIDE_STREAM");
        // every return after the fork joins the side stream back into ctx->stream, so nothing later on
        // ctx->stream (an upload into d_in, a free) overtakes the side kernel
        struct SideJoin {
            kg_ctx* ctx;
            bool on = false;
            ~SideJoin() {
                if (on) hipStreamWaitEvent(ctx->stream, ctx->join, 0);
            }
        } join{ctx};
        if (side) {
            st0 = ext_gate_local(s, p);
            if (st0 != KG_OK) return st0;
            st0 = launch_plain_side(s, p, kk, d_out);
            join.on = ctx->join != nullptr;
            if (st0 != KG_OK) return st0;
        }
        st0 = ext_stats_local(s, p, side);
        if (st0 != KG_OK) return st0;
        st0 = ext_select_local(s, p, kk, d_out, false, side);
        if (st0 != KG_OK) return st0;
        return record_end(ctx, e0, e1);
    }
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    p->k_last = k;
    p->kk_last = kk;
    if (p->n == 0) return KG_OK;
    HIP_TRY(ctx, hipMemsetAsync(p->d_pstat, 0, sizeof(uint32_t) * p->n, ctx->stream));
    if (s->n == 0) {
        HIP_TRY(ctx, hipMemsetAsync(d_out, 0, sizeof(uint64_t) * kk * p->n, ctx->stream));
        return KG_OK;
    }
    // per pod: fast lanes (float64 fast path + F_BIG records on the integer path), then the integer lanes
    uint32_t parts = 0;
    LaunchSelect a = make_select(s, p->dev, p->d_order, p->n, p->n_fast, p->n, kk, true, d_out, nullptr, p->d_pstat, &parts);
    kg_status st = ensure_partial(p, std::max<size_t>((size_t)parts * p->n * kk, 1));
    if (st != KG_OK) return st;
    a.partial = p->d_partial;
    const uint32_t n_int = a.n_pods - a.n_fast;
    if (n_int && !a.exact && s->weights_small && (kk == 1 || a.fused_k) && !std::getenv("KG_NO_IPRUNE")) {
        // room for every (lane, record) pair the filter walks (lanes padded to workgroups, records to chunks);
        // a launch that needs more than 2^26 slots keeps the unpruned kernel
        const size_t cap = std::min<size_t>((size_t)(n_int + 255) / 256 * 256 * ((size_t)s->n + 4096), (size_t)1 << 26);
        if (p->ipairs_cap < cap) {
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            hipFree(p->d_ipairs);
            hipFree(p->d_ipair_count);
            p->d_ipairs = nullptr;
            p->d_ipair_count = nullptr;
            p->ipairs_cap = 0;
            HIP_TRY(ctx, hipMalloc(&p->d_ipairs, sizeof(uint64_t) * cap));
            HIP_TRY(ctx, hipMalloc(&p->d_ipair_count, sizeof(uint32_t) * (cap / (256 * 64) + 1)));
            p->ipairs_cap = cap;
        }
        a.ipairs = p->d_ipairs;
        a.ipair_count = p->d_ipair_count;
        a.ipairs_cap = p->ipairs_cap;
        a.iseg_cap = (uint32_t)(p->ipairs_cap / (256 * 64) + 1);
        a.iseed = 256;
    }
    if (!std::getenv("KG_NO_SIDE_STREAM")) {
        // beside the fast lanes' kernels: the pruned integer lanes (disjoint rows of out) or, without them, the
        // fused top-1 select of storage class 1 (atomicMax into the same rows)
        st = ensure_side(ctx);
        if (st != KG_OK) return st;
        a.side = ctx->side;
        a.fork = ctx->fork;
        a.join = ctx->join;
    }
    hipEvent_t e0, e1;
    st = record_begin(ctx, &e0, &e1);
    if (st != KG_OK) return st;
    const hipError_t le = launch_select(a, ctx->stream);
    // a launch error after the fork leaves the pruned lanes' kernels unjoined: drain the side stream before anything
    // later on ctx->stream (an upload into the pod columns, a free) can overtake them
    if (le != hipSuccess && a.side) hipStreamSynchronize(a.side);
    HIP_TRY(ctx, le);
    return record_end(ctx, e0, e1);
}

kg_status kg_eval_select(kg_snap* s, kg_pods* p, uint32_t k) {
    kg_status st = check_pair(s, p);
    if (st != KG_OK) return st;
    std::lock_guard<std::mutex> g(s->ctx->mu);
    st = check_views(s);
    if (st != KG_OK) return st;
    return select_local(s, p, k, p->d_keys);
}

kg_status kg_result_keys(kg_pods* p, uint64_t* out) {
    if (!p || !out) return KG_INVALID_ARG;
    kg_ctx* ctx = p->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (p->k_last == 0) return fail(ctx, KG_INVALID_ARG, "no selection result");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const uint64_t* h = p->h_keys;  // pinned staging
    HIP_TRY(ctx, hipMemcpyAsync(p->h_keys, p->d_keys, sizeof(uint64_t) * p->kk_last * p->n, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (p->k_last == p->kk_last) {
        std::memcpy(out, h, sizeof(uint64_t) * p->k_last * p->n);
        return KG_OK;
    }
    for (uint32_t j = 0; j < p->n; j++)
        for (uint32_t t = 0; t < p->k_last; t++) out[(size_t)j * p->k_last + t] = h[(size_t)j * p->kk_last + t];
    return KG_OK;
}

kg_status kg_result_status(kg_pods* p, uint32_t* out) {
    if (!p || !out) return KG_INVALID_ARG;
    kg_ctx* ctx = p->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (p->k_last == 0) return fail(ctx, KG_INVALID_ARG, "no selection result");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (p->n) HIP_TRY(ctx, hipMemcpyAsync(out, p->d_pstat, sizeof(uint32_t) * p->n, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return KG_OK;
}

}  // extern "C"

namespace {
constexpr uint32_t REPLAY_G = 256;  // replay steps per captured graph

// pod binds cpusets on (local) node: its Reserve allocated CPUs the Unreserve would have to know
bool cpuset_bound(const kg_snap* s, const kg_pods* p, uint32_t pod, uint32_t node) {
    if (!s->has_cpu || !(s->kcfg.plugins & KG_PLUGIN_NUMA) || pod >= p->h_flags.size()) return false;
    const ZoneRec& z = s->h_zones[s->pos[node]];
    const bool node_bind = ((z.cpu_meta >> CPU_META_BIND_SHIFT) & 3u) != 0;
    return z.cpu_topo >= 0 && ((p->h_flags[pod] & KG_POD_CPU_BIND) || (node_bind && p->h_req_cpu[pod] != 0));
}

// NodeNUMAResource of pod `pod` on `node` reads the restore of reservations holding NUMA / cpuset allocations there
// (kg_node_columns.rsv_numa, nodenumaresource/reservation.go:188-262), which the device does not follow: the pod binds
// CPUs there or its merged NUMA policy is not None (the pairs the select reports KG_ST_UNSUPPORTED)
bool rsv_numa_pair(const kg_snap* s, const kg_pods* p, uint32_t pod, uint32_t node) {
    if (!(s->kcfg.plugins & KG_PLUGIN_NUMA) || node >= s->n || pod >= p->h_flags.size()) return false;
    const uint32_t f = (uint32_t)s->h_nodes[s->pos[node]].v[N_FLAGS];
    if (!(f & F_RSV_NUMA) || (p->h_flags[pod] & KG_POD_NUMA_SKIP)) return false;
    const uint32_t node_pol = (f >> F_NUMA_POLICY_SHIFT) & 15u, pod_pol = (p->h_flags[pod] >> 16) & 15u;
    return node_pol != KG_NUMA_NONE || pod_pol != KG_NUMA_NONE || cpuset_bound(s, p, pod, node);
}

// some pod of the batch may meet such a pair in a sequential call (kg_replay): it refuses the batch
bool rsv_numa_batch(const kg_snap* s, const kg_pods* p) {
    if (!(s->kcfg.plugins & KG_PLUGIN_NUMA)) return false;
    bool any = false;
    for (uint32_t r = 0; r < s->n; r++) {
        const uint32_t f = (uint32_t)s->h_nodes[r].v[N_FLAGS];
        if (!(f & F_RSV_NUMA)) continue;
        any = true;
        if (((f >> F_NUMA_POLICY_SHIFT) & 15u) != KG_NUMA_NONE) return true;
        if (r < s->h_zones.size() && ((s->h_zones[r].cpu_meta >> CPU_META_BIND_SHIFT) & 3u) != 0u) return true;
    }
    return any && (p->pod_policy || p->any_cpu_bind);
}

// cpuset Reserves happen in this (snapshot, batch): the replay runs the device accumulator between steps
bool cpuset_active(const kg_snap* s, const kg_pods* p) {
    return s->has_cpu && (s->kcfg.plugins & KG_PLUGIN_NUMA) && (p->any_cpu_bind || s->node_bind);
}

std::vector<uint8_t> replay_key(const kg_snap* s, const kg_pods* p, bool exact, bool reasons = false) {
    std::vector<uint8_t> k;
    auto put = [&k](const void* x, size_t n) { k.insert(k.end(), (const uint8_t*)x, (const uint8_t*)x + n); };
    put(&reasons, sizeof(reasons));
    put(&s->d_nodes, sizeof(s->d_nodes));
    put(&s->d_zones, sizeof(s->d_zones));
    put(&s->d_zsel, sizeof(s->d_zsel));
    put(&s->n, sizeof(s->n));
    put(&s->base, sizeof(s->base));
    put(&s->kcfg, sizeof(s->kcfg));
    put(&p->n, sizeof(p->n));
    put(&exact, sizeof(exact));
    const bool cs = cpuset_active(s, p);
    put(&cs, sizeof(cs));
    put(&s->d_cpu_alloc, sizeof(s->d_cpu_alloc));
    put(&s->d_cpu_topos, sizeof(s->d_cpu_topos));
    put(&s->d_pos, sizeof(s->d_pos));
    return k;
}

// Capture REPLAY_G steps that read their base step from device memory, plus the bump of that base.
kg_status replay_graph(kg_snap* s, kg_pods* p, bool exact, bool reasons) {
    kg_ctx* ctx = s->ctx;
    std::vector<uint8_t> key = replay_key(s, p, exact, reasons);
    if (p->rexec && key == p->rkey) return KG_OK;
    if (p->rexec) {
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        hipGraphExecDestroy(p->rexec);
        p->rexec = nullptr;
    }
    hipGraph_t graph = nullptr;
    HIP_TRY(ctx, hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
    hipError_t e = hipSuccess;
    const bool cs = cpuset_active(s, p);
    for (uint32_t t = 0; t < REPLAY_G && e == hipSuccess; t++) {
        // the previous pod's cpuset Reserve runs before the step that applies its other Reserves
        if (cs)
            e = launch_cpuset_reserve(s->d_nodes, s->d_zones, s->d_cpu_alloc, s->d_cpu_topos, p->dev, s->kcfg, 0, 0,
                                      p->d_winners, p->d_step, t, s->d_pos, s->base, p->n, s->d_zsel, nullptr,
                                      ctx->stream);
        if (e == hipSuccess)
            e = launch_replay_step(s->d_nodes, s->d_zones, p->dev, p->n, s->n, s->base, s->kcfg, exact, p->d_step, t,
                                   p->d_winners, s->d_zsel, reasons ? p->d_reason : nullptr, ctx->stream);
    }
    if (e == hipSuccess) e = launch_bump(p->d_step, REPLAY_G, ctx->stream);
    hipError_t ec = hipStreamEndCapture(ctx->stream, &graph);
    if (e == hipSuccess) e = ec;
    if (e == hipSuccess) e = hipGraphInstantiate(&p->rexec, graph, nullptr, nullptr, 0);
    if (graph) hipGraphDestroy(graph);
    HIP_TRY(ctx, e);
    p->rkey = std::move(key);
    return KG_OK;
}

constexpr uint32_t RB_R = 8;  // replay windows per captured graph

// Records per k_rb_top wave of storage class c (one wave per chunk: the pass is latency-bound, so the
// costlier SingleNUMANode records take shorter chunks and more waves). KG_RB_CHUNK0 / KG_RB_CHUNK1:
// tuning aids, 1..RB_CHUNK.
uint32_t rb_chunk(int c) {
    static uint32_t v[2] = {0, 0};
    if (v[c] == 0) {
        const char* e = std::getenv(c == 0 ? "KG_RB_CHUNK0" : "KG_RB_CHUNK1");
        const long x = e ? std::strtol(e, nullptr, 10) : 0;
        // defaults from a sweep on config 3 (MI355X, 32/32 .. 8/4): 12 / 6 records, 165k -> 191k pods/s
        v[c] = (x >= 1 && x <= (long)RB_CHUNK) ? (uint32_t)x : (c == 0 ? 12u : 6u);
    }
    return v[c];
}

// Window replay: RB_R windows of (k_rb_top per storage class, k_rb_merge, k_rb_fix) per graph; each
// window reads the next pod to place from p->d_step and advances it by 1..RB_W pods.
kg_status rb_graph(kg_snap* s, kg_pods* p, bool exact) {
    kg_ctx* ctx = s->ctx;
    LaunchRb a{};
    a.nodes = s->d_nodes;
    a.zones = s->d_zones;
    a.nodes_rw = s->d_nodes;
    a.zones_rw = s->d_zones;
    a.pods = p->dev;
    a.n_pods = p->n;
    a.n_nodes = s->n;
    a.index_base = s->base;
    const uint32_t bounds[3] = {0, s->n0, s->n};
    uint32_t n_parts = 0;
    for (int c = 0; c < 2; c++) {
        const uint32_t chunk = rb_chunk(c);
        SelectRange& r = a.range[c];
        r.begin = bounds[c];
        r.end = bounds[c + 1];
        r.chunk = chunk;
        r.n_chunks = (r.end - r.begin + chunk - 1) / chunk;
        r.part0 = n_parts;
        n_parts += r.n_chunks;
    }
    a.n_parts = n_parts;
    a.exact = exact;
    a.fast = !exact && !force_int() && s->weights_small && p->fast_ok && (s->kcfg.plugins & 7u) == 7u;
    a.cfg = s->kcfg;
    a.pos = s->d_pos;
    a.step = p->d_step;
    a.winners = p->d_winners;
    const size_t need = (size_t)std::max<uint32_t>(n_parts, 1) * RB_W * RB_K;
    if (p->rbpart_cap < need) {
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        hipFree(p->d_rbpart);
        p->d_rbpart = nullptr;
        p->rbpart_cap = 0;
        HIP_TRY(ctx, hipMalloc(&p->d_rbpart, sizeof(uint64_t) * need));
        p->rbpart_cap = need;
    }
    if (!p->d_rbtops) HIP_TRY(ctx, hipMalloc(&p->d_rbtops, sizeof(uint64_t) * RB_W * RB_K));
    a.partial = p->d_rbpart;
    a.tops = p->d_rbtops;
    p->rb_args = a;
    std::vector<uint8_t> key = replay_key(s, p, exact);
    auto put = [&key](const void* x, size_t n) { key.insert(key.end(), (const uint8_t*)x, (const uint8_t*)x + n); };
    put(&s->d_pos, sizeof(s->d_pos));
    put(&s->n0, sizeof(s->n0));
    put(&a.fast, sizeof(a.fast));
    put(&p->d_rbpart, sizeof(p->d_rbpart));
    put(&p->d_rbtops, sizeof(p->d_rbtops));
    if (p->bexec && key == p->bkey) return KG_OK;
    if (p->bexec) {
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        hipGraphExecDestroy(p->bexec);
        p->bexec = nullptr;
    }
    hipGraph_t graph = nullptr;
    HIP_TRY(ctx, hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
    hipError_t e = hipSuccess;
    for (uint32_t t = 0; t < RB_R && e == hipSuccess; t++) e = launch_rb_window(a, ctx->stream);
    hipError_t ec = hipStreamEndCapture(ctx->stream, &graph);
    if (e == hipSuccess) e = ec;
    if (e == hipSuccess) e = hipGraphInstantiate(&p->bexec, graph, nullptr, nullptr, 0);
    if (graph) hipGraphDestroy(graph);
    HIP_TRY(ctx, e);
    p->bkey = std::move(key);
    return KG_OK;
}

// the replay follows reservation views (their Reservation score term and Reservation.Reserve)
bool rsv_replay(const kg_snap* s) { return (s->cfg.plugins & KG_PLUGIN_RSV) && s->n_views; }

// config-5 replay steps (DeviceShare minors, ElasticQuota used, NormalizeScore via score buckets)
kg_status ext_replay_graph(kg_snap* s, kg_pods* p, bool exact, bool reasons) {
    kg_ctx* ctx = s->ctx;
    std::vector<uint8_t> key = replay_key(s, p, exact, reasons);
    auto put = [&key](const void* x, size_t n) { key.insert(key.end(), (const uint8_t*)x, (const uint8_t*)x + n); };
    // every ExtDev field the captured launches take by value (tables re-uploaded in place keep their pointers)
    ExtDev e = s->ext_dev();
    e.dsum = replay_dsum(s, p) ? p->d_devsum : nullptr;
    const bool fb = replay_fb(s, p, exact, reasons);
    e.gz = replay_gz(s, p, exact, reasons) ? p->d_gz : nullptr;
    put(&e.dev, sizeof(e.dev));
    put(&e.dsum, sizeof(e.dsum));
    put(&e.gz, sizeof(e.gz));
    put(&fb, sizeof(fb));
    put(&s->n0, sizeof(s->n0));
    put(&p->d_dclass, sizeof(p->d_dclass));
    put(&p->n_dclass, sizeof(p->n_dclass));
    put(&e.graw, sizeof(e.graw));
    put(&e.gnodes, sizeof(e.gnodes));
    put(&e.grsv, sizeof(e.grsv));
    put(&e.qlim, sizeof(e.qlim));
    put(&e.qstate, sizeof(e.qstate));
    put(&e.n_quotas, sizeof(e.n_quotas));
    put(&e.views, sizeof(e.views));
    put(&e.infos, sizeof(e.infos));
    put(&e.cls_begin, sizeof(e.cls_begin));
    put(&e.rdev, sizeof(e.rdev));
    put(&e.parts, sizeof(e.parts));
    put(&e.n_parts, sizeof(e.n_parts));
    put(&e.part_rng, sizeof(e.part_rng));
    put(&e.binpack, sizeof(e.binpack));
    RsvStep* rs = rsv_replay(s) ? s->d_rstep : nullptr;
    put(&rs, sizeof(rs));
    put(&s->d_rlist, sizeof(s->d_rlist));
    const bool cs = cpuset_active(s, p);
    put(&cs, sizeof(cs));
    put(&s->d_cpu_alloc, sizeof(s->d_cpu_alloc));
    put(&s->d_cpu_topos, sizeof(s->d_cpu_topos));
    put(&s->d_pos, sizeof(s->d_pos));
    put(&p->d_done, sizeof(p->d_done));
    if (p->xexec && key == p->xkey) return KG_OK;
    if (p->xexec) {
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        hipGraphExecDestroy(p->xexec);
        p->xexec = nullptr;
    }
    hipGraph_t graph = nullptr;
    HIP_TRY(ctx, hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
    hipError_t err = hipSuccess;
    for (uint32_t t = 0; t < REPLAY_G && err == hipSuccess; t++) {
        // the previous pod's cpuset Reserve runs before the step that applies its other Reserves (zone codes of its
        // step in the step-parity half of zsel)
        if (cs)
            err = launch_cpuset_reserve(s->d_nodes, s->d_zones, s->d_cpu_alloc, s->d_cpu_topos, p->dev, s->kcfg, 0, 0,
                                        p->d_winners, p->d_step, t, s->d_pos, s->base, p->n, s->d_zsel, nullptr, ctx->stream,
                                        s->n);
        if (err == hipSuccess)
            err = launch_ext_replay_step(s->d_nodes, s->d_zones, s->d_dev, e, p->dev, p->n, s->n, s->base, s->kcfg, exact,
                                         p->d_step, t, p->d_winners, p->d_minors, p->d_buckets, s->d_zsel,
                                         reasons ? p->d_reason : nullptr, s->d_pos,
                                         (s->cfg.plugins & KG_PLUGIN_RSV) ? s->d_nsel : nullptr, rs, s->d_rlist,
                                         p->d_done, p->d_dclass, p->n_dclass, fb, s->n0, ctx->stream);
    }
    if (err == hipSuccess) err = launch_bump(p->d_step, REPLAY_G, ctx->stream);
    hipError_t ec = hipStreamEndCapture(ctx->stream, &graph);
    if (err == hipSuccess) err = ec;
    if (err == hipSuccess) err = hipGraphInstantiate(&p->xexec, graph, nullptr, nullptr, 0);
    if (graph) hipGraphDestroy(graph);
    HIP_TRY(ctx, err);
    p->xkey = std::move(key);
    return KG_OK;
}
}  // namespace

extern "C" {

static kg_status ext_replay(kg_snap* s, kg_pods* p, int32_t* out_node, int64_t* out_total, uint32_t* out_reason);

kg_status kg_replay(kg_snap* s, kg_pods* p, int32_t* out_node, int64_t* out_total, uint32_t* out_reason) {
    kg_status st = check_pair(s, p);
    if (st != KG_OK) return st;
    kg_ctx* ctx = s->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    st = check_views(s);
    if (st != KG_OK) return st;
    if (rsv_numa_batch(s, p))
        return fail(ctx, KG_UNSUPPORTED, "replay over nodes whose reservations hold NUMA / cpuset allocations "
                                         "(kg_node_columns.rsv_numa) with pods that bind CPUs or a NUMA policy");
    if (s->ext()) return ext_replay(s, p, out_node, out_total, out_reason);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const uint32_t n = p->n;
    const bool exact = force_exact();
    const bool reasons = out_reason != nullptr;
    // window replay needs the changed-row bitmap in LDS; every config-3 plugin scores a pair from its own row.
    // The FitError diagnosis (out_reason) needs every node's status in each pod's cycle: one pod per launch.
    const bool windows = !reasons && !force_step_replay() && !cpuset_active(s, p) && s->n <= 32u * (uint32_t)RB_BITMAP_WORDS;
    st = windows ? rb_graph(s, p, exact) : replay_graph(s, p, exact, reasons);
    if (st != KG_OK) return st;
    HIP_TRY(ctx, hipMemsetAsync(p->d_winners, 0, sizeof(uint64_t) * (n + 1), ctx->stream));
    if (reasons) HIP_TRY(ctx, hipMemsetAsync(p->d_reason, 0, sizeof(uint32_t) * (n + 1), ctx->stream));
    s->gen++;
    HIP_TRY(ctx, hipMemsetAsync(p->d_step, 0, sizeof(uint32_t), ctx->stream));
    hipEvent_t e0, e1;
    st = record_begin(ctx, &e0, &e1);
    if (st != KG_OK) return st;
    if (windows) {
        // every window places 1..RB_W pods: launch the windows the remaining pods need at least, then look
        uint32_t placed = 0;
        while (placed < n) {
            const uint32_t before = placed;
            const uint32_t windows_min = (n - placed + RB_W - 1) / RB_W;
            if (replay_no_graph()) {  // profiling aid: the same launches, not captured
                for (uint32_t w = 0; w < windows_min; w++) HIP_TRY(ctx, launch_rb_window(p->rb_args, ctx->stream));
            } else {
                for (uint32_t w = 0; w < windows_min; w += RB_R) HIP_TRY(ctx, hipGraphLaunch(p->bexec, ctx->stream));
            }
            HIP_TRY(ctx, hipMemcpyAsync(&placed, p->d_step, sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            if (placed <= before || placed > n) return fail(ctx, KG_DEVICE_ERROR, "window replay stalled at pod %u", placed);
        }
    } else {
        // steps 0..n: step i Assumes pod i-1 and evaluates pod i
        for (uint32_t done = 0; done <= n; done += REPLAY_G) HIP_TRY(ctx, hipGraphLaunch(p->rexec, ctx->stream));
    }
    HIP_TRY(ctx, launch_big_scan(s->d_nodes, s->n, s->d_big + 1, s->d_big, ctx->stream));
    st = record_end(ctx, e0, e1);
    if (st != KG_OK) return st;
    std::vector<uint64_t> w(std::max<uint32_t>(n, 1));
    HIP_TRY(ctx, hipMemcpyAsync(w.data(), p->d_winners, sizeof(uint64_t) * n, hipMemcpyDeviceToHost, ctx->stream));
    if (out_reason && n)
        HIP_TRY(ctx, hipMemcpyAsync(out_reason, p->d_reason, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    for (uint32_t j = 0; j < n; j++) {
        if (out_node) out_node[j] = kg_key_node(w[j]);
        if (out_total) out_total[j] = kg_key_total(w[j]);
    }
    return KG_OK;
}

// Reserve of (pod, node); split != nullptr: the NUMA allocation's per-zone amounts (2 x KG_MAX_ZONES) are returned.
static kg_status assume_impl(kg_snap* s, kg_pods* p, uint32_t pod, uint32_t node, int32_t* out_zone, int64_t* out_split) {
    kg_status st = check_pair(s, p);
    if (st != KG_OK) return st;
    kg_ctx* ctx = s->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (pod >= p->n || node >= s->n) return fail(ctx, KG_INVALID_ARG, "pod %u / node %u out of range", pod, node);
    if (rsv_numa_pair(s, p, pod, node))
        return fail(ctx, KG_UNSUPPORTED, "pod %u on node %u: NUMA / cpuset restore of its reservations", pod, node);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (out_split && !p->d_split) HIP_TRY(ctx, hipMalloc(&p->d_split, sizeof(int64_t) * 2 * KG_MAX_ZONES));
    touch_views(s, node);
    HIP_TRY(ctx, hipMemsetAsync(p->d_aout, 0, sizeof(int32_t) * 2, ctx->stream));
    if (out_split) HIP_TRY(ctx, hipMemsetAsync(p->d_split, 0, sizeof(int64_t) * 2 * KG_MAX_ZONES, ctx->stream));
    if (s->has_cpu)
        HIP_TRY(ctx, launch_cpuset_reserve(s->d_nodes, s->d_zones, s->d_cpu_alloc, s->d_cpu_topos, p->dev, s->kcfg, pod,
                                           s->pos[node], nullptr, nullptr, 0, s->d_pos, s->base, p->n, nullptr, p->d_aout,
                                           ctx->stream));
    HIP_TRY(ctx, launch_assume(s->d_nodes, s->d_zones, p->dev, pod, s->pos[node], -1, 1, s->kcfg, force_exact(), p->d_aout,
                               ctx->stream, out_split ? p->d_split : nullptr));
    s->gen++;
    HIP_TRY(ctx, launch_big_scan(s->d_nodes, s->n, s->d_big + 1, s->d_big, ctx->stream));
    int32_t zone = -1;
    HIP_TRY(ctx, hipMemcpyAsync(&zone, p->d_aout, sizeof(zone), hipMemcpyDeviceToHost, ctx->stream));
    if (out_split)
        HIP_TRY(ctx, hipMemcpyAsync(out_split, p->d_split, sizeof(int64_t) * 2 * KG_MAX_ZONES, hipMemcpyDeviceToHost,
                                    ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (out_zone) *out_zone = zone;
    if (zone_reserve_fails(zone))
        return fail(ctx, KG_RESERVE_FAILED, "Reserve of pod %u on node %u failed: NUMA status 0x%x", pod, node, zone_fail_status(zone));
    return KG_OK;
}

kg_status kg_assume(kg_snap* s, kg_pods* p, uint32_t pod, uint32_t node) { return assume_impl(s, p, pod, node, nullptr, nullptr); }

kg_status kg_assume_numa(kg_snap* s, kg_pods* p, uint32_t pod, uint32_t node, int32_t* out_zone, int64_t* out_zone_amounts) {
    if (!out_zone || !out_zone_amounts) return s && s->ctx ? fail(s->ctx, KG_INVALID_ARG, "null output") : KG_INVALID_ARG;
    return assume_impl(s, p, pod, node, out_zone, out_zone_amounts);
}

static kg_status forget_impl(kg_snap* s, kg_pods* p, uint32_t pod, uint32_t node, int32_t zone, const int64_t* split) {
    kg_status st = check_pair(s, p);
    if (st != KG_OK) return st;
    kg_ctx* ctx = s->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (pod >= p->n || node >= s->n) return fail(ctx, KG_INVALID_ARG, "pod %u / node %u out of range", pod, node);
    const bool multi = zone >= 0x40 && zone < 0x80;
    if (zone >= KG_MAX_ZONES && !(multi && split))
        return fail(ctx, KG_UNSUPPORTED, "Unreserve of a multi-zone NUMA allocation (zone code 0x%x) needs its per-zone "
                                         "amounts (kg_forget_numa)", zone);
    if (cpuset_bound(s, p, pod, node)) return fail(ctx, KG_UNSUPPORTED, "Unreserve of a cpuset allocation");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (multi && !p->d_split) HIP_TRY(ctx, hipMalloc(&p->d_split, sizeof(int64_t) * 2 * KG_MAX_ZONES));
    touch_views(s, node);
    if (multi)
        HIP_TRY(ctx, hipMemcpyAsync(p->d_split, split, sizeof(int64_t) * 2 * KG_MAX_ZONES, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, launch_assume(s->d_nodes, s->d_zones, p->dev, pod, s->pos[node], zone, -1, s->kcfg, force_exact(), nullptr,
                               ctx->stream, multi ? p->d_split : nullptr));
    s->gen++;
    HIP_TRY(ctx, launch_big_scan(s->d_nodes, s->n, s->d_big + 1, s->d_big, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return KG_OK;
}

kg_status kg_forget(kg_snap* s, kg_pods* p, uint32_t pod, uint32_t node, int32_t zone) {
    return forget_impl(s, p, pod, node, zone, nullptr);
}

kg_status kg_forget_numa(kg_snap* s, kg_pods* p, uint32_t pod, uint32_t node, int32_t zone, const int64_t* zone_amounts) {
    if (!zone_amounts) return s && s->ctx ? fail(s->ctx, KG_INVALID_ARG, "null zone amounts") : KG_INVALID_ARG;
    return forget_impl(s, p, pod, node, zone, zone_amounts);
}

static kg_status ext_replay(kg_snap* s, kg_pods* p, int32_t* out_node, int64_t* out_total, uint32_t* out_reason) {
    kg_ctx* ctx = s->ctx;
    if ((s->cfg.plugins & KG_PLUGIN_RSV) && s->n_views && !s->rsv_follow())
        return fail(ctx, KG_UNSUPPORTED, "replay with reservations holding GPUs and no restore inputs "
                                         "(kg_snapshot_upload_rsv_gpu)");
    kg_status st = check_ext(s);
    if (st != KG_OK) return st;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const uint32_t n = p->n;
    const bool exact = force_exact();
    if (rsv_replay(s) && !s->d_rstep) {
        HIP_TRY(ctx, hipMalloc(&s->d_rstep, sizeof(RsvStep) * 3));
        HIP_TRY(ctx, hipMalloc(&s->d_rlist, sizeof(uint64_t) * 2 * 3 * (size_t)std::max<uint32_t>(s->n, 1)));
    }
    if (!p->d_done) HIP_TRY(ctx, hipMalloc(&p->d_done, REPLAY_DONE_WORDS * sizeof(uint32_t)));
    HIP_TRY(ctx, hipMemsetAsync(p->d_done, 0, REPLAY_DONE_WORDS * sizeof(uint32_t), ctx->stream));
    const bool reasons = out_reason != nullptr;
    if (replay_dsum(s, p)) {
        st = devsum_reserve(s, p);
        if (st != KG_OK) return st;
    }
    if (replay_gz(s, p, exact, reasons)) {
        st = gz_reserve(s, p);
        if (st != KG_OK) return st;
    }
    st = ext_replay_graph(s, p, exact, reasons);
    if (st != KG_OK) return st;
    if (rsv_replay(s)) {
        RsvStep z[3];
        for (RsvStep& x : z) x.win = 0, x.pref = ~0ull, x.cnt = 0, x.rmax = 0;
        HIP_TRY(ctx, hipMemcpyAsync(s->d_rstep, z, sizeof(z), hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // z is on this stack
    }
    if (out_reason) HIP_TRY(ctx, hipMemsetAsync(p->d_reason, 0, sizeof(uint32_t) * (n + 1), ctx->stream));
    HIP_TRY(ctx, hipMemsetAsync(p->d_winners, 0, sizeof(uint64_t) * (n + 1), ctx->stream));
    HIP_TRY(ctx, hipMemsetAsync(p->d_minors, 0, sizeof(uint32_t) * (n + 1), ctx->stream));
    s->gen++;
    HIP_TRY(ctx, hipMemsetAsync(p->d_buckets, 0, sizeof(uint64_t) * REPLAY_BUCKET_WORDS, ctx->stream));
    HIP_TRY(ctx, hipMemsetAsync(p->d_step, 0, sizeof(uint32_t), ctx->stream));
    hipEvent_t e0, e1;
    st = record_begin(ctx, &e0, &e1);
    if (st != KG_OK) return st;
    // the tables of the replay's starting state (inside the timed region)
    if (replay_dsum(s, p))
        HIP_TRY(ctx, launch_dev_sum(s->d_nodes, s->d_zones, s->d_dev, s->n, s->n0, p->d_dclass, p->n_dclass, s->kcfg,
                                    s->ext_dev(), p->d_devsum, spec_cls_max(p), ctx->stream));
    if (replay_gz(s, p, exact, reasons))
        HIP_TRY(ctx, launch_gpu_zone_sum(s->d_nodes, s->d_zones, s->d_dev, s->n, s->n0, p->d_dclass, p->n_dclass, s->kcfg,
                                         s->ext_dev(), p->d_gz, ctx->stream));
    for (uint32_t done = 0; done <= n; done += REPLAY_G) HIP_TRY(ctx, hipGraphLaunch(p->xexec, ctx->stream));
    HIP_TRY(ctx, launch_big_scan(s->d_nodes, s->n, s->d_big + 1, s->d_big, ctx->stream));
    st = record_end(ctx, e0, e1);
    if (st != KG_OK) return st;
    if ((s->cfg.plugins & KG_PLUGIN_RSV) && s->n_views) s->views_on_device = true;  // Reservation.Reserve ran there
    if ((s->cfg.plugins & KG_PLUGIN_QUOTA) && s->n_quotas) {
        // the final state sits in buffer n & 1; make both buffers agree again
        const size_t qb = sizeof(QuotaState) * s->n_quotas;
        QuotaState* fin = s->d_qstate + (size_t)(n & 1u) * s->n_quotas;
        QuotaState* other = s->d_qstate + (size_t)((n & 1u) ^ 1u) * s->n_quotas;
        HIP_TRY(ctx, hipMemcpyAsync(other, fin, qb, hipMemcpyDeviceToDevice, ctx->stream));
    }
    std::vector<uint64_t> w(std::max<uint32_t>(n, 1));
    HIP_TRY(ctx, hipMemcpyAsync(w.data(), p->d_winners, sizeof(uint64_t) * n, hipMemcpyDeviceToHost, ctx->stream));
    if (out_reason && n)
        HIP_TRY(ctx, hipMemcpyAsync(out_reason, p->d_reason, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    for (uint32_t j = 0; j < n; j++) {
        if (out_node) out_node[j] = kg_key_node(w[j]);
        if (out_total) out_total[j] = kg_key_total(w[j]);
    }
    return KG_OK;
}

kg_status kg_replay_minors(kg_pods* p, uint32_t* out) {
    if (!p || !out) return KG_INVALID_ARG;
    kg_ctx* ctx = p->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (p->n) HIP_TRY(ctx, hipMemcpyAsync(out, p->d_minors, sizeof(uint32_t) * p->n, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return KG_OK;
}

static kg_status assume_ext(kg_snap* s, kg_pods* p, uint32_t pod, uint32_t node, int32_t zone, uint32_t minors,
                            int64_t sign, int32_t* out_zone, uint32_t* out_minors) {
    kg_status st = check_pair(s, p);
    if (st != KG_OK) return st;
    kg_ctx* ctx = s->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (pod >= p->n || node >= s->n) return fail(ctx, KG_INVALID_ARG, "pod %u / node %u out of range", pod, node);
    st = check_ext(s);
    if (st != KG_OK) return st;
    if (sign > 0 && rsv_numa_pair(s, p, pod, node))
        return fail(ctx, KG_UNSUPPORTED, "pod %u on node %u: NUMA / cpuset restore of its reservations", pod, node);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    // a Reserve follows Reservation.Reserve on the device's views (k_ext_assume, rsv_reserve_dev) unless a reservation
    // holds GPUs; an Unreserve does not know the reservation: the node's views are stale then
    if (sign < 0 || !s->rsv_follow() || !(s->cfg.plugins & KG_PLUGIN_RSV)) touch_views(s, node);
    else if (s->n_views && node < s->cls_mask.size() && s->cls_mask[node]) s->views_on_device = true;
    HIP_TRY(ctx, hipMemsetAsync(p->d_aout, 0, sizeof(int32_t) * 4, ctx->stream));
    if (sign > 0 && s->has_cpu) {
        // the pair evaluated before the cpuset take changes the counts it reads (zone and minors preset in d_aout)
        HIP_TRY(ctx, launch_ext_assume(s->d_nodes, s->d_zones, s->d_dev, s->ext_dev(), p->dev, pod, s->pos[node], zone,
                                       minors, 0, s->kcfg, force_exact(), p->d_aout, ctx->stream));
        HIP_TRY(ctx, launch_cpuset_reserve(s->d_nodes, s->d_zones, s->d_cpu_alloc, s->d_cpu_topos, p->dev, s->kcfg, pod,
                                           s->pos[node], nullptr, nullptr, 0, s->d_pos, s->base, p->n, nullptr, p->d_aout,
                                           ctx->stream));
    }
    HIP_TRY(ctx, launch_ext_assume(s->d_nodes, s->d_zones, s->d_dev, s->ext_dev(), p->dev, pod, s->pos[node], zone, minors,
                                   sign, s->kcfg, force_exact(), p->d_aout, ctx->stream, nullptr, sign > 0));
    s->gen++;
    HIP_TRY(ctx, launch_big_scan(s->d_nodes, s->n, s->d_big + 1, s->d_big, ctx->stream));
    int32_t o[2] = {-1, 0};
    HIP_TRY(ctx, hipMemcpyAsync(o, p->d_aout, sizeof(o), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (out_zone) *out_zone = o[0];
    if (out_minors) *out_minors = (uint32_t)o[1];
    if (sign > 0 && zone_reserve_fails(o[0]))
        return fail(ctx, KG_RESERVE_FAILED, "Reserve of pod %u on node %u failed: NUMA status 0x%x", pod, node, zone_fail_status(o[0]));
    return KG_OK;
}

kg_status kg_assume_ext(kg_snap* s, kg_pods* p, uint32_t pod, uint32_t node, int32_t* out_zone, uint32_t* out_minors) {
    return assume_ext(s, p, pod, node, -1, 0, 1, out_zone, out_minors);
}

kg_status kg_forget_ext(kg_snap* s, kg_pods* p, uint32_t pod, uint32_t node, int32_t zone, uint32_t minors) {
    if (s && zone >= KG_MAX_ZONES)
        return fail(s->ctx, KG_UNSUPPORTED, "Unreserve of a multi-zone NUMA allocation (zone code 0x%x)", zone);
    if (s && p && node < s->n && cpuset_bound(s, p, pod, node))
        return fail(s->ctx, KG_UNSUPPORTED, "Unreserve of a cpuset allocation");
    return assume_ext(s, p, pod, node, zone, minors, -1, nullptr, nullptr);
}

// ---- Reserve / Unreserve with the allocation record -------------------------------------------------------------

kg_status kg_reserve(kg_snap* s, kg_pods* p, uint32_t pod, uint32_t node, kg_reserve_record* out) {
    kg_status st = check_pair(s, p);
    if (st != KG_OK) return st;
    kg_ctx* ctx = s->ctx;
    if (!out) return fail(ctx, KG_INVALID_ARG, "null record");
    std::lock_guard<std::mutex> g(ctx->mu);
    if (pod >= p->n || node >= s->n) return fail(ctx, KG_INVALID_ARG, "pod %u / node %u out of range", pod, node);
    if (rsv_numa_pair(s, p, pod, node))
        return fail(ctx, KG_UNSUPPORTED, "pod %u on node %u: NUMA / cpuset restore of its reservations", pod, node);
    if (s->ext()) {
        st = check_ext(s);
        if (st != KG_OK) return st;
    }
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (!p->d_rec) HIP_TRY(ctx, hipMalloc(&p->d_rec, sizeof(uint64_t) * 16));
    // Reservation.Reserve follows the node's views on the device unless a reservation there holds GPUs (their DeviceShare
    // restore tables follow the reserve pods' allocations: the caller re-uploads the node's views)
    const bool rsv = (s->cfg.plugins & KG_PLUGIN_RSV) && s->n_views && s->rsv_follow();
    if (!rsv) touch_views(s, node);
    else if (node < s->cls_mask.size() && s->cls_mask[node]) s->views_on_device = true;
    HIP_TRY(ctx, hipMemsetAsync(p->d_aout, 0, sizeof(int32_t) * 4, ctx->stream));
    HIP_TRY(ctx, hipMemsetAsync(p->d_rec, 0, sizeof(uint64_t) * 16, ctx->stream));
    const ExtDev e = s->ext_dev();
    const uint32_t rec = s->pos[node];
    if (s->has_cpu) {
        // the pair evaluated before the cpuset take changes the counts it reads (zone, minors, reservation preset)
        HIP_TRY(ctx, launch_ext_assume(s->d_nodes, s->d_zones, s->d_dev, e, p->dev, pod, rec, -1, 0, 0, s->kcfg,
                                       force_exact(), p->d_aout, ctx->stream, nullptr, rsv));
        HIP_TRY(ctx, launch_cpuset_reserve(s->d_nodes, s->d_zones, s->d_cpu_alloc, s->d_cpu_topos, p->dev, s->kcfg, pod, rec,
                                           nullptr, nullptr, 0, s->d_pos, s->base, p->n, nullptr, p->d_aout, ctx->stream, 0,
                                           p->d_rec));
    }
    HIP_TRY(ctx, launch_ext_assume(s->d_nodes, s->d_zones, s->d_dev, e, p->dev, pod, rec, -1, 0, 1, s->kcfg, force_exact(),
                                   p->d_aout, ctx->stream, reinterpret_cast<int64_t*>(p->d_rec + 4), rsv));
    s->gen++;
    HIP_TRY(ctx, launch_big_scan(s->d_nodes, s->n, s->d_big + 1, s->d_big, ctx->stream));
    int32_t o[4] = {-1, 0, -1, -1};
    uint64_t r[16];
    HIP_TRY(ctx, hipMemcpyAsync(o, p->d_aout, sizeof(o), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(r, p->d_rec, sizeof(r), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    std::memset(out, 0, sizeof(*out));
    out->numa_zone = o[0];
    out->rsv_rid = -1;
    if (zone_reserve_fails(o[0]))
        return fail(ctx, KG_RESERVE_FAILED, "Reserve of pod %u on node %u failed: NUMA status 0x%x", pod, node, zone_fail_status(o[0]));
    out->gpu_minors = (uint32_t)o[1];
    out->rsv_rid = rsv ? o[3] : -1;
    for (int w = 0; w < 4; w++) out->cpus[w] = r[w];
    for (int z = 0; z < 2 * KG_MAX_ZONES; z++) out->zone_amounts[z] = (int64_t)r[4 + z];
    if (r[0] | r[1] | r[2] | r[3]) out->flags |= KG_RECORD_CPUSET;
    if (s->ext() && (s->cfg.plugins & KG_PLUGIN_QUOTA) && s->n_quotas) out->flags |= KG_RECORD_QUOTA;
    return KG_OK;
}

kg_status kg_unreserve(kg_snap* s, kg_pods* p, uint32_t pod, uint32_t node, kg_reserve_record* rec) {
    kg_status st = check_pair(s, p);
    if (st != KG_OK) return st;
    kg_ctx* ctx = s->ctx;
    if (!rec) return fail(ctx, KG_INVALID_ARG, "null record");
    std::lock_guard<std::mutex> g(ctx->mu);
    if (pod >= p->n || node >= s->n) return fail(ctx, KG_INVALID_ARG, "pod %u / node %u out of range", pod, node);
    if (zone_reserve_fails(rec->numa_zone)) return fail(ctx, KG_INVALID_ARG, "the record's Reserve failed: nothing to give back");
    if (rec->flags & KG_RECORD_RELEASED) return fail(ctx, KG_INVALID_ARG, "the record was already given back");
    if (s->ext()) {
        st = check_ext(s);
        if (st != KG_OK) return st;
    }
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (!p->d_rec) HIP_TRY(ctx, hipMalloc(&p->d_rec, sizeof(uint64_t) * 16));
    const bool rsv = (s->cfg.plugins & KG_PLUGIN_RSV) && s->n_views && s->rsv_follow();
    if (!rsv) touch_views(s, node);
    else if (node < s->cls_mask.size() && s->cls_mask[node]) s->views_on_device = true;
    uint64_t r[16] = {0};
    for (int w = 0; w < 4; w++) r[w] = s->has_cpu ? rec->cpus[w] : 0;
    bool any = false;
    for (int z = 0; z < 2 * KG_MAX_ZONES; z++) {
        r[4 + z] = (uint64_t)rec->zone_amounts[z];
        any = any || rec->zone_amounts[z] != 0;
    }
    HIP_TRY(ctx, hipMemcpyAsync(p->d_rec, r, sizeof(r), hipMemcpyHostToDevice, ctx->stream));
    // the NUMA allocation is given back by its recorded per-zone amounts (zone code 0x40 | every zone)
    const int32_t zone = rec->numa_zone < 0 ? -1 : any ? 0x4F : rec->numa_zone;
    HIP_TRY(ctx, launch_ext_assume(s->d_nodes, s->d_zones, s->d_dev, s->ext_dev(), p->dev, pod, s->pos[node], zone,
                                   rec->gpu_minors, -1, s->kcfg, force_exact(), nullptr, ctx->stream,
                                   reinterpret_cast<int64_t*>(p->d_rec + 4), rsv, rec->rsv_rid, s->d_cpu_alloc,
                                   s->d_cpu_topos, (rec->flags & KG_RECORD_CPUSET) ? p->d_rec : nullptr));
    s->gen++;
    HIP_TRY(ctx, launch_big_scan(s->d_nodes, s->n, s->d_big + 1, s->d_big, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // r is on this stack
    rec->flags |= KG_RECORD_RELEASED;
    return KG_OK;
}

// ---- cpuset accumulator (batch entry) -----------------------------------------------------------------

static const char* cpu_topo_problem(const kg_cpu_topo& t) {
    if (t.n_cpus > KG_MAX_CPUS) return "more than 256 CPUs";
    if (t.n_nodes > 8 || t.n_sockets > 8) return "more than 8 NUMA nodes or sockets";
    int per_core[KG_MAX_CPUS] = {0};
    for (int c = 0; c < t.n_cpus; c++) {
        if (t.core[c] >= t.n_cores || t.numa[c] >= t.n_nodes || t.socket[c] >= t.n_sockets) return "id out of range";
        if (++per_core[t.core[c]] > 8) return "more than 8 CPUs per core";
    }
    return nullptr;
}

kg_status kg_cpuset_take(kg_ctx* ctx, const kg_cpu_topo* topos, uint32_t n_topos, const kg_cpu_alloc* allocs,
                         uint32_t n_allocs, const kg_cpuset_request* reqs, uint32_t n, uint64_t* out, int32_t* rc) {
    if (!ctx || (n && (!topos || !reqs || !out || !rc))) return KG_INVALID_ARG;
    std::lock_guard<std::mutex> g(ctx->mu);
    for (uint32_t t = 0; t < n_topos; t++)
        if (const char* why = cpu_topo_problem(topos[t])) return fail(ctx, KG_UNSUPPORTED, "CPU topology %u: %s", t, why);
    for (uint32_t i = 0; i < n; i++) {
        const kg_cpuset_request& q = reqs[i];
        if (q.topo >= n_topos || (q.alloc >= 0 && (!allocs || (uint32_t)q.alloc >= n_allocs)))
            return fail(ctx, KG_INVALID_ARG, "request %u: topology / allocation index out of range", i);
        if (q.needed < 0 || q.needed > KG_MAX_CPUS || q.max_ref < 1 || q.bind < 0 || q.bind > 2 || q.excl < 0 ||
            q.excl > 2 || q.strategy < 0 || q.strategy > 1)
            return fail(ctx, KG_INVALID_ARG, "request %u: bad arguments", i);
    }
    if (n == 0) return KG_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const size_t bt = sizeof(kg_cpu_topo) * n_topos, ba = sizeof(kg_cpu_alloc) * (allocs ? n_allocs : 0),
                 bq = sizeof(kg_cpuset_request) * n, bo = sizeof(uint64_t) * 4 * n, br = sizeof(int32_t) * n;
    uint8_t* d = nullptr;
    HIP_TRY(ctx, hipMalloc(&d, bt + ba + bq + bo + br + 64));
    kg_status st = KG_OK;
    uint8_t* p = d;
    auto* d_topo = reinterpret_cast<kg_cpu_topo*>(p);
    p += bt;
    auto* d_alloc = ba ? reinterpret_cast<kg_cpu_alloc*>(p) : nullptr;
    p += ba;
    p = reinterpret_cast<uint8_t*>((reinterpret_cast<uintptr_t>(p) + 7) & ~(uintptr_t)7);
    auto* d_req = reinterpret_cast<kg_cpuset_request*>(p);
    p += bq;
    auto* d_out = reinterpret_cast<uint64_t*>(p);
    p += bo;
    auto* d_rc = reinterpret_cast<int32_t*>(p);
    hipError_t e = hipMemcpyAsync(d_topo, topos, bt, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess && ba) e = hipMemcpyAsync(d_alloc, allocs, ba, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(d_req, reqs, bq, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = launch_cpuset_take(d_topo, d_alloc, d_req, n, d_out, d_rc, ctx->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(out, d_out, bo, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(rc, d_rc, br, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) st = fail(ctx, KG_DEVICE_ERROR, "kg_cpuset_take: %s", hipGetErrorString(e));
    hipFree(d);
    return st;
}

// ---- checkpoint / rollback and the inline batch cycle ------------------------------------------------

static kg_status save_state(kg_snap* s, kg_snap::Saved& k) {
    kg_ctx* ctx = s->ctx;
    const size_t n = std::max<uint32_t>(s->n, 1);
    if (!k.nodes) {
        HIP_TRY(ctx, hipMalloc(&k.nodes, sizeof(NodeRec) * n));
        HIP_TRY(ctx, hipMalloc(&k.zones, sizeof(ZoneRec) * n));
        if (s->d_dev) HIP_TRY(ctx, hipMalloc(&k.dev, sizeof(DevRec) * n));
    }
    if (s->d_cpu_alloc && !k.cpu) HIP_TRY(ctx, hipMalloc(&k.cpu, sizeof(kg_cpu_alloc) * n));
    if (k.nq < s->n_quotas || (s->n_quotas && !k.q)) {
        hipFree(k.q);
        k.q = nullptr;
        HIP_TRY(ctx, hipMalloc(&k.q, sizeof(QuotaState) * 2 * (size_t)s->n_quotas));
    }
    k.nq = s->n_quotas;
    HIP_TRY(ctx, hipMemcpyAsync(k.nodes, s->d_nodes, sizeof(NodeRec) * s->n, hipMemcpyDeviceToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(k.zones, s->d_zones, sizeof(ZoneRec) * s->n, hipMemcpyDeviceToDevice, ctx->stream));
    if (s->d_dev) HIP_TRY(ctx, hipMemcpyAsync(k.dev, s->d_dev, sizeof(DevRec) * s->n, hipMemcpyDeviceToDevice, ctx->stream));
    if (s->d_cpu_alloc)
        HIP_TRY(ctx, hipMemcpyAsync(k.cpu, s->d_cpu_alloc, sizeof(kg_cpu_alloc) * s->n, hipMemcpyDeviceToDevice, ctx->stream));
    if (s->n_quotas && s->d_qstate)
        HIP_TRY(ctx, hipMemcpyAsync(k.q, s->d_qstate, sizeof(QuotaState) * 2 * (size_t)s->n_quotas, hipMemcpyDeviceToDevice,
                                    ctx->stream));
    const uint32_t ni = (uint32_t)s->h_infos.size();
    if (s->n_views && (k.nv < s->n_views || k.ni < ni || !k.views)) {
        hipFree(k.views);
        hipFree(k.infos);
        k.views = nullptr;
        k.infos = nullptr;
        HIP_TRY(ctx, hipMalloc(&k.views, sizeof(RsvView) * s->n_views));
        HIP_TRY(ctx, hipMalloc(&k.infos, sizeof(RsvInfo) * std::max<uint32_t>(ni, 1)));
    }
    k.nv = s->n_views;
    k.ni = ni;
    if (s->n_views) {
        HIP_TRY(ctx, hipMemcpyAsync(k.views, s->d_views, sizeof(RsvView) * s->n_views, hipMemcpyDeviceToDevice, ctx->stream));
        if (ni) HIP_TRY(ctx, hipMemcpyAsync(k.infos, s->d_infos, sizeof(RsvInfo) * ni, hipMemcpyDeviceToDevice, ctx->stream));
    }
    if (s->gpu_raw) {  // the GPU restore tables and inputs a Reserve rebuilds
        if (k.nrd < s->n_rdev || k.ngn < s->n_gnodes || k.ngr < s->n_grsv || !k.rdev) {
            for (void* b : {(void*)k.rdev, (void*)k.gnodes, (void*)k.grsv}) hipFree(b);
            k.rdev = nullptr, k.gnodes = nullptr, k.grsv = nullptr;
            HIP_TRY(ctx, hipMalloc(&k.rdev, sizeof(DevRec) * std::max<uint32_t>(s->n_rdev, 1)));
            HIP_TRY(ctx, hipMalloc(&k.gnodes, sizeof(GpuRawNode) * std::max<uint32_t>(s->n_gnodes, 1)));
            HIP_TRY(ctx, hipMalloc(&k.grsv, sizeof(GpuRawRsv) * std::max<uint32_t>(s->n_grsv, 1)));
        }
        k.nrd = s->n_rdev, k.ngn = s->n_gnodes, k.ngr = s->n_grsv;
        if (s->n_rdev) HIP_TRY(ctx, hipMemcpyAsync(k.rdev, s->d_rdev, sizeof(DevRec) * s->n_rdev, hipMemcpyDeviceToDevice, ctx->stream));
        if (s->n_gnodes)
            HIP_TRY(ctx, hipMemcpyAsync(k.gnodes, s->d_gnodes, sizeof(GpuRawNode) * s->n_gnodes, hipMemcpyDeviceToDevice, ctx->stream));
        if (s->n_grsv)
            HIP_TRY(ctx, hipMemcpyAsync(k.grsv, s->d_grsv, sizeof(GpuRawRsv) * s->n_grsv, hipMemcpyDeviceToDevice, ctx->stream));
    } else {
        k.nrd = k.ngn = k.ngr = 0;
    }
    k.views_on_device = s->views_on_device;
    k.views_stale = s->views_stale;
    k.stale = s->stale;
    k.n_stale = s->n_stale;
    k.valid = true;
    return KG_OK;
}

static kg_status restore_state(kg_snap* s, kg_snap::Saved& k) {
    kg_ctx* ctx = s->ctx;
    HIP_TRY(ctx, hipMemcpyAsync(s->d_nodes, k.nodes, sizeof(NodeRec) * s->n, hipMemcpyDeviceToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(s->d_zones, k.zones, sizeof(ZoneRec) * s->n, hipMemcpyDeviceToDevice, ctx->stream));
    if (s->d_dev) HIP_TRY(ctx, hipMemcpyAsync(s->d_dev, k.dev, sizeof(DevRec) * s->n, hipMemcpyDeviceToDevice, ctx->stream));
    if (s->d_cpu_alloc && k.cpu)
        HIP_TRY(ctx, hipMemcpyAsync(s->d_cpu_alloc, k.cpu, sizeof(kg_cpu_alloc) * s->n, hipMemcpyDeviceToDevice, ctx->stream));
    if (k.nq && s->d_qstate)
        HIP_TRY(ctx, hipMemcpyAsync(s->d_qstate, k.q, sizeof(QuotaState) * 2 * (size_t)k.nq, hipMemcpyDeviceToDevice,
                                    ctx->stream));
    HIP_TRY(ctx, launch_big_scan(s->d_nodes, s->n, s->d_big + 1, s->d_big, ctx->stream));
    if (k.nv && k.nv == s->n_views && k.views) {
        HIP_TRY(ctx, hipMemcpyAsync(s->d_views, k.views, sizeof(RsvView) * k.nv, hipMemcpyDeviceToDevice, ctx->stream));
        if (k.ni) HIP_TRY(ctx, hipMemcpyAsync(s->d_infos, k.infos, sizeof(RsvInfo) * k.ni, hipMemcpyDeviceToDevice, ctx->stream));
        s->views_on_device = k.views_on_device;
    }
    if (s->gpu_raw && k.rdev && k.nrd == s->n_rdev && k.ngn == s->n_gnodes && k.ngr == s->n_grsv) {
        if (k.nrd) HIP_TRY(ctx, hipMemcpyAsync(s->d_rdev, k.rdev, sizeof(DevRec) * k.nrd, hipMemcpyDeviceToDevice, ctx->stream));
        if (k.ngn)
            HIP_TRY(ctx, hipMemcpyAsync(s->d_gnodes, k.gnodes, sizeof(GpuRawNode) * k.ngn, hipMemcpyDeviceToDevice, ctx->stream));
        if (k.ngr) HIP_TRY(ctx, hipMemcpyAsync(s->d_grsv, k.grsv, sizeof(GpuRawRsv) * k.ngr, hipMemcpyDeviceToDevice, ctx->stream));
    }
    s->views_stale = k.views_stale;
    s->stale = k.stale;
    s->n_stale = k.n_stale;
    s->gen++;
    return KG_OK;
}

kg_status kg_snapshot_checkpoint(kg_snap* s) {
    if (!s) return KG_INVALID_ARG;
    kg_ctx* ctx = s->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (!s->uploaded) return fail(ctx, KG_INVALID_ARG, "snapshot not uploaded");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    kg_status st = save_state(s, s->ck);
    if (st != KG_OK) return st;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    s->gen++;
    return KG_OK;
}

kg_status kg_snapshot_rollback(kg_snap* s) {
    if (!s) return KG_INVALID_ARG;
    kg_ctx* ctx = s->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (!s->ck.valid)
        return fail(ctx, KG_INVALID_ARG, "no checkpoint (none taken, or the snapshot / its tables were re-uploaded since)");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    kg_status st = restore_state(s, s->ck);
    if (st != KG_OK) return st;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return KG_OK;
}

kg_status kg_batch_schedule(kg_snap* s, kg_pods* p, const int32_t* plan_node, uint32_t* out_result, uint32_t* out_status,
                            int32_t* out_zone, uint32_t* out_minors) {
    kg_status st = check_pair(s, p);
    if (st != KG_OK) return st;
    kg_ctx* ctx = s->ctx;
    if ((!plan_node || !out_result || !out_status) && p->n) return fail(ctx, KG_INVALID_ARG, "null plan / result buffer");
    std::lock_guard<std::mutex> g(ctx->mu);
    if ((s->cfg.plugins & KG_PLUGIN_RSV) && s->n_views && !s->rsv_follow())
        return fail(ctx, KG_UNSUPPORTED, "batch schedule with reservations holding GPUs and no restore inputs "
                                         "(kg_snapshot_upload_rsv_gpu)");
    if (s->ext()) {
        st = check_ext(s);
        if (st != KG_OK) return st;
    }
    const uint32_t n = p->n;
    for (uint32_t j = 0; j < n; j++)
        if (plan_node[j] >= (int32_t)s->n) return fail(ctx, KG_INVALID_ARG, "pod %u: planned node %d >= %u", j, plan_node[j], s->n);
    auto set_all = [&](uint32_t code) {
        for (uint32_t j = 0; j < n; j++) {
            out_result[j] = code;
            out_status[j] = 0;
            if (out_zone) out_zone[j] = -1;
            if (out_minors) out_minors[j] = 0;
        }
    };
    for (uint32_t j = 0; j < n; j++)
        if (plan_node[j] < 0) {  // "batch schedule plan missing node for pod": nothing is assumed
            set_all(KG_BATCH_NO_PLAN);
            return KG_OK;
        }
    if (n == 0) return KG_OK;
    // podRequestsByNode: groups in order of first appearance, each in batch order
    std::vector<uint32_t> gid(s->n, UINT32_MAX), begin, rec, count;
    for (uint32_t j = 0; j < n; j++) {
        uint32_t& x = gid[plan_node[j]];
        if (x == UINT32_MAX) {
            x = (uint32_t)rec.size();
            rec.push_back(s->pos[plan_node[j]]);
            count.push_back(0);
        }
        count[x]++;
    }
    const uint32_t G = (uint32_t)rec.size();
    begin.assign(G + 1, 0);
    for (uint32_t q = 0; q < G; q++) begin[q + 1] = begin[q] + count[q];
    std::vector<uint32_t> fill(begin.begin(), begin.end() - 1), order(n);
    for (uint32_t j = 0; j < n; j++) order[fill[gid[plan_node[j]]]++] = j;
    // device scratch: [begin G+1][pods n][rec G] + outputs [result n][status n][zone n][minors n]
    const size_t words = (size_t)G + 1 + n + G + 4 * (size_t)n;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (!p->d_batch) HIP_TRY(ctx, hipMalloc(&p->d_batch, sizeof(uint32_t) * (7 * (size_t)p->cap + 1)));
    uint32_t* d = p->d_batch;
    if (words > 7 * (size_t)p->cap + 1) return fail(ctx, KG_INVALID_ARG, "batch scratch");
    std::vector<uint32_t> h(G + 1 + n + G);
    std::copy(begin.begin(), begin.end(), h.begin());
    std::copy(order.begin(), order.end(), h.begin() + G + 1);
    std::copy(rec.begin(), rec.end(), h.begin() + G + 1 + n);
    uint32_t* d_res = d + G + 1 + n + G;
    HIP_TRY(ctx, hipMemcpyAsync(d, h.data(), sizeof(uint32_t) * h.size(), hipMemcpyHostToDevice, ctx->stream));
    st = save_state(s, s->bk);  // CleanupAssumedPods restores this
    if (st != KG_OK) return st;
    hipEvent_t e0, e1;
    st = record_begin(ctx, &e0, &e1);
    if (st != KG_OK) return st;
    const bool cs = cpuset_active(s, p);  // cpuset-binding pods: the cooperative cycle takes their CPUs on the device
    HIP_TRY(ctx, launch_batch(s->d_nodes, s->d_zones, s->d_dev, s->ext_dev(), p->dev, d, d + G + 1, d + G + 1 + n, G, s->ext(),
                              s->kcfg, force_exact(), d_res, d_res + n, (int32_t*)(d_res + 2 * n), d_res + 3 * n, ctx->stream,
                              cs ? s->d_cpu_alloc : nullptr, cs ? s->d_cpu_topos : nullptr));
    st = record_end(ctx, e0, e1);
    if (st != KG_OK) return st;
    std::vector<uint32_t> out(4 * (size_t)n);
    HIP_TRY(ctx, hipMemcpyAsync(out.data(), d_res, sizeof(uint32_t) * 4 * n, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    s->gen++;
    bool failed = false, unsup = false;
    for (uint32_t j = 0; j < n; j++) {
        failed |= out[j] != KG_BATCH_ASSUMED;
        unsup |= (out[n + j] & KG_ST_UNSUPPORTED) != 0;
    }
    if (failed) {  // the job failed: Unreserve + ForgetPod every assumed pod
        st = restore_state(s, s->bk);
        if (st != KG_OK) return st;
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        for (uint32_t j = 0; j < n; j++)
            if (out[j] == KG_BATCH_ASSUMED) out[j] = KG_BATCH_ROLLED_BACK;
    } else {
        HIP_TRY(ctx, launch_big_scan(s->d_nodes, s->n, s->d_big + 1, s->d_big, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        if ((s->cfg.plugins & KG_PLUGIN_RSV) && s->n_views) s->views_on_device = true;  // Reservation.Reserve ran there
    }
    s->bk.valid = false;
    for (uint32_t j = 0; j < n; j++) {
        out_result[j] = out[j];
        out_status[j] = out[n + j];
        if (out_zone) out_zone[j] = (int32_t)out[2 * (size_t)n + j];
        if (out_minors) out_minors[j] = out[3 * (size_t)n + j];
    }
    if (unsup) return fail(ctx, KG_UNSUPPORTED, "a pod of the plan needs the host path on its planned node");
    return KG_OK;
}

kg_status kg_snapshot_upload_quotas(kg_snap* s, const kg_quota_columns* c, uint32_t nq) {
    if (!s || (!c && nq)) return KG_INVALID_ARG;
    kg_ctx* ctx = s->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    std::vector<QuotaLim> lim(std::max<uint32_t>(nq, 1));
    std::vector<QuotaState> qs(2 * (size_t)std::max<uint32_t>(nq, 1));
    for (uint32_t q = 0; q < nq; q++) {
        QuotaLim& L = lim[q];
        QuotaState& S = qs[q];
        std::memset(&L, 0, sizeof(L));
        std::memset(&S, 0, sizeof(S));
        for (int r = 0; r < QUOTA_R; r++) {
            const size_t x = (size_t)q * QUOTA_R + r;
            L.limit[r] = c->used_limit ? c->used_limit[x] : 0;
            L.min[r] = c->min ? c->min[x] : 0;
            S.used[r] = c->used ? c->used[x] : 0;
            S.np_used[r] = c->np_used ? c->np_used[x] : 0;
        }
        L.limit_keys = c->limit_keys ? c->limit_keys[q] : 0u;
        L.min_keys = c->min_keys ? c->min_keys[q] : 0u;
        S.used_keys = c->used_keys ? c->used_keys[q] : 0u;
        S.np_keys = c->np_used_keys ? c->np_used_keys[q] : 0u;
        qs[nq + q] = S;
    }
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    s->gen++;
    hipFree(s->d_qlim);
    hipFree(s->d_qstate);
    s->d_qlim = nullptr;
    s->d_qstate = nullptr;
    HIP_TRY(ctx, hipMalloc(&s->d_qlim, sizeof(QuotaLim) * lim.size()));
    HIP_TRY(ctx, hipMalloc(&s->d_qstate, sizeof(QuotaState) * qs.size()));
    HIP_TRY(ctx, hipMemcpyAsync(s->d_qlim, lim.data(), sizeof(QuotaLim) * lim.size(), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(s->d_qstate, qs.data(), sizeof(QuotaState) * qs.size(), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    s->n_quotas = nq;
    s->invalidate_saved();
    return KG_OK;
}

kg_status kg_snapshot_read_quotas(kg_snap* s, int64_t* used, uint32_t* used_keys, int64_t* np_used, uint32_t* np_keys) {
    if (!s) return KG_INVALID_ARG;
    kg_ctx* ctx = s->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (!s->n_quotas) return KG_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    std::vector<QuotaState> qs(s->n_quotas);
    HIP_TRY(ctx, hipMemcpyAsync(qs.data(), s->d_qstate, sizeof(QuotaState) * s->n_quotas, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    for (uint32_t q = 0; q < s->n_quotas; q++) {
        for (int r = 0; r < QUOTA_R; r++) {
            if (used) used[(size_t)q * QUOTA_R + r] = qs[q].used[r];
            if (np_used) np_used[(size_t)q * QUOTA_R + r] = qs[q].np_used[r];
        }
        if (used_keys) used_keys[q] = qs[q].used_keys;
        if (np_keys) np_keys[q] = qs[q].np_keys;
    }
    return KG_OK;
}

// After Reservation.Reserve ran on the device (kg_replay / kg_assume_ext), bring the host copies of the views and
// reservations up to date (caller holds the lock)
static kg_status sync_views_from_device(kg_snap* s) {
    if (!s->views_on_device || !s->n_views) return KG_OK;
    kg_ctx* ctx = s->ctx;
    std::vector<RsvView> dv(s->n_views);
    std::vector<RsvInfo> di(s->h_infos.size());
    HIP_TRY(ctx, hipMemcpyAsync(dv.data(), s->d_views, sizeof(RsvView) * dv.size(), hipMemcpyDeviceToHost, ctx->stream));
    if (!di.empty())
        HIP_TRY(ctx, hipMemcpyAsync(di.data(), s->d_infos, sizeof(RsvInfo) * di.size(), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    for (uint32_t t = 0; t < s->n_views && t < s->view_order.size(); t++) {
        kg_rsv_view& h = s->h_views[s->view_order[t]];
        for (int k = 0; k < RSV_R; k++) {
            h.req[k] = dv[t].req[k];
            h.pod_requested[k] = dv[t].pod_requested[k];
            h.r_allocated[k] = dv[t].r_allocated[k];
        }
        h.nz_cpu = dv[t].nz_cpu;
        h.nz_mem = dv[t].nz_mem;
        h.num_pods = dv[t].num_pods;
    }
    for (size_t t = 0; t < di.size(); t++) {
        kg_rsv_info& h = s->h_infos[t];
        for (int k = 0; k < RSV_R; k++) h.allocated[k] = di[t].allocated[k];
        h.allocated_pods = di[t].allocated_pods;
        h.allocated_keys = di[t].allocated_keys;
    }
    // the GPU restore tables a Reserve into a node with GPU-holding reservations rebuilt (gpu_restore_rebuild): a later
    // kg_snapshot_update_views keeps the other nodes' tables from these copies
    if (s->gpu_raw && s->d_rdev && s->n_rdev && s->h_rdevs.size() == s->n_rdev) {
        HIP_TRY(ctx, hipMemcpyAsync(s->h_rdevs.data(), s->d_rdev, sizeof(DevRec) * s->n_rdev, hipMemcpyDeviceToHost,
                                    ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    s->views_on_device = false;
    return KG_OK;
}

kg_status kg_snapshot_read_reservations(kg_snap* s, kg_rsv_view* views, uint32_t n_views, kg_rsv_info* infos,
                                        uint32_t n_infos) {
    if (!s) return KG_INVALID_ARG;
    kg_ctx* ctx = s->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (n_views != s->h_views.size() || n_infos != s->h_infos.size() || (n_views && !views) || (n_infos && !infos))
        return fail(ctx, KG_INVALID_ARG, "%u views / %u infos uploaded", (uint32_t)s->h_views.size(), (uint32_t)s->h_infos.size());
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    kg_status st = sync_views_from_device(s);
    if (st != KG_OK) return st;
    std::copy(s->h_views.begin(), s->h_views.end(), views);
    std::copy(s->h_infos.begin(), s->h_infos.end(), infos);
    return KG_OK;
}

kg_status kg_snapshot_read_rsv_devs(kg_snap* s, kg_rsv_dev* devs, uint32_t n_devs) {
    if (!s) return KG_INVALID_ARG;
    kg_ctx* ctx = s->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (n_devs != s->h_rdevs.size() || (n_devs && !devs))
        return fail(ctx, KG_INVALID_ARG, "%u GPU restore tables uploaded", (uint32_t)s->h_rdevs.size());
    if (!n_devs) return KG_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipMemcpyAsync(devs, s->d_rdev, sizeof(DevRec) * n_devs, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return KG_OK;
}

// the views / reservations / GPU restore tables of the whole snapshot onto the device (caller holds the lock)
static kg_status upload_views(kg_snap* s, const kg_rsv_view* views, uint32_t nv, const kg_rsv_info* infos, uint32_t ni,
                              const kg_rsv_dev* devs, uint32_t nd) {
    kg_ctx* ctx = s->ctx;
    // views sorted by (class, record position); node class masks
    std::vector<uint32_t> order(nv);
    std::vector<uint64_t> mask(s->n, 0);
    for (uint32_t v = 0; v < nv; v++) {
        const kg_rsv_view& x = views[v];
        if (x.node >= s->n) return fail(ctx, KG_INVALID_ARG, "view %u: node %u >= %u", v, x.node, s->n);
        if (x.cls >= (uint32_t)RSV_MAX_CLASSES) return fail(ctx, KG_UNSUPPORTED, "view %u: class %u >= %d", v, x.cls, RSV_MAX_CLASSES);
        if (x.count > (uint32_t)RSV_MAX_PER_VIEW || (uint64_t)x.first + x.count > ni)
            return fail(ctx, KG_INVALID_ARG, "view %u: reservations [%u, %u+%u) invalid", v, x.first, x.first, x.count);
        if ((mask[x.node] >> x.cls) & 1ull) return fail(ctx, KG_INVALID_ARG, "view %u: duplicate (class %u, node %u)", v, x.cls, x.node);
        if (x.dev_base < -1 || x.dev_base >= (int64_t)nd) return fail(ctx, KG_INVALID_ARG, "view %u: GPU table %d of %u", v, x.dev_base, nd);
        mask[x.node] |= 1ull << x.cls;
        order[v] = v;
    }
    for (uint32_t t = 0; t < ni; t++) {
        const int64_t o = infos[t].order;
        if (o <= -(1ll << 31) || o >= (1ll << 31)) return fail(ctx, KG_INVALID_ARG, "reservation %u: order outside int32", t);
        if (infos[t].dev < -1 || infos[t].dev >= (int64_t)nd)
            return fail(ctx, KG_INVALID_ARG, "reservation %u: GPU table %d of %u", t, infos[t].dev, nd);
    }
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        if (views[a].cls != views[b].cls) return views[a].cls < views[b].cls;
        return s->pos[views[a].node] < s->pos[views[b].node];
    });
    std::vector<RsvView> dv(std::max<uint32_t>(nv, 1));
    std::vector<uint32_t> cb(RSV_MAX_CLASSES + 1, 0);
    for (uint32_t t = 0; t < nv; t++) {
        const kg_rsv_view& x = views[order[t]];
        RsvView& d = dv[t];
        std::memset(&d, 0, sizeof(d));
        d.rec = s->pos[x.node];
        d.first = x.first;
        d.count = x.count;
        d.cls = x.cls;
        for (int k = 0; k < RSV_R; k++) {
            d.req[k] = x.req[k];
            d.pod_requested[k] = x.pod_requested[k];
            d.r_allocated[k] = x.r_allocated[k];
        }
        d.nz_cpu = x.nz_cpu;
        d.nz_mem = x.nz_mem;
        d.num_pods = x.num_pods;
        d.dev_base = x.dev_base;
        cb[x.cls + 1]++;
    }
    for (int c = 0; c < RSV_MAX_CLASSES; c++) cb[c + 1] += cb[c];
    std::vector<RsvInfo> di(std::max<uint32_t>(ni, 1));
    for (uint32_t t = 0; t < ni; t++) {
        const kg_rsv_info& x = infos[t];
        RsvInfo& d = di[t];
        std::memset(&d, 0, sizeof(d));
        d.policy = x.policy;
        d.names = x.names;
        d.allocate_once = x.allocate_once;
        d.dev = x.dev;
        d.order = x.order;
        for (int k = 0; k < RSV_R; k++) {
            d.allocatable[k] = x.allocatable[k];
            d.allocated[k] = x.allocated[k];
            d.reserved[k] = x.reserved[k];
        }
        d.max_pods = x.max_pods;
        d.allocated_pods = x.allocated_pods;
        d.rid = x.rid;
        d.allocated_keys = x.allocated_keys;
        d.dev_pref = x.dev_minors;
    }
    // the node record of every GPU restore table (a table belongs to one view: its base or one of its reservations)
    std::vector<uint32_t> rrec(std::max<uint32_t>(nd, 1), 0u);
    for (uint32_t v = 0; v < nv; v++) {
        const uint32_t rec = s->pos[views[v].node];
        if (views[v].dev_base >= 0) rrec[views[v].dev_base] = rec;
        for (uint32_t t = views[v].first; t < views[v].first + views[v].count; t++)
            if (infos[t].dev >= 0) rrec[infos[t].dev] = rec;
    }
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    for (void* b : {(void*)s->d_views, (void*)s->d_infos, (void*)s->d_cls_begin, (void*)s->d_rdev, (void*)s->d_rdev_rec,
                    (void*)s->d_vfirst, (void*)s->d_vmap})
        hipFree(b);
    s->d_vfirst = nullptr;
    s->d_vmap = nullptr;
    s->d_views = nullptr;
    s->d_infos = nullptr;
    s->d_cls_begin = nullptr;
    s->d_rdev = nullptr;
    s->d_rdev_rec = nullptr;
    s->n_rdev = nd;
    HIP_TRY(ctx, hipMalloc(&s->d_rdev_rec, sizeof(uint32_t) * rrec.size()));
    HIP_TRY(ctx, hipMemcpyAsync(s->d_rdev_rec, rrec.data(), sizeof(uint32_t) * rrec.size(), hipMemcpyHostToDevice, ctx->stream));
    static_assert(sizeof(DevRec) == sizeof(kg_rsv_dev), "kg_rsv_dev is a DevRec");
    HIP_TRY(ctx, hipMalloc(&s->d_rdev, sizeof(DevRec) * std::max<uint32_t>(nd, 1)));
    if (nd) HIP_TRY(ctx, hipMemcpyAsync(s->d_rdev, devs, sizeof(DevRec) * nd, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMalloc(&s->d_views, sizeof(RsvView) * dv.size()));
    HIP_TRY(ctx, hipMalloc(&s->d_infos, sizeof(RsvInfo) * di.size()));
    HIP_TRY(ctx, hipMalloc(&s->d_cls_begin, sizeof(uint32_t) * cb.size()));
    HIP_TRY(ctx, hipMemcpyAsync(s->d_views, dv.data(), sizeof(RsvView) * dv.size(), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(s->d_infos, di.data(), sizeof(RsvInfo) * di.size(), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(s->d_cls_begin, cb.data(), sizeof(uint32_t) * cb.size(), hipMemcpyHostToDevice, ctx->stream));
    // direct view lookup (find_view): per record the start of its views in vmap, in class order
    std::vector<uint32_t> vfirst(std::max<uint32_t>(s->n, 1), 0u), vmap(std::max<uint32_t>(nv, 1), 0u);
    {
        std::vector<uint64_t> rmask(s->n, 0);
        for (uint32_t i = 0; i < s->n; i++) rmask[s->pos[i]] = mask[i];
        uint32_t at = 0;
        for (uint32_t r = 0; r < s->n; r++) {
            vfirst[r] = at;
            at += (uint32_t)__builtin_popcountll(rmask[r]);
        }
        for (uint32_t t = 0; t < nv; t++) {
            const uint32_t r = dv[t].rec;
            vmap[vfirst[r] + (uint32_t)__builtin_popcountll(rmask[r] & ((1ull << dv[t].cls) - 1ull))] = t;
        }
    }
    HIP_TRY(ctx, hipMalloc(&s->d_vfirst, sizeof(uint32_t) * vfirst.size()));
    HIP_TRY(ctx, hipMalloc(&s->d_vmap, sizeof(uint32_t) * vmap.size()));
    HIP_TRY(ctx, hipMemcpyAsync(s->d_vfirst, vfirst.data(), sizeof(uint32_t) * vfirst.size(), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(s->d_vmap, vmap.data(), sizeof(uint32_t) * vmap.size(), hipMemcpyHostToDevice, ctx->stream));
    // class masks into slot N_RSV_CLASSES of every record (a strided 8-byte column copy)
    s->cls_mask = mask;
    s->n_view_nodes = 0;
    for (uint32_t i = 0; i < s->n; i++) s->n_view_nodes += mask[i] != 0;
    std::vector<int64_t> col(s->n);
    for (uint32_t i = 0; i < s->n; i++) {
        col[s->pos[i]] = (int64_t)mask[i];
        s->h_nodes[s->pos[i]].v[N_RSV_CLASSES] = (int64_t)mask[i];
    }
    if (s->n)
        HIP_TRY(ctx, hipMemcpy2DAsync(&s->d_nodes[0].v[N_RSV_CLASSES], sizeof(NodeRec), col.data(), sizeof(int64_t),
                                      sizeof(int64_t), s->n, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    s->n_views = nv;
    s->views_stale = false;
    s->gpu_raw = false;  // the restore inputs of GPU-holding reservations go with the views they were given for
    s->rsv_gpu = false;
    for (uint32_t v = 0; v < nv; v++) s->rsv_gpu = s->rsv_gpu || views[v].dev_base >= 0;
    for (uint32_t t = 0; t < ni; t++) s->rsv_gpu = s->rsv_gpu || infos[t].dev >= 0;
    s->view_order = order;
    s->views_on_device = false;
    s->h_views.assign(views, views + nv);
    s->h_infos.assign(infos, infos + ni);
    s->h_rdevs.assign(devs, devs + nd);
    s->stale.assign(s->n, 0);
    s->n_stale = 0;
    s->gen++;
    s->invalidate_saved();
    s->max_cls_views = 0;
    for (int c = 0; c < RSV_MAX_CLASSES; c++) s->max_cls_views = std::max(s->max_cls_views, cb[c + 1] - cb[c]);
    return KG_OK;
}

kg_status kg_snapshot_upload_reservations(kg_snap* s, const kg_rsv_view* views, uint32_t nv, const kg_rsv_info* infos,
                                          uint32_t ni, const kg_rsv_dev* devs, uint32_t nd) {
    if (!s || (!views && nv) || (!infos && ni) || (!devs && nd)) return KG_INVALID_ARG;
    kg_ctx* ctx = s->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (!s->uploaded) return fail(ctx, KG_INVALID_ARG, "snapshot not uploaded");
    return upload_views(s, views, nv, infos, ni, devs, nd);
}

kg_status kg_snapshot_upload_rsv_gpu(kg_snap* s, const kg_rsv_gpu* g, uint32_t n) {
    if (!s || (!g && n)) return KG_INVALID_ARG;
    kg_ctx* ctx = s->ctx;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!s->uploaded) return fail(ctx, KG_INVALID_ARG, "snapshot not uploaded");
    if (!s->d_dev) {  // DeviceShare is off here: the GPU restore tables matter to no plugin
        s->gpu_raw = true;
        return KG_OK;
    }
    // node entries (rid -1) and each node's reservation entries, grouped by node
    std::vector<int32_t> node_entry(s->n, -1);
    std::vector<std::vector<uint32_t>> rsv_of(s->n);
    for (uint32_t k = 0; k < n; k++) {
        if (g[k].node >= s->n) return fail(ctx, KG_INVALID_ARG, "entry %u: node %u >= %u", k, g[k].node, s->n);
        if (g[k].rid < 0) {
            if (node_entry[g[k].node] >= 0) return fail(ctx, KG_INVALID_ARG, "node %u: two used entries", g[k].node);
            node_entry[g[k].node] = (int32_t)k;
        } else {
            rsv_of[g[k].node].push_back(k);
        }
    }
    // the inputs must cover every GPU-holding view and reservation: a node left out would keep stale restore tables
    // after a Reserve there (its record has no raw entry), so a partial upload is refused and the calls keep refusing
    for (const kg_rsv_view& v : s->h_views) {
        if (v.node >= s->n) continue;
        if (v.dev_base >= 0 && node_entry[v.node] < 0)
            return fail(ctx, KG_INVALID_ARG, "node %u: a view holds GPU restore tables but no used entry was given", v.node);
        for (uint32_t t = v.first; t < v.first + v.count && t < s->h_infos.size(); t++) {
            if (s->h_infos[t].dev < 0) continue;
            if (node_entry[v.node] < 0)
                return fail(ctx, KG_INVALID_ARG, "node %u: reservation %u holds GPUs but no used entry was given", v.node,
                            s->h_infos[t].rid);
            bool found = false;
            for (uint32_t k : rsv_of[v.node]) found = found || (uint32_t)g[k].rid == s->h_infos[t].rid;
            if (!found)
                return fail(ctx, KG_INVALID_ARG, "node %u: reservation %u holds GPUs but has no entry", v.node,
                            s->h_infos[t].rid);
        }
    }
    std::vector<GpuRawNode> gn;
    std::vector<GpuRawRsv> gr;
    std::vector<int32_t> graw(std::max<uint32_t>(s->n, 1), -1);
    for (uint32_t i = 0; i < s->n; i++) {
        if (rsv_of[i].empty() && node_entry[i] < 0) continue;
        if (node_entry[i] < 0) return fail(ctx, KG_INVALID_ARG, "node %u: reservation entries without its used entry", i);
        GpuRawNode x;
        std::memset(&x, 0, sizeof(x));
        std::memcpy(x.used, g[node_entry[i]].a, sizeof(x.used));
        x.first = (uint32_t)gr.size();
        x.count = (uint32_t)rsv_of[i].size();
        for (uint32_t k : rsv_of[i]) {
            GpuRawRsv r;
            std::memset(&r, 0, sizeof(r));
            std::memcpy(r.alloc, g[k].a, sizeof(r.alloc));
            std::memcpy(r.allocated, g[k].b, sizeof(r.allocated));
            r.rid = (uint32_t)g[k].rid;
            r.policy = g[k].policy;
            r.pods = g[k].allocated_pods;
            gr.push_back(r);
        }
        graw[s->pos[i]] = (int32_t)gn.size();
        gn.push_back(x);
    }
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    for (void* b : {(void*)s->d_graw, (void*)s->d_gnodes, (void*)s->d_grsv}) hipFree(b);
    s->d_graw = nullptr, s->d_gnodes = nullptr, s->d_grsv = nullptr;
    HIP_TRY(ctx, hipMalloc(&s->d_graw, sizeof(int32_t) * graw.size()));
    HIP_TRY(ctx, hipMalloc(&s->d_gnodes, sizeof(GpuRawNode) * std::max<size_t>(gn.size(), 1)));
    HIP_TRY(ctx, hipMalloc(&s->d_grsv, sizeof(GpuRawRsv) * std::max<size_t>(gr.size(), 1)));
    HIP_TRY(ctx, hipMemcpy(s->d_graw, graw.data(), sizeof(int32_t) * graw.size(), hipMemcpyHostToDevice));
    if (!gn.empty()) HIP_TRY(ctx, hipMemcpy(s->d_gnodes, gn.data(), sizeof(GpuRawNode) * gn.size(), hipMemcpyHostToDevice));
    if (!gr.empty()) HIP_TRY(ctx, hipMemcpy(s->d_grsv, gr.data(), sizeof(GpuRawRsv) * gr.size(), hipMemcpyHostToDevice));
    s->n_gnodes = (uint32_t)gn.size();
    s->n_grsv = (uint32_t)gr.size();
    s->gpu_raw = true;
    s->gen++;
    s->invalidate_saved();
    return KG_OK;
}

kg_status kg_snapshot_update_views(kg_snap* s, const uint32_t* nodes, uint32_t n_nodes, const kg_rsv_view* views, uint32_t nv,
                                   const kg_rsv_info* infos, uint32_t ni, const kg_rsv_dev* devs, uint32_t nd) {
    if (!s || (!nodes && n_nodes) || (!views && nv) || (!infos && ni) || (!devs && nd)) return KG_INVALID_ARG;
    kg_ctx* ctx = s->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (!s->uploaded) return fail(ctx, KG_INVALID_ARG, "snapshot not uploaded");
    kg_status sst = sync_views_from_device(s);
    if (sst != KG_OK) return sst;
    std::vector<uint8_t> listed(s->n, 0);
    for (uint32_t k = 0; k < n_nodes; k++) {
        if (nodes[k] >= s->n) return fail(ctx, KG_INVALID_ARG, "node %u >= %u", nodes[k], s->n);
        listed[nodes[k]] = 1;
    }
    for (uint32_t v = 0; v < nv; v++)
        if (views[v].node >= s->n || !listed[views[v].node])
            return fail(ctx, KG_INVALID_ARG, "view %u: node %u is not among the updated nodes", v, views[v].node);
    // the kept views of the other nodes (their reservations and GPU tables re-indexed), then the new ones
    std::vector<kg_rsv_view> av;
    std::vector<kg_rsv_info> ai;
    std::vector<kg_rsv_dev> ad;
    std::vector<int32_t> dmap(s->h_rdevs.size(), -1);
    auto dev_of = [&](int32_t d) {
        if (d < 0) return d;
        if (dmap[d] < 0) {
            dmap[d] = (int32_t)ad.size();
            ad.push_back(s->h_rdevs[d]);
        }
        return dmap[d];
    };
    for (const kg_rsv_view& x : s->h_views) {
        if (listed[x.node]) continue;
        kg_rsv_view y = x;
        y.first = (uint32_t)ai.size();
        y.dev_base = dev_of(x.dev_base);
        for (uint32_t t = x.first; t < x.first + x.count; t++) {
            kg_rsv_info r = s->h_infos[t];
            r.dev = dev_of(r.dev);
            ai.push_back(r);
        }
        av.push_back(y);
    }
    const uint32_t i0 = (uint32_t)ai.size(), d0 = (uint32_t)ad.size();
    for (uint32_t v = 0; v < nv; v++) {
        kg_rsv_view y = views[v];
        if ((uint64_t)y.first + y.count > ni) return fail(ctx, KG_INVALID_ARG, "view %u: reservations out of range", v);
        y.first += i0;
        if (y.dev_base >= 0) y.dev_base += (int32_t)d0;
        av.push_back(y);
    }
    for (uint32_t t = 0; t < ni; t++) {
        kg_rsv_info r = infos[t];
        if (r.dev >= 0) r.dev += (int32_t)d0;
        ai.push_back(r);
    }
    ad.insert(ad.end(), devs, devs + nd);
    const std::vector<uint8_t> keep = s->stale;
    kg_status st = upload_views(s, av.data(), (uint32_t)av.size(), ai.data(), (uint32_t)ai.size(), ad.data(),
                                (uint32_t)ad.size());
    if (st != KG_OK) return st;
    // the listed nodes are fresh; any other stale node stays stale
    for (uint32_t i = 0; i < s->n && i < keep.size(); i++)
        if (keep[i] && !listed[i] && s->cls_mask[i]) {
            s->stale[i] = 1;
            s->n_stale++;
        }
    s->views_stale = s->n_stale != 0;
    return KG_OK;
}

kg_status kg_profile_enable(kg_ctx* ctx, int enable) {
    if (!ctx) return KG_INVALID_ARG;
    std::lock_guard<std::mutex> g(ctx->mu);
    ctx->profiling = enable != 0;
    return KG_OK;
}

kg_status kg_profile_read(kg_ctx* ctx, double* total_ms, uint64_t* launches, int reset) {
    if (!ctx) return KG_INVALID_ARG;
    std::lock_guard<std::mutex> g(ctx->mu);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    for (auto& e : ctx->ev_live) {
        HIP_TRY(ctx, hipEventSynchronize(e.second));
        float ms = 0.f;
        HIP_TRY(ctx, hipEventElapsedTime(&ms, e.first, e.second));
        ctx->prof_ms += ms;
        ctx->prof_launches++;
        ctx->ev_free.push_back(e);
    }
    ctx->ev_live.clear();
    if (total_ms) *total_ms = ctx->prof_ms;
    if (launches) *launches = ctx->prof_launches;
    if (reset) {
        ctx->prof_ms = 0.0;
        ctx->prof_launches = 0;
    }
    return KG_OK;
}

kg_status kg_shard_unique_id(uint8_t out[128]) {
    if (!out) return KG_INVALID_ARG;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return KG_DEVICE_ERROR;
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(out, &id, 128);
    return KG_OK;
}

kg_status kg_shard_init(kg_ctx* ctx, const uint8_t id[128], int rank, int world) {
    if (!ctx || !id || world < 1 || rank < 0 || rank >= world) return KG_INVALID_ARG;
    std::lock_guard<std::mutex> g(ctx->mu);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    ncclUniqueId uid;
    std::memcpy(&uid, id, 128);
    if (ctx->comm) {
        ncclCommDestroy(ctx->comm);
        ctx->comm = nullptr;
    }
    NCCL_TRY(ctx, ncclCommInitRank(&ctx->comm, world, uid, rank));
    ctx->rank = rank;
    ctx->world = world;
    return KG_OK;
}

kg_status kg_shard_select(kg_snap* s, kg_pods* p, uint32_t k, uint64_t* out_keys) {
    kg_status st = check_pair(s, p);
    if (st != KG_OK) return st;
    kg_ctx* ctx = s->ctx;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (!ctx->comm) return fail(ctx, KG_INVALID_ARG, "kg_shard_init not called");
    if (k == 0 || k > (uint32_t)KG_TOPK_MAX) return fail(ctx, KG_INVALID_ARG, "k=%u outside [1, %d]", k, KG_TOPK_MAX);
    st = check_views(s);
    if (st != KG_OK) return st;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const uint32_t n = p->n;
    const uint32_t kk = k == 1 ? 1 : KG_TOPK_MAX;  // kernels keep 1 or KG_TOPK_MAX keys per pod
    const size_t need = (size_t)n * kk * (ctx->world + 1);
    if (need > p->gather_cap) {
        if (p->d_gather) {
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            HIP_TRY(ctx, hipFree(p->d_gather));
            p->d_gather = nullptr;
        }
        HIP_TRY(ctx, hipMalloc(&p->d_gather, sizeof(uint64_t) * std::max<size_t>(need, 1)));
        p->gather_cap = need;
    }
    uint64_t* local = p->d_gather + (size_t)n * kk * ctx->world;  // this shard's per-pod top-kk keys
    if (s->ext()) {
        // NormalizeScore maxima and the Reservation preferred node are global over all shards: one
        // all-reduce per statistic between the two passes (a real exchange step)
        st = check_ext(s);
        if (st != KG_OK) return st;
        p->k_last = k;
        p->kk_last = kk;
        if (n == 0) return KG_OK;
        hipEvent_t e0, e1;  // bracket: the whole shard step (its all-reduces included)
        st = record_begin(ctx, &e0, &e1);
        if (st != KG_OK) return st;
        st = ext_stats_local(s, p);
        if (st != KG_OK) return st;
        NCCL_TRY(ctx, ncclAllReduce(p->d_dev_max, p->d_dev_max, n, ncclUint32, ncclMax, ctx->comm, ctx->stream));
        NCCL_TRY(ctx, ncclAllReduce(p->d_rsv_max, p->d_rsv_max, n, ncclUint32, ncclMax, ctx->comm, ctx->stream));
        NCCL_TRY(ctx, ncclAllReduce(p->d_pref, p->d_pref, n, ncclUint64, ncclMin, ctx->comm, ctx->stream));
        // the one-pass select's per-class bounds (k_dev_sum; zero on a shard that built none)
        if (!(s->d_dev && ext_fast_base(s, p)))
            HIP_TRY(ctx, hipMemsetAsync(spec_cls_max(p), 0, sizeof(uint32_t) * DEV_CLASSES, ctx->stream));
        NCCL_TRY(ctx, ncclAllReduce(spec_cls_max(p), spec_cls_max(p), DEV_CLASSES, ncclUint32, ncclMax, ctx->comm,
                                    ctx->stream));
        if (s->n == 0) {
            HIP_TRY(ctx, hipMemsetAsync(local, 0, sizeof(uint64_t) * n * kk, ctx->stream));
            NCCL_TRY(ctx, ncclAllReduce(spec_fb_max(p), spec_fb_max(p), n, ncclUint32, ncclMax, ctx->comm, ctx->stream));
        } else
            st = ext_select_local(s, p, kk, local, true);
        if (st != KG_OK) return st;
        st = record_end(ctx, e0, e1);
    } else {
        st = select_local(s, p, k, local);
    }
    if (st != KG_OK) return st;
    if (n == 0) return KG_OK;
    // per-pod outcome flags: the quota verdict is the same on every rank and KG_ST_UNSUPPORTED is the
    // top bit, so the max over ranks is their OR
    NCCL_TRY(ctx, ncclAllReduce(p->d_pstat, p->d_pstat, n, ncclUint32, ncclMax, ctx->comm, ctx->stream));
    // exchange the per-shard top-kk keys (8 B x kk per pod per shard) and run the same global selectHost
    NCCL_TRY(ctx, ncclAllGather(local, p->d_gather, (size_t)n * kk, ncclUint64, ctx->comm, ctx->stream));
    HIP_TRY(ctx, launch_merge(p->d_gather, (uint32_t)ctx->world, n, kk, p->d_keys, ctx->stream));
    p->k_last = k;
    p->kk_last = kk;
    if (out_keys) {
        std::vector<uint64_t> h((size_t)n * kk);
        HIP_TRY(ctx, hipMemcpyAsync(h.data(), p->d_keys, sizeof(uint64_t) * n * kk, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        for (uint32_t j = 0; j < n; j++)
            for (uint32_t t = 0; t < k; t++) out_keys[(size_t)j * k + t] = h[(size_t)j * kk + t];
    }
    return KG_OK;
}

uint64_t kg_make_key(int64_t total, uint32_t node) {
    return ((uint64_t)total << 32) | (uint64_t)(0xFFFFFFFFu - node);
}

int32_t kg_key_node(uint64_t key) { return key ? (int32_t)(0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFull)) : -1; }

int64_t kg_key_total(uint64_t key) { return key ? (int64_t)(key >> 32) : -1; }

kg_status kg_merge_keys(const uint64_t* keys, uint32_t n_shards, uint32_t n_pods, uint32_t k, uint64_t* out) {
    if ((!keys && n_shards && n_pods) || (!out && n_pods) || k == 0) return KG_INVALID_ARG;
    std::vector<uint64_t> top(k);
    for (uint32_t j = 0; j < n_pods; j++) {
        std::fill(top.begin(), top.end(), 0ull);
        for (uint32_t sh = 0; sh < n_shards; sh++) {
            const uint64_t* src = keys + ((size_t)sh * n_pods + j) * k;
            for (uint32_t t = 0; t < k; t++) {
                uint64_t key = src[t];
                for (uint32_t u = 0; u < k; u++) {
                    if (key > top[u]) std::swap(key, top[u]);
                }
            }
        }
        for (uint32_t t = 0; t < k; t++) out[(size_t)j * k + t] = top[t];
    }
    return KG_OK;
}

}  // extern "C"
