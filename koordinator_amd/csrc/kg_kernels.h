// kg_kernels.h — host-side launch interface of the device kernels (internal to libkoordgpu.so).
#pragma once
#include <hip/hip_runtime_api.h>

#include "kg_layout.h"
#include "../../include/koordgpu.h"

namespace kg {

constexpr int KG_TOPK_MAX = 4;  // select kernels are instantiated for K = 1 and K = 4 (k <= 4)

// One storage class of node records: [begin, end) walked in n_chunks chunks of `chunk` records,
// written to partial rows [part0, part0 + n_chunks).
struct SelectRange {
    uint32_t begin, end, chunk, n_chunks, part0;
};

// Matrix-mode select of one pod batch against one snapshot (launch_select). The batch is split per pod:
// lanes [0, n_fast) of `order` take the float64 fast path (k_select1 / k_select<FAST>) on the records of
// each storage class plus the integer path on the F_BIG records (k_big_sel, chunked over the device's
// F_BIG list); lanes [n_fast, n_pods) — pods outside the fast domain (a NUMA policy of their own, cpuset
// binding, values >= 2^44) — take the integer path on every record (k_select<!FAST>). Final keys go to
// out[row][K] (row = the lane's pod; K = 1 or KG_TOPK_MAX); K > 1 (and the unfused top-1 fast path)
// goes through per-chunk partial rows [part][ld][K] and list merges.
struct LaunchSelect {
    const NodeRec* nodes;
    const ZoneRec* zones;
    PodsDev pods;
    uint32_t n_pods;       // lanes: fast lanes then integer lanes
    uint32_t n_rows;       // row space of out / partial (the pod batch): row stride of the partials
    uint32_t index_base, k;
    SelectRange range[2];  // fast sub-batch: records of storage class 0 / 1
    SelectRange irange;    // integer sub-batch: every record
    bool exact, fast;
    KCfg cfg;
    uint64_t* partial;     // [parts][n_rows][K]
    const uint32_t* pmap;  // sub-batch row -> batch position for pstat (nullptr: identity)
    uint32_t* pstat;       // per batch position: KG_ST_UNSUPPORTED when some pair needs the host path
    bool fused;            // K == 1 fast path: atomicMax straight into out, no partials
    bool fused_k;          // K > 1: every lane inserts its top-K into out[row] by the atomicMax cascade
                           // (topk_atomic, kg_kernels.hip), no partials, no merge
    uint64_t* out;
    const uint32_t* big_list;
    const uint32_t* big_count;
    uint32_t big_y, big_part0;  // F_BIG chunks (blockIdx.y) and their first partial row (unfused)
    const uint32_t* order;  // lane -> row: fast lanes (grouped by wave kind) then integer lanes; nullptr: identity
    uint32_t n_fast;        // fast lanes (0 unless `fast`)
    // integer lanes with atomics into out (K == 1, or fused_k): pruned evaluation when ipairs is set -- records
    // [0, iseed) seed each lane's top-K on the integer path, then only the pairs whose fast-path NodeResourcesFit /
    // LoadAware bound can still enter it (survivors, (lane << 32) | record, at most ipairs_cap) are evaluated
    uint64_t* ipairs;       // per filter workgroup a segment of 256 x chunk slots
    uint32_t* ipair_count;  // per segment: survivors
    uint64_t ipairs_cap;    // slots of ipairs
    uint32_t iseg_cap, iseed;  // entries of ipair_count; seed records
    // optional second stream for the pruned integer lanes (they write only their own rows of out): forked from
    // the launch stream before the fast kernels, joined back after them
    hipStream_t side;
    hipEvent_t fork, join;
};
inline uint32_t select_fparts(const LaunchSelect& a) { return a.big_part0 + a.big_y; }

// Block replay (k_rb_top / k_rb_merge / k_rb_fix): window of RB_W pods, RB_K keys kept per pod,
// changed-row bitmap in LDS (snapshots up to 32 x RB_BITMAP_WORDS records).
constexpr int RB_W = 64;
constexpr int RB_K = 16;
constexpr int RB_BITMAP_WORDS = 8192;
constexpr int RB_CHUNK = 32;  // records per k_rb_top wave (fast blocks staged in LDS)

struct LaunchRb {
    const NodeRec* nodes;
    const ZoneRec* zones;
    NodeRec* nodes_rw;
    ZoneRec* zones_rw;
    PodsDev pods;
    uint32_t n_pods, n_nodes, index_base, n_parts;
    SelectRange range[2];
    bool exact, fast;
    KCfg cfg;
    const uint32_t* pos;  // snapshot index -> record
    uint32_t* step;       // next pod to place
    uint64_t* partial;    // [n_parts][RB_W][RB_K]
    uint64_t* tops;       // [RB_W][RB_K]
    uint64_t* winners;
};

struct VerifyDev {
    uint32_t* status;
    int64_t *s_nrf, *s_la, *s_numa, *total;
    int8_t* zone;
};

struct ExtVerifyDev {
    uint32_t* status;
    int64_t *s_nrf, *s_la, *s_numa, *s_dev, *s_rsv, *order, *total;
    int8_t* zone;
};

hipError_t launch_select(const LaunchSelect& a, hipStream_t s);

// config-5 plugin set (kg_ext.hip)
hipError_t launch_ext_gate(const PodsDev& pods, uint32_t n_pods, const ExtDev& e, uint32_t plugins, uint32_t* qst,
                           uint32_t* pstat, hipStream_t s);
hipError_t launch_ext_verify(const NodeRec* nodes, const ZoneRec* zones, const ExtDev& e, const PodsDev& pods,
                             uint32_t n_pods, uint32_t n_nodes, uint32_t index_base, const KCfg& cfg, bool exact,
                             const uint32_t* qst, const ExtVerifyDev& o, hipStream_t s);
// A second stream for one independent kernel of a launcher (forked from and joined back into the launch stream
// inside the launcher; nullptr / null members: everything on the launch stream).
struct SideLane {
    hipStream_t s;
    hipEvent_t fork, join;
};
hipError_t launch_ext_stats(const NodeRec* nodes, const ZoneRec* zones, const ExtDev& e, const PodsDev& pods,
                            const uint32_t* list, uint32_t n_list, uint32_t n_nodes, uint32_t n0, uint32_t chunk,
                            uint32_t index_base, const KCfg& cfg, bool exact, bool topo, bool fb, const uint32_t* qst,
                            uint32_t* dev_max, uint32_t* rsv_max, uint64_t* pref, const uint32_t* special,
                            uint32_t special_est, const uint32_t* c1, uint32_t c1_est, hipStream_t s, const SideLane* lane = nullptr);
hipError_t launch_ext_stats_views(const NodeRec* nodes, const ZoneRec* zones, const ExtDev& e, const PodsDev& pods,
                                  const uint32_t* list, uint32_t n_list, uint32_t max_views, uint32_t index_base,
                                  const KCfg& cfg, bool exact,
                                  bool topo, const uint32_t* qst, uint32_t* dev_max, uint32_t* rsv_max, uint64_t* pref,
                                  hipStream_t s);
hipError_t launch_ext_select(const NodeRec* nodes, const ZoneRec* zones, const ExtDev& e, const PodsDev& pods,
                             const uint32_t* list, uint32_t n_pods, uint32_t n_nodes, uint32_t n0, uint32_t chunk, uint32_t k,
                             uint32_t index_base, const KCfg& cfg, bool exact, bool topo, bool fb, const uint32_t* qst, const uint32_t* dev_max,
                             const uint32_t* rsv_max, const uint64_t* pref, uint64_t* partial, uint32_t* pstat, hipStream_t s);
// dst[i] = max(dst[i], src[i])
hipError_t launch_max_fold(uint32_t* dst, const uint32_t* src, uint32_t n, hipStream_t s);
// One-pass fast-base select, second half: final DeviceShare maxima into dev_max, re-run of the rows whose guess
// was wrong (fb launches; k = 1: partial = the fused keys by row).
hipError_t launch_ext_fix(const NodeRec* nodes, const ZoneRec* zones, const ExtDev& e, const PodsDev& pods,
                          const uint32_t* list, uint32_t n_pods, uint32_t n_nodes, uint32_t n0, uint32_t chunk, uint32_t k,
                          uint32_t index_base, const KCfg& cfg, const uint32_t* qst, uint32_t* dev_max,
                          const uint32_t* rsv_max, const uint64_t* pref, uint64_t* partial, uint32_t* pstat,
                          uint32_t* rows, uint32_t* n_rows, hipStream_t s);
// General records of a fast-base select (F_BIG, class 1 unless split off into c1, the lane's views); k > 1: partial
// chunks after the fast-base kernel's (n_nodes / chunk of them), then the class-1 kernel's (c1 != nullptr:
// k_special_scan's c1 list, evaluated by the light k_ext_select_c1).
// k_ext_select_c1 at top-1 straight into keys: beside the one-pass select (e.cls_max: its guessed maxima) or, with
// e.rows, on the rows k_ext_fix_rows listed
hipError_t launch_ext_select_c1_top1(const NodeRec* nodes, const ZoneRec* zones, const ExtDev& e, const PodsDev& pods,
                                     const uint32_t* list, uint32_t n_pods, uint32_t n0, uint32_t index_base, const KCfg& cfg,
                                     const uint32_t* qst, const uint32_t* dev_max, const uint64_t* pref, uint64_t* keys,
                                     const uint32_t* c1, uint32_t c1_est, hipStream_t s);
hipError_t launch_ext_select_sp(const NodeRec* nodes, const ZoneRec* zones, const ExtDev& e, const PodsDev& pods,
                                const uint32_t* list, uint32_t n_pods, uint32_t n_nodes, uint32_t n0, uint32_t chunk, uint32_t k,
                                uint32_t index_base, const KCfg& cfg, const uint32_t* qst, const uint32_t* dev_max,
                                const uint32_t* rsv_max, const uint64_t* pref, uint64_t* partial, uint32_t* pstat,
                                const uint32_t* special, uint32_t special_est, const uint32_t* c1, uint32_t c1_est, uint32_t live_est, bool c1_split,
                                hipStream_t s, const SideLane* lane = nullptr);
// out[map[t]] = rows t of src (k keys each; row map[t] with src_by_map, src may then be out); rows whose pod
// has a nonzero qst[pod] get zero keys and pstat[pod] = qst[pod] (the gate decided the pod: no pair needs the
// host path)
hipError_t launch_scatter_keys(const uint64_t* src, const uint32_t* map, uint32_t n, uint32_t k, bool src_by_map,
                               const uint32_t* qst, uint64_t* out, uint32_t* pstat, hipStream_t s);
// arrival counters of a replay step launch (the last workgroup picks): REPLAY_DONE_SHARDS shard counters and one top
// counter, each on a 128-B line of its own; uint32 words, zeroed once, left zeroed by every launch
constexpr uint32_t REPLAY_DONE_SHARDS = 32, REPLAY_DONE_STRIDE = 32;
constexpr uint32_t REPLAY_WG = 256;  // threads (node records) per workgroup of a replay step launch
// score buckets of a replay step: [3 steps][128 scores], one bucket per 128-B line (every workgroup's atomicMax on a
// bucket would otherwise queue behind the other buckets of its line)
constexpr uint32_t REPLAY_BUCKET_STRIDE = 16;
constexpr size_t REPLAY_BUCKET_WORDS = (size_t)3 * 128 * REPLAY_BUCKET_STRIDE;
constexpr uint32_t REPLAY_DONE_WORDS = (REPLAY_DONE_SHARDS + 1) * REPLAY_DONE_STRIDE;
hipError_t launch_ext_replay_step(NodeRec* nodes, ZoneRec* zones, DevRec* devs, const ExtDev& e, const PodsDev& pods,
                                  uint32_t n_pods, uint32_t n_nodes, uint32_t index_base, const KCfg& cfg, bool exact,
                                  const uint32_t* step_base, uint32_t step_off, uint64_t* winners, uint32_t* minors,
                                  uint64_t* buckets, int8_t* zsel, uint32_t* reason, const uint32_t* pos, int32_t* nsel,
                                  RsvStep* rs, uint64_t* rlist, uint32_t* done, const DevClass* dclass, uint32_t n_dclass,
                                  bool fb, uint32_t n0, hipStream_t s);
// k_ext_assume: Reserve (sign 1, sign 0 = its evaluation pass) / Unreserve (sign -1) with every enabled plugin; rsv:
// Reservation.Reserve / Unreserve on the node's views (rid: the reservation an Unreserve leaves); split: the NUMA
// allocation's per-zone amounts; cpus: the cpuset CPUs an Unreserve releases
hipError_t launch_ext_assume(NodeRec* nodes, ZoneRec* zones, DevRec* devs, const ExtDev& e, const PodsDev& pods,
                             uint32_t pod, uint32_t rec, int32_t zone, uint32_t minors, int64_t sign, const KCfg& cfg,
                             bool exact, int32_t* out, hipStream_t s, int64_t* split = nullptr, bool rsv = true,
                             int32_t rid = -1, kg_cpu_alloc* allocs = nullptr, const kg_cpu_topo* topos = nullptr,
                             const uint64_t* cpus = nullptr);
// batch of cpuset accumulator requests (kg_cpuset.hip)
hipError_t launch_cpuset_take(const kg_cpu_topo* topos, const kg_cpu_alloc* allocs, const kg_cpuset_request* reqs,
                              uint32_t n, uint64_t* out, int32_t* rc, hipStream_t s);
// NodeNUMAResource cpuset Reserve of (pod, rec), or with winners != nullptr of replay step's previous pod
hipError_t launch_cpuset_reserve(NodeRec* nodes, ZoneRec* zones, kg_cpu_alloc* allocs, const kg_cpu_topo* topos,
                                 const PodsDev& pods, const KCfg& cfg, uint32_t pod, uint32_t rec, const uint64_t* winners,
                                 const uint32_t* step_base, uint32_t step_off, const uint32_t* pos, uint32_t index_base,
                                 uint32_t n_pods, int8_t* zsel, int32_t* fail_out, hipStream_t s, uint32_t zsel_stride = 0,
                                 uint64_t* taken_out = nullptr);
// inline batch cycle of a whole-job plan (k_batch); ext = the snapshot carries the config-5 tables
hipError_t launch_batch(NodeRec* nodes, ZoneRec* zones, DevRec* devs, const ExtDev& e, const PodsDev& pods,
                        const uint32_t* grp_begin, const uint32_t* grp_pods, const uint32_t* grp_rec, uint32_t n_groups,
                        bool ext, const KCfg& cfg, bool exact, uint32_t* result, uint32_t* status, int32_t* zone,
                        uint32_t* minors, hipStream_t s, kg_cpu_alloc* allocs = nullptr,
                        const kg_cpu_topo* topos = nullptr);
hipError_t launch_merge(const uint64_t* partial, uint32_t n_parts, uint32_t n_pods, uint32_t k, uint64_t* out,
                        hipStream_t s);
// merge of partial rows [part0, part0 + n_parts) (row stride ld pods) for the rows list[0..n) (nullptr: 0..n)
hipError_t launch_merge_list(const uint64_t* partial, uint32_t part0, uint32_t n_parts, uint32_t ld, const uint32_t* list,
                             uint32_t n, uint32_t k, uint64_t* out, hipStream_t s);
hipError_t launch_big_scan(const NodeRec* nodes, uint32_t n_nodes, uint32_t* big_list, uint32_t* big_count,
                           hipStream_t s);
// Grid of the PART 2 ext kernels (special records, grid-stride): chunk and chunk count for an estimate
// of the special-record count and the pod blocks of the launch (~2048 workgroups in all).
inline void ext_part2_grid(uint32_t special_est, uint32_t pod_blocks, uint32_t* chunk, uint32_t* n_chunks,
                           uint32_t target = 2048u, uint32_t min_chunk = 4u) {
    const uint32_t want = pod_blocks ? (target + pod_blocks - 1) / pod_blocks : 1u;
    const uint32_t est = special_est ? special_est : 1u;
    *chunk = est / want < min_chunk ? min_chunk : (est + want - 1) / want;
    *n_chunks = (est + *chunk - 1) / *chunk;
}
hipError_t launch_special_scan(const NodeRec* nodes, uint32_t n_nodes, uint32_t n0, uint32_t* special, uint32_t* c1,
                               hipStream_t s);
hipError_t launch_rdev_codes(const NodeRec* nodes, const ZoneRec* zones, const DevRec* devs, const DevRec* rdev,
                             const uint32_t* rdev_rec, uint32_t n_rdev, const DevClass* cls, uint32_t n_cls,
                             const KCfg& cfg, const ExtDev& e, uint8_t* out, hipStream_t s);
hipError_t launch_gpu_zone_sum(const NodeRec* nodes, const ZoneRec* zones, const DevRec* devs, uint32_t n_nodes,
                               uint32_t n0, const DevClass* cls, uint32_t n_cls, const KCfg& cfg, const ExtDev& e,
                               uint64_t* out, hipStream_t s);
hipError_t launch_dev_sum(const NodeRec* nodes, const ZoneRec* zones, const DevRec* devs, uint32_t n_nodes, uint32_t n0,
                          const DevClass* cls, uint32_t n_cls, const KCfg& cfg, const ExtDev& e, DevSum* out,
                          uint32_t* cls_max, hipStream_t s, bool zero_cls_max = true);
hipError_t launch_scatter_rows(const void* stage, const uint32_t* pos, uint32_t n, bool dev, NodeRec* nodes,
                               ZoneRec* zones, DevRec* devs, hipStream_t s);
hipError_t launch_verify(const NodeRec* nodes, const ZoneRec* zones, const PodsDev& pods, uint32_t n_pods,
                         uint32_t n_nodes, const KCfg& cfg, bool exact, const VerifyDev& o, hipStream_t s);
hipError_t launch_replay_step(NodeRec* nodes, ZoneRec* zones, const PodsDev& pods, uint32_t n_pods, uint32_t n_nodes,
                              uint32_t index_base, const KCfg& cfg, bool exact, const uint32_t* step_base,
                              uint32_t step_off, uint64_t* winners, int8_t* zsel, uint32_t* reason, hipStream_t s);
hipError_t launch_bump(uint32_t* step_base, uint32_t by, hipStream_t s);
hipError_t launch_rb_window(const LaunchRb& a, hipStream_t s);
hipError_t launch_assume(NodeRec* nodes, ZoneRec* zones, const PodsDev& pods, uint32_t pod, uint32_t node,
                         int32_t zone, int64_t sign, const KCfg& cfg, bool exact, int32_t* zone_out, hipStream_t s,
                         int64_t* split = nullptr);

}  // namespace kg
