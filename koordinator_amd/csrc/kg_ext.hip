// kg_ext.hip — CDNA4 (gfx950) kernels of the config-5 plugin set (DeviceShare, Reservation,
// ElasticQuota on top of NodeResourcesFit / LoadAware / NodeNUMAResource), integer path.
//
// DeviceShare and Reservation normalise their scores by the per-pod maximum over the feasible nodes
// (DefaultNormalizeScore, frameworkext/normalize_score.go:24-52) and Reservation gives its PreScore
// preferredNode 1000 (reservation/scoring.go:113-121,191-198), so matrix mode runs in two passes:
//   k_ext_stats   lane = pod (of the pods that carry a GPU request or a reservation class), wave walks
//                 a chunk of node records: feasibility + raw DeviceShare score, nominated reservation
//                 score and the node order -> per-pod max / min by atomics;
//   k_ext_select  lane = pod, wave walks a chunk of records: weighted total with the normalised terms,
//                 running top-K per lane -> per-(chunk, pod) partials (merged by k_merge), or at K = 1 on
//                 fast-base batches an atomicMax into the pod's key.
// Fast-base batches (every base plugin on the fast block, GPU pods classed) run pass 1 on the general records
// only (F_BIG, storage class 1, the pod's views): on the fast-base records k_ext_select takes the DeviceShare
// maximum to be the class's best fitting score (k_dev_sum's cls_max), records the real one, and k_ext_fix_rows
// re-runs the rows whose guess was wrong, so no pair is evaluated twice unless its pod's guess failed.
// Between the passes the multi-GPU path all-reduces the per-pod maxima over RCCL.
// The sequential replay's step kernel (k_ext_replay, k_ext_assume) lives in kg_ext_replay.hip, the batch cycle
// (k_batch, k_batch_coop) in kg_ext_batch.hip.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kg_cpuset_reserve.h"
#include "kg_ext.h"
#include "kg_ext_wave.h"
#include "kg_kernels.h"
#include <cstdlib>

namespace kg {

// DevSum of every record for the pod batch's GPU request classes: thread = record; it loads the record's minors
// once and, per class, runs the GPU allocator's Filter and scores one instance (codes / scores stored 8 classes at
// a time). The kernel is bound by the latency of the record loads (lanes are a record apart), not by arithmetic, so
// the classes are not split over more threads. cls_max[class] = the best score over the fast-base records (below n0,
// not F_BIG, with GPUs) the class fits on: the one-pass select's guess of the DeviceShare maximum.
__global__ __launch_bounds__(256) void k_dev_sum(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                 const DevRec* __restrict__ devs, uint32_t n_nodes, uint32_t n0,
                                                 const DevClass* __restrict__ cls, uint32_t n_cls, KCfg cfg, ExtDev e,
                                                 DevSum* __restrict__ out, uint32_t* __restrict__ cls_max) {
    // the partition tables in LDS: allocateByPartition walks them per class in a dependent chain of loads
    __shared__ kg_gpu_partition lparts[KG_GPU_MAX_PARTS];
    __shared__ uint32_t lrng[KG_GPU_MAX_TABLES * 9];
    if (e.parts) {
        const uint32_t np = min(e.n_parts, (uint32_t)KG_GPU_MAX_PARTS);
        for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) lparts[i] = e.parts[i];
        for (uint32_t i = threadIdx.x; i < (uint32_t)KG_GPU_MAX_TABLES * 9u; i += blockDim.x) lrng[i] = e.part_rng[i];
        __syncthreads();
        e.parts = lparts;
        e.part_rng = lrng;
    }
    const uint32_t rec0 = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = rec0 < n_nodes;
    const uint32_t rec = live ? rec0 : n_nodes - 1;  // dead lanes compute a copy for the wave reductions
    const DevRec& d = devs[rec];
    const int32_t D = (int32_t)nodes[rec].v[N_DEV_MINORS];
    const bool fbrec = live && rec < n0 && !((uint32_t)nodes[rec].v[N_FLAGS] & F_BIG) && D > 0;
    const uint64_t topo = zones[rec].dev_topo;
    const uint32_t part = zones[rec].dev_part;
    // the record's minors once, in registers (16-B loads; lanes are 384 B apart, so every load instruction
    // touches 64 lines: the per-class allocator reads them from here instead): free per (resource, minor), the
    // class-independent minor sets, the sums of the Score
    int64_t fr[DEV_R][DEV_MINORS];
    uint32_t used = 0u, total = 0u, nonzero = 0u;
    DevSum o;
#pragma unroll
    for (int r = 0; r < DEV_R; r++) {
        int64_t t = 0, f = 0;
#pragma unroll
        for (int m = 0; m < DEV_MINORS; m += 2) {
            const longlong2 tv = *reinterpret_cast<const longlong2*>(&d.total[r][m]);
            const longlong2 fv = *reinterpret_cast<const longlong2*>(&d.free_[r][m]);
            fr[r][m] = fv.x;
            fr[r][m + 1] = fv.y;
            t += tv.x + tv.y;
            f += fv.x + fv.y;
            const uint32_t b0 = m < D ? 1u << m : 0u, b1 = m + 1 < D ? 2u << m : 0u;
            used |= (fv.x != tv.x ? b0 : 0u) | (fv.y != tv.y ? b1 : 0u);
            total |= (tv.x != 0 ? b0 : 0u) | (tv.y != 0 ? b1 : 0u);
            nonzero |= (fv.x != 0 ? b0 : 0u) | (fv.y != 0 ? b1 : 0u);
        }
        o.T[r] = t;
        o.F[r] = f;
        o.rcp[r] = t != 0 ? 1.0 / (double)t : 0.0;
    }
    DevSum& w = out[rec];
    if (live) {
        for (int r = 0; r < DEV_R; r++) {
            w.T[r] = o.T[r];
            w.F[r] = o.F[r];
            w.rcp[r] = o.rcp[r];
        }
    }
    static_assert(DSUM_CHUNK == 8 && offsetof(DevSum, code) % 8 == 0 && offsetof(DevSum, score) % 8 == 0, "packed stores");
    const uint32_t nc = min(n_cls, (uint32_t)DEV_CLASSES);
    for (uint32_t k0 = 0; k0 < nc; k0 += DSUM_CHUNK) {
        uint64_t codes = 0, scores = 0;  // DSUM_CHUNK = 8 bytes each: one store per chunk
#pragma unroll 1
        for (uint32_t i = 0; i < DSUM_CHUNK; i++) {
            const uint32_t k = k0 + i;
            if (k >= nc) break;
            PodX x{};
            x.dkeys = cls[k].dkeys;
            x.dcount = cls[k].dcount;
            x.dflags = cls[k].dflags;
            x.dtmpl = cls[k].dtmpl;
            x.dbw = cls[k].dbw;
            for (int r = 0; r < DEV_R; r++) x.dreq[r] = cls[k].dreq[r];
            uint32_t le = 0u;
#pragma unroll
            for (int m = 0; m < DEV_MINORS; m++) {
                bool ok = m < D;
#pragma unroll
                for (int r = 0; r < DEV_R; r++) ok &= !(((x.dkeys >> r) & 1u) && x.dreq[r] > fr[r][m]);
                le |= ok ? 1u << m : 0u;
            }
            const GpuMinors g{used, total, total & le, nonzero & le};
            // D <= 0 never reads the code (the pair is decided first)
            const uint32_t code = D > 0 ? gpu_allocate_code(e, D, topo, part, x, g) : 0u;
            const uint32_t score = (uint32_t)dev_sum_score(cfg, &o, x);
            codes |= (uint64_t)(code & 0xFFu) << (8 * i);
            scores |= (uint64_t)(score & 0xFFu) << (8 * i);
            const int32_t best = wmax_i32((fbrec && code == 0u) ? (int32_t)score : 0);
            if (best > 0 && (threadIdx.x & 63u) == 0) atomicMax(cls_max + k, (uint32_t)best);
        }
        if (live) {
            *reinterpret_cast<uint64_t*>(&w.code[k0]) = codes;
            *reinterpret_cast<uint64_t*>(&w.score[k0]) = scores;
        }
    }
}

// GPU allocator outcome of every reservation restore table for every GPU request class of the batch (thread =
// (table, chunk of classes)): the view pairs of the select / stats kernels then read a code instead of running the allocator.
__global__ __launch_bounds__(256) void k_rdev_codes(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                    const DevRec* __restrict__ devs, const DevRec* __restrict__ rdev,
                                                    const uint32_t* __restrict__ rdev_rec, uint32_t n_rdev,
                                                    const DevClass* __restrict__ cls, uint32_t n_cls, KCfg cfg, ExtDev e,
                                                    uint8_t* __restrict__ out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_rdev) return;
    const uint32_t rec = rdev_rec[t];
    const int32_t D = (int32_t)nodes[rec].v[N_DEV_MINORS];
    const DevRec* tab = rdev + t;
    const uint32_t outside = D > 0 ? dev_outside_used(devs + rec, tab, D) : 0u;
    const uint32_t k0 = blockIdx.y * DSUM_CHUNK, k1 = min(k0 + DSUM_CHUNK, (uint32_t)DEV_CLASSES);
    for (uint32_t k = k0; k < k1; k++) {
        uint8_t code = 0;
        if (k < n_cls && D > 0) {
            PodX x{};
            x.dkeys = cls[k].dkeys;
            x.dcount = cls[k].dcount;
            x.dflags = cls[k].dflags;
            x.dtmpl = cls[k].dtmpl;
            x.dbw = cls[k].dbw;
            for (int r = 0; r < DEV_R; r++) x.dreq[r] = cls[k].dreq[r];
            code = (uint8_t)gpu_allocate(cfg, e, tab, D, zones[rec].dev_topo, zones[rec].dev_part, x, outside, false).code;
        }
        out[(size_t)t * DEV_CLASSES + k] = code;
    }
}

// gpu_zone_sum of every storage-class-1 record (SingleNUMANode, [n0, n_nodes)) for every GPU request class of the
// batch: thread = (record, class). The special-record kernels of a fast-base launch merge it into the fast block's
// zone walk (eval_c1) instead of running DeviceShare's hint provider per pair.
__global__ __launch_bounds__(64) void k_gpu_zone_sum(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                     const DevRec* __restrict__ devs, uint32_t n_nodes, uint32_t n0,
                                                     const DevClass* __restrict__ cls, KCfg cfg, ExtDev e,
                                                     uint64_t* __restrict__ out) {
    const uint32_t rec = n0 + blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t k = blockIdx.y;
    if (rec >= n_nodes) return;
    PodX x{};
    x.dkeys = cls[k].dkeys;
    x.dcount = cls[k].dcount;
    x.dflags = cls[k].dflags;
    x.dtmpl = cls[k].dtmpl;
    x.dbw = cls[k].dbw;
    for (int r = 0; r < DEV_R; r++) x.dreq[r] = cls[k].dreq[r];
    out[(size_t)(rec - n0) * DEV_CLASSES + k] = gpu_zone_sum(cfg, e, nodes[rec].v, zones + rec, devs + rec, x);
}

// Records the fast-base kernels (PART 1) take for no pod: F_BIG or storage class 1. special[0] = count,
// special[1..] = records (any order: keys are order-free). c1 (nullable): the storage-class-1 records that are not
// F_BIG go to their own list (c1[0] = count), for the light class-1 kernels (eval_c1); special then holds F_BIG only.
__global__ __launch_bounds__(256) void k_special_scan(const NodeRec* __restrict__ nodes, uint32_t n_nodes, uint32_t n0,
                                                      uint32_t* __restrict__ special, uint32_t* __restrict__ c1) {
    const uint32_t rec0 = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = rec0 < n_nodes;
    const uint32_t rec = live ? rec0 : 0u;  // every lane takes part in the ballots
    const int64_t* n = nodes[rec].v;
    const bool big = ((uint32_t)n[N_FLAGS] & F_BIG) != 0;
    const bool to_c1 = live && c1 && rec >= n0 && !big, to_sp = live && !to_c1 && (rec >= n0 || big);
    // one atomic per wave and list: the lanes' slots from the ballot's prefix counts
    const uint64_t bc = __ballot(to_c1), bs = __ballot(to_sp);
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t below = lane ? (~0ull >> (64u - lane)) : 0ull;
    const uint32_t leader_c = bc ? (uint32_t)__ffsll((unsigned long long)bc) - 1u : 64u;
    const uint32_t leader_s = bs ? (uint32_t)__ffsll((unsigned long long)bs) - 1u : 64u;
    uint32_t base_c = 0, base_s = 0;
    if (lane == leader_c) base_c = atomicAdd(c1, (uint32_t)__popcll(bc));
    if (lane == leader_s) base_s = atomicAdd(special, (uint32_t)__popcll(bs));
    base_c = __shfl(base_c, (int)(leader_c & 63u), 64);
    base_s = __shfl(base_s, (int)(leader_s & 63u), 64);
    if (to_c1) c1[1 + base_c + (uint32_t)__popcll(bc & below)] = rec;
    if (to_sp) special[1 + base_s + (uint32_t)__popcll(bs & below)] = rec;
}

// Weighted total of a fast-base pair (FB paths): base total from the fast block + the normalised
// DeviceShare term + the Reservation term, which off a view is 0 or the preferred node's 100 (total_ext
// with s_rsv = 0). mag = ceil(2^32 / dev_max) for dev_max >= 2: floor(s * 100 / dev_max) exactly for
// s * 100 <= 10^4 (the error term s * 100 * (mag * dev_max - 2^32) stays below 2^32).
__device__ __forceinline__ int64_t total_fb(const KCfg& c, uint64_t base_key, int64_t s_dev, uint32_t dm, uint32_t mag,
                                            uint32_t g, uint64_t pf) {
    const uint32_t n100 = (uint32_t)s_dev * 100u;
    const uint32_t nd = dm == 0 ? (uint32_t)s_dev : (dm == 1 ? n100 : __umulhi(n100, mag));
    const int64_t rsv = (pf != PREF_NONE && (uint32_t)pf == g) ? (int64_t)c.w_rsv * 100 : 0;
    return (int64_t)(base_key >> 32) + (int64_t)c.w_dev * nd + rsv;
}

__device__ __forceinline__ uint32_t norm_magic(uint32_t dm) {
    return dm >= 2 ? (uint32_t)(((1ull << 32) + dm - 1) / dm) : 0u;
}

// ElasticQuota PreFilter of every pod against the batch-start quota state (matrix mode).
__global__ __launch_bounds__(256) void k_ext_gate(PodsDev pods, uint32_t n_pods, ExtDev e, uint32_t plugins,
                                                  uint32_t* __restrict__ qst, uint32_t* __restrict__ pstat) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_pods) return;
    uint32_t s = 0;
    if (plugins & KG_PLUGIN_QUOTA) {
        const PodX x = load_podx(pods, j);
        if (x.quota >= 0 && (uint32_t)x.quota < e.n_quotas)
            s = quota_gate(e.qlim[x.quota], e.qstate[x.quota], load_pod(pods, j), x);
    }
    qst[j] = s;
    if (pstat) pstat[j] = s;  // a rejected pod is decided; the select kernels OR in KG_ST_UNSUPPORTED
}

// Verify: raw per-plugin results of every (pod, record) pair, [pod][snapshot index].
template <bool EXACT>
__global__ __launch_bounds__(256) void k_ext_verify_raw(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                        ExtDev e, PodsDev pods, uint32_t n_pods, uint32_t n_nodes, KCfg cfg,
                                                        const uint32_t* __restrict__ qst, ExtVerifyDev o) {
    const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= (size_t)n_pods * n_nodes) return;
    const uint32_t j = (uint32_t)(x / n_nodes), rec = (uint32_t)(x % n_nodes);
    const PodV p = load_pod(pods, j);
    const PodX px = load_podx(pods, j);
    const PairX r = eval_pair_ext<EXACT>(cfg, e, nodes[rec].v, zones + rec, dev_of(e, rec), rec, p, px, qst[j]);
    const size_t y = (size_t)j * n_nodes + node_index(nodes[rec]);
    o.status[y] = r.status;
    o.s_nrf[y] = r.s_nrf;
    o.s_la[y] = r.s_la;
    o.s_numa[y] = r.s_numa;
    o.s_dev[y] = r.s_dev;
    o.s_rsv[y] = r.s_rsv;
    o.order[y] = r.order;
    o.zone[y] = (int8_t)r.zone;
}

// Verify: per pod, PreScore preferredNode + NormalizeScore maxima, then the weighted totals.
__global__ __launch_bounds__(256) void k_ext_verify_fin(uint32_t n_pods, uint32_t n_nodes, uint32_t index_base, KCfg cfg,
                                                        ExtVerifyDev o) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_pods) return;
    const size_t row = (size_t)j * n_nodes;
    uint32_t dmax = 0, rmax = 0;
    uint64_t pref = PREF_NONE;
    for (uint32_t i = 0; i < n_nodes; i++) {
        if (o.status[row + i]) continue;
        dmax = max(dmax, (uint32_t)o.s_dev[row + i]);
        rmax = max(rmax, (uint32_t)o.s_rsv[row + i]);
        if (o.order[row + i] != 0) {
            const uint64_t k = pref_key(o.order[row + i], index_base + i);
            pref = k < pref ? k : pref;
        }
    }
    for (uint32_t i = 0; i < n_nodes; i++) {
        PairX r;
        r.status = o.status[row + i];
        if (r.status) {
            o.total[row + i] = -1;
            continue;
        }
        r.s_nrf = o.s_nrf[row + i];
        r.s_la = o.s_la[row + i];
        r.s_numa = o.s_numa[row + i];
        r.s_dev = o.s_dev[row + i];
        r.s_rsv = o.s_rsv[row + i];
        o.total[row + i] = total_ext(cfg, r, index_base + i, dmax, rmax, pref);
        if (pref != PREF_NONE && (uint32_t)pref == index_base + i) o.s_rsv[row + i] = 1000;
    }
}

// Pass 1: per-pod NormalizeScore inputs over the feasible nodes of records [lo, hi) of chunk blockIdx.y
// (fast-base batches: k_ext_stats_sp over the general records only; the fast-base records' DeviceShare
// maximum comes out of k_ext_select itself).
template <bool EXACT, bool TOPO>
__global__ __launch_bounds__(256) void k_ext_stats(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                   ExtDev e, PodsDev pods, const uint32_t* __restrict__ list,
                                                   uint32_t n_list, uint32_t n_nodes, uint32_t chunk, uint32_t index_base,
                                                   KCfg cfg, const uint32_t* __restrict__ qst, uint32_t* __restrict__ dev_max,
                                                   uint32_t* __restrict__ rsv_max, uint64_t* __restrict__ pref) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = t < n_list;
    const uint32_t j = live ? list[t] : 0;
    const PodV p = load_pod(pods, j);
    const PodX px = load_podx(pods, j);
    const uint32_t q = live ? qst[j] : 1u;
    const uint32_t lo = blockIdx.y * chunk, hi = min(n_nodes, lo + chunk);
    const uint32_t dcls = pods.dev_cls ? pods.dev_cls[j] : (uint32_t)DEV_CLASSES;
    uint32_t dmax = 0, rmax = 0;
    uint64_t pk = PREF_NONE;
    for (uint32_t rec = lo; rec < hi; rec++) {
        const PairX r = eval_pair_ext<EXACT, TOPO, false>(cfg, e, nodes[rec].v, zones + rec, dev_of(e, rec), rec, p, px, q, dcls);
        if (r.status) continue;
        dmax = max(dmax, (uint32_t)r.s_dev);
        rmax = max(rmax, (uint32_t)r.s_rsv);
        if (r.order != 0) {
            const uint64_t k = pref_key(r.order, index_base + node_index(nodes[rec]));
            pk = k < pk ? k : pk;
        }
    }
    if (!live) return;
    if (dmax) atomicMax(dev_max + j, dmax);
    if (rmax) atomicMax(rsv_max + j, rmax);
    if (pk != PREF_NONE) atomicMin((unsigned long long*)(pref + j), (unsigned long long)pk);
}

// The kernels around the whole evaluator (eval_pair_ext) need the full 256 VGPRs; its one accumulation register took
// them to one wave per SIMD, with every dependent load chain of the evaluator (views -> infos -> restore tables)
// exposed. Two waves per SIMD keep every register and hide half of that latency.
#define KG_EVAL_ATTR __attribute__((amdgpu_waves_per_eu(2, 2)))

// The records a fast-base pass leaves to the general path for lane t: the special records (F_BIG, and class
// 1 unless c1_split; grid-stride over chunks of `chunk`) for every lane, then the views of the lane's reservation
// class that are not in the special list, positions below lim. fn(rec, position) evaluates one pair.
template <typename Fn>
__device__ __forceinline__ void for_general_records(const NodeRec* __restrict__ nodes, const ExtDev& e,
                                                    const uint32_t* __restrict__ special, uint32_t n0, uint32_t chunk,
                                                    uint32_t by, int32_t cls, bool c1_split, uint32_t lim, Fn&& fn) {
    // one iteration space (the special list, then the class's views) and one call site of fn: with two, the
    // compiler outlined the evaluation lambda (an out-of-line call, its state through scratch memory)
    const uint32_t nsp = special[0], step = gridDim.y * chunk;
    uint32_t cb = 0, ce = 0;
    if (cls >= 0 && cls < RSV_MAX_CLASSES && e.cls_begin) {
        cb = e.cls_begin[cls];
        ce = e.cls_begin[cls + 1];
    }
    const uint32_t total = min(nsp + (ce - cb), lim);  // lim: the lane's positions end there
    for (uint32_t x = by * chunk; x < total; x += step)
        for (uint32_t u = x, ue = min(x + chunk, total); u < ue; u++) {
            uint32_t rec;
            if (u < nsp) {
                rec = special[1 + u];
            } else {
                rec = e.views[cb + (u - nsp)].rec;
                if (((uint32_t)nodes[rec].v[N_FLAGS] & F_BIG) || (rec >= n0 && !c1_split)) continue;  // special list
            }
            fn(rec, u);
        }
}

// The class-1 records of a split fast-base pass (k_special_scan's c1 list) for lane t, grid-stride over chunks.
template <typename Fn>
__device__ __forceinline__ void for_c1_records(const uint32_t* __restrict__ c1, uint32_t chunk, uint32_t by, Fn&& fn) {
    const uint32_t nc = c1[0], step = gridDim.y * chunk;
    for (uint32_t x = by * chunk; x < nc; x += step)
        for (uint32_t y = x, ye = min(x + chunk, nc); y < ye; y++) fn(c1[1 + y]);
}

// A storage-class-1 (SingleNUMANode) record of a fast-base launch for a pod off its reservation views, with DeviceShare's hints from e.gz: the fast block's base key (0 = infeasible with the
// NodeResourcesFit / LoadAware / NodeNUMAResource Filters, the quota gate or a required reservation affinity, as
// k_ext_select<FB> has them) and, when feasible, DeviceShare's Filter under the admitted zone and its raw score.
// Returns false when the pair takes the general path instead.
struct C1Pair {
    uint64_t bk;
    int64_t s_dev;
    uint32_t st, g;
};

__device__ __forceinline__ bool eval_c1(const KCfg& cfg, const KCfg& cv, const ExtDev& e, const int64_t* __restrict__ n,
                                        const ZoneRec* __restrict__ zr, uint32_t rec, uint32_t n0, const PodF& pff,
                                        const PodX& px, uint32_t dcls, uint32_t q, bool req_aff, uint32_t index_base,
                                        C1Pair& o) {
    const uint32_t fl = (uint32_t)n[N_FLAGS];
    if (rec < n0 || (fl & F_BIG)) return false;
    if ((cfg.plugins & KG_PLUGIN_RSV) && px.cls >= 0 && px.cls < RSV_MAX_CLASSES &&
        (((uint64_t)n[N_RSV_CLASSES] >> px.cls) & 1ull))
        return false;  // a view of the pod's class
    const FastRec fr = *reinterpret_cast<const FastRec*>(&n[FAST_BEGIN]);
    o.g = index_base + (uint32_t)((uint64_t)fr.flags >> 32);
    o.s_dev = 0;
    const bool dev = (cfg.plugins & KG_PLUGIN_DEV) && px.dcount != 0 && dcls < (uint32_t)DEV_CLASSES;
    if (!dev) {
        o.bk = eval_fast_key<7u, 1>(cv, fr, zr, pff, o.g);
        o.st = (o.bk == 0ull || q != 0u || req_aff) ? 1u : 0u;
        return true;
    }
    if (!e.gz) return false;  // (not in a split pass: k_special_scan splits only with the table or without GPU pods)
    const uint64_t gz = e.gz[(size_t)(rec - n0) * DEV_CLASSES + dcls];
    int32_t zone = -1;
    o.bk = eval_fast_key<7u, 1, true>(cv, fr, zr, pff, o.g, &zone, gz);
    o.st = (o.bk == 0ull || q != 0u || req_aff) ? 1u : 0u;
    if (o.st) return true;
    if (zone >= 0 && !(gz & GZ_NODEV)) {  // DeviceShare's Allocate under the admitted zone, its Score there
        o.st = ((gz >> (12 + zone)) & 1ull) ? 0u : 1u;
        o.s_dev = (int64_t)((gz >> (16 + 8 * zone)) & 0xFFull);
    } else {  // no affinity (one zone) or no provider: the allocation on the node's devices
        o.st = dev_eval_cls(n, e.dsum + rec, px, dcls, o.s_dev);
    }
    return true;
}

// Pass 1, general records of a fast-base launch (the complement of k_ext_stats<.., 1>).
__global__ __launch_bounds__(256) void k_ext_stats_sp(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                      ExtDev e, PodsDev pods, const uint32_t* __restrict__ list,
                                                      uint32_t n_list, uint32_t n0, uint32_t chunk, uint32_t index_base,
                                                      KCfg cfg, const uint32_t* __restrict__ qst,
                                                      uint32_t* __restrict__ dev_max, uint32_t* __restrict__ rsv_max,
                                                      uint64_t* __restrict__ pref, const uint32_t* __restrict__ special,
                                                      bool c1_split) {
    // launch order (not xcd_block): its work sits in the few pod blocks of the class pods, and whole chunks per XCD
    // measured slower (1.58 vs 1.13 ms on config 5)
    const GridBlock b{blockIdx.x, blockIdx.y};
    const uint32_t t = b.x * blockDim.x + threadIdx.x;
    const bool live = t < n_list;
    const uint32_t j = live ? list[t] : 0;
    const PodV p = load_pod(pods, j);
    const PodX px = load_podx(pods, j);
    const uint32_t q = live ? qst[j] : 1u;
    const uint32_t dcls = pods.dev_cls ? (uint32_t)pods.dev_cls[j] : (uint32_t)DEV_CLASSES;
    uint32_t dmax = 0, rmax = 0;
    uint64_t pk = PREF_NONE;
    const uint32_t xp = (e.xpairs && live) ? (e.xpos ? e.xpos[j] : j) : 0xFFFFFFFFu;
    uint64_t* const xcol = xp < e.xn ? e.xpairs + xp : nullptr;  // position u at xcol[u * xn]
    bool xlive = false;  // a pair the select pass must evaluate again (not stored, or outside the packing)
    for_general_records(nodes, e, special, n0, chunk, b.y, (cfg.plugins & KG_PLUGIN_RSV) ? px.cls : -1, c1_split, 0xFFFFFFFFu,
                        [&](uint32_t rec, uint32_t u) {
        // the whole pair (the select pass reads it back instead of evaluating it again)
        const PairX r = eval_pair_ext<false, false, true>(cfg, e, nodes[rec].v, zones + rec, dev_of(e, rec), rec, p, px, q,
                                                          dcls);
        if (xcol) {
            const uint64_t x = xpair_pack(cfg, r);
            if (u < e.xT) xcol[(size_t)u * e.xn] = x;
            xlive |= u >= e.xT || x == XPAIR_LIVE;
        }
        if (r.status) return;
        dmax = max(dmax, (uint32_t)r.s_dev);
        rmax = max(rmax, (uint32_t)r.s_rsv);
        if (r.order != 0) {
            const uint64_t k = pref_key(r.order, index_base + node_index(nodes[rec]));
            pk = k < pk ? k : pk;
        }
    });
    if (!live) return;
    if (xlive) xcol[(size_t)e.xT * e.xn] = 1ull;  // the lane's flag row (zeroed before the pass)
    if (dmax) atomicMax(dev_max + j, dmax);
    if (rmax) atomicMax(rsv_max + j, rmax);
    if (pk != PREF_NONE) atomicMin((unsigned long long*)(pref + j), (unsigned long long)pk);
}

// Pass 1, class-1 records of a split fast-base launch (k_special_scan's c1 list): eval_c1 with DeviceShare's hints
// from e.gz; a record holding a view of the pod's class is left to k_ext_stats_sp's view walk. Off a view the
// Reservation score and order are 0: only DeviceShare's maximum comes out.
__global__ __launch_bounds__(256) void k_ext_stats_c1(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                      ExtDev e, PodsDev pods, const uint32_t* __restrict__ list,
                                                      uint32_t n_list, uint32_t n0, uint32_t chunk, uint32_t index_base,
                                                      KCfg cfg, const uint32_t* __restrict__ qst,
                                                      uint32_t* __restrict__ dev_max, const uint32_t* __restrict__ c1) {
    const GridBlock b = xcd_block();  // whole record chunks per XCD (kg_eval.h)
    const uint32_t t = b.x * blockDim.x + threadIdx.x;
    const bool live = t < n_list;
    const uint32_t j = live ? list[t] : 0;
    const PodV p = load_pod(pods, j);
    const PodX px = load_podx(pods, j);
    if (!((cfg.plugins & KG_PLUGIN_DEV) && px.dcount != 0)) return;  // s_dev = 0 everywhere
    const uint32_t q = live ? qst[j] : 1u;
    const uint32_t dcls = pods.dev_cls ? (uint32_t)pods.dev_cls[j] : (uint32_t)DEV_CLASSES;
    const PodF pff = to_podf(p, cfg);
    const KCfg cv = cfg_in_vgprs(cfg);
    const bool req_aff = (cfg.plugins & KG_PLUGIN_RSV) && (p.flags & KG_POD_RSV_REQUIRED);
    uint32_t dmax = 0;
    for_c1_records(c1, chunk, b.y, [&](uint32_t rec) {
        C1Pair o;
        if (eval_c1(cfg, cv, e, nodes[rec].v, zones + rec, rec, n0, pff, px, dcls, q, req_aff, index_base, o) && !o.st)
            dmax = max(dmax, (uint32_t)o.s_dev);
    });
    if (live && dmax) atomicMax(dev_max + j, dmax);
}

// Pass 1 for pods without a GPU request: only the nodes holding a view of the pod's reservation class
// can carry a Reservation score or order, so lane t walks chunk b.y of that class's views
// (record order) instead of every record.
template <bool EXACT, bool TOPO>
__global__ __launch_bounds__(256) KG_EVAL_ATTR void k_ext_stats_views(const NodeRec* __restrict__ nodes,
                                                         const ZoneRec* __restrict__ zones, ExtDev e, PodsDev pods,
                                                         const uint32_t* __restrict__ list, uint32_t n_list,
                                                         uint32_t chunk, uint32_t index_base, KCfg cfg,
                                                         const uint32_t* __restrict__ qst,
                                                         uint32_t* __restrict__ rsv_max, uint64_t* __restrict__ pref) {
    const GridBlock b = xcd_block();  // whole view chunks per XCD (kg_eval.h)
    const uint32_t t = b.x * blockDim.x + threadIdx.x;
    if (t >= n_list) return;
    const uint32_t j = list[t];
    const PodV p = load_pod(pods, j);
    const PodX px = load_podx(pods, j);
    const uint32_t q = qst[j];
    if (q || px.cls < 0 || px.cls >= RSV_MAX_CLASSES) return;
    uint32_t rmax = 0;
    uint64_t pk = PREF_NONE;
    // stored pairs: position = the special list's length + the view's rank in its class (for_general_records)
    const uint32_t xp = (e.xpairs && e.xsp) ? (e.xpos ? e.xpos[j] : j) : 0xFFFFFFFFu;
    uint64_t* const xcol = xp < e.xn ? e.xpairs + xp : nullptr;  // position u at xcol[u * xn]
    const uint32_t nsp = xcol ? e.xsp[0] : 0u;
    const uint32_t dcls = pods.dev_cls ? (uint32_t)pods.dev_cls[j] : (uint32_t)DEV_CLASSES;
    bool xlive = false;  // as in k_ext_stats_sp
    const uint32_t cb = e.cls_begin[px.cls], ce = e.cls_begin[px.cls + 1];
    const uint32_t vb = cb + b.y * chunk, ve = min(ce, vb + chunk);
    for (uint32_t v = vb; v < ve; v++) {
        const uint32_t rec = e.views[v].rec;
        const PairX r = eval_pair_ext<EXACT, TOPO, true>(cfg, e, nodes[rec].v, zones + rec, dev_of(e, rec), rec, p, px, q,
                                                         dcls);
        if (xcol) {
            const uint64_t x = xpair_pack(cfg, r);
            const uint32_t u = nsp + (v - cb);
            if (u < e.xT) xcol[(size_t)u * e.xn] = x;
            xlive |= u >= e.xT || x == XPAIR_LIVE;
        }
        if (r.status) continue;
        rmax = max(rmax, (uint32_t)r.s_rsv);
        if (r.order != 0) {
            const uint64_t k = pref_key(r.order, index_base + node_index(nodes[rec]));
            pk = k < pk ? k : pk;
        }
    }
    if (xlive) xcol[(size_t)e.xT * e.xn] = 1ull;
    if (rmax) atomicMax(rsv_max + j, rmax);
    if (pk != PREF_NONE) atomicMin((unsigned long long*)(pref + j), (unsigned long long)pk);
}

template <int K>
__device__ __forceinline__ void topk_ins(uint64_t (&top)[K], uint64_t key) {
#pragma unroll
    for (int t = 0; t < K; t++) {
        const uint64_t cur = top[t];
        const bool gt = key > cur;
        top[t] = gt ? key : cur;
        key = gt ? cur : key;
    }
}

// Pass 2: weighted totals with the normalised DeviceShare / Reservation terms, top-K per (chunk, pod).
// FB (host: fast path valid, all three base plugins, no general topology manager): on class-0 records
// that are not F_BIG and hold no view of the lane's reservation class, the NodeResourcesFit / LoadAware
// / NodeNUMAResource part of the pair comes from the fast block (eval_fast_key, the base select's
// arithmetic: same feasibility and weighted total as eval_pair), and only DeviceShare, the
// reservation-affinity check and the normalised terms are evaluated on top.
template <int K, bool EXACT, bool TOPO, bool FB, int PART = 0>
__global__ __launch_bounds__(256, 3) void k_ext_select(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                    ExtDev e, PodsDev pods, const uint32_t* __restrict__ list,
                                                    uint32_t n_pods, uint32_t n_nodes, uint32_t n0,
                                                    uint32_t chunk, uint32_t index_base, KCfg cfg,
                                                    const uint32_t* __restrict__ qst, const uint32_t* __restrict__ dev_max,
                                                    const uint32_t* __restrict__ rsv_max, const uint64_t* __restrict__ pref,
                                                    uint64_t* __restrict__ partial, uint32_t* __restrict__ pstat) {
    // lane = row j of the output; the pod is list[j] (list == nullptr: the batch in order). Re-run launch
    // (e.rows): lane t takes row e.rows[t] of the *e.n_rows rows k_ext_fix_rows listed.
    constexpr bool FUSED = FB && PART == 1 && K == 1;  // top-1 straight into partial[row] by atomicMax
    const GridBlock b = xcd_block();
    const uint32_t t0 = b.x * blockDim.x + threadIdx.x;
    uint32_t j = t0;
    bool live = j < n_pods;
    if constexpr (FB) {
        if (e.rows) {
            const uint32_t nr = *e.n_rows, t = t0 + e.rows_from;
            if (b.x * blockDim.x + e.rows_from >= nr) return;  // whole workgroup idle (no barrier in this kernel)
            live = t < nr;
            j = live ? e.rows[t] : 0u;
        }
    }
    const uint32_t jj = live ? (list ? list[j] : j) : 0;
    const PodV p = load_pod(pods, jj);
    const PodX px = load_podx(pods, jj);
    const uint32_t q = live ? qst[jj] : 1u;
    const uint32_t rm = rsv_max[jj];
    uint32_t dm = dev_max[jj];
    const uint32_t dcls = pods.dev_cls ? pods.dev_cls[jj] : (uint32_t)DEV_CLASSES;
    // one-pass mode: the fast-base maximum is guessed as the class bound, the real one is collected
    const bool guess = FB && e.cls_max && (cfg.plugins & KG_PLUGIN_DEV) && px.dcount != 0 && dcls < (uint32_t)DEV_CLASSES;
    if (guess) dm = max(dm, e.cls_max[dcls]);
    uint32_t fbmax = 0;
    const uint64_t pf = pref[jj];
    uint64_t top[K];
#pragma unroll
    for (int t = 0; t < K; t++) top[t] = 0;
    const uint32_t lo = b.y * chunk, hi = min(n_nodes, lo + chunk);
    PodF pff{};
    KCfg cv = cfg;
    if constexpr (FB) {
        pff = to_podf(p, cfg);
        cv = cfg_in_vgprs(cfg);
    }
    const bool req_aff = (cfg.plugins & KG_PLUGIN_RSV) && (p.flags & KG_POD_RSV_REQUIRED);
    const uint32_t mag = norm_magic(dm);
    // pairs that need the host path come from eval_pair_ext only: FB records never do (a batch with a
    // cpuset-binding pod is not fast_ok, nodes with a CPU bind policy are F_BIG)
    uint32_t unsup = 0;
    for (uint32_t rec = lo; rec < hi; rec++) {
        const int64_t* __restrict__ n = nodes[rec].v;
        if constexpr (FB) {
            const uint32_t fl = (uint32_t)n[N_FLAGS];
            const bool view = (cfg.plugins & KG_PLUGIN_RSV) && px.cls >= 0 && px.cls < RSV_MAX_CLASSES &&
                              (((uint64_t)n[N_RSV_CLASSES] >> px.cls) & 1ull);
            const bool fbrec = rec < n0 && !(fl & F_BIG) && !view;
            if (PART == 1 && !fbrec) continue;
            if (fbrec) {
                const FastRec fr = *reinterpret_cast<const FastRec*>(&n[FAST_BEGIN]);
                const uint32_t g = index_base + (uint32_t)((uint64_t)fr.flags >> 32);
                const uint64_t bk = eval_fast_key<7u, 0>(cv, fr, zones + rec, pff, g);
                uint32_t st = (bk == 0ull || q != 0u || req_aff) ? 1u : 0u;
                int64_t s_dev = 0;
                if ((cfg.plugins & KG_PLUGIN_DEV) && !st)  // only the key's zero-ness matters once st != 0
                    st |= dev_eval_cls(n, e.dsum + rec, px, dcls, s_dev);
                if (!st) fbmax = max(fbmax, (uint32_t)s_dev);
                const int64_t tot = total_fb(cfg, bk, s_dev, dm, mag, g, pf);
                topk_ins<K>(top, st ? 0ull : (((uint64_t)tot << 32) | (uint64_t)(0xFFFFFFFFu - g)));
                continue;
            }
        }
        if constexpr (PART != 1) {
            const PairX r = eval_pair_ext<EXACT, TOPO>(cfg, e, n, zones + rec, dev_of(e, rec), rec, p, px, q, dcls);
            unsup |= r.status & KG_ST_UNSUPPORTED;
            const uint32_t g = index_base + node_index(nodes[rec]);
            const uint64_t key = ((uint64_t)total_ext(cfg, r, g, dm, rm, pf) << 32) | (uint64_t)(0xFFFFFFFFu - g);
            topk_ins<K>(top, r.status ? 0ull : key);
        }
    }
    if (live) {
        if constexpr (FUSED) {
            if (top[0]) atomicMax((unsigned long long*)(partial + j), (unsigned long long)top[0]);
        } else {
            uint64_t* dst = partial + ((size_t)b.y * n_pods + j) * K;
#pragma unroll
            for (int t = 0; t < K; t++) dst[t] = top[t];
        }
        if (unsup) atomicOr(pstat + jj, unsup);
        if (guess && fbmax) atomicMax(e.fb_max + jj, fbmax);
    }
}

// One-pass fast-base select: per GPU pod of the x list, the final DeviceShare maximum (general records' from
// pass 1, fast-base records' from k_ext_select) goes to dev_max for the general-record kernel; rows whose
// guessed maximum was not the final one are listed for a re-run (their fused key reset first). A pod the
// quota gate rejected or with a required reservation affinity has no feasible fast-base pair: any guess holds.
__global__ __launch_bounds__(256) void k_ext_fix_rows(PodsDev pods, const uint32_t* __restrict__ list, uint32_t n_pods,
                                                      ExtDev e, uint32_t plugins, const uint32_t* __restrict__ qst,
                                                      uint32_t* __restrict__ dev_max, uint32_t* __restrict__ rows,
                                                      uint32_t* __restrict__ n_rows, uint64_t* __restrict__ fused) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_pods || !(plugins & KG_PLUGIN_DEV)) return;
    const uint32_t jj = list ? list[j] : j;
    const PodX px = load_podx(pods, jj);
    const uint32_t dcls = pods.dev_cls ? pods.dev_cls[jj] : (uint32_t)DEV_CLASSES;
    if (px.dcount == 0 || dcls >= (uint32_t)DEV_CLASSES) return;
    const uint32_t gen = dev_max[jj], fin = max(gen, e.fb_max[jj]);
    dev_max[jj] = fin;
    const bool req_aff = (plugins & KG_PLUGIN_RSV) && (load_pod(pods, jj).flags & KG_POD_RSV_REQUIRED);
    if (qst[jj] != 0u || req_aff || fin == max(gen, e.cls_max[dcls])) return;
    if (fused) fused[j] = 0ull;
    rows[atomicAdd(n_rows, 1u)] = j;
}

// Pass 2, general records of a fast-base launch (the complement of k_ext_select<.., 1>), in two kernels: the pairs
// the statistics pass stored (k_ext_select_xs: a load and the weighted total, no evaluator in the kernel, so its
// occupancy is not the evaluator's one wave per SIMD) and the pairs evaluated here (k_ext_select_sp). A lane's stored
// column: a GPU pod's every general pair, a class pod's views (positions from the special list's length on); a pod its
// quota gate rejected was not evaluated there (its keys are 0, k_ext_gate wrote its status). The flag row (position xT)
// marks the lanes with a pair outside the stored form: k_ext_select_sp then takes the lane's every pair.
// Partials of chunk b.y go after the fast kernel's (part_off); top-1 is fused (partial = the keys by row).
struct XLane {
    const uint64_t* col;  // the lane's stored column (position u at col[u * xn]), nullptr = none
    bool all, flagged;    // every general pair stored (a GPU pod); a pair to evaluate again
};

__device__ __forceinline__ XLane xlane(const ExtDev& e, const PodX& px, uint32_t jj, bool live, uint32_t q) {
    XLane l{nullptr, false, false};
    const uint32_t xp = (e.xpairs && live && q == 0u) ? (e.xpos ? e.xpos[jj] : jj) : 0xFFFFFFFFu;
    if (xp < e.xn) {
        l.col = e.xpairs + xp;
        l.all = px.dcount > 0;
        l.flagged = l.col[(size_t)e.xT * e.xn] != 0ull;
    }
    return l;
}

template <int K>
__device__ __forceinline__ void put_partial(uint64_t* partial, const uint64_t (&top)[K], uint32_t j, uint32_t n_pods,
                                            uint32_t by, uint32_t part_off) {
    if constexpr (K == 1) {  // fused top-1 like k_ext_select<1, .., FB>
        if (top[0]) atomicMax((unsigned long long*)(partial + j), (unsigned long long)top[0]);
    } else {
        uint64_t* dst = partial + (((size_t)by + part_off) * n_pods + j) * K;
#pragma unroll
        for (int t = 0; t < K; t++) dst[t] = top[t];
    }
}

template <int K>
__global__ __launch_bounds__(256) void k_ext_select_xs(const NodeRec* __restrict__ nodes, ExtDev e, PodsDev pods,
                                                       const uint32_t* __restrict__ list, uint32_t n_pods, uint32_t n0,
                                                       uint32_t chunk, uint32_t index_base, KCfg cfg,
                                                       const uint32_t* __restrict__ qst,
                                                       const uint32_t* __restrict__ dev_max,
                                                       const uint32_t* __restrict__ rsv_max,
                                                       const uint64_t* __restrict__ pref, uint64_t* __restrict__ partial,
                                                       uint32_t* __restrict__ pstat, const uint32_t* __restrict__ special,
                                                       uint32_t part_off, bool c1_split) {
    const GridBlock b = xcd_block();
    const uint32_t j = b.x * blockDim.x + threadIdx.x;
    const bool live = j < n_pods;
    const uint32_t jj = live ? (list ? list[j] : j) : 0;
    const PodX px = load_podx(pods, jj);
    const uint32_t q = live ? qst[jj] : 1u;
    const XLane l = xlane(e, px, jj, live, q);
    uint64_t top[K];
#pragma unroll
    for (int t = 0; t < K; t++) top[t] = 0;
    uint32_t unsup = 0;
    if (l.col && !l.flagged) {
        const uint32_t dm = dev_max[jj], rm = rsv_max[jj];
        const uint64_t pf = pref[jj];
        const uint32_t nsp = special[0];
        for_general_records(nodes, e, special, n0, chunk, b.y, (cfg.plugins & KG_PLUGIN_RSV) ? px.cls : -1, c1_split,
                            0xFFFFFFFFu, [&](uint32_t rec, uint32_t u) {
            if (!l.all && u < nsp) return;  // k_ext_select_sp's
            const uint64_t x = l.col[(size_t)u * e.xn];
            if (!(x >> 63)) {  // infeasible (XPAIR_LIVE only in flagged lanes)
                unsup |= x == XPAIR_UNSUP ? (uint32_t)KG_ST_UNSUPPORTED : 0u;
                return;
            }
            const uint32_t g = index_base + node_index(nodes[rec]);
            topk_ins<K>(top, ((uint64_t)total_xpair(cfg, x, g, dm, rm, pf) << 32) | (uint64_t)(0xFFFFFFFFu - g));
        });
    }
    if (live) {
        put_partial<K>(partial, top, j, n_pods, b.y, part_off);
        if (unsup) atomicOr(pstat + jj, unsup);
    }
}

template <int K>
__global__ __launch_bounds__(256) KG_EVAL_ATTR void k_ext_select_sp(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                       ExtDev e, PodsDev pods, const uint32_t* __restrict__ list,
                                                       uint32_t n_pods, uint32_t n0, uint32_t chunk, uint32_t index_base,
                                                       KCfg cfg, const uint32_t* __restrict__ qst,
                                                       const uint32_t* __restrict__ dev_max,
                                                       const uint32_t* __restrict__ rsv_max,
                                                       const uint64_t* __restrict__ pref, uint64_t* __restrict__ partial,
                                                       uint32_t* __restrict__ pstat, const uint32_t* __restrict__ special,
                                                       uint32_t part_off, bool c1_split) {
    const GridBlock b = xcd_block();
    const uint32_t j = b.x * blockDim.x + threadIdx.x;
    const bool live = j < n_pods;
    const uint32_t jj = live ? (list ? list[j] : j) : 0;
    const PodV p = load_pod(pods, jj);
    const PodX px = load_podx(pods, jj);
    const uint32_t q = live ? qst[jj] : 1u;
    const XLane l = xlane(e, px, jj, live, q);
    uint64_t top[K];
#pragma unroll
    for (int t = 0; t < K; t++) top[t] = 0;
    uint32_t unsup = 0;
    const uint32_t nsp = special[0];
    // a flagged or unstored lane: every pair (the stored ones read back); a stored class pod: its special-list pairs
    const uint32_t lim = (q != 0u || !live) ? 0u : (l.col && !l.flagged) ? (l.all ? 0u : nsp) : 0xFFFFFFFFu;
    if (lim) {
        const uint32_t dm = dev_max[jj], rm = rsv_max[jj];
        const uint64_t pf = pref[jj];
        const uint32_t dcls = pods.dev_cls ? (uint32_t)pods.dev_cls[jj] : (uint32_t)DEV_CLASSES;
        for_general_records(nodes, e, special, n0, chunk, b.y, (cfg.plugins & KG_PLUGIN_RSV) ? px.cls : -1, c1_split, lim,
                            [&](uint32_t rec, uint32_t u) {
            const uint64_t x = (l.col && u < e.xT && (l.all || u >= nsp)) ? l.col[(size_t)u * e.xn] : XPAIR_LIVE;
            const uint32_t g = index_base + node_index(nodes[rec]);
            uint64_t key = 0;
            if (x >> 63) {
                key = ((uint64_t)total_xpair(cfg, x, g, dm, rm, pf) << 32) | (uint64_t)(0xFFFFFFFFu - g);
            } else if (x == XPAIR_LIVE) {
                const PairX r = eval_pair_ext<false, false>(cfg, e, nodes[rec].v, zones + rec, dev_of(e, rec), rec, p, px,
                                                            q, dcls);
                unsup |= r.status & KG_ST_UNSUPPORTED;
                key = r.status ? 0ull : ((uint64_t)total_ext(cfg, r, g, dm, rm, pf) << 32) | (uint64_t)(0xFFFFFFFFu - g);
            } else if (x == XPAIR_UNSUP) {
                unsup |= KG_ST_UNSUPPORTED;
            }
            topk_ins<K>(top, key);
        });
    }
    if (live) {
        put_partial<K>(partial, top, j, n_pods, b.y, part_off);
        if (unsup) atomicOr(pstat + jj, unsup);
    }
}

// Pass 2, class-1 records of a split fast-base launch (the light complement of k_ext_select_sp): eval_c1 per pair,
// a record holding a view of the pod's class left to k_ext_select_sp's view walk. Partials of chunk b.y go
// after part_off; top-1 is fused.
template <int K>
__global__ __launch_bounds__(256) void k_ext_select_c1(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                       ExtDev e, PodsDev pods, const uint32_t* __restrict__ list,
                                                       uint32_t n_pods, uint32_t n0, uint32_t chunk, uint32_t index_base,
                                                       KCfg cfg, const uint32_t* __restrict__ qst,
                                                       const uint32_t* __restrict__ dev_max, const uint64_t* __restrict__ pref,
                                                       uint64_t* __restrict__ partial, const uint32_t* __restrict__ c1,
                                                       uint32_t part_off) {
    const GridBlock b = xcd_block();  // whole record chunks per XCD (kg_eval.h)
    uint32_t j = b.x * blockDim.x + threadIdx.x;
    bool live = j < n_pods;
    if (e.rows) {  // re-run of the rows k_ext_fix_rows listed (top-1), as k_ext_select<FB>'s
        const uint32_t nr = *e.n_rows, t = j + e.rows_from;
        if (b.x * blockDim.x + e.rows_from >= nr) return;  // whole workgroup idle (no barrier in this kernel)
        live = t < nr;
        j = live ? e.rows[t] : 0u;
    }
    const uint32_t jj = live ? (list ? list[j] : j) : 0;
    const PodV p = load_pod(pods, jj);
    const PodX px = load_podx(pods, jj);
    const uint32_t q = live ? qst[jj] : 1u;
    uint32_t dm = dev_max[jj];
    const uint64_t pf = pref[jj];
    const uint32_t dcls = pods.dev_cls ? (uint32_t)pods.dev_cls[jj] : (uint32_t)DEV_CLASSES;
    // beside the one-pass select: the same guessed maximum (its wrong rows are re-run after k_ext_fix_rows)
    if (e.cls_max && (cfg.plugins & KG_PLUGIN_DEV) && px.dcount != 0 && dcls < (uint32_t)DEV_CLASSES)
        dm = max(dm, e.cls_max[dcls]);
    const PodF pff = to_podf(p, cfg);
    const KCfg cv = cfg_in_vgprs(cfg);
    const bool req_aff = (cfg.plugins & KG_PLUGIN_RSV) && (p.flags & KG_POD_RSV_REQUIRED);
    const uint32_t mag = norm_magic(dm);
    uint64_t top[K];
#pragma unroll
    for (int t = 0; t < K; t++) top[t] = 0;
    for_c1_records(c1, chunk, b.y, [&](uint32_t rec) {
        C1Pair o;
        if (!eval_c1(cfg, cv, e, nodes[rec].v, zones + rec, rec, n0, pff, px, dcls, q, req_aff, index_base, o)) return;
        const int64_t tot = total_fb(cfg, o.bk, o.s_dev, dm, mag, o.g, pf);
        topk_ins<K>(top, o.st ? 0ull : (((uint64_t)tot << 32) | (uint64_t)(0xFFFFFFFFu - o.g)));
    });
    if (!live) return;
    if constexpr (K == 1) {
        if (top[0]) atomicMax((unsigned long long*)(partial + j), (unsigned long long)top[0]);
    } else {
        uint64_t* dst = partial + (((size_t)b.y + part_off) * n_pods + j) * K;
#pragma unroll
        for (int t = 0; t < K; t++) dst[t] = top[t];
    }
}

// Rows of a sub-batch select (plain pods / config-5 pods) back to their batch positions; a pod the
// ElasticQuota PreFilter rejected has no feasible node.
__global__ __launch_bounds__(256) void k_scatter_keys(const uint64_t* src, const uint32_t* __restrict__ map,
                                                      uint32_t n, uint32_t k, bool src_by_map, const uint32_t* __restrict__ qst,
                                                      uint64_t* out, uint32_t* __restrict__ pstat) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint32_t j = map[t];
    const bool rejected = qst && qst[j] != 0;
    const size_t r = src_by_map ? j : t;
    for (uint32_t i = 0; i < k; i++) out[(size_t)j * k + i] = rejected ? 0ull : src[r * k + i];
    if (rejected && pstat) pstat[j] = qst[j];
}

// ------------------------------------------------------------------------------------------------
// launchers

static uint32_t env_u32(const char* name, uint32_t dflt) {
    const char* v = std::getenv(name);
    return v ? (uint32_t)std::strtoul(v, nullptr, 10) : dflt;
}

hipError_t launch_ext_gate(const PodsDev& pods, uint32_t n_pods, const ExtDev& e, uint32_t plugins, uint32_t* qst,
                           uint32_t* pstat, hipStream_t s) {
    if (n_pods == 0) return hipSuccess;
    k_ext_gate<<<(n_pods + 255) / 256, 256, 0, s>>>(pods, n_pods, e, plugins, qst, pstat);
    return hipGetLastError();
}

hipError_t launch_ext_verify(const NodeRec* nodes, const ZoneRec* zones, const ExtDev& e, const PodsDev& pods,
                             uint32_t n_pods, uint32_t n_nodes, uint32_t index_base, const KCfg& cfg, bool exact,
                             const uint32_t* qst, const ExtVerifyDev& o, hipStream_t s) {
    const size_t pairs = (size_t)n_pods * n_nodes;
    if (pairs == 0) return hipSuccess;
    dim3 grid((unsigned)((pairs + 255) / 256));
    if (exact)
        k_ext_verify_raw<true><<<grid, 256, 0, s>>>(nodes, zones, e, pods, n_pods, n_nodes, cfg, qst, o);
    else
        k_ext_verify_raw<false><<<grid, 256, 0, s>>>(nodes, zones, e, pods, n_pods, n_nodes, cfg, qst, o);
    k_ext_verify_fin<<<(n_pods + 255) / 256, 256, 0, s>>>(n_pods, n_nodes, index_base, cfg, o);
    return hipGetLastError();
}

// An error after the fork of a side lane: its kernels may still run with no join back into the main stream, so the
// lane is drained before the error goes up (the caller may free the buffers they write).
static hipError_t drain_lane(const SideLane* lane, hipError_t err) {
    hipStreamSynchronize(lane->s);
    return err;
}

hipError_t launch_ext_stats(const NodeRec* nodes, const ZoneRec* zones, const ExtDev& e, const PodsDev& pods,
                            const uint32_t* list, uint32_t n_list, uint32_t n_nodes, uint32_t n0, uint32_t chunk,
                            uint32_t index_base, const KCfg& cfg, bool exact, bool topo, bool fb, const uint32_t* qst,
                            uint32_t* dev_max, uint32_t* rsv_max, uint64_t* pref, const uint32_t* special,
                            uint32_t special_est, const uint32_t* c1, uint32_t c1_est, hipStream_t s, const SideLane* lane) {
    if (n_list == 0 || n_nodes == 0) return hipSuccess;
    dim3 grid((n_list + 255) / 256, (n_nodes + chunk - 1) / chunk);
    if (fb) {  // the general records only (the fast-base records' maximum: k_ext_select)
        // the class-1 kernel on the side lane beside the general one (both only atomicMax / atomicMin per pod)
        const bool two = c1 && lane && lane->s && lane->fork && lane->join;
        hipStream_t s3 = two ? lane->s : s;
        if (two) {
            hipError_t err = hipEventRecord(lane->fork, s);
            if (err == hipSuccess) err = hipStreamWaitEvent(lane->s, lane->fork, 0);
            if (err != hipSuccess) return err;
        }
        if (c1) {
            uint32_t chunk3, y3;
            ext_part2_grid(c1_est, grid.x, &chunk3, &y3);
            k_ext_stats_c1<<<dim3(grid.x, y3), 256, 0, s3>>>(nodes, zones, e, pods, list, n_list, n0, chunk3, index_base, cfg,
                                                             qst, dev_max, c1);
            if (two) {
                hipError_t err = hipEventRecord(lane->join, lane->s);
                if (err != hipSuccess) return drain_lane(lane, err);
            }
        }
        uint32_t chunk2, y2;
        // short chunks: a wave's pairs run one after another, each a chain of dependent loads through the views, the
        // reservations and their GPU tables (config 5: ~8k workgroups of 3 positions 0.60 ms, ~2k of 9 1.12 ms)
        ext_part2_grid(special_est, grid.x, &chunk2, &y2, env_u32("KG_SP_TARGET", 8192u), env_u32("KG_SP_MIN", 1u));
        k_ext_stats_sp<<<dim3(grid.x, y2), 256, 0, s>>>(nodes, zones, e, pods, list, n_list, n0, chunk2, index_base, cfg,
                                                        qst, dev_max, rsv_max, pref, special, c1 != nullptr);
        if (two) {
            hipError_t err = hipStreamWaitEvent(s, lane->join, 0);
            if (err != hipSuccess) return drain_lane(lane, err);
        }
        return hipGetLastError();
    }
#define KG_EXT_ST(EX, TP)                                                                                              \
    k_ext_stats<EX, TP><<<grid, 256, 0, s>>>(nodes, zones, e, pods, list, n_list, n_nodes, chunk, index_base, cfg, qst, \
                                             dev_max, rsv_max, pref)
    if (exact) {
        if (topo) KG_EXT_ST(true, true);
        else KG_EXT_ST(true, false);
    } else {
        if (topo) KG_EXT_ST(false, true);
        else KG_EXT_ST(false, false);
    }
#undef KG_EXT_ST
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_max_fold(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = max(dst[i], src[i]);
}

hipError_t launch_max_fold(uint32_t* dst, const uint32_t* src, uint32_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    k_max_fold<<<(n + 255) / 256, 256, 0, s>>>(dst, src, n);
    return hipGetLastError();
}

hipError_t launch_special_scan(const NodeRec* nodes, uint32_t n_nodes, uint32_t n0, uint32_t* special, uint32_t* c1,
                               hipStream_t s) {
    hipError_t e = hipMemsetAsync(special, 0, sizeof(uint32_t), s);
    if (e == hipSuccess && c1) e = hipMemsetAsync(c1, 0, sizeof(uint32_t), s);
    if (e != hipSuccess || n_nodes == 0) return e;
    k_special_scan<<<(n_nodes + 255) / 256, 256, 0, s>>>(nodes, n_nodes, n0, special, c1);
    return hipGetLastError();
}

hipError_t launch_rdev_codes(const NodeRec* nodes, const ZoneRec* zones, const DevRec* devs, const DevRec* rdev,
                             const uint32_t* rdev_rec, uint32_t n_rdev, const DevClass* cls, uint32_t n_cls,
                             const KCfg& cfg, const ExtDev& e, uint8_t* out, hipStream_t s) {
    if (n_rdev == 0) return hipSuccess;
    const uint32_t chunks = ((uint32_t)DEV_CLASSES + DSUM_CHUNK - 1) / DSUM_CHUNK;
    k_rdev_codes<<<dim3((n_rdev + 63) / 64, chunks), 64, 0, s>>>(nodes, zones, devs, rdev, rdev_rec, n_rdev, cls, n_cls, cfg, e,
                                                                 out);
    return hipGetLastError();
}

hipError_t launch_gpu_zone_sum(const NodeRec* nodes, const ZoneRec* zones, const DevRec* devs, uint32_t n_nodes,
                               uint32_t n0, const DevClass* cls, uint32_t n_cls, const KCfg& cfg, const ExtDev& e,
                               uint64_t* out, hipStream_t s) {
    if (n_nodes <= n0 || n_cls == 0) return hipSuccess;
    k_gpu_zone_sum<<<dim3((n_nodes - n0 + 63) / 64, std::min<uint32_t>(n_cls, (uint32_t)DEV_CLASSES)), 64, 0, s>>>(
        nodes, zones, devs, n_nodes, n0, cls, cfg, e, out);
    return hipGetLastError();
}

hipError_t launch_dev_sum(const NodeRec* nodes, const ZoneRec* zones, const DevRec* devs, uint32_t n_nodes, uint32_t n0,
                          const DevClass* cls, uint32_t n_cls, const KCfg& cfg, const ExtDev& e, DevSum* out,
                          uint32_t* cls_max, hipStream_t s, bool zero_cls_max) {
    hipError_t err = zero_cls_max ? hipMemsetAsync(cls_max, 0, sizeof(uint32_t) * DEV_CLASSES, s) : hipSuccess;
    if (err != hipSuccess || n_nodes == 0) return err;
    // the batch's classes only (a class's code / score is read only by pods of that class)
    k_dev_sum<<<(n_nodes + 255) / 256, 256, 0, s>>>(nodes, zones, devs, n_nodes, n0, cls, n_cls, cfg, e, out,
                                                                  cls_max);
    return hipGetLastError();
}

hipError_t launch_scatter_keys(const uint64_t* src, const uint32_t* map, uint32_t n, uint32_t k, bool src_by_map,
                               const uint32_t* qst, uint64_t* out, uint32_t* pstat, hipStream_t s) {
    if (n == 0) return hipSuccess;
    k_scatter_keys<<<(n + 255) / 256, 256, 0, s>>>(src, map, n, k, src_by_map, qst, out, pstat);
    return hipGetLastError();
}

hipError_t launch_ext_stats_views(const NodeRec* nodes, const ZoneRec* zones, const ExtDev& e, const PodsDev& pods,
                                  const uint32_t* list, uint32_t n_list, uint32_t max_views, uint32_t index_base,
                                  const KCfg& cfg, bool exact,
                                  bool topo, const uint32_t* qst, uint32_t* dev_max, uint32_t* rsv_max, uint64_t* pref,
                                  hipStream_t s) {
    (void)dev_max;  // no GPU request: the DeviceShare maximum stays 0
    if (n_list == 0 || max_views == 0) return hipSuccess;
    // split every class's views over enough chunks to fill the chip (~2048 workgroups)
    const uint32_t pod_blocks = (n_list + 255) / 256;
    const uint32_t want = std::max<uint32_t>(1, env_u32("KG_SV_TARGET", 2048u) / pod_blocks);
    const uint32_t chunk = std::max<uint32_t>(env_u32("KG_SV_MIN", 4u), (max_views + want - 1) / want);
    dim3 grid(pod_blocks, (max_views + chunk - 1) / chunk);
#define KG_EXT_SV(EX, TP)                                                                                        \
    k_ext_stats_views<EX, TP><<<grid, 256, 0, s>>>(nodes, zones, e, pods, list, n_list, chunk, index_base, cfg, qst, \
                                                   rsv_max, pref)
    if (exact) {
        if (topo) KG_EXT_SV(true, true);
        else KG_EXT_SV(true, false);
    } else {
        if (topo) KG_EXT_SV(false, true);
        else KG_EXT_SV(false, false);
    }
#undef KG_EXT_SV
    return hipGetLastError();
}

hipError_t launch_ext_select(const NodeRec* nodes, const ZoneRec* zones, const ExtDev& e, const PodsDev& pods,
                             const uint32_t* list, uint32_t n_pods, uint32_t n_nodes, uint32_t n0, uint32_t chunk, uint32_t k,
                             uint32_t index_base, const KCfg& cfg, bool exact, bool topo, bool fb, const uint32_t* qst, const uint32_t* dev_max,
                             const uint32_t* rsv_max, const uint64_t* pref, uint64_t* partial, uint32_t* pstat, hipStream_t s) {
    if (n_pods == 0 || n_nodes == 0) return hipSuccess;
    dim3 grid((n_pods + 255) / 256, (n_nodes + chunk - 1) / chunk);
#define KG_EXT_SEL(KK, EX, TP, F, ...)                                                                       \
    k_ext_select<KK, EX, TP, F, ##__VA_ARGS__><<<grid, 256, 0, s>>>(nodes, zones, e, pods, list, n_pods, n_nodes, n0, chunk, index_base, \
                                                     cfg, qst, dev_max, rsv_max, pref, partial, pstat)
#define KG_EXT_SEL_K(KK)                              \
    if (fb) {                                         \
        KG_EXT_SEL(KK, false, false, true, 1);        \
    } else if (exact) {                               \
        if (topo) KG_EXT_SEL(KK, true, true, false);  \
        else KG_EXT_SEL(KK, true, false, false);      \
    } else {                                          \
        if (topo) KG_EXT_SEL(KK, false, true, false); \
        else KG_EXT_SEL(KK, false, false, false);     \
    }
    if (k == 1) {
        KG_EXT_SEL_K(1)
    } else {
        KG_EXT_SEL_K(KG_TOPK_MAX)
    }
#undef KG_EXT_SEL_K
#undef KG_EXT_SEL
    return hipGetLastError();
}

hipError_t launch_ext_fix(const NodeRec* nodes, const ZoneRec* zones, const ExtDev& e, const PodsDev& pods,
                          const uint32_t* list, uint32_t n_pods, uint32_t n_nodes, uint32_t n0, uint32_t chunk, uint32_t k,
                          uint32_t index_base, const KCfg& cfg, const uint32_t* qst, uint32_t* dev_max,
                          const uint32_t* rsv_max, const uint64_t* pref, uint64_t* partial, uint32_t* pstat,
                          uint32_t* rows, uint32_t* n_rows, hipStream_t s) {
    if (n_pods == 0 || n_nodes == 0) return hipSuccess;
    hipError_t err = hipMemsetAsync(n_rows, 0, sizeof(uint32_t), s);
    if (err != hipSuccess) return err;
    k_ext_fix_rows<<<(n_pods + 255) / 256, 256, 0, s>>>(pods, list, n_pods, e, cfg.plugins, qst, dev_max, rows, n_rows,
                                                        k == 1 ? partial : nullptr);
    ExtDev f = e;
    f.cls_max = nullptr;
    f.rows = rows;
    f.n_rows = n_rows;
    f.rows_from = 0;
    if (k == 1) {
        // a handful of rows (the guesses the class bound missed): the launch takes as long as one workgroup's walk of
        // its record chunk, so the first 256 rows go over short chunks in one pod block, the rest (if any) as before
        const uint32_t c1 = std::max<uint32_t>(16u, chunk / 8u), gx = (n_pods + 255) / 256;
        k_ext_select<1, false, false, true, 1><<<dim3(1, (n_nodes + c1 - 1) / c1), 256, 0, s>>>(
            nodes, zones, f, pods, list, n_pods, n_nodes, n0, c1, index_base, cfg, qst, dev_max, rsv_max, pref, partial, pstat);
        if (gx > 1) {
            f.rows_from = 256;
            k_ext_select<1, false, false, true, 1><<<dim3(gx - 1, (n_nodes + chunk - 1) / chunk), 256, 0, s>>>(
                nodes, zones, f, pods, list, n_pods, n_nodes, n0, chunk, index_base, cfg, qst, dev_max, rsv_max, pref, partial,
                pstat);
        }
        return hipGetLastError();
    }
    return launch_ext_select(nodes, zones, f, pods, list, n_pods, n_nodes, n0, chunk, k, index_base, cfg, false, false, true,
                             qst, dev_max, rsv_max, pref, partial, pstat, s);
}

hipError_t launch_ext_select_c1_top1(const NodeRec* nodes, const ZoneRec* zones, const ExtDev& e, const PodsDev& pods,
                                     const uint32_t* list, uint32_t n_pods, uint32_t n0, uint32_t index_base, const KCfg& cfg,
                                     const uint32_t* qst, const uint32_t* dev_max, const uint64_t* pref, uint64_t* keys,
                                     const uint32_t* c1, uint32_t c1_est, hipStream_t s) {
    if (n_pods == 0 || !c1) return hipSuccess;
    const uint32_t gx = (n_pods + 255) / 256;
    uint32_t chunk3, y3;
    ext_part2_grid(c1_est, gx, &chunk3, &y3);
    if (!e.rows) {
        k_ext_select_c1<1><<<dim3(gx, y3), 256, 0, s>>>(nodes, zones, e, pods, list, n_pods, n0, chunk3, index_base, cfg, qst,
                                                        dev_max, pref, keys, c1, 0);
        return hipGetLastError();
    }
    // re-run rows: the first 256 over short chunks in one pod block (as launch_ext_fix), the rest as before
    ExtDev f = e;
    f.rows_from = 0;
    uint32_t cs, ys;
    ext_part2_grid(c1_est, 1, &cs, &ys, 4096u, 8u);
    k_ext_select_c1<1><<<dim3(1, ys), 256, 0, s>>>(nodes, zones, f, pods, list, n_pods, n0, cs, index_base, cfg, qst, dev_max,
                                                   pref, keys, c1, 0);
    if (gx > 1) {
        f.rows_from = 256;
        k_ext_select_c1<1><<<dim3(gx - 1, y3), 256, 0, s>>>(nodes, zones, f, pods, list, n_pods, n0, chunk3, index_base, cfg,
                                                            qst, dev_max, pref, keys, c1, 0);
    }
    return hipGetLastError();
}

hipError_t launch_ext_select_sp(const NodeRec* nodes, const ZoneRec* zones, const ExtDev& e, const PodsDev& pods,
                                const uint32_t* list, uint32_t n_pods, uint32_t n_nodes, uint32_t n0, uint32_t chunk, uint32_t k,
                                uint32_t index_base, const KCfg& cfg, const uint32_t* qst, const uint32_t* dev_max,
                                const uint32_t* rsv_max, const uint64_t* pref, uint64_t* partial, uint32_t* pstat,
                                const uint32_t* special, uint32_t special_est, const uint32_t* c1, uint32_t c1_est, uint32_t live_est,
                                bool c1_split, hipStream_t s, const SideLane* lane) {
    if (n_pods == 0 || n_nodes == 0) return hipSuccess;
    const uint32_t gx = (n_pods + 255) / 256, y1 = (n_nodes + chunk - 1) / chunk;
    uint32_t chunk2, y2, chunk3 = 0, y3 = 0;
    ext_part2_grid(special_est, gx, &chunk2, &y2);
    if (c1) ext_part2_grid(c1_est, gx, &chunk3, &y3);
    const bool sp = c1_split;  // (c1 == nullptr with c1_split: k_ext_select_c1 ran beside the one-pass select)
    // the class-1 kernel on the side lane beside the general one (disjoint partial rows: y1 + y2 on)
    const bool two = c1 && lane && lane->s && lane->fork && lane->join;
    hipStream_t s3 = two ? lane->s : s;
    if (two) {
        hipError_t err = hipEventRecord(lane->fork, s);
        if (err == hipSuccess) err = hipStreamWaitEvent(lane->s, lane->fork, 0);
        if (err != hipSuccess) return err;
    }
    if (c1) {
        if (k == 1)
            k_ext_select_c1<1><<<dim3(gx, y3), 256, 0, s3>>>(nodes, zones, e, pods, list, n_pods, n0, chunk3, index_base, cfg,
                                                             qst, dev_max, pref, partial, c1, y1 + y2);
        else
            k_ext_select_c1<KG_TOPK_MAX><<<dim3(gx, y3), 256, 0, s3>>>(nodes, zones, e, pods, list, n_pods, n0, chunk3,
                                                                       index_base, cfg, qst, dev_max, pref, partial, c1,
                                                                       y1 + y2);
        if (two) {
            hipError_t err = hipEventRecord(lane->join, lane->s);
            if (err != hipSuccess) return drain_lane(lane, err);
        }
    }
    // the stored pairs (rows y1..), then the ones evaluated here (rows after the class-1 kernel's) over a grid sized
    // for live_est positions (with stored pairs: the special list; the kernel's 256-VGPR workgroups would otherwise
    // queue behind the class-1 kernel on the side lane only to find nothing to do)
    const uint32_t y4 = y1 + y2 + y3;
    uint32_t chunk5, y5;
    ext_part2_grid(live_est, gx, &chunk5, &y5);
    if (k == 1) {
        if (e.xpairs)
            k_ext_select_xs<1><<<dim3(gx, y2), 256, 0, s>>>(nodes, e, pods, list, n_pods, n0, chunk2, index_base, cfg, qst,
                                                            dev_max, rsv_max, pref, partial, pstat, special, y1, sp);
        k_ext_select_sp<1><<<dim3(gx, y5), 256, 0, s>>>(nodes, zones, e, pods, list, n_pods, n0, chunk5, index_base, cfg, qst,
                                                        dev_max, rsv_max, pref, partial, pstat, special, y4, sp);
    } else {
        // (without stored pairs it writes its rows' zero keys)
        k_ext_select_xs<KG_TOPK_MAX><<<dim3(gx, y2), 256, 0, s>>>(nodes, e, pods, list, n_pods, n0, chunk2, index_base, cfg,
                                                                  qst, dev_max, rsv_max, pref, partial, pstat, special, y1,
                                                                  sp);
        k_ext_select_sp<KG_TOPK_MAX><<<dim3(gx, y5), 256, 0, s>>>(nodes, zones, e, pods, list, n_pods, n0, chunk5, index_base,
                                                                  cfg, qst, dev_max, rsv_max, pref, partial, pstat, special, y4,
                                                                  sp);
    }
    if (two) {
        hipError_t err = hipStreamWaitEvent(s, lane->join, 0);
        if (err != hipSuccess) return drain_lane(lane, err);
    }
    return hipGetLastError();
}

}  // namespace kg
