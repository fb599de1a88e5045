// kg_kernels.hip — CDNA4 (gfx950) kernels of the Filter/Score evaluation engine.
//
//   k_select   matrix mode: lane = pending pod, wave walks a chunk of node records in uniform order
//              (each record's 256-byte fast block arrives by wide scalar loads into SGPRs), running
//              top-K per lane; per-(chunk, pod) partial keys. Specialised per node storage class
//              (records are stored grouped by class) and per enabled-plugin set.
//   k_big_sel  the nodes outside the float64 fast path (F_BIG records) for the fast lanes, on the
//              integer path, chunked over the device's F_BIG list.
//   k_merge    per pod: top-K over partial keys (global selectHost of one shard or of the
//              all-gathered shards).
//   k_verify   lane = (pod, node record): every plugin's status / score (FilterPlugin / ScorePlugin
//              results) for parity dumps.
//   k_replay   one pod per launch, lane = node record: applies the previous pod's Assume to the
//              winning node in place, evaluates the pod on every node, block max -> atomicMax.
//   k_assume   Reserve / Unreserve of one pod on one node.
// No MFMA: this is integer / IEEE-double scalar work bound by VALU issue and on-chip bandwidth.
#include <hip/hip_runtime.h>

#include "kg_eval.h"
#include "kg_kernels.h"

namespace kg {

template <int K>
__device__ __forceinline__ void topk_insert(uint64_t (&top)[K], uint64_t key) {
    if constexpr (K == 1) {
        top[0] = key > top[0] ? key : top[0];
    } else {
        // a wave-uniform skip when no lane's key enters its top-K (most records once the lists have filled): the
        // cascade below leaves top unchanged for a key not above top[K-1], so the lanes that do not insert may run it
        if (!__any(key > top[K - 1])) return;
#pragma unroll
        for (int t = 0; t < K; t++) {
            const uint64_t cur = top[t];
            const bool gt = key > cur;
            top[t] = gt ? key : cur;
            key = gt ? cur : key;
        }
    }
}

// Insert a lane's top-K (descending, zeros = none) into the K shared slots of its pod, out[0..K), by an
// atomicMax cascade: each key goes down the slots, an atomicMax at slot u keeps the larger of (slot, key) and
// the smaller continues to slot u + 1. Whatever the interleaving of the lanes (chunks) that insert into one
// pod, slot u ends as the u-th largest key inserted (the values passed below slot u are exactly its arrivals
// minus their maximum), and slot u >= slot u + 1 at every instant; slots only grow. So a key that is not
// above slot K-1 (read once, a lower bound of every slot from then on) can stop.
template <int K>
__device__ __forceinline__ void topk_atomic(uint64_t* out, const uint64_t (&top)[K]) {
    if (top[0] == 0ull) return;
    const uint64_t floor = __hip_atomic_load(out + (K - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int t = 0; t < K; t++) {
        uint64_t carry = top[t];
        if (carry <= floor) break;  // top is descending: every later key stops too
#pragma unroll
        for (int u = 0; u < K; u++) {
            if (carry <= floor) break;
            const uint64_t old = atomicMax((unsigned long long*)(out + u), (unsigned long long)carry);
            carry = old < carry ? old : carry;
        }
    }
}

__device__ __forceinline__ uint32_t rec_gidx(const NodeRec& r, uint32_t index_base) {
    return index_base + node_index(r);
}

// Records [begin, end) are walked in chunks of `chunk`; blockIdx.y = chunk, partial row = part0 + chunk.
// FAST: pods and weights fit the float64 fast path (host check); records flagged F_BIG are skipped
// and evaluated on the integer path by k_big_sel.
template <int K, uint32_t PM, int CLS, int KIND>
__device__ __forceinline__ void select_fast_loop(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                 uint32_t lo, uint32_t hi, uint32_t index_base, const KCfg& cv,
                                                 const PodF& pf, uint64_t (&top)[K]) {
    for (uint32_t i = lo; i < hi; i++) {
        const FastRec r = *reinterpret_cast<const FastRec*>(&nodes[i].v[FAST_BEGIN]);
        uint32_t total;
        const bool ok = fast_eval<PM, CLS, KIND>(cv, r, zones + i, pf, total);
        const uint64_t key = ((uint64_t)total << 32) | (uint64_t)(0xFFFFFFFFu - (index_base + (uint32_t)((uint64_t)r.flags >> 32)));
        // F_BIG records (integer path in k_big_sel) are masked, not branched around: one wait
        // for the whole record
        topk_insert<K>(top, (ok & !((uint32_t)r.flags & F_BIG)) ? key : 0ull);
    }
}

// Records [begin, end) are walked in chunks of `chunk`; blockIdx.y = chunk. Lane j serves pod
// row = order[j] (order nullable: row j). FAST: the pod is in the float64 fast domain (host check) and
// records flagged F_BIG are masked out (k_big_sel evaluates them on the integer path); otherwise every
// record is evaluated on the integer path. K == 1 with `out`: atomicMax of the lane's best key into
// out[row] (zeroed by the launcher); else the lane's top-K goes to partial row part0 + chunk (row
// stride ld pods).
template <int K, bool EXACT, bool FAST, uint32_t PM, int CLS>
__global__ __launch_bounds__(256) void k_select(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                PodsDev pods, uint32_t n_lanes, uint32_t ld, uint32_t begin, uint32_t end,
                                                uint32_t chunk, uint32_t part0, uint32_t index_base, KCfg cfg,
                                                uint64_t* __restrict__ partial, uint64_t* __restrict__ out,
                                                const uint32_t* __restrict__ pmap, uint32_t* __restrict__ pstat,
                                                const uint32_t* __restrict__ order) {
    const GridBlock b = xcd_block();  // whole record chunks per XCD (kg_eval.h)
    const uint32_t j = b.x * blockDim.x + threadIdx.x;
    const uint32_t c = b.y;
    const bool live = j < n_lanes;
    const uint32_t row = live ? (order ? order[j] : j) : 0u;
    const PodV p = load_pod(pods, row);
    uint64_t top[K];
#pragma unroll
    for (int t = 0; t < K; t++) top[t] = 0;
    const uint32_t lo = begin + c * chunk;
    const uint32_t hi = min(end, lo + chunk);
    uint32_t unsup = 0;
    if constexpr (FAST) {
        const PodF pf = to_podf(p, cfg);
        const KCfg cv = cfg_in_vgprs(cfg);
        if (__all(!live || fast_kind_match(FK_PROD, p)))
            select_fast_loop<K, PM, CLS, FK_PROD>(nodes, zones, lo, hi, index_base, cv, pf, top);
        else if (__all(!live || fast_kind_match(FK_BATCH, p)))
            select_fast_loop<K, PM, CLS, FK_BATCH>(nodes, zones, lo, hi, index_base, cv, pf, top);
        else
            select_fast_loop<K, PM, CLS, FK_ANY>(nodes, zones, lo, hi, index_base, cv, pf, top);
    } else {
        for (uint32_t i = lo; i < hi; i++) {
            const PairOut o = eval_pair<EXACT, false, true, true, false>(cfg, nodes[i].v, zones + i, p);
            unsup |= o.status & KG_ST_UNSUPPORTED;
            topk_insert<K>(top, pair_key(cfg, o, rec_gidx(nodes[i], index_base)));
        }
    }
    if (live) {
        if (K == 1 && out) {
            if (top[0]) atomicMax((unsigned long long*)(out + row), (unsigned long long)top[0]);
        } else if (out) {
            topk_atomic<K>(out + (size_t)row * K, top);
        } else {
            uint64_t* dst = partial + ((size_t)(part0 + c) * ld + row) * K;
#pragma unroll
            for (int t = 0; t < K; t++) dst[t] = top[t];
        }
        if (unsup) atomicOr(pstat + (pmap ? pmap[row] : row), unsup);
    }
}

// ---- integer lanes, pruned (LaunchSelect.ipairs) ------------------------------------------------------------
// The lanes whose pods cannot take the fast path (a NUMA policy of their own, cpuset binding) evaluate every record on
// the integer path. Pruned form, exact for top-K into out: (1) k_int_seed: records [0, iseed) on the integer path,
// their keys into out (real pairs: out's K-th key is then a lower bound of the pod's final K-th key); (2)
// k_int_filter: records [iseed, end) with the fast path's NodeResourcesFit / LoadAware part (exact for a pod in the
// fast value domain on a record that is not F_VBIG): a pair failing those filters has key 0, and one whose total
// cannot exceed that part + the NUMA weight x 100 is dropped when that bound is below out's K-th key; the rest are
// appended to ipairs (a full list: the lane evaluates them itself); (3) k_int_pairs: the survivors on the integer
// path, one pair per lane. (NodeNUMAResource's KG_ST_UNSUPPORTED is never produced for a pair these filters drop:
// it is not reached on the device.)
template <int K>
__device__ __forceinline__ void int_insert(uint64_t* out, uint32_t row, const uint64_t (&top)[K]) {
    if constexpr (K == 1) {
        if (top[0]) atomicMax((unsigned long long*)(out + row), (unsigned long long)top[0]);
    } else {
        topk_atomic<K>(out + (size_t)row * K, top);
    }
}

template <int K>
__global__ __launch_bounds__(256) void k_int_seed(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                  PodsDev pods, uint32_t n_lanes, const uint32_t* __restrict__ order,
                                                  uint32_t seed, uint32_t index_base, KCfg cfg, uint64_t* __restrict__ out,
                                                  const uint32_t* __restrict__ pmap, uint32_t* __restrict__ pstat) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_lanes) return;
    const uint32_t row = order ? order[j] : j;
    const PodV p = load_pod(pods, row);
    uint64_t top[K];
#pragma unroll
    for (int t = 0; t < K; t++) top[t] = 0;
    uint32_t unsup = 0;
    const uint32_t lo = blockIdx.y * ((seed + gridDim.y - 1) / gridDim.y), hi = min(seed, lo + (seed + gridDim.y - 1) / gridDim.y);
    for (uint32_t i = lo; i < hi; i++) {
        const PairOut o = eval_pair<false, false, true, true, false>(cfg, nodes[i].v, zones + i, p);
        unsup |= o.status & KG_ST_UNSUPPORTED;
        topk_insert<K>(top, pair_key(cfg, o, rec_gidx(nodes[i], index_base)));
    }
    int_insert<K>(out, row, top);
    if (unsup) atomicOr(pstat + (pmap ? pmap[row] : row), unsup);
}

template <int K>
__global__ __launch_bounds__(256) void k_int_filter(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                    PodsDev pods, uint32_t n_lanes, const uint32_t* __restrict__ order,
                                                    uint32_t begin, uint32_t end, uint32_t chunk, uint32_t index_base,
                                                    KCfg cfg, uint64_t* __restrict__ out, uint64_t* __restrict__ pairs,
                                                    uint32_t* __restrict__ seg_count) {
    // survivors go to this workgroup's own segment of `pairs` (256 x chunk slots: room for every pair it walks),
    // counted in LDS; no global atomics
    __shared__ uint32_t cnt;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    const uint32_t seg = blockIdx.y * gridDim.x + blockIdx.x;
    uint64_t* dst = pairs + (size_t)seg * 256u * chunk;
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = j < n_lanes;
    const uint32_t row = live ? (order ? order[j] : j) : 0u;
    const PodV p = load_pod(pods, row);
    const bool fastv = live && (p.flags & POD_FASTV) != 0;
    const PodF pf = to_podf(p, cfg);
    const KCfg cv = cfg_in_vgprs(cfg);
    const uint64_t floor_key = live ? out[(size_t)row * K + (K - 1)] : ~0ull;
    const uint32_t bonus = (uint32_t)cfg.w_numa * 100u;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t below = lane ? (~0ull >> (64u - lane)) : 0ull;
    const uint32_t lo = begin + blockIdx.y * chunk, hi = min(end, lo + chunk);
    for (uint32_t i = lo; i < hi; i++) {
        const int64_t* nv = nodes[i].v;
        bool keep = live;
        if (fastv && !((uint32_t)nv[N_FLAGS] & F_VBIG)) {
            const FastRec& fr = *reinterpret_cast<const FastRec*>(&nv[FAST_BEGIN]);
            uint32_t part = 0;
            const bool ok = fast_eval<KG_PLUGIN_NRF | KG_PLUGIN_LA, 0>(cv, fr, zones + i, pf, part);
            keep = ok && ((((uint64_t)(part + bonus)) << 32) | 0xFFFFFFFFull) >= floor_key;
        }
        const uint64_t bk = __ballot(keep);
        if (bk == 0ull) continue;
        const uint32_t leader = (uint32_t)__ffsll((unsigned long long)bk) - 1u;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&cnt, (uint32_t)__popcll(bk));
        base = __shfl(base, (int)leader, 64);
        if (keep) dst[base + (uint32_t)__popcll(bk & below)] = ((uint64_t)j << 32) | i;
    }
    __syncthreads();
    if (threadIdx.x == 0) seg_count[seg] = cnt;
}

template <int K>
__global__ __launch_bounds__(256) void k_int_pairs(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                   PodsDev pods, const uint32_t* __restrict__ order,
                                                   const uint64_t* __restrict__ pairs, const uint32_t* __restrict__ seg_count,
                                                   uint32_t n_segs, uint32_t seg_cap, uint32_t index_base, KCfg cfg,
                                                   uint64_t* __restrict__ out, const uint32_t* __restrict__ pmap,
                                                   uint32_t* __restrict__ pstat) {
    // one workgroup per segment at a time, its lanes over the segment's survivors
    for (uint32_t seg = blockIdx.x; seg < n_segs; seg += gridDim.x) {
        const uint32_t n = seg_count[seg];
        for (uint32_t t = threadIdx.x; t < n; t += blockDim.x) {
            const uint64_t e = pairs[(size_t)seg * seg_cap + t];
            const uint32_t j = (uint32_t)(e >> 32), i = (uint32_t)e;
            const uint32_t row = order ? order[j] : j;
            const PodV p = load_pod(pods, row);
            const PairOut o = eval_pair<false, false, true, true, false>(cfg, nodes[i].v, zones + i, p);
            uint64_t top[K];
#pragma unroll
            for (int u = 0; u < K; u++) top[u] = 0;
            top[0] = pair_key(cfg, o, rec_gidx(nodes[i], index_base));
            int_insert<K>(out, row, top);
            if (o.status & KG_ST_UNSUPPORTED) atomicOr(pstat + (pmap ? pmap[row] : row), o.status & KG_ST_UNSUPPORTED);
        }
    }
}

// Fused top-1 select of one storage class: lane = pod, blockIdx.y = chunk of records [begin, end); the
// lane's best key goes to out[pod] by atomicMax (out zeroed by the launcher; the F_BIG records come from
// k_big_sel); no per-chunk partials, no merge pass. `order` (nullable) lists the fast lanes grouped by
// wave kind (kg_pods_upload), so most waves run a kind-specialised loop.
template <uint32_t PM, int CLS, int KIND>
__device__ __forceinline__ uint64_t select1_loop(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                 uint32_t lo, uint32_t hi, uint32_t index_base, const KCfg& cv,
                                                 const PodF& pf) {
    uint64_t top = 0;
    for (uint32_t i = lo; i < hi; i++) {
        const FastRec r = *reinterpret_cast<const FastRec*>(&nodes[i].v[FAST_BEGIN]);
        uint32_t total;
        const bool ok = fast_eval<PM, CLS, KIND>(cv, r, zones + i, pf, total);
        const uint64_t key = ((uint64_t)total << 32) | (uint64_t)(0xFFFFFFFFu - (index_base + (uint32_t)((uint64_t)r.flags >> 32)));
        // F_BIG records: k_big_sel; feasibility and the record test fold into the update's lane mask
        const bool better = ok & !((uint32_t)r.flags & F_BIG) & (key > top);
        top = better ? key : top;
    }
    return top;
}

// (round 6: amdgpu_waves_per_eu(8) -> 78 SGPRs, 8 instead of 6 workgroups per CU, measured no faster: 0.2238 / 0.2251
// vs 0.2231 / 0.2217 ms per config-2 step; the loop is VALU-issue bound, not latency bound)
#ifndef KG_SEL1_ATTR
#define KG_SEL1_ATTR
#endif
template <uint32_t PM, int CLS>
__global__ __launch_bounds__(256) KG_SEL1_ATTR void k_select1(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                 PodsDev pods, uint32_t n_pods, uint32_t begin, uint32_t end,
                                                 uint32_t chunk, uint32_t index_base, KCfg cfg,
                                                 uint64_t* __restrict__ out, const uint32_t* __restrict__ order) {
    const GridBlock b = xcd_block();
    const uint32_t j = b.x * blockDim.x + threadIdx.x;
    const bool live = j < n_pods;
    const uint32_t o = live ? (order ? order[j] : j) : 0u;
    const PodV p = load_pod(pods, o);
    const uint32_t lo = begin + b.y * chunk;
    const uint32_t hi = min(end, lo + chunk);
    const PodF pf = to_podf(p, cfg);
    const KCfg cv = cfg_in_vgprs(cfg);
    uint64_t top;
    // wave-uniform dispatch (idle lanes match any kind)
    if (__all(!live || fast_kind_match(FK_PROD, p)))
        top = select1_loop<PM, CLS, FK_PROD>(nodes, zones, lo, hi, index_base, cv, pf);
    else if (__all(!live || fast_kind_match(FK_BATCH, p)))
        top = select1_loop<PM, CLS, FK_BATCH>(nodes, zones, lo, hi, index_base, cv, pf);
    else
        top = select1_loop<PM, CLS, FK_ANY>(nodes, zones, lo, hi, index_base, cv, pf);
    if (live && top) atomicMax((unsigned long long*)(out + o), (unsigned long long)top);
}

// The F_BIG records (integer path) for the fast lanes: lane = pod (via order), blockIdx.y = chunk of the
// device's F_BIG list (k_big_scan), whose length is only known on the device: gridDim.y chunks of
// ceil(count / gridDim.y) records each. K == 1 with `out`: atomicMax into out[row]; else the lane's top-K
// into partial row part0 + blockIdx.y (empty chunks write zeros).
template <int K>
__global__ __launch_bounds__(256) void k_big_sel(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                 PodsDev pods, uint32_t n_lanes, uint32_t ld,
                                                 const uint32_t* __restrict__ big_list,
                                                 const uint32_t* __restrict__ big_count, uint32_t index_base, KCfg cfg,
                                                 uint64_t* __restrict__ partial, uint32_t part0, uint64_t* __restrict__ out,
                                                 const uint32_t* __restrict__ pmap, uint32_t* __restrict__ pstat,
                                                 const uint32_t* __restrict__ order) {
    const uint32_t nb = *big_count;
    const bool direct = out != nullptr;
    if (nb == 0 && direct) return;  // uniform
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_lanes) return;
    const uint32_t row = order ? order[j] : j;
    const uint32_t chunk = (nb + gridDim.y - 1) / gridDim.y;
    const uint32_t lo = blockIdx.y * chunk, hi = min(nb, lo + chunk);
    uint64_t top[K];
#pragma unroll
    for (int t = 0; t < K; t++) top[t] = 0;
    uint32_t unsup = 0;
    if (lo < hi) {
        const PodV p = load_pod(pods, row);
        // direct (fused) launches run after the fast records' kernels: a record whose NodeResourcesFit / LoadAware
        // part fails, or whose best possible total (that part + the NUMA weight x 100) stays below the pod's current
        // K-th best key, cannot change the result and skips the integer path. The fast block's NRF / LA part is exact
        // on records that are F_BIG only for their NUMA / CPU bind policies (not F_VBIG); prune is off for a pod
        // outside the fast domain (the lanes here are fast lanes).
        uint64_t floor_key = 0;
        if (direct) {
            floor_key = ~0ull;
#pragma unroll
            for (int t = 0; t < K; t++) floor_key = min(floor_key, (uint64_t)out[(size_t)row * K + t]);
        }
        const PodF pf = to_podf(p, cfg);
        const KCfg cv = cfg_in_vgprs(cfg);  // the fast path's form of the weights
        for (uint32_t b = lo; b < hi; b++) {
            const uint32_t i = big_list[b];
            const int64_t* nv = nodes[i].v;
            const uint32_t fl = (uint32_t)nv[N_FLAGS];
            if (direct && !(fl & F_VBIG)) {
                const FastRec& fr = *reinterpret_cast<const FastRec*>(&nv[FAST_BEGIN]);
                uint32_t part = 0;
                const bool ok = fast_eval<KG_PLUGIN_NRF | KG_PLUGIN_LA, 0>(cv, fr, zones + i, pf, part);
                if (!ok) continue;  // the pair fails NodeResourcesFit / LoadAware: key 0
                const uint64_t bound = ((uint64_t)(part + (uint32_t)cfg.w_numa * 100u) << 32) | 0xFFFFFFFFull;
                if (bound < floor_key) continue;
            }
            const PairOut o = eval_pair<false, false, true, true, false>(cfg, nv, zones + i, p);
            unsup |= o.status & KG_ST_UNSUPPORTED;
            topk_insert<K>(top, pair_key(cfg, o, rec_gidx(nodes[i], index_base)));
        }
    }
    if (direct) {
        if constexpr (K == 1) {
            if (top[0]) atomicMax((unsigned long long*)(out + row), (unsigned long long)top[0]);
        } else {
            topk_atomic<K>(out + (size_t)row * K, top);
        }
    } else {
        uint64_t* dst = partial + ((size_t)(part0 + blockIdx.y) * ld + row) * K;
#pragma unroll
        for (int t = 0; t < K; t++) dst[t] = top[t];
    }
    if (unsup) atomicOr(pstat + (pmap ? pmap[row] : row), unsup);
}

// Per pod row (lane j -> list[j], or j): top-K over partial rows [part0, part0 + n_parts) of stride ld.
template <int K>
__global__ __launch_bounds__(256) void k_merge(const uint64_t* __restrict__ partial, uint32_t part0, uint32_t n_parts,
                                               uint32_t ld, const uint32_t* __restrict__ list, uint32_t n,
                                               uint64_t* __restrict__ out) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t row = list ? list[j] : j;
    uint64_t top[K];
#pragma unroll
    for (int t = 0; t < K; t++) top[t] = 0;
    for (uint32_t c = 0; c < n_parts; c++) {
        const uint64_t* src = partial + ((size_t)(part0 + c) * ld + row) * K;
#pragma unroll
        for (int t = 0; t < K; t++) topk_insert<K>(top, src[t]);
    }
#pragma unroll
    for (int t = 0; t < K; t++) out[(size_t)row * K + t] = top[t];
}

// Rebuild the list of F_BIG records (after any change of node state).
__global__ __launch_bounds__(256) void k_big_scan(const NodeRec* __restrict__ nodes, uint32_t n_nodes,
                                                  uint32_t* __restrict__ big_list, uint32_t* __restrict__ big_count) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_nodes) return;
    if ((uint32_t)nodes[i].v[N_FLAGS] & F_BIG) {
        const uint32_t slot = atomicAdd(big_count, 1u);
        big_list[slot] = i;
    }
}

// Outputs are indexed by the node's snapshot index (record orig), [pod][node].
template <bool EXACT>
__global__ __launch_bounds__(256) void k_verify(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                PodsDev pods, uint32_t n_pods, uint32_t n_nodes, KCfg cfg,
                                                uint32_t* __restrict__ status, int64_t* __restrict__ s_nrf,
                                                int64_t* __restrict__ s_la, int64_t* __restrict__ s_numa,
                                                int64_t* __restrict__ total, int8_t* __restrict__ zone) {
    const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= (size_t)n_pods * n_nodes) return;
    const uint32_t j = (uint32_t)(x / n_nodes), i = (uint32_t)(x % n_nodes);
    const PodV p = load_pod(pods, j);
    const PairOut o = eval_pair<EXACT>(cfg, nodes[i].v, zones + i, p);
    const size_t y = (size_t)j * n_nodes + node_index(nodes[i]);
    status[y] = o.status;
    s_nrf[y] = o.s_nrf;
    s_la[y] = o.s_la;
    s_numa[y] = o.s_numa;
    total[y] = o.status ? -1 : pair_total(cfg, o);
    zone[y] = (int8_t)o.zone;
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(v, off, 64);
        v = o > v ? o : v;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v |= (uint32_t)__shfl_xor((int)v, off, 64);
    return v;
}

// Ordering of LDS accesses between the lanes of a one-wave workgroup: the LDS serves a wave's
// operations in order, so waiting for this wave's own LDS operations is enough. Unlike
// __syncthreads(), it leaves the wave's global loads (row prefetches) and stores in flight.
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Wave max by DPP (row-local steps, then row broadcasts; result read from lane 63). Call with all
// 64 lanes active.
__device__ __forceinline__ uint32_t wave_max_u32_dpp(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false));  // row_half_mirror
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false));  // row_mirror
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false));  // row_bcast:15
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false));  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// max of 64-bit selection keys: the high halves (totals), then the low halves of the lanes that hold it
__device__ __forceinline__ uint64_t wave_max_key(uint64_t k) {
    const uint32_t hi = wave_max_u32_dpp((uint32_t)(k >> 32));
    const uint32_t lo = wave_max_u32_dpp((uint32_t)(k >> 32) == hi ? (uint32_t)k : 0u);
    return ((uint64_t)hi << 32) | lo;
}

// Step `step` of the sequential replay: Assume(pod step-1 -> its winner), then evaluate pod `step`.
// One wave per workgroup (no LDS, no barrier): lane = node record. The zone each lane chose for its
// node in the previous step is kept in zsel, so the winner's Reserve needs no re-evaluation; the
// winner key and both pods are loaded up front, independently of each other.
template <bool EXACT>
__global__ __launch_bounds__(64) void k_replay(NodeRec* __restrict__ nodes, ZoneRec* __restrict__ zones, PodsDev pods,
                                               uint32_t n_pods, uint32_t n_nodes, uint32_t index_base, KCfg cfg,
                                               const uint32_t* __restrict__ step_base, uint32_t step_off,
                                               uint64_t* __restrict__ winners, int8_t* __restrict__ zsel,
                                               uint32_t* __restrict__ reason) {
    const uint32_t step = (step_base ? *step_base : 0u) + step_off;
    if (step > n_pods) return;  // uniform: past the end of the batch
    const uint32_t i = blockIdx.x * 64u + threadIdx.x;
    const bool live = i < n_nodes;
    const bool has_next = step < n_pods;
    const uint64_t prev = step > 0 ? __hip_atomic_load(&winners[step - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    const PodV q = load_pod(pods, step > 0 ? step - 1 : 0);
    const PodV p = load_pod(pods, has_next ? step : 0);
    if (live && prev != 0ull) {
        const uint32_t g = 0xFFFFFFFFu - (uint32_t)(prev & 0xFFFFFFFFull);
        if (g == rec_gidx(nodes[i], index_base)) {
            const int32_t z = zsel[i];
            if (zone_reserve_fails(z)) {  // the Reserve fails (BestEffort allocation): the pod stays unscheduled
                winners[step - 1] = 0ull;
                if (reason) atomicOr(reason + step - 1, zone_fail_status(z));
            } else {
                apply_assume(cfg, nodes[i].v, zones + i, q, z, 1);
            }
        }
    }
    if (!has_next) return;  // uniform: the final step only applies the last Assume
    uint64_t key = 0;
    uint32_t st = 0;
    if (live) {
        const PairOut o = eval_pair<EXACT>(cfg, nodes[i].v, zones + i, p);
        key = pair_key(cfg, o, rec_gidx(nodes[i], index_base));
        zsel[i] = (int8_t)o.zone;
        st = o.status;
    }
    key = wave_max_u64(key);
    if (threadIdx.x == 0 && key) atomicMax((unsigned long long*)&winners[step], (unsigned long long)key);
    if (reason) {  // FitError diagnosis: OR of the filter status bits over the nodes
        st = wave_or_u32(st);
        if (threadIdx.x == 0 && st) atomicOr(reason + step, st);
    }
}

__global__ void k_bump(uint32_t* step_base, uint32_t by) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *step_base += by;
}

template <bool EXACT>
__global__ void k_assume(NodeRec* __restrict__ nodes, ZoneRec* __restrict__ zones, PodsDev pods, uint32_t pod,
                         uint32_t node, int32_t zone_in, int64_t sign, KCfg cfg, int32_t* __restrict__ zone_out,
                         int64_t* __restrict__ split) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const PodV q = load_pod(pods, pod);
    int64_t* n = nodes[node].v;
    int32_t zone = zone_in;
    if (sign > 0) {
        // a cpuset Reserve that ran first hands over the zone of the pre-take state (or its failure)
        const int32_t w = zone_out ? *zone_out : 0;
        zone = zone_is_preset(w) ? zone_of_preset(w) : eval_pair<EXACT>(cfg, n, zones + node, q).zone;
    }
    if (!zone_reserve_fails(zone)) apply_assume(cfg, n, zones + node, q, zone, sign, split);  // else nothing is applied
    if (zone_out) *zone_out = zone;
}

// ------------------------------------------------------------------------------------------------
// Block replay (config 3): the pods of a window [base, base + RB_W) are placed one by one, exactly as
// the sequential replay places them, from one matrix pass over the window. A placement changes the
// row of its winner only, and every config-3 plugin scores a pair from that pair's row alone, so for
// pod base + t only the nodes already chosen in the window (the set C, at most t rows) can have new
// keys; every other node keeps the key the window pass computed. The pass keeps each pod's top RB_K
// keys; pod base + t's best unchanged node is the first of them outside C, unless all RB_K are in C
// (the window ends before that pod: the next window starts there). k_rb_fix re-evaluates C plus
// that candidate on the updated rows, staged in LDS, and applies the Assume.

// Integer-path key of one pair, out of line: keeps the fast loops' register allocation free of the
// integer path's (records flagged F_BIG are rare).
template <bool EXACT>
__device__ __forceinline__ uint64_t int_key(const KCfg& cfg, const int64_t* n, const ZoneRec* zr, const PodV& p, uint32_t g) {
    return pair_key(cfg, eval_pair<EXACT, false, true, true, false>(cfg, n, zr, p), g);
}

// Pass 1: per-(chunk, pod) top-RB_K over node records [begin, end); lane = pod of the window. Each
// wave first stages its chunk's fast blocks (and zone tables for SingleNUMANode records) in LDS with
// all lanes, so the walk pays one memory latency instead of one per record.
template <bool EXACT, bool FAST, int CLS>
__global__ __launch_bounds__(64) void k_rb_top(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                               PodsDev pods, uint32_t n_pods, uint32_t begin, uint32_t end,
                                               uint32_t chunk, uint32_t part0, uint32_t index_base, KCfg cfg,
                                               const uint32_t* __restrict__ step, uint64_t* __restrict__ partial) {
    __shared__ FastRec sfr[FAST ? RB_CHUNK : 1];
    __shared__ ZoneRec szr[(FAST && CLS == 1) ? RB_CHUNK : 1];
    const uint32_t base = *step;
    if (base >= n_pods) return;  // uniform: batch done
    const uint32_t t = threadIdx.x, j = base + t;
    const bool live = j < n_pods;
    const PodV p = load_pod(pods, live ? j : base);
    uint64_t top[RB_K];
#pragma unroll
    for (int k = 0; k < RB_K; k++) top[k] = 0;
    const uint32_t lo = begin + blockIdx.x * chunk;
    const uint32_t hi = min(end, lo + chunk);
    if constexpr (FAST) {
        const uint32_t n = hi - lo;  // <= RB_CHUNK (host)
        constexpr uint32_t QF = sizeof(FastRec) / 16, QZ = sizeof(ZoneRec) / 16;
        for (uint32_t q = t; q < n * QF; q += 64u)
            reinterpret_cast<uint4*>(sfr)[q] = reinterpret_cast<const uint4*>(&nodes[lo + q / QF].v[FAST_BEGIN])[q % QF];
        if constexpr (CLS == 1)
            for (uint32_t q = t; q < n * QZ; q += 64u)
                reinterpret_cast<uint4*>(szr)[q] = reinterpret_cast<const uint4*>(&zones[lo + q / QZ])[q % QZ];
        __syncthreads();
        const PodF pf = to_podf(p, cfg);
        const KCfg cv = cfg_in_vgprs(cfg);
        for (uint32_t x = 0; x < n; x++) {
            const FastRec& r = sfr[x];
            const uint32_t f = (uint32_t)r.flags;
            const uint32_t g = index_base + (uint32_t)((uint64_t)r.flags >> 32);
            uint64_t key;
            if (f & F_BIG)  // uniform branch: lane = pod, the record is the wave's
                key = int_key<false>(cfg, nodes[lo + x].v, zones + lo + x, p, g);
            else
                key = eval_fast_key<7u, CLS>(cv, r, CLS == 1 ? &szr[x] : zones + lo + x, pf, g);
            if (key > top[RB_K - 1]) topk_insert<RB_K>(top, key);
        }
    } else {
        for (uint32_t i = lo; i < hi; i++) {
            const uint64_t key = pair_key(cfg, eval_pair<EXACT, false, true, true, false>(cfg, nodes[i].v, zones + i, p),
                                          rec_gidx(nodes[i], index_base));
            if (key > top[RB_K - 1]) topk_insert<RB_K>(top, key);
        }
    }
    uint64_t* dst = partial + ((size_t)(part0 + blockIdx.x) * RB_W + t) * RB_K;
#pragma unroll
    for (int k = 0; k < RB_K; k++) dst[k] = live ? top[k] : 0ull;
}

// Pass 2: per pod of the window (one workgroup each), top-RB_K over the chunk lists.
__global__ __launch_bounds__(256) void k_rb_merge(const uint64_t* __restrict__ partial, uint32_t n_parts, uint32_t n_pods,
                                                  const uint32_t* __restrict__ step, uint64_t* __restrict__ tops) {
    __shared__ uint64_t cand[4 * RB_K];
    const uint32_t base = *step;
    if (base >= n_pods) return;
    const uint32_t t = blockIdx.x, lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint64_t top[RB_K];
#pragma unroll
    for (int k = 0; k < RB_K; k++) top[k] = 0;
    for (uint32_t c = threadIdx.x; c < n_parts; c += blockDim.x) {
        const uint64_t* src = partial + ((size_t)c * RB_W + t) * RB_K;
        uint64_t in[RB_K];
#pragma unroll
        for (int k = 0; k < RB_K; k++) in[k] = src[k];  // one wait for the whole list
#pragma unroll
        for (int k = 0; k < RB_K; k++) {
            if (in[k] <= top[RB_K - 1]) break;  // lists are sorted: the rest is smaller
            topk_insert<RB_K>(top, in[k]);
        }
    }
    // wave: RB_K rounds of max extraction (keys are unique: the node index is in the low half)
    for (int r = 0; r < RB_K; r++) {
        const uint64_t m = wave_max_key(top[0]);
        if (m != 0 && top[0] == m) {
#pragma unroll
            for (int k = 0; k < RB_K - 1; k++) top[k] = top[k + 1];
            top[RB_K - 1] = 0;
        }
        if (lane == 0) cand[w * RB_K + r] = m;
    }
    __syncthreads();
    if (w == 0) {
        uint64_t v = cand[lane];  // 4 waves x RB_K = 64 candidates
        for (int r = 0; r < RB_K; r++) {
            const uint64_t m = wave_max_key(v);
            if (m != 0 && v == m) v = 0;
            if (lane == 0) tops[t * RB_K + r] = m;
        }
    }
}

// Integer-path key and zone of one pair, out of line: rows flagged F_BIG and the integer variant.
// Keeps the integer path's registers and private arrays out of the window loop.
template <bool EXACT>
__device__ __forceinline__ uint64_t rb_int_eval(const KCfg* cfg, const NodeRec* n, const ZoneRec* zr, PodV p, uint32_t g,
                                             int32_t* zone) {
    const PairOut o = eval_pair<EXACT>(*cfg, n->v, zr, p);
    *zone = o.zone;
    return pair_key(*cfg, o, g);
}

// Lane-parallel Reserve of pod j on one LDS-staged row for the window replay's serial loop: the same
// bits as apply_assume (sign +1; kg_eval.h) followed by derive_node (kg_layout.h), with the int-slot
// updates, the F_BIG checks, the four zone headrooms and the derived fast slots spread over the
// wave's lanes instead of one lane's chain of dependent LDS accesses. Multi-zone NUMA splits
// (zone >= 0x40) keep the one-lane apply_assume. Call with all 64 lanes active.
enum : uint8_t { DER_FIT = 0, DER_DIFF = 1, DER_HEAD = 2, DER_AMP_FIT = 3, DER_AMP_DELTA = 4 };
constexpr int N_DER = 21;
__constant__ uint8_t DER_DST[N_DER] = {D_FIT_CPU, D_FIT_MEM, D_FIT_EPH, D_FIT_SC0, D_FIT_SC1, D_LR_NZ_CPU, D_LR_NZ_MEM,
                                      D_LR_SC0, D_LR_SC1, D_LA_HEAD_NP0, D_LA_HEAD_NP1, D_LA_HEAD_PROD0, D_LA_HEAD_PROD1,
                                      D_LA_SFREE_NP0, D_LA_SFREE_NP1, D_LA_SDELTA0, D_LA_SDELTA1, D_NUMA_FREE_CPU,
                                      D_NUMA_FREE_MEM, D_AMP_FIT, D_AMP_DELTA};
__constant__ uint8_t DER_A[N_DER] = {N_ALLOC_CPU, N_ALLOC_MEM, N_ALLOC_EPH, N_SC_ALLOC0, N_SC_ALLOC1, N_ALLOC_CPU,
                                    N_ALLOC_MEM, N_SC_ALLOC0, N_SC_ALLOC1, N_LA_FCUT_NP0, N_LA_FCUT_NP1, N_LA_FCUT_PROD0,
                                    N_LA_FCUT_PROD1, N_LA_ALLOC0, N_LA_ALLOC1, N_LA_SBASE_NP0, N_LA_SBASE_NP1, N_ALLOC_CPU,
                                    N_ALLOC_MEM, N_ALLOC_CPU, N_CPUSET};
__constant__ uint8_t DER_B[N_DER] = {N_REQ_CPU, N_REQ_MEM, N_REQ_EPH, N_SC_REQ0, N_SC_REQ1, N_NZ_CPU, N_NZ_MEM,
                                    N_SC_REQ0, N_SC_REQ1, N_LA_FBASE_NP0, N_LA_FBASE_NP1, N_LA_FBASE_PROD0,
                                    N_LA_FBASE_PROD1, N_LA_SBASE_NP0, N_LA_SBASE_NP1, N_LA_SBASE_PROD0, N_LA_SBASE_PROD1,
                                    N_REQ_CPU, N_REQ_MEM, N_REQ_CPU, N_AMP_CPUSET};
__constant__ uint8_t DER_OP[N_DER] = {DER_FIT, DER_FIT, DER_FIT, DER_FIT, DER_FIT, DER_DIFF, DER_DIFF, DER_DIFF, DER_DIFF,
                                     DER_HEAD, DER_HEAD, DER_HEAD, DER_HEAD, DER_DIFF, DER_DIFF, DER_DIFF, DER_DIFF,
                                     DER_DIFF, DER_DIFF, DER_AMP_FIT, DER_AMP_DELTA};

// The lane's derived-slot operation (DER_* tables), loaded once per kernel.
struct DerLane {
    uint32_t dst, a, b, op;
};

__device__ __forceinline__ DerLane der_lane(uint32_t lane) {
    DerLane d{0, 0, 0, 0};
    if (lane < (uint32_t)N_DER) d = {DER_DST[lane], DER_A[lane], DER_B[lane], DER_OP[lane]};
    return d;
}

// 64-bit lane broadcast / gather
__device__ __forceinline__ int64_t readlane64(int64_t x, uint32_t src) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, (int)src);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)x >> 32), (int)src);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ int64_t shfl64(int64_t x, uint32_t src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)x, (int)src, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)((uint64_t)x >> 32), (int)src, 64);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Reserve of pod pt (its columns broadcast from the lane that holds it) on an LDS-staged row, then
// derive_node: one round of LDS reads (lane k: int slot k; lanes 32..35: zone k - 32), the new int
// values exchanged between lanes by shuffles, one round of writes.
__device__ __forceinline__ void assume_wave(const KCfg& c, NodeRec& r, ZoneRec& z, const PodV& pt, int32_t zone,
                                            uint32_t lane, const DerLane& dl) {
    int64_t* v = r.v;
    const uint64_t fl = (uint64_t)v[N_FLAGS];
    const int64_t old = lane < (uint32_t)N_INT_SLOTS ? v[lane] : 0;
    const bool zl = lane >= 32u && lane < 32u + (uint32_t)MAX_ZONES;
    const uint32_t q = zl ? lane - 32u : 0u;
    int64_t tc = 0, tm = 0, uc = 0, um = 0;
    if (zl) tc = z.cpu[q], tm = z.mem[q], uc = z.cpu_used[q], um = z.mem_used[q];
    const uint32_t meta = z.cpu_meta;
    // apply_assume (sign +1): the int slot updates
    const uint32_t flags = (uint32_t)fl;
    const bool la = (c.plugins & KG_PLUGIN_LA) && (flags & F_LA_HAS_METRIC);
    const bool prod = (pt.flags & KG_POD_PROD) != 0;
    const int64_t e0 = pt.est0 > 0 ? pt.est0 : 0, e1 = pt.est1 > 0 ? pt.est1 : 0;
    int64_t add = 0;
    add = lane == (uint32_t)N_REQ_CPU ? pt.req_cpu : add;
    add = lane == (uint32_t)N_REQ_MEM ? pt.req_mem : add;
    add = lane == (uint32_t)N_REQ_EPH ? pt.req_eph : add;
    add = lane == (uint32_t)N_SC_REQ0 ? pt.sc0 : add;
    add = lane == (uint32_t)N_SC_REQ1 ? pt.sc1 : add;
    add = lane == (uint32_t)N_NZ_CPU ? pt.nz_cpu : add;
    add = lane == (uint32_t)N_NZ_MEM ? pt.nz_mem : add;
    add = lane == (uint32_t)N_NUM_PODS ? 1 : add;
    if (la) {
        add = (lane == (uint32_t)N_LA_FBASE_NP0 || lane == (uint32_t)N_LA_SBASE_NP0) ? e0 : add;
        add = (lane == (uint32_t)N_LA_FBASE_NP1 || lane == (uint32_t)N_LA_SBASE_NP1) ? e1 : add;
        if (prod) {
            add = (lane == (uint32_t)N_LA_FBASE_PROD0 || lane == (uint32_t)N_LA_SBASE_PROD0) ? e0 : add;
            add = (lane == (uint32_t)N_LA_FBASE_PROD1 || lane == (uint32_t)N_LA_SBASE_PROD1) ? e1 : add;
        }
    }
    const int64_t nv = old + add;
    const bool zone_hit = zl && (c.plugins & KG_PLUGIN_NUMA) && zone >= 0 && zone < MAX_ZONES && (uint32_t)zone == q;
    if (zone_hit) uc += pt.req_cpu, um += pt.req_mem;
    // the zone's allocation record (apply_assume) and the amplified accounting of zone_cpu_alloc on the new state
    const uint32_t st0 = z.status;
    const uint32_t st = st0 | ((uint32_t)((__ballot(zone_hit && (pt.req_cpu | pt.req_mem)) >> 32) & 0xFull)
                               << ZONE_RECORD_SHIFT);
    int64_t ua = uc;
    if (zl && ((st >> (ZONE_RECORD_SHIFT + q)) & 1u) && z.amp_ratio > 1.0) {
        const int64_t cz = 1000 * (int64_t)z.cz_alloc[q];
        ua = uc - cz + amp_i64(cz, z.amp_ratio);
    }
    // derive_node on the new values
    const int64_t always_fail = kg_bits(-1.0), never_fail = kg_bits(4611686018427387904.0);
    const uint32_t f0 = flags & ~(uint32_t)F_DERIVED_MASK;
    const bool full = shfl64(nv, N_NUM_PODS) + 1 > shfl64(nv, N_ALLOC_PODS);
    const int64_t cs = shfl64(nv, N_CPUSET), acs = shfl64(nv, N_AMP_CPUSET);
    bool big = false;
    if (lane <= (uint32_t)N_LA_SBASE_PROD1 && lane != (uint32_t)N_ALLOC_PODS && lane != (uint32_t)N_NUM_PODS &&
        !(lane >= (uint32_t)N_LA_FCUT_NP0 && lane <= (uint32_t)N_LA_FCUT_PROD1))
        big = kg_big(nv) || nv < 0;
    if (lane == 63) big = kg_big(cs) || kg_big(acs) || cs < 0 || acs < cs;
    double zv[6] = {0, 0, 0, 0, 0, 0};
    if (zl) {
        big = kg_big(tc) || kg_big(tm) || kg_big(ua) || kg_big(um) || uc < 0 || um < 0;
        const int64_t ac = tc - ua < 0 ? 0 : tc - ua, am = tm - um < 0 ? 0 : tm - um;
        const int64_t rc = tc - ac < 0 ? 0 : tc - ac, rm = tm - am < 0 ? 0 : tm - am;
        zv[0] = ac != 0 ? x100(ac) : -1.0;
        zv[1] = am != 0 ? x100(am) : -1.0;
        zv[2] = x100(tc - rc);
        zv[3] = x100(tm - rm);
        zv[4] = x100(tc - ua);
        zv[5] = x100(tm - um);
    }
    const uint32_t pol0 = (f0 >> F_NUMA_POLICY_SHIFT) & 15u;
    const bool pol_host = pol0 == 2u /* KG_NUMA_RESTRICTED */;
    const bool vbig = __ballot(big) != 0ull;
    const bool big_all = vbig || pol_host || ((meta >> CPU_META_BIND_SHIFT) & 3u) != 0u;
    const uint32_t f = f0 | (full ? (uint32_t)F_PODS_FULL : 0u) | (big_all ? (uint32_t)F_BIG : 0u) |
                       (vbig ? (uint32_t)F_VBIG : 0u);
    // derived slot dl.dst of this lane (lanes < N_DER)
    uint32_t a = dl.a, b = dl.b, mode = (f >> F_LA_FMODE_NP_SHIFT) & 3u;
    if (dl.op == DER_HEAD && a >= (uint32_t)N_LA_FCUT_PROD0) {  // prod heads: the non-prod ones without prod thresholds
        if (f & F_LA_PROD_THR) mode = (f >> F_LA_FMODE_PROD_SHIFT) & 3u;
        else a -= 2u, b -= 2u;
    }
    const int64_t va = shfl64(nv, a), vb = shfl64(nv, b);
    const bool amp = (f & F_AMP) != 0;
    int64_t val;
    if (dl.op == DER_FIT) {
        const int64_t d = va - vb;
        val = (lane == 0 && full) ? always_fail : kg_bits(x100(d < 0 ? 0 : d));
    } else if (dl.op == DER_DIFF) {
        val = kg_bits(x100(va - vb));
    } else if (dl.op == DER_HEAD) {
        val = mode == FMODE_PASS ? never_fail
            : mode == FMODE_FAIL_EXPIRED ? always_fail : kg_bits(((double)va - (double)vb) * 100.0);
    } else if (dl.op == DER_AMP_FIT) {
        const int64_t req_f = (vb >= cs && cs > 0) ? vb - cs + acs : vb;
        const int64_t d = va - req_f;
        val = pol_host ? always_fail : amp ? kg_bits(x100(d < 0 ? 0 : d)) : never_fail;
    } else {  // DER_AMP_DELTA: 0 on BestEffort nodes (node-level score without amplification)
        val = kg_bits((amp && pol0 != 1u) ? x100(va - vb) : 0.0);
    }
    // writes
    if (lane < (uint32_t)N_INT_SLOTS && add) v[lane] = nv;
    if (lane < (uint32_t)N_DER) v[dl.dst] = val;
    if (zl) {
        if (zone_hit) z.cpu_used[q] = uc, z.mem_used[q] = um;
        ZoneFast& zf = z.zf[q];
        zf.avail_cpu = zv[0];
        zf.avail_mem = zv[1];
        zf.hint_cpu = zv[2];
        zf.hint_mem = zv[3];
        zf.free_cpu = zv[4];
        zf.free_mem = zv[5];
    }
    if (lane == 32u && st != st0) z.status = st;
    if (lane == 63) v[N_FLAGS] = (int64_t)((fl & 0xFFFFFFFF00000000ull) | f);
    wave_lds_sync();
}

// Pass 3 (one wave, lane = pod base + lane of the window): the sequential placements of the window.
// Rows of C (the nodes placed on so far in this window) live in LDS slots [0, nc), and ckey[c][t] holds
// pod t's key on slot c as the row is now. Pod t's winner is the larger of its best key over C (a
// column read and a DPP max) and its candidate: the first entry of its list outside C, whose key the
// window pass computed on an unchanged row. After the Assume, the one changed row is re-evaluated
// for every later pod of the window at once (lane = pod, row uniform). While pod t is placed, the
// rows of the first two entries of pod t+1's list outside C are loaded into registers: whichever
// node pod t takes, pod t+1's candidate is one of them. FAST: keys from the float64 fast path (rows
// not flagged F_BIG), else the integer path. Ends by writing the rows of C back and advancing *step.
template <bool EXACT, bool FAST>
__global__ __launch_bounds__(64) void k_rb_fix(NodeRec* __restrict__ nodes, ZoneRec* __restrict__ zones, PodsDev pods,
                                               uint32_t n_pods, uint32_t n_nodes, uint32_t index_base, KCfg cfg,
                                               const uint32_t* __restrict__ pos, const uint64_t* __restrict__ tops,
                                               uint32_t* __restrict__ step, uint64_t* __restrict__ winners) {
    __shared__ NodeRec snode[RB_W];
    __shared__ ZoneRec szone[RB_W];
    __shared__ uint32_t changed[RB_BITMAP_WORDS];
    __shared__ uint32_t crec[RB_W];
    __shared__ uint64_t skey[RB_W * RB_K];
    __shared__ uint32_t srec[RB_W * RB_K];
    __shared__ uint64_t ckey[RB_W][RB_W];  // [slot][pod]
    __shared__ int8_t czone[RB_W][RB_W];
    __shared__ KCfg scfg;  // for the out-of-line integer path
    constexpr uint32_t NN = sizeof(NodeRec) / 16, NZ = sizeof(ZoneRec) / 16, NQ = NN + NZ;  // 16-B pieces
    static_assert(NQ <= 128, "row staging: two pieces per lane");
    const uint32_t lane = threadIdx.x;
    const uint32_t base = *step;
    if (base >= n_pods) return;  // uniform
    const uint32_t words = (n_nodes + 31u) >> 5;
    for (uint32_t w = lane; w < words; w += 64u) changed[w] = 0;
    const bool live = base + lane < n_pods;
    const PodV mp = load_pod(pods, live ? base + lane : base);  // this lane's pod
    {
        uint64_t kk[RB_K];
#pragma unroll
        for (int k = 0; k < RB_K; k++) kk[k] = tops[lane * RB_K + k];
        uint32_t rr[RB_K];
#pragma unroll
        for (int k = 0; k < RB_K; k++)  // branch-free index: the RB_K loads are in flight together
            rr[k] = pos[kk[k] ? 0xFFFFFFFFu - (uint32_t)(kk[k] & 0xFFFFFFFFull) - index_base : 0u];
#pragma unroll
        for (int k = 0; k < RB_K; k++) {
            skey[lane * RB_K + k] = kk[k];
            srec[lane * RB_K + k] = kk[k] ? rr[k] : 0u;
        }
    }
    if (lane == 0) scfg = cfg;
    __syncthreads();
    const KCfg cv = cfg_in_vgprs(cfg);
    const PodF mpf = to_podf(mp, cfg);
    const DerLane der = der_lane(lane);
    // key and zone of this lane's pod on slot s (row uniform across the wave)
    auto eval_slot = [&](uint32_t s, int32_t* zone) -> uint64_t {
        const uint32_t f = (uint32_t)snode[s].v[N_FLAGS];
        const uint32_t g = index_base + node_index(snode[s]);
        if (FAST && !(f & (F_BIG | F_TOPO))) {
            const FastRec& r = *reinterpret_cast<const FastRec*>(&snode[s].v[FAST_BEGIN]);
            *zone = -1;
            if (node_class(snode[s]) == 1) return eval_fast_key<7u, 1>(cv, r, &szone[s], mpf, g, zone);
            return eval_fast_key<7u, 0>(cv, r, &szone[s], mpf, g);
        }
        return rb_int_eval<EXACT>(&scfg, &snode[s], &szone[s], mp, g, zone);
    };
    auto piece = [&](uint32_t r, uint32_t q) -> uint4 {
        return q < NN ? reinterpret_cast<const uint4*>(&nodes[r])[q] : reinterpret_cast<const uint4*>(&zones[r])[q - NN];
    };
    auto put = [&](uint32_t slot, uint32_t q, uint4 v) {
        if (q < NN) reinterpret_cast<uint4*>(&snode[slot])[q] = v;
        else reinterpret_cast<uint4*>(&szone[slot])[q - NN] = v;
    };
    // prefetched rows: two candidates (e1, e2) of the next pod, two pieces per lane each
    // (named registers, not arrays: a dynamically indexed private array would live in scratch)
    uint32_t rec1 = 0, rec2 = 0;
    int k1 = -1, k2 = -1;
    uint4 pa1 = {}, pb1 = {}, pa2 = {}, pb2 = {};
    auto prefetch = [&](uint32_t t) {
        const uint64_t ck = lane < (uint32_t)RB_K ? skey[t * RB_K + lane] : 0ull;
        const uint32_t rec = lane < (uint32_t)RB_K ? srec[t * RB_K + lane] : 0u;
        uint64_t m = __ballot(ck != 0ull && ((changed[rec >> 5] >> (rec & 31u)) & 1u) == 0u);
        k1 = m ? (int)(__ffsll((long long)m) - 1) : -1;
        if (m) m &= m - 1;
        k2 = m ? (int)(__ffsll((long long)m) - 1) : -1;
        rec1 = (uint32_t)__builtin_amdgcn_readlane((int)rec, k1 >= 0 ? k1 : 0);
        rec2 = (uint32_t)__builtin_amdgcn_readlane((int)rec, k2 >= 0 ? k2 : 0);
        if (k1 >= 0) {
            pa1 = piece(rec1, lane);
            if (lane + 64u < NQ) pb1 = piece(rec1, lane + 64u);
        }
        if (k2 >= 0) {
            pa2 = piece(rec2, lane);
            if (lane + 64u < NQ) pb2 = piece(rec2, lane + 64u);
        }
    };
    prefetch(0);
    uint32_t nc = 0, done = 0, last = 0xFFFFFFFFu;  // last: the record the previous pod added to C
    for (uint32_t t = 0; t < (uint32_t)RB_W && base + t < n_pods; t++) {
        const uint32_t j = base + t;
        // candidate: e1 unless the previous pod just took it
        const bool second = k1 >= 0 && rec1 == last;
        const int ck_k = second ? k2 : k1;
        const bool has_cand = ck_k >= 0;
        const bool full = skey[t * RB_K + RB_K - 1] != 0ull;
        if (!has_cand && full) break;  // every listed node changed: this pod starts the next window
        const uint32_t cand = second ? rec2 : rec1;
        const uint64_t cand_key = has_cand ? skey[t * RB_K + ck_k] : 0ull;
        const uint4 cpre0 = second ? pa2 : pa1, cpre1 = second ? pb2 : pb1;
        // pod t+1's first two entries outside C_t: their rows load while pod t is placed
        if (t + 1 < (uint32_t)RB_W && j + 1 < n_pods) prefetch(t + 1);
        // best key over C
        const uint64_t kc = lane < nc ? ckey[lane][t] : 0ull;
        const uint64_t best_c = wave_max_key(kc);
        const uint64_t best = best_c > cand_key ? best_c : cand_key;
        last = 0xFFFFFFFFu;
        uint64_t placed = best;
        if (best != 0ull) {
            uint32_t slot;
            int32_t zone;
            if (best == cand_key) {  // the candidate wins: it joins C in slot nc (unless its Reserve fails)
                slot = nc;
                put(slot, lane, cpre0);
                if (lane + 64u < NQ) put(slot, lane + 64u, cpre1);
                wave_lds_sync();
                // pod t's zone on the candidate (class-0 rows on the fast path never allocate one; BestEffort
                // rows take the integer path for their Reserve's zone)
                const uint32_t cf = (uint32_t)snode[slot].v[N_FLAGS];
                int32_t z = -1;
                if (!(FAST && !(cf & (F_BIG | F_TOPO)) && node_class(snode[slot]) == 0) && lane == t) eval_slot(slot, &z);
                zone = __shfl(z, (int)t, 64);
                if (!zone_reserve_fails(zone)) {
                    if (lane == 0) {
                        crec[slot] = cand;
                        changed[cand >> 5] |= 1u << (cand & 31u);
                    }
                    last = cand;
                    nc++;
                }
            } else {
                slot = (uint32_t)(__ffsll((long long)__ballot(lane < nc && kc == best)) - 1);
                zone = czone[slot][t];
            }
            if (zone_reserve_fails(zone)) {
                placed = 0ull;  // the Reserve fails (BestEffort allocation): nothing changes, the pod stays unscheduled
            } else if (zone >= 0x40) {  // multi-zone NUMA split: one lane (lane t holds pod t)
                if (lane == t) apply_assume(cfg, snode[slot].v, &szone[slot], mp, zone, 1);
            } else {
                PodV pt;
                pt.req_cpu = readlane64(mp.req_cpu, t);
                pt.req_mem = readlane64(mp.req_mem, t);
                pt.req_eph = readlane64(mp.req_eph, t);
                pt.sc0 = readlane64(mp.sc0, t);
                pt.sc1 = readlane64(mp.sc1, t);
                pt.nz_cpu = readlane64(mp.nz_cpu, t);
                pt.nz_mem = readlane64(mp.nz_mem, t);
                pt.est0 = readlane64(mp.est0, t);
                pt.est1 = readlane64(mp.est1, t);
                pt.flags = (uint32_t)__builtin_amdgcn_readlane((int)mp.flags, (int)t);
                assume_wave(cfg, snode[slot], szone[slot], pt, zone, lane, der);
            }
            wave_lds_sync();
            // later pods of the window on the changed row
            if (placed && lane > t && live) {
                int32_t z = -1;
                ckey[slot][lane] = eval_slot(slot, &z);
                czone[slot][lane] = (int8_t)z;
            }
        }
        if (lane == 0) winners[j] = placed;
        wave_lds_sync();
        done = t + 1;
    }
    // write the changed rows back
    for (uint32_t s2 = 0; s2 < nc; s2++) {
        const uint32_t r = crec[s2];
        uint4* dn = reinterpret_cast<uint4*>(&nodes[r]);
        uint4* dz = reinterpret_cast<uint4*>(&zones[r]);
        const uint4* sn = reinterpret_cast<const uint4*>(&snode[s2]);
        const uint4* sz = reinterpret_cast<const uint4*>(&szone[s2]);
        for (uint32_t q = lane; q < NQ; q += 64u) {
            if (q < NN) dn[q] = sn[q];
            else dz[q - NN] = sz[q - NN];
        }
    }
    if (lane == 0) *step = base + done;
}

// ------------------------------------------------------------------------------------------------
// launchers

#define KG_LAUNCH_CHECK() (hipGetLastError())

template <int K, bool EXACT, bool FAST, uint32_t PM, int CLS>
static void select_instance(const LaunchSelect& a, const SelectRange& r, uint32_t lane0, uint32_t n_lanes, bool atom,
                            hipStream_t s) {
    dim3 grid((n_lanes + 255) / 256, r.n_chunks), block(256);
    k_select<K, EXACT, FAST, PM, CLS><<<grid, block, 0, s>>>(a.nodes, a.zones, a.pods, n_lanes, a.n_rows, r.begin, r.end,
                                                             r.chunk, r.part0, a.index_base, a.cfg, a.partial,
                                                             atom ? a.out : nullptr, a.pmap, a.pstat,
                                                             a.order ? a.order + lane0 : nullptr);
}

// K > 1 fused (a.fused_k): the lanes insert into out by the atomic cascade, no partial rows exist
template <int K, int CLS>
static void select_fast(const LaunchSelect& a, const SelectRange& r, hipStream_t s) {
    const bool atom = K > 1 && a.fused_k;
    switch (a.cfg.plugins & 7u) {
        case 0: select_instance<K, false, true, 0, CLS>(a, r, 0, a.n_fast, atom, s); break;
        case 1: select_instance<K, false, true, 1, CLS>(a, r, 0, a.n_fast, atom, s); break;
        case 2: select_instance<K, false, true, 2, CLS>(a, r, 0, a.n_fast, atom, s); break;
        case 3: select_instance<K, false, true, 3, CLS>(a, r, 0, a.n_fast, atom, s); break;
        case 4: select_instance<K, false, true, 4, CLS>(a, r, 0, a.n_fast, atom, s); break;
        case 5: select_instance<K, false, true, 5, CLS>(a, r, 0, a.n_fast, atom, s); break;
        case 6: select_instance<K, false, true, 6, CLS>(a, r, 0, a.n_fast, atom, s); break;
        default: select_instance<K, false, true, 7, CLS>(a, r, 0, a.n_fast, atom, s); break;
    }
}

hipError_t launch_select(const LaunchSelect& a, hipStream_t s) {
    const uint32_t K = a.k == 1 ? 1u : (uint32_t)KG_TOPK_MAX;
    const uint32_t n_fast = a.fast ? a.n_fast : 0u, n_int = a.n_pods - n_fast;
    // K == 1: the fused fast path and the integer lanes update out[row] by atomicMax; K > 1 fused: every lane
    // by the atomicMax cascade
    if ((K == 1 && (a.fused || n_int)) || (K > 1 && a.fused_k)) {
        hipError_t e = hipMemsetAsync(a.out, 0, sizeof(uint64_t) * a.n_rows * K, s);
        if (e != hipSuccess) return e;
    }
    const uint32_t seed_n = a.irange.n_chunks ? min(a.iseed, a.irange.end) : 0u;
    const uint32_t i_lb = (n_int + 255) / 256;
    const uint32_t i_chunk = max(64u, (a.irange.end - seed_n + max(1u, 2048u / max(1u, i_lb)) - 1) / max(1u, 2048u / max(1u, i_lb)));
    const uint32_t i_fy = a.irange.n_chunks ? (a.irange.end - seed_n + i_chunk - 1) / i_chunk : 0u;
    const bool pruned = n_int && a.irange.n_chunks && a.ipairs && !a.exact && (K == 1 || a.fused_k) &&
                        (uint64_t)i_lb * i_fy * 256u * i_chunk <= a.ipairs_cap && (uint64_t)i_lb * i_fy <= a.iseg_cap;
    // the side stream (when the caller gives one) takes the pruned integer lanes or, without them, the fused top-1
    // select of storage class 1 (both write out by atomics only; k_big_sel reads out's keys as a lower bound)
    const bool c1_side = !pruned && K == 1 && a.fused && n_fast && a.range[1].n_chunks && a.range[0].n_chunks;
    const bool side = (pruned || c1_side) && a.side && a.fork && a.join;
    hipStream_t si = side ? a.side : s;
    if (side) {
        hipError_t e = hipEventRecord(a.fork, s);
        if (e == hipSuccess) e = hipStreamWaitEvent(a.side, a.fork, 0);
        if (e != hipSuccess) return e;
    }
    if (pruned) {
        // pruned integer lanes (see k_int_seed): seed, filter into per-workgroup segments, survivors
        const uint32_t* io = a.order ? a.order + n_fast : nullptr;
        const uint32_t sy = max(1u, min(64u, (2048u + i_lb - 1) / i_lb));
        const uint32_t n_segs = i_lb * i_fy;
        if (K == 1) {
            if (seed_n) k_int_seed<1><<<dim3(i_lb, sy), 256, 0, si>>>(a.nodes, a.zones, a.pods, n_int, io, seed_n, a.index_base,
                                                                     a.cfg, a.out, a.pmap, a.pstat);
            if (i_fy) k_int_filter<1><<<dim3(i_lb, i_fy), 256, 0, si>>>(a.nodes, a.zones, a.pods, n_int, io, seed_n,
                                                                       a.irange.end, i_chunk, a.index_base, a.cfg, a.out,
                                                                       a.ipairs, a.ipair_count);
            if (n_segs) k_int_pairs<1><<<min(n_segs, 4096u), 256, 0, si>>>(a.nodes, a.zones, a.pods, io, a.ipairs, a.ipair_count,
                                                                          n_segs, 256u * i_chunk, a.index_base, a.cfg, a.out,
                                                                          a.pmap, a.pstat);
        } else {
            if (seed_n)
                k_int_seed<KG_TOPK_MAX><<<dim3(i_lb, sy), 256, 0, si>>>(a.nodes, a.zones, a.pods, n_int, io, seed_n, a.index_base,
                                                                       a.cfg, a.out, a.pmap, a.pstat);
            if (i_fy)
                k_int_filter<KG_TOPK_MAX><<<dim3(i_lb, i_fy), 256, 0, si>>>(a.nodes, a.zones, a.pods, n_int, io, seed_n,
                                                                           a.irange.end, i_chunk, a.index_base, a.cfg, a.out,
                                                                           a.ipairs, a.ipair_count);
            if (n_segs)
                k_int_pairs<KG_TOPK_MAX><<<min(n_segs, 4096u), 256, 0, si>>>(a.nodes, a.zones, a.pods, io, a.ipairs,
                                                                            a.ipair_count, n_segs, 256u * i_chunk,
                                                                            a.index_base, a.cfg, a.out, a.pmap, a.pstat);
        }
        if (side) {
            hipError_t e = hipEventRecord(a.join, a.side);
            if (e != hipSuccess) return e;
        }
    }
    if (n_fast) {
        const uint32_t pod_blocks = (n_fast + 255) / 256;
        for (int cls = 0; cls < 2; cls++) {
            const SelectRange& r = a.range[cls];
            if (r.n_chunks == 0) continue;
            if (a.fused) {
                dim3 grid(pod_blocks, r.n_chunks), block(256);
                hipStream_t sc = (cls == 1 && c1_side && side) ? si : s;
#define KG_SEL1(PMV)                                                                                               \
    do {                                                                                                           \
        if (cls == 0)                                                                                              \
            k_select1<PMV, 0><<<grid, block, 0, sc>>>(a.nodes, a.zones, a.pods, n_fast, r.begin, r.end, r.chunk,   \
                                                      a.index_base, a.cfg, a.out, a.order);                        \
        else                                                                                                       \
            k_select1<PMV, 1><<<grid, block, 0, sc>>>(a.nodes, a.zones, a.pods, n_fast, r.begin, r.end, r.chunk,   \
                                                      a.index_base, a.cfg, a.out, a.order);                        \
    } while (0)
                switch (a.cfg.plugins & 7u) {
                    case 0: KG_SEL1(0); break;
                    case 1: KG_SEL1(1); break;
                    case 2: KG_SEL1(2); break;
                    case 3: KG_SEL1(3); break;
                    case 4: KG_SEL1(4); break;
                    case 5: KG_SEL1(5); break;
                    case 6: KG_SEL1(6); break;
                    default: KG_SEL1(7); break;
                }
#undef KG_SEL1
                if (cls == 1 && c1_side && side) {
                    hipError_t e = hipEventRecord(a.join, a.side);
                    if (e != hipSuccess) return e;
                }
            } else if (K == 1) {
                if (cls == 0) select_fast<1, 0>(a, r, s);
                else select_fast<1, 1>(a, r, s);
            } else {
                if (cls == 0) select_fast<KG_TOPK_MAX, 0>(a, r, s);
                else select_fast<KG_TOPK_MAX, 1>(a, r, s);
            }
        }
        // F_BIG records of the fast lanes: integer path, chunked over the device's list; after the fast records'
        // kernels, whose keys in out let a direct launch skip records that cannot enter the pod's top-K
        {
            dim3 grid(pod_blocks, a.big_y), block(256);
            if (K == 1)
                k_big_sel<1><<<grid, block, 0, s>>>(a.nodes, a.zones, a.pods, n_fast, a.n_rows, a.big_list, a.big_count,
                                                    a.index_base, a.cfg, a.partial, a.big_part0, a.fused ? a.out : nullptr,
                                                    a.pmap, a.pstat, a.order);
            else
                k_big_sel<KG_TOPK_MAX><<<grid, block, 0, s>>>(a.nodes, a.zones, a.pods, n_fast, a.n_rows, a.big_list,
                                                              a.big_count, a.index_base, a.cfg, a.partial, a.big_part0,
                                                              a.fused_k ? a.out : nullptr, a.pmap, a.pstat, a.order);
        }
        if (!a.fused && !a.fused_k) {
            hipError_t e = launch_merge_list(a.partial, 0, select_fparts(a), a.n_rows, a.order, n_fast, K, a.out, s);
            if (e != hipSuccess) return e;
        }
    }
    if (pruned) {
        // launched above (before the fast lanes)
    } else if (n_int && a.irange.n_chunks) {
        const SelectRange& r = a.irange;
        if (a.exact) {
            if (K == 1) select_instance<1, true, false, 0, 0>(a, r, n_fast, n_int, true, s);
            else select_instance<KG_TOPK_MAX, true, false, 0, 0>(a, r, n_fast, n_int, a.fused_k, s);
        } else {
            if (K == 1) select_instance<1, false, false, 0, 0>(a, r, n_fast, n_int, true, s);
            else select_instance<KG_TOPK_MAX, false, false, 0, 0>(a, r, n_fast, n_int, a.fused_k, s);
        }
        if (K > 1 && !a.fused_k) {
            hipError_t e = launch_merge_list(a.partial, r.part0, r.n_chunks, a.n_rows, a.order ? a.order + n_fast : nullptr,
                                             n_int, K, a.out, s);
            if (e != hipSuccess) return e;
        }
    } else if (n_int && K > 1 && !a.fused_k) {  // no records: no feasible node (fused: out is zeroed)
        hipError_t e = launch_merge_list(a.partial, 0, 0, a.n_rows, a.order ? a.order + n_fast : nullptr, n_int, K, a.out, s);
        if (e != hipSuccess) return e;
    }
    if (side) {
        hipError_t e = hipStreamWaitEvent(s, a.join, 0);
        if (e != hipSuccess) return e;
    }
    return KG_LAUNCH_CHECK();
}

hipError_t launch_merge_list(const uint64_t* partial, uint32_t part0, uint32_t n_parts, uint32_t ld, const uint32_t* list,
                             uint32_t n, uint32_t k, uint64_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    dim3 grid((n + 255) / 256), block(256);
    if (k == 1)
        k_merge<1><<<grid, block, 0, s>>>(partial, part0, n_parts, ld, list, n, out);
    else
        k_merge<KG_TOPK_MAX><<<grid, block, 0, s>>>(partial, part0, n_parts, ld, list, n, out);
    return KG_LAUNCH_CHECK();
}

hipError_t launch_merge(const uint64_t* partial, uint32_t n_parts, uint32_t n_pods, uint32_t k, uint64_t* out,
                        hipStream_t s) {
    return launch_merge_list(partial, 0, n_parts, n_pods, nullptr, n_pods, k, out, s);
}

// Batched row update (kg_snapshot_update_rows): record r of the staged block (NodeRec, ZoneRec and, with
// DeviceShare, DevRec of each row back to back) goes to record position pos[r]. One 16-byte word per lane:
// a 512-B node record is 32 consecutive lanes, so each wave writes two whole records with full-line stores.
__global__ __launch_bounds__(256) void k_scatter_rows(const uint4* __restrict__ stage, const uint32_t* __restrict__ pos,
                                                      uint32_t n, uint32_t dev_words, uint4* __restrict__ nodes,
                                                      uint4* __restrict__ zones, uint4* __restrict__ devs) {
    constexpr uint32_t NW = sizeof(NodeRec) / 16, ZW = sizeof(ZoneRec) / 16;
    const uint32_t rw = NW + ZW + dev_words;
    const size_t total = (size_t)n * rw;
    for (size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += (size_t)gridDim.x * blockDim.x) {
        const uint32_t r = (uint32_t)(x / rw), w = (uint32_t)(x % rw);
        const size_t p = pos[r];
        const uint4 v = stage[x];
        if (w < NW)
            nodes[p * NW + w] = v;
        else if (w < NW + ZW)
            zones[p * ZW + (w - NW)] = v;
        else
            devs[p * dev_words + (w - NW - ZW)] = v;
    }
}

hipError_t launch_scatter_rows(const void* stage, const uint32_t* pos, uint32_t n, bool dev, NodeRec* nodes,
                               ZoneRec* zones, DevRec* devs, hipStream_t s) {
    static_assert(sizeof(NodeRec) % 16 == 0 && sizeof(ZoneRec) % 16 == 0 && sizeof(DevRec) % 16 == 0, "16-B words");
    if (n == 0) return hipSuccess;
    const uint32_t dw = dev ? (uint32_t)(sizeof(DevRec) / 16) : 0u;
    const size_t words = (size_t)n * (sizeof(NodeRec) / 16 + sizeof(ZoneRec) / 16 + dw);
    const unsigned grid = (unsigned)std::min<size_t>((words + 255) / 256, 4096);
    k_scatter_rows<<<grid, 256, 0, s>>>(static_cast<const uint4*>(stage), pos, n, dw, reinterpret_cast<uint4*>(nodes),
                                        reinterpret_cast<uint4*>(zones), reinterpret_cast<uint4*>(devs));
    return KG_LAUNCH_CHECK();
}

hipError_t launch_big_scan(const NodeRec* nodes, uint32_t n_nodes, uint32_t* big_list, uint32_t* big_count,
                           hipStream_t s) {
    hipError_t e = hipMemsetAsync(big_count, 0, sizeof(uint32_t), s);
    if (e != hipSuccess || n_nodes == 0) return e;
    k_big_scan<<<(n_nodes + 255) / 256, 256, 0, s>>>(nodes, n_nodes, big_list, big_count);
    return KG_LAUNCH_CHECK();
}

hipError_t launch_verify(const NodeRec* nodes, const ZoneRec* zones, const PodsDev& pods, uint32_t n_pods,
                         uint32_t n_nodes, const KCfg& cfg, bool exact, const VerifyDev& o, hipStream_t s) {
    const size_t pairs = (size_t)n_pods * n_nodes;
    dim3 grid((unsigned)((pairs + 255) / 256)), block(256);
    if (exact)
        k_verify<true><<<grid, block, 0, s>>>(nodes, zones, pods, n_pods, n_nodes, cfg, o.status, o.s_nrf, o.s_la,
                                              o.s_numa, o.total, o.zone);
    else
        k_verify<false><<<grid, block, 0, s>>>(nodes, zones, pods, n_pods, n_nodes, cfg, o.status, o.s_nrf, o.s_la,
                                               o.s_numa, o.total, o.zone);
    return KG_LAUNCH_CHECK();
}

hipError_t launch_replay_step(NodeRec* nodes, ZoneRec* zones, const PodsDev& pods, uint32_t n_pods, uint32_t n_nodes,
                              uint32_t index_base, const KCfg& cfg, bool exact, const uint32_t* step_base,
                              uint32_t step_off, uint64_t* winners, int8_t* zsel, uint32_t* reason, hipStream_t s) {
    dim3 grid((n_nodes + 63) / 64), block(64);
    if (exact)
        k_replay<true><<<grid, block, 0, s>>>(nodes, zones, pods, n_pods, n_nodes, index_base, cfg, step_base,
                                              step_off, winners, zsel, reason);
    else
        k_replay<false><<<grid, block, 0, s>>>(nodes, zones, pods, n_pods, n_nodes, index_base, cfg, step_base,
                                               step_off, winners, zsel, reason);
    return KG_LAUNCH_CHECK();
}

template <bool EXACT, bool FAST, int CLS>
static void rb_top_instance(const LaunchRb& a, const SelectRange& r, hipStream_t s) {
    k_rb_top<EXACT, FAST, CLS><<<r.n_chunks, 64, 0, s>>>(a.nodes, a.zones, a.pods, a.n_pods, r.begin, r.end, r.chunk,
                                                         r.part0, a.index_base, a.cfg, a.step, a.partial);
}

hipError_t launch_rb_window(const LaunchRb& a, hipStream_t s) {
    for (int cls = 0; cls < 2; cls++) {
        const SelectRange& r = a.range[cls];
        if (r.n_chunks == 0) continue;
        if (a.exact) rb_top_instance<true, false, 0>(a, r, s);
        else if (a.fast && cls == 0) rb_top_instance<false, true, 0>(a, r, s);
        else if (a.fast) rb_top_instance<false, true, 1>(a, r, s);
        else rb_top_instance<false, false, 0>(a, r, s);
    }
    k_rb_merge<<<RB_W, 256, 0, s>>>(a.partial, a.n_parts, a.n_pods, a.step, a.tops);
    if (a.exact)
        k_rb_fix<true, false><<<1, 64, 0, s>>>(a.nodes_rw, a.zones_rw, a.pods, a.n_pods, a.n_nodes, a.index_base, a.cfg,
                                               a.pos, a.tops, a.step, a.winners);
    else if (a.fast)
        k_rb_fix<false, true><<<1, 64, 0, s>>>(a.nodes_rw, a.zones_rw, a.pods, a.n_pods, a.n_nodes, a.index_base, a.cfg,
                                               a.pos, a.tops, a.step, a.winners);
    else
        k_rb_fix<false, false><<<1, 64, 0, s>>>(a.nodes_rw, a.zones_rw, a.pods, a.n_pods, a.n_nodes, a.index_base, a.cfg,
                                                a.pos, a.tops, a.step, a.winners);
    return KG_LAUNCH_CHECK();
}

hipError_t launch_bump(uint32_t* step_base, uint32_t by, hipStream_t s) {
    k_bump<<<1, 64, 0, s>>>(step_base, by);
    return KG_LAUNCH_CHECK();
}

hipError_t launch_assume(NodeRec* nodes, ZoneRec* zones, const PodsDev& pods, uint32_t pod, uint32_t node,
                         int32_t zone, int64_t sign, const KCfg& cfg, bool exact, int32_t* zone_out, hipStream_t s,
                         int64_t* split) {
    if (exact)
        k_assume<true><<<1, 64, 0, s>>>(nodes, zones, pods, pod, node, zone, sign, cfg, zone_out, split);
    else
        k_assume<false><<<1, 64, 0, s>>>(nodes, zones, pods, pod, node, zone, sign, cfg, zone_out, split);
    return KG_LAUNCH_CHECK();
}

}  // namespace kg
