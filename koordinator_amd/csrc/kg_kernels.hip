// kg_kernels.hip — CDNA4 (gfx950) kernels of the Filter/Score evaluation engine.
//
//   k_select   matrix mode: lane = pending pod, wave walks a chunk of node records in uniform order
//              (each record's 256-byte fast block arrives by wide scalar loads into SGPRs), running
//              top-K per lane; per-(chunk, pod) partial keys. Specialised per node storage class
//              (records are stored grouped by class) and per enabled-plugin set.
//   k_merge    per pod: top-K over partial keys (global selectHost of one shard or of the
//              all-gathered shards); k_merge_big adds the nodes outside the float64 fast path.
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
#pragma unroll
        for (int t = 0; t < K; t++) {
            const uint64_t cur = top[t];
            const bool gt = key > cur;
            top[t] = gt ? key : cur;
            key = gt ? cur : key;
        }
    }
}

__device__ __forceinline__ uint32_t rec_gidx(const NodeRec& r, uint32_t index_base) {
    return index_base + node_index(r);
}

// Records [begin, end) are walked in chunks of `chunk`; blockIdx.y = chunk, partial row = part0 + chunk.
// FAST: pods and weights fit the float64 fast path (host check); records flagged F_BIG are skipped
// and evaluated on the integer path by k_merge_big.
template <int K, bool EXACT, bool FAST, uint32_t PM, int CLS>
__global__ __launch_bounds__(256) void k_select(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                PodsDev pods, uint32_t n_pods, uint32_t begin, uint32_t end,
                                                uint32_t chunk, uint32_t part0, uint32_t index_base, KCfg cfg,
                                                uint64_t* __restrict__ partial) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t c = blockIdx.y;
    const bool live = j < n_pods;
    const PodV p = load_pod(pods, live ? j : 0);
    uint64_t top[K];
#pragma unroll
    for (int t = 0; t < K; t++) top[t] = 0;
    const uint32_t lo = begin + c * chunk;
    const uint32_t hi = min(end, lo + chunk);
    if constexpr (FAST) {
        const PodF pf = to_podf(p, cfg);
        const KCfg cv = cfg_in_vgprs(cfg);
        for (uint32_t i = lo; i < hi; i++) {
            const FastRec r = *reinterpret_cast<const FastRec*>(&nodes[i].v[FAST_BEGIN]);
            const uint64_t key = eval_fast_key<PM, CLS>(cv, r, zones + i, pf, index_base + (uint32_t)((uint64_t)r.flags >> 32));
            // F_BIG records (integer path in k_merge_big) are masked, not branched around: one wait
            // for the whole record
            topk_insert<K>(top, ((uint32_t)r.flags & F_BIG) ? 0ull : key);
        }
    } else {
        for (uint32_t i = lo; i < hi; i++) {
            const PairOut o = eval_pair<EXACT>(cfg, nodes[i].v, zones + i, p);
            topk_insert<K>(top, pair_key(cfg, o, rec_gidx(nodes[i], index_base)));
        }
    }
    if (live) {
        uint64_t* dst = partial + ((size_t)(part0 + c) * n_pods + j) * K;
#pragma unroll
        for (int t = 0; t < K; t++) dst[t] = top[t];
    }
}

template <int K>
__global__ __launch_bounds__(256) void k_merge(const uint64_t* __restrict__ partial, uint32_t n_parts, uint32_t n_pods,
                                               uint64_t* __restrict__ out) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_pods) return;
    uint64_t top[K];
#pragma unroll
    for (int t = 0; t < K; t++) top[t] = 0;
    for (uint32_t c = 0; c < n_parts; c++) {
        const uint64_t* src = partial + ((size_t)c * n_pods + j) * K;
#pragma unroll
        for (int t = 0; t < K; t++) topk_insert<K>(top, src[t]);
    }
#pragma unroll
    for (int t = 0; t < K; t++) out[(size_t)j * K + t] = top[t];
}

// Merge of the fast select: top-K over the chunk partials plus the BIG records (integer path) listed
// by k_big_scan.
template <int K>
__global__ __launch_bounds__(256) void k_merge_big(const uint64_t* __restrict__ partial, uint32_t n_parts,
                                                   uint32_t n_pods, const NodeRec* __restrict__ nodes,
                                                   const ZoneRec* __restrict__ zones, PodsDev pods,
                                                   const uint32_t* __restrict__ big_list,
                                                   const uint32_t* __restrict__ big_count, uint32_t index_base,
                                                   KCfg cfg, uint64_t* __restrict__ out) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_pods) return;
    uint64_t top[K];
#pragma unroll
    for (int t = 0; t < K; t++) top[t] = 0;
    for (uint32_t c = 0; c < n_parts; c++) {
        const uint64_t* src = partial + ((size_t)c * n_pods + j) * K;
#pragma unroll
        for (int t = 0; t < K; t++) topk_insert<K>(top, src[t]);
    }
    const uint32_t nb = *big_count;
    if (nb) {
        const PodV p = load_pod(pods, j);
        for (uint32_t b = 0; b < nb; b++) {
            const uint32_t i = big_list[b];
            const PairOut o = eval_pair<false>(cfg, nodes[i].v, zones + i, p);
            topk_insert<K>(top, pair_key(cfg, o, rec_gidx(nodes[i], index_base)));
        }
    }
#pragma unroll
    for (int t = 0; t < K; t++) out[(size_t)j * K + t] = top[t];
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

// Step `step` of the sequential replay: Assume(pod step-1 -> its winner), then evaluate pod `step`.
// One wave per workgroup (no LDS, no barrier): lane = node record. The zone each lane chose for its
// node in the previous step is kept in zsel, so the winner's Reserve needs no re-evaluation; the
// winner key and both pods are loaded up front, independently of each other.
template <bool EXACT>
__global__ __launch_bounds__(64) void k_replay(NodeRec* __restrict__ nodes, ZoneRec* __restrict__ zones, PodsDev pods,
                                               uint32_t n_pods, uint32_t n_nodes, uint32_t index_base, KCfg cfg,
                                               const uint32_t* __restrict__ step_base, uint32_t step_off,
                                               uint64_t* __restrict__ winners, int8_t* __restrict__ zsel) {
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
        if (g == rec_gidx(nodes[i], index_base)) apply_assume(cfg, nodes[i].v, zones + i, q, zsel[i], 1);
    }
    if (!has_next) return;  // uniform: the final step only applies the last Assume
    uint64_t key = 0;
    if (live) {
        const PairOut o = eval_pair<EXACT>(cfg, nodes[i].v, zones + i, p);
        key = pair_key(cfg, o, rec_gidx(nodes[i], index_base));
        zsel[i] = (int8_t)o.zone;
    }
    key = wave_max_u64(key);
    if (threadIdx.x == 0 && key) atomicMax((unsigned long long*)&winners[step], (unsigned long long)key);
}

__global__ void k_bump(uint32_t* step_base, uint32_t by) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *step_base += by;
}

template <bool EXACT>
__global__ void k_assume(NodeRec* __restrict__ nodes, ZoneRec* __restrict__ zones, PodsDev pods, uint32_t pod,
                         uint32_t node, int32_t zone_in, int64_t sign, KCfg cfg, int32_t* __restrict__ zone_out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const PodV q = load_pod(pods, pod);
    int64_t* n = nodes[node].v;
    int32_t zone = zone_in;
    if (sign > 0) {
        const PairOut o = eval_pair<EXACT>(cfg, n, zones + node, q);
        zone = o.zone;
    }
    apply_assume(cfg, n, zones + node, q, zone, sign);
    if (zone_out) *zone_out = zone;
}

// ------------------------------------------------------------------------------------------------
// launchers

#define KG_LAUNCH_CHECK() (hipGetLastError())

template <int K, bool EXACT, bool FAST, uint32_t PM, int CLS>
static void select_instance(const LaunchSelect& a, const SelectRange& r, hipStream_t s) {
    dim3 grid((a.n_pods + 255) / 256, r.n_chunks), block(256);
    k_select<K, EXACT, FAST, PM, CLS><<<grid, block, 0, s>>>(a.nodes, a.zones, a.pods, a.n_pods, r.begin, r.end,
                                                             r.chunk, r.part0, a.index_base, a.cfg, a.partial);
}

template <int K, int CLS>
static void select_fast(const LaunchSelect& a, const SelectRange& r, hipStream_t s) {
    switch (a.cfg.plugins & 7u) {
        case 0: select_instance<K, false, true, 0, CLS>(a, r, s); break;
        case 1: select_instance<K, false, true, 1, CLS>(a, r, s); break;
        case 2: select_instance<K, false, true, 2, CLS>(a, r, s); break;
        case 3: select_instance<K, false, true, 3, CLS>(a, r, s); break;
        case 4: select_instance<K, false, true, 4, CLS>(a, r, s); break;
        case 5: select_instance<K, false, true, 5, CLS>(a, r, s); break;
        case 6: select_instance<K, false, true, 6, CLS>(a, r, s); break;
        default: select_instance<K, false, true, 7, CLS>(a, r, s); break;
    }
}

hipError_t launch_select(const LaunchSelect& a, hipStream_t s) {
    for (int cls = 0; cls < 2; cls++) {
        const SelectRange& r = a.range[cls];
        if (r.n_chunks == 0) continue;
        if (a.exact) {
            if (a.k == 1) select_instance<1, true, false, 0, 0>(a, r, s);
            else select_instance<KG_TOPK_MAX, true, false, 0, 0>(a, r, s);
        } else if (a.fast) {
            if (a.k == 1) {
                if (cls == 0) select_fast<1, 0>(a, r, s);
                else select_fast<1, 1>(a, r, s);
            } else {
                if (cls == 0) select_fast<KG_TOPK_MAX, 0>(a, r, s);
                else select_fast<KG_TOPK_MAX, 1>(a, r, s);
            }
        } else {
            if (a.k == 1) select_instance<1, false, false, 0, 0>(a, r, s);
            else select_instance<KG_TOPK_MAX, false, false, 0, 0>(a, r, s);
        }
    }
    return KG_LAUNCH_CHECK();
}

hipError_t launch_merge(const uint64_t* partial, uint32_t n_parts, uint32_t n_pods, uint32_t k, uint64_t* out,
                        hipStream_t s) {
    dim3 grid((n_pods + 255) / 256), block(256);
    if (k == 1)
        k_merge<1><<<grid, block, 0, s>>>(partial, n_parts, n_pods, out);
    else
        k_merge<KG_TOPK_MAX><<<grid, block, 0, s>>>(partial, n_parts, n_pods, out);
    return KG_LAUNCH_CHECK();
}

hipError_t launch_merge_big(const uint64_t* partial, uint32_t n_parts, uint32_t n_pods, uint32_t k,
                            const NodeRec* nodes, const ZoneRec* zones, const PodsDev& pods, const uint32_t* big_list,
                            const uint32_t* big_count, uint32_t index_base, const KCfg& cfg, uint64_t* out,
                            hipStream_t s) {
    dim3 grid((n_pods + 255) / 256), block(256);
    if (k == 1)
        k_merge_big<1><<<grid, block, 0, s>>>(partial, n_parts, n_pods, nodes, zones, pods, big_list, big_count,
                                              index_base, cfg, out);
    else
        k_merge_big<KG_TOPK_MAX><<<grid, block, 0, s>>>(partial, n_parts, n_pods, nodes, zones, pods, big_list,
                                                        big_count, index_base, cfg, out);
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
                              uint32_t step_off, uint64_t* winners, int8_t* zsel, hipStream_t s) {
    dim3 grid((n_nodes + 63) / 64), block(64);
    if (exact)
        k_replay<true><<<grid, block, 0, s>>>(nodes, zones, pods, n_pods, n_nodes, index_base, cfg, step_base,
                                              step_off, winners, zsel);
    else
        k_replay<false><<<grid, block, 0, s>>>(nodes, zones, pods, n_pods, n_nodes, index_base, cfg, step_base,
                                               step_off, winners, zsel);
    return KG_LAUNCH_CHECK();
}

hipError_t launch_bump(uint32_t* step_base, uint32_t by, hipStream_t s) {
    k_bump<<<1, 64, 0, s>>>(step_base, by);
    return KG_LAUNCH_CHECK();
}

hipError_t launch_assume(NodeRec* nodes, ZoneRec* zones, const PodsDev& pods, uint32_t pod, uint32_t node,
                         int32_t zone, int64_t sign, const KCfg& cfg, bool exact, int32_t* zone_out, hipStream_t s) {
    if (exact)
        k_assume<true><<<1, 64, 0, s>>>(nodes, zones, pods, pod, node, zone, sign, cfg, zone_out);
    else
        k_assume<false><<<1, 64, 0, s>>>(nodes, zones, pods, pod, node, zone, sign, cfg, zone_out);
    return KG_LAUNCH_CHECK();
}

}  // namespace kg
