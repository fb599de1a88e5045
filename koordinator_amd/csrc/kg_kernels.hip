// kg_kernels.hip — CDNA4 (gfx950) kernels of the Filter/Score evaluation engine.
//
//   k_select   matrix mode: lane = pending pod, wave walks a chunk of nodes in uniform order
//              (node records arrive through the scalar cache into SGPRs), running top-K per lane;
//              per-(chunk, pod) partial keys -> k_merge.
//   k_merge    per pod: top-K over the chunks' partial keys (global selectHost of one shard or of
//              the all-gathered shards).
//   k_verify   lane = (pod, node) pair: every plugin's status / score (FilterPlugin / ScorePlugin
//              results) for parity dumps.
//   k_replay   one pod per launch, lane = node: applies the previous pod's Assume to the winning
//              node in place, evaluates the pod on every node, block max -> atomicMax.
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

template <int K, bool EXACT>
__global__ __launch_bounds__(256) void k_select(const NodeRec* __restrict__ nodes, const ZoneRec* __restrict__ zones,
                                                PodsDev pods, uint32_t n_pods, uint32_t n_nodes, uint32_t chunk,
                                                uint32_t index_base, KCfg cfg, uint64_t* __restrict__ partial) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t c = blockIdx.y;
    const bool live = j < n_pods;
    const PodV p = load_pod(pods, live ? j : 0);
    uint64_t top[K];
#pragma unroll
    for (int t = 0; t < K; t++) top[t] = 0;
    const uint32_t lo = c * chunk;
    const uint32_t hi = min(n_nodes, lo + chunk);
    for (uint32_t i = lo; i < hi; i++) {
        const int64_t* n = nodes[i].v;
        const PairOut o = eval_pair<EXACT>(cfg, n, zones + i, p);
        topk_insert<K>(top, pair_key(cfg, o, index_base + i));
    }
    if (live) {
        uint64_t* dst = partial + ((size_t)c * n_pods + j) * K;
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
    status[x] = o.status;
    s_nrf[x] = o.s_nrf;
    s_la[x] = o.s_la;
    s_numa[x] = o.s_numa;
    total[x] = o.status ? -1 : pair_total(cfg, o);
    zone[x] = (int8_t)o.zone;
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
template <bool EXACT>
__global__ __launch_bounds__(256) void k_replay(NodeRec* __restrict__ nodes, ZoneRec* __restrict__ zones, PodsDev pods,
                                                uint32_t n_pods, uint32_t n_nodes, uint32_t index_base, KCfg cfg,
                                                const uint32_t* __restrict__ step_base, uint32_t step_off,
                                                uint64_t* __restrict__ winners) {
    __shared__ uint64_t red[4];
    const uint32_t step = (step_base ? *step_base : 0u) + step_off;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (step > n_pods) return;  // uniform: past the end of the batch
    const bool live = i < n_nodes;
    if (step > 0 && live) {
        const uint64_t prev = winners[step - 1];
        if (prev != 0ull) {
            const uint32_t g = 0xFFFFFFFFu - (uint32_t)(prev & 0xFFFFFFFFull);
            if (g - index_base == i) {
                const PodV q = load_pod(pods, step - 1);
                int64_t* n = nodes[i].v;
                const PairOut o = eval_pair<EXACT>(cfg, n, zones + i, q);
                apply_assume(cfg, n, zones + i, q, o.zone, 1);
            }
        }
    }
    if (step == n_pods) return;  // uniform: final step only applies the last Assume
    uint64_t key = 0;
    if (live) {
        const PodV p = load_pod(pods, step);
        const PairOut o = eval_pair<EXACT>(cfg, nodes[i].v, zones + i, p);
        key = pair_key(cfg, o, index_base + i);
    }
    key = wave_max_u64(key);
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = key;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t m = red[0];
        for (uint32_t w = 1; w < (blockDim.x >> 6); w++) m = red[w] > m ? red[w] : m;
        if (m) atomicMax((unsigned long long*)&winners[step], (unsigned long long)m);
    }
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

hipError_t launch_select(const LaunchSelect& a, hipStream_t s) {
    dim3 grid((a.n_pods + 255) / 256, a.n_chunks), block(256);
    if (a.exact) {
        if (a.k == 1)
            k_select<1, true><<<grid, block, 0, s>>>(a.nodes, a.zones, a.pods, a.n_pods, a.n_nodes, a.chunk,
                                                    a.index_base, a.cfg, a.partial);
        else
            k_select<KG_TOPK_MAX, true><<<grid, block, 0, s>>>(a.nodes, a.zones, a.pods, a.n_pods, a.n_nodes, a.chunk,
                                                              a.index_base, a.cfg, a.partial);
    } else {
        if (a.k == 1)
            k_select<1, false><<<grid, block, 0, s>>>(a.nodes, a.zones, a.pods, a.n_pods, a.n_nodes, a.chunk,
                                                     a.index_base, a.cfg, a.partial);
        else
            k_select<KG_TOPK_MAX, false><<<grid, block, 0, s>>>(a.nodes, a.zones, a.pods, a.n_pods, a.n_nodes,
                                                               a.chunk, a.index_base, a.cfg, a.partial);
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
                              uint32_t step_off, uint64_t* winners, hipStream_t s) {
    dim3 grid((n_nodes + 255) / 256), block(256);
    if (exact)
        k_replay<true><<<grid, block, 0, s>>>(nodes, zones, pods, n_pods, n_nodes, index_base, cfg, step_base,
                                              step_off, winners);
    else
        k_replay<false><<<grid, block, 0, s>>>(nodes, zones, pods, n_pods, n_nodes, index_base, cfg, step_base,
                                               step_off, winners);
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
