// kg_ext_wave.h — wave-level helpers shared by the config-5 kernel files (kg_ext.hip, kg_ext_replay.hip,
// kg_ext_batch.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "kg_ext.h"

namespace kg {

// agent-scope relaxed accesses: global_store / global_load with sc1 (write-through / L1-bypassing), for data handed
// from one workgroup to another inside a launch
template <typename T>
__device__ __forceinline__ void st_agent(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
    return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t wmax_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(v, off, 64);
        v = o > v ? o : v;
    }
    return v;
}

__device__ __forceinline__ int32_t wmax_i32(int32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off, 64));
    return v;
}

__device__ __forceinline__ const DevRec* dev_of(const ExtDev& e, uint32_t rec) { return e.dev ? e.dev + rec : nullptr; }

constexpr uint32_t DSUM_CHUNK = 8;  // GPU request classes per thread of k_dev_sum / k_rdev_codes

// DevSum of one record for every GPU request class of a batch (k_dev_sum's arithmetic, thread = record there), by a
// whole wave: lane = class. The replay refreshes its winner's entry after a Reserve that changed the record's minors,
// so that every step's DeviceShare Filter / Score off reservation views reads the table (dev_eval_sum) instead of
// running the allocator per pair.
__device__ __forceinline__ void dev_sum_refresh(const KCfg& cfg, const ExtDev& e, const int64_t* __restrict__ n,
                                                const ZoneRec* __restrict__ zr, const DevRec* __restrict__ d,
                                                const DevClass* __restrict__ cls, uint32_t n_cls, DevSum* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u;
    const int32_t D = (int32_t)n[N_DEV_MINORS];
    DevSum o;
    uint32_t used = 0u, total = 0u, nonzero = 0u;
#pragma unroll
    for (int r = 0; r < DEV_R; r++) {
        int64_t t = 0, f = 0;
#pragma unroll
        for (int m = 0; m < DEV_MINORS; m++) {
            const int64_t tv = d->total[r][m], fv = d->free_[r][m];
            t += tv;
            f += fv;
            const uint32_t b = m < D ? 1u << m : 0u;
            used |= fv != tv ? b : 0u;
            total |= tv != 0 ? b : 0u;
            nonzero |= fv != 0 ? b : 0u;
        }
        o.T[r] = t;
        o.F[r] = f;
        o.rcp[r] = t != 0 ? 1.0 / (double)t : 0.0;
    }
    if (lane == 0) {
        for (int r = 0; r < DEV_R; r++) {
            out->T[r] = o.T[r];
            out->F[r] = o.F[r];
            out->rcp[r] = o.rcp[r];
        }
    }
    const uint32_t nc = min(n_cls, (uint32_t)DEV_CLASSES);
    for (uint32_t k = lane; k < nc; k += 64u) {
        PodX x{};
        x.dkeys = cls[k].dkeys;
        x.dcount = cls[k].dcount;
        x.dflags = cls[k].dflags;
        x.dtmpl = cls[k].dtmpl;
        x.dbw = cls[k].dbw;
        for (int r = 0; r < DEV_R; r++) x.dreq[r] = cls[k].dreq[r];
        uint32_t le = 0u;
        for (int m = 0; m < DEV_MINORS; m++) {
            bool ok = m < D;
#pragma unroll
            for (int r = 0; r < DEV_R; r++) ok &= !(((x.dkeys >> r) & 1u) && x.dreq[r] > d->free_[r][m]);
            le |= ok ? 1u << m : 0u;
        }
        const GpuMinors g{used, total, total & le, nonzero & le};
        const uint32_t code = D > 0 ? gpu_allocate_code(e, D, zr->dev_topo, zr->dev_part, x, g) : 0u;
        out->code[k] = (uint8_t)(code & 0xFFu);
        out->score[k] = (uint8_t)((uint32_t)dev_sum_score(cfg, &o, x) & 0xFFu);
    }
}

}  // namespace kg
