// Reproducer of a gfx950 device-code discrepancy met while building the GPU partition allocator (round 3):
// gpu_partition_a below (the first form of kg_ext.h's gpu_partition) picks partition {0,1} (mask 0x3) on the
// reference case allocator_gpu_test.go:516 (Hopper table, minor 4 used, 2 GPUs) where the host build of the
// same source and the current kg_ext.h gpu_partition pick {6,7} (mask 0xc0, the reference's answer). Built at
// -O1 and -O3 (ROCm 7.2 hipcc) it is wrong; adding a printf inside its scoring loop makes it right.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize tools/dbg_part.hip -o dbg_part
// Expected output: "form A 3 (wrong: c0 expected) | kg_ext.h c0"
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../koordinator_amd/csrc/kg_ext.h"
namespace kg {
// The earlier form of gpu_partition (local weight arrays indexed by the loop counter, compound loop condition).
__device__ __forceinline__ GpuAlloc gpu_partition_a(const ExtDev& e, uint32_t tbl, const PodX& x, const GpuMinors& g) {
    if (tbl == 0u || !e.parts) return {KG_DEV_CODE_NO_PARTITION, 0u};
    const uint32_t N = x.dcount;
    if (N > 8u) return {KG_DEV_CODE_PART_COUNT, 0u};
    const uint32_t rng = e.part_rng[(tbl - 1u) * 9u + N];
    const uint32_t b = rng & 0xFFFFu, en = rng >> 16;
    if (b >= en) return {KG_DEV_CODE_PART_COUNT, 0u};
    const bool restricted = (x.dflags & KG_GPU_POD_RESTRICTED) != 0, has_bw = (x.dflags & KG_GPU_POD_RING_BW) != 0;
    // the feasible partitions all come from one AllocationScore group: the first that has any (only the
    // first group under the Restricted policy)
    uint32_t gb = b, ge = b, nfeas = 0;
    while (gb < en) {
        ge = gb;
        while (ge < en && e.parts[ge].alloc_score == e.parts[gb].alloc_score) ge++;
        for (uint32_t t = gb; t < ge; t++) {
            const kg_gpu_partition& q = e.parts[t];
            const bool ok = !(q.minors & g.used) && (g.total & q.minors) == q.minors &&
                            (!has_bw || (q.ring_bw >= 0 && x.dbw <= q.ring_bw));
            nfeas += ok ? 1u : 0u;
        }
        if (nfeas > 0u || restricted) break;
        gb = ge;
    }
    if (nfeas == 0u) return {KG_DEV_CODE_PARTITIONED, 0u};
    // selectPartitionByBinPack (:261-296): the first of the highest bin-pack scores (sort.Slice of <= 12
    // elements is an insertion sort, stable)
    uint32_t best_mask = 0u;
    int64_t best = -1;
    for (uint32_t t = gb; t < ge; t++) {
        const kg_gpu_partition& q = e.parts[t];
        const bool ok = !(q.minors & g.used) && (g.total & q.minors) == q.minors &&
                        (!has_bw || (q.ring_bw >= 0 && x.dbw <= q.ring_bw));
        if (!ok) continue;
        if (nfeas == 1u) return {0u, q.minors};
        const uint32_t allocated = g.used | q.minors;
        int64_t score = 0;
        const uint32_t sizes[3] = {8u, 4u, 2u};
        const int64_t wts[3] = {10000, 100, 1};
        for (int k = 0; k < 3; k++) {
            if (sizes[k] < N) continue;
            const uint32_t r2 = e.part_rng[(tbl - 1u) * 9u + sizes[k]];
            const uint32_t b2 = r2 & 0xFFFFu, e2 = r2 >> 16;
            for (uint32_t u = b2; u < e2 && e.parts[u].alloc_score == e.parts[b2].alloc_score; u++) {
                if (e.parts[u].minors & allocated) continue;
                score += wts[k] * (int64_t)e.parts[u].alloc_score;
            }
        }
        if (score > best) {
            best = score;
            best_mask = q.minors;
        }
    }
    return {0u, best_mask};
}

}  // namespace kg
using namespace kg;

__global__ void k(ExtDev e, const DevRec* d, uint32_t* out) {
    if (threadIdx.x) return;
    PodX x{};
    x.dcount = 2;
    x.dkeys = 3;
    x.dreq[0] = 100;
    x.dreq[1] = 100;
    const GpuMinors g = gpu_minors(d, 8, x, 0u);
    out[0] = gpu_partition_a(e, 1u, x, g).mask;
    out[1] = gpu_partition(e, 1u, x, g).mask;
}

int main() {
    kg_gpu_partition P[15];
    int n = 0;
    for (int m = 0; m < 8; m++) P[n++] = {0, 1, (uint8_t)(1 << m), 0, 1, -1};
    for (int m = 0; m < 4; m++) P[n++] = {0, 2, (uint8_t)(3 << (2 * m)), 0, 1, -1};
    P[n++] = {0, 4, 15, 0, 1, -1};
    P[n++] = {0, 4, 240, 0, 1, -1};
    P[n++] = {0, 8, 255, 0, 1, -1};
    uint32_t rng[16 * 9] = {0};
    rng[1] = 0 | 8 << 16;
    rng[2] = 8 | 12 << 16;
    rng[4] = 12 | 14 << 16;
    rng[8] = 14 | 15 << 16;
    DevRec d{};
    for (int r = 0; r < 3; r++)
        for (int m = 0; m < 8; m++) {
            d.total[r][m] = 100;
            d.free_[r][m] = m == 4 ? 0 : 100;
        }
    kg_gpu_partition* dP;
    uint32_t *dr, *dout;
    DevRec* dd;
    if (hipMalloc(&dP, sizeof(P)) || hipMalloc(&dr, sizeof(rng)) || hipMalloc(&dd, sizeof(d)) || hipMalloc(&dout, 64)) return 1;
    hipMemcpy(dP, P, sizeof(P), hipMemcpyHostToDevice);
    hipMemcpy(dr, rng, sizeof(rng), hipMemcpyHostToDevice);
    hipMemcpy(dd, &d, sizeof(d), hipMemcpyHostToDevice);
    static int64_t bp[3 * 256];
    const uint32_t sizes[3] = {8, 4, 2};
    for (int k = 0; k < 3; k++)
        for (uint32_t mask = 0; mask < 256; mask++) {
            const uint32_t b = rng[sizes[k]] & 0xFFFF, en = rng[sizes[k]] >> 16;
            int64_t sum = 0;
            for (uint32_t u = b; u < en; u++)
                if (!(P[u].minors & mask)) sum += P[u].alloc_score;
            bp[k * 256 + mask] = sum;
        }
    int64_t* dbp;
    if (hipMalloc(&dbp, sizeof(bp))) return 1;
    hipMemcpy(dbp, bp, sizeof(bp), hipMemcpyHostToDevice);
    ExtDev e{};
    e.parts = dP;
    e.part_rng = dr;
    e.binpack = dbp;
    k<<<1, 64>>>(e, dd, dout);
    uint32_t o[2];
    hipMemcpy(o, dout, 8, hipMemcpyDeviceToHost);
    printf("form A %x (%s) | kg_ext.h %x\n", o[0], o[0] == 0xc0 ? "right" : "wrong: c0 expected", o[1]);
    return o[1] == 0xc0 ? 0 : 2;
}
