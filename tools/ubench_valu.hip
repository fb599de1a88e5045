// Issue cost of the VALU instructions the select loop uses (gfx950), one wave per SIMD vs four waves per
// SIMD: s_memtime around 64 x 8 independent instructions. Build: hipcc --offload-arch=gfx950 -O2
// tools/ubench_valu.hip -o /tmp/ubench_valu ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(X) X X X X X X X X
#define REP64(X) REP8(REP8(X))

template <int OP>
__global__ void kern(unsigned long long* out, double* dsink, float* fsink, unsigned* usink) {
    double a0 = threadIdx.x * 1.5 + 1, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    double b = 3.25;
    unsigned u0 = threadIdx.x + 1, u1 = u0 + 1, u2 = u0 + 2, u3 = u0 + 3, u4 = u0 + 4, u5 = u0 + 5, u6 = u0 + 6, u7 = u0 + 7;
    unsigned long long x0 = threadIdx.x * 77ull + 1, y = 12345678901ull;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < 16; it++) {
        if constexpr (OP == 0) {  // v_add_f64
            REP64(asm volatile("v_add_f64 %0, %0, %8\n v_add_f64 %1, %1, %8\n v_add_f64 %2, %2, %8\n v_add_f64 %3, %3, %8\n v_add_f64 %4, %4, %8\n v_add_f64 %5, %5, %8\n v_add_f64 %6, %6, %8\n v_add_f64 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
        } else if constexpr (OP == 1) {  // v_cmp_lt_f64 -> sgpr pair
            REP64(asm volatile("v_cmp_lt_f64_e64 s[44:45], %0, %8\n v_cmp_lt_f64_e64 s[46:47], %1, %8\n v_cmp_lt_f64_e64 s[48:49], %2, %8\n v_cmp_lt_f64_e64 s[50:51], %3, %8\n v_cmp_lt_f64_e64 s[52:53], %4, %8\n v_cmp_lt_f64_e64 s[54:55], %5, %8\n v_cmp_lt_f64_e64 s[56:57], %6, %8\n v_cmp_lt_f64_e64 s[58:59], %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "s44","s45","s46","s47","s48","s49","s50","s51","s52","s53","s54","s55","s56","s57","s58","s59");)
        } else if constexpr (OP == 2) {  // v_cmp_lt_u64 -> sgpr pair
            REP64(asm volatile("v_cmp_lt_u64_e64 s[44:45], %0, %1\n v_cmp_lt_u64_e64 s[46:47], %0, %1\n v_cmp_lt_u64_e64 s[48:49], %0, %1\n v_cmp_lt_u64_e64 s[50:51], %0, %1\n v_cmp_lt_u64_e64 s[52:53], %0, %1\n v_cmp_lt_u64_e64 s[54:55], %0, %1\n v_cmp_lt_u64_e64 s[56:57], %0, %1\n v_cmp_lt_u64_e64 s[58:59], %0, %1" : "+v"(x0) : "v"(y) : "s44","s45","s46","s47","s48","s49","s50","s51","s52","s53","s54","s55","s56","s57","s58","s59");)
        } else if constexpr (OP == 3) {  // v_cvt_u32_f64
            REP64(asm volatile("v_cvt_u32_f64 %8, %0\n v_cvt_u32_f64 %9, %1\n v_cvt_u32_f64 %10, %2\n v_cvt_u32_f64 %11, %3\n v_cvt_u32_f64 %12, %4\n v_cvt_u32_f64 %13, %5\n v_cvt_u32_f64 %14, %6\n v_cvt_u32_f64 %15, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "=v"(u0), "=v"(u1), "=v"(u2), "=v"(u3), "=v"(u4), "=v"(u5), "=v"(u6), "=v"(u7));)
        } else if constexpr (OP == 4) {  // v_mul_u32_u24
            REP64(asm volatile("v_mul_u32_u24 %0, %0, %8\n v_mul_u32_u24 %1, %1, %8\n v_mul_u32_u24 %2, %2, %8\n v_mul_u32_u24 %3, %3, %8\n v_mul_u32_u24 %4, %4, %8\n v_mul_u32_u24 %5, %5, %8\n v_mul_u32_u24 %6, %6, %8\n v_mul_u32_u24 %7, %7, %8" : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(u4), "+v"(u5), "+v"(u6), "+v"(u7) : "v"(3u));)
        } else if constexpr (OP == 5) {  // v_cmp_lt_u32 -> sgpr pair
            REP64(asm volatile("v_cmp_lt_u32_e64 s[44:45], %0, %8\n v_cmp_lt_u32_e64 s[46:47], %1, %8\n v_cmp_lt_u32_e64 s[48:49], %2, %8\n v_cmp_lt_u32_e64 s[50:51], %3, %8\n v_cmp_lt_u32_e64 s[52:53], %4, %8\n v_cmp_lt_u32_e64 s[54:55], %5, %8\n v_cmp_lt_u32_e64 s[56:57], %6, %8\n v_cmp_lt_u32_e64 s[58:59], %7, %8" : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(u4), "+v"(u5), "+v"(u6), "+v"(u7) : "v"(9u) : "s44","s45","s46","s47","s48","s49","s50","s51","s52","s53","s54","s55","s56","s57","s58","s59");)
        } else if constexpr (OP == 6) {  // v_fma_f64
            REP64(asm volatile("v_fma_f64 %0, %0, %8, %8\n v_fma_f64 %1, %1, %8, %8\n v_fma_f64 %2, %2, %8, %8\n v_fma_f64 %3, %3, %8, %8\n v_fma_f64 %4, %4, %8, %8\n v_fma_f64 %5, %5, %8, %8\n v_fma_f64 %6, %6, %8, %8\n v_fma_f64 %7, %7, %8, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
        } else if constexpr (OP == 7) {  // v_mul_f32
            float f0 = a0, f1 = a1, f2 = a2, f3 = a3, f4 = a4, f5 = a5, f6 = a6, f7 = a7;
            REP64(asm volatile("v_mul_f32 %0, %0, %8\n v_mul_f32 %1, %1, %8\n v_mul_f32 %2, %2, %8\n v_mul_f32 %3, %3, %8\n v_mul_f32 %4, %4, %8\n v_mul_f32 %5, %5, %8\n v_mul_f32 %6, %6, %8\n v_mul_f32 %7, %7, %8" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7) : "v"(1.0001f));)
            fsink[threadIdx.x] = f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7;
        } else if constexpr (OP == 8) {  // v_mul_hi_u32
            REP64(asm volatile("v_mul_hi_u32 %0, %0, %8\n v_mul_hi_u32 %1, %1, %8\n v_mul_hi_u32 %2, %2, %8\n v_mul_hi_u32 %3, %3, %8\n v_mul_hi_u32 %4, %4, %8\n v_mul_hi_u32 %5, %5, %8\n v_mul_hi_u32 %6, %6, %8\n v_mul_hi_u32 %7, %7, %8" : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(u4), "+v"(u5), "+v"(u6), "+v"(u7) : "v"(0x9999999u));)
        } else if constexpr (OP == 9) {  // v_cmp_lt_f32
            float f0 = a0, f1 = a1, f2 = a2, f3 = a3, f4 = a4, f5 = a5, f6 = a6, f7 = a7;
            REP64(asm volatile("v_cmp_lt_f32_e64 s[44:45], %0, %8\n v_cmp_lt_f32_e64 s[46:47], %1, %8\n v_cmp_lt_f32_e64 s[48:49], %2, %8\n v_cmp_lt_f32_e64 s[50:51], %3, %8\n v_cmp_lt_f32_e64 s[52:53], %4, %8\n v_cmp_lt_f32_e64 s[54:55], %5, %8\n v_cmp_lt_f32_e64 s[56:57], %6, %8\n v_cmp_lt_f32_e64 s[58:59], %7, %8" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7) : "v"(2.0f) : "s44","s45","s46","s47","s48","s49","s50","s51","s52","s53","s54","s55","s56","s57","s58","s59");)
            fsink[threadIdx.x] = f0 + f1;
        } else if constexpr (OP == 10) {  // v_cndmask_b32 with sgpr-pair mask
            REP64(asm volatile("v_cndmask_b32_e64 %0, %0, %8, s[44:45]\n v_cndmask_b32_e64 %1, %1, %8, s[44:45]\n v_cndmask_b32_e64 %2, %2, %8, s[44:45]\n v_cndmask_b32_e64 %3, %3, %8, s[44:45]\n v_cndmask_b32_e64 %4, %4, %8, s[44:45]\n v_cndmask_b32_e64 %5, %5, %8, s[44:45]\n v_cndmask_b32_e64 %6, %6, %8, s[44:45]\n v_cndmask_b32_e64 %7, %7, %8, s[44:45]" : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3), "+v"(u4), "+v"(u5), "+v"(u6), "+v"(u7) : "v"(3u) : "s44","s45");)
        } else if constexpr (OP == 11) {  // v_cvt_f64_u32
            REP64(asm volatile("v_cvt_f64_u32 %0, %8\n v_cvt_f64_u32 %1, %9\n v_cvt_f64_u32 %2, %10\n v_cvt_f64_u32 %3, %11\n v_cvt_f64_u32 %4, %12\n v_cvt_f64_u32 %5, %13\n v_cvt_f64_u32 %6, %14\n v_cvt_f64_u32 %7, %15" : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7) : "v"(u0), "v"(u1), "v"(u2), "v"(u3), "v"(u4), "v"(u5), "v"(u6), "v"(u7));)
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = t1 - t0;
        out[2 * blockIdx.x + 1] = r1 - r0;
    }
    dsink[threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    usink[threadIdx.x] = u0 + u1 + u2 + u3 + u4 + u5 + u6 + u7 + (unsigned)x0;
}

template <int OP>
void run(const char* name, unsigned long long* d, double* ds, float* fs, unsigned* us) {
    for (int waves : {1, 4, 8, 16}) {
        // one workgroup of `waves` waves per CU x 256 CUs: waves per SIMD = waves / 4 rounded up
        hipLaunchKernelGGL(kern<OP>, dim3(256), dim3(64 * waves), 0, 0, d, ds, fs, us);
        hipDeviceSynchronize();
        unsigned long long h[512];
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        double avg = 0, rt = 0;
        for (int i = 0; i < 256; i++) {
            avg += h[2 * i];
            rt += h[2 * i + 1];
        }
        avg /= 256;
        rt /= 256;
        const double per_simd = waves < 4 ? 1.0 : waves / 4.0;  // waves sharing one SIMD's issue
        printf("%-16s waves/CU=%2d  %.2f ticks per wave-instruction per SIMD (clock %.0f MHz)\n", name, waves,
               avg / (16.0 * 512 * per_simd), avg / rt * 100.0);
    }
}

// Chip-wide rate: a grid far larger than the chip (4096 x 256 threads = 16 waves per SIMD over time),
// timed by events; cycles per wave-instruction per SIMD at the in-kernel clock.
template <int OP>
void run_grid(const char* name, unsigned long long* d, double* ds, float* fs, unsigned* us) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int blocks = 4096, threads = 256;
    hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(threads), 0, 0, d, ds, fs, us);  // warm
    hipEventRecord(a);
    for (int r = 0; r < 10; r++) hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(threads), 0, 0, d, ds, fs, us);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    unsigned long long h[512];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    double tk = 0, rt = 0;
    for (int i = 0; i < 256; i++) {
        tk += h[2 * i];
        rt += h[2 * i + 1];
    }
    const double mhz = tk / rt * 100.0;
    const double insts = 10.0 * blocks * (threads / 64) * 16.0 * 512;
    const double cyc = (ms * 1e-3) * mhz * 1e6 * 1024.0 / insts;
    printf("%-16s grid: %.3f ms for %.3g wave-inst = %.3g T/s; %.2f cycles per wave-instruction per SIMD at %.0f MHz\n",
           name, ms / 10, insts / 10, insts / (ms * 1e-3) / 1e12, cyc, mhz);
    hipEventDestroy(a);
    hipEventDestroy(b);
}

int main() {
    unsigned long long* d;
    double* ds;
    float* fs;
    unsigned* us;
    hipMalloc(&d, 512 * 8);
    hipMalloc(&ds, 8192 * 8);
    hipMalloc(&fs, 8192 * 4);
    hipMalloc(&us, 8192 * 4);
    run<0>("v_add_f64", d, ds, fs, us);
    run<1>("v_cmp_lt_f64", d, ds, fs, us);
    run<2>("v_cmp_lt_u64", d, ds, fs, us);
    run<3>("v_cvt_u32_f64", d, ds, fs, us);
    run<4>("v_mul_u32_u24", d, ds, fs, us);
    run<5>("v_cmp_lt_u32", d, ds, fs, us);
    run<6>("v_fma_f64", d, ds, fs, us);
    run<7>("v_mul_f32", d, ds, fs, us);
    run<8>("v_mul_hi_u32", d, ds, fs, us);
    run<9>("v_cmp_lt_f32", d, ds, fs, us);
    run<10>("v_cndmask_b32", d, ds, fs, us);
    run<11>("v_cvt_f64_u32", d, ds, fs, us);
    hipMalloc(&d, 8192 * 8);
    run_grid<0>("v_add_f64", d, ds, fs, us);
    run_grid<1>("v_cmp_lt_f64", d, ds, fs, us);
    run_grid<2>("v_cmp_lt_u64", d, ds, fs, us);
    run_grid<3>("v_cvt_u32_f64", d, ds, fs, us);
    run_grid<4>("v_mul_u32_u24", d, ds, fs, us);
    run_grid<5>("v_cmp_lt_u32", d, ds, fs, us);
    run_grid<6>("v_fma_f64", d, ds, fs, us);
    run_grid<7>("v_mul_f32", d, ds, fs, us);
    run_grid<8>("v_mul_hi_u32", d, ds, fs, us);
    run_grid<10>("v_cndmask_b32", d, ds, fs, us);
    return 0;
}
