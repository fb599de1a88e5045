// Hardware probe for the gfx950 scalar-load addressing behind the round-3 gpu_partition discrepancy
// (tools/dbg_part.hip, DESIGN.md "Toolchain findings"): the compiler emitted s_load_dword with an SGPR base of
// struct + 2 and an immediate offset of 2 (a dword-aligned sum). This kernel issues exactly that form -- a scalar
// LOAD, nothing is written through the scalar cache -- and reports which dword came back.
//   out[0] = dword read from base(buf + 2 bytes) + 0x2   (buf[1] if the sum is used; buf[0] if SBASE[1:0] is dropped)
//   out[1] = dword read from base(buf + 4 bytes) + 0x0   (control: buf[1])
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void k_sload_probe(const uint32_t* buf, uint32_t* out) {
    const uint64_t b2 = (uint64_t)buf + 2, b4 = (uint64_t)buf + 4;
    uint32_t v0, v1;
    asm volatile("s_load_dword %0, %1, 0x2\n\ts_waitcnt lgkmcnt(0)" : "=s"(v0) : "s"(b2) : "memory");
    asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v1) : "s"(b4) : "memory");
    if (threadIdx.x == 0) {
        out[0] = v0;
        out[1] = v1;
    }
}

extern "C" int sload_probe(uint32_t* host_out) {
    uint32_t h[4] = {0x11111111u, 0x22222222u, 0x33333333u, 0x44444444u};
    uint32_t *d = nullptr, *o = nullptr;
    if (hipMalloc(&d, sizeof(h)) != hipSuccess || hipMalloc(&o, 8) != hipSuccess) return 1;
    if (hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) return 2;
    k_sload_probe<<<1, 64>>>(d, o);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    if (hipMemcpy(host_out, o, 8, hipMemcpyDeviceToHost) != hipSuccess) return 4;
    hipFree(d);
    hipFree(o);
    return 0;
}
