"""Step timing of the config-5 replay kernel (profiling only, never shipped): writes tools/timing/kg_ext_replay_t.hip,
koordinator_amd/csrc/kg_ext_replay.hip with wall-clock stamps (s_memrealtime, 100 MHz) per step: first / last wave
start, last wave past the Reserve, past the evaluation, at the arrival, and the pick's end; links
tools/timing/libkoordgpu_t.so (load it with KG_LIB_PATH) exporting kg_step_timing_reset / kg_step_timing_read."""
import os
import subprocess

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
src = open(os.path.join(R, "koordinator_amd/csrc/kg_ext_replay.hip")).read()
HDR = """
#define KG_T_N 16384
__device__ unsigned long long kg_step_t[6][KG_T_N];
__device__ __forceinline__ void kg_stamp(int k, uint32_t step, bool mn) {
    // one wave in 16 workgroups stamps (same-address atomics from every wave would serialise and skew the clock)
    if ((threadIdx.x & 63u) != 0 || step >= KG_T_N || (k != 5 && (blockIdx.x & 15u) != 0)) return;
    const unsigned long long t = (unsigned long long)wall_clock64();
    if (mn) atomicMin(&kg_step_t[k][step], t); else atomicMax(&kg_step_t[k][step], t);
}
"""
edits = [
    ("namespace kg {\n", "namespace kg {\n" + HDR, 1),
    ("    const bool has_next = step < n_pods;\n    const uint64_t prev",
     "    const bool has_next = step < n_pods;\n    kg_stamp(0, step, true);\n    kg_stamp(1, step, false);\n    const uint64_t prev", 1),
    ("    // pod `step` on every record, before its ElasticQuota gate", "    kg_stamp(2, step, false);\n    // pod `step` on every record, before its ElasticQuota gate", 1),
    ("    // the previous Reserve's outcome, from the zone code", "    kg_stamp(3, step, false);\n    // the previous Reserve's outcome, from the zone code", 1),
    ("    __shared__ int last;\n", "    kg_stamp(4, step, false);\n    __shared__ int last;\n", 1),
    ("        if (lane == 0) winners[step] = w;\n    }\n", "        if (lane == 0) winners[step] = w;\n    }\n    kg_stamp(5, step, false);\n", 1),
]
import sys
if "--split" in sys.argv:  # the two-launch fast-base step: stamps of k_ext_replay_pre and k_ext_replay_fast
    edits = [edits[0],
        ("    const PodX px = load_podx(pods, has_next ? step : 0);\n    if (blockIdx.x == 0) {\n        uint64_t* Z",
         "    const PodX px = load_podx(pods, has_next ? step : 0);\n    kg_stamp(0, step, true);\n    if (blockIdx.x == 0) {\n        uint64_t* Z", 1),
        ("            ctl[step & 1u] = qst;\n", "            ctl[step & 1u] = qst;\n            kg_stamp(1, step, false);\n", 1),
        ("        replay_general_contrib<EXACT>(cfg, e, nodes, zones, devs, pods, step, rec, n_nodes, index_base, p, px, buckets, zsel,\n                                      nsel, rs, rlist);\n    }\n",
         "        replay_general_contrib<EXACT>(cfg, e, nodes, zones, devs, pods, step, rec, n_nodes, index_base, p, px, buckets, zsel,\n                                      nsel, rs, rlist);\n    }\n    kg_stamp(2, step, false);\n", 1),
        ("    const uint32_t qst = ctl[step & 1u];\n    uint64_t kb = 0;", "    const uint32_t qst = ctl[step & 1u];\n    if ((blockIdx.x & 15u) == 0) { kg_stamp(3, step, true); kg_stamp(4, step, false); }\n    uint64_t kb = 0;", 1),
        ("    if (!last || threadIdx.x >= 64u) return;\n    const uint64_t w = qst", "    if (!last || threadIdx.x >= 64u) return;\n    kg_stamp(5, step, false);\n    const uint64_t w = qst", 1),
    ]
if "--stub" in sys.argv:  # no out-of-line paths: the fast pairs alone (timing of a scratch-free kernel)
    edits += [
        ("            refresh = replay_reserve(cfg, e, nodes, zones, devs, pods, step - 1, i, prev_zone, nom, minors + step - 1);",
         "            refresh = false;", 1),
        ("    if (const uint64_t own = __ballot(refresh))  // uniform per wave: the winner's workgroup\n        replay_refresh(",
         "    if (const uint64_t own = __ballot(refresh) & 0ull)\n        replay_refresh(", 1),
        ("            const PairX r = replay_general_pair<EXACT>(cfg, e, nodes[i].v, zones + i, devs ? devs + i : nullptr, i, p, px, dcls);",
         "            PairX r{}; r.status = 1; r.zone = -1; r.nom = -1;", 1),
    ]
for a, b, n in edits:
    assert src.count(a) >= 1, a
    src = src.replace(a, b, n)
src += """
extern "C" int kg_step_timing_reset() {
    static unsigned long long h[6][KG_T_N];
    for (int k = 0; k < 6; k++)
        for (int s = 0; s < KG_T_N; s++) h[k][s] = k == 0 ? ~0ull : 0ull;
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(kg::kg_step_t), h, sizeof(h));
}
extern "C" int kg_step_timing_read(unsigned long long* out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(kg::kg_step_t), sizeof(unsigned long long) * 6 * KG_T_N);
}
"""
out = os.path.join(R, "tools/timing/kg_ext_replay_t.hip")
open(out, "w").write(src)
flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-fPIC", "-Wno-unused-value",
         "-I" + os.path.join(R, "koordinator_amd/csrc")]
objs = [os.path.join(R, "build", f) for f in ("kg_kernels.hip.o", "kg_ext.hip.o", "kg_ext_batch.hip.o", "kg_cpuset.hip.o",
                                              "kg_runtime.cpp.o")]
subprocess.check_call(["/opt/rocm/bin/hipcc", *flags, "-c", out, "-o", out + ".o"])
subprocess.check_call(["/opt/rocm/bin/hipcc", *flags, "-shared", out + ".o", *objs, "-o",
                       os.path.join(R, "tools/timing/libkoordgpu_t%s.so" % ("_stub" if "--stub" in sys.argv else "_split" if "--split" in sys.argv else "")), "-L/opt/rocm/lib", "-lrccl",
                       "-Wl,-rpath,/opt/rocm/lib"])
os.remove(out + ".o")
print("built tools/timing/libkoordgpu_t.so")
