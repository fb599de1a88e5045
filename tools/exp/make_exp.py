"""A/B variants of the replay step kernel (timing experiments only; never shipped): writes tools/exp/kg_ext_v<N>.hip
from koordinator_amd/csrc/kg_ext.hip with one piece of k_ext_replay cut, and links tools/exp/lib_v<N>.so."""
import os, subprocess, sys
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
src = open(os.path.join(R, "koordinator_amd/csrc/kg_ext.hip")).read()
EVAL = "            const PairX r = eval_pair_ext<EXACT>(cfg, e, nodes[i].v, zones + i, devs ? devs + i : nullptr, i, p, px, qst);\n            zsel["
RES = "    if (live && prev != 0ull) {\n        const uint32_t g = 0xFFFFFFFFu - (uint32_t)(prev & 0xFFFFFFFFull);\n        if (g == index_base + node_index(nodes[i])) {"
assert EVAL in src and RES in src
BASE = ("            PairX r; { const PairOut b = eval_pair<EXACT>(cfg, nodes[i].v, zones + i, p); r.status = b.status | qst; r.zone = b.zone;"
        " r.s_nrf = b.s_nrf; r.s_la = b.s_la; r.s_numa = b.s_numa; r.s_dev = 0; r.s_rsv = 0; r.order = 0; r.nom = -1; }\n            zsel[")
NORES = RES.replace("if (live && prev != 0ull)", "if (false && live && prev != 0ull)")
CONST = "            PairX r; r.status = 1; r.zone = -1; r.nom = -1; r.s_nrf = r.s_la = r.s_numa = r.s_dev = r.s_rsv = r.order = 0;\n            zsel["
TICK = "    if (lane == 0) ticket = atomicAdd(done, 1u);"
assert TICK in src
variants = {
    1: [(EVAL, EVAL.replace("const PairX r = eval_pair_ext", "PairX r = eval_pair_ext").replace(";\n", "; r.status = 1;\n", 1))],
    2: [(EVAL, BASE)],
    3: [(RES, RES.replace("if (live && prev != 0ull)", "if (false && live && prev != 0ull)"))],
    4: [(EVAL, BASE), (RES, NORES)],
    5: [(EVAL, BASE.replace("eval_pair<EXACT>(cfg,", "eval_pair<EXACT>(cfgn,").replace("PairX r; {", "PairX r; { KCfg cfgn = cfg; cfgn.plugins &= ~KG_PLUGIN_NUMA;")), (RES, NORES)],
    6: [(EVAL, CONST), (RES, NORES)],
    7: [(EVAL, CONST), (RES, NORES), (TICK, "    if (lane == 0) ticket = 0;")],
}
objs = [os.path.join(R, "build", f) for f in ("kg_kernels.hip.o", "kg_cpuset.hip.o", "kg_runtime.cpp.o")]
flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-fPIC", "-Wno-unused-value",
         "-I" + os.path.join(R, "koordinator_amd/csrc")]
procs = []
for v in map(int, sys.argv[1:] or variants):
    s = src
    for a, b in variants[v]:
        s = s.replace(a, b)
    f = os.path.join(R, "tools/exp", f"kg_ext_v{v}.hip")
    open(f, "w").write(s)
    o = f + ".o"
    procs.append((v, o, subprocess.Popen(["/opt/rocm/bin/hipcc", *flags, "-c", f, "-o", o])))
for v, o, p in procs:
    assert p.wait() == 0
    subprocess.check_call(["/opt/rocm/bin/hipcc", *flags, "-shared", o, *objs, "-o", os.path.join(R, "tools/exp", f"lib_v{v}.so"),
                           "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"])
    print("built", v)
