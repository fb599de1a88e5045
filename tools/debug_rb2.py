import ctypes as C
import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np
import oracle_lib
from koordinator_amd import engine, synth, abi
cfg, nodes, pods = synth.topology(1200, 2500, seed=5)
cfg.numa_strategy = sys.argv[1]
kc = cfg.kg_config()
ctx = engine.Context(0)
w = abi.take(pods, np.arange(64))
v = oracle_lib.eval_verify(kc, nodes, w)
snap = engine.Snapshot(ctx, kc, nodes)
b = engine.PodBatch(ctx, w)
lists = np.zeros((64, 16), np.uint64)
placed = np.zeros(1, np.uint32)
win = np.zeros(64, np.uint64)
L = ctx.L
L.kg_debug_rb_window.argtypes = [C.c_void_p] * 5
L.kg_debug_rb_window(snap.h, b.h, lists.ctypes.data, placed.ctypes.data, win.ctypes.data)
for t in range(4):
    row = []
    for k in lists[t][:8]:
        i = int(abi.key_node(k)); g = int(abi.key_total(k))
        row.append((i, g, int(v.total[t, i]), int(nodes["numa_policy"][i]), int(nodes["numa_zones"][i]), int(v.score_numa[t, i])))
    print("pod", t, "pol", int(pods["numa_policy"][t]), row)
