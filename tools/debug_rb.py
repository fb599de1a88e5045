import ctypes as C
import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np
import oracle_lib
from koordinator_amd import engine, synth, abi
strategy = sys.argv[1]
cfg, nodes, pods = synth.topology(1200, 2500, seed=5)
cfg.numa_strategy = strategy
kc = cfg.kg_config()
ctx = engine.Context(0)
snap = engine.Snapshot(ctx, kc, nodes)
w = abi.take(pods, np.arange(64))
b = engine.PodBatch(ctx, w)
lists = np.zeros((64, 16), np.uint64)
placed = np.zeros(1, np.uint32)
win = np.zeros(64, np.uint64)
L = ctx.L
L.kg_debug_rb_window.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
rc = L.kg_debug_rb_window(snap.h, b.h, lists.ctypes.data, placed.ctypes.data, win.ctypes.data)
print("rc", rc, "placed", placed[0])
want = oracle_lib.select(kc, nodes, w, 16)
print("lists equal", np.array_equal(lists, want))
for t in range(3):
    print(t, "gpu", [(int(abi.key_node(k)), int(abi.key_total(k))) for k in lists[t][:4]])
    print(t, "orc", [(int(abi.key_node(k)), int(abi.key_total(k))) for k in want[t][:4]])
bad = np.nonzero((lists != want).any(axis=1))[0]
print("pods with different lists", bad[:10], len(bad))
# hypotheses: lists of another pod, or lists under the other NUMA strategy
for t in range(3):
    hits = [u for u in range(64) if np.array_equal(lists[t], want[u])]
    print("pod", t, "matches oracle pod", hits)
cfg.numa_strategy = "LeastAllocated"
kl = cfg.kg_config()
wl = oracle_lib.select(kl, nodes, w, 16)
print("vs LeastAllocated oracle:", int((lists == wl).all(axis=1).sum()), "of 64 pods equal")
cfg.numa_strategy = strategy
cfg.numa_hint_strategy = "MostAllocated"
km = cfg.kg_config()
wm = oracle_lib.select(km, nodes, w, 16)
print("vs hint-Most oracle:", int((lists == wm).all(axis=1).sum()), "of 64 pods equal")
v = oracle_lib.eval_verify(kc, nodes, w)
gv = engine.eval_verify(snap, b)
print("verify equal on same snapshot after the window:", all(np.array_equal(getattr(gv, f), getattr(v, f)) for f in ("status", "total")))
