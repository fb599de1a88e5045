"""Per-step stamps of the config-5 replay (GPU box): KG_LIB_PATH=tools/timing/libkoordgpu_t.so python3 this.py
-> gpurun_out/step_timing.npz (6 x steps, 100 MHz ticks) and a summary line per pod kind."""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from koordinator_amd import abi, engine, synth  # noqa: E402

ctx = engine.Context(0)
L = ctx.L
cfg, nodes, pods, quotas, rsv = synth.config5()
snap = engine.Snapshot(ctx, cfg.kg_config(), nodes)
snap.upload_quotas(quotas)
snap.upload_reservations(rsv)
engine.replay(snap, engine.PodBatch(ctx, abi.take(pods, np.arange(256))))
snap.upload(nodes)
snap.upload_quotas(quotas)
snap.upload_reservations(rsv)
batch = engine.PodBatch(ctx, pods)
assert L.kg_step_timing_reset() == 0
node, _ = engine.replay(snap, batch)
T = np.zeros((6, 16384), np.uint64)
assert L.kg_step_timing_read(T.ctypes.data_as(C.POINTER(C.c_ulonglong))) == 0
n = batch.n
T = T[:, :n].astype(np.int64)
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/step_timing.npz", T=T)
us = lambda a: float(np.median(a)) / 100.0 * 1e6 / 1e6 * 1e0  # ticks (10 ns) -> us
if len(sys.argv) > 1 and sys.argv[1] == "split":  # pre start / WG0 done / specials done / fast start min, max / pick
    d = {"pre_wg0": np.median(T[1] - T[0]) / 100, "pre_spec": np.median(T[2] - T[0]) / 100,
         "fast_start": np.median(T[3] - T[0]) / 100, "fast_start_max": np.median(T[4] - T[0]) / 100,
         "pick": np.median(T[5] - T[0]) / 100, "gap_to_next": np.median(T[0][1:] - T[5][:-1]) / 100,
         "mean_step": float(np.mean(T[0][1:] - T[0][:-1])) / 100}
    print(json.dumps({k: round(float(v), 2) for k, v in d.items()}), flush=True)
    sys.exit(0)
d = {"start_spread": np.median(T[1] - T[0]) / 100, "reserve": np.median(T[2] - T[0]) / 100,
     "eval": np.median(T[3] - T[0]) / 100, "arrive": np.median(T[4] - T[0]) / 100, "pick": np.median(T[5] - T[0]) / 100,
     "gap_to_next": np.median(T[0][1:] - T[5][:-1]) / 100}
print(json.dumps({k: round(float(v), 2) for k, v in d.items()}), flush=True)
ctx.close()
