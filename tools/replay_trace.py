"""Config-3 replay alone (for rocprofv3 kernel traces: run with KG_REPLAY_NOGRAPH=1 so the tracer sees
the window kernels as direct launches).  python tools/replay_trace.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from koordinator_amd import abi, engine, synth  # noqa: E402

cfg, nodes, pods = synth.cluster(3)
ctx = engine.Context(0)
snap = engine.Snapshot(ctx, cfg.kg_config(), nodes)
batch = engine.PodBatch(ctx, pods)
engine.replay(snap, engine.PodBatch(ctx, abi.take(pods, np.arange(512))))
snap.upload(nodes)
t0 = time.perf_counter()
node, _ = engine.replay(snap, batch)
dt = time.perf_counter() - t0
print(f"{batch.n / dt:.0f} pods/s, {int((node >= 0).sum())} placed, {dt:.3f} s")
ctx.close()
