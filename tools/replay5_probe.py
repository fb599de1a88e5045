"""The config-5 replay (bench.replay5_rate: 100k nodes x 10k pods, every plugin, GPU-holding reservations) as one
program, for a rocprofv3 kernel trace of its captured step graphs.
Usage (GPU box): rocprofv3 --kernel-trace --stats -d gpurun_out/r5trace -o run --output-format csv -- \\
                     python3 tools/replay5_probe.py
       python3 tools/replay5_probe.py --pods 1024   (the first 1024 pods only: PMC passes, one dispatch per step)"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from koordinator_amd import engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pods", type=int, default=0, help="replay only the first N pods of the sequence (0 = all)")
a = ap.parse_args()
ctx = engine.Context(0)
if a.pods:
    import numpy as np

    from koordinator_amd import abi, synth

    cfg, nodes, pods, quotas, rsv = synth.config5()
    snap = engine.Snapshot(ctx, cfg.kg_config(), nodes)
    snap.upload_quotas(quotas)
    snap.upload_reservations(rsv)
    batch = engine.PodBatch(ctx, abi.take(pods, np.arange(a.pods)))
    t0 = time.perf_counter()
    node, _ = engine.replay(snap, batch)
    dt = time.perf_counter() - t0
    print(json.dumps({"pods": a.pods, "seconds": dt, "placed": int((node >= 0).sum())}), flush=True)
else:
    print(json.dumps(bench.replay5_rate(ctx, False, 0.0)), flush=True)
ctx.close()
