"""The config-5 replay (bench.replay5_rate: 100k nodes x 10k pods, every plugin, GPU-holding reservations) as one
program, for a rocprofv3 kernel trace of its captured step graphs.
Usage (GPU box): rocprofv3 --kernel-trace --stats -d gpurun_out/r5trace -o run --output-format csv -- \\
                     python3 tools/replay5_probe.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from koordinator_amd import engine  # noqa: E402

ctx = engine.Context(0)
print(json.dumps(bench.replay5_rate(ctx, False, 0.0)), flush=True)
ctx.close()
