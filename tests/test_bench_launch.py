"""bench.py's multi-GPU entry point on CPU: `bench.py --gpus N` without a launcher starts N rank
processes with the rendezvous environment, and every rank reaches the gloo bootstrap and then the device
open (which fails here, without a GPU, with the library's KG_NO_DEVICE) — the parent itself never
touches the device."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_spawns_ranks_without_launcher():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                              "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0  # no GPU in this container
    err = r.stderr
    for dev in (0, 1):
        assert f"kg_open(device={dev})" in err, err[-2000:]
