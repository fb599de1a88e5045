"""Writes tests/golden/config3_replay.npz: the oracle's one-pod-per-cycle placements (global node index,
-1 = unschedulable) and totals for the whole config-3 sequence (synth.cluster(3): 50k pods on 10k nodes),
plus a digest of the generated cluster so a generator change is detected. The oracle's kgo_replay is the
checker (oracle/kg_oracle.c); replay_parallel runs the same cycles on 16 threads (equal placements, see
tests/test_host.py). Usage: python tests/golden/make_config3_golden.py"""
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle_lib  # noqa: E402
from koordinator_amd import abi, synth  # noqa: E402


def digest(nodes, pods) -> str:
    h = hashlib.sha256()
    for t in (nodes, pods):
        for k in sorted(t):
            h.update(k.encode())
            h.update(np.ascontiguousarray(t[k]).tobytes())
    return h.hexdigest()[:32]


def main():
    cfg, nodes, pods = synth.cluster(3)
    kc = cfg.kg_config()
    t0 = time.time()
    node, total = oracle_lib.OracleState(kc, nodes).replay_parallel(pods, 8)
    out = os.path.join(HERE, "config3_replay.npz")
    np.savez_compressed(out, node=node, total=total, digest=np.array(digest(nodes, pods)))
    print(out, f"{time.time() - t0:.1f}s placed {(node >= 0).sum()} / {abi.table_len(pods)}")


if __name__ == "__main__":
    main()
