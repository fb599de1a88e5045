"""Writes tests/golden/replay5_head.npz: the oracle's one-pod-per-cycle config-5 replay at the BASELINE size
(synth.config5(): 100k nodes, every plugin, reservations holding GPUs with their DeviceShare restore inputs, ElasticQuota)
for the first N_HEAD pods of the batch: per pod the global node index (-1 = unschedulable), the total, the GPU minors
chosen and the FitError reason bits, plus the final quota used and a digest of the generated cluster (the select
golden's digest, make_select_golden._digest) so a generator change is detected. The checker is the oracle's
kgo_ext_replay_parallel (oracle/kg_oracle.c; placements equal the serial kgo_ext_replay, tests/test_rsv_replay.py).
Usage: python tests/golden/make_replay5_golden.py"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)

import oracle_lib  # noqa: E402
from koordinator_amd import abi, synth  # noqa: E402
from make_select_golden import _digest  # noqa: E402

N_HEAD = 3000
PATH = os.path.join(HERE, "replay5_head.npz")


def workload():
    cfg, nodes, pods, quotas, rsv = synth.config5()
    return cfg.kg_config(), nodes, pods, quotas, rsv


def main():
    kc, nodes, pods, quotas, rsv = workload()
    head = abi.take(pods, np.arange(N_HEAD))
    t0 = time.time()
    node, total, minors, qu, qn, why = oracle_lib.OracleState(kc, nodes).ext_replay(
        head, quotas, rsv=rsv, reasons=True, workers=os.cpu_count() or 8)
    np.savez_compressed(PATH, node=node, total=total, minors=minors, reason=why, quota_used=qu, quota_np_used=qn,
                        digest=np.array(_digest(nodes, pods, quotas, rsv)))
    print(PATH, f"{time.time() - t0:.1f}s placed {(node >= 0).sum()} / {N_HEAD}")


if __name__ == "__main__":
    main()
