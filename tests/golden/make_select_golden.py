"""Writes tests/golden/select_config{2,4,5}.npz: the oracle's per-pod top-3 selection keys (packed
(total << 32) | (0xFFFFFFFF - node), descending, 0 = no feasible node) for the WHOLE pod batch of the
BASELINE configurations that are evaluated in matrix mode:

  config 2  synth.cluster(2):  10k nodes x 10k pods, NodeResourcesFit + LoadAware + NodeNUMAResource
  config 4  synth.cluster(4):  100k nodes x 10k pods, same plugins
  config 5  synth.config5(): + DeviceShare, Reservation, ElasticQuota
  config 6  synth.mixed():     config 2 with Restricted / BestEffort nodes, node CPU bind policies and LSR
                               (cpuset-binding) pods (bench config 6)

plus a digest of the generated cluster (make_config3_golden.digest), so a generator change is detected
and the GPU box only compares (tests/test_select_golden.py). Top-1 is the first column (keys are unique:
the node index sits in the low half). The oracle (oracle/kg_oracle.c kgo_select / kgo_ext_select) is the
checker; pods are independent in matrix mode, so the batch is cut into pod ranges evaluated on a thread
pool (ctypes drops the GIL for the call). Usage: python tests/golden/make_select_golden.py [2 4 5 6]"""
import ctypes
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)

import oracle_lib  # noqa: E402
from koordinator_amd import abi, synth  # noqa: E402
from make_config3_golden import digest  # noqa: E402

K = 3


def path(config: int) -> str:
    return os.path.join(HERE, f"select_config{config}.npz")


def workload(config: int):
    """(kg_config, nodes, pods, quotas, reservations) of a matrix-mode configuration."""
    if config == 5:
        cfg, nodes, pods, quotas, rsv = synth.config5()
        return cfg.kg_config(), nodes, pods, quotas, rsv
    if config == 6:
        cfg, nodes, pods = synth.mixed()
        return cfg.kg_config(), nodes, pods, None, None
    cfg, nodes, pods = synth.cluster(config)
    return cfg.kg_config(), nodes, pods, None, None


def oracle_keys(kc, nodes, pods, quotas, rsv, idx, k=K):
    """Oracle top-k keys of pods[idx] (the whole snapshot, index base 0)."""
    sub = abi.take(pods, np.asarray(idx))
    if quotas is None and rsv is None:
        return oracle_lib.select(kc, nodes, sub, k)
    return oracle_lib.ext_select(kc, nodes, sub, k, 0, quotas, rsv)


def make(config: int, workers: int = os.cpu_count() or 8):
    kc, nodes, pods, quotas, rsv = workload(config)
    n = abi.table_len(pods)
    parts = np.array_split(np.arange(n), max(1, 8 * workers))
    t0 = time.time()
    with ThreadPoolExecutor(workers) as ex:
        keys = np.concatenate(list(ex.map(lambda ix: oracle_keys(kc, nodes, pods, quotas, rsv, ix), parts)))
    dig = _digest(nodes, pods, quotas, rsv)
    np.savez_compressed(path(config), keys=keys, digest=np.array(dig))
    print(path(config), f"{time.time() - t0:.1f}s", f"pods with a node {(keys[:, 0] != 0).sum()} / {n}")


def _digest(nodes, pods, quotas, rsv) -> str:
    if quotas is None and rsv is None:
        return digest(nodes, pods)
    extra = {f"q_{k}": v for k, v in (quotas or {}).items()}
    if rsv is not None:  # the reservation tables as the ABI sees them
        for name, arr, n in (("views", rsv.views, rsv.n_views), ("infos", rsv.infos, rsv.n_infos),
                             ("devs", rsv.devs, rsv.n_devs)):
            extra[f"r_{name}"] = np.frombuffer(bytes(arr), np.uint8)[: n * ctypes.sizeof(arr._type_)]
    return digest(nodes, {**pods, **extra})


def cluster_digest(config: int) -> str:
    _, nodes, pods, quotas, rsv = workload(config)
    return _digest(nodes, pods, quotas, rsv)


def load(config: int):
    g = np.load(path(config), allow_pickle=False)
    return g["keys"], str(g["digest"])


if __name__ == "__main__":
    for c in [int(a) for a in sys.argv[1:]] or [2, 4, 5, 6]:
        make(c)
