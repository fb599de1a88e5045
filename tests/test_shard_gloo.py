"""Node-sharded selectHost across ranks on CPU: world_size 2 over gloo.

Each rank evaluates its contiguous node shard (snapshot indices [start, end), index_base = start)
with the oracle, the per-pod top-k keys are all-gathered exactly as kg_shard_select exchanges them
over RCCL, and every rank merges them with the library's kg_merge_keys (host code of
libkoordgpu.so, no device needed). The merged keys must equal the unsharded selection.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n_nodes, n_pods, k, bounds, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_lib
        from koordinator_amd import abi, engine, synth

        cfg, nodes, pods = synth.small(n_nodes, n_pods, seed=31, numa=True, scale=4.0)
        kc = cfg.kg_config()
        lo, hi = bounds[rank], bounds[rank + 1]
        shard = abi.take(nodes, np.arange(lo, hi))
        local = oracle_lib.select(kc, shard, pods, k, index_base=lo)  # [pods, k] uint64
        gathered = [torch.zeros(n_pods * k, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(gathered, torch.from_numpy(local.reshape(-1).view(np.int64).copy()))
        allk = np.stack([g.numpy().view(np.uint64).reshape(n_pods, k) for g in gathered])
        merged = engine.merge_keys(allk)
        want = oracle_lib.select(kc, nodes, pods, k)
        q.put((rank, bool(np.array_equal(merged, want)), int((want[:, 0] != 0).sum())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bounds,k", [((0, 500, 1000), 1), ((0, 333, 1000), 3), ((0, 1, 1000), 2),
                                     ((0, 250, 500, 750, 1000), 3), ((0, 100, 101, 600, 1000), 3)])
def test_sharded_select_matches_global(bounds, k):
    """P x k per-shard keys all-gathered (world 2 and 4, k up to 3 = numberOfHighestScoredNodesToReport)
    and merged: the global top-k, including an empty shard's contribution."""
    world = len(bounds) - 1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 1000, 128, k, bounds, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    for p in procs:
        if p.is_alive():
            p.kill()
        assert p.exitcode == 0
    res = sorted(q.get(timeout=5) for _ in range(world))
    assert all(ok for _, ok, _ in res), res
    assert res[0][2] > 0  # some pods are schedulable


def _ext_worker(rank, world, port, n_nodes, n_pods, k, bounds, q):
    """Config 5 sharded: per-shard NormalizeScore inputs all-reduced (MAX / MIN) exactly as
    kg_shard_select does over RCCL, then per-shard top-k, all-gather, merge."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_lib
        from koordinator_amd import abi, engine, synth

        cfg, nodes, pods, quotas, rsv = synth.cluster5(n_nodes, n_pods, seed_config=51, rsv_frac=0.3)
        kc = cfg.kg_config()
        lo, hi = bounds[rank], bounds[rank + 1]
        shard = abi.take(nodes, np.arange(lo, hi))
        srsv = rsv.shard(lo, hi)
        dm, rm, pf = oracle_lib.ext_shard_stats(kc, shard, pods, lo, quotas, srsv)
        tdm = torch.from_numpy(dm.astype(np.int64))
        trm = torch.from_numpy(rm.astype(np.int64))
        tpf = torch.from_numpy(pf.view(np.int64) ^ np.int64(-2**63))  # unsigned order as signed
        dist.all_reduce(tdm, op=dist.ReduceOp.MAX)
        dist.all_reduce(trm, op=dist.ReduceOp.MAX)
        dist.all_reduce(tpf, op=dist.ReduceOp.MIN)
        gpf = (tpf.numpy() ^ np.int64(-2**63)).view(np.uint64)
        local = oracle_lib.ext_shard_select(kc, shard, pods, lo, tdm.numpy().astype(np.uint32),
                                            trm.numpy().astype(np.uint32), gpf, k, quotas, srsv)
        gathered = [torch.zeros(n_pods * k, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(gathered, torch.from_numpy(local.reshape(-1).view(np.int64).copy()))
        allk = np.stack([g.numpy().view(np.uint64).reshape(n_pods, k) for g in gathered])
        merged = engine.merge_keys(allk)
        want = oracle_lib.ext_select(kc, nodes, pods, k, 0, quotas, rsv)
        q.put((rank, bool(np.array_equal(merged, want)), int((want[:, 0] != 0).sum()),
               int((abi.key_total(want[:, 0]) >= 500000).sum())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bounds,k", [((0, 400, 900), 1), ((0, 450, 900), 3), ((0, 200, 450, 700, 900), 3)])
def test_sharded_ext_select_matches_global(bounds, k):
    world = len(bounds) - 1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ext_worker, args=(r, world, port, 900, 160, k, bounds, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    for p in procs:
        if p.is_alive():
            p.kill()
        assert p.exitcode == 0
    res = sorted(q.get(timeout=5) for _ in range(world))
    assert all(ok for _, ok, _, _ in res), res
    assert res[0][2] > 0 and res[0][3] > 0  # schedulable pods, some on their preferred reservation node
