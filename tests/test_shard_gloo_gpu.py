"""Node-sharded selectHost with DEVICE-computed shard keys: world_size 2 over gloo.

test_shard_gloo.py merges oracle-computed shard keys; here each rank is its own process with its own
koordgpu context on cuda:0 (one box has one GPU, and RCCL refuses two ranks on one device, so the
exchange runs over gloo). Each rank evaluates its contiguous node shard on the GPU through the C-ABI
(kg_snapshot_create with index_base = shard start, kg_eval_select), the per-pod top-k keys are
all-gathered exactly as kg_shard_select exchanges them, and kg_merge_keys merges them. The merged
keys must equal the oracle's unsharded selection (bit-exact). Reference: upstream selectHost over
one cycle's nodes (k8s.io/kubernetes pkg/scheduler, SURVEY.md:40 and :140), sharded as SURVEY.md:236.
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

        cfg, nodes, pods = synth.small(n_nodes, n_pods, seed=37, numa=True, scale=4.0)
        kc = cfg.kg_config()
        lo, hi = bounds[rank], bounds[rank + 1]
        ctx = engine.Context(0)
        try:
            batch = engine.PodBatch(ctx, pods)
            snap = engine.Snapshot(ctx, kc, abi.take(nodes, np.arange(lo, hi)), index_base=int(lo))
            local = engine.eval_select(snap, batch, k)  # [pods, k] uint64, computed on the GPU
            snap.close()
        finally:
            ctx.close()
        gathered = [torch.zeros(n_pods * k, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(gathered, torch.from_numpy(np.ascontiguousarray(local).reshape(-1).view(np.int64).copy()))
        allk = np.stack([g.numpy().view(np.uint64).reshape(n_pods, k) for g in gathered])
        merged = engine.merge_keys(allk)
        want = oracle_lib.select(kc, nodes, pods, k)
        q.put((rank, bool(np.array_equal(merged, want)), int((want[:, 0] != 0).sum())))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("bounds,k", [((0, 1000, 2000), 1), ((0, 700, 2000), 3)])
def test_device_sharded_select_matches_global(bounds, k):
    world = len(bounds) - 1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 2000, 256, k, bounds, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
    for p in procs:
        if p.is_alive():
            p.kill()
        assert p.exitcode == 0
    res = sorted(q.get(timeout=5) for _ in range(world))
    assert all(ok for _, ok, _ in res), res
    assert res[0][2] > 0
