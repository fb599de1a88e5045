"""Benchmark of the MI355X Filter/Score evaluation engine (BASELINE.json metric).

One step = one pass of the hot path over one batch: Filter + Score of every pending pod against
every node of the snapshot (NodeResourcesFit + LoadAwareScheduling + NodeNUMAResource) and the
selectHost of each pod — config 2 of BASELINE.md (10k nodes x 10k pods) per GPU. With --gpus N the
nodes are sharded (10k per GPU, weak scaling): each rank evaluates its shard, the per-pod best keys
are all-gathered over RCCL and every rank runs the same global selectHost.

Prints ONE JSON line on rank 0 (value = evals/s over all ranks, inputs resident in HBM).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from koordinator_amd import abi, engine, synth  # noqa: E402

HBM_PEAK = 8.0e12  # MI355X HBM3E peak B/s (MI355X_MICROARCH.md, chip-level parameters)
# Algorithmic bytes per (pod, node) eval, SURVEY.md §8d (scan model, node row read once per eval):
# NodeResourcesFit 120 B + LoadAware 52 B + NodeNUMAResource 4 B + 0.2 x 64 B zone table = 188.8 B.
B_EVAL = {1: 172.0, 2: 188.8, 4: 188.8,
          # config 5: + DeviceShare 384 B x 30% GPU pods + Reservation 4 B node flag (308 B)
          5: 308.0}
METRIC = "Filter+Score pod-node evals/sec"
PLUGINS = {1: "+LoadAware", 2: "+LoadAware+NodeNUMAResource", 4: "+LoadAware+NodeNUMAResource",
           5: "+LoadAware+NodeNUMAResource+DeviceShare+Reservation+ElasticQuota"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=[1, 2, 4, 5],
                    help="2: 10k nodes per GPU x 10k pods (weak scaling, default); 4: 100k nodes split over "
                         "the GPUs x 10k pods (strong scaling); 5: config 4 + DeviceShare / Reservation / "
                         "ElasticQuota; 1: the 1k x 500 CPU-harness case")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-replay", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    return ap.parse_args()


# VALU issue peak in wave-instructions/s: 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU
# instruction (MI355X_MICROARCH.md: a wave issues each VALU instruction over 2 cycles)
VALU_PEAK = 256 * 4 * 2.4e9 / 2


def load_pmc():
    """The committed rocprofv3 PMC summary of the select kernels (tools/pmc_summary.py), or {}."""
    path = os.path.join(ROOT, "profiles", "select_pmc.json")
    if not os.path.exists(path):
        return {}
    try:
        with open(path) as f:
            return json.load(f)
    except Exception:
        return {}


def load_traffic():
    """HBM bytes per select launch from the committed rocprofv3 PMC summary (or None)."""
    return load_pmc().get("hbm_bytes_per_launch")


def valu_issue(avg_kernel_s):
    """The select's actual ceiling: VALU wave-instructions per launch (SQ_INSTS_VALU of the committed
    PMC pass, summed over the k_select kernels of one step) / the live kernel time, against VALU_PEAK."""
    ks = load_pmc().get("kernels", {})
    insts = sum(v["counters"].get("SQ_INSTS_VALU", 0.0) for k, v in ks.items() if "k_select<" in k)
    if not insts or not avg_kernel_s:
        return None
    a = insts / avg_kernel_s
    return {"bound": "valu", "achieved": a / 1e12, "peak": VALU_PEAK / 1e12, "unit": "T wave-inst/s",
            "frac": a / VALU_PEAK, "insts_per_launch": insts,
            "note": "pod tiling serves one node read to 64 pods, so the scan-model HBM frac exceeds 1; the "
                    "kernel is VALU-issue bound (float64 ops issue over 4 cycles, so this frac is a lower bound)"}


def cpu_baseline(cfg, nodes, pods, target_s):
    """Oracle (C restatement, upstream-shaped 16-worker parallelizer) on a bounded pod sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib  # test infrastructure: the CPU baseline leg only

    workers = 16
    kc = cfg.kg_config()
    n_nodes = abi.table_len(nodes)
    probe = 8
    t0 = time.perf_counter()
    oracle_lib.select_parallel(kc, nodes, abi.take(pods, np.arange(probe)), workers)
    dt = max(time.perf_counter() - t0, 1e-6)
    n = int(min(abi.table_len(pods), max(probe, target_s / (dt / probe))))
    sample = abi.take(pods, np.arange(n))
    t0 = time.perf_counter()
    oracle_lib.select_parallel(kc, nodes, sample, workers)
    dt = time.perf_counter() - t0
    return {"value": n * n_nodes / dt, "unit": "evals/s", "cores": workers, "kind": "port",
            "sample": f"{n} pods x {n_nodes} nodes ({n * n_nodes} evals) in {dt:.2f} s; oracle/kg_oracle.c "
                      f"kgo_select_parallel: per pod parallel Filter then parallel Score over nodes, "
                      f"{workers} workers, chunked like pkg/util/parallelize/parallelism.go:29-49"}


def cpu_baseline_ext(kc, nodes, pods, quotas, rsv, target_s):
    """Config 5: the oracle's restatement (one thread) on a bounded pod sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib  # test infrastructure: the CPU baseline leg only

    n_nodes = abi.table_len(nodes)
    probe = 4
    t0 = time.perf_counter()
    oracle_lib.ext_select(kc, nodes, abi.take(pods, np.arange(probe)), 1, 0, quotas, rsv)
    dt = max(time.perf_counter() - t0, 1e-6)
    n = int(min(abi.table_len(pods), max(probe, target_s / (dt / probe))))
    t0 = time.perf_counter()
    oracle_lib.ext_select(kc, nodes, abi.take(pods, np.arange(n)), 1, 0, quotas, rsv)
    dt = time.perf_counter() - t0
    return {"value": n * n_nodes / dt, "unit": "evals/s", "cores": 1, "kind": "port",
            "sample": f"{n} pods x {n_nodes} nodes ({n * n_nodes} evals) in {dt:.2f} s; oracle/kg_oracle.c "
                      f"kgo_ext_select (all six plugins, NormalizeScore, selectHost), one thread"}


def replay_rate(ctx, cfg, with_cpu):
    """Config 3: 50k pods placed one by one on 10k nodes with device-resident Assume."""
    _, nodes, pods = synth.cluster(3)
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, nodes)
    batch = engine.PodBatch(ctx, pods)
    small = engine.PodBatch(ctx, abi.take(pods, np.arange(512)))
    engine.replay(snap, small)  # warm-up (graph instantiate, code load)
    snap.upload(nodes)
    t0 = time.perf_counter()
    node, _ = engine.replay(snap, batch)
    dt = time.perf_counter() - t0
    placed = int((node >= 0).sum())
    out = {"pods_placed_per_s": batch.n / dt, "pods": batch.n, "placed": placed,
           "unschedulable": batch.n - placed, "seconds": round(dt, 4),
           "workload": "config3: 10k nodes x 50k pods, one pod per cycle, Assume on device"}
    if with_cpu:
        # CPU baseline: the oracle's sequential replay (one thread) of the first pods of the same sequence
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib  # test infrastructure: the CPU baseline leg only

        n = 1500
        st = oracle_lib.OracleState(kc, nodes)
        t0 = time.perf_counter()
        want, _ = st.replay(abi.take(pods, np.arange(n)))
        cdt = time.perf_counter() - t0
        assert np.array_equal(want, node[:n])  # same placements as the device replay
        out["cpu_baseline"] = {"value": n / cdt, "unit": "pods/s", "cores": 1, "kind": "port",
                               "sample": f"first {n} pods of the config-3 sequence, oracle/kg_oracle.c kgo_replay "
                                         f"(sequential Filter+Score over all nodes + Assume), {cdt:.2f} s"}
    return out


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(a.gpus)))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # bootstrap + host barriers only (data path is RCCL in the library)

        dist.init_process_group("gloo")
    ctx = engine.Context(local)
    quotas = rsv = None
    if a.config == 5:
        cfg, nodes, pods, quotas, rsv = synth.cluster5(100_000, 10_000)
    else:
        cfg, nodes, pods = synth.cluster(a.config)
    if a.config in (4, 5):
        # one 100k-node cluster, contiguous shard per rank (strong scaling)
        bounds = np.linspace(0, abi.table_len(nodes), world + 1).astype(np.int64)
        base = int(bounds[rank])
        nodes = abi.take(nodes, np.arange(bounds[rank], bounds[rank + 1]))
        if rsv is not None:
            rsv = rsv.shard(int(bounds[rank]), int(bounds[rank + 1]))
        n_local = abi.table_len(nodes)
        n_total = int(bounds[-1])
    else:
        # one 10k-node shard per rank (weak scaling)
        n_local = abi.table_len(nodes)
        if world > 1:
            nodes = synth.nodes(n_local, a.config + 10 * rank, numa=(a.config == 2))
        base = rank * n_local
        n_total = n_local * world
    if world > 1:
        uid = [engine.shard_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ctx.shard_init(uid[0], rank, world)
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, nodes, index_base=base)
    if quotas is not None:
        snap.upload_quotas(quotas)
    if rsv is not None:
        snap.upload_reservations(rsv)
    batch = engine.PodBatch(ctx, pods)
    n_pods = batch.n

    def step():
        if world > 1:
            engine.shard_select(snap, batch, download=False)
        else:
            engine.eval_select_async(snap, batch, 1)

    for _ in range(a.warmup):
        step()
    ctx.sync()
    ctx.profile(True)
    ctx.profile_read(reset=True)
    if dist:
        dist.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    ctx.sync()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    kern_ms, launches = ctx.profile_read(reset=True)
    ctx.profile(False)
    elapsed = t1 - t0
    if dist:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # check the result of the last step is sane (feasible keys point into the cluster)
    keys = engine.result_keys(batch, 1)[:, 0]
    idx = abi.key_node(keys)
    assert np.all(idx[keys != 0] < n_total)

    evals = float(n_pods) * n_total * a.steps
    value = evals / elapsed
    avg_kernel_s = (kern_ms / 1e3) / max(launches, 1)
    achieved = (float(n_pods) * n_local * B_EVAL[a.config]) / avg_kernel_s if launches else None
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "evals/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if a.config in (4, 5) else "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (PCG64 seed 0x6B6F6F7264, SURVEY.md §8d distributions)",
        "config": {"workload": f"config{a.config}: {n_local} nodes/GPU x {n_pods} pods, Filter+Score+selectHost "
                               f"(NodeResourcesFit{PLUGINS[a.config]})",
                   "nodes_per_gpu": n_local, "nodes_total": n_total, "pods": n_pods,
                   "parallelism": f"node-shard x{world}" + (" + RCCL all-gather of per-pod best keys" if world > 1 else "")},
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9 if achieved else None, "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": (achieved / HBM_PEAK) if achieved else None,
                     "traffic": load_traffic() if a.config != 5 else None,
                     "kernel": "k_select" if a.config != 5 else "k_ext_select + k_select (plain-pod split, one bracket)", "kernel_avg_ms": avg_kernel_s * 1e3,
                     "bytes_per_eval": B_EVAL[a.config], "evals_per_launch": n_pods * n_local,
                     "issue": valu_issue(avg_kernel_s) if a.config == 2 and world == 1 else None},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1:
        if a.config == 5:
            if not a.no_cpu_baseline:
                out["cpu_baseline"] = cpu_baseline_ext(kc, nodes, pods, quotas, rsv, a.cpu_seconds)
        else:
            if not a.no_replay:
                out["replay"] = replay_rate(ctx, cfg, not a.no_cpu_baseline)
            if not a.no_cpu_baseline:
                out["cpu_baseline"] = cpu_baseline(cfg, nodes, pods, a.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
