"""Benchmark of the MI355X Filter/Score evaluation engine (BASELINE.json metric).

One step = one pass of the hot path over one batch: Filter + Score of every pending pod against
every node of the snapshot and the selectHost of each pod.

  N = 1 (default): config 2 of BASELINE.md — 10k nodes x 10k pods, NodeResourcesFit + LoadAware +
          NodeNUMAResource, on one GPU.
  N > 1 (default): config 4 — one 100k-node cluster split contiguously over the N GPUs (strong
          scaling). Each rank evaluates its shard, the per-pod top-k keys (k = 3, upstream
          numberOfHighestScoredNodesToReport) are all-gathered over RCCL and every rank runs the same
          global selectHost (kg_shard_select).

`python bench.py --gpus N` with no launcher environment starts N rank processes itself (RANK,
WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT set per child) before anything touches the GPU; under
`torch.distributed.run` each process is one rank. Prints ONE JSON line on rank 0 (value = evals/s over
all ranks, inputs resident in HBM).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK = 8.0e12  # MI355X HBM3E peak B/s (MI355X_MICROARCH.md, chip-level parameters)
# VALU issue: 256 CUs x 4 SIMDs at 2.4 GHz. A wave64 instruction holds its SIMD for 2 cycles when it is
# f32 arithmetic and 4 cycles when it is f64, 64-bit or 32-bit integer, a compare, a conversion or a
# v_cndmask (chip-wide measurement, tools/ubench_valu.hip -> profiles/r2/ubench_valu.txt); the select
# kernels' loops are ~95 % of the latter, so the peak is priced per kernel from its ISA mix (roofline).
SIMD_CYCLES = 256 * 4 * 2.4e9
VALU_PEAK = SIMD_CYCLES / 2  # the all-f32 ceiling, for reference
# SALU issue peak: one scalar instruction per cycle per CU.
SALU_PEAK = 256 * 2.4e9
# Algorithmic bytes per (pod, node) eval, SURVEY.md §8d (scan model, node row read once per eval):
# NodeResourcesFit 120 B + LoadAware 52 B + NodeNUMAResource 4 B + 0.2 x 64 B zone table = 188.8 B.
B_EVAL = {1: 172.0, 2: 188.8, 4: 188.8, 6: 188.8,
          # config 5: + DeviceShare 384 B x 30% GPU pods + Reservation 4 B node flag (308 B)
          5: 308.0}
METRIC = "Filter+Score pod-node evals/sec"
PLUGINS = {1: "+LoadAware", 2: "+LoadAware+NodeNUMAResource", 4: "+LoadAware+NodeNUMAResource",
           6: "+LoadAware+NodeNUMAResource; mixed: 20% SingleNUMANode, 10% Restricted, 10% BestEffort, 5% CPU-bind-"
              "policy nodes, 5% LSR cpuset pods",
           5: "+LoadAware+NodeNUMAResource+DeviceShare+Reservation+ElasticQuota"}
KERNEL_SOURCES = ("kg_eval.h", "kg_ext.h", "kg_ext_wave.h", "kg_kernels.h", "kg_layout.h", "kg_kernels.hip", "kg_ext.hip")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=None, choices=[1, 2, 4, 5, 6],
                    help="2: 10k nodes x 10k pods (default at 1 GPU); 4: 100k nodes split over the GPUs x 10k "
                         "pods (strong scaling, default at N > 1); 5: config 4 + DeviceShare / Reservation / "
                         "ElasticQuota; 1: the 1k x 500 CPU-harness case; 6: config 2 on a mixed cluster "
                         "(Restricted / BestEffort / CPU-bind-policy nodes, LSR pods: synth.mixed)")
    ap.add_argument("--k", type=int, default=None, help="per-pod top-k (default 3 for config 4, else 1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-replay", action="store_true")
    ap.add_argument("--no-cycle", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    return ap.parse_args()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """Start n rank processes of this script (one per GPU) and wait for them. The parent never
    initialises the GPU: it only spawns children with the rendezvous environment."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc = 0
    for p in procs:
        code = p.wait()
        rc = rc or code
    return rc


def kernel_source_hash() -> str:
    h = hashlib.sha256()
    for name in KERNEL_SOURCES:
        with open(os.path.join(ROOT, "koordinator_amd", "csrc", name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def load_pmc(name: str):
    """A committed rocprofv3 PMC summary (tools/pmc_summary.py) if it was taken on these kernel sources."""
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            pmc = json.load(f)
    except Exception:
        return None
    if pmc.get("kernel_source_hash") != kernel_source_hash():
        return None  # stale: taken on other kernel code
    return pmc


def roofline(pmc, kernel_s, evals_per_launch, b_eval, kernel_name):
    """The dominant kernel's ceiling. The select kernels are bound by instruction issue (VALU, with the
    CU's single scalar unit as co-limit), not by HBM: pod tiling serves each node record to 64 pods, so
    the HBM traffic is a few MB per launch. The primary figure is therefore the VALU issue fraction
    (instructions per launch from the committed PMC pass on these kernel sources / the live average
    kernel time); the measured HBM bytes and the SURVEY §8d scan model are reported next to it."""
    out = {"bound": "valu-issue", "achieved": None, "peak": VALU_PEAK / 1e12, "unit": "T wave-inst/s", "frac": None,
           "traffic": None, "kernel": kernel_name, "kernel_avg_ms": kernel_s * 1e3 if kernel_s else None,
           "evals_per_launch": evals_per_launch}
    scan = evals_per_launch * b_eval / kernel_s if kernel_s else None
    out["scan_model"] = {"bytes_per_eval": b_eval, "effective_GBps": scan / 1e9 if scan else None,
                         "note": "SURVEY §8d scan model (node row read once per eval); pod tiling reads a row "
                                 "once per 64 pods, so this is not an HBM utilisation and may exceed 8 TB/s"}
    if not pmc or not kernel_s:
        out["note"] = ("no PMC summary for these kernel sources and this configuration (N = 1, configs 2, 4, 5, 6): "
                       "issue / HBM fractions not available")
        return out
    valu = pmc.get("valu_insts_per_launch")
    salu = pmc.get("salu_insts_per_launch")
    hbm = pmc.get("hbm_bytes_per_launch")
    if valu:
        # price each kernel's VALU count with its loop's issue cost (profiles/valu_mix.json: 2 cycles per f32
        # wave64 instruction, 4 for f64 / integer / compare / convert, measured by tools/ubench_valu.hip)
        mix = load_pmc("valu_mix.json")
        cyc = None
        if mix:
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            from valu_mix import canon_demangled

            cyc = 0.0
            for name, k in (pmc.get("kernels") or {}).items():
                v = (k.get("counters") or {}).get("SQ_INSTS_VALU", 0.0)
                m = mix["kernels"].get(canon_demangled(name) or "")
                cyc += v * (m["cyc_per_valu"] if m else 4.0)
        cpi = cyc / valu if cyc else 4.0
        peak = SIMD_CYCLES / cpi
        out["achieved"] = valu / kernel_s / 1e12
        out["peak"] = peak / 1e12
        out["frac"] = valu / kernel_s / peak
        out["issue_model"] = {"cycles_per_valu": cpi, "simd_cycles_per_s": SIMD_CYCLES,
                              "source": "profiles/valu_mix.json (ISA mix) x profiles/r2/ubench_valu.txt (costs)"
                                        if mix else "4 cycles per VALU (no ISA mix for these sources)",
                              "frac_at_2_cycles": valu / kernel_s / (SIMD_CYCLES / 2)}
    if salu:
        out["salu"] = {"achieved": salu / kernel_s / 1e12, "peak": SALU_PEAK / 1e12, "unit": "T inst/s",
                       "frac": salu / kernel_s / SALU_PEAK}
    if hbm:
        out["traffic"] = hbm
        out["hbm"] = {"achieved": hbm / kernel_s / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                      "frac": hbm / kernel_s / HBM_PEAK,
                      "note": "rocprofv3 FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE per launch"}
    out["pmc"] = pmc.get("source")
    return out


def cpu_baseline(cfg, nodes, pods, target_s):
    """Oracle (C restatement, upstream-shaped 16-worker parallelizer) on a bounded pod sample."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib  # test infrastructure: the CPU baseline leg only
    from koordinator_amd import abi

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
    return {"value": n * n_nodes / dt, "unit": "evals/s", "cores": os.cpu_count(), "workers": workers,
            "kind": "port",
            "sample": f"{n} pods x {n_nodes} nodes ({n * n_nodes} evals) in {dt:.2f} s; oracle/kg_oracle.c "
                      f"kgo_select_parallel: per pod parallel Filter then parallel Score over nodes on {workers} "
                      f"worker threads (upstream parallelism 16, chunked like pkg/util/parallelize/"
                      f"parallelism.go:29-49) on a host with {os.cpu_count()} logical CPUs"}


def cpu_baseline_ext(kc, nodes, pods, quotas, rsv, target_s, workers: int = 16):
    """Config 5: the oracle's restatement on a bounded pod sample, pods split over 16 worker threads (each pod's
    Filter / Score / NormalizeScore / selectHost is independent of the others; the C calls release the GIL)."""
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib  # test infrastructure: the CPU baseline leg only
    from koordinator_amd import abi

    n_nodes = abi.table_len(nodes)

    def run(n):
        parts = [ix for ix in np.array_split(np.arange(n), min(n, 4 * workers)) if len(ix)]
        with ThreadPoolExecutor(workers) as ex:
            list(ex.map(lambda ix: oracle_lib.ext_select(kc, nodes, abi.take(pods, ix), 1, 0, quotas, rsv), parts))

    probe = workers
    t0 = time.perf_counter()
    run(probe)
    dt = max(time.perf_counter() - t0, 1e-6)
    n = int(min(abi.table_len(pods), max(probe, target_s / (dt / probe))))
    t0 = time.perf_counter()
    run(n)
    dt = time.perf_counter() - t0
    return {"value": n * n_nodes / dt, "unit": "evals/s", "cores": os.cpu_count(), "workers": workers, "kind": "port",
            "sample": f"{n} pods x {n_nodes} nodes ({n * n_nodes} evals) in {dt:.2f} s; oracle/kg_oracle.c "
                      f"kgo_ext_select (all six plugins, NormalizeScore, selectHost), pods split over {workers} worker "
                      f"threads on a host with {os.cpu_count()} logical CPUs"}


def replay_rate(ctx, cfg, with_cpu, cpu_s, config=3):
    """Pods placed one by one with device-resident Assume: config 3 (50k pods on 10k nodes) or, for the
    BASELINE metric's 100k-node half, the config-4 cluster (10k pods on 100k nodes, one GPU)."""
    import numpy as np

    from koordinator_amd import abi, engine, synth

    _, nodes, pods = synth.cluster(config)
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
           "workload": (f"config{config}: {snap.n // 1000}k nodes x {batch.n // 1000}k pods, one pod per cycle, "
                        "Assume on device")}
    if with_cpu:
        # CPU baseline: every cycle's Filter / Score on the upstream 16-worker parallelizer, then the
        # Reserve, for the first pods of the same sequence (bounded sample)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib  # test infrastructure: the CPU baseline leg only

        probe = 50 if config == 3 else 8
        st = oracle_lib.OracleState(kc, nodes)
        t0 = time.perf_counter()
        st.replay_parallel(abi.take(pods, np.arange(probe)), 16)
        per = max(time.perf_counter() - t0, 1e-6) / probe
        n = int(min(batch.n, max(probe * 2, cpu_s / per)))
        st = oracle_lib.OracleState(kc, nodes)
        t0 = time.perf_counter()
        want, _ = st.replay_parallel(abi.take(pods, np.arange(n)), 16)
        cdt = time.perf_counter() - t0
        assert np.array_equal(want, node[:n])  # same placements as the device replay
        out["cpu_baseline"] = {"value": n / cdt, "unit": "pods/s", "cores": os.cpu_count(), "workers": 16,
                               "kind": "port",
                               "sample": f"first {n} pods of the config-{config} sequence in {cdt:.2f} s; oracle/kg_oracle.c "
                                         f"kgo_replay_parallel: each cycle's Filter then Score over all nodes on 16 "
                                         f"worker threads (parallelism.go:29-49), then the Reserve"}
    snap.close()
    batch.close()
    return out


def replay5_rate(ctx, with_cpu, cpu_s):
    """Config 5 one pod per cycle: the config-5 cluster of the select (100k nodes x 10k pods, every plugin, reservations
    holding GPUs with their DeviceShare restore inputs), kg_replay running every plugin's Reserve on the device between
    pods: NodeInfo, LoadAware, NUMA, GPU minors (and the GPU-holding reservations' restore tables), ElasticQuota and
    Reservation.Reserve."""
    import numpy as np

    from koordinator_amd import abi, engine, synth

    cfg, nodes, pods, quotas, rsv = synth.config5()
    kc = cfg.kg_config()
    snap = engine.Snapshot(ctx, kc, nodes)
    snap.upload_quotas(quotas)
    snap.upload_reservations(rsv)
    small = engine.PodBatch(ctx, abi.take(pods, np.arange(256)))
    engine.replay(snap, small)  # warm-up (graph instantiate, code load)
    snap.upload(nodes)
    snap.upload_quotas(quotas)
    snap.upload_reservations(rsv)
    batch = engine.PodBatch(ctx, pods)
    t0 = time.perf_counter()
    node, _ = engine.replay(snap, batch)
    dt = time.perf_counter() - t0
    placed = int((node >= 0).sum())
    out = {"pods_placed_per_s": batch.n / dt, "pods": batch.n, "placed": placed, "seconds": round(dt, 4),
           "workload": (f"config5: {snap.n // 1000}k nodes x {batch.n // 1000}k pods, one pod per cycle, Reserve of "
                        "every plugin (NodeInfo, LoadAware, NUMA, GPU minors, ElasticQuota, Reservation) on device; "
                        "reservations holding GPUs followed through their restore tables")}
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib  # test infrastructure: the CPU baseline leg only

        workers = 16  # upstream parallelism 16 (pkg/util/parallelize/parallelism.go:29-49)
        probe = 8
        t0 = time.perf_counter()
        oracle_lib.OracleState(kc, nodes).ext_replay(abi.take(pods, np.arange(probe)), quotas, rsv=rsv, workers=workers)
        per = max(time.perf_counter() - t0, 1e-6) / probe
        n = int(min(batch.n, max(probe * 2, cpu_s / 2 / per)))
        t0 = time.perf_counter()
        want = oracle_lib.OracleState(kc, nodes).ext_replay(abi.take(pods, np.arange(n)), quotas, rsv=rsv,
                                                            workers=workers)[0]
        cdt = time.perf_counter() - t0
        assert np.array_equal(want, node[:n])  # same placements as the device replay
        out["cpu_baseline"] = {"value": n / cdt, "unit": "pods/s", "cores": os.cpu_count(), "workers": workers,
                               "kind": "port",
                               "sample": f"first {n} pods of the sequence in {cdt:.2f} s; oracle/kg_oracle.c "
                                         f"kgo_ext_replay_parallel: each cycle's Filter / Score over the nodes on "
                                         f"{workers} worker threads (parallelism.go:29-49), then the Reserve"}
    snap.close()
    batch.close()
    small.close()
    return out


def cycle_rate(ctx, snap, pods_table, steps):
    """One end-to-end PreFilter cycle as the plugin pays it: pod batch upload (host columns -> HBM), the
    select over every node, and the download of the per-pod keys."""
    from koordinator_amd import engine

    batch = engine.PodBatch(ctx, pods_table)
    engine.eval_select(snap, batch, 1)  # warm-up
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        batch.upload(pods_table)
        engine.eval_select(snap, batch, 1)  # includes kg_result_keys (device -> host)
    dt = (time.perf_counter() - t0) / steps
    n = batch.n
    batch.close()
    return {"ms_per_cycle": dt * 1e3, "evals_per_s": n * snap.n / dt, "pods": n, "nodes": snap.n,
            "note": "kg_pods_upload (host columns copied into pinned staging, one async copy) + kg_eval_select + kg_result_keys per cycle"}


def main():
    a = parse()
    if a.gpus > 1 and "RANK" not in os.environ:
        sys.exit(launch_ranks(a.gpus))

    import numpy as np

    from koordinator_amd import abi, engine, synth

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    config = a.config if a.config is not None else (2 if world == 1 else 4)
    k = a.k if a.k is not None else (3 if config == 4 else 1)
    dist = None
    if world > 1:
        import torch.distributed as dist  # bootstrap + host barriers only (data path is RCCL in the library)

        dist.init_process_group("gloo")
    ctx = engine.Context(local)
    quotas = rsv = None
    if config == 5:
        cfg, nodes, pods, quotas, rsv = synth.config5()
    elif config == 6:
        cfg, nodes, pods = synth.mixed()
    else:
        cfg, nodes, pods = synth.cluster(config)
    all_nodes = nodes
    if config in (4, 5):
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
            nodes = synth.mixed(n_local, 1, seed=6 + 10 * rank)[1] if config == 6 else \
                synth.nodes(n_local, config + 10 * rank, numa=(config == 2))
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
            engine.shard_select(snap, batch, k, download=False)
        else:
            engine.eval_select_async(snap, batch, k)

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
    # the result of the last step is sane (descending keys pointing into the cluster)
    keys = engine.result_keys(batch, k)
    idx = abi.key_node(keys)
    assert np.all(idx[keys != 0] < n_total)
    assert np.all(keys[:, :-1] >= keys[:, 1:])

    evals = float(n_pods) * n_total * a.steps
    value = evals / elapsed
    avg_kernel_s = (kern_ms / 1e3) / max(launches, 1) if launches else None
    # the committed PMC passes are per launch of one configuration (profiles/run_profile.sh: 2, 4 and 5)
    pmc = load_pmc({2: "select_pmc.json", 4: "select4_pmc.json", 5: "ext_pmc.json", 6: "select6_pmc.json"}[config]) \
        if world == 1 and config in (2, 4, 5, 6) else None
    fused = k == 1 and os.environ.get("KG_SELECT_UNFUSED", "0") in ("", "0")
    base = "k_big_sel + k_select1 (fused top-1)" if fused else "k_select + k_big_sel + k_merge"
    if config == 6:
        base += " + k_int_seed / k_int_filter / k_int_pairs (pruned LSR lanes)"
    kname = base if config != 5 else (f"config-5 step: k_dev_sum + k_rdev_codes + k_ext_stats_sp/views + k_ext_select "
                                      f"(one pass + re-run) + k_ext_select_sp + plain pods' {base} (one bracket)")
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "evals/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if config in (4, 5) else "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (PCG64 seed 0x6B6F6F7264, SURVEY.md §8d distributions)",
        "config": {"workload": f"config{config}: {n_total} nodes ({n_local}/GPU) x {n_pods} pods, "
                               f"Filter+Score+selectHost top-{k} (NodeResourcesFit{PLUGINS[config]})",
                   "nodes_per_gpu": n_local, "nodes_total": n_total, "pods": n_pods, "k": k,
                   "parallelism": f"node-shard x{world}" + (f" + RCCL all-gather of per-pod top-{k} keys" if world > 1 else "")},
        "roofline": roofline(pmc, avg_kernel_s, n_pods * n_local, B_EVAL[config], kname),
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1:
        if config != 5 and not a.no_cycle:
            out["cycle"] = cycle_rate(ctx, snap, pods, 10)
        if config == 5:
            if not a.no_cpu_baseline:
                out["cpu_baseline"] = cpu_baseline_ext(kc, nodes, pods, quotas, rsv, a.cpu_seconds)
            if not a.no_replay:
                snap.close()
                batch.close()
                out["replay"] = replay5_rate(ctx, not a.no_cpu_baseline, a.cpu_seconds)
        else:
            if not a.no_replay and config in (1, 2):
                out["replay"] = replay_rate(ctx, cfg, not a.no_cpu_baseline, a.cpu_seconds)
                out["replay_100k"] = replay_rate(ctx, cfg, not a.no_cpu_baseline, a.cpu_seconds / 2, config=4)
            if not a.no_cpu_baseline:
                out["cpu_baseline"] = cpu_baseline(cfg, all_nodes, pods, a.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
