"""Deterministic synthetic clusters for the benchmark configurations.

Columns are generated directly (vectorised numpy, PCG64 seeded with 0x6B6F6F7264 + config index)
with the distributions of §8d; they are what the host decode would produce for such a cluster.
"""
from __future__ import annotations

import numpy as np

from . import abi
from .config import SchedulerConfig, bench_profile
from .decode import amplify

SEED = 0x6B6F6F7264
GI = 1 << 30
MI = 1 << 20
DEFAULT_EST_MILLI_CPU = 250
DEFAULT_EST_MEMORY = 200 * MI
NZ_CPU = 100
NZ_MEM = 200 * MI


def _rng(config: int, extra: int = 0):
    return np.random.Generator(np.random.PCG64(SEED + config + 1000 * extra))


def _go_round_half_away(x: np.ndarray) -> np.ndarray:
    return np.where(x >= 0, np.floor(x + 0.5), np.ceil(x - 0.5))


def _estimate(q: np.ndarray, lim: np.ndarray, factor: int, default: int) -> np.ndarray:
    """estimatedUsedByResource on integer quantities (milli-cpu or bytes)."""
    est = _go_round_half_away(q.astype(np.float64) * float(factor) / 100.0).astype(np.int64)
    est = np.where((lim > 0) & (est > lim), lim, est)
    return np.where(q == 0, default, est)


def nodes(n: int, config: int = 1, numa: bool = False, rng=None) -> abi.Table:
    r = rng or _rng(config)
    t = abi.empty_nodes(n)
    cores = r.choice([32, 64, 96], n)
    mem_gi = r.choice([128, 256, 512], n)
    amp = np.zeros(n, bool)
    if numa:
        amp = r.random(n) < 0.10
    ratio = np.where(amp, 1.5, 1.0)
    alloc_cpu = np.array([amplify(int(c) * 1000, float(q)) for c, q in zip(cores, ratio)], np.int64)
    t["alloc_cpu"] = alloc_cpu
    t["alloc_mem"] = mem_gi.astype(np.int64) * GI
    t["alloc_eph"] = r.choice([100, 200, 400], n).astype(np.int64) * GI
    t["alloc_pods"] = np.full(n, 110, np.int64)
    frac = r.random(n) * 0.7
    t["req_cpu"] = (alloc_cpu * frac).astype(np.int64)
    t["req_mem"] = (t["alloc_mem"] * (r.random(n) * 0.7)).astype(np.int64)
    t["req_eph"] = (t["alloc_eph"] * (r.random(n) * 0.3)).astype(np.int64)
    t["num_pods"] = r.integers(0, 80, n).astype(np.int64)
    t["nz_cpu"] = t["req_cpu"] + r.integers(0, 5, n) * NZ_CPU
    t["nz_mem"] = t["req_mem"] + r.integers(0, 5, n) * NZ_MEM
    for k, base in enumerate((alloc_cpu, t["alloc_mem"])):
        sc = (base * (r.random(n) * 0.4)).astype(np.int64)
        t[f"sc_alloc{k}"] = sc
        t[f"sc_req{k}"] = (sc * (r.random(n) * 0.7)).astype(np.int64)
    # LoadAware: EstimateNode allocatable = allocatable; NodeMetric usage U(0, 0.8); 5% nodes without a
    # NodeMetric, 2% expired; delta of recently assigned pods up to 5%.
    has_metric = r.random(n) >= 0.05
    expired = has_metric & (r.random(n) < 0.02)
    flags = np.where(has_metric, abi.KG_LA_HAS_METRIC, 0) | np.where(expired, abi.KG_LA_EXPIRED, 0)
    t["la_flags"] = flags.astype(np.uint32)
    for k, a in enumerate((alloc_cpu, t["alloc_mem"])):
        t[f"la_alloc{k}"] = a
        t[f"la_thr_usage{k}"] = np.full(n, (65, 95)[k], np.int64)
        usage = (a * (r.random(n) * 0.8)).astype(np.int64)
        delta = (a * (r.random(n) * 0.05)).astype(np.int64)
        prod_usage = (usage * r.random(n)).astype(np.int64)
        prod_delta = (delta * r.random(n)).astype(np.int64)
        base = np.where(has_metric, usage + delta, 0)
        pbase = np.where(has_metric, prod_usage + prod_delta, 0)
        t[f"la_fbase_np{k}"] = base
        t[f"la_sbase_np{k}"] = base
        t[f"la_fbase_prod{k}"] = pbase
        t[f"la_sbase_prod{k}"] = pbase
    t["cpu_amp_ratio"] = ratio
    if numa:
        single = r.random(n) < 0.20
        t["numa_policy"] = np.where(single, abi.KG_NUMA_SINGLE_NODE, abi.KG_NUMA_NONE).astype(np.uint32)
        t["numa_zones"] = np.full(n, 2, np.uint32)
        for z in range(2):
            zc = alloc_cpu // 2
            zm = t["alloc_mem"] // 2
            t[f"zone_cpu{z}"] = zc
            t[f"zone_mem{z}"] = zm
            t[f"zone_cpu_used{z}"] = (zc * (r.random(n) * 0.7)).astype(np.int64)
            t[f"zone_mem_used{z}"] = (zm * (r.random(n) * 0.7)).astype(np.int64)
        # half of the amplified nodes carry cpuset-allocated cpus (whole cores)
        cs = np.where(amp & (r.random(n) < 0.5), (t["req_cpu"] // 2000) * 1000, 0)
        t["cpuset_alloc_milli"] = cs.astype(np.int64)
    return t


def pods(p: int, config: int = 1, scale: float = 1.0, rng=None, la_factors=(85, 70)) -> abi.Table:
    r = rng or _rng(config, 1)
    t = abi.empty_pods(p)
    cpu = (r.choice([100, 250, 500, 1000, 2000, 4000], p) * scale).astype(np.int64)
    mem = (r.choice([128 * MI, 512 * MI, GI, 2 * GI, 4 * GI, 8 * GI], p) * scale).astype(np.int64)
    two = r.random(p) < 0.5
    lim_cpu = np.where(two, 2 * cpu, cpu)
    lim_mem = np.where(two, 2 * mem, mem)
    prod = r.random(p) < 0.70
    empty = r.random(p) < 0.05
    prod &= ~empty
    batch = ~prod & ~empty
    z = np.zeros(p, np.int64)
    t["req_cpu"] = np.where(prod, cpu, z)
    t["req_mem"] = np.where(prod, mem, z)
    t["sc_req0"] = np.where(batch, cpu, z)  # kubernetes.io/batch-cpu (milli-core count)
    t["sc_req1"] = np.where(batch, mem, z)  # kubernetes.io/batch-memory
    t["nz_cpu"] = np.where(prod, cpu, NZ_CPU)
    t["nz_mem"] = np.where(prod, mem, NZ_MEM)
    # EstimatePod: prod pods estimate cpu/memory, batch pods batch-cpu/batch-memory, empty pods defaults
    q_cpu = np.where(empty, 0, np.maximum(lim_cpu, cpu))
    q_mem = np.where(empty, 0, np.maximum(lim_mem, mem))
    t["la_est0"] = _estimate(q_cpu, np.where(empty, 0, lim_cpu), la_factors[0], DEFAULT_EST_MILLI_CPU)
    t["la_est1"] = _estimate(q_mem, np.where(empty, 0, lim_mem), la_factors[1], DEFAULT_EST_MEMORY)
    flags = np.where(prod, abi.KG_POD_PROD | abi.KG_POD_HAS_CPU | abi.KG_POD_HAS_MEM, 0)
    flags |= np.where(empty, abi.KG_POD_NUMA_SKIP, 0)
    t["flags"] = flags.astype(np.uint32)
    return t


def cluster(config: int):
    """(SchedulerConfig, nodes, pods) of a BASELINE configuration (1: 1k x 500, 2: 10k x 10k,
    3: 10k nodes x 50k replay pods, 4: 100k nodes x 10k pods)."""
    if config == 1:
        return bench_profile(numa=False), nodes(1000, 1), pods(500, 1)
    if config == 2:
        return bench_profile(numa=True), nodes(10_000, 2, numa=True), pods(10_000, 2)
    if config == 3:
        # pods scaled so that the 50k placements saturate the cluster: LoadAware usage thresholds bind first
        # (cpu requested levels off near 51%), the last ~1.3k pods are unschedulable
        return bench_profile(numa=True), nodes(10_000, 3, numa=True), pods(50_000, 3, scale=2.5)
    if config == 4:
        return bench_profile(numa=True), nodes(100_000, 4, numa=True), pods(10_000, 4)
    raise ValueError(config)


def small(n_nodes: int, n_pods: int, seed: int = 0, numa: bool = True, scale: float = 1.0) -> tuple:
    """Small synthetic cluster for parity tests."""
    cfg: SchedulerConfig = bench_profile(numa=numa)
    return cfg, nodes(n_nodes, 100 + seed, numa=numa), pods(n_pods, 100 + seed, scale=scale)
