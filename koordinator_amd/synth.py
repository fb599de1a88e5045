"""Deterministic synthetic clusters for the benchmark configurations.

Columns are generated directly (vectorised numpy, PCG64 seeded with 0x6B6F6F7264 + config index)
with the distributions of §8d; they are what the host decode would produce for such a cluster.
"""
from __future__ import annotations

import numpy as np

from . import abi
from .config import GPU_CORE, GPU_MEMORY, GPU_MEMORY_RATIO, SchedulerConfig, bench_profile, config5_profile
from . import decode
from .decode import amplify, gpu_requirements, quota_keys, reservation_gpu_raw, reservation_restore

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


GPU_MEM_PER_MINOR = 192 * GI
N_RSV_CLASSES = 8


def cluster5(n_nodes: int, n_pods: int, seed_config: int = 5, n_quotas: int = 100, rsv_frac: float = 0.05,
             numa: str = "none", usage: str = "mixed", rsv_gpu: bool = True, raw: bool = False):
    """Config 5: configs 1-2's plugins plus DeviceShare (8 GPU minors per node: gpu-core
    100, gpu-memory-ratio 100, gpu-memory 192Gi; minors 40% idle, 30% fully used, 30% partially used),
    Reservation (5% of nodes hold 1-4 reservations of one of 8 owner classes, a third of them reserving
    1-2 whole GPUs of the node's idle minors, their assigned pods using part of them; 20% of all pods, GPU
    pods included, match one class, a quarter of them with a required reservation affinity) and
    ElasticQuota (100 flat quotas, every pod in one; 10% non-preemptible pods). 30% of the pods request
    GPUs: 60% whole GPUs (1/2/4/8), 40% shared (gpu-core 50 + gpu-memory-ratio 50, or gpu-core 50 +
    gpu-memory 24Gi). NUMA policy None on every node (the NUMA zone restore of reservations and the
    DeviceShare NUMA hints stay on the host path).

    usage: "mixed" (above) or "u01": each minor's used fraction U(0, 1) (gpu-core / ratio
    int(100 u), gpu-memory the same percentage), so whole-GPU pods fit only the rare idle minors.
    numa: "none" (above), "single" (the 20% SingleNUMANode nodes of configs 2-3 kept), or "mix" (own random
    stream: None 40%, SingleNUMANode / Restricted / BestEffort 20% each, 10% of the pods with a NUMA policy of
    their own, 5% of the GPU nodes with a GPU whose Topology.NodeID is -1): GPU pods on NUMA-policy nodes join
    DeviceShare's NUMA hints (deviceshare/topology_hint.go) to the topology manager.

    rsv_gpu=False: no reservation holds GPUs (the replay follows reservation Reserves on the device only then).

    Returns (cfg, nodes, pods, quotas, reservations): nodes already restored to the view of pods that
    match no reservation (decode.reservation_restore), reservations = abi.Reservations; raw=True appends the
    true NodeInfo table and the reservation dicts the restore was computed from."""
    cfg = config5_profile()
    r = _rng(seed_config)
    t = nodes(n_nodes, seed_config, numa=True, rng=r)
    n = n_nodes
    if numa == "none":
        t["numa_policy"][:] = abi.KG_NUMA_NONE
    # DeviceShare minors
    t["dev_minors"] = np.full(n, abi.KG_DEV_MINORS, np.int32)
    tot = np.zeros((n, abi.KG_DEV_R, abi.KG_DEV_MINORS), np.int64)
    tot[:, abi.KG_DEV_CORE, :] = 100
    tot[:, abi.KG_DEV_RATIO, :] = 100
    tot[:, abi.KG_DEV_MEM, :] = GPU_MEM_PER_MINOR
    state = r.random((n, abi.KG_DEV_MINORS))
    if usage == "u01":
        used_pct = (state * 100).astype(np.int64)
    else:
        used_pct = np.where(state < 0.4, 0, np.where(state < 0.7, 100, (r.random((n, abi.KG_DEV_MINORS)) * 20).astype(np.int64) * 5))
    free = tot.copy()
    free[:, abi.KG_DEV_CORE, :] -= used_pct
    free[:, abi.KG_DEV_RATIO, :] -= used_pct
    free[:, abi.KG_DEV_MEM, :] -= used_pct * GPU_MEM_PER_MINOR // 100
    used = tot - free
    # Reservations on 5% of the nodes (counted in the true NodeInfo: reserve pod + assigned pods)
    resv = []
    holders = np.nonzero(r.random(n) < rsv_frac)[0]
    for i in holders:
        idle = [m for m in range(abi.KG_DEV_MINORS) if used_pct[i, m] == 0]
        for _ in range(int(r.integers(1, 5))):
            cpu = int(r.choice([2000, 4000, 8000]))
            mem = int(r.choice([4, 8, 16])) * GI
            alloc = [cpu, mem, 0, 0, 0]
            ap = int(r.integers(1, 3)) if r.random() < 0.5 else 0
            allocated = None
            if ap:
                f = float(r.choice([0.25, 0.5, 0.75]))
                allocated = [int(cpu * f), int(mem * f), 0, 0, 0]
            pol = r.random()
            policy = abi.KG_RSV_DEFAULT if pol < 0.6 else (abi.KG_RSV_ALIGNED if pol < 0.8 else abi.KG_RSV_RESTRICTED)
            order = int(r.integers(1, 11)) if r.random() < 0.3 else 0
            # GPUs: the reserve pod holds whole idle minors; assigned pods use part of them (both counted
            # in the node's used, as nodeDevice.deviceUsed counts every allocation)
            dev_alloc = dev_allocated = None
            if idle and r.random() < 1 / 3 and rsv_gpu:
                k = min(len(idle), int(r.integers(1, 3)))
                ms = [idle.pop(int(r.integers(0, len(idle)))) for _ in range(k)]
                dev_alloc = np.zeros((abi.KG_DEV_R, abi.KG_DEV_MINORS), np.int64)
                dev_alloc[:, ms] = tot[i][:, ms]
                used[i] += dev_alloc
                if ap:
                    part = int(r.choice([25, 50, 100]))
                    dev_allocated = np.zeros_like(dev_alloc)
                    m0 = ms[0]
                    dev_allocated[abi.KG_DEV_CORE, m0] = part
                    dev_allocated[abi.KG_DEV_RATIO, m0] = part
                    dev_allocated[abi.KG_DEV_MEM, m0] = part * GPU_MEM_PER_MINOR // 100
                    used[i] += dev_allocated
            resv.append(dict(node=int(i), cls=int(r.integers(0, N_RSV_CLASSES)), allocatable=alloc,
                             allocated=allocated, reserved=None, allocated_pods=ap, policy=policy, order=order,
                             allocate_once=ap == 0, max_pods=-1, dev_alloc=dev_alloc, dev_allocated=dev_allocated))
            t["req_cpu"][i] += cpu + (allocated[0] if allocated else 0)
            t["req_mem"][i] += mem + (allocated[1] if allocated else 0)
            t["nz_cpu"][i] += cpu + (allocated[0] if allocated else 0)
            t["nz_mem"][i] += mem + (allocated[1] if allocated else 0)
            t["num_pods"][i] += 1 + ap
    t["dev_total"], t["dev_free"], t["dev_used"] = tot, np.maximum(tot - used, 0), used
    true_t = {k: np.array(v, copy=True) for k, v in t.items()}
    gpu_raw = reservation_gpu_raw(t, resv)
    t, views, infos, devs = reservation_restore(t, resv)
    # Pods
    pr = _rng(seed_config, 1)
    p = pods(n_pods, seed_config, rng=pr)
    gpu = pr.random(n_pods) < 0.30
    whole = pr.random(n_pods) < 0.60
    count = pr.choice([1, 2, 4, 8], n_pods, p=[0.5, 0.25, 0.15, 0.10])
    by_mem = pr.random(n_pods) < 0.25
    for j in np.nonzero(gpu)[0]:
        if whole[j]:
            req = {GPU_CORE: 100 * int(count[j]), GPU_MEMORY_RATIO: 100 * int(count[j])}
        elif by_mem[j]:
            req = {GPU_CORE: 50, GPU_MEMORY: 24 * GI}
        else:
            req = {GPU_CORE: 50, GPU_MEMORY_RATIO: 50}
        vec, keys, cnt, _ = gpu_requirements(req)
        p["dev_req"][j] = vec
        p["dev_keys"][j] = keys
        p["dev_count"][j] = cnt
    # reservation owner classes
    cls_on = pr.random(n_pods) < 0.20
    p["rsv_class"] = np.where(cls_on, pr.integers(0, N_RSV_CLASSES, n_pods), -1).astype(np.int32)
    p["flags"] |= np.where(cls_on & (pr.random(n_pods) < 0.25), abi.KG_POD_RSV_REQUIRED, 0).astype(np.uint32)
    # ElasticQuota: flat quotas with Max over cpu + memory (10%: also the batch resources)
    q = abi.empty_quotas(n_quotas)
    maxk = np.where(pr.random(n_quotas) < 0.10, 0b1111, 0b0011).astype(np.uint32)
    lim = np.stack([pr.integers(50, 500, n_quotas) * 1000, pr.integers(100, 2000, n_quotas) * GI,
                    pr.integers(50, 500, n_quotas) * 1000, pr.integers(100, 2000, n_quotas) * GI], 1).astype(np.int64)
    used = (lim * pr.uniform(0.5, 1.0, (n_quotas, 1))).astype(np.int64)
    q["used_limit"], q["used"] = lim, used
    q["limit_keys"], q["used_keys"] = maxk, maxk
    q["min"] = (lim * 0.6).astype(np.int64)
    q["np_used"] = (q["min"] * pr.uniform(0.0, 1.1, (n_quotas, 1))).astype(np.int64)
    q["min_keys"], q["np_used_keys"] = maxk, maxk
    p["quota"] = pr.integers(0, n_quotas, n_pods).astype(np.int32)
    p["flags"] |= np.where(pr.random(n_pods) < 0.10, abi.KG_POD_NON_PREEMPTIBLE, 0).astype(np.uint32)
    p["quota_keys"] = quota_keys(p, maxk)
    gpu_topology5(t, p, seed_config, any_numa=numa == "mix")
    if numa == "mix":
        rm = _rng(seed_config, 3)
        t["numa_policy"] = rm.choice([abi.KG_NUMA_NONE, abi.KG_NUMA_SINGLE_NODE, abi.KG_NUMA_RESTRICTED,
                                      abi.KG_NUMA_BEST_EFFORT], n, p=[0.4, 0.2, 0.2, 0.2]).astype(np.uint32)
        own = rm.random(n_pods) < 0.10
        p["numa_policy"] = np.where(own, rm.choice([abi.KG_NUMA_SINGLE_NODE, abi.KG_NUMA_RESTRICTED], n_pods),
                                    abi.KG_NUMA_NONE).astype(np.uint32)
    if raw:
        for k in set(t) - set(true_t):  # columns set after the restore (GPU topology) hold for the true table too
            true_t[k] = np.array(t[k], copy=True)
        return cfg, t, p, q, abi.Reservations(views, infos, devs, gpu_raw), true_t, resv
    return cfg, t, p, q, abi.Reservations(views, infos, devs, gpu_raw)


def config5(n_nodes: int = 100_000, n_pods: int = 10_000, rsv_gpu: bool = True):
    """BASELINE config 5 as SURVEY.md §8d states it: cluster5 with per-minor GPU usage U(0, 1) and the 20%
    SingleNUMANode nodes of configs 2-3 (GPU pods there join DeviceShare's NUMA hints to the topology manager).
    rsv_gpu=False: no reservation holds GPUs (the form kg_replay follows through Reservation.Reserve)."""
    return cluster5(n_nodes, n_pods, numa="single", usage="u01", rsv_gpu=rsv_gpu)


def gpu_topology5(t: abi.Table, p: abi.Table, seed_config: int = 5, any_numa: bool = False):
    """GPU topology and partitions of a config-5 cluster (own random stream, so the other draws do not
    move): 90% of the nodes report GPU topology (two NUMA nodes of four minors; half of them two GPUs per PCIe
    switch, half one, like the reference's fakeDeviceCR / fakeH800DeviceCR), 30% are labelled H100 (the
    Hopper partition table), a third of those with the Honor partition policy. GPU pods: whole-GPU pods carry a
    GPUPartitionSpec 10% of the time (a third Restricted), and 10% of the GPU pods require a NUMANode or PCIe
    topology scope."""
    n, n_pods = abi.table_len(t), abi.table_len(p)
    r = _rng(seed_config, 2)
    has = r.random(n) < 0.90
    pair = r.random(n) < 0.5
    h100 = r.random(n) < 0.30
    honor = h100 & (r.random(n) < 1 / 3)
    layouts = [[(m // 4, str(m // 2)) for m in range(8)], [(m // 4, str(m)) for m in range(8)]]
    topos = [decode.gpu_topology([{"minor": m, "topology": {"nodeID": q, "pcieID": pc}} for m, (q, pc) in enumerate(l)])[0]
             for l in layouts]
    tabs = decode.GpuPartitionTables()
    hop = tabs.add(decode.gpu_partition_table(None, {"metadata": {"labels": {decode.LABEL_GPU_MODEL: "H100"}}})[0])
    t["dev_topo"] = np.where(has, np.where(pair, np.uint64(topos[0]), np.uint64(topos[1])),
                             np.uint64((1 << 64) - 1)).astype(np.uint64)
    # the GPUs' NUMA node ids (NUMATopology.deviceToNodeID): minors 0-3 on NUMA node 0, 4-7 on node 1
    numa_ids = decode.gpu_numa([{"minor": m, "topology": {"nodeID": q}} for m, (q, _) in enumerate(layouts[0])])
    t["dev_numa"] = np.where(has, np.uint32(numa_ids), np.uint32(0xFFFFFFFF)).astype(np.uint32)
    if any_numa:  # (own stream) minor 7 reports Topology.NodeID -1 on 5% of the GPU nodes
        ra = _rng(seed_config, 4)
        anyn = has & (ra.random(n) < 0.05)
        l2 = [(q if m != 7 else -1, pc) for m, (q, pc) in enumerate(layouts[0])]
        infos = [{"minor": m, "topology": {"nodeID": q, "pcieID": pc}} for m, (q, pc) in enumerate(l2)]
        t["dev_topo"] = np.where(anyn, np.uint64(decode.gpu_topology(infos)[0]), t["dev_topo"]).astype(np.uint64)
        t["dev_numa"] = np.where(anyn, np.uint32(decode.gpu_numa(infos)), t["dev_numa"]).astype(np.uint32)
    t["dev_part"] = (np.where(has, abi.KG_GPU_TREE, 0) | np.where(h100, hop, 0) |
                     np.where(honor, abi.KG_GPU_HONOR, 0)).astype(np.uint32)
    t["gpu_parts"] = tabs.array()
    flags = np.zeros(n_pods, np.uint32)
    gpu = p["dev_count"] > 0
    # gpuShared as calcDesiredRequestsAndCountForGPU decides it (decode.gpu_requirements)
    has_ratio = ((p["dev_keys"] >> abi.KG_DEV_RATIO) & 1) != 0
    shared = gpu & np.where(has_ratio, p["dev_req"][:, abi.KG_DEV_RATIO] < 100, ((p["dev_keys"] >> abi.KG_DEV_MEM) & 1) != 0)
    flags |= np.where(shared, abi.KG_GPU_POD_SHARED, 0).astype(np.uint32)
    spec = gpu & ~shared & (r.random(n_pods) < 0.10)
    flags |= np.where(spec, abi.KG_GPU_POD_HONOR, 0).astype(np.uint32)
    flags |= np.where(spec & (r.random(n_pods) < 1 / 3), abi.KG_GPU_POD_RESTRICTED, 0).astype(np.uint32)
    scope = np.where(r.random(n_pods) < 0.5, 2, 3)
    req_scope = gpu & (r.random(n_pods) < 0.10)
    flags |= np.where(req_scope, scope << abi.KG_GPU_POD_SCOPE_SHIFT, 0).astype(np.uint32)
    p["dev_flags"] = flags


def topology(n_nodes: int, n_pods: int, seed: int = 0, pod_policy_frac: float = 0.3):
    """NUMA topology-manager workload: nodes with 1-4 zones under every policy
    (None / BestEffort / Restricted / SingleNUMANode), zone statuses (idle / single / shared), pods
    with and without their own NUMA policy and large enough that multi-zone hints are needed."""
    r = _rng(900 + seed, 0)
    t = nodes(n_nodes, 900 + seed, numa=True, rng=r)
    n = n_nodes
    Z = r.integers(1, 5, n).astype(np.uint32)
    Z[r.random(n) < 0.03] = 0  # a few nodes without NUMA resources
    t["numa_zones"] = Z
    t["numa_policy"] = r.choice([abi.KG_NUMA_NONE, abi.KG_NUMA_BEST_EFFORT, abi.KG_NUMA_RESTRICTED,
                                 abi.KG_NUMA_SINGLE_NODE], n, p=[0.25, 0.25, 0.25, 0.25]).astype(np.uint32)
    zs = np.maximum(Z, 1).astype(np.int64)
    status = np.zeros(n, np.uint32)
    for z in range(abi.KG_MAX_ZONES):
        on = z < Z
        zc = np.where(on, t["alloc_cpu"] // zs, 0)
        zm = np.where(on, t["alloc_mem"] // zs, 0)
        t[f"zone_cpu{z}"] = zc
        t[f"zone_mem{z}"] = zm
        lvl = r.choice([0.0, 0.3, 0.6, 0.9, 1.0], n)
        t[f"zone_cpu_used{z}"] = (zc * lvl * r.random(n)).astype(np.int64)
        t[f"zone_mem_used{z}"] = (zm * lvl * r.random(n)).astype(np.int64)
        full = r.random(n) < 0.05  # a zone with no cpu left
        t[f"zone_cpu_used{z}"] = np.where(full & on, zc, t[f"zone_cpu_used{z}"])
        status |= (np.where(on, r.choice([0, 1, 2], n, p=[0.6, 0.2, 0.2]), 0).astype(np.uint32) << (2 * z))
    t["numa_zone_status"] = status
    used_cpu = sum(t[f"zone_cpu_used{z}"] for z in range(abi.KG_MAX_ZONES))
    used_mem = sum(t[f"zone_mem_used{z}"] for z in range(abi.KG_MAX_ZONES))
    t["req_cpu"] = np.maximum(t["req_cpu"], used_cpu)
    t["req_mem"] = np.maximum(t["req_mem"], used_mem)
    t["nz_cpu"] = np.maximum(t["nz_cpu"], t["req_cpu"])
    t["nz_mem"] = np.maximum(t["nz_mem"], t["req_mem"])
    pr = _rng(900 + seed, 1)
    p = pods(n_pods, 900 + seed, scale=4.0, rng=pr)
    pol = pr.choice([abi.KG_NUMA_BEST_EFFORT, abi.KG_NUMA_RESTRICTED, abi.KG_NUMA_SINGLE_NODE], n_pods)
    p["numa_policy"] = np.where(pr.random(n_pods) < pod_policy_frac, pol, abi.KG_NUMA_NONE).astype(np.uint32)
    return bench_profile(numa=True), t, p


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


CPU_SHAPES = ((1, 1, 16, 2), (2, 1, 16, 2), (2, 2, 12, 2), (2, 2, 8, 1))  # buildCPUTopologyForTest shapes


def cpuset_cluster(n_nodes: int, n_pods: int, seed: int = 0, bind_frac: float = 0.3, node_bind_frac: float = 0.06,
                   no_topo_frac: float = 0.08):
    """A small cluster with cpuset binding: CPU topologies of CPU_SHAPES on most nodes, an
    existing allocation per node (cpuset_alloc_milli = 1000 x allocated CPUs, RefCount up to maxRefCount 1 or
    2, random exclusive policies), node CPU bind policies on a few nodes, both NUMA allocate strategies; pods
    from pods() with a share turned into LSE/LSR cpuset pods (whole cores, Full/Spread policy, required or
    preferred, random exclusive policy)."""
    cfg, t, pt = small(n_nodes, n_pods, seed=seed, numa=True)
    r = _rng(200 + seed, 7)
    topos = [abi.cpu_topo_for_test(*sh) for sh in CPU_SHAPES]
    n = n_nodes
    ti = r.integers(0, len(topos), n).astype(np.int32)
    ti[r.random(n) < no_topo_frac] = -1
    max_ref = np.where(r.random(n) < 0.15, 2, 1).astype(np.uint8)
    alloc = np.zeros((n, 2 * abi.KG_MAX_CPUS), np.uint8)
    cs = np.zeros(n, np.int64)
    for i in range(n):
        if ti[i] < 0:
            continue
        nc = topos[ti[i]].n_cpus
        k = int(r.integers(0, int(nc * 0.6) + 1))
        k = min(k, int(t["req_cpu"][i] // 1000))
        cpus = r.choice(nc, size=k, replace=False)
        for c in cpus:
            alloc[i, c] = 1 if max_ref[i] == 1 else int(r.integers(1, 3))
            alloc[i, abi.KG_MAX_CPUS + c] = int(r.integers(0, 3))
        cs[i] = 1000 * k
    t["cpu_topo"] = ti
    t["cpu_topos"] = abi.cpu_topos_array(topos)
    t["cpu_alloc"] = alloc
    t["cpu_max_ref"] = max_ref
    nb = np.zeros(n, np.uint8)
    u = r.random(n)
    nb[u < node_bind_frac / 2] = abi.KG_NODE_CPU_BIND_FULL_PCPUS_ONLY
    nb[(u >= node_bind_frac / 2) & (u < node_bind_frac)] = abi.KG_NODE_CPU_BIND_SPREAD_BY_PCPUS
    t["cpu_bind_policy"] = nb
    t["cpu_strategy"] = r.integers(0, 2, n).astype(np.uint8)
    t["cpuset_alloc_milli"] = cs
    # cpuset pods: prod pods with whole-core requests
    m = len(pt["req_cpu"])
    bind = (r.random(m) < bind_frac) & ((pt["flags"] & abi.KG_POD_PROD) != 0)
    cores = r.choice([1, 2, 4, 6, 8, 16], m)
    pt["req_cpu"] = np.where(bind, cores * 1000, pt["req_cpu"]).astype(np.int64)
    pt["nz_cpu"] = np.where(bind, cores * 1000, pt["nz_cpu"]).astype(np.int64)
    pol = r.integers(1, 3, m).astype(np.uint32)
    req = r.random(m) < 0.35
    excl = r.integers(0, 3, m).astype(np.uint32)
    f = pt["flags"].astype(np.uint32)
    f = np.where(bind, f | abi.KG_POD_CPU_BIND | (pol << abi.KG_POD_CPU_POLICY_SHIFT) |
                 np.where(req, abi.KG_POD_CPU_REQUIRED, 0).astype(np.uint32) | (excl << abi.KG_POD_CPU_EXCL_SHIFT), f)
    pt["flags"] = f.astype(np.uint32)
    return cfg, t, pt


def add_cpusets(t: abi.Table, p: abi.Table, seed: int = 0, bind_frac: float = 0.08, node_bind_frac: float = 0.05):
    """Cpuset binding on any cluster (own random stream): a CPU topology on every node (2 sockets x 1 NUMA node x
    cores/2 cores x 2 threads, matching its cpu allocatable before amplification), an existing allocation of up to
    half the CPUs where cpuset_alloc_milli holds one, node CPU bind policies on a few policy-None nodes, and LSR pods
    (prod pods with whole-core cpu requests binding cpusets, Full / Spread, a third required, random exclusive
    policy). Used to put cpuset pods into the config-5 replay and batch cycle."""
    r = _rng(300 + seed, 9)
    n, m = abi.table_len(t), abi.table_len(p)
    ratio = np.where(t["cpu_amp_ratio"] > 1, t["cpu_amp_ratio"], 1.0) if "cpu_amp_ratio" in t else np.ones(n)
    cores = np.rint(t["alloc_cpu"] / ratio / 1000).astype(np.int64)
    shapes = {32: 0, 64: 1, 96: 2}
    topos = [abi.cpu_topo_for_test(2, 1, c // 4, 2) for c in (32, 64, 96)]
    ti = np.array([shapes.get(int(c), 0) for c in cores], np.int32)
    ncpu = np.array([32, 64, 96])[ti]
    alloc = np.zeros((n, 2 * abi.KG_MAX_CPUS), np.uint8)
    cs = np.zeros(n, np.int64)
    have = t["cpuset_alloc_milli"] if "cpuset_alloc_milli" in t else np.zeros(n, np.int64)
    for i in np.nonzero(have > 0)[0]:
        k = int(min(have[i] // 1000, ncpu[i] // 2))
        cpus = r.choice(int(ncpu[i]), size=k, replace=False)
        alloc[i, cpus] = 1
        alloc[i, abi.KG_MAX_CPUS + cpus] = r.integers(0, 3, k)
        cs[i] = 1000 * k
    t["cpu_topo"] = ti
    t["cpu_topos"] = abi.cpu_topos_array(topos)
    t["cpu_alloc"] = alloc
    t["cpu_max_ref"] = np.ones(n, np.uint8)
    t["cpuset_alloc_milli"] = cs
    nb = np.zeros(n, np.uint8)
    pick = (t["numa_policy"] == abi.KG_NUMA_NONE) & (r.random(n) < node_bind_frac)
    nb[pick & (r.random(n) < 0.5)] = abi.KG_NODE_CPU_BIND_FULL_PCPUS_ONLY
    nb[pick & (nb == 0)] = abi.KG_NODE_CPU_BIND_SPREAD_BY_PCPUS
    t["cpu_bind_policy"] = nb
    t["cpu_strategy"] = r.integers(0, 2, n).astype(np.uint8)
    bind = (r.random(m) < bind_frac) & ((p["flags"] & abi.KG_POD_PROD) != 0)
    whole = r.choice([1, 2, 4, 8], m)
    p["req_cpu"] = np.where(bind, whole * 1000, p["req_cpu"]).astype(np.int64)
    p["nz_cpu"] = np.where(bind, whole * 1000, p["nz_cpu"]).astype(np.int64)
    cpol = r.integers(1, 3, m).astype(np.uint32)
    req = r.random(m) < 1 / 3
    excl = r.integers(0, 3, m).astype(np.uint32)
    f = p["flags"].astype(np.uint32)
    p["flags"] = np.where(bind, f | abi.KG_POD_CPU_BIND | (cpol << abi.KG_POD_CPU_POLICY_SHIFT) |
                          np.where(req, abi.KG_POD_CPU_REQUIRED, 0).astype(np.uint32) | (excl << abi.KG_POD_CPU_EXCL_SHIFT),
                          f).astype(np.uint32)
    return t, p


def mixed(n_nodes: int = 10_000, n_pods: int = 10_000, seed: int = 6):
    """A realistic mixed cluster (bench config 6): config 2's nodes and pods, plus
    - kubelet topology-manager policies: 20% SingleNUMANode (as config 2), 10% Restricted, 10% BestEffort;
    - CPU topologies on every node (2 sockets x 1 NUMA node x cores/2 cores x 2 threads, matching the node's
      cpu allocatable before amplification), existing cpuset allocations as nodes() sets them;
    - 5% of the nodes (NUMA policy None) with a node CPU bind policy (FullPCPUsOnly / SpreadByPCPUs), where
      every pod with a cpu request binds cpusets;
    - 5% LSR pods: prod pods with whole-core cpu requests binding cpusets (Full / Spread, a third required).
    Restricted / BestEffort nodes and CPU-bind-policy nodes are outside the float64 fast path (F_BIG: the
    integer path with the general NUMA topology manager / cpuset checks); LSR pods take the integer path on
    every node."""
    cfg = bench_profile(numa=True)
    r = _rng(seed)
    t = nodes(n_nodes, seed, numa=True, rng=r)
    n = n_nodes
    pol = t["numa_policy"].copy()
    u = r.random(n)
    none = pol == abi.KG_NUMA_NONE
    pol[none & (u < 0.125)] = abi.KG_NUMA_RESTRICTED  # 0.8 x 0.125 = 10% of all nodes
    pol[none & (u >= 0.125) & (u < 0.25)] = abi.KG_NUMA_BEST_EFFORT
    t["numa_policy"] = pol.astype(np.uint32)
    # CPU topologies by core count (alloc before amplification: 32 / 64 / 96 cores)
    cores = np.rint(t["alloc_cpu"] / np.where(t["cpu_amp_ratio"] > 1, t["cpu_amp_ratio"], 1.0) / 1000).astype(np.int64)
    shapes = {32: 0, 64: 1, 96: 2}
    topos = [abi.cpu_topo_for_test(2, 1, c // 4, 2) for c in (32, 64, 96)]
    ti = np.array([shapes.get(int(c), 0) for c in cores], np.int32)
    alloc = np.zeros((n, 2 * abi.KG_MAX_CPUS), np.uint8)
    cs = np.zeros(n, np.int64)
    ncpu = np.array([32, 64, 96])[ti]
    for i in np.nonzero(t["cpuset_alloc_milli"] > 0)[0]:
        k = int(min(t["cpuset_alloc_milli"][i] // 1000, ncpu[i] // 2))
        cpus = r.choice(int(ncpu[i]), size=k, replace=False)
        alloc[i, cpus] = 1
        cs[i] = 1000 * k
    t["cpu_topo"] = ti
    t["cpu_topos"] = abi.cpu_topos_array(topos)
    t["cpu_alloc"] = alloc
    t["cpu_max_ref"] = np.ones(n, np.uint8)
    t["cpuset_alloc_milli"] = cs
    nb = np.zeros(n, np.uint8)
    v = r.random(n)
    pick = (t["numa_policy"] == abi.KG_NUMA_NONE) & (v < 0.05 / 0.6)  # policy None is 60% of the nodes
    nb[pick & (r.random(n) < 0.5)] = abi.KG_NODE_CPU_BIND_FULL_PCPUS_ONLY
    nb[pick & (nb == 0)] = abi.KG_NODE_CPU_BIND_SPREAD_BY_PCPUS
    t["cpu_bind_policy"] = nb
    t["cpu_strategy"] = r.integers(0, 2, n).astype(np.uint8)
    pr = _rng(seed, 1)
    p = pods(n_pods, seed, rng=pr)
    m = n_pods
    bind = (pr.random(m) < 0.05 / 0.7) & ((p["flags"] & abi.KG_POD_PROD) != 0)
    whole = pr.choice([1, 2, 4, 8], m)
    p["req_cpu"] = np.where(bind, whole * 1000, p["req_cpu"]).astype(np.int64)
    p["nz_cpu"] = np.where(bind, whole * 1000, p["nz_cpu"]).astype(np.int64)
    cpol = pr.integers(1, 3, m).astype(np.uint32)
    req = pr.random(m) < 1 / 3
    f = p["flags"].astype(np.uint32)
    p["flags"] = np.where(bind, f | abi.KG_POD_CPU_BIND | (cpol << abi.KG_POD_CPU_POLICY_SHIFT) |
                          np.where(req, abi.KG_POD_CPU_REQUIRED, 0).astype(np.uint32), f).astype(np.uint32)
    return cfg, t, p


def small(n_nodes: int, n_pods: int, seed: int = 0, numa: bool = True, scale: float = 1.0) -> tuple:
    """Small synthetic cluster for parity tests."""
    cfg: SchedulerConfig = bench_profile(numa=numa)
    return cfg, nodes(n_nodes, 100 + seed, numa=numa), pods(n_pods, 100 + seed, scale=scale)
