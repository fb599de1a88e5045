"""Builders for the known-answer cases of tests/golden/pin_kat.json (see make_pin_kat.py).

Each builder restates the fixture set-up of the reference test runner it cites and returns
(kg_config, nodes table, pods table, reservations or None, expectation dict). The expectations are
checked on the oracle (CPU) and on the device through the C ABI by tests/test_pin_kat.py.
"""
import json
import os

import numpy as np

from koordinator_amd import abi, decode
from koordinator_amd.config import BATCH_CPU, BATCH_MEMORY, SchedulerConfig

HERE = os.path.dirname(os.path.abspath(__file__))
GI = 1 << 30
MI = 1 << 20


def load():
    with open(os.path.join(HERE, "golden", "pin_kat.json")) as f:
        return json.load(f)


def _nodes(n):
    t = abi.empty_nodes(n)
    t["alloc_pods"][:] = 110
    return t


def _add_existing(t, i, cpu_m=0, mem_b=0, sc=(0, 0), has_mem=True):
    """NodeInfo.AddPod of an existing pod: Requested, NonZeroRequested (100m / 200Mi defaults), len(Pods)."""
    t["req_cpu"][i] += cpu_m
    t["req_mem"][i] += mem_b
    t["nz_cpu"][i] += cpu_m if cpu_m else 100
    t["nz_mem"][i] += mem_b if has_mem and mem_b else 200 * MI
    for k in range(2):
        t[f"sc_req{k}"][i] += sc[k]
    t["num_pods"][i] += 1


def _pod(cpu_m=0, mem_b=0, eph_b=0, sc=(0, 0), has_cpu=None, has_mem=None, prod=True):
    p = abi.empty_pods(1)
    p["req_cpu"][0], p["req_mem"][0], p["req_eph"][0] = cpu_m, mem_b, eph_b
    p["sc_req0"][0], p["sc_req1"][0] = sc
    p["nz_cpu"][0] = cpu_m if (has_cpu if has_cpu is not None else cpu_m) else 100
    p["nz_mem"][0] = mem_b if (has_mem if has_mem is not None else mem_b) else 200 * MI
    f = abi.KG_POD_PROD if prod else 0
    if has_cpu if has_cpu is not None else cpu_m:
        f |= abi.KG_POD_HAS_CPU
    if has_mem if has_mem is not None else mem_b:
        f |= abi.KG_POD_HAS_MEM
    if not (cpu_m or mem_b or eph_b or sc[0] or sc[1]):
        f |= abi.KG_POD_NUMA_SKIP
    p["flags"][0] = f
    return p


# ---- NodeResourcesFit ------------------------------------------------------------------------------

def nrf_fits(case):
    """job_nominated_pods_test.go:355-386: NodeInfo of test-node plus the nominated pods not removed."""
    kc = SchedulerConfig(plugins=abi.KG_PLUGIN_NRF).kg_config()
    t = _nodes(1)
    t["alloc_cpu"][0] = case["node"]["cpu"] * 1000
    t["alloc_pods"][0] = case["node"]["pods"]
    for c in case["existing_cpu"]:
        _add_existing(t, 0, cpu_m=c * 1000, has_mem=False)
    pods = _pod(cpu_m=case["pod_cpu"] * 1000)
    return kc, t, pods, None, {"nrf_reasons": case["want"]}


FITS_SCALARS = ("example.com/gpu", "other.io/fpga")


def fits_ignored(case, plugin):
    """reservation/plugin_test.go:6839-6847: fitsNode(podRequest, nodeAlloc, allPodsRequested, nil, nil, 0, 1,
    ...), on the device either as NodeResourcesFit Fits (plugin "nrf", ignored scalars from the Fits args)
    or as the Reservation Filter's node-alone fitsNode (plugin "rsv": a view with no matched reservation
    and a pod without reservation affinity)."""
    cfg = SchedulerConfig(plugins=abi.KG_PLUGIN_NRF if plugin == "nrf" else abi.KG_PLUGIN_RSV,
                          scalar_resources=FITS_SCALARS, nrf_resources=[("cpu", 1), ("memory", 1)],
                          nrf_ignored=tuple(case["ignored"]), nrf_ignored_groups=tuple(case["ignored_groups"]),
                          rsv_ignored=tuple(case["ignored"]), rsv_ignored_groups=tuple(case["ignored_groups"]))
    kc = cfg.kg_config()
    a = case["alloc"]
    t = _nodes(1)
    t["alloc_cpu"][0] = a.get("cpu", 0) * 1000
    t["alloc_mem"][0] = a.get("mem", 0) * GI
    t["alloc_pods"][0] = a.get("pods", 0)
    t["sc_alloc0"][0] = a.get("sc0", 0)
    t["sc_alloc1"][0] = a.get("sc1", 0)
    r = case["requested"]
    t["req_cpu"][0] = r.get("cpu", 0) * 1000
    t["num_pods"][0] = 1  # allocatedPods = 1
    pr = case["pod"]
    pods = _pod(cpu_m=pr.get("cpu", 0) * 1000, sc=(pr.get("sc0", 0), pr.get("sc1", 0)))
    rsv = None
    if plugin == "rsv":
        pods["rsv_class"][0] = 0
        view = dict(node=0, cls=0, first=0, count=0, req=[t["req_cpu"][0], 0, 0, 0, 0], nz_cpu=0, nz_mem=0,
                    num_pods=1, pod_requested=[t["req_cpu"][0], 0, 0, 0, 0], r_allocated=[0] * 5)
        rsv = abi.Reservations([view], [])
    want = case["want"]
    if plugin == "nrf":
        names = {"cpu": "Insufficient cpu", FITS_SCALARS[0]: f"Insufficient {FITS_SCALARS[0]}",
                 FITS_SCALARS[1]: f"Insufficient {FITS_SCALARS[1]}"}
        return kc, t, pods, rsv, {"nrf_reasons": [names[w] for w in want], "scalars": FITS_SCALARS}
    return kc, t, pods, rsv, {"status": abi.KG_ST_RSV_NODE if want else 0}


def nrfp_score(case):
    """node_resources_fit_plus_test.go:140-318: testNode1 / testNode2 and the incoming pod; cpu / memory on
    NonZeroRequested, nvidia.com/gpu on Requested (node_resource_fit_plus_utils.go:114-139)."""
    res = case["resources"]
    cfg = SchedulerConfig(plugins=abi.KG_PLUGIN_NRF, scalar_resources=("nvidia.com/gpu", "xx.xx/xx"),
                          nrf_resources=[(n, w) for n, w, _ in res],
                          nrf_most=tuple(n for n, _, ty in res if ty == "MostAllocated"))
    kc = cfg.kg_config()
    t = _nodes(len(case["nodes"]))
    for i, nd in enumerate(case["nodes"]):
        t["alloc_cpu"][i] = nd["cpu"] * 1000
        t["alloc_mem"][i] = nd["mem"] * GI
        t["alloc_eph"][i] = nd["eph"] * GI
        t["sc_alloc0"][i] = nd["gpu"]
        t["alloc_pods"][i] = 0  # the test nodes list no "pods" allocatable (Score only)
        ex = nd["existing"]
        if ex:
            _add_existing(t, i, cpu_m=ex["cpu"] * 1000, mem_b=ex["mem"] * GI, sc=(ex["gpu"], 0))
    p = case["pod"]
    pods = _pod(cpu_m=p["cpu"] * 1000, mem_b=p["mem"] * GI, eph_b=p["eph"] * GI, sc=(p["gpu"], 0))
    return kc, t, pods, None, {"score_nrf": case["want_scores"], "order": case["want"]}


# ---- NodeNUMAResource with amplified CPUs --------------------------------------------------------------

def _amp_pod(p):
    if p is None:
        return _pod()
    pods = _pod(cpu_m=p["cpu"] * 1000, mem_b=p.get("mem", 0) * GI)
    if p.get("cpuset"):
        pods["flags"][0] |= abi.KG_POD_CPU_BIND  # LSR prod pod: AllowUseCPUSet (nodenumaresource/util.go:49-56)
    return pods


def numa_amp_filter(case):
    """plugin_test.go:1207-1232: node-1 = makeNode(cpu 32, memory 40Gi, ratio); existing pods through the
    NodeInfo and the pod event handler (cpuset pods count as the resource manager's allocated CPUs)."""
    kc = SchedulerConfig(plugins=abi.KG_PLUGIN_NUMA).kg_config()
    t = _nodes(1)
    ratio = case["ratio"]
    t["alloc_cpu"][0] = decode.amplify(32 * 1000, ratio)
    t["alloc_mem"][0] = 40 * GI
    t["cpu_amp_ratio"][0] = ratio
    for e in case["existing"]:
        _add_existing(t, 0, cpu_m=e["cpu"] * 1000, has_mem=False)
        if e["cpuset"] and case["nrt"]:
            t["cpuset_alloc_milli"][0] += e["cpu"] * 1000
    pods = _amp_pod(case["pod"])
    want = case["want"]
    exp = {"numa_reasons": want}
    if not want and case["pod"] and case["pod"].get("cpuset"):
        exp = {"host_path": True}
    return kc, t, pods, None, exp


def numa_amp_score(case):
    """scoring_test.go:947-1006: nodes from makeNode (allocatable cpu amplified by the ratio), topology
    options with the node's CPU topology for the nodes in nodeHasNRT, existing pods via the NodeInfo and
    the pod event handler."""
    cfg = SchedulerConfig(plugins=abi.KG_PLUGIN_NUMA, numa_strategy=case["strategy"])
    kc = cfg.kg_config()
    n = len(case["nodes"])
    t = _nodes(n)
    names = [f"node{i + 1}" for i in range(n)]
    for i, (cpu, mem, ratio) in enumerate(case["nodes"]):
        t["alloc_cpu"][i] = decode.amplify(cpu * 1000, ratio)
        t["alloc_mem"][i] = mem * GI
        t["cpu_amp_ratio"][i] = ratio
    # nodes in nodeHasNRT carry the CPU topology buildCPUTopologyForTest(2, 1, 8, 2) (scoring_test.go:982-996);
    # an existing cpuset pod holds that many CPUs in the resource manager (the count is what the Score reads)
    t["cpu_topo"] = np.array([0 if nm in case["nrt"] else -1 for nm in names], np.int32)
    t["cpu_topos"] = abi.cpu_topos_array([abi.cpu_topo_for_test(2, 1, 8, 2)])
    t["cpu_alloc"] = np.zeros((n, 2 * abi.KG_MAX_CPUS), np.uint8)
    held = [0] * n
    for node, cpu, mem, cpuset in case["existing"]:
        i = names.index(node)
        _add_existing(t, i, cpu_m=cpu * 1000, mem_b=mem * GI)
        if cpuset and node in case["nrt"]:
            t["cpuset_alloc_milli"][i] += cpu * 1000
            t["cpu_alloc"][i, held[i]:held[i] + cpu] = 1
            held[i] += cpu
    pods = _amp_pod(case["pod"])
    return kc, t, pods, None, {"score_numa": case["want"]}


# ---- Reservation -----------------------------------------------------------------------------------------

RSV_KEYS = ("cpu", "mem", "eph", "bcpu", "bmem")


def _rsv_vec(d):
    """{cpu | cpu_m, mem, bcpu_m, bmem} -> [cpu milli, memory B, ephemeral B, batch-cpu, batch-memory B]"""
    v = [0] * 5
    v[0] = d.get("cpu", 0) * 1000 + d.get("cpu_m", 0)
    v[1] = d.get("mem", 0) * GI
    v[3] = d.get("bcpu_m", 0)
    v[4] = d.get("bmem", 0) * GI
    return v


def rsv_filter(case):
    """plugin_test.go:2522-2544: test-node (:1162-1174) with an empty NodeInfo, the case's stateData; the
    ReservationInfo fields as frameworkext.NewReservationInfo / AddAssignedPod derive them
    (reservation_info.go:92-132,490-500, RefreshPreCalculated :516-529)."""
    kc = SchedulerConfig(plugins=abi.KG_PLUGIN_RSV, scalar_resources=(BATCH_CPU, BATCH_MEMORY)).kg_config()
    t = _nodes(1)
    t["alloc_cpu"][0] = 32000
    t["alloc_mem"][0] = 32 * GI
    t["alloc_pods"][0] = 100
    t["sc_alloc0"][0] = 7500
    t["sc_alloc1"][0] = 10 * GI
    r = case["rsv"]
    alloc = _rsv_vec(r["allocatable"])
    names = sum(1 << k for k in range(5) if alloc[k] != 0)
    allocated = [0] * 5
    for c in r.get("assigned_cpu", []):
        allocated[0] += c * 1000  # quotav1.Mask(requests, ResourceNames): cpu is a name
    info = dict(policy=getattr(abi, "KG_RSV_" + r["policy"].upper()), names=names, allocate_once=1, order=0,
                allocatable=alloc, allocated=allocated, reserved=_rsv_vec(r.get("reserved", {})),
                max_pods=r["allocatable"].get("pods", -1), allocated_pods=len(r.get("assigned_cpu", [])))
    view = dict(node=0, cls=0, first=0, count=1, req=[0] * 5, nz_cpu=0, nz_mem=0, num_pods=0,
                pod_requested=_rsv_vec(case["pod_requested"]), r_allocated=_rsv_vec(case["r_allocated"]))
    rsvs = abi.Reservations([view], [info])
    pr = case["pod"]
    v = _rsv_vec(pr)
    pods = _pod(cpu_m=v[0], mem_b=v[1], sc=(v[3], v[4]), has_cpu="cpu" in pr or "cpu_m" in pr, has_mem="mem" in pr)
    pods["rsv_class"][0] = 0
    if case["affinity"]:
        pods["flags"][0] |= abi.KG_POD_RSV_REQUIRED
    st = 0
    for w in case["want"]:
        st |= abi.KG_ST_RSV_RESERVATION if w.startswith("Reservation(s)") else abi.KG_ST_RSV_NODE
    return kc, t, pods, rsvs, {"status": st}


# ---- DeviceShare -----------------------------------------------------------------------------------------

def _dev(minors, pod, strategy="LeastAllocated"):
    kc = SchedulerConfig(plugins=abi.KG_PLUGIN_DEV, dev_strategy=strategy).kg_config()
    t = _nodes(1)
    t["alloc_cpu"][0] = 64000
    t["alloc_mem"][0] = 256 * GI
    t["dev_minors"][0] = len(minors)
    for m, x in enumerate(minors):
        t["dev_total"][0, :, m] = [x["total"][0], x["total"][1], x["total"][2] * GI]
        t["dev_free"][0, :, m] = [x["free"][0], x["free"][1], x["free"][2] * GI]
    pods = abi.empty_pods(1)
    req = {("koordinator.sh/" + k): (v * GI if k == "gpu-memory" else v) for k, v in pod.items()}
    vec, keys, cnt, _ = decode.gpu_requirements(req)
    pods["dev_req"][0] = vec
    pods["dev_keys"][0] = keys
    pods["dev_count"][0] = cnt
    return kc, t, pods


def dev_filter(case):
    """deviceshare/plugin_test.go:3181-3220: Filter on test-node with the case's nodeDevice."""
    kc, t, pods = _dev(case["minors"], case["pod"])
    w = case["want"]
    return kc, t, pods, None, {"status": getattr(abi, w) if isinstance(w, str) else w}


def dev_score_device(case):
    """deviceshare/scoring_test.go:1319-1333: scoreDevice(requests, total, free) of one minor that only
    has gpu-memory-ratio; the node score of a one-minor node is that minor's score."""
    minor = {"total": [0, case["total"], 0], "free": [0, case["free"], 0]}
    kc, t, pods = _dev([minor], {"gpu-memory-ratio": case["req"]}, case["strategy"])
    if case.get("infeasible"):
        return kc, t, pods, None, {"status": abi.KG_ST_DEV_INSUFFICIENT, "score_dev": [case["want"]]}
    return kc, t, pods, None, {"status": 0, "score_dev": [case["want"]]}


def dev_score_most(case):
    """deviceshare/scoring_test.go:562-599 (TestScore runner) with ScoringStrategy MostAllocated."""
    kc, t, pods = _dev(case["minors"], case["pod"], "MostAllocated")
    return kc, t, pods, None, {"status": 0, "score_dev": [case["want"]]}


def dev_normalize(case):
    """deviceshare/scoring_test.go:660-666: NormalizeScore over the node scores; here every node's raw score
    comes from one ratio-only minor (free, request) and the normalised term is the weighted total (weight 1,
    the other plugins off)."""
    raws = case["raw"]
    kc = SchedulerConfig(plugins=abi.KG_PLUGIN_DEV).kg_config()
    t = _nodes(len(raws))
    t["alloc_cpu"][:] = 64000
    t["alloc_mem"][:] = 256 * GI
    t["dev_minors"][:] = 1
    req = raws[0][1]
    for i, (free, r) in enumerate(raws):
        assert r == req  # one pod
        t["dev_total"][i, 1, 0] = 100
        t["dev_free"][i, 1, 0] = free
    pods = abi.empty_pods(1)
    vec, keys, cnt, _ = decode.gpu_requirements({"koordinator.sh/gpu-memory-ratio": req})
    pods["dev_req"][0] = vec
    pods["dev_keys"][0] = keys
    pods["dev_count"][0] = cnt
    return kc, t, pods, None, {"status": 0, "total": case["want"]}


BUILDERS = {
    "nrf_fits": nrf_fits,
    "fits_ignored_nrf": lambda c: fits_ignored(c, "nrf"),
    "fits_ignored_rsv": lambda c: fits_ignored(c, "rsv"),
    "nrfp_score": nrfp_score,
    "numa_amp_filter": numa_amp_filter,
    "numa_amp_score": numa_amp_score,
    "rsv_filter": rsv_filter,
    "dev_filter": dev_filter,
    "dev_score_device": dev_score_device,
    "dev_score_most": dev_score_most,
    "dev_normalize": dev_normalize,
}
SECTION = {"fits_ignored_nrf": "fits_ignored", "fits_ignored_rsv": "fits_ignored"}


def all_cases():
    data = load()
    out = []
    for key, fn in BUILDERS.items():
        for case in data[SECTION.get(key, key)]:
            out.append((f"{key}:{case['name']}", key, case))
    return out


def is_ext(kc):
    return (kc.plugins & abi.KG_PLUGIN_EXT) != 0
