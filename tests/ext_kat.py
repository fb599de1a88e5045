"""Builders for the config-5 known-answer cases of tests/golden/ext_kat.json (see make_ext_kat.py)."""
import json
import os

from koordinator_amd import abi, decode
from koordinator_amd.config import config5_profile

HERE = os.path.dirname(os.path.abspath(__file__))


def load():
    with open(os.path.join(HERE, "golden", "ext_kat.json")) as f:
        return json.load(f)


def _cfg(plugins):
    kc = config5_profile().kg_config()
    kc.plugins = plugins
    return kc


def _nodes(n, cpu=64000, mem=256 << 30):
    t = abi.empty_nodes(n)
    t["alloc_cpu"][:] = cpu
    t["alloc_mem"][:] = mem
    t["alloc_pods"][:] = 110
    return t


def deviceshare(case):
    kc = _cfg(abi.KG_PLUGIN_DEV)
    nodes = _nodes(1)
    nodes["dev_minors"][0] = len(case["minors"])
    for m, x in enumerate(case["minors"]):
        nodes["dev_total"][0, :, m] = x["total"]
        nodes["dev_free"][0, :, m] = x["free"]
    pods = abi.empty_pods(1)
    vec, keys, cnt, _ = decode.gpu_requirements(case["pod"])
    pods["dev_req"][0] = vec
    pods["dev_keys"][0] = keys
    pods["dev_count"][0] = cnt
    return kc, nodes, pods


def _info(alloc, allocated=None, order=0):
    return dict(policy=abi.KG_RSV_DEFAULT, names=0b11, allocate_once=1, order=order,
                allocatable=list(alloc) + [0, 0, 0], allocated=(list(allocated) if allocated else [0, 0]) + [0, 0, 0],
                reserved=[0] * 5, max_pods=-1, allocated_pods=0)


def _view(node, first, count):
    return dict(node=node, cls=0, first=first, count=count, req=[0] * 5, nz_cpu=0, nz_mem=0, num_pods=0,
                pod_requested=[0] * 5, r_allocated=[0] * 5)


def _pod(req):
    pods = abi.empty_pods(1)
    pods["rsv_class"][0] = 0
    if req is not None:
        pods["req_cpu"][0], pods["req_mem"][0] = req
        pods["nz_cpu"][0], pods["nz_mem"][0] = req
        pods["flags"][0] = abi.KG_POD_HAS_CPU | abi.KG_POD_HAS_MEM
    return pods


def reservation_score(case):
    kc = _cfg(abi.KG_PLUGIN_RSV)
    nodes = _nodes(1, *case["node"])
    infos = [_info(r["allocatable"], r.get("allocated")) for r in case["reservations"]]
    views = [_view(0, 0, len(infos))] if infos else []
    return kc, nodes, _pod(case["pod"]), abi.Reservations(views, infos)


def reservation_order(case):
    kc = _cfg(abi.KG_PLUGIN_RSV)
    n = case["nodes"]
    nodes = _nodes(n, 0, 0)
    nodes["alloc_pods"][:] = 0  # nodes without status: no allocatable at all
    infos = [_info(case["allocatable"], order=o) for o in case["orders"]]
    views = [_view(i, i, 1) for i in range(n)]
    return kc, nodes, _pod(case["pod"]), abi.Reservations(views, infos)


def elasticquota(case):
    kc = _cfg(abi.KG_PLUGIN_QUOTA)
    nodes = _nodes(1)
    q = abi.empty_quotas(1)
    q["used_limit"][0, :2] = case["limit"]
    q["limit_keys"][0] = 0b11
    pods = abi.empty_pods(1)
    pods["req_cpu"][0], pods["req_mem"][0] = case["pod"]
    pods["flags"][0] = abi.KG_POD_HAS_CPU | abi.KG_POD_HAS_MEM
    pods["quota"][0] = 0
    pods["quota_keys"][0] = 0b11
    return kc, nodes, pods, q
