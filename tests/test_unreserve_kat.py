"""The reference's Reserve / Unreserve and DeviceShare restore known answers (tests/golden/unreserve_kat.json, transcribed
by tests/golden/make_unreserve_kat.py from reservation/plugin_test.go TestUnreserve, deviceshare/plugin_test.go
Test_Plugin_Unreserve, deviceshare/reservation_test.go Test_Plugin_ReservationRestore and Test_allocateWithNominated),
run on the oracle session (kgo_ext_reserve / kgo_ext_unreserve, CPU) and on the device through the C ABI (kg_reserve /
kg_unreserve, GPU). Each case is one node of a small config-5 cluster (a second node holds nothing) built the way the
reference test builds its fixture: the node's GPUs and their used amounts (nodeDevice.updateCacheUsed of the reserve pod
and its assigned pods), the reservation, the pods of the case.

Checked per pod: the Reserve's minors and nominated reservation (the expected ones), the GPU restore tables after the
Reserve equal the host restore (decode.reservation_restore) recomputed from the reference's expected bookkeeping, the
reservation's Allocated / assigned pods after Reserve and after Unreserve, and the whole state given back."""
import json
import os

import numpy as np
import pytest

import oracle_lib
from koordinator_amd import abi, decode, synth
from koordinator_amd.config import GPU_CORE, GPU_MEMORY, GPU_MEMORY_RATIO

GI = 1 << 30
HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "unreserve_kat.json")) as f:
    CASES = json.load(f)
POLICY = {"Default": abi.KG_RSV_DEFAULT, "Aligned": abi.KG_RSV_ALIGNED, "Restricted": abi.KG_RSV_RESTRICTED}


def _tab(minors):
    t = np.zeros((abi.KG_DEV_R, abi.KG_DEV_MINORS), np.int64)
    for m, (c, r, g) in (minors or {}).items():
        t[abi.KG_DEV_CORE, int(m)], t[abi.KG_DEV_RATIO, int(m)], t[abi.KG_DEV_MEM, int(m)] = c, r, g * GI
    return t


def _rsv_dict(spec):
    if spec is None:
        return []
    r = dict(node=0, cls=int(spec["cls"]), allocatable=[int(spec["cpu_m"]), int(spec["mem"]) * GI, 0, 0, 0],
             allocated=None, reserved=None, allocated_pods=int(spec.get("allocated_pods", 0)),
             policy=POLICY[spec["policy"]], order=0, allocate_once=False, max_pods=-1, dev_alloc=None,
             dev_allocated=None)
    if r["allocated_pods"]:
        r["allocated"], r["allocated_keys"] = [0] * abi.KG_RSV_R, 0  # its assigned pod requests nothing but GPUs
    if spec.get("dev_alloc"):
        r["dev_alloc"] = _tab(spec["dev_alloc"])
        r["dev_allocated"] = _tab(spec.get("dev_allocated"))
    return [r]


def _build(case, pod_specs):
    """(cfg, true node table, reservation dicts, pods): node 0 as the case describes it, node 1 without GPUs."""
    cfg, _, p, _, _, T, _ = synth.cluster5(2, max(1, len(pod_specs)), seed_config=7, rsv_frac=0.0, raw=True,
                                           usage="u01")
    T = {k: np.array(v, copy=True) for k, v in T.items()}
    T["numa_policy"][:] = abi.KG_NUMA_NONE
    T["dev_minors"] = np.array([len(case["node"]["minors"]), -1], np.int32)
    tot = np.zeros((2, abi.KG_DEV_R, abi.KG_DEV_MINORS), np.int64)
    used = np.zeros_like(tot)
    tot[0], used[0] = _tab(case["node"]["minors"]), _tab(case.get("used"))
    T["dev_total"], T["dev_used"], T["dev_free"] = tot, used, np.maximum(tot - used, 0)
    T["dev_topo"][:] = np.uint64((1 << 64) - 1)  # no GPU topology reported
    T["dev_part"][:] = 0
    T["dev_numa"][:] = np.uint32(0xFFFFFFFF)
    resv = _rsv_dict(case.get("reservation"))
    p = {k: np.array(v, copy=True) for k, v in p.items()}
    n = abi.table_len(p)
    p["flags"] = ((p["flags"] & ~np.uint32(abi.KG_POD_NUMA_SKIP | abi.KG_POD_RSV_REQUIRED | abi.KG_POD_CPU_BIND))
                  | abi.KG_POD_HAS_CPU | abi.KG_POD_HAS_MEM).astype(np.uint32)
    p["quota"][:] = -1
    p["dev_req"][:] = 0
    p["dev_keys"][:] = 0
    p["dev_count"][:] = 0
    p["dev_flags"][:] = 0
    for j, s in enumerate(pod_specs):
        p["req_cpu"][j] = p["nz_cpu"][j] = int(s.get("cpu_m", 100))
        p["req_mem"][j] = p["nz_mem"][j] = int(s.get("mem", 1)) * GI
        for k in ("req_eph", "sc_req0", "sc_req1"):
            p[k][j] = 0
        p["rsv_class"][j] = int(s.get("cls", -1))
        g = s.get("gpu")
        if g:
            req = {GPU_CORE: g["core"] * g.get("count", 1)}
            if "ratio" in g:
                req[GPU_MEMORY_RATIO] = g["ratio"] * g.get("count", 1)
            if "mem" in g:
                req[GPU_MEMORY] = g["mem"] * GI
            vec, keys, cnt, shared = decode.gpu_requirements(req)
            p["dev_req"][j], p["dev_keys"][j], p["dev_count"][j] = vec, keys, cnt
            p["dev_flags"][j] = abi.KG_GPU_POD_SHARED if shared else 0
    assert n >= len(pod_specs)
    return cfg, T, resv, p


def _restore(T, resv):
    t, views, infos, devs = decode.reservation_restore(T, resv)
    return t, abi.Reservations(views, infos, devs, decode.reservation_gpu_raw(T, resv))


def _mask(ms):
    return sum(1 << int(m) for m in ms)


def _info_of(rsv_tab, cls):
    """The reservation's copy in the pod's view on node 0 (-1 = the pod's class has no view)."""
    for v in range(rsv_tab.n_views):
        w = rsv_tab.views[v]
        if w.node == 0 and w.cls == cls and w.count:
            return w.first
    return -1


def _check_info(infos, x, want):
    if x < 0 or want is None:
        return
    assert [int(a) for a in infos[x].allocated[:2]] == [want["allocated"][0], want["allocated"][1] * GI]
    assert infos[x].allocated_pods == want["allocated_pods"]


def _devs(r):
    return [np.ctypeslib.as_array(r.devs[x].free).copy() for x in range(r.n_devs)]


NODE_COLS = ("req_cpu", "req_mem", "req_eph", "sc_req0", "sc_req1", "nz_cpu", "nz_mem", "num_pods", "dev_free")


def _after_unreserve(T, resv, p, j, rec):
    """The snapshot columns after the pod's Reserve + Unreserve as the restore sees them: NodeInfo as before, the
    reservation it joined back to its Allocated (SubtractWithNonNegativeResult) with the keys the pod's requests added
    (quotav1.Add then Subtract keep them: an explicit zero's NonZeroRequested is 0, no longer the default)."""
    r2 = [dict(r) for r in resv]
    x = int(rec.rsv_rid)
    if x >= 0:
        alloc = r2[x]["allocatable"]
        names = sum(1 << k for k in range(abi.KG_RSV_R) if alloc[k] != 0)
        f = int(p["flags"][j])
        keys_m = (1 if (f & abi.KG_POD_HAS_CPU) and (names & 1) else 0) | (2 if (f & abi.KG_POD_HAS_MEM) and (names & 2) else 0)
        keys0 = int(r2[x].get("allocated_keys", 3)) if r2[x].get("allocated") is not None else 0
        r2[x]["allocated"] = list(r2[x].get("allocated") or [0] * abi.KG_RSV_R)
        r2[x]["allocated_keys"] = keys0 | keys_m
    return decode.reservation_restore(T, r2)[0]


def _run(case, device):
    from koordinator_amd import engine  # noqa: F401  (the GPU leg)
    if "want_parts" in case:  # RestoreReservation's reusableAlloc and merged tables for the one matched reservation
        (alloc, _), (allocated, _), (rem, _), _ = decode.dev_reservation_parts(_rsv_dict(case["reservation"])[0])
        w = case["want_parts"]
        assert np.array_equal(alloc, _tab(w["allocatable"])) and np.array_equal(allocated, _tab(w["allocated"]))
        assert np.array_equal(rem, _tab(w["remained"]))
        assert np.array_equal(alloc, _tab(w["merged_matched_allocatable"]))
        assert np.array_equal(allocated, _tab(w["merged_matched_allocated"]))
    if "unreserve_only" in case:
        u = case["unreserve_only"]
        specs = [{"cls": -1, "gpu": u["gpu"]}]
        cfg, T, resv, p = _build(case, specs)
        kc = cfg.kg_config()
        kc.plugins &= ~abi.KG_PLUGIN_QUOTA
        t, rsv = _restore(T, resv)
        rec = abi.KgReserveRecord()
        rec.numa_zone, rec.rsv_rid, rec.gpu_minors = -1, -1, _mask(u["minors"])
        want_free = _tab(u["want_free"])
        if device:
            ctx = engine.Context(0)
            try:
                snap = engine.Snapshot(ctx, kc, t)
                batch = engine.PodBatch(ctx, p)
                engine.unreserve(snap, batch, 0, 0, rec)
                got = snap.read_state()["dev_free"][0]
            finally:
                ctx.close()
        else:
            st = oracle_lib.OracleState(kc, t)
            st.unreserve(0, p, 0, rec)
            got = st.dev_free()[0]
        assert np.array_equal(got, want_free)
        return
    specs = case["pods"]
    cfg, T, resv, p = _build(case, specs)
    kc = cfg.kg_config()
    kc.plugins &= ~abi.KG_PLUGIN_QUOTA
    t, rsv = _restore(T, resv)
    for j, s in enumerate(specs):
        st = oracle_lib.OracleState(kc, t)
        sess = oracle_lib.ExtSession(st, None, rsv)
        assert sess.filter(0, p, j) == 0, s["name"]
        before = st.table()
        ok, rec = sess.reserve(0, p, j)
        assert ok, s["name"]
        if "want_minors" in s:
            assert rec.gpu_minors == _mask(s["want_minors"]), (s["name"], rec.gpu_minors)
        assert (rec.rsv_rid >= 0) == s["want_nominated"], s["name"]
        x = _info_of(rsv, int(s["cls"]))
        mid = sess.read_reservations()
        _check_info(mid.infos, x, s.get("want_info_after_reserve"))
        if "want_rsv_allocated_after" in s:
            # the reservation's tables after the Reserve: the restore of the reference's expected bookkeeping
            r2 = [dict(r) for r in resv]
            r2[0]["dev_allocated"] = _tab(s["want_rsv_allocated_after"])
            T2 = {k: np.array(v, copy=True) for k, v in T.items()}
            T2["dev_used"][0] += _tab(s["want_rsv_allocated_after"]) - _tab(case["reservation"]["dev_allocated"])
            T2["dev_free"][0] = np.maximum(T2["dev_total"][0] - T2["dev_used"][0], 0)
            _, want2 = _restore(T2, r2)
            for a, b in zip(_devs(mid), _devs(want2)):
                assert np.array_equal(a, b), s["name"]
        drec = None
        if device:
            ctx = engine.Context(0)
            try:
                snap = engine.Snapshot(ctx, kc, t)
                snap.upload_reservations(rsv)
                batch = engine.PodBatch(ctx, p)
                drec = engine.reserve(snap, batch, j, 0)
                for f in ("numa_zone", "gpu_minors", "rsv_rid", "flags"):
                    assert getattr(drec, f) == getattr(rec, f), (s["name"], f)
                dmid = snap.read_reservations(rsv)
                _check_info(dmid.infos, x, s.get("want_info_after_reserve"))
                for a, b in zip(_devs(dmid), _devs(mid)):
                    assert np.array_equal(a, b), s["name"]
                assert np.array_equal(snap.read_state()["dev_free"], st.table()["dev_free"])
                engine.unreserve(snap, batch, j, 0, drec)
                dend = snap.read_reservations(rsv)
                _check_info(dend.infos, x, s.get("want_info_after_unreserve"))
                for a, b in zip(_devs(dend), _devs(rsv)):
                    assert np.array_equal(a, b), s["name"]
                want_end, got_end = _after_unreserve(T, resv, p, j, rec), snap.read_state()
                for c in NODE_COLS:
                    assert np.array_equal(got_end[c], want_end[c]), (s["name"], c)
            finally:
                ctx.close()
        assert sess.unreserve(0, p, j, rec)
        end = sess.read_reservations()
        _check_info(end.infos, x, s.get("want_info_after_unreserve"))
        for a, b in zip(_devs(end), _devs(rsv)):
            assert np.array_equal(a, b), s["name"]
        want_end, got_end = _after_unreserve(T, resv, p, j, rec), st.table()
        for c in NODE_COLS:
            assert np.array_equal(got_end[c], want_end[c]), (s["name"], c)
        if rec.rsv_rid < 0:  # nothing but the pod changed: the state is the one before
            oracle_lib.assert_state_restored(before, got_end)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_unreserve_kat_oracle(case):
    _run(case, device=False)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_unreserve_kat_device(case):
    _run(case, device=True)
