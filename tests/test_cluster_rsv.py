"""f1 remainder: reservation and ElasticQuota events in the host cache layer (cluster.ReservationCache /
QuotaCache): the reservation cache's writers (reservation/cache.go:785-1104: updateReservation,
DeleteReservation, addPod / updatePod / deletePod of pods allocated to a reservation, IsMatchable) and the
quota handler's (elasticquota/quota_handler.go: quota add / update / delete, pod used), checked against the
restore / quota tables built directly from the same objects."""
import json

import numpy as np

from koordinator_amd import abi, decode
from koordinator_amd.cluster import ANN_RESERVATION_ALLOCATED, ClusterState, LABEL_QUOTA_NAME
from koordinator_amd.config import bench_profile

GI = 1 << 30


def _node(name, cpu="32", mem="64Gi"):
    return {"metadata": {"name": name, "labels": {}},
            "status": {"allocatable": {"cpu": cpu, "memory": mem, "pods": "110"}}}


def _pod(name, node="", cpu="1", mem="2Gi", labels=None, rsv=None):
    ann = {}
    if rsv is not None:
        ann[ANN_RESERVATION_ALLOCATED] = json.dumps({"uid": rsv, "name": rsv})
    return {"metadata": {"name": name, "namespace": "default", "uid": "uid-" + name, "labels": labels or {},
                         "annotations": ann},
            "spec": {"nodeName": node, "containers": [{"resources": {"requests": {"cpu": cpu, "memory": mem}}}]},
            "status": {"phase": "Running"}}


def _rsv(name, node, cpu="4", mem="8Gi", phase="Available", allocate_once=True, owners=None):
    return {"metadata": {"name": name, "uid": name, "labels": {}},
            "spec": {"owners": owners if owners is not None else [{"labelSelector": {"matchLabels": {"app": "a"}}}],
                     "allocateOnce": allocate_once},
            "status": {"phase": phase, "nodeName": node, "allocatable": {"cpu": cpu, "memory": mem}}}


def _state():
    return ClusterState(bench_profile(numa=False), [_node("n0"), _node("n1"), _node("n2")])


def test_reservation_events_restore_views():
    st = _state()
    g0 = st.generation
    st.on_reservation(_rsv("r1", "n1", allocate_once=False))
    assert list(st.rsv_rows_since(g0)) == [1]
    assert st.req[1][0] == 4000  # the reserve pod counts in NodeInfo
    pending = [_pod("p-a", labels={"app": "a"}), _pod("p-b", labels={"app": "b"})]
    cls, t, rsv = st.reservation_restore(pending)
    assert list(cls) == [0, -1]
    assert rsv.n_views == 1 and rsv.views[0].node == 1 and rsv.views[0].count == 1
    assert rsv.views[0].req[0] == 0  # the matched reserve pod is removed from the restored Requested
    # a pod allocated to the reservation: Allocated grows, the default view gives back the double count
    st.on_pod_add(_pod("p-in", node="n1", cpu="1", labels={"app": "a"}, rsv="r1"))
    ri = st.reservations.infos["r1"]
    assert ri.allocated[0] == 1000 and ri.allocated[1] == 2 * GI and ri.matchable()
    cls, t, rsv = st.reservation_restore(pending)
    assert t["req_cpu"][1] == 4000  # 4000 reserve + 1000 pod - 1000 (unmatched: its allocated counted once)
    v = rsv.views[0]
    assert v.req[0] == 1000 and v.r_allocated[0] == 1000
    want_t, want_views, _, _ = decode.reservation_restore(st.table(), [dict(
        node=1, cls=[0], allocatable=[4000, 8 * GI, 0, 0, 0], allocated=[1000, 2 * GI, 0, 0, 0], reserved=None,
        allocated_pods=1, policy=abi.KG_RSV_DEFAULT, order=0, allocate_once=False, max_pods=-1, names=3)])
    assert np.array_equal(t["req_cpu"], want_t["req_cpu"]) and want_views[0]["req"] == list(v.req)
    # the pod leaves: allocated back to zero
    st.on_pod_delete(_pod("p-in", node="n1", rsv="r1"))
    assert st.reservations.infos["r1"].allocated == [0] * abi.KG_RSV_R
    st.on_reservation_delete(_rsv("r1", "n1"))
    assert st.req[1][0] == 0
    assert st.reservation_restore(pending)[2].n_views == 0


def test_allocate_once_reservation_stops_matching():
    st = _state()
    st.on_reservation(_rsv("r2", "n2"))  # allocateOnce default
    st.on_pod_add(_pod("p-in", node="n2", labels={"app": "a"}, rsv="r2"))
    assert not st.reservations.infos["r2"].matchable()  # IsMatchable: allocate-once with an assigned pod
    # matchableOnNode is refreshed by reservation events only (cache.go:1020-1045 addPods leaves it): the restore still
    # visits r2 (FilterNominateReservation, plugin.go:1197, is what refuses it) until its status update
    assert "r2" in st.reservations.matchable_on_node["n2"]
    st.on_reservation(_rsv("r2", "n2", phase="Succeeded"))
    assert "n2" not in st.reservations.matchable_on_node
    cls, _, rsv = st.reservation_restore([_pod("p-a", labels={"app": "a"})])
    assert list(cls) == [-1] and rsv.n_views == 0
    assert st.req[2][0] == 1000  # the reserve pod left NodeInfo, the assigned pod stays


def test_pod_moves_between_reservations():
    st = _state()
    st.on_reservation(_rsv("ra", "n0", allocate_once=False))
    st.on_reservation(_rsv("rb", "n0", allocate_once=False))
    old = _pod("p", node="n0", labels={"app": "a"}, rsv="ra")
    st.on_pod_add(old)
    new = _pod("p", node="n0", labels={"app": "a"}, rsv="rb")
    st.on_pod_update(old, new)
    assert st.reservations.infos["ra"].allocated[0] == 0 and st.reservations.infos["rb"].allocated[0] == 1000


def test_quota_events():
    st = _state()
    q = {"metadata": {"name": "q1"}, "spec": {"max": {"cpu": "10", "memory": "20Gi"}, "min": {"cpu": "4", "memory": "8Gi"}}}
    st.on_quota(q)
    st.on_pod_add(_pod("x", node="n0", cpu="2", labels={LABEL_QUOTA_NAME: "q1"}))
    st.on_pod_add(_pod("y", node="n1", cpu="1", labels={LABEL_QUOTA_NAME: "q1",
                                                        "quota.scheduling.koordinator.sh/preemptible": "false"}))
    st.on_pod_add(_pod("z", node="", cpu="8", labels={LABEL_QUOTA_NAME: "q1"}))  # pending: not used yet
    t = st.quotas.columns()
    assert list(t["used_limit"][0][:2]) == [10000, 20 * GI] and t["limit_keys"][0] == 0b11
    assert list(t["used"][0][:2]) == [3000, 4 * GI] and list(t["np_used"][0][:2]) == [1000, 2 * GI]
    st.on_pod_delete(_pod("x", node="n0", labels={LABEL_QUOTA_NAME: "q1"}))
    assert st.quotas.columns()["used"][0][0] == 1000
    st.on_quota({"metadata": {"name": "q1"}, "spec": {"max": {"cpu": "12"}}})
    assert st.quotas.columns()["limit_keys"][0] == 0b01
    st.on_quota_delete("q1")
    assert st.quotas.columns()["limit_keys"][0] == 0


def test_restricted_resources_kat():
    """TestGetReservationRestrictedResources (util/reservation/reservation_test.go:997-1042), through the
    annotation NewReservationInfo reads (frameworkext/reservation_info.go:99-106)."""
    from koordinator_amd.cluster import ANN_RESERVATION_RESTRICTED_OPTIONS, restricted_resources
    names = ["cpu", "memory"]
    cases = [(None, ["cpu", "memory"]), (["cpu", "memory"], ["cpu", "memory"]), (["cpu"], ["cpu"]), ([], ["cpu", "memory"])]
    for opt, want in cases:
        ann = {} if opt is None else {ANN_RESERVATION_RESTRICTED_OPTIONS: json.dumps({"resources": opt})}
        assert restricted_resources(names, ann) == want
    # an annotation that does not parse keeps every name (the parse error is recorded, names unchanged)
    assert restricted_resources(names, {ANN_RESERVATION_RESTRICTED_OPTIONS: "{bad"}) == names


def test_restricted_reservation_masks_allocated():
    """A Restricted reservation restricted to cpu: Allocated = Mask(requests, [cpu]) and the restore's names
    bitmask carries cpu only (reservation_info.go:92-107)."""
    from koordinator_amd.cluster import ANN_RESERVATION_RESTRICTED_OPTIONS
    st = _state()
    r = _rsv("r3", "n0", allocate_once=False)
    r["spec"]["allocatePolicy"] = "Restricted"
    r["metadata"]["annotations"] = {ANN_RESERVATION_RESTRICTED_OPTIONS: json.dumps({"resources": ["cpu"]})}
    st.on_reservation(r)
    ri = st.reservations.infos["r3"]
    assert ri.names == ["cpu"]
    st.on_pod_add(_pod("p-in", node="n0", cpu="1", mem="2Gi", labels={"app": "a"}, rsv="r3"))
    assert ri.allocated[0] == 1000 and ri.allocated[1] == 0
    _, _, rsv = st.reservation_restore([_pod("p-a", labels={"app": "a"})])
    assert rsv.n_views == 1
    # the plain variant (no annotation) keeps both names
    r2 = _rsv("r4", "n1", allocate_once=False)
    r2["spec"]["allocatePolicy"] = "Restricted"
    st.on_reservation(r2)
    assert st.reservations.infos["r4"].names == ["cpu", "memory"]
