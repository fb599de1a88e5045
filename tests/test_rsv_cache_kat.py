"""f1: the reservation cache (cluster.ReservationCache) against the reference's own tests of reservationCache
(pkg/scheduler/plugins/reservation/cache_test.go) and ReservationInfo (frameworkext/reservation_info.go).

Each test restates one Go test's scenario on Reservation / Pod dicts and checks the same expectations:
ResourceNames, Allocatable, Allocated (nil until the first assigned pod, zero-valued keys after the last one
leaves), AssignedPods, the matchable / allocated node sets, ListAllNodes, ForEachMatchableReservationOnNode and
ListAvailableReservationInfosOnNode. Quantities are compared as exact values (Fraction) the way
resource.Quantity compares them."""
from fractions import Fraction

from koordinator_amd.cluster import ReservationCache
from koordinator_amd.config import bench_profile

GI = 1 << 30


def _cache():
    return ReservationCache(bench_profile(numa=False))


def _rsv(uid, name, node, cpu, mem, phase="Available", allocatable=True, allocated=None, allocate_once=None):
    spec = {"template": {"spec": {"containers": [{"resources": {"requests": {"cpu": cpu, "memory": mem}}}]}}}
    if allocate_once is not None:
        spec["allocateOnce"] = allocate_once
    status = {"nodeName": node}
    if phase:
        status["phase"] = phase
    if allocatable:
        status["allocatable"] = {"cpu": cpu, "memory": mem}
    if allocated:
        status["allocated"] = allocated
    return {"metadata": {"uid": uid, "name": name}, "spec": spec, "status": status}


def _pod(uid, name, cpu, mem):
    return {"metadata": {"uid": uid, "name": name, "namespace": "default"},
            "spec": {"containers": [{"resources": {"requests": {"cpu": cpu, "memory": mem}}}]}}


def q(v):
    return Fraction(v)


def test_cache_update_reservation():
    """TestCacheUpdateReservation (cache_test.go:41-110): status.allocated is not Allocated (nil without pods);
    a repeated update leaves the info as it was."""
    c = _cache()
    r = _rsv("u1", "test-reservation", "test-node-1", "4", "4Gi", allocated={"cpu": "2", "memory": "2Gi"})
    for _ in range(2):
        c.update_reservation(r)
        infos = c.list_available("test-node-1", True)
        assert len(infos) == 1
        ri = infos[0]
        assert ri.names == ["cpu", "memory"]
        assert ri.allocatable_rl == {"cpu": q(4), "memory": q(4 * GI)}
        assert ri.allocated_rl is None and ri.assigned == {}


def test_cache_delete_reservation():
    """TestCacheDeleteReservation (cache_test.go:112-174): a reservation without a phase (Allocatable from its
    template), then DeleteReservation removes it."""
    c = _cache()
    r = _rsv("u1", "test-reservation", "test-node-1", "4", "4Gi", phase="", allocated={"cpu": "2", "memory": "2Gi"})
    c.update_reservation(r)
    ri = c.get("u1")
    assert ri is not None
    assert ri.names == ["cpu", "memory"] and ri.allocatable_rl == {"cpu": q(4), "memory": q(4 * GI)}
    assert ri.allocated_rl is None and ri.assigned == {}
    c.delete_reservation(r)
    assert c.get("u1") is None


def test_cache_update_reservation_if_exists():
    """TestCacheUpdateReservationIfExists (cache_test.go:176-275)."""
    c = _cache()
    r = _rsv("u1", "test-reservation", "test-node-1", "4", "4Gi")
    c.update_reservation_if_exists(r)
    assert c.get("u1") is None  # not created
    c.update_reservation(r)
    assert c.get("u1") is not None and c.get("u1").phase == "Available"
    r2 = _rsv("u1", "test-reservation", "test-node-1", "4", "4Gi", phase="Succeeded",
              allocated={"cpu": "2", "memory": "2Gi"})
    c.update_reservation_if_exists(r2)
    assert c.get("u1").phase == "Succeeded"
    assert "u1" not in c.matchable_on_node.get("test-node-1", set())
    # matchable -> not matchable
    c2 = _cache()
    rr = _rsv("u2", "test-reservation-2", "test-node-2", "2", "0")
    rr["spec"]["template"]["spec"]["containers"][0]["resources"]["requests"] = {"cpu": "2"}
    rr["status"]["allocatable"] = {"cpu": "2"}
    c2.update_reservation(rr)
    assert "u2" in c2.matchable_on_node["test-node-2"]
    rr["status"]["phase"] = "Failed"
    c2.update_reservation_if_exists(rr)
    assert "u2" not in c2.matchable_on_node.get("test-node-2", set())


def test_cache_add_or_update_or_delete_pod():
    """TestCacheAddOrUpdateOrDeletePod (cache_test.go:277-396): Allocated = the pod's masked requests; an update
    within the same reservation keeps it; after deletePod Allocated is {cpu: 0, memory: 0} (not nil) and
    AssignedPods is empty."""
    c = _cache()
    r = _rsv("u1", "test-reservation", "test-node-1", "4000m", "4Gi", phase="",
             allocated={"cpu": "2000m", "memory": "2Gi"})
    c.update_reservation(r)
    assert c.get("u1") is not None
    pod = _pod("p1", "test-pod-1", "2000m", "2Gi")
    assert c.assume_pod("u1", pod)
    ri = c.get("u1")
    assert ri.names == ["cpu", "memory"] and ri.allocatable_rl == {"cpu": q(4), "memory": q(4 * GI)}
    assert ri.allocated_rl == {"cpu": q(2), "memory": q(2 * GI)}
    assert ri.assigned == {"p1": {"cpu": q(2), "memory": q(2 * GI)}}
    c.update_pod_in("u1", "u1", pod, pod)
    assert ri.allocated_rl == {"cpu": q(2), "memory": q(2 * GI)} and list(ri.assigned) == ["p1"]
    c.forget_pod("u1", pod)
    assert ri.allocated_rl == {"cpu": q(0), "memory": q(0)} and ri.assigned == {}
    assert ri.allocated == [0] * len(ri.allocated)


def test_cache_update_pod_across_reservations():
    """TestCacheUpdatePodAcrossReservations (cache_test.go:398-500)."""
    c = _cache()
    c.update_reservation(_rsv("u1", "test-reservation-1", "test-node-1", "4000m", "4Gi", phase=""))
    c.update_reservation(_rsv("u2", "test-reservation-2", "test-node-1", "2000m", "2Gi", phase=""))
    pod = _pod("p1", "test-pod-1", "2000m", "2Gi")
    c.assume_pod("u1", pod)
    assert list(c.get("u1").assigned) == ["p1"]
    c.update_pod_in("u1", "u2", pod, pod)
    assert c.get("u1").assigned == {} and list(c.get("u2").assigned) == ["p1"]
    c.update_pod_in("u2", "u2", pod, pod)
    assert list(c.get("u2").assigned) == ["p1"]


def test_cache_list_all_nodes():
    """TestCacheListAllNodes (cache_test.go:502-612)."""
    c = _cache()
    c.update_reservation(_rsv("u1", "test-reservation-1", "test-node-1", "4", "4Gi", allocate_once=False))
    c.update_reservation(_rsv("u2", "test-reservation-2", "test-node-2", "2", "2Gi", allocate_once=False))
    assert c.list_all_nodes(True) == ["test-node-1", "test-node-2"]
    assert c.list_all_nodes(False) == []  # no allocated pods yet
    c.assume_pod("u1", _pod("p", "test-pod", "1", "1Gi"))
    assert c.list_all_nodes(False) == ["test-node-1"]
    assert len(c.list_all_nodes(True)) == 2


def test_cache_for_each_matchable_reservation_on_node():
    """TestCacheForEachMatchableReservationOnNode (cache_test.go:614-699): a Failed reservation is not visited;
    returning False stops the walk."""
    c = _cache()
    c.update_reservation(_rsv("u1", "test-reservation-1", "test-node-1", "4", "4Gi"))
    c.update_reservation(_rsv("u2", "test-reservation-2", "test-node-1", "2", "2Gi", phase="Failed"))
    seen = []
    c.for_each_matchable("test-node-1", lambda ri: seen.append(ri.uid) or True)
    assert seen == ["u1"]
    seen = []
    c.for_each_matchable("test-node-1", lambda ri: seen.append(ri.uid) and False)
    assert len(seen) == 1


def test_cache_list_available_reservation_infos_on_node():
    """TestCacheListAvailableReservationInfosOnNode (cache_test.go:701-776)."""
    c = _cache()
    c.update_reservation(_rsv("u1", "test-reservation", "test-node-1", "4", "4Gi"))
    c.update_reservation(_rsv("u2", "test-reservation-failed", "test-node-1", "2", "2Gi", phase="Failed"))
    got = c.list_available("test-node-1", False)
    assert [ri.uid for ri in got] == ["u1"]
    assert len(c.list_available("test-node-1", True)) == 2


def test_allocated_masked_on_resource_name_change():
    """UpdateReservation (reservation_info.go:400-428): Allocated is re-masked by the new ResourceNames, and a pod
    removed afterwards subtracts its requests masked by the current names (SubtractWithNonNegativeResult keeps a
    zero for keys only in the subtrahend)."""
    import json
    from koordinator_amd.cluster import ANN_RESERVATION_RESTRICTED_OPTIONS
    c = _cache()
    r = _rsv("u1", "r", "n", "4", "4Gi", allocate_once=False)
    c.update_reservation(r)
    pod = _pod("p1", "p", "1", "1Gi")
    c.assume_pod("u1", pod)
    ri = c.get("u1")
    assert ri.allocated_rl == {"cpu": q(1), "memory": q(GI)} and ri.allocated_keys() == 3
    r2 = json.loads(json.dumps(r))
    r2["spec"]["allocatePolicy"] = "Restricted"
    r2["metadata"]["annotations"] = {ANN_RESERVATION_RESTRICTED_OPTIONS: json.dumps({"resources": ["cpu"]})}
    c.update_reservation(r2)
    assert ri.names == ["cpu"] and ri.allocated_rl == {"cpu": q(1)} and ri.allocated_keys() == 1
    c.forget_pod("u1", pod)
    assert ri.allocated_rl == {"cpu": q(0)}
    # a Restricted reservation whose options do not parse has a ParseError: not matchable
    r3 = json.loads(json.dumps(r2))
    r3["metadata"]["annotations"] = {ANN_RESERVATION_RESTRICTED_OPTIONS: "{bad"}
    c.update_reservation(r3)
    assert not ri.is_matchable() and "u1" not in c.matchable_on_node.get("n", set())


# ---- ElasticQuota handler (elasticquota/quota_handler_test.go) -------------------------------------------------
# The flat cache (cluster.QuotaCache: EnableCheckParentQuota off, one tree) restates the handler's per-quota part;
# the parent / tree-ID cases (MultiQuotaTree, runtime refresh up a quota tree) are outside it (parity unpinned).

def _quota(name, cpu, mem, deleting=False):
    md = {"name": name}
    if deleting:
        md["deletionTimestamp"] = "2024-01-01T00:00:00Z"
    return {"metadata": md, "spec": {"max": {"cpu": cpu, "memory": mem}, "min": {"cpu": "0", "memory": "0"}}}


def test_quota_add_ignores_deleting_quota():
    """TestPlugin_OnQuotaAddWithTreeID (quota_handler_test.go:43-50): quota "1" is added; a copy named "2" carrying a
    DeletionTimestamp is not (OnQuotaAdd, quota_handler.go:42-45); nor is an update of a deleting quota (:70-73)."""
    from koordinator_amd.cluster import QuotaCache
    c = QuotaCache(bench_profile(numa=False))
    c.on_quota(_quota("1", "0", "0"), add=True)
    assert "1" in c.index
    c.on_quota(_quota("2", "0", "0", deleting=True), add=True)
    assert "2" not in c.index
    c.on_quota(_quota("1", "8", "8Gi", deleting=True))
    assert c.max[c.index["1"]] == {"cpu": "0", "memory": "0"}
    # an Add of a quota already held does not overwrite it (:54-57); an Update does
    c.on_quota(_quota("1", "4", "4Gi"), add=True)
    assert c.max[c.index["1"]] == {"cpu": "0", "memory": "0"}
    c.on_quota(_quota("1", "4", "4Gi"))
    assert c.max[c.index["1"]] == {"cpu": "4", "memory": "4Gi"}
    # the default and system quotas are updated by an Add too (quota_handler.go:55)
    for name in ("koordinator-default-quota", "koordinator-system-quota"):
        c.on_quota(_quota(name, "1", "1Gi"), add=True)
        c.on_quota(_quota(name, "2", "2Gi"), add=True)
        assert c.max[c.index[name]] == {"cpu": "2", "memory": "2Gi"}


def test_quota_pod_used_flat():
    """TestPlugin_ReplaceQuotas's flat part (quota_handler_test.go:329-358): a pod labelled with a quota counts its
    request in that quota's used, another quota stays at zero."""
    from koordinator_amd.cluster import LABEL_QUOTA_NAME, QuotaCache
    c = QuotaCache(bench_profile(numa=False))
    c.on_quota(_quota("test1", "100", "200"), add=True)
    c.on_quota(_quota("test2", "200", "400"), add=True)
    pod = {"metadata": {"uid": "p", "name": "pod", "labels": {LABEL_QUOTA_NAME: "test1"}},
           "spec": {"nodeName": "n0", "containers": [{"resources": {"requests": {"cpu": "40", "memory": "100"}}}]},
           "status": {"phase": "Running"}}
    c.on_pod(None, pod)
    t = c.columns()
    assert list(t["used"][c.index["test1"]][:2]) == [40000, 100]
    assert list(t["used"][c.index["test2"]][:2]) == [0, 0]


def test_cache_reservation_node_move_walks_both_nodes():
    """updateReservation (cache.go:793-844) adds a moved reservation to its new node's sets and removes nothing from
    the old node's: ForEachMatchableReservationOnNode visits it on both nodes, and the restore inputs key each entry
    by the node walked, so the reservation is restored once per node (never twice on the new one)."""
    c = _cache()
    c.update_reservation(_rsv("u1", "r1", "node-a", "4", "4Gi"))
    c.update_reservation(_rsv("u1", "r1", "node-b", "4", "4Gi"))
    assert "u1" in c.matchable_on_node["node-a"] and "u1" in c.matchable_on_node["node-b"]
    index = {"node-a": 0, "node-b": 1}
    pairs = c.matchable_infos(index)
    assert [(n, ri.uid) for n, ri in pairs] == [("node-a", "u1"), ("node-b", "u1")]
    entries = c.restore_inputs(index)
    assert sorted(e["node"] for e in entries) == [0, 1]


def test_cache_delete_tombstone_without_node():
    """DeleteReservation clears the sets of the object's nodeName only (cache.go:893-918): a tombstone without one
    leaves the uid on the node, and the walk skips it instead of failing on the missing info."""
    c = _cache()
    c.update_reservation(_rsv("u1", "r1", "node-a", "4", "4Gi"))
    c.update_reservation(_rsv("u2", "r2", "node-a", "2", "2Gi"))
    tomb = _rsv("u1", "r1", "", "4", "4Gi")
    c.delete_reservation(tomb)
    assert c.get("u1") is None
    seen = []
    c.for_each_matchable("node-a", lambda ri: seen.append(ri.uid) or True)
    assert seen == ["u2"]
    assert [e["uid"] for e in c.restore_inputs({"node-a": 0})] == ["u2"]
