"""Reservation matching (koordinator_amd/rsvmatch.py) against the reference's owner-match and
reservation-affinity tests (tests/golden/rsvmatch_kat.json), plus the owner-match classes it hands the device."""
import json
import os

import pytest

from koordinator_amd import rsvmatch

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "rsvmatch_kat.json")) as f:
    K = json.load(f)


@pytest.mark.parametrize("c", K["owners"], ids=[c["name"] for c in K["owners"]])
def test_match_reservation_owners(c):
    assert rsvmatch.match_owners(c["pod"], c["owners"]) == c["want"]


@pytest.mark.parametrize("c", K["affinity"], ids=[c["name"] for c in K["affinity"]])
def test_before_prefilter_with_reservation_affinity(c):
    nodes = {c["node"]["metadata"]["name"]: c["node"]}
    cls, rsv_cls, sets = rsvmatch.match_classes([c["pod"]], [c["requests"]], c["reservations"], nodes)
    assert (cls[0] >= 0) == c["want_restored"]


def test_classes_group_equal_matched_sets():
    owners_a = [{"labelSelector": {"matchLabels": {"app": "a"}}}]
    owners_ab = [{"labelSelector": {"matchExpressions": [{"key": "app", "operator": "In", "values": ["a", "b"]}]}}]
    rs = [{"metadata": {"name": "r0"}, "spec": {"owners": owners_a}, "status": {"nodeName": "n0"}},
          {"metadata": {"name": "r1"}, "spec": {"owners": owners_ab}, "status": {"nodeName": "n1"}},
          {"metadata": {"name": "r2"}, "spec": {"owners": None}, "status": {"nodeName": "n1"}}]
    pods = [{"metadata": {"labels": {"app": a}}} for a in ("a", "b", "c", "a")]
    cls, rsv_cls, sets = rsvmatch.match_classes(pods, [{}] * 4, rs, {})
    assert cls == [0, 1, -1, 0]
    assert sets == [(0, 1), (1,)]
    assert rsv_cls == [[0], [0, 1], []]
    ignored = {"metadata": {"labels": {rsvmatch.LABEL_RESERVATION_IGNORED: "true"}}}
    assert rsvmatch.match_classes([ignored], [{}], rs, {})[2] == [(0, 1, 2)]  # ignored: every reservation


def test_exact_match_quirk():
    # a resource in neither list ends the check as a match (apis/extension/reservation.go:263-267)
    assert rsvmatch.exact_match({"cpu": "4"}, {"cpu": "8"}, ["nvidia.com/gpu", "cpu"])
    assert not rsvmatch.exact_match({"cpu": "4"}, {"cpu": "8"}, ["cpu"])
    assert rsvmatch.exact_match({"cpu": "8"}, {"cpu": "8000m"}, ["cpu"])


def test_restore_with_shared_reservations_matches_per_pod_restore():
    """A reservation matched by several classes: the shared-class restore gives every pod the same Filter /
    Score results as restoring that pod alone (one class per pod), on the oracle."""
    import numpy as np
    import oracle_lib
    from koordinator_amd import abi, decode, synth
    cfg, nodes, pods, quotas, rsv = synth.cluster5(60, 12, seed_config=91, rsv_frac=0.0)
    kc = cfg.kg_config()
    kc.plugins &= ~abi.KG_PLUGIN_QUOTA
    GI = 1 << 30
    resv = [dict(node=n, cls=None, allocatable=[4000, 8 * GI, 0, 0, 0], allocated=None, reserved=None, allocated_pods=0,
                 policy=abi.KG_RSV_DEFAULT, order=0, allocate_once=True, max_pods=-1) for n in (3, 3, 7, 11)]
    sets = [(0, 1), (1, 2, 3), (0, 1)]  # matched sets of three pod classes
    pod_cls = [0, 1, 2, 0, -1, 1, 2, 2, -1, 0, 1, 0]
    for x, r in enumerate(resv):
        r["cls"] = [c for c, st in enumerate(sets) if x in st]
    pods["rsv_class"] = np.array(pod_cls, np.int32)
    t, views, infos, devs = decode.reservation_restore(nodes, resv)
    shared = oracle_lib.ext_verify(kc, t, pods, None, abi.Reservations(views, infos, devs))
    for j, c in enumerate(pod_cls):
        one = [dict(r, cls=[0] if (c >= 0 and x in sets[c]) else []) for x, r in enumerate(resv)]
        pj = abi.take(pods, [j])
        pj["rsv_class"] = np.array([0 if c >= 0 else -1], np.int32)
        t1, v1, i1, d1 = decode.reservation_restore(nodes, one)
        alone = oracle_lib.ext_verify(kc, t1, pj, None, abi.Reservations(v1, i1, d1))
        assert np.array_equal(shared.status[j], alone.status[0])
        assert np.array_equal(shared.total[j], alone.total[0])
