"""Known answers of the reservation matching restatement (koordinator_amd/rsvmatch.py), transcribed from
  /root/reference/pkg/util/reservation/reservation_test.go:258-445 TestMatchReservationOwners and
  /root/reference/pkg/scheduler/plugins/reservation/transformer_test.go:743-1040
      TestBeforePreFilterWithReservationAffinity (restored == some reservation matched).
Writes rsvmatch_kat.json next to this file. Objects are the tests' Go literals written as Kubernetes JSON."""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def owners_cases():
    pod1 = {"metadata": {"name": "test-pod-1", "namespace": "test", "labels": {"aaa": "bbb", "ccc": "ddd"}}}
    return [
        {"name": "no owner to match", "line": 268, "pod": {}, "owners": None, "want": False},
        {"name": "match objRef", "line": 280, "pod": {"metadata": {"name": "test-pod-0", "namespace": "test"}},
         "owners": [{"object": {"name": "test-pod-0", "namespace": "test"}}], "want": True},
        {"name": "match controllerRef", "line": 304,
         "pod": {"metadata": {"name": "test-sts-0-0", "namespace": "test", "ownerReferences": [
             {"name": "test-sts-0", "controller": True, "kind": "StatefulSet", "apiVersion": "apps/v1"}]}},
         "owners": [{"controller": {"name": "test-sts-0", "controller": True, "namespace": "test"}}], "want": True},
        {"name": "match labels", "line": 337, "pod": pod1,
         "owners": [{"labelSelector": {"matchLabels": {"aaa": "bbb"}}}], "want": True},
        {"name": "fail on one term of owner spec", "line": 365, "pod": pod1,
         "owners": [{"object": {"name": "test-pod-2"}, "labelSelector": {"matchLabels": {"aaa": "bbb", "xxx": "yyy"}}}],
         "want": False},
        {"name": "match one of owner specs", "line": 397,
         "pod": {"metadata": {"name": "test-pod-2", "namespace": "test", "labels": {"aaa": "bbb", "ccc": "ddd"}}},
         "owners": [{"object": {"name": "test-pod-0", "namespace": "test"}},
                    {"labelSelector": {"matchLabels": {"aaa": "bbb"}}}], "want": True},
    ]


def affinity_cases():
    """transformer_test.go:743-1040: node1 (labels test=true); reservation8C16G (labels reservation-a=true,
    owners label test-reservation=true, allocatable 8 cpu / 16Gi); unschedulable-reservation (labels
    reservation-b=true, spec.unschedulable); the test pod (labels test-reservation=true, requests 4 cpu / 8Gi)."""
    node = {"metadata": {"name": "node1", "labels": {"test": "true"}}}
    owners = [{"labelSelector": {"matchLabels": {"test-reservation": "true"}}}]
    matched = {"metadata": {"name": "reservation8C16G", "labels": {"reservation-a": "true"}},
               "spec": {"owners": owners}, "status": {"nodeName": "node1", "allocatable": {"cpu": "8", "memory": "16Gi"}}}
    unsched = {"metadata": {"name": "unschedulable-reservation", "labels": {"reservation-b": "true"}},
               "spec": {"owners": owners, "unschedulable": True},
               "status": {"nodeName": "node1", "allocatable": {"cpu": "8", "memory": "16Gi"}}}

    def term(key, value):
        return {"requiredDuringSchedulingIgnoredDuringExecution": {"reservationSelectorTerms": [
            {"matchExpressions": [{"key": key, "operator": "In", "values": [value]}]}]}}

    tol = [{"key": "node.kubernetes.io/unschedulable", "operator": "Exists", "effect": "NoSchedule"}]
    cases = [
        ("pod has no reservation affinity", 857, None, None, False, True),
        ("pod has reservation affinity and matched", 861, term("reservation-a", "true"), None, False, True),
        ("pod has reservation affinity but failed to match", 880, term("reservation-a", "false"), None, False, False),
        ("pod has reservation affinity but failed to exact match", 899, term("reservation-a", "false"), ["cpu"], False,
         False),
        ("pod specifies a reservation name and matched", 923, {"name": "reservation8C16G"}, None, False, True),
        ("pod specifies a reservation name but failed to match", 930, {"name": "not-reservation8C16G"}, None, False,
         False),
        ("pod specifies a reservation name but failed to exact match", 937, {"name": "reservation8C16G"}, ["cpu"],
         False, False),
        ("pod matches unschedulable reservation without toleration", 949, term("reservation-b", "true"), None, True,
         False),
        ("pod matches unschedulable reservation with toleration", 970, dict(term("reservation-b", "true"),
                                                                           tolerations=tol), None, True, True),
    ]
    out = []
    for name, line, aff, exact, use_unsched, want in cases:
        ann = {}
        if aff is not None:
            ann["scheduling.koordinator.sh/reservation-affinity"] = json.dumps(aff)
        if exact is not None:
            ann["scheduling.koordinator.sh/exact-match-reservation"] = json.dumps({"resourceNames": exact})
        pod = {"metadata": {"labels": {"test-reservation": "true"}, "annotations": ann}}
        out.append({"name": name, "line": line, "pod": pod, "requests": {"cpu": "4", "memory": "8Gi"},
                    "reservations": [matched] + ([unsched] if use_unsched else []), "node": node,
                    "want_restored": want})
    return out


def main():
    with open(os.path.join(HERE, "rsvmatch_kat.json"), "w") as f:
        json.dump({"owners": owners_cases(), "affinity": affinity_cases()}, f, indent=1)


if __name__ == "__main__":
    main()
