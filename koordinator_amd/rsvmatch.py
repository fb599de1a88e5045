"""Reservation matching: which reservations a pending pod may allocate from.

Host restatement of the Reservation transformer's per-(pod, reservation) decision
(reservation/transformer.go:147-350 prepareMatchReservationStateForNormalPod, :637-681
checkReservationMatchedOrIgnored) and the helpers it calls:
  * owners: util/reservation/reservation.go:416-503 (ReservationOwnerMatcher.Match, MatchObjectRef,
    MatchReservationControllerReference, MatchLabels) — DNF of ObjectReference / ControllerReference /
    LabelSelector;
  * reservation affinity: reservation.go:520-624 (GetRequiredReservationAffinity, MatchAffinity,
    FindMatchingUntoleratedTaint, TolerateUnschedulable) over the reservation's labels merged onto the node's
    (frameworkext/reservation_info.go:330-358, OmitNodeLabelsForReservation off);
  * apis/extension/reservation.go: IsReservationIgnored (:111), GetReservationAffinity (:171),
    ExactMatchReservation (:256-276).

The result feeds the device path as owner-match classes: pods whose matched-reservation sets are equal form one
class (kg_pod_columns.rsv_class); each reservation lists the classes that match it, and the restore
(decode.reservation_restore) builds one view per (class, node). Objects are plain dicts shaped like the
Kubernetes JSON (metadata / spec / status)."""
from __future__ import annotations

import json
from typing import Dict, List, Optional, Sequence, Tuple

from .decode import parse_quantity

ANN_RESERVATION_AFFINITY = "scheduling.koordinator.sh/reservation-affinity"
ANN_EXACT_MATCH = "scheduling.koordinator.sh/exact-match-reservation"
LABEL_RESERVATION_IGNORED = "scheduling.koordinator.sh/reservation-ignored"
TAINT_NODE_UNSCHEDULABLE = "node.kubernetes.io/unschedulable"


# ---- label selectors (k8s.io/apimachinery labels, metav1.LabelSelectorAsSelector) --------------------------

def label_selector_matches(sel: Optional[dict], labels: Optional[dict]) -> bool:
    """metav1.LabelSelector: matchLabels AND matchExpressions (In / NotIn / Exists / DoesNotExist). An empty
    selector matches everything; None (no selector) is handled by the callers."""
    labels = labels or {}
    for k, v in (sel.get("matchLabels") or {}).items():
        if labels.get(k) != v:
            return False
    for req in sel.get("matchExpressions") or []:
        k, op, vals = req["key"], req["operator"], req.get("values") or []
        has = k in labels
        if op == "In" and not (has and labels[k] in vals):
            return False
        if op == "NotIn" and has and labels[k] in vals:
            return False
        if op == "Exists" and not has:
            return False
        if op == "DoesNotExist" and has:
            return False
    return True


def _node_requirement(req: dict, labels: dict) -> bool:
    """v1.NodeSelectorRequirement over labels (nodeaffinity: In, NotIn, Exists, DoesNotExist, Gt, Lt)."""
    k, op, vals = req["key"], req["operator"], req.get("values") or []
    has = k in labels
    if op == "In":
        return has and labels[k] in vals
    if op == "NotIn":
        return not has or labels[k] not in vals
    if op == "Exists":
        return has
    if op == "DoesNotExist":
        return not has
    if op in ("Gt", "Lt"):
        if not has or len(vals) != 1:
            return False
        try:
            a, b = int(labels[k]), int(vals[0])
        except ValueError:
            return False
        return a > b if op == "Gt" else a < b
    return False


def node_selector_matches(terms: Sequence[dict], labels: dict, name: str) -> bool:
    """nodeaffinity.NodeSelector.Match: terms ORed; a term's matchExpressions (labels) and matchFields
    (metadata.name) ANDed; a term with neither matches nothing."""
    for term in terms:
        exprs, fields = term.get("matchExpressions") or [], term.get("matchFields") or []
        if not exprs and not fields:
            continue
        if all(_node_requirement(r, labels) for r in exprs) and \
                all(_node_requirement(r, {"metadata.name": name}) for r in fields):
            return True
    return False


# ---- owners (util/reservation/reservation.go:416-503) -------------------------------------------------------

def match_object_ref(pod: dict, ref: Optional[dict]) -> bool:
    if ref is None:
        return True
    m = pod.get("metadata", {})
    for field, have in (("uid", m.get("uid", "")), ("name", m.get("name", "")),
                        ("namespace", m.get("namespace", "")), ("apiVersion", pod.get("apiVersion", ""))):
        if ref.get(field) and ref[field] != have:
            return False
    return True


def match_controller_ref(pod: dict, cref: Optional[dict]) -> bool:
    if cref is None:
        return True
    m = pod.get("metadata", {})
    if cref.get("namespace") and cref["namespace"] != m.get("namespace", ""):
        return False
    for owner in m.get("ownerReferences") or []:
        if cref.get("controller") is not None and (owner.get("controller") is None or
                                                   bool(owner["controller"]) != bool(cref["controller"])):
            continue
        if any(cref.get(f) and cref[f] != owner.get(f, "") for f in ("uid", "name", "kind", "apiVersion")):
            continue
        return True
    return False


def match_owners(pod: dict, owners: Optional[Sequence[dict]]) -> bool:
    """MatchReservationOwners: owners == nil matches nothing, [{}] everything; each owner ANDs its parts."""
    labels = pod.get("metadata", {}).get("labels") or {}
    for o in owners or []:
        if match_object_ref(pod, o.get("object")) and match_controller_ref(pod, o.get("controller")) and \
                (o.get("labelSelector") is None or label_selector_matches(o["labelSelector"], labels)):
            return True
    return False


# ---- reservation affinity (util/reservation/reservation.go:520-624) ----------------------------------------

def _tolerates(tol: dict, taint: dict) -> bool:
    """v1.Toleration.ToleratesTaint."""
    if tol.get("effect") and tol["effect"] != taint.get("effect"):
        return False
    if tol.get("key") and tol["key"] != taint.get("key"):
        return False
    op = tol.get("operator") or "Equal"
    if op == "Exists":
        return True
    return op == "Equal" and (tol.get("value") or "") == (taint.get("value") or "")


class ReservationAffinity:
    """RequiredReservationAffinity of a pod (None when the pod has no reservation-affinity annotation)."""

    def __init__(self, raw: dict):
        self.name = raw.get("name", "")
        self.selector = raw.get("reservationSelector") or None
        req = raw.get("requiredDuringSchedulingIgnoredDuringExecution")
        self.terms = req.get("reservationSelectorTerms") if req else None
        self.tolerations = raw.get("tolerations") or []
        self.tolerate_unschedulable = any(
            _tolerates(t, {"key": TAINT_NODE_UNSCHEDULABLE, "effect": "NoSchedule"}) for t in self.tolerations)

    @staticmethod
    def of(pod: dict) -> Optional["ReservationAffinity"]:
        ann = pod.get("metadata", {}).get("annotations") or {}
        if ANN_RESERVATION_AFFINITY not in ann:
            return None
        s = ann[ANN_RESERVATION_AFFINITY]
        return ReservationAffinity(json.loads(s) if s else {})

    def match_affinity(self, labels: dict, name: str) -> bool:
        if self.selector and any(labels.get(k) != v for k, v in self.selector.items()):
            return False
        if self.terms is not None:
            return node_selector_matches(self.terms, labels, name)
        return True

    def untolerated_taint(self, taints: Sequence[dict]) -> Optional[dict]:
        """FindMatchingUntoleratedTaint with DoNotScheduleTaintsFilter (NoSchedule / NoExecute)."""
        for t in taints or []:
            if t.get("effect") not in ("NoSchedule", "NoExecute"):
                continue
            if not any(_tolerates(tol, t) for tol in self.tolerations):
                return t
        return None


def exact_match(pod_requests: Dict[str, int], allocatable: Dict[str, object], names: Optional[Sequence[str]]) -> bool:
    """ExactMatchReservation (apis/extension/reservation.go:256-276), including its early `return true` when a
    resource is in neither list."""
    if not names:
        return True
    for r in names:
        in_r, in_p = r in allocatable, r in pod_requests
        if not in_r or not in_p:
            return not in_r and not in_p
        if parse_quantity(allocatable[r]) != parse_quantity(pod_requests[r]):
            return False
    return True


def reservation_ignored(pod: dict) -> bool:
    return (pod.get("metadata", {}).get("labels") or {}).get(LABEL_RESERVATION_IGNORED) == "true"


def exact_match_spec(pod: dict) -> Optional[List[str]]:
    s = (pod.get("metadata", {}).get("annotations") or {}).get(ANN_EXACT_MATCH)
    return (json.loads(s).get("resourceNames") or []) if s else None


def check_matched_or_ignored(pod: dict, r: dict, node: dict, pod_requests: Dict[str, object],
                             affinity: Optional[ReservationAffinity] = None, exact: Optional[List[str]] = None,
                             ignored: Optional[bool] = None) -> Tuple[bool, str]:
    """checkReservationMatchedOrIgnored (transformer.go:637-681): (matched or ignored, diagnosis bucket).
    `r` is a Reservation object (metadata.name / labels / deletionTimestamp, spec.owners / unschedulable /
    taints, status.allocatable); `node` the Node it sits on."""
    if ignored is None:
        ignored = reservation_ignored(pod)
    if ignored:
        return True, "ignored"
    if not match_owners(pod, r.get("spec", {}).get("owners")):
        return False, "ownerUnmatched"
    meta, spec = r.get("metadata", {}), r.get("spec", {})
    alloc = (r.get("status") or {}).get("allocatable") or {}
    name = affinity.name if affinity else ""
    if name:
        if meta.get("name", "") != name:
            return False, "nameUnmatched"
        if not exact_match(pod_requests, alloc, exact):
            return False, "notExactMatched"
        return True, "nameMatched"
    unschedulable = bool(spec.get("unschedulable")) or meta.get("deletionTimestamp") is not None
    if unschedulable and not (affinity is not None and affinity.tolerate_unschedulable):
        return False, "isUnschedulableUnmatched"
    if affinity is not None and affinity.untolerated_taint(spec.get("taints")) is not None:
        return False, "taintsUnmatched"
    if affinity is not None:
        labels = dict(node.get("metadata", {}).get("labels") or {})
        labels.update(meta.get("labels") or {})
        if not affinity.match_affinity(labels, meta.get("name", "")):
            return False, "affinityUnmatched"
    if not exact_match(pod_requests, alloc, exact):
        return False, "notExactMatched"
    return True, "matched"


def match_classes(pods: Sequence[dict], pod_requests: Sequence[Dict[str, object]], reservations: Sequence[dict],
                  nodes: Dict[str, dict]) -> Tuple[List[int], List[List[int]], List[Tuple[int, ...]]]:
    """Owner-match classes of a pod batch: (rsv_class per pod, -1 = no reservation matched or ignored; per
    reservation the classes that match it; per class its matched reservation indices). Pods with equal matched
    sets share a class (the device's restore views are per (class, node))."""
    by_set: Dict[Tuple[int, ...], int] = {}
    pod_class, class_sets = [], []
    rsv_classes: List[List[int]] = [[] for _ in reservations]
    for pod, req in zip(pods, pod_requests):
        aff = ReservationAffinity.of(pod)
        exact = exact_match_spec(pod)
        ign = reservation_ignored(pod)
        matched = tuple(x for x, r in enumerate(reservations)
                        if check_matched_or_ignored(pod, r, nodes.get(r.get("status", {}).get("nodeName", ""), {}),
                                                    req, aff, exact, ign)[0])
        if not matched:
            pod_class.append(-1)
            continue
        if matched not in by_set:
            by_set[matched] = len(class_sets)
            class_sets.append(matched)
            for x in matched:
                rsv_classes[x].append(by_set[matched])
        pod_class.append(by_set[matched])
    return pod_class, rsv_classes, class_sets
