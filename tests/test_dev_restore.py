"""DeviceShare reservation restore on the host (decode.dev_reusable / dev_effective), pinned by the reference's
Test_tryAllocateFromReservation (deviceshare/reservation_test.go:414-1124).

Each case gives the node's GPU usage and a restore state (matched reservations with allocatable / allocated /
remained, merged tables); tryAllocateFromReusable either allocates from the first matched reservation that
fits (wantResult: its minor), returns nothing (no reservation fits and none is required), or fails (required).
Here: the effective tables of dev_reusable, the DeviceShare fit of kg_ext.h (dev_minor_fits per minor), and the
Reserve order of dev_choose (score desc, minor asc). Not transcribed: the two reservation-ignored pods and the
pre-allocatable case (neither is on the device path)."""
import numpy as np
import pytest

from koordinator_amd import abi, decode

GI = 1 << 30
R, M = abi.KG_DEV_R, abi.KG_DEV_MINORS
CORE, RATIO, MEM = abi.KG_DEV_CORE, abi.KG_DEV_RATIO, abi.KG_DEV_MEM


def tab(minors):
    """{minor: (core, ratio, mem_gi)} -> (table, mask)"""
    t = np.zeros((R, M), np.int64)
    for m, (c, r, g) in (minors or {}).items():
        t[CORE, m], t[RATIO, m], t[MEM, m] = c, r, g * GI
    return t, decode._dmask(t) if minors else np.zeros(M, bool)


ONE = {0: (100, 100, 8), 1: (100, 100, 8)}
HALF = {0: (50, 50, 4)}
P75 = {0: (75, 75, 6)}
P25 = {0: (25, 25, 2)}
P25_1 = {0: (25, 25, 2), 1: (100, 100, 8)}
TOTAL = tab(ONE)[0]

DEFAULT, ALIGNED, RESTRICTED = abi.KG_RSV_DEFAULT, abi.KG_RSV_ALIGNED, abi.KG_RSV_RESTRICTED
HALF_GPU = {CORE: 50, MEM: 4 * GI}  # podRequestsHalfGPU: gpu-core 50, gpu-memory 4Gi

# name, request, matched [(policy, allocatable, allocated, remained)], merged (unmatchedUsed, matchedAllocatable,
# matchedAllocated), deviceUsed, required, want (minor | None = no allocation, "fail")
CASES = [
    ("no matched reservations", HALF_GPU, [], ({}, {}, {}), {}, False, None),
    ("allocate from default policy reservation", HALF_GPU, [(DEFAULT, P25, None, P25)], ({}, P25, {}), {}, False, 0),
    ("allocate from default policy reservation and required from reservation", HALF_GPU,
     [(DEFAULT, HALF, P25, HALF)], ({}, HALF, P25), {0: (50, 50, 4)}, True, 0),
    ("allocate from default policy reservation and required from reservation and reservation empty", HALF_GPU,
     [(DEFAULT, HALF, HALF, None)], ({}, HALF, HALF), {0: (150, 150, 12)}, True, 1),
    ("allocate from Aligned policy reservation", HALF_GPU, [(ALIGNED, HALF, None, HALF)], ({}, HALF, None),
     {0: (100, 100, 8), 1: (100, 100, 8)}, False, 0),
    ("failed to allocate from Aligned policy reservation with bigger request but no remaining resources on node",
     {CORE: 60, MEM: 5 * GI}, [(ALIGNED, HALF, None, HALF)], ({}, HALF, None),
     {0: (100, 100, 8), 1: (100, 100, 8)}, True, "fail"),
    ("failed to allocate from Aligned policy reservation that remaining little not fits request",
     {CORE: 30, MEM: 1 * GI}, [(ALIGNED, HALF, P25, P25)], ({}, HALF, P25),
     {0: (125, 125, 10), 1: (100, 100, 8)}, True, "fail"),
    ("allocate from Restricted policy reservation", HALF_GPU, [(RESTRICTED, HALF, None, HALF)], ({}, HALF, None),
     {0: (100, 100, 8), 1: (100, 100, 8)}, False, 0),
    ("failed to allocate from Restricted policy reservation since node remains resources but reservation not fits",
     HALF_GPU, [(RESTRICTED, HALF, P25, P25)], ({}, HALF, P25), {0: (75, 75, 6), 1: (100, 100, 8)}, True, "fail"),
    ("allocate from Restricted policy reservation with reservation-ignored pods", HALF_GPU,
     [(RESTRICTED, ONE, None, ONE)], ({}, HALF, None), {0: (175, 175, 14), 1: (150, 150, 12)}, False, 1),
]


def fits_minor(free, m, req):
    f = free[:, m]
    if not f.any():
        return False
    return all(req[k] <= f[k] for k in req)


def least(req, total):
    if total == 0 or req > total:
        return 0
    return (total - req) * 100 // total


def minor_score(total, free, m, req):
    """dev_least on one minor with the shipped DeviceShare weights (gpu-memory-ratio 1, gpu-memory 1)."""
    s = w = 0
    for k in (RATIO, MEM):
        t, f = total[k, m], free[k, m]
        if t == 0:
            continue
        r = t - f + req.get(k, 0) if t >= f else t
        s += least(r, t)
        w += 1
    return s // w if w else 0


def choose(total, free, req):
    cand = [m for m in range(M) if fits_minor(free, m, req)]
    if not cand:
        return None
    return sorted(cand, key=lambda m: (-minor_score(total, free, m, req), m))[0]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_try_allocate_from_reservation(case):
    name, req, matched, (uu, mal, ma), used, required, want = case
    used_t = tab(used)[0]
    free = np.maximum(TOTAL - used_t, 0)
    parts = []
    for policy, alloc, _allocated, rem in matched:
        parts.append((policy, tab(alloc), tab(rem)))
    per, _base = decode.dev_reusable(TOTAL, used_t, free, tab(uu), tab(ma), tab(mal), parts)
    got = None
    for T, F in per:
        m = choose(T, F, req)
        if m is not None:
            got = m
            break
    if got is None and required and matched:
        got = "fail"
    assert got == want, name


def test_reservation_parts_follow_restore():
    """RestoreReservation's filterFn: remained = allocatable - allocated on the reservation's minors, and an
    unmatched reservation gives back what its pods use inside it."""
    r = {"dev_alloc": tab(HALF)[0], "dev_allocated": tab(P25)[0] + tab({1: (10, 10, 1)})[0]}
    (alloc, am), (allocated, alm), (rem, rm), (used, um) = decode.dev_reservation_parts(r)
    assert list(np.nonzero(am)[0]) == [0]
    assert allocated[:, 1].sum() == 0  # minor 1 is not the reservation's: not counted (appendAllocatedByHints)
    assert np.array_equal(rem, tab({0: (25, 25, 2)})[0]) and list(np.nonzero(rm)[0]) == [0]
    assert np.array_equal(used, tab(P25)[0]) and list(np.nonzero(um)[0]) == [0]
    assert decode.dev_reservation_parts({"dev_alloc": None}) is None
