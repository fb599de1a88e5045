"""Reference known answers that pin NodeResourcesFit (a1, a2), amplified-CPU NodeNUMAResource (a7, a8),
Reservation fit (a10) and DeviceShare fit / score / NormalizeScore (a12, a13): tests/golden/pin_kat.json,
transcribed from the Go tests cited per case (tests/golden/make_pin_kat.py), built as the test runners
build their fixtures (tests/pin_kat.py).

Each case runs on the oracle (CPU) and, with -m gpu, on the device through the C ABI, where the whole
verify row must also equal the oracle's."""
import numpy as np
import pytest

import oracle_lib
import pin_kat
from koordinator_amd import abi, reasons

CASES = pin_kat.all_cases()
IDS = [c[0] for c in CASES]


def oracle_verify(kc, nodes, pods, rsv):
    if pin_kat.is_ext(kc):
        return oracle_lib.ext_verify(kc, nodes, pods, None, rsv)
    return oracle_lib.eval_verify(kc, nodes, pods)


def check(res, exp):
    st = int(res.status[0, 0])
    if "nrf_reasons" in exp:
        got = reasons.plugin_reasons(st & abi.KG_ST_NRF_MASK, exp.get("scalars", reasons.DEFAULT_SCALARS))
        assert got.get("NodeResourcesFit", []) == exp["nrf_reasons"]
    if "numa_reasons" in exp:
        got = reasons.plugin_reasons(st & abi.KG_ST_NUMA_MASK)
        assert got.get("NodeNUMAResource", []) == exp["numa_reasons"]
        assert not (st & abi.KG_ST_UNSUPPORTED)
    if exp.get("host_path"):
        assert np.all(res.status[0] & abi.KG_ST_UNSUPPORTED)
    if "status" in exp:
        assert st == exp["status"], hex(st)
    if "score_nrf" in exp:
        assert list(res.score_nrf[0]) == exp["score_nrf"]
        if exp.get("order") == "node0 > node1":
            assert res.score_nrf[0, 0] > res.score_nrf[0, 1]
    if "score_numa" in exp:
        assert np.all(res.status[0] == 0)
        assert list(res.score_numa[0]) == exp["score_numa"]
    if "score_dev" in exp:
        assert list(res.score_dev[0]) == exp["score_dev"]
    if "total" in exp:
        assert list(res.total[0]) == exp["total"]


@pytest.mark.parametrize("name,key,case", CASES, ids=IDS)
def test_pin_kat_oracle(name, key, case):
    kc, nodes, pods, rsv, exp = pin_kat.BUILDERS[key](case)
    check(oracle_verify(kc, nodes, pods, rsv), exp)


def test_pin_kat_covers_every_transcribed_case():
    data = pin_kat.load()
    n = sum(len(v) for v in data.values())
    assert len(CASES) == n + len(data["fits_ignored"])  # fits_ignored runs through two plugins
    assert n >= 45


@pytest.fixture(scope="module")
def ctx():
    from koordinator_amd import engine

    c = engine.Context(0)
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name,key,case", CASES, ids=IDS)
def test_pin_kat_gpu(ctx, name, key, case):
    from koordinator_amd import engine

    kc, nodes, pods, rsv, exp = pin_kat.BUILDERS[key](case)
    snap = engine.Snapshot(ctx, kc, nodes)
    if rsv is not None:
        snap.upload_reservations(rsv)
    batch = engine.PodBatch(ctx, pods)
    got = engine.eval_verify(snap, batch)
    check(got, exp)
    ref = oracle_verify(kc, nodes, pods, rsv)
    for f in ("status", "score_nrf", "score_la", "score_numa", "score_dev", "score_rsv", "total", "numa_zone"):
        assert np.array_equal(getattr(got, f), getattr(ref, f)), f
