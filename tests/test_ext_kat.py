"""Config-5 known answers from the reference's Go tests (tests/golden/ext_kat.json), checked on the
oracle (CPU) and through the C ABI on the device (-m gpu)."""
import pytest

import ext_kat
import oracle_lib
from koordinator_amd import abi

K = ext_kat.load()


def _engine_verify(kc, nodes, pods, quotas=None, rsv=None):
    from koordinator_amd import engine
    ctx = engine.Context(0)
    try:
        snap = engine.Snapshot(ctx, kc, nodes)
        if quotas is not None:
            snap.upload_quotas(quotas)
        if rsv is not None:
            snap.upload_reservations(rsv)
        return engine.eval_verify(snap, engine.PodBatch(ctx, pods))
    finally:
        ctx.close()


def _run(backend, kc, nodes, pods, quotas=None, rsv=None):
    if backend == "oracle":
        return oracle_lib.ext_verify(kc, nodes, pods, quotas, rsv)
    return _engine_verify(kc, nodes, pods, quotas, rsv)


BACKENDS = ["oracle", pytest.param("gpu", marks=pytest.mark.gpu)]


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("case", K["deviceshare_score"], ids=[c["name"] for c in K["deviceshare_score"]])
def test_deviceshare_score_kat(backend, case):
    kc, nodes, pods = ext_kat.deviceshare(case)
    got = _run(backend, kc, nodes, pods)
    if "status" in case["want"]:
        assert got.status[0, 0] & getattr(abi, case["want"]["status"]), case["ref"]
    else:
        assert got.status[0, 0] == 0 and got.score_dev[0, 0] == case["want"]["score"], case["ref"]


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("case", K["reservation_score"], ids=[c["name"] for c in K["reservation_score"]])
def test_reservation_score_kat(backend, case):
    kc, nodes, pods, rsv = ext_kat.reservation_score(case)
    got = _run(backend, kc, nodes, pods, rsv=rsv)
    assert got.status[0, 0] == 0
    assert list(got.score_rsv[0]) == case["want"], case["ref"]


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("case", K["reservation_order"], ids=[c["name"] for c in K["reservation_order"]])
def test_reservation_order_kat(backend, case):
    kc, nodes, pods, rsv = ext_kat.reservation_order(case)
    got = _run(backend, kc, nodes, pods, rsv=rsv)
    assert (got.status[0] == 0).all()
    assert list(got.score_rsv[0]) == case["want_score"], case["ref"]
    assert list(got.total[0]) == [kc.weight_rsv * s for s in case["want_normalized"]], case["ref"]


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("case", K["elasticquota_prefilter"], ids=[c["name"] for c in K["elasticquota_prefilter"]])
def test_elasticquota_prefilter_kat(backend, case):
    kc, nodes, pods, q = ext_kat.elasticquota(case)
    got = _run(backend, kc, nodes, pods, quotas=q)
    assert (got.status[0, 0] == 0) == case["want_pass"], case["ref"]
    if not case["want_pass"]:
        assert got.status[0, 0] == abi.KG_ST_QUOTA
