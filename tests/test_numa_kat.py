"""NodeNUMAResource known answers from the reference's Go tests (tests/golden/numa_kat.json) on the
oracle (CPU) and through the C ABI on the device (-m gpu): SingleNUMANode / Restricted hint merge
and the NUMA scores."""
import pytest

import numa_kat
import oracle_lib

K = numa_kat.load()
BACKENDS = ["oracle", pytest.param("gpu", marks=pytest.mark.gpu)]


def _verify(backend, kc, nodes, pods):
    if backend == "oracle":
        return oracle_lib.eval_verify(kc, nodes, pods)
    from koordinator_amd import engine
    ctx = engine.Context(0)
    try:
        return engine.eval_verify(engine.Snapshot(ctx, kc, nodes), engine.PodBatch(ctx, pods))
    finally:
        ctx.close()


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("case", K["affinity"], ids=[c["name"] for c in K["affinity"]])
def test_numa_affinity_kat(backend, case):
    kc, nodes, pods = numa_kat.affinity(case)
    got = _verify(backend, kc, nodes, pods)
    assert got.status[0, 0] == 0, case["ref"]
    assert got.numa_zone[0, 0] == case["want_zone"], case["ref"]


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("case", K["score"], ids=[c["name"] for c in K["score"]])
def test_numa_score_kat(backend, case):
    kc, nodes, pods = numa_kat.score(case)
    got = _verify(backend, kc, nodes, pods)
    assert (got.status[0] == 0).all(), case["ref"]
    assert list(got.score_numa[0]) == case["want"], case["ref"]
