"""DeviceShare GPU allocator (partition tables, topology scopes, shared-GPU bin-packing) against the known
answers of allocator_gpu_test.go (tests/golden/gpu_alloc_kat.json): the oracle on the CPU and the device
through the C ABI (-m gpu). Filter status from the verify matrix, minors from the Reserve."""
import pytest

import gpu_alloc_kat
import oracle_lib
from koordinator_amd import abi

K = gpu_alloc_kat.load()
CASES = K["cases"]


def _check(c, status, minors):
    if c["error"]:
        assert status != 0 and abi.dev_code(status) == gpu_alloc_kat.CODES[c["error"]], hex(status)
    else:
        assert status == 0, hex(status)
        assert gpu_alloc_kat.minors_of(minors) == c["want"]


@pytest.mark.parametrize("c", CASES, ids=[f'{x["line"]}-{x["name"][:40]}' for x in CASES])
def test_gpu_alloc_kat_oracle(c):
    kc, nodes, pods = gpu_alloc_kat.build(K, c)
    v = oracle_lib.ext_verify(kc, nodes, pods)
    st = oracle_lib.OracleState(kc, nodes)
    node, _, minors, _, _ = st.ext_replay(pods)
    _check(c, int(v.status[0, 0]), int(minors[0]))
    assert (node[0] == 0) == (c["error"] is None)


@pytest.mark.gpu
@pytest.mark.parametrize("c", CASES, ids=[f'{x["line"]}-{x["name"][:40]}' for x in CASES])
def test_gpu_alloc_kat_device(c):
    from koordinator_amd import engine
    kc, nodes, pods = gpu_alloc_kat.build(K, c)
    ctx = engine.Context(0)
    try:
        snap = engine.Snapshot(ctx, kc, nodes)
        batch = engine.PodBatch(ctx, pods)
        v = engine.eval_verify(snap, batch)
        minors = 0
        if v.status[0, 0] == 0:
            _, minors = engine.assume_ext(snap, batch, 0, 0)
        _check(c, int(v.status[0, 0]), minors)
        snap2 = engine.Snapshot(ctx, kc, nodes)
        batch2 = engine.PodBatch(ctx, pods)
        node, _ = engine.replay(snap2, batch2)
        assert (node[0] == 0) == (c["error"] is None)
        if c["error"] is None:  # the replay's in-kernel Reserve takes the same minors
            assert gpu_alloc_kat.minors_of(int(engine.replay_minors(batch2)[0])) == c["want"]
    finally:
        ctx.close()
