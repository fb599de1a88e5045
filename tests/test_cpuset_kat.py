"""cpuset accumulator against the reference's own KATs (cpu_accumulator_test.go):
the CPU oracle (oracle/kg_cpuset.c) here; the device accumulator with -m gpu (tests/test_cpuset_gpu.py)."""
import pytest

import cpuset_kat
import oracle_lib

KAT = cpuset_kat.load()


def oracle_take(topo, max_ref, avail, alloc, needed, bind, excl, strategy, preferred=None):
    return oracle_lib.take_cpus(topo, max_ref, avail, alloc, needed, bind, excl, strategy, preferred)


@pytest.mark.parametrize("case", KAT["takes"], ids=lambda c: f'{c["source"].split()[-1]}:{c["name"]}')
def test_take_kat_oracle(case):
    cpuset_kat.check_take(lambda *a: oracle_take(*a), case)


@pytest.mark.parametrize("seq", KAT["sequences"], ids=lambda s: s["name"])
def test_take_sequence_oracle(seq):
    cpuset_kat.run_sequence(oracle_take, seq)


def test_take_preferred_oracle():
    cpuset_kat.run_preferred(oracle_take, KAT["preferred"])


# ---- device accumulator (kg_cpuset_take), -m gpu ----------------------------------------------------

@pytest.fixture(scope="module")
def ctx():
    from koordinator_amd import engine
    c = engine.Context(0)
    yield c
    c.close()


def device_take(ctx):
    from koordinator_amd import abi, engine

    def take(topo, max_ref, avail, alloc, needed, bind, excl, strategy, preferred=None):
        q = abi.KgCpusetRequest()
        q.topo, q.alloc = 0, 0 if alloc is not None else -1
        for w in range(4):
            q.avail[w] = int(avail[w])
            q.preferred[w] = int(preferred[w]) if preferred is not None else 0
        q.needed, q.max_ref, q.bind, q.excl, q.strategy = needed, max_ref, bind, excl, strategy
        q.has_preferred = 1 if preferred is not None else 0
        out, rc = engine.cpuset_take(ctx, [topo], [alloc] if alloc is not None else [], [q])
        return int(rc[0]), abi.mask_cpus(out[0])
    return take


@pytest.mark.gpu
def test_take_kat_gpu(ctx):
    take = device_take(ctx)
    for case in KAT["takes"]:
        cpuset_kat.check_take(take, case)
    for seq in KAT["sequences"]:
        cpuset_kat.run_sequence(take, seq)
    cpuset_kat.run_preferred(take, KAT["preferred"])


@pytest.mark.gpu
def test_take_random_batch_gpu(ctx):
    """Many requests in one launch (one workgroup each) on random topologies, allocations, policies and
    preferred sets: bit-identical to the oracle, error codes included."""
    import numpy as np
    from koordinator_amd import abi, engine
    rng = np.random.default_rng(7)
    topos, allocs, reqs, args = [], [], [], []
    shapes = [(1, 1, 8, 2), (2, 1, 8, 2), (2, 2, 4, 2), (2, 2, 16, 2), (1, 2, 12, 1), (2, 4, 8, 2), (4, 2, 8, 2)]
    for k in range(600):
        t = abi.cpu_topo_for_test(*shapes[k % len(shapes)])
        n = t.n_cpus
        max_ref = int(rng.choice([1, 1, 2]))
        al = abi.KgCpuAlloc()
        ref = rng.choice([0, 0, 0, 1, 2], size=n) if max_ref > 1 else rng.choice([0, 0, 1], size=n)
        for c in range(n):
            al.ref[c] = int(ref[c])
            al.excl[c] = int(rng.integers(0, 3)) if ref[c] else 0
        avail = abi.cpu_mask([c for c in range(n) if ref[c] < max_ref])
        pref = abi.cpu_mask(rng.choice(n, size=int(rng.integers(0, 6)), replace=False)) if k % 3 == 0 else None
        needed = int(rng.integers(0, n // 2 + 2))
        bind, excl, strat = int(rng.integers(0, 3)), int(rng.integers(0, 3)), int(rng.integers(0, 2))
        topos.append(t)
        allocs.append(al)
        q = abi.KgCpusetRequest()
        q.topo, q.alloc = k, k
        for w in range(4):
            q.avail[w] = int(avail[w])
            q.preferred[w] = int(pref[w]) if pref is not None else 0
        q.needed, q.max_ref, q.bind, q.excl, q.strategy = needed, max_ref, bind, excl, strat
        q.has_preferred = 1 if pref is not None else 0
        reqs.append(q)
        args.append((t, max_ref, avail, al, needed, bind, excl, strat, pref))
    out, rc = engine.cpuset_take(ctx, topos, allocs, reqs)
    ok = 0
    for k, a in enumerate(args):
        wrc, want = oracle_take(*a)
        assert int(rc[k]) == wrc, (k, int(rc[k]), wrc)
        if wrc == 0:
            assert abi.mask_cpus(out[k]) == want, (k, abi.mask_cpus(out[k]), want)
            ok += 1
    assert ok > 400
