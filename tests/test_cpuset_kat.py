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
