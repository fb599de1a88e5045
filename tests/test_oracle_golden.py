"""Pins the CPU oracle (and the host decode) to the reference's own known-answer tests."""
import pytest

import kat
import oracle_lib
from koordinator_amd import abi

LA = kat.load("loadaware_kat.json")


@pytest.mark.parametrize("case", LA["cases"], ids=[c["name"] for c in LA["cases"]])
def test_loadaware_kat_oracle(case):
    cfg, nodes, pods = kat.la_case(case, LA["node_default"])
    kc = cfg.kg_config()
    r = oracle_lib.eval_pair(kc, nodes, 0, pods, 0)
    if case["kind"] == "filter":
        code, reason = kat.la_status(r.status & abi.KG_ST_LA_MASK)
        assert code == case["want"]["code"], (case["ref"], hex(r.status))
        if "reason" in case["want"]:
            assert reason == case["want"]["reason"]
    else:
        assert r.s_la == case["want"]["score"], case["ref"]
