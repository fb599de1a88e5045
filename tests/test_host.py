"""CPU-side tests: the C-ABI library loads and exports the header's symbols, host-only helpers,
host decode known answers, oracle self-consistency."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import kat
import oracle_lib
from koordinator_amd import abi, decode, engine, synth
from koordinator_amd.config import LoadAwareArgs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "koordgpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kg_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    L = engine.lib()
    names = header_functions()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert L.kg_abi_version() == abi.KG_ABI_VERSION


def test_struct_layouts_match_header(tmp_path):
    """ctypes mirrors have the C sizes of include/koordgpu.h (compiled with gcc here)."""
    import subprocess
    names = ["kg_config", "kg_node_columns", "kg_node_state", "kg_pod_columns", "kg_verify_out",
             "kg_quota_columns", "kg_rsv_view", "kg_rsv_info", "kg_rsv_dev", "kg_cpu_topo", "kg_cpu_alloc",
             "kg_cpuset_request", "kg_reserve_record"]
    src = tmp_path / "sz.c"
    hdr = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "koordgpu.h")
    src.write_text(f'#include "{hdr}"\n#include <stdio.h>\nint main(void){{' +
                   "".join(f'printf("%zu\\n", sizeof({n}));' for n in names) + "return 0;}\n")
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", str(src), "-o", str(exe)])
    sizes = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    mirrors = [abi.KgConfig, abi.KgNodeColumns, abi.KgNodeState, abi.KgPodColumns, abi.KgVerifyOut,
               abi.KgQuotaColumns, abi.KgRsvView, abi.KgRsvInfo, abi.KgRsvDev, abi.KgCpuTopo, abi.KgCpuAlloc,
               abi.KgCpusetRequest, abi.KgReserveRecord]
    for n, c_size, m in zip(names, sizes, mirrors):
        assert C.sizeof(m) == c_size, n


def test_keys_host_helpers():
    L = engine.lib()
    for total, node in [(0, 0), (190, 5), (500_000, 99_999), (1, 0x7FFFFFFE)]:
        key = L.kg_make_key(total, node)
        assert key == abi.make_key(total, node)
        assert L.kg_key_node(key) == node and L.kg_key_total(key) == total
    assert L.kg_key_node(0) == -1 and L.kg_key_total(0) == -1
    # higher total wins, then lower index
    assert abi.make_key(10, 7) > abi.make_key(9, 0)
    assert abi.make_key(10, 3) > abi.make_key(10, 4)


def test_merge_keys_is_global_select_host():
    rng = np.random.default_rng(3)
    keys = np.zeros((4, 100, 3), np.uint64)
    for s in range(4):
        for j in range(100):
            ks = sorted((abi.make_key(int(rng.integers(0, 300)), s * 1000 + int(i)) for i in rng.choice(1000, 3, False)),
                        reverse=True)
            keys[s, j] = ks
    keys[2, 10] = 0  # shard with no feasible node
    out = engine.merge_keys(keys)
    flat = np.sort(keys.transpose(1, 0, 2).reshape(100, -1), axis=1)[:, ::-1][:, :3]
    assert np.array_equal(out, flat)


def test_device_count_without_gpu_is_safe():
    assert engine.device_count() >= 0


def test_oracle_parallel_baseline_equals_sequential():
    cfg, nodes, pods = synth.small(800, 120, seed=21)
    kc = cfg.kg_config()
    seq = oracle_lib.select(kc, nodes, pods, 1)[:, 0]
    for workers in (1, 3, 16):
        par = oracle_lib.select_parallel(kc, nodes, pods, workers)
        assert np.array_equal(seq, par)


def test_oracle_replay_consistent_with_assume():
    cfg, nodes, pods = synth.small(120, 200, seed=22, scale=3.0)
    kc = cfg.kg_config()
    st = oracle_lib.OracleState(kc, nodes)
    node, total = st.replay(pods)
    st2 = oracle_lib.OracleState(kc, nodes)
    for j in range(200):
        view = st2.table()
        keys = oracle_lib.select(kc, view, abi.take(pods, [j]), 1)[0, 0]
        assert abi.key_node(keys) == node[j]
        if node[j] >= 0:
            st2.assume(int(node[j]), pods, j)
    assert (node < 0).any()


EST_CASES = [
    # default_estimator_test.go:33-283 (TestDefaultEstimatorEstimatePod)
    ("estimate empty pod", {"containers": [{}]}, None, False, [250, 200 * 1024 * 1024]),
    ("estimate guaranteed pod", {"containers": [{"requests": {"cpu": "4", "memory": "8Gi"}, "limits": {"cpu": "4", "memory": "8Gi"}}]},
     None, False, [3400, 6012954214]),
    ("estimate burstable pod", {"containers": [{"requests": {"cpu": "4", "memory": "8Gi"}, "limits": {"cpu": "8", "memory": "8Gi"}}]},
     None, False, [6800, 6012954214]),
    ("zoomed cpu factors", {"containers": [{"requests": {"cpu": "4", "memory": "8Gi"}, "limits": {"cpu": "4", "memory": "8Gi"}}]},
     {"cpu": 110}, False, [4000, 6012954214]),
    ("zoomed memory factors", {"containers": [{"requests": {"cpu": "4", "memory": "8Gi"}, "limits": {"cpu": "4", "memory": "8Gi"}}]},
     {"memory": 110}, False, [3400, 8589934592]),
    ("estimate Batch pod", {"labels": {"koordinator.sh/qosClass": "BE"}, "priority": 5000,
                            "containers": [{"requests": {"kubernetes.io/batch-cpu": "4000", "kubernetes.io/batch-memory": "8Gi"},
                                            "limits": {"kubernetes.io/batch-cpu": "4000", "kubernetes.io/batch-memory": "8Gi"}}]},
     None, False, [3400, 6012954214]),
    ("estimate pod only has request", {"labels": {"koordinator.sh/qosClass": "LS"}, "priority": 9999,
                                       "containers": [{"requests": {"cpu": "4", "memory": "8Gi"}}]},
     {"cpu": 80, "memory": 80}, False, [3200, 6871947674]),
    ("estimate pod with customized factors", {"labels": {"koordinator.sh/qosClass": "LS"}, "priority": 9999,
                                              "annotations": {"scheduling.koordinator.sh/load-estimated-scaling-factors": '{"cpu":100}'},
                                              "containers": [{"requests": {"cpu": "4", "memory": "8Gi"}}]},
     {"cpu": 80, "memory": 80}, True, [4000, 6871947674]),
]


@pytest.mark.parametrize("name,pod,factors,custom,want", EST_CASES, ids=[c[0] for c in EST_CASES])
def test_estimator_known_answers(name, pod, factors, custom, want):
    la = LoadAwareArgs(estimated_scaling_factors=dict(factors) if factors else None,
                       allow_customize_estimation=custom).defaulted()
    assert decode.estimate_pod(kat.make_pod(pod), la) == want


@pytest.mark.parametrize("ann,alloc,want", [
    # default_estimator_test.go:291-360 (TestDefaultEstimatorEstimateNode)
    (None, {"cpu": "32"}, {"cpu": 32000}),
    ('{"cpu":28,"memory":"32Gi"}', {"cpu": "32", "memory": "42Gi"}, {"cpu": 28000, "memory": 32 << 30}),
    ('{"cpu":32,"memory":"42Gi"}', {"cpu": "32", "memory": "42Gi"}, {"cpu": 32000, "memory": 42 << 30}),
])
def test_estimate_node_known_answers(ann, alloc, want):
    node = {"metadata": {"annotations": {decode.ANN_RAW_ALLOCATABLE: ann} if ann else {}}, "status": {"allocatable": alloc}}
    got = {k: decode.vec_value(k, v) for k, v in decode.estimate_node_allocatable(node).items()}
    assert got == want


@pytest.mark.parametrize("q,value,milli", [
    ("1", 1, 1000), ("100m", 1, 100), ("0.5", 1, 500), ("1Gi", 1 << 30, 1000 << 30), ("20k", 20000, 20_000_000),
    ("1.5Mi", 1572864, 1572864000), ("2e3", 2000, 2_000_000), ("0", 0, 0), ("250m", 1, 250)])
def test_quantity(q, value, milli):
    assert decode.value(q) == value and decode.milli_value(q) == milli


def test_pod_requests_sidecars_and_overhead():
    pod = kat.make_pod({"containers": [{"requests": {"cpu": "1", "memory": "1Gi"}}],
                        "init_containers": [{"requests": {"cpu": "3"}},
                                            {"requests": {"cpu": "500m", "memory": "2Gi"}, "restartPolicy": "Always"},
                                            {"requests": {"cpu": "2"}}],
                        "overhead": {"cpu": "100m"}})
    r = decode.pod_requests(pod)
    # containers 1 + sidecar 0.5 = 1.5 cpu; init max(3, 2 + 0.5) = 3 -> max(1.5, 3) = 3; + overhead
    assert decode.milli_value(r["cpu"]) == 3100
    assert decode.value(r["memory"]) == 3 << 30
    nz = decode.pod_requests(kat.make_pod({"containers": [{"requests": {"cpu": "1"}}, {}]}), decode.NON_MISSING)
    assert decode.milli_value(nz["cpu"]) == 1100 and decode.value(nz["memory"]) == 400 << 20


@pytest.mark.parametrize("spec,want", [
    ({}, "koord-batch"),                                                        # BestEffort -> BE -> batch
    ({"containers": [{"requests": {"cpu": "1"}}]}, "koord-prod"),               # Burstable -> LS -> prod
    ({"priority": 7000}, "koord-mid"),
    ({"priority": 100, "containers": [{"requests": {"cpu": "1"}}]}, "koord-prod"),
    ({"labels": {"koordinator.sh/priority-class": "koord-free"}}, "koord-free"),
    ({"labels": {"koordinator.sh/qosClass": "BE"}, "containers": [{"requests": {"cpu": "1"}}]}, "koord-batch"),
])
def test_priority_class_with_default(spec, want):
    assert decode.priority_class(kat.make_pod(spec)) == want


def test_oracle_parallel_replay_equals_sequential():
    """The replay CPU baseline (each cycle on the 16-worker parallelizer) places exactly like kgo_replay."""
    cfg, nodes, pods = synth.small(300, 400, seed=24, scale=6.0, numa=True)
    kc = cfg.kg_config()
    want, wtot = oracle_lib.OracleState(kc, nodes).replay(pods)
    for workers in (1, 5, 16):
        got, gtot = oracle_lib.OracleState(kc, nodes).replay_parallel(pods, workers)
        assert np.array_equal(got, want) and np.array_equal(gtot, wtot)
    assert (want < 0).any() and (want >= 0).any()


def test_reason_strings():
    from koordinator_amd import reasons
    bits = abi.KG_ST_NRF_CPU | abi.KG_ST_LA_MEM | abi.KG_ST_LA_AGG | abi.KG_ST_NUMA_AMP_CPU
    got = reasons.plugin_reasons(bits)
    assert got["NodeResourcesFit"] == ["Insufficient cpu"]
    assert got["LoadAwareScheduling"] == ["node(s) memory aggregated usage exceed threshold"]
    assert got["NodeNUMAResource"] == ["Insufficient amplified cpu"]
    assert reasons.reasons(0) == []
    assert reasons.loadaware_status(abi.KG_ST_LA_EXPIRED) == ("Unschedulable", "node(s) nodeMetric expired")


def test_non_zero_requests_rule():
    """NonZeroRequested's rule, as koordinator restates it in GetNonZeroRequestForResource
    (frameworkext/reservation_info.go:579-600, pinned by reservation_info_test.go:934-1003 where a reserve pod
    without requests gets Non0AllocatedMilliCPU / Non0AllocatedMem = schedutil's defaults): a cpu / memory key
    that is absent takes the default, one explicitly set to zero stays zero; per container, so a pod's
    non-zero request is the sum over containers. The default values themselves (100m, 200Mi) are upstream
    constants (k8s.io/kubernetes v1.35.6 pkg/scheduler/util) not present in the reference tree: parity of the
    values is unpinned."""
    from koordinator_amd.config import SchedulerConfig

    def pod(*reqs):
        return {"metadata": {"name": "p", "namespace": "d"},
                "spec": {"containers": [{"name": f"c{k}", "resources": {"requests": r}} for k, r in enumerate(reqs)]}}

    cfg = SchedulerConfig()
    row = decode.pod_row(pod({}, {"cpu": "0", "memory": "0"}, {"cpu": "250m"}), cfg)
    assert (row["req_cpu"], row["req_mem"]) == (250, 0)
    # container 0: both defaults; container 1: explicit zeros; container 2: its cpu, the memory default
    assert row["nz_cpu"] == 100 + 0 + 250
    assert row["nz_mem"] == 2 * 200 * 1024 * 1024


def test_default_cpu_bind_policy_from_profile():
    """A "" / "Default" bind policy takes NodeNUMAResourceArgs.DefaultCPUBindPolicy (plugin.go:327-334,
    FullPCPUs by default, v1/defaults.go:50); an explicit policy is kept; a required policy marks REQUIRED."""
    import json

    from koordinator_amd.config import SchedulerConfig

    def lsr(spec):
        ann = {decode.ANN_RESOURCE_SPEC: json.dumps(spec)} if spec is not None else {}
        return {"metadata": {"name": "p", "namespace": "d", "annotations": ann,
                             "labels": {"koordinator.sh/qosClass": "LSR"}},
                "spec": {"priority": 9500, "containers": [{"name": "c", "resources": {"requests": {"cpu": "4"}}}]}}

    def policy(flags):
        return (flags >> abi.KG_POD_CPU_POLICY_SHIFT) & 3

    full, spread = abi.KG_CPU_BIND["FullPCPUs"], abi.KG_CPU_BIND["SpreadByPCPUs"]
    for default, want in (("FullPCPUs", full), ("SpreadByPCPUs", spread)):
        cfg = SchedulerConfig(default_cpu_bind_policy=default)
        for spec in (None, {}, {"preferredCPUBindPolicy": "Default"}):
            f = decode.pod_row(lsr(spec), cfg)["flags"]
            assert f & abi.KG_POD_CPU_BIND and policy(f) == want and not f & abi.KG_POD_CPU_REQUIRED
        f = decode.pod_row(lsr({"preferredCPUBindPolicy": "FullPCPUs"}), cfg)["flags"]
        assert policy(f) == full
        f = decode.pod_row(lsr({"requiredCPUBindPolicy": "Default"}), cfg)["flags"]
        assert policy(f) == want and f & abi.KG_POD_CPU_REQUIRED
