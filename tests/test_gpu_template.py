"""f4: GPU shared-resource templates (deviceshare/gpu_shared_resource_templates_cache.go, allocator_gpu.go:135-168,
utils.go:540-547).

- The host decode of the template cache against the reference's known answers: findMatchedTemplates
  (gpu_shared_resource_templates_cache_test.go:84-190 on testTemplatesInfos :31-75), the configmap loader (:199-240),
  the key builder (:242-244) and parseGPURequirements' candidates / PreFilter error (utils_test.go:768-819,
  plugin_test.go:656-681).
- allocateByTemplate on the device path: the candidates of the node's vendor-model key decide (none: the allocation
  fails with ErrNoMatchedGPUSharedResourceTemplate, UnschedulableAndUnresolvable — TestAllocateByTemplate's "no matched
  template" case, allocator_gpu_test.go:1871-1883; one: generalAllocate; several: the plain allocator). The oracle
  restates it; the device matches the oracle bit for bit on config-5 clusters with template pods.

TestAllocateByTemplate's other cases (:1718-1870) decide on Huawei NPU dimensions (npu-core / npu-cpu / npu-dvpp) the
device tables do not hold (KG_DEV_R = gpu-core, gpu-memory-ratio, gpu-memory): parity unpinned for those dimensions;
templates over the GPU dimensions are pinned through the control flow above.
"""
import numpy as np
import pytest
import yaml

import oracle_lib
from koordinator_amd import abi, decode, synth

GM, CORE, CPU, DVPP = "koordinator.sh/gpu-memory", "huawei.com/npu-core", "huawei.com/npu-cpu", "huawei.com/npu-dvpp"


def _t(mem, core, cpu, dvpp=None):
    t = {GM: mem, CORE: core, CPU: cpu}
    if dvpp is not None:
        t[DVPP] = dvpp
    return t


# testTemplatesInfos (gpu_shared_resource_templates_cache_test.go:31-75)
INFOS = {"huawei-Ascend-310P": {
    "vir01": _t("3Gi", "1", "1", "12"),
    "vir02": _t("6Gi", "2", "2", "25"),
    "vir02_1c": _t("6Gi", "2", "1", "25"),
    "vir04": _t("12Gi", "4", "4", "50"),
    "vir04_3c": _t("12Gi", "4", "3", "50"),
    "vir04_3c_ndvpp": _t("12Gi", "4", "3"),
    "vir04_4c_dvpp": _t("12Gi", "4", "4", "100"),
}}
MATCHED = [CORE]  # testGPUSharedResourceTemplatesMatchedResources (plugin_test.go:85)

FIND_CASES = [  # (line, resources, strict, {key: [names]})
    (96, _t("6Gi", "2", "2", "25"), True, {"huawei-Ascend-310P": ["vir02"]}),
    (119, _t("6Gi", "2", "3", "25"), True, {}),
    (133, {CORE: "2"}, True, {}),
    (144, {CORE: "2"}, False, {"huawei-Ascend-310P": ["vir02", "vir02_1c"]}),
    (170, {CORE: "3"}, False, {}),
]


@pytest.mark.parametrize("line,res,strict,want", FIND_CASES, ids=[str(c[0]) for c in FIND_CASES])
def test_find_matched_templates_kat(line, res, strict, want):
    cache = decode.GpuSharedResourceTemplates(INFOS)
    got = cache.find_matched(res, strict)
    assert {k: sorted(v) for k, v in got.items()} == want
    for k, names in want.items():  # the matched templates are the whole templates, not the masked ones
        for n in names:
            assert got[k][n] == {r: decode.parse_quantity(q) for r, q in INFOS[k][n].items()}


def test_templates_configmap_and_key():
    data = yaml.safe_dump(INFOS)
    cache = decode.GpuSharedResourceTemplates.from_configmap({"data": {"data.yaml": data}})
    assert cache.infos == decode.GpuSharedResourceTemplates(INFOS).infos
    with pytest.raises(ValueError):
        decode.GpuSharedResourceTemplates.from_configmap({"data": {"data.yaml": "invalid yaml"}})
    node = {"metadata": {"labels": {decode.LABEL_GPU_VENDOR: "huawei", decode.LABEL_GPU_MODEL: "Ascend-310P"}}}
    assert decode.gpu_template_key(node) == "huawei-Ascend-310P"
    assert cache.node_key(node) == 0
    assert cache.node_key({"metadata": {}}) == abi.KG_GPU_TMPL_NONE


def test_parse_gpu_requirements_templates_kat():
    """utils_test.go:768-803: a shared NPU request matches vir04 only; :804-819 and plugin_test.go:656-681: no
    template matches, PreFilter fails with ErrNoMatchedGPUSharedResourceTemplate."""
    cache = decode.GpuSharedResourceTemplates(INFOS, MATCHED)
    flags, tmpl, cands = cache.pod_template(_t("12Gi", "4", "4", "50"), shared=True)
    assert flags == abi.KG_GPU_POD_TEMPLATE and tmpl == 1
    assert {k: sorted(v) for k, v in cands.items()} == {"huawei-Ascend-310P": ["vir04"]}
    node = {"metadata": {"labels": {decode.LABEL_GPU_VENDOR: "huawei", decode.LABEL_GPU_MODEL: "Ascend-310P"}}}
    assert cache.allocation_template(cands, node) == "vir04"
    with pytest.raises(decode.NoMatchedTemplate):
        cache.pod_template(_t("12Gi", "5", "4", "50"), shared=True)
    # not shared, or no matched resource named: no template enforced
    assert cache.pod_template(_t("12Gi", "5", "4", "50"), shared=False)[:2] == (0, 0)
    assert cache.pod_template({GM: "12Gi"}, shared=True)[:2] == (0, 0)


# ---- allocateByTemplate in the allocator (oracle, then the device) --------------------------------------------------

GPU_TEMPLATES = {  # templates over the device's GPU dimensions: a vendor-model key per GPU model of the cluster
    "nvidia-A100": {"1g.10gb": {"koordinator.sh/gpu-core": 14, GM: "10Gi"},
                    "2g.20gb": {"koordinator.sh/gpu-core": 28, GM: "20Gi"}},
    "nvidia-H100": {"1g.10gb": {"koordinator.sh/gpu-core": 14, GM: "10Gi"},
                    "1g.10gb+me": {"koordinator.sh/gpu-core": 14, GM: "10Gi"}},
}


def _one_node_case():
    """One 8-GPU node (80Gi each, no topology tree) and a shared pod of one 10Gi / core-14 instance."""
    nodes = abi.empty_nodes(1)
    nodes["alloc_cpu"][:] = 64000
    nodes["alloc_mem"][:] = 256 << 30
    nodes["alloc_pods"][:] = 110
    nodes["dev_minors"][0] = 8
    for m in range(8):
        nodes["dev_total"][0, :, m] = [100, 100, 80 << 30]
        nodes["dev_free"][0, :, m] = [100, 100, 80 << 30]
    pods = abi.empty_pods(1)
    vec, keys, cnt, shared = decode.gpu_requirements({"koordinator.sh/gpu-core": 14, GM: 10 << 30})
    assert shared and cnt == 1
    pods["dev_req"][0] = vec
    pods["dev_keys"][0] = keys
    pods["dev_count"][0] = cnt
    pods["dev_flags"] = np.array([abi.KG_GPU_POD_SHARED], np.uint32)
    return nodes, pods, decode.GpuSharedResourceTemplates(GPU_TEMPLATES, [GM]).requests_per_gpu(vec, keys)


def _kc():
    from koordinator_amd.config import config5_profile
    kc = config5_profile().kg_config()
    kc.plugins = abi.KG_PLUGIN_NRF | abi.KG_PLUGIN_DEV
    return kc


@pytest.mark.parametrize("model,cands", [("A100", 1), ("H100", 2), ("V100", 0), ("", 0)])
def test_allocate_by_template_oracle(model, cands):
    """The node key's candidates: none fails (TestAllocateByTemplate "no matched template",
    allocator_gpu_test.go:1871-1883: an unlabelled node), one or several allocate as the plain allocator does."""
    cache = decode.GpuSharedResourceTemplates(GPU_TEMPLATES, [GM])
    nodes, pods, rpg = _one_node_case()
    flags, tmpl, cand = cache.pod_template(rpg, shared=True)
    assert flags == abi.KG_GPU_POD_TEMPLATE
    node = {"metadata": {"labels": {decode.LABEL_GPU_VENDOR: "nvidia", decode.LABEL_GPU_MODEL: model} if model else {}}}
    kc = _kc()
    plain = oracle_lib.ext_verify(kc, nodes, pods)
    nodes["dev_part"] = np.array([cache.node_key(node) << abi.KG_GPU_TMPL_SHIFT], np.uint32)
    pods["dev_flags"] = pods["dev_flags"] | np.uint32(flags)
    pods["dev_tmpl"] = np.array([tmpl], np.uint32)
    got = oracle_lib.ext_verify(kc, nodes, pods)
    if cands == 0:
        assert abi.dev_code(int(got.status[0, 0])) == abi.KG_DEV_CODE_NO_TEMPLATE
        assert cache.allocation_template(cand, node) is None
    else:
        assert got.status[0, 0] == 0 and plain.status[0, 0] == 0
        assert np.array_equal(got.total, plain.total)
        assert (cache.allocation_template(cand, node) is not None) == (cands == 1)


def _template_cluster(seed, n_nodes=900, n_pods=192, rsv_frac=0.2, numa="none"):
    """cluster5 with template keys on the GPU nodes (two configured keys, 20% of the nodes with no templates) and
    the shared GPU pods enforcing templates (random candidate counts per key, some with none on a key)."""
    cfg, nodes, pods, quotas, rsv = synth.cluster5(n_nodes, n_pods, seed_config=seed, rsv_frac=rsv_frac, numa=numa)
    nodes = {k: v.copy() for k, v in nodes.items()}
    pods = {k: v.copy() for k, v in pods.items()}
    r = np.random.default_rng(seed)
    key = r.choice([0, 1, abi.KG_GPU_TMPL_NONE], len(nodes["alloc_cpu"]), p=[0.45, 0.35, 0.2]).astype(np.uint32)
    nodes["dev_part"] = (nodes["dev_part"] | (key << abi.KG_GPU_TMPL_SHIFT)).astype(np.uint32)
    shared = (pods["dev_count"] > 0) & ((pods["dev_flags"] & abi.KG_GPU_POD_SHARED) != 0)
    tmpl = (r.integers(0, 3, len(shared)) | (r.integers(0, 3, len(shared)) << 2)).astype(np.uint32)
    pods["dev_tmpl"] = np.where(shared, tmpl, 0).astype(np.uint32)
    pods["dev_flags"] = np.where(shared, pods["dev_flags"] | abi.KG_GPU_POD_TEMPLATE, pods["dev_flags"]).astype(np.uint32)
    return cfg, nodes, pods, quotas, rsv


def test_template_cluster_oracle():
    """Template pods in a config-5 cluster: on the device path everywhere; ErrNoMatchedGPUSharedResourceTemplate exactly
    on the nodes whose key holds no candidate; elsewhere the outcome of the same pod without a template."""
    cfg, nodes, pods, quotas, rsv = _template_cluster(41, 500, 128)
    kc = cfg.kg_config()
    v = oracle_lib.ext_verify(kc, nodes, pods, quotas, rsv)
    assert not (v.status & abi.KG_ST_UNSUPPORTED).any()
    plain = {k: a.copy() for k, a in pods.items()}
    plain["dev_flags"] = (plain["dev_flags"] & ~np.uint32(abi.KG_GPU_POD_TEMPLATE)).astype(np.uint32)
    w = oracle_lib.ext_verify(kc, nodes, plain, quotas, rsv)
    t = (pods["dev_flags"] & abi.KG_GPU_POD_TEMPLATE) != 0
    key = (nodes["dev_part"] >> abi.KG_GPU_TMPL_SHIFT) & 15
    cand = np.where(key[None, :] == abi.KG_GPU_TMPL_NONE, 0,
                    (pods["dev_tmpl"][:, None] >> (2 * np.minimum(key, 14)[None, :])) & 3)
    none = t[:, None] & (cand == 0) & (nodes["dev_minors"] > 0)[None, :]
    codes = np.vectorize(abi.dev_code)(v.status)
    quota = (v.status & abi.KG_ST_QUOTA) != 0  # ElasticQuota's PreFilter rejects the pod before any Filter
    assert t.sum() >= 10 and (none & ~quota).sum() > 100
    # (a pod that must allocate from a reservation reports makeReasonsByReservation's reason instead)
    rsv_reason = (v.status & abi.KG_ST_DEV_RSV) != 0
    assert (codes[none & ~quota & ~rsv_reason] == abi.KG_DEV_CODE_NO_TEMPLATE).all()
    same = ~none | quota
    assert np.array_equal(v.status[same], w.status[same])
    rows = ~(none & ~quota).any(axis=1)  # NormalizeScore runs over the feasible nodes: rows without a template miss
    assert rows.sum() >= 20 and np.array_equal(v.total[rows], w.total[rows])


FIELDS = ("status", "score_nrf", "score_la", "score_numa", "score_dev", "score_rsv", "total", "numa_zone")


@pytest.fixture(scope="module")
def ctx():
    from koordinator_amd import engine
    c = engine.Context(0)
    yield c
    c.close()


def _make(ctx, kc, nodes, pods, quotas, rsv):
    from koordinator_amd import engine
    snap = engine.Snapshot(ctx, kc, nodes)
    if kc.plugins & abi.KG_PLUGIN_QUOTA:
        snap.upload_quotas(quotas)
    if kc.plugins & abi.KG_PLUGIN_RSV:
        snap.upload_reservations(rsv)
    return snap, engine.PodBatch(ctx, pods)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,numa", [(42, "none"), (43, "mix")])
def test_template_verify_device(ctx, seed, numa):
    from koordinator_amd import engine
    cfg, nodes, pods, quotas, rsv = _template_cluster(seed, numa=numa)
    kc = cfg.kg_config()
    snap, batch = _make(ctx, kc, nodes, pods, quotas, rsv)
    got = engine.eval_verify(snap, batch)
    ref = oracle_lib.ext_verify(kc, nodes, pods, quotas, rsv)
    for name in FIELDS:
        a, b = getattr(got, name), getattr(ref, name)
        if not np.array_equal(a, b):
            j, i = np.argwhere(a != b)[0]
            raise AssertionError(f"{name} differs, first pod {j} node {i}: gpu={a[j, i]} oracle={b[j, i]}")
    assert (np.vectorize(abi.dev_code)(ref.status) == abi.KG_DEV_CODE_NO_TEMPLATE).any()


@pytest.mark.gpu
def test_template_select_and_replay_device(ctx):
    from koordinator_amd import engine
    cfg, nodes, pods, quotas, rsv = _template_cluster(44, 1500, 400, rsv_frac=0.0)
    kc = cfg.kg_config()
    kc.plugins &= ~abi.KG_PLUGIN_RSV
    snap, batch = _make(ctx, kc, nodes, pods, quotas, rsv)
    got = engine.eval_select(snap, batch, 3)
    assert np.array_equal(got, oracle_lib.ext_select(kc, nodes, pods, 3, 0, quotas, rsv))
    node, total, reason = engine.replay(snap, batch, reasons=True)
    minors = engine.replay_minors(batch)
    st = oracle_lib.OracleState(kc, nodes)
    rnode, rtotal, rminors, qu, qnp, rreason = st.ext_replay(pods, quotas, reasons=True)
    assert np.array_equal(node, rnode) and np.array_equal(total, rtotal)
    assert np.array_equal(minors, rminors) and np.array_equal(reason, rreason)
