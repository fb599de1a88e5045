"""Debug aid: first divergence of the config-5 NUMA-mix replay (tests/test_gpu_numa.py::test_gpu_numa_replay_device).
Replays the first K pods on the device and in the oracle, then compares the node state (zone used, GPU free) and
pod K's verify row on both states."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import oracle_lib  # noqa: E402
from koordinator_amd import abi, engine, synth  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 2
cfg, nodes, pods, quotas, rsv = synth.cluster5(700, 600, seed_config=34, rsv_frac=0.0, numa="mix")
kc = cfg.kg_config()
kc.plugins &= ~abi.KG_PLUGIN_RSV
ctx = engine.Context(0)
snap = engine.Snapshot(ctx, kc, nodes)
snap.upload_quotas(quotas)
head = abi.take(pods, np.arange(K))
b = engine.PodBatch(ctx, head)
node, total, reason = engine.replay(snap, b, reasons=True)
minors = engine.replay_minors(b)
st = oracle_lib.OracleState(kc, nodes)
rnode, rtotal, rminors, qu, qnp, rreason = st.ext_replay(head, quotas, reasons=True)
print("device", node.tolist(), [hex(m) for m in minors], total.tolist())
print("oracle", rnode.tolist(), [hex(m) for m in rminors], rtotal.tolist())
ds = snap.read_state()
ot = st.table()
odf = st.dev_free()
for k in sorted(ot):
    if k in ds and ds[k].shape == ot[k].shape and not np.array_equal(ds[k], ot[k]):
        bad = np.argwhere(ds[k] != ot[k])
        print("state differs", k, bad[:4].tolist(), ds[k][tuple(bad[0])], ot[k][tuple(bad[0])])
if odf is not None and not np.array_equal(ds["dev_free"], odf):
    bad = np.argwhere(ds["dev_free"] != odf)
    print("dev_free differs", bad[:8].tolist())
    i = bad[0][0]
    print("device", ds["dev_free"][i].tolist())
    print("oracle", odf[i].tolist())
print("policy of placed nodes", [int(nodes["numa_policy"][i]) for i in node if i >= 0])
# pod K on both states
nxt = abi.take(pods, np.array([K]))
b2 = engine.PodBatch(ctx, nxt)
g = engine.eval_verify(snap, b2)
otab = dict(nodes)
otab.update(ot)
if odf is not None:
    otab["dev_free"] = odf
r = oracle_lib.ext_verify(kc, otab, nxt, quotas, None)
for name in ("status", "score_nrf", "score_numa", "score_dev", "total", "numa_zone"):
    a, c = getattr(g, name), getattr(r, name)
    if not np.array_equal(a, c):
        bad = np.argwhere(a != c)
        print("verify differs", name, len(bad), [(int(i), a[0, i].item(), c[0, i].item()) for _, i in bad[:6]])
print("done")
print("verify pod K totals at", [(i, int(g.total[0, i]), int(r.total[0, i]), int(g.score_dev[0, i]), int(g.status[0, i])) for i in (513, 271)])
print("pod K", {k: (v[K].tolist() if hasattr(v[K], "tolist") else v[K]) for k, v in pods.items() if k in ("dev_count", "dev_keys", "dev_flags", "numa_policy", "flags", "quota")})
print("verify argmax", int(np.argmax(g.total[0])), int(np.argmax(r.total[0])), "max score_dev", int(g.score_dev[0][g.status[0] == 0].max()))
snap2 = engine.Snapshot(ctx, kc, nodes)
snap2.upload_quotas(quotas)
b3 = engine.PodBatch(ctx, abi.take(pods, np.arange(K + 1)))
n3, t3, r3 = engine.replay(snap2, b3, reasons=True)
print("replay K+1", n3.tolist(), t3.tolist())
