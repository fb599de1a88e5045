"""Diagnostic: first divergence of kg_replay from the oracle replay with reservation views, per plugin subset."""
import sys
sys.path[:0] = ["/root/repo", "/root/repo/tests"]
import numpy as np  # noqa: E402
import oracle_lib  # noqa: E402
import test_rsv_replay as T  # noqa: E402
from koordinator_amd import abi, engine  # noqa: E402

ctx = engine.Context(0)
for name, drop, cls_off in [("all", 0, False), ("no-quota", abi.KG_PLUGIN_QUOTA, False),
                            ("no-dev", abi.KG_PLUGIN_DEV, False), ("no-quota-dev", abi.KG_PLUGIN_QUOTA | abi.KG_PLUGIN_DEV, False),
                            ("no-class", 0, True)]:
    cfg, nodes, pods, quotas, rsv, _, _ = T._cluster(1200, 300, 81)
    if cls_off:
        pods["rsv_class"][:] = -1
    kc = cfg.kg_config()
    kc.plugins &= ~drop
    snap = engine.Snapshot(ctx, kc, nodes)
    if kc.plugins & abi.KG_PLUGIN_QUOTA:
        snap.upload_quotas(quotas)
    snap.upload_reservations(rsv)
    node, total, why = engine.replay(snap, engine.PodBatch(ctx, pods), reasons=True)
    onode, ototal, _, _, _, owhy = oracle_lib.OracleState(kc, nodes).ext_replay(
        pods, quotas if kc.plugins & abi.KG_PLUGIN_QUOTA else None, rsv=rsv, reasons=True)
    d = np.nonzero((node != onode) | (total != ototal))[0]
    j = int(d[0]) if len(d) else -1
    print(name, "first diff", j, (node[j], onode[j], total[j], ototal[j], pods["rsv_class"][j]) if j >= 0 else "", flush=True)
    snap.close()
ctx.close()
