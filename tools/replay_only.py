"""Config-3 replay alone (10k nodes x 50k pods), for kernel traces: python tools/replay_only.py [reps]."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from koordinator_amd import engine, synth  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    cfg, nodes, pods = synth.cluster(3)
    kc = cfg.kg_config()
    ctx = engine.Context(0)
    batch = engine.PodBatch(ctx, pods)
    for r in range(reps):
        snap = engine.Snapshot(ctx, kc, nodes)
        t = time.perf_counter()
        node, _ = engine.replay(snap, batch)
        dt = time.perf_counter() - t
        print(f"rep {r}: {len(node) / dt:.0f} pods/s ({dt * 1e6 / len(node):.2f} us/pod), placed {(node >= 0).sum()}",
              flush=True)
        snap.close()
    ctx.close()


if __name__ == "__main__":
    main()
