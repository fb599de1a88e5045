#!/bin/bash
# Every bench line on one GPU: config 2 (with replay at 10k / 100k nodes, cycle and CPU baselines), 4, 5, 6.
#   bash tools/gpu_bench_all.sh <tag>
set -o pipefail
TAG=${1:-b}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 2
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline > gpurun_out/bench4_$TAG.json 2> gpurun_out/bench4_$TAG.err || exit 3
timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 > gpurun_out/bench5_$TAG.json 2> gpurun_out/bench5_$TAG.err || exit 4
timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline > gpurun_out/bench6_$TAG.json 2> gpurun_out/bench6_$TAG.err || exit 5
for f in bench bench4 bench5 bench6; do python -c "
import json;d=json.loads(open('gpurun_out/${f}_$TAG.json').read().strip().splitlines()[-1])
print('$f', round(d['ms_per_step'],4), '%.4g'%d['value'], d['roofline'].get('kernel_avg_ms'), (d.get('cycle') or {}).get('ms_per_cycle'),
      (d.get('replay') or {}).get('pods_placed_per_s'), (d.get('replay_100k') or {}).get('pods_placed_per_s'), (d.get('cpu_baseline') or {}).get('value'))"; done
