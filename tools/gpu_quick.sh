#!/bin/bash
# Quick GPU check: the -m gpu suite (optionally a -k filter) and config-2 / config-5 bench lines.
#   bash tools/gpu_quick.sh <tag> [pytest -k expression]
set -o pipefail
TAG=${1:-q}
K=${2:-}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
fi
tail -2 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-replay > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 2
KG_SELECT_UNFUSED=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-replay --no-cycle > gpurun_out/benchu_$TAG.json 2> gpurun_out/benchu_$TAG.err || exit 3
timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench5_$TAG.json 2> gpurun_out/bench5_$TAG.err || exit 4
for f in bench benchu bench5; do python -c "import json;d=json.loads(open('gpurun_out/${f}_$TAG.json').read().strip().splitlines()[-1]);print('$f', round(d['ms_per_step'],4), '%.4g'%d['value'], d['roofline'].get('kernel_avg_ms'))"; done
