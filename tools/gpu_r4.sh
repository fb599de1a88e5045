#!/bin/bash
# Round-4 GPU call: the -m gpu suite (optional -k), then the named bench lines.
#   bash tools/gpu_r4.sh <tag> "<pytest -k expr or ALL or NONE>" [bench configs...]
set -o pipefail
TAG=${1:-r4}
K=${2:-ALL}
shift 2
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ "$K" != "NONE" ]; then
  if [ "$K" = "ALL" ]; then KA=(); else KA=(-k "$K"); fi
  timeout -k 10 600 python -u -m pytest tests -m gpu --maxfail=${MAXFAIL:-1} -q --timeout 120 --timeout-method thread "${KA[@]}" \
    > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
  tail -2 gpurun_out/gpu_tests_$TAG.log
fi
for c in "$@"; do
  case $c in
    2) timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err || exit 2 ;;
    4) timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline > gpurun_out/bench4_$TAG.json 2> gpurun_out/bench4_$TAG.err || exit 4 ;;
    5) timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench5_$TAG.json 2> gpurun_out/bench5_$TAG.err || exit 5 ;;
    6) timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline > gpurun_out/bench6_$TAG.json 2> gpurun_out/bench6_$TAG.err || exit 6 ;;
    full) timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 7 ;;
  esac
  f=gpurun_out/bench${c}_$TAG.json; [ "$c" = full ] && f=gpurun_out/bench_$TAG.json
  python -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$c', round(d['ms_per_step'],4), '%.4g'%d['value'], (d.get('roofline') or {}).get('kernel_avg_ms'))"
done
echo done
