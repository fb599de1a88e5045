#!/bin/bash
# Mixed-cluster check: its parity tests, the config-6 bench line and a kernel trace of it.
#   bash tools/gpu_mixed.sh <tag>
set -o pipefail
TAG=${1:-m}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mixed.py tests/test_select_golden.py tests/test_numa_topology.py tests/test_numa_kat.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 \
    --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python bench.py --config 6 --no-replay --no-cpu-baseline > gpurun_out/bench6_$TAG.json 2> gpurun_out/bench6_$TAG.err || exit 2
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof6_$TAG" -o run --output-format csv -- \
    python3 "$R/bench.py" --config 6 --steps 10 --warmup 2 --no-replay --no-cpu-baseline --no-cycle > /dev/null || exit 3
cd "$R" || exit 1
f=$(find gpurun_out/prof6_$TAG -name "run_kernel_stats.csv" | head -1)
head -12 "$f"
python -c "import json;d=json.loads(open('gpurun_out/bench6_$TAG.json').read().strip().splitlines()[-1]);print('bench6', round(d['ms_per_step'],4), '%.4g'%d['value'], d['roofline'].get('kernel_avg_ms'), d.get('cycle',{}).get('ms_per_cycle'))"
