#!/bin/bash
# GPU allocator check: its KATs, the config-5 parity tests (topology / partition clusters), the golden select.
#   bash tools/gpu_f4.sh <tag>
set -o pipefail
TAG=${1:-f4}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_alloc_kat.py tests/test_ext_parity.py tests/test_ext_kat.py tests/test_batch.py \
    tests/test_select_golden.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 \
    || { tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench5_$TAG.json 2> gpurun_out/bench5_$TAG.err || exit 2
python -c "import json;d=json.loads(open('gpurun_out/bench5_$TAG.json').read().strip().splitlines()[-1]);print('bench5', round(d['ms_per_step'],4), '%.4g'%d['value'])"
KG_TRACE_FIX=1 timeout -k 10 300 python bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline --no-cycle --no-replay 2>&1 >/dev/null | grep "re-ran" | head -3 || true
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof5_$TAG" -o run --output-format csv -- \
    python3 "$R/bench.py" --config 5 --steps 5 --warmup 1 --no-cpu-baseline --no-cycle > /dev/null || exit 3
cd "$R" || exit 1
f=$(find gpurun_out/prof5_$TAG -name "run_kernel_stats.csv" | head -1)
head -14 "$f"
