#!/bin/bash
# One GPU call: GPU parity suite, default bench line, config-5 bench, rocprofv3 summaries.
#   bash tools/gpu_full_run.sh <tag>
set -o pipefail
TAG=${1:-r1}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 2
timeout -k 10 400 python bench.py --config 5 --steps 5 --warmup 1 > gpurun_out/bench5_$TAG.json 2> gpurun_out/bench5_$TAG.err || exit 3
bash profiles/run_profile.sh $TAG || exit 4
