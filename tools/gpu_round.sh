#!/bin/bash
# One GPU call: the -m gpu parity suite, the default bench line, config 4 / 5 bench lines and the
# rocprofv3 summaries of the config-2 select (each step under its own time limit; stops at the first failure).
#   bash tools/gpu_round.sh <tag> [steps...]   steps: tests bench bench4 bench5 prof2 prof4 prof5 (default: all)
set -o pipefail
TAG=${1:-r2}
shift
STEPS=${*:-tests bench bench4 bench5 prof2 prof4 prof5}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for s in $STEPS; do
  echo "== $s $(date +%T)"
  case $s in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
             > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; } ;;
    bench) timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 2 ;;
    bench4) timeout -k 10 400 python bench.py --config 4 --no-cpu-baseline > gpurun_out/bench4_$TAG.json 2> gpurun_out/bench4_$TAG.err || exit 3 ;;
    bench5) timeout -k 10 400 python bench.py --config 5 --steps 5 --warmup 1 > gpurun_out/bench5_$TAG.json 2> gpurun_out/bench5_$TAG.err || exit 4 ;;
    prof2) bash profiles/run_profile.sh ${TAG}_c2 2 > gpurun_out/prof2_$TAG.log 2>&1 || exit 5 ;;
    prof4) bash profiles/run_profile.sh ${TAG}_c4 4 > gpurun_out/prof4_$TAG.log 2>&1 || exit 7 ;;
    prof5) bash profiles/run_profile.sh ${TAG}_c5 5 > gpurun_out/prof5_$TAG.log 2>&1 || exit 6 ;;
  esac
done
echo "== done $(date +%T)"
