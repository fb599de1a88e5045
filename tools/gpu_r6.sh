#!/bin/bash
# Round-6 GPU steps (each under its own limit; the script stops at the first failure):
#   bash tools/gpu_r6.sh <tag> [steps...]   steps: probe5 trace5 bench2 bench4 bench5 bench6 tests sel smoke
#   (sel: the tests named by $KG_TESTS)
set -o pipefail
TAG=${1:-r6}
shift
STEPS=${*:-probe5 trace5}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in $STEPS; do
  echo "== $s $(date +%T)"
  case $s in
    probe5) timeout -k 10 300 python3 tools/replay5_probe.py > gpurun_out/replay5_$TAG.json 2> gpurun_out/replay5_$TAG.err || exit 1 ;;
    trace5) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r5trace_$TAG" -o run \
              --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/replay5_probe.py" > gpurun_out/replay5_trace_$TAG.json \
              2> gpurun_out/replay5_trace_$TAG.err || exit 2 ;;
    bench2) timeout -k 10 400 python3 bench.py > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err || exit 3 ;;
    bench4) timeout -k 10 400 python3 bench.py --config 4 --no-cpu-baseline > gpurun_out/bench4_$TAG.json 2> gpurun_out/bench4_$TAG.err || exit 4 ;;
    bench5) timeout -k 10 400 python3 bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench5_$TAG.json 2> gpurun_out/bench5_$TAG.err || exit 5 ;;
    bench6) timeout -k 10 400 python3 bench.py --config 6 --no-cpu-baseline --no-cycle > gpurun_out/bench6_$TAG.json 2> gpurun_out/bench6_$TAG.err || exit 6 ;;
    tests) timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 7; } ;;
    sel) timeout -k 10 600 python3 -u -m pytest $KG_TESTS -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_sel_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_sel_$TAG.log; exit 9; } ;;
    smoke) timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 8 ;;
  esac
done
echo "== done $(date +%T)"
