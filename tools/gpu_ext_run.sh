# One GPU call: whole GPU parity suite, config-5 bench, rocprofv3 kernel stats of the config-5 bench.
#   bash tools/gpu_ext_run.sh <tag>
set -o pipefail
TAG=${1:-r1}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config 5 --steps 5 --warmup 1 > gpurun_out/bench5_$TAG.json 2> gpurun_out/bench5_$TAG.err || exit 2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof5_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config 5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench5t_$TAG.json 2>gpurun_out/bench5t_$TAG.err || exit 3
