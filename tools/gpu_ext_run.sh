set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_ext_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ext_tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --config 5 --steps 5 --warmup 1 > gpurun_out/bench5.json 2> gpurun_out/bench5.err || exit 2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof5 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config 5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench5_trace.json 2>&1 || exit 3
