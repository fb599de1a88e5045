set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_ext_parity.py tests/test_numa_topology.py tests/test_ext_kat.py tests/test_numa_kat.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ext_tests.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof5b -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config 5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench5b.json 2>gpurun_out/bench5b.err || exit 3
