# Sweep KG_SELECT_BLOCKS (base select workgroup target) on config 2, then the GPU suite once.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in 2048 4096 8192 1024; do
  KG_SELECT_BLOCKS=$b timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-replay > gpurun_out/tune_$b.json 2>gpurun_out/tune_$b.err || exit 1
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_tune.log 2>&1 || exit 2
