#!/bin/bash
# Sweep KG_SELECT_BLOCKS (workgroup target of the base select launches) on config 2.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for b in ${*:-2048 4096 8192 16384}; do
  KG_SELECT_BLOCKS=$b timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-replay --no-cycle > gpurun_out/tune_$b.json 2>gpurun_out/tune_$b.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/tune_$b.json').read().strip().splitlines()[-1]);print($b, round(d['ms_per_step'],4), d['roofline'].get('kernel_avg_ms'))"
done
