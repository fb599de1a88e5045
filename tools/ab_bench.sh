#!/bin/bash
# A/B of two engine builds on the GPU box: bench.py config 2 (and 5) with tools/ab/libkoordgpu_base.so
# (KG_LIB_PATH) and with the in-tree library, alternating, each run under its own time limit.
#   bash tools/ab_bench.sh <tag> [configs...]
set -o pipefail
TAG=${1:-ab}
shift
CFGS=${*:-2}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for c in $CFGS; do
  for round in 1 2; do
    KG_LIB_PATH=$PWD/tools/ab/libkoordgpu_base.so timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-replay --no-cycle \
      > gpurun_out/ab_${TAG}_c${c}_base_$round.json 2> gpurun_out/ab_${TAG}_c${c}_base_$round.err || exit 2
    timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-replay --no-cycle \
      > gpurun_out/ab_${TAG}_c${c}_new_$round.json 2> gpurun_out/ab_${TAG}_c${c}_new_$round.err || exit 3
  done
done
for f in gpurun_out/ab_${TAG}_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],4), d['roofline'].get('kernel_avg_ms'))"; done
