#!/bin/bash
# Round-6 A/B of the config-2 select: koordinator_amd/ab/libkoordgpu_base.so (KG_LIB_PATH) vs the in-tree library,
# and KG_SELECT_BLOCKS variants of the in-tree one; each run under its own limit.  bash tools/ab_sel.sh <tag> [config]
set -o pipefail
TAG=${1:-ab}
C=${2:-2}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --config $C --steps 40 --warmup 5 --no-cpu-baseline --no-replay --no-cycle \
    > gpurun_out/ab_${TAG}_$name.json 2> gpurun_out/ab_${TAG}_$name.err || exit 2
  python3 -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_$name.json')); print('$name', round(d['ms_per_step'],4), d['roofline'].get('kernel_avg_ms'))"
}
for r in 1 2; do
  run base$r KG_LIB_PATH=$PWD/koordinator_amd/ab/libkoordgpu_base.so
  run new$r KG_X=0
done
for b in 4096 2048 1024; do run blk$b KG_SELECT_BLOCKS=$b; done
echo done
