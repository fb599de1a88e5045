#!/bin/bash
# PMC passes over the first 1024 pods of the config-5 replay (one step kernel per pod; gfx950 slot limits per pass):
#   bash tools/pmc_replay5.sh <tag>      -> gpurun_out/pmc5_<tag>/{sq,fetch,tcc}/run_counter_collection.csv
set -uo pipefail
TAG=${1:-r5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc5_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
P=("$R/tools/replay5_probe.py" --pods 1024)
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    SQ_WAIT_INST_ANY SQ_INSTS_VMEM -d "$OUT/sq" -o run --output-format csv -- python3 "${P[@]}" || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 "${P[@]}" || exit $?
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d "$OUT/tcc" -o run --output-format csv -- \
    python3 "${P[@]}" || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY -d "$OUT/sq2" -o run \
    --output-format csv -- python3 "${P[@]}" || exit $?
echo "pmc done: $OUT"
