#!/bin/bash
# rocprofv3 collection for the select kernel (run on the GPU box from the repo root):
#   bash profiles/run_profile.sh <tag>
# 1) kernel trace + stats of a bench run (per-kernel average durations);
# 2) separate PMC passes (gfx950 slot limits): FETCH_SIZE, WRITE_SIZE, SQ instruction mix / cycles.
set -uo pipefail
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
BENCH=("$R/bench.py" --steps 20 --warmup 2 --no-cpu-baseline --no-replay)
PMC_BENCH=("$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline --no-replay)

timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "${BENCH[@]}" > "$OUT/bench_under_trace.json" || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
    python3 "${PMC_BENCH[@]}" > /dev/null || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
    python3 "${PMC_BENCH[@]}" > /dev/null || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d "$OUT/pmc_sq" -o run --output-format csv -- \
    python3 "${PMC_BENCH[@]}" > /dev/null || exit $?
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INST_CYCLES_VMEM -d "$OUT/pmc_clk" \
    -o run --output-format csv -- python3 "${PMC_BENCH[@]}" > /dev/null || exit $?
echo "profile done: $OUT"
