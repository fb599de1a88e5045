#!/bin/bash
# rocprofv3 collection for the select kernels (run on the GPU box from the repo root):
#   bash profiles/run_profile.sh <tag> [config]      (config 2 default; 4 = 100k nodes top-3; 5 = the config-5 plugin set; 6 = mixed)
# 1) kernel trace + stats of a bench run (per-kernel average durations);
# 2) separate PMC passes (gfx950 slot limits): FETCH_SIZE, WRITE_SIZE, SQ instruction mix / cycles;
# 3) tools/pmc_summary.py -> gpurun_out/prof_<tag>/summary.json (copy it to profiles/ to commit).
set -uo pipefail
TAG=${1:-r2}
CFG=${2:-2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
BENCH=("$R/bench.py" --config "$CFG" --steps 20 --warmup 2 --no-cpu-baseline --no-replay --no-cycle)
PMC_BENCH=("$R/bench.py" --config "$CFG" --steps 4 --warmup 1 --no-cpu-baseline --no-replay --no-cycle)

timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "${BENCH[@]}" > "$OUT/bench_under_trace.json" || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
    python3 "${PMC_BENCH[@]}" > /dev/null || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
    python3 "${PMC_BENCH[@]}" > /dev/null || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d "$OUT/pmc_sq" -o run --output-format csv -- \
    python3 "${PMC_BENCH[@]}" > /dev/null || exit $?
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INST_CYCLES_VMEM -d "$OUT/pmc_clk" \
    -o run --output-format csv -- python3 "${PMC_BENCH[@]}" > /dev/null || exit $?
cd "$R" || exit 1
if [ "$CFG" = "4" ]; then  # top-3: per-chunk partials merged by k_merge_list inside the bracket
    python3 tools/pmc_summary.py "$OUT" "$OUT/summary.json" "k_select<" "k_select1<" "k_big_sel" "k_merge" || exit $?
elif [ "$CFG" = "5" ]; then
    python3 tools/pmc_summary.py "$OUT" "$OUT/summary.json" "k_ext_select" "k_ext_stats" "k_ext_fix_rows" "k_dev_sum" "k_gpu_zone_sum" \
        "k_rdev_codes" "k_ext_gate" "k_special_scan" "k_scatter_keys" "k_select<" "k_select1<" "k_big_sel" || exit $?
elif [ "$CFG" = "6" ]; then  # mixed cluster: fast lanes, pruned F_BIG pairs, pruned integer (LSR) lanes
    python3 tools/pmc_summary.py "$OUT" "$OUT/summary.json" "k_select<" "k_select1<" "k_big_init" "k_big_sel" \
        "k_int_seed" "k_int_filter" "k_int_pairs" "k_merge" || exit $?
else
    python3 tools/pmc_summary.py "$OUT" "$OUT/summary.json" "k_select<" "k_select1<" "k_big_init" || exit $?
fi
echo "profile done: $OUT"
