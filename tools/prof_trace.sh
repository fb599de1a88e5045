#!/bin/bash
# Kernel trace + stats of short bench runs, one per config, with the top kernels printed:
#   bash tools/prof_trace.sh <tag> <config>...      (on the GPU box, from the repo root)
set -o pipefail
TAG=$1
shift
export TMPDIR=/tmp
R=$PWD
for c in "$@"; do
  O=$R/gpurun_out/trace${c}_$TAG
  mkdir -p "$O"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O" -o run --output-format csv -- \
      python3 "$R/bench.py" --config "$c" --steps 5 --warmup 1 --no-cpu-baseline --no-replay --no-cycle > "$O/bench.json") || exit 1
  python3 - "$O" "$c" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
r = list(csv.DictReader(open(f)))
tot = sum(float(x["TotalDurationNs"]) for x in r)
for x in sorted(r, key=lambda x: -float(x["TotalDurationNs"]))[:10]:
    print(sys.argv[2], x["Name"][:70], x["Calls"], round(float(x["AverageNs"]) / 1e6, 4), f'{100 * float(x["TotalDurationNs"]) / tot:.1f}%')
PY
done
echo done
