#!/bin/bash
# Config-5 A/B: bench lines with the pass-1 pair table (default) and without it (KG_PAIRS_GB=0), and a kernel
# trace of each.   bash tools/gpu_c5.sh <tag>
set -o pipefail
TAG=${1:-c5}
R=$GRAFT_REPO_ROOT
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in pairs nopairs; do
  if [ $v = nopairs ]; then export KG_PAIRS_GB=0; fi
  timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench5_${TAG}_$v.json 2> gpurun_out/bench5_${TAG}_$v.err || exit 2
  cd /tmp || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof5_${TAG}_$v" -o run --output-format csv -- \
      python3 "$R/bench.py" --config 5 --steps 10 --warmup 2 --no-cpu-baseline > /dev/null || exit 3
  cd "$R" || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/bench5_${TAG}_$v.json').read().strip().splitlines()[-1]);print('bench5 $v', round(d['ms_per_step'],4), '%.4g'%d['value'])"
  f=$(find gpurun_out/prof5_${TAG}_$v -name "run_kernel_stats.csv" | head -1)
  cut -c1-60,200-260 "$f" | head -14
done
