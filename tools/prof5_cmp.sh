export TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out/prof5_r4b gpurun_out/prof5_r4c
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof5_r4b -o run --output-format csv -- python3 $R/bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline --no-replay --no-cycle > $R/gpurun_out/prof5_r4b/bench.json || exit 1
KG_NO_GZ=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof5_r4c -o run --output-format csv -- python3 $R/bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline --no-replay --no-cycle > $R/gpurun_out/prof5_r4c/bench.json || exit 2
cd $R
python3 - <<'PY'
import csv
for d in ("prof5_r4b", "prof5_r4c"):
    r = list(csv.DictReader(open(f"gpurun_out/{d}/run_kernel_stats.csv")))
    for x in sorted(r, key=lambda x: -float(x["TotalDurationNs"]))[:6]:
        print(d, x["Name"][:60], x["Calls"], round(float(x["AverageNs"]) / 1e6, 3))
PY
