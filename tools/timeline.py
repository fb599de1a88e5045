"""Print one step's kernel timeline from a rocprofv3 kernel trace: python3 tools/timeline.py <run_kernel_trace.csv> [step]
(steps are split at each k_ext_gate dispatch; times in us relative to the step's first kernel start)."""
import csv
import sys

r = sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: int(x["Start_Timestamp"]))
step = int(sys.argv[2]) if len(sys.argv) > 2 else 3
starts = [i for i, x in enumerate(r) if "k_ext_gate" in x["Kernel_Name"]]
a = starts[step]
b = starts[step + 1] if step + 1 < len(starts) else len(r)
t0 = int(r[a]["Start_Timestamp"])
for x in r[a:b]:
    s, e = int(x["Start_Timestamp"]) - t0, int(x["End_Timestamp"]) - t0
    print(f'{x["Queue_Id"]:>3} {s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f}  grid {x["Grid_Size_X"]}x{x["Grid_Size_Y"]} '
          f'vgpr {x["VGPR_Count"]}  {x["Kernel_Name"][:60]}')
