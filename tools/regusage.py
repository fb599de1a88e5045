"""Tabulate per-kernel register usage of the engine's gfx950 code object (compiler resource remarks)."""
import re
import subprocess
import sys

SRC = sys.argv[2] if len(sys.argv) > 2 else "koordinator_amd/csrc/kg_kernels.hip"


def main(pattern=""):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-fno-slp-vectorize",
           "--cuda-device-only", "-c", SRC, "-o", "/tmp/kg_regusage.o", "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    for r in rows:
        if pattern in r["name"]:
            print(f'{r["name"][:70]:70s} S={r.get("TotalSGPRs")} V={r.get("VGPRs")} '
                  f'Sspill={r.get("SGPRs Spill")} Vspill={r.get("VGPRs Spill")} occ={r.get("Occupancy [waves/SIMD]")} '
                  f'LDS={r.get("LDS Size [bytes/block]")}')


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "")
