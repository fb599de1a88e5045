"""VALU issue-cost model of the select kernels from their ISA (hipcc -S of the kernel sources, the build's
flags): per kernel, the main loop's VALU instructions split into f32 arithmetic (2 cycles per wave64
instruction on a SIMD) and the rest (4 cycles: f64, 64-bit and 32-bit integer, compares, conversions,
v_cndmask), the costs measured chip-wide by tools/ubench_valu.hip (profiles/r2/ubench_valu.txt).
Writes profiles/valu_mix.json stamped with bench.kernel_source_hash(); bench.py prices the PMC VALU
counts with it (roofline.issue).
Usage: python tools/valu_mix.py [out.json]"""
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import isa_mix  # noqa: E402

CYC_F32, CYC_OTHER = 2.0, 4.0
KERNELS = ("k_select1", "k_select", "k_ext_select", "k_ext_select_sp", "k_ext_stats", "k_ext_stats_sp", "k_ext_stats_views",
           "k_dev_sum", "k_rdev_codes", "k_big_init", "k_big_sel")


def canon_mangled(nm):
    """_ZN2kg9k_select1ILj7ELi0EEEv... -> k_select1<7,0>; _ZN2kg9k_dev_sumEPK... -> k_dev_sum"""
    m = re.match(r"_ZN2kg(\d+)", nm)
    if not m:
        return None
    name = nm[m.end():m.end() + int(m.group(1))]
    rest = nm[m.end() + int(m.group(1)):]
    if not rest.startswith("I"):
        return name
    m = re.match(r"I(.*?)EEv", rest)
    if not m:
        return None
    args = re.findall(r"L([jib])(\d+)E", m.group(1))
    out = []
    for t, v in args:
        out.append(("true" if v == "1" else "false") if t == "b" else v)
    return f"{name}<{','.join(out)}>"


def canon_demangled(nm):
    """void kg::k_select1<7u, 0>(...) -> k_select1<7,0>"""
    m = re.search(r"kg::(\w+)<([^>]*)>", nm)
    if not m:
        m2 = re.search(r"kg::(\w+)\(", nm)
        return m2.group(1) if m2 else None
    args = [a.strip().rstrip("u") for a in m.group(2).split(",")]
    return f"{m.group(1)}<{','.join(args)}>"


def main(out):
    import __graft_entry__ as g
    import bench

    res = {"kernel_source_hash": bench.kernel_source_hash(), "cycles": {"f32": CYC_F32, "other": CYC_OTHER},
           "note": "main-loop VALU mix per kernel; cycles per wave64 VALU instruction on one SIMD measured by "
                   "tools/ubench_valu.hip (profiles/r2/ubench_valu.txt: v_mul_f32 2.2, f64 / integer / compare / "
                   "convert / cndmask 4.0-4.2 chip-wide)",
           "kernels": {}}
    with tempfile.TemporaryDirectory() as td:
        for src in ("kg_kernels.hip", "kg_ext.hip"):
            s = os.path.join(g.CSRC, src)
            asm = os.path.join(td, src + ".s")
            flags = [f for f in g.HIP_FLAGS if f not in ("-fPIC",)]
            subprocess.check_call([g.HIPCC, *flags, "-S", "--cuda-device-only", s, "-o", asm],
                                  stderr=subprocess.DEVNULL)
            for nm, lo, hi, ins in isa_mix.loops(asm, "k_"):
                key = canon_mangled(nm)
                if key is None or key.split("<")[0] not in KERNELS:
                    continue
                v, sa, sm = isa_mix.mix(ins)
                f32 = sum(c for i, c in v.items() if re.search(r"_f32(_e\d+)?$", i) and "cvt" not in i and "cmp" not in i)
                tot = sum(v.values())
                cur = res["kernels"].get(key)
                if cur is None or tot > cur["valu"]:  # the kernel's largest loop
                    res["kernels"][key] = {"valu": tot, "f32": f32, "salu": sa,
                                           "cyc_per_valu": (CYC_F32 * f32 + CYC_OTHER * (tot - f32)) / max(tot, 1)}
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    for k, v in sorted(res["kernels"].items()):
        print(k, v)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "valu_mix.json"))
