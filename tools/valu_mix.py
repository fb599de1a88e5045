"""VALU issue-cost model of the select kernels from their ISA (hipcc -S of the kernel sources, the build's
flags): per kernel, the main loop's VALU instructions, each priced by its opcode's chip-wide issue cost measured on
the MI355X (tools/gen_ubench_ops.py -> profiles/r5/ubench_ops.jsonl: cycles per wave64 instruction per SIMD at the
in-kernel clock). Measured on gfx950: 32-bit add / sub / and / or / xor / lshrrev / mov and f32 add / mul issue every
~2.3 cycles; 64-bit, f64, compares, conversions, cndmask, 32-bit multiplies, shifts left, min / max, bfe, add3 and the
carry forms every ~4.1; rcp_f32 8.2, rcp_f64 16.2. Opcodes the table does not hold are priced at 4.1 (their class).
Writes profiles/valu_mix.json stamped with bench.kernel_source_hash(); bench.py prices the PMC VALU counts with it
(roofline.issue).
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

OPS_TABLE = os.path.join(ROOT, "profiles", "r5", "ubench_ops.jsonl")
CYC_DEFAULT = 4.1
KERNELS = ("k_select1", "k_select", "k_ext_select", "k_ext_select_sp", "k_ext_select_xs", "k_ext_select_c1", "k_ext_stats", "k_ext_stats_sp",
           "k_ext_stats_c1", "k_ext_stats_views", "k_dev_sum", "k_rdev_codes", "k_gpu_zone_sum", "k_big_init", "k_big_sel",
           "k_int_seed", "k_int_filter", "k_int_pairs", "k_ext_replay", "k_replay")


def op_costs():
    """opcode -> cycles from the committed microbenchmark (v_cndmask_b32_e32 is priced like its e64 form: the
    benchmark's e32 loop ran 19.7 cycles, an artefact of that loop the compiled kernels do not show)."""
    cost = {}
    with open(OPS_TABLE) as f:
        for line in f:
            d = json.loads(line)
            cost[d["op"]] = d["cycles"]
    cost["v_cndmask_b32_e32"] = cost.get("v_cndmask_b32_e64", CYC_DEFAULT)
    return cost


def price(op, cost):
    """Issue cost of one opcode of the ISA listing (suffixes _e32 / _e64 / _dpp / _sdwa folded where the table has the
    plain form)."""
    if op in cost:
        return cost[op]
    base = re.sub(r"_(e32|e64|dpp|sdwa)$", "", op)
    if base in cost:
        return cost[base]
    if base in ("v_subrev_u32",):
        return cost.get("v_sub_u32", CYC_DEFAULT)
    if base in ("v_sub_f32", "v_subrev_f32"):
        return cost.get("v_add_f32", CYC_DEFAULT)
    if base in ("v_fmac_f32", "v_mac_f32"):
        return cost.get("v_fma_f32", CYC_DEFAULT)
    if base.startswith(("v_rcp_", "v_rsq_", "v_sqrt_")):
        return cost.get("v_rcp_f64" if base.endswith("f64") else "v_rcp_f32", CYC_DEFAULT)
    return CYC_DEFAULT


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

    cost = op_costs()
    res = {"kernel_source_hash": bench.kernel_source_hash(), "cycles": {"table": "profiles/r5/ubench_ops.jsonl",
                                                                        "default": CYC_DEFAULT},
           "note": "main-loop VALU mix per kernel, each opcode priced by its measured chip-wide issue cost on MI355X "
                   "(tools/gen_ubench_ops.py: ~2.3 cycles for 32-bit add / logic / lshr / mov and f32 add / mul, ~4.1 "
                   "for 64-bit, f64, compare, convert, cndmask, mul / shl / min / max forms)",
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
                tot = sum(v.values())
                cyc = sum(c * price(i, cost) for i, c in v.items())
                fast = sum(c for i, c in v.items() if price(i, cost) < 3.0)
                cur = res["kernels"].get(key)
                if cur is None or tot > cur["valu"]:  # the kernel's largest loop
                    res["kernels"][key] = {"valu": tot, "fast": fast, "salu": sa, "cyc_per_valu": cyc / max(tot, 1)}
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    for k, v in sorted(res["kernels"].items()):
        print(k, v)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "valu_mix.json"))
