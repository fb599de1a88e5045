"""VALU / SALU mix of a kernel's loops from hipcc -S output (issue-cost model of the select kernels).
Usage: python tools/isa_mix.py <file.s> <kernel-name-substring> [top]"""
import collections
import re
import sys


def loops(path, key):
    s = open(path).read()
    out = []
    for m in re.finditer(r"^(_Z\S+):\s*;", s, re.M):
        nm = m.group(1)
        if key not in nm:
            continue
        a = m.end()
        b = s.index(".Lfunc_end", a)
        lines = [l.split(";")[0].strip() for l in s[a:b].split("\n")]
        lines = [l for l in lines if l and not l.startswith(".") or re.match(r"^\.LBB\S+:$", l)]
        pos = {}
        for k, l in enumerate(lines):
            if re.match(r"^\.LBB\S+:$", l):
                pos[l[:-1]] = k
        regions = []
        for k, l in enumerate(lines):
            mm = re.match(r"^s_(cbranch_\w+|branch)\s+(\.LBB\S+)$", l)
            if mm and mm.group(2) in pos and pos[mm.group(2)] < k:
                regions.append((pos[mm.group(2)], k))
        for lo, hi in regions:
            ins = [l.split()[0] for l in lines[lo:hi + 1] if not l.endswith(":")]
            out.append((nm, lo, hi, ins))
    return out


def mix(ins):
    v = collections.Counter(i for i in ins if i.startswith("v_"))
    sa = sum(1 for i in ins if i.startswith("s_") and not i.startswith(("s_load", "s_buffer_load", "s_waitcnt", "s_cbranch", "s_branch")))
    sm = sum(1 for i in ins if i.startswith(("s_load", "s_buffer_load")))
    return v, sa, sm


if __name__ == "__main__":
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    found = loops(sys.argv[1], sys.argv[2])
    found.sort(key=lambda x: -len(x[3]))
    for nm, lo, hi, ins in found[:top]:
        v, sa, sm = mix(ins)
        f32 = sum(c for i, c in v.items() if re.search(r"_f32(_e\d+)?$", i) and "cvt" not in i and "cmp" not in i)
        print(f"{nm[:60]} lines {lo}-{hi}: {len(ins)} instructions, VALU {sum(v.values())} (f32 arith {f32}), "
              f"SALU {sa}, SMEM {sm}")
        print("  ", ", ".join(f"{i} {c}" for i, c in v.most_common()))
