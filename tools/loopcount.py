"""Count the instructions of each basic block of one kernel in an assembly listing (loop sizing)."""
import collections
import re
import sys


def blocks(asm_path, kernel):
    s = open(asm_path).read()
    i = s.index(kernel + ":")
    j = s.index(".Lfunc_end", i)
    cur, out = "entry", collections.OrderedDict()
    for line in s[i:j].splitlines():
        t = line.strip()
        m = re.match(r"^(\.LBB\w+):", t)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        out.setdefault(cur, []).append(t.split()[0])
    return out


if __name__ == "__main__":
    for name, ins in blocks(sys.argv[1], sys.argv[2]).items():
        v = sum(1 for x in ins if x.startswith("v_"))
        sm = sum(1 for x in ins if x.startswith("s_"))
        print(f"{name:12s} total={len(ins):4d} valu={v:4d} salu/smem={sm:4d}")
