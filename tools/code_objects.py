"""Extract the gfx950 code objects embedded in a host ELF (.hip_fatbin clang offload bundles) and disassemble them.

    python tools/code_objects.py koordinator_amd/libkoordgpu.so OUTDIR   -> OUTDIR/co<k>.elf, OUTDIR/co<k>.s
"""
import os
import struct
import subprocess
import sys

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def bundles(data: bytes):
    pos = 0
    while True:
        at = data.find(MAGIC, pos)
        if at < 0:
            return
        n, = struct.unpack_from("<Q", data, at + 24)
        off = at + 32
        for _ in range(n):
            o, size, tlen = struct.unpack_from("<QQQ", data, off)
            triple = data[off + 24: off + 24 + tlen].decode()
            off += 24 + tlen
            if "gfx950" in triple and size:
                yield triple, data[at + o: at + o + size]
        pos = at + len(MAGIC)


def extract(path: str, out: str):
    os.makedirs(out, exist_ok=True)
    data = open(path, "rb").read()
    files = []
    for k, (triple, blob) in enumerate(bundles(data)):
        elf = os.path.join(out, f"co{k}.elf")
        open(elf, "wb").write(blob)
        asm = os.path.join(out, f"co{k}.s")
        with open(asm, "w") as f:
            subprocess.check_call([OBJDUMP, "-d", "--mcpu=gfx950", elf], stdout=f)
        files.append(asm)
    return files


if __name__ == "__main__":
    print("\n".join(extract(sys.argv[1], sys.argv[2])))
