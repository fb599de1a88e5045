"""Per-kernel resource usage (VGPRs, SGPRs, scratch, spills, LDS) from the AMDGPU metadata of the gfx950 code
objects in a host ELF:  python tools/kernel_resources.py koordinator_amd/libkoordgpu.so [name-substring ...]"""
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from code_objects import bundles  # noqa: E402

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def kernels(elf_bytes: bytes):
    with tempfile.NamedTemporaryFile(suffix=".elf") as f:
        f.write(elf_bytes)
        f.flush()
        txt = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True).stdout
    for blk in re.split(r"\n  - \.agpr_count:", txt)[1:]:
        def g(key):
            m = re.search(r"\n    \." + key + r":\s+(\S+)", blk)
            return m.group(1) if m else "?"
        yield dict(name=g("name"), vgpr=g("vgpr_count"), sgpr=g("sgpr_count"), scratch=g("private_segment_fixed_size"),
                   vspill=g("vgpr_spill_count"), sspill=g("sgpr_spill_count"), lds=g("group_segment_fixed_size"))


if __name__ == "__main__":
    data = open(sys.argv[1], "rb").read()
    subs = sys.argv[2:]
    for _, blob in bundles(data):
        for k in kernels(blob):
            if not subs or any(s in k["name"] for s in subs):
                print(f'{k["name"][:90]:90s} vgpr {k["vgpr"]:>4} sgpr {k["sgpr"]:>4} scratch {k["scratch"]:>6} '
                      f'vspill {k["vspill"]:>4} sspill {k["sspill"]:>4} lds {k["lds"]:>6}')
