"""Regression guard for the round-1 miscompile (commit f4efa99): with the NUMA topology manager
(`numa_topology`) and the multi-zone Reserve split (`numa_reserve_split`) compiled as out-of-line device
functions, the round-1 build's device results stopped matching the oracle on gfx950 (ROCm 7.2 hipcc / clang).
The fault was not isolated to a smaller reproducer; the functions were made __forceinline__ and the results
matched again. This CPU test compiles the integer evaluation path (eval_pair + apply_assume, which contain both
functions) for gfx950 to assembly and fails if any out-of-line call (s_swappc_b64 / s_setpc_b64) appears in
it, so a toolchain or source change cannot bring the out-of-line form back silently. A self-check compiles a
deliberately __noinline__ helper and expects the call to show up."""
import os
import shutil
import subprocess

import pytest

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "koordinator_amd", "csrc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", f"-I{CSRC}",
         "--cuda-device-only", "-S"]

PROBE = r"""
#include <hip/hip_runtime.h>
#include "kg_eval.h"
namespace kg {
%s
__global__ void probe(NodeRec* nodes, ZoneRec* zones, PodsDev pods, KCfg cfg, uint64_t* out) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    const PodV p = load_pod(pods, 0);
    const PairOut o = eval_pair<false>(cfg, nodes[i].v, zones + i, p);
    apply_assume(cfg, nodes[i].v, zones + i, p, o.zone, 1);
    out[i] = pair_key(cfg, o, i) %s;
}
}
"""


def _compile(tmp_path, extra_fn="", extra_use=""):
    src = tmp_path / "probe.hip"
    src.write_text(PROBE % (extra_fn, extra_use))
    asm = tmp_path / "probe.s"
    subprocess.check_call([HIPCC, *FLAGS, str(src), "-o", str(asm)], stderr=subprocess.DEVNULL)
    return asm.read_text()


def _calls(asm: str) -> int:
    """Calls (s_swappc_b64) plus device functions emitted besides the kernel. s_setpc_b64 alone is not counted: the
    kernel's own long branches (beyond the 16-bit branch offset, s_getpc + s_add to a local .LBB label) use it."""
    lines = asm.splitlines()
    calls = sum(1 for line in lines if line.strip().startswith("s_swappc_b64"))
    funcs = sum(1 for line in lines if line.strip().startswith(".type") and line.strip().endswith("@function"))
    return calls + max(0, funcs - 1)


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc not in this image")
def test_eval_path_has_no_out_of_line_calls(tmp_path):
    asm = _compile(tmp_path)
    ver = subprocess.run([HIPCC, "--version"], capture_output=True, text=True).stdout.splitlines()[:1]
    assert _calls(asm) == 0, f"out-of-line device call in the evaluation path ({ver})"


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc not in this image")
def test_guard_detects_a_call(tmp_path):
    asm = _compile(tmp_path, "__device__ __attribute__((noinline)) uint64_t twist(uint64_t x) { return x * 3 + 1; }",
                   "^ twist(i)")
    assert _calls(asm) >= 1


# ---- the round-3 gpu_partition discrepancy: misaligned scalar-load bases ------------------------------------------
# Root cause (tools/dbg_part.hip, DESIGN.md "Toolchain findings"): for a loop over an array of 16-byte partition
# records reading a byte field (offset 2) and an int field (offset 4) at a wave-uniform index, the gfx950 backend
# strength-reduced both to one pointer (record + 2) and read the int with `s_load_dword sX, s[base], 0x2`. The sum is
# dword aligned, but the hardware drops SBASE[1:0] before adding the offset (tools/sload_probe.hip measures it), so
# the load returned the record's first dword and every score comparison failed. Fingerprint: a scalar load whose
# immediate offset is not a multiple of 4 (its base must then be misaligned for the access to be aligned).
_SLOAD = None


def _misaligned_sloads(asm_lines):
    import re
    global _SLOAD
    if _SLOAD is None:
        _SLOAD = re.compile(r"^\s*(s_(?:load|buffer_load)_\S+)\s+[^,]+,\s*[^,]+,\s*(\S+)(?:\s+offset:(0x[0-9a-fA-F]+))?")
    bad = []
    for line in asm_lines:
        m = _SLOAD.match(line)
        if m and any(g and g.startswith("0x") and int(g, 16) % 4 for g in (m.group(2), m.group(3))):
            bad.append(line.strip())
    return bad


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc not in this image")
def test_reproducer_shows_misaligned_sload(tmp_path):
    """Self-check of the detector: the reproducer's first gpu_partition form compiles to scalar loads at offset 2."""
    root = os.path.dirname(CSRC.rstrip("/").rsplit("/", 1)[0])
    asm = tmp_path / "part.s"
    subprocess.check_call([HIPCC, *FLAGS, os.path.join(root, "tools", "dbg_part.hip"), "-o", str(asm)],
                          stderr=subprocess.DEVNULL)
    assert len(_misaligned_sloads(asm.read_text().splitlines())) >= 1


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"), reason="llvm-objdump not in this image")
def test_library_has_no_misaligned_sloads(tmp_path):
    """The built engine (every gfx950 code object in libkoordgpu.so) carries no scalar load of the miscompiled form,
    and no out-of-line device call (s_swappc_b64): round 4 found the config-5 view kernels calling their evaluation
    lambda out of line (its state through scratch memory) when it had two call sites."""
    root = os.path.dirname(CSRC.rstrip("/").rsplit("/", 1)[0])
    lib = os.path.join(root, "koordinator_amd", "libkoordgpu.so")
    if not os.path.exists(lib):
        pytest.skip("libkoordgpu.so not built")
    import sys
    sys.path.insert(0, os.path.join(root, "tools"))
    from code_objects import extract
    files = extract(lib, str(tmp_path))
    assert files
    import re
    for f in files:
        with open(f) as fh:
            lines = fh.read().splitlines()
        bad = _misaligned_sloads(lines)
        assert not bad, (f, bad[:4])
        calls, cur = [], None
        for line in lines:
            m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
            if m:
                cur = m.group(1)
            elif "s_swappc_b64" in line:
                calls.append(cur)
        assert not calls, (f, sorted(set(calls))[:4])
