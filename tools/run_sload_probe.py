"""Run tools/sload_probe.hip's kernel once and print which dword the misaligned-base scalar load returned."""
import ctypes as C
import os
import sys

lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsload_probe.so"))
out = (C.c_uint32 * 2)()
rc = lib.sload_probe(out)
if rc:
    sys.exit(f"probe failed: {rc}")
v0, v1 = out[0], out[1]
print(f"s_load_dword base=buf+2 offset=0x2 -> {v0:#010x} ({'buf[0]: SBASE[1:0] dropped' if v0 == 0x11111111 else 'buf[1]: sum used' if v0 == 0x22222222 else 'other'}); control base=buf+4 -> {v1:#010x}")
