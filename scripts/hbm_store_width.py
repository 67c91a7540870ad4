"""Achievable HBM rates with 16-byte vs 8-byte non-temporal stores (scripts/micro/
libhbm_probe.so modes 2/3 vs 7/8): does the decoder's 8-byte row store width cap it?"""
import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "micro", "libhbm_probe.so"))
lib.hbm_probe.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
for rep in range(2):
    for mode, name in ((2, "write 16B"), (7, "write 8B"), (3, "mix 2r3w 16B"), (8, "mix 2r3w 8B")):
        g = ctypes.c_double()
        rc = lib.hbm_probe(mode, 1 << 30, 10, ctypes.byref(g))
        print(f"{name:14s} {g.value:8.1f} GB/s rc={rc}")
