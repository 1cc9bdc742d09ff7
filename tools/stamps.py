"""Phase clocks of the fused encoder (diagnostic build lib/libbic_stamps.so, make stamps).
Runs one C3-sized encode and prints the median/mean per-wave time of each phase."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["BIC_LIB_PATH"] = os.path.join(ROOT, "binary-image-compression_amd", "lib", "libbic_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
import pybic  # noqa: E402

rows, cols, nplanes = 16384, 16384, 8
ctx = pybic.Context(0)
t = ctx.torch
g = t.Generator(device=ctx.dev)
g.manual_seed(1)
gray = t.randint(0, 256, (rows, cols), dtype=t.uint8, device=ctx.dev, generator=g)
planes = ctx.bitplanes_u8(gray, nplanes=8)
for _ in range(3):
    ctx.encode_planes2(planes, cols, True)
ctx.sync()
n = rows * nplanes * 8
buf = np.zeros(n, np.uint64)
lib = pybic.load()
lib.bic_debug_stamps.argtypes = [C.c_void_p, C.c_size_t]
assert lib.bic_debug_stamps(buf.ctypes.data, n) == 0
S = buf.reshape(-1, 8).astype(np.int64)
names = ["load", "wait_ones", "len+eg", "golomb", "barrier", "write"]
d = np.diff(S[:, :7], axis=1)
ok = (S[:, 0] > 0) & (d >= 0).all(axis=1)
d = d[ok]
tot = S[ok, 6] - S[ok, 0]
print(f"waves {ok.sum()}  per-wave total: median {np.median(tot):.0f}  mean {tot.mean():.0f} clk")
for i, nm in enumerate(names):
    print(f"{nm:10s} median {np.median(d[:, i]):9.0f}  mean {d[:, i].mean():9.0f}  share {d[:, i].sum() / tot.sum():6.3f}")
span = S[ok, 6].max() - S[ok, 0].min()
print("kernel span (clk)", span)
