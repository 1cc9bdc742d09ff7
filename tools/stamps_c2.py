"""Phase clocks of the single-kernel encoder at C2 (one 4096^2 plane, Golomb only, no predictor; the
diagnostic build lib/libbic_stamps.so): per-wave time of each phase and the launch's span."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["BIC_LIB_PATH"] = os.path.join(ROOT, "binary-image-compression_amd", "lib", "libbic_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
import pybic  # noqa: E402

rows, cols = 4096, 4096
ctx = pybic.Context(0)
t = ctx.torch
g = t.Generator(device=ctx.dev)
g.manual_seed(1)
planes = t.randint(0, 256, (rows * cols // 8,), dtype=t.uint8, device=ctx.dev, generator=g).view(t.int64).view(1, rows, cols // 64)
slot = ctx.slot_words(rows, cols, pybic.CODER_GOLOMB)
out, bits = ctx.empty_i64(1, slot), ctx.empty_i64(1)
for _ in range(5):
    ctx.encode_planes(planes, cols, False, pybic.CODER_GOLOMB, slot, out, bits)
ctx.sync()
n = rows * 8
buf = np.zeros(n, np.uint64)
lib = pybic.load()
lib.bic_debug_stamps.argtypes = [C.c_void_p, C.c_size_t]
assert lib.bic_debug_stamps(buf.ctypes.data, n) == 0
S = buf.reshape(-1, 8).astype(np.int64)
names = ["load+count", "ones lookback", "len", "bits lookback", "emit", "write"]
d = np.diff(S[:, :7], axis=1)
ok = (S[:, 0] > 0) & (d >= 0).all(axis=1)
d = d[ok]
tot = S[ok, 6] - S[ok, 0]
print(f"waves {ok.sum()}  per-wave total: median {np.median(tot):.0f}  mean {tot.mean():.0f} clk")
for i, nm in enumerate(names):
    print(f"{nm:14s} median {np.median(d[:, i]):9.0f}  mean {d[:, i].mean():9.0f}  max {d[:, i].max():9.0f}")
st = S[ok, 0] - S[ok, 0].min()
print("start offsets (clk): median", np.median(st), "max", st.max())
print("kernel span (clk)", S[ok, 6].max() - S[ok, 0].min())
