"""Per-row phase clocks of k_emit_known (diagnostic build lib/libbic_stamps.so, make stamps): one
C3 encode_gray; per row: start, after EG, end, and its class (k = 0 copy, k = 1 image, other). Prints
the row cost by class and how unevenly the persistent waves finish (the tail of the launch)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["BIC_LIB_PATH"] = os.path.join(ROOT, "binary-image-compression_amd", "lib", "libbic_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
import pybic  # noqa: E402

rows, cols = 16384, 16384
ctx = pybic.Context(0)
t = ctx.torch
g = t.Generator(device=ctx.dev)
g.manual_seed(1)
gray = t.randint(0, 256, (rows, cols), dtype=t.uint8, device=ctx.dev, generator=g)
for _ in range(3):
    ctx.encode_gray(gray, nplanes=8)
ctx.sync()
n = rows * 8 * 8
buf = np.zeros(n, np.uint64)
lib = pybic.load()
lib.bic_debug_stamps.argtypes = [C.c_void_p, C.c_size_t]
assert lib.bic_debug_stamps(buf.ctypes.data, n) == 0
S = buf.reshape(-1, 8)
t0, t1, t2, info = (S[:, k].astype(np.int64) for k in range(4))
cls = (info & 3)
blk = (info >> 8) & 0xffffffff
wv = (info >> 40) & 0xff
ok = t0 > 0
base = t0[ok].min()
print("rows", ok.sum(), "kernel span clk", t2[ok].max() - base)
for c, name in ((1, "k=0 copy"), (2, "k=1 image"), (0, "other/rest")):
    m = ok & (cls == c)
    if m.any():
        print(f"{name:11s} rows {m.sum():7d}  row clk median {np.median(t2[m] - t0[m]):8.0f} mean {np.mean(t2[m] - t0[m]):8.0f}"
              f"  (EG part median {np.median(t1[m] - t0[m]):6.0f})")
wid = blk * 4 + wv
ends = {}
starts = {}
busy = {}
for i in np.nonzero(ok)[0]:
    w = int(wid[i])
    ends[w] = max(ends.get(w, 0), int(t2[i]))
    starts[w] = min(starts.get(w, 1 << 62), int(t0[i]))
    busy[w] = busy.get(w, 0) + int(t2[i] - t0[i])
e = np.array(sorted(v - base for v in ends.values()))
b = np.array(list(busy.values()))
print("waves", len(e), " finish clk: min", e.min(), "p10", int(np.percentile(e, 10)), "median", int(np.median(e)),
      "p90", int(np.percentile(e, 90)), "max", e.max())
print("busy clk per wave: min", b.min(), "median", int(np.median(b)), "max", b.max())
