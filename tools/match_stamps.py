"""Phase clocks of the row workgroup of bic_match_encode (diagnostic build lib/libbic_stamps.so,
make stamps): per tile, the clocks between the phase marks of k_match_team's main workgroup."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["BIC_LIB_PATH"] = os.path.join(ROOT, "binary-image-compression_amd", "lib", "libbic_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pybic  # noqa: E402
from oracle_lib import text_plane, pack_rows  # noqa: E402

rows = int(os.environ.get("ROWS", "512"))
cols = int(os.environ.get("COLS", "512"))
W, R = 16, 128
ctx = pybic.Context(0)
ctx.set_match_parts(int(os.environ.get("PARTS", "0")))
rng = np.random.default_rng(1)
kind = os.environ.get("INPUT", "rand50")
I = {"text": lambda: text_plane(1, rows, cols), "blank": lambda: np.zeros((rows, (cols + 63) // 64), np.uint64),
     "rand50": lambda: pack_rows(rng.random((rows, cols)) < 0.5)}[kind]()
d = ctx.to_dev(I)
e = pybic.enum_table(W)
for _ in range(3):
    ctx.match_encode(d, cols, W, 0, R, e)
ctx.sync()
nt = (rows // W) * (cols // W)
buf = np.zeros(nt * 16, np.uint64)
lib = pybic.load()
lib.bic_debug_match_stamps.argtypes = [C.c_void_p, C.c_size_t]
assert lib.bic_debug_match_stamps(buf.ctypes.data, nt * 16) == 0
S16 = buf.reshape(-1, 16).astype(np.int64)
S = S16[:, :8]
X = S16[:, 8:11]
names = ["wait+load", "P", "publish", "scan", "helpers", "decide", "barrier", "next"]
d = np.diff(S, axis=1)
nxt = np.r_[S[1:, 0] - S[:-1, 7], 0]
nx = cols // W
print(f"{kind} {rows}x{cols}: tiles {nt}, span {S[:, 7].max() - S[:, 0].min()} clk")
for ti in [0, 1, rows // W // 2, rows // W - 1]:
    sl = slice(ti * nx + 2, (ti + 1) * nx)
    med = [int(np.median(d[sl, i])) for i in range(7)]
    print(f"row {ti:3d}: " + "  ".join(f"{n}={m}" for n, m in zip(names, med)) +
          f"  next={int(np.median(nxt[sl][:-1]))}  tile={int(np.median(S[sl, 7] - S[sl, 0]))}")
    print(f"        scan: pre={int(np.median(X[sl, 0] - S[sl, 3]))} tasks={int(np.median(X[sl, 1] - X[sl, 0]))} "
          f"wavemin={int(np.median(X[sl, 2] - X[sl, 1]))} red={int(np.median(S[sl, 4] - X[sl, 2]))}")
