"""diagnostic: the FIRST encode of a process -- bad Golomb planes for one configuration (argv: rows cols
mode one_stream warm) -- warm: 0 none, 1 an encode of another shape first, 2 a 1 s sleep after the
context is made"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pybic  # noqa: E402
from oracle_lib import Oracle  # noqa: E402

rows, cols, mode, one, warm = (int(x) for x in sys.argv[1:6])
o = Oracle()
img = o.gen_bytes(rows * 13 + cols, rows * cols).reshape(rows, cols)
P = o.bitplanes(img, 8)
exp = [o.encode_plane(P[k], cols, 1, 0) for k in range(8)]
ctx = pybic.Context(0)
ctx.set_encoder("staged")
ctx.set_eg_source(mode)
ctx.set_one_stream(bool(one))
g = ctx.torch.from_numpy(img).to(ctx.dev)
if warm == 1:
    w = ctx.torch.zeros((64, 8192), dtype=ctx.torch.uint8, device=ctx.dev)
    ctx.encode_gray(w, store_planes=False)
    ctx.sync()
elif warm == 2:
    ctx.sync()
    time.sleep(1.0)
_, (og, bg), _ = ctx.encode_gray(g, store_planes=False)
ctx.sync()
bad = [k for k in range(8) if pybic.stream_bytes(og[k], exp[k][0]) != exp[k][1].tobytes()]
print(f"{rows}x{cols} mode {mode} one_stream {one} warm {warm}: bad planes {bad}", flush=True)
