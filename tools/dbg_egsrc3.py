"""diagnostic: first encode of a fresh context -- bad Golomb rows per encode, per EG-source mode"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pybic  # noqa: E402
from oracle_lib import Oracle  # noqa: E402

rows, cols = int(sys.argv[1]), int(sys.argv[2])
o = Oracle()
img = o.gen_bytes(rows * 13 + cols, rows * cols).reshape(rows, cols)
P = o.bitplanes(img, 8)
exp = [o.encode_plane(P[k], cols, 1, 0) for k in range(8)]


def bad_planes(ctx, g, mode, one=False, sync_first=False):
    ctx.set_eg_source(mode)
    ctx.set_one_stream(one)
    if sync_first:
        ctx.sync()
    _, (og, bg), _ = ctx.encode_gray(g, store_planes=False)
    ctx.sync()
    bad = []
    for k in range(8):
        eb, est, _ = exp[k]
        if pybic.stream_bytes(og[k], eb) != est.tobytes():
            bad.append(k)
    return bad


for trial, first in enumerate((1, 2, 1, 0, 1, 2)):
    ctx = pybic.Context(0)
    ctx.set_encoder("staged")
    g = ctx.torch.from_numpy(img).to(ctx.dev)
    r = [bad_planes(ctx, g, first)]
    for m in (1, 2, 1):
        r.append(bad_planes(ctx, g, m))
    print(f"trial {trial}: first mode {first}: bad planes per encode (modes {first},1,2,1): {r}", flush=True)
    ctx.close()
