"""Golomb k classes of the rows of the bench's C3 input (diagnostic): per plane, the share of rows
whose codewords all have k = 0, all k = 1, or mixed, from the exact coder walk
(A_i - N_i = A0 - N0 + j_{i-1} + 1 - 2i over the row's samples)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
import pybic  # noqa: E402

rows, cols = 16384, 16384
ctx = pybic.Context(0)
t = ctx.torch
g = t.Generator(device=ctx.dev)
g.manual_seed(0x5EED0000)
gray = t.randint(0, 256, (rows, cols), dtype=t.uint8, device=ctx.dev, generator=g)
planes = ctx.bitplanes_u8(gray, nplanes=8)
resid, _ = ctx.med_residual(planes, cols, True, want_resid=True, want_weight=False)
ctx.sync()
R = pybic.as_u64(resid).reshape(8, rows, cols // 64)
for p in range(8):
    N0 = 0
    O = 0
    cnt = np.zeros(3, np.int64)
    for r0 in range(0, rows, 512):
        bits = np.unpackbits(R[p, r0:r0 + 512].byteswap().view(np.uint8), axis=1).astype(bool)
        rr, cc = np.nonzero(bits)
        ones = bits.sum(1)
        start = np.concatenate([[0], np.cumsum(ones)[:-1]])
        rank = np.arange(len(rr)) - start[rr]
        c2 = cc + 1 - 2 * (rank + 1)
        c3 = cc + 1 - 3 * (rank + 1)
        mx2 = np.full(512, -10**9)
        mn2 = np.full(512, 10**9)
        mx3 = np.full(512, -10**9)
        np.maximum.at(mx2, rr, c2)
        np.minimum.at(mn2, rr, c2)
        np.maximum.at(mx3, rr, c3)
        for i in range(512):
            row = r0 + i
            N0 = O + row
            A0 = row * (cols + 1) - N0
            d = A0 - N0
            hi = d + max(0, mx2[i])
            lo = d + min(0, mn2[i])
            hi2 = A0 - 2 * N0 + max(0, mx3[i])
            if N0 > 0 and hi <= 0:
                cnt[0] += 1
            elif N0 > 0 and lo > 0 and hi2 <= 0:
                cnt[1] += 1
            else:
                cnt[2] += 1
            O += ones[i]
    print(f"plane {p}: k0 {cnt[0] / rows:.3f}  k1 {cnt[1] / rows:.3f}  mixed {cnt[2] / rows:.3f}", flush=True)
