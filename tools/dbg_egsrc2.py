"""diagnostic: the class emission kernels (EG source mode 1) row by row -- per bad Golomb row its
start, length, whether it is a k = 0 copy (R then '1'), the differing bit range; three encodes."""
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
ctx = pybic.Context(0)
ctx.set_encoder("staged")
img = o.gen_bytes(rows * 13 + cols, rows * cols).reshape(rows, cols)
g = ctx.torch.from_numpy(img).to(ctx.dev)
P = o.bitplanes(img, 8)


def bits_of(b, n):
    return np.unpackbits(np.frombuffer(b, np.uint8))[:n]


shown = False
for rep in range(12):
    mode, one = ((1, False), (1, True), (2, False))[rep % 3]
    ctx.set_eg_source(mode)
    ctx.set_one_stream(one)
    _, (og, bg), _ = ctx.encode_gray(g, store_planes=False)
    ctx.sync()
    for k in range(8):
        eb, est, _ = o.encode_plane(P[k], cols, 1, 0)
        got = bits_of(pybic.stream_bytes(og[k], eb), eb)
        exp = bits_of(est.tobytes(), eb)
        if np.array_equal(got, exp):
            continue
        ri = list(o.row_index(P[k], cols, 1)[0::2]) + [eb]
        # residual rows on the CPU: the med residual of the plane
        R = o.med(P[k], cols)
        Rb = np.unpackbits(R.astype(">u8").view(np.uint8).reshape(rows, -1), axis=1)[:, :cols]
        for r in range(rows):
            a, b = int(ri[r]), int(ri[r + 1])
            d = np.nonzero(got[a:b] != exp[a:b])[0]
            if not len(d):
                continue
            L = b - a
            k0 = L == cols + 1 and np.array_equal(exp[a:b - 1], Rb[r]) and exp[b - 1] == 1
            if not shown:
                shown = True
                for q in range(0, L, 64):
                    print("  exp", "".join(map(str, exp[a + q:a + q + 64])))
                    print("  got", "".join(map(str, got[a + q:a + q + 64])))
            print(f"rep {rep} mode {mode} one_stream {one} plane {k} row {r}: start {a} (mod64 {a % 64}) len {L} k0 {k0} "
                  f"diffs {len(d)} first {int(d[0])} last {int(d[-1])} "
                  f"exp {''.join(map(str, exp[a:a + 24]))} got {''.join(map(str, got[a:a + 24]))}"
                  f" | around first: exp {''.join(map(str, exp[a + d[0]:a + d[0] + 16]))} got {''.join(map(str, got[a + d[0]:a + d[0] + 16]))}")
