import sys
sys.path.insert(0, "binary-image-compression_amd"); sys.path.insert(0, "tests")
import numpy as np, pybic
from oracle_lib import Oracle
o = Oracle(); ctx = pybic.Context(0); t = ctx.torch
for (rows, cols, pitch) in [(2, 4096, 4096), (300, 64, 64), (1, 128, 128), (1, 64, 64), (1, 80, 80)]:
    gray = o.gen_bytes(77 + rows, rows * pitch).reshape(rows, pitch)
    exp = o.bitplanes(np.ascontiguousarray(gray[:, :cols]), 8)
    g = t.from_numpy(gray).to(ctx.dev)
    got = pybic.as_u64(ctx.bitplanes_u8(g, cols=cols, nplanes=8)); ctx.sync()
    bad = np.argwhere(got != exp)
    print(rows, cols, "bad", len(bad), "of", got.size)
    for (b, r, w) in bad[:4]:
        print("  plane", b, "row", r, "word", w)
        print("   got", format(int(got[b, r, w]), "064b"))
        print("   exp", format(int(exp[b, r, w]), "064b"))
    # which expected word does got match?
    if len(bad):
        b, r, w = bad[0]
        hits = np.argwhere(exp == got[b, r, w])
        print("  got[bad0] equals exp at", hits[:4].tolist())
