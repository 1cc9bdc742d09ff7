"""C2 diagnostic: the single-kernel encoder's phase clocks (lib/libbic_stamps.so) for the three planes of
tools/c2_alt.py (whose launch takes 33 / 18.6 / 33 us by input): kernel span, phase medians and the
slowest rows' phases and start offsets."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["BIC_LIB_PATH"] = os.path.join(ROOT, "binary-image-compression_amd", "lib", "libbic_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
import pybic  # noqa: E402

rows = cols = 4096
wpr = cols // 64
ctx = pybic.Context(0)
t = ctx.torch
g = t.Generator(device=ctx.dev)
g.manual_seed(0x5EED0000)
planes = [t.randint(0, 256, (rows * wpr * 8,), dtype=t.uint8, device=ctx.dev, generator=g).view(t.int64).view(1, rows, wpr)
          for _ in range(3)]
slot = ctx.slot_words(rows, cols, pybic.CODER_GOLOMB)
out, bits = ctx.empty_i64(1, slot), ctx.empty_i64(1)
lib = pybic.load()
lib.bic_debug_stamps.argtypes = [C.c_void_p, C.c_size_t]
names = ["load+count", "ones lb", "len", "bits lb", "emit", "write"]
for pi, pl in enumerate(planes):
    for _ in range(5):
        ctx.encode_planes(pl, cols, False, pybic.CODER_GOLOMB, slot, out, bits)
    ctx.sync()
    n = rows * 8
    buf = np.zeros(n, np.uint64)
    assert lib.bic_debug_stamps(buf.ctypes.data, n) == 0
    S = buf.reshape(-1, 8).astype(np.int64)
    d = np.diff(S[:, :7], axis=1)
    ok = (S[:, 0] > 0) & (d >= 0).all(axis=1)
    t0 = S[ok, 0].min()
    print(f"== plane {pi}: waves {ok.sum()} span {S[ok, 6].max() - t0} clk; slow-path word counts col 7")
    for i, nm in enumerate(names):
        print(f"   {nm:10s} median {np.median(d[ok][:, i]):8.0f} max {d[ok][:, i].max():8.0f}")
    end = np.where(ok, S[:, 6] - t0, -1)
    top = np.argsort(end)[-6:][::-1]
    for r in top:
        print(f"   row {r:5d} start {S[r, 0] - t0:7d} end {end[r]:7d} phases {list(d[r])} s7 {S[r, 7]}")
    s7 = S[:, 7]
    p1 = s7 // 1000000
    p3 = s7 % 1000
    lng = (s7 // 1000) % 1000
    for nm_, sel in (("all copy-path words", ok & (p1 == 64)), ("no copy-path word", ok & (p1 == 0)),
                     ("mixed paths", ok & (p1 > 0) & (p1 < 64)), ("any per-codeword word", ok & (p3 > 0))):
        if sel.any():
            print(f"   {nm_:22s} rows {sel.sum():5d}  emit median {np.median(d[sel][:, 4]):7.0f}  len median {np.median(d[sel][:, 2]):7.0f}"
                  f"  bits lb median {np.median(d[sel][:, 3]):7.0f}")
    print(f"   per-codeword words per row: mean {p3[ok].mean():.2f}; long words {lng[ok].sum()}")
    print(f"   rows by end > 20k clk: {(end > 20000).sum()}, start offsets median {np.median(S[ok, 0] - t0):.0f} max {(S[ok, 0] - t0).max()}",
          flush=True)
