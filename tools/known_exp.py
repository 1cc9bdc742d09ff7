"""Diagnostic: cost of the fused encoder's look-back waits. With the stamps build, a normal
launch records every tile's prefixes; BIC_KNOWN=1 launches replay them instead of looking back.
Prints the encoder time of both and the phase clocks of the replayed launch."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["BIC_LIB_PATH"] = os.path.join(ROOT, "binary-image-compression_amd", "lib", "libbic_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
import ctypes as C  # noqa: E402

import pybic  # noqa: E402

rows, cols, nplanes = 16384, 16384, 8
ctx = pybic.Context(0)
t = ctx.torch
g = t.Generator(device=ctx.dev)
g.manual_seed(1)
gray = t.randint(0, 256, (rows, cols), dtype=t.uint8, device=ctx.dev, generator=g)
planes = ctx.bitplanes_u8(gray, nplanes=8)
ctx.reserve(8, rows, cols)
res = {}
for mode in ("0", "1", "0", "1"):
    os.environ["BIC_KNOWN"] = mode
    ctx.prof_enable(True)
    for _ in range(5):
        (og, bg), (oe, be) = ctx.encode_planes2(planes, cols, True)
    ctx.sync()
    prof = ctx.prof_collect()
    ctx.prof_enable(False)
    res[mode] = (pybic.as_u64(bg).copy(), pybic.as_u64(be).copy(), og.clone(), oe.clone())
    print("known" if mode == "1" else "normal", prof)
same = all(np.array_equal(res["0"][i], res["1"][i]) for i in range(2)) and bool((res["0"][2] == res["1"][2]).all()) \
    and bool((res["0"][3] == res["1"][3]).all())
print("streams identical:", same)
n = rows * nplanes * 8
buf = np.zeros(n, np.uint64)
lib = pybic.load()
lib.bic_debug_stamps.argtypes = [C.c_void_p, C.c_size_t]
assert lib.bic_debug_stamps(buf.ctypes.data, n) == 0
S = buf.reshape(-1, 8).astype(np.int64)
names = ["load", "wait_ones", "eg", "golomb", "wait_bits", "write"]
d = np.diff(S[:, :7], axis=1)
ok = (S[:, 0] > 0) & (d >= 0).all(axis=1)
d = d[ok]
tot = S[ok, 6] - S[ok, 0]
print(f"(known launch) waves {ok.sum()}  per-wave total: median {np.median(tot):.0f}  mean {tot.mean():.0f} clk")
for i, nm in enumerate(names):
    print(f"{nm:10s} median {np.median(d[:, i]):9.0f}  mean {d[:, i].mean():9.0f}  share {d[:, i].sum() / tot.sum():6.3f}")
# where the time goes: per-phase percentiles, by wave slot in the tile and by claim order
ids = np.nonzero(ok)[0]
plane, row = ids // rows, ids % rows
wave = row % 16
claim = (row // 16) * nplanes + plane
gol = d[:, 3]
for nm, i in (("load", 0), ("eg", 2), ("golomb", 3), ("write", 5)):
    print(nm, "p10/p50/p90/p99:", np.percentile(d[:, i], [10, 50, 90, 99]).astype(int))
print("golomb mean by wave slot:", [int(gol[wave == q].mean()) for q in range(16)])
nb = 8
edges = np.linspace(0, claim.max() + 1, nb + 1)
print("golomb mean by claim-order octile:", [int(gol[(claim >= edges[q]) & (claim < edges[q + 1])].mean()) for q in range(nb)])
start = S[ok, 0]
order = np.argsort(start)
print("golomb mean by start-time octile:", [int(gol[order[q * len(order) // nb:(q + 1) * len(order) // nb]].mean()) for q in range(nb)])
cnt = S[ok, 7]
gen, lng, cp = cnt % 1000, (cnt // 1000) % 1000, cnt // 1000000
print("words per row: general loop mean %.2f (rows with any %.3f), long lanes mean %.3f, copy mode mean %.1f"
      % (gen.mean(), (gen > 0).mean(), lng.mean(), cp.mean()))
for lo, hi in ((0, 1), (1, 2), (2, 5), (5, 1000)):
    m = (gen >= lo) & (gen < hi)
    if m.any():
        print(f"general words in [{lo},{hi}): rows {m.sum():7d}  golomb mean {gol[m].mean():8.0f}")
m = lng > 0
if m.any():
    print(f"rows with long lanes: {m.sum()}  golomb mean {gol[m].mean():.0f}")
