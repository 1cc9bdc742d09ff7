"""Phase clocks of the staged prefix (diagnostic build lib/libbic_stamps.so, make stamps): one C3
encode_gray (the bench's default call), then per walked row of k_row_walk its entry, residual-word,
walked and stored times on the shared 100 MHz clock (slots 4-7 of bic_fused.hip WSTAMP), and per
workgroup of the two k_scan_rows launches (SSTAMP) its entry, own rows loaded, earlier rows summed,
block scans done and end. Prints spans, phase durations and how the start times spread."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["BIC_LIB_PATH"] = os.path.join(ROOT, "binary-image-compression_amd", "lib", "libbic_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
import pybic  # noqa: E402

C4 = len(sys.argv) > 1 and sys.argv[1] == "c4"  # bench.py's C4 call instead: 64 frames of 4096^2, packed
ctx = pybic.Context(0)
t = ctx.torch
g = t.Generator(device=ctx.dev)
g.manual_seed(0x5EED0000)
if C4:
    rows = cols = 4096
    nplanes = 64
    planes = t.randint(-2**62, 2**62, (nplanes, rows, cols // 64), dtype=t.int64, device=ctx.dev, generator=g)
else:
    rows = cols = 16384
    nplanes = 8
    gray = t.randint(0, 256, (rows, cols), dtype=t.uint8, device=ctx.dev, generator=g)
lib = pybic.load()
lib.bic_debug_stamps.argtypes = [C.c_void_p, C.c_size_t]
n = (1 << 21) + 16384
out = {}
for rep in range(3):
    if C4:
        ctx.encode_planes_packed(planes, cols, True, golomb=True, eg=False)
    else:
        ctx.encode_gray(gray, store_planes=False)
    ctx.sync()
    buf = np.zeros(n, np.uint64)
    assert lib.bic_debug_stamps(buf.ctypes.data, n) == 0
    S = buf[:rows * nplanes * 8].reshape(-1, 8).astype(np.int64)[:, 4:8]
    ok = (S[:, 0] > 0) & (S[:, 3] >= S[:, 0])
    if rep == 0:
        first = S[:, 0].copy()
    else:  # rows stamped by this call only (the array keeps older values)
        ok &= S[:, 0] != first
        first = S[:, 0].copy()
    W = S[ok]
    t0 = W[:, 0].min()
    d = lambda a: np.percentile(a, [10, 50, 90, 100]).round(2).tolist()  # noqa: E731
    out = dict(rep=rep, rows=int(ok.sum()), span_us=float((W[:, 3].max() - t0) / 100),
               load_us=d((W[:, 1] - W[:, 0]) / 100), walk_us=d((W[:, 2] - W[:, 1]) / 100),
               store_us=d((W[:, 3] - W[:, 2]) / 100), start_us=d((W[:, 0] - t0) / 100),
               end_us=d((W[:, 3] - t0) / 100), planes=np.bincount(np.nonzero(ok)[0] // rows, minlength=nplanes).tolist()[:8])
    print(json.dumps(out), flush=True)
    for name, off in (("ones_scan", 0), ("len_scan", 8192)):
        T = buf[(1 << 21) + off:(1 << 21) + off + 8192].reshape(-1, 8).astype(np.int64)[:, :5]
        T = T[T[:, 0] > 0]
        t0 = T[:, 0].min()
        print(json.dumps(dict(rep=rep, kernel=name, wgs=len(T), span_us=float((T[:, 4].max() - t0) / 100),
                              own_us=d((T[:, 1] - T[:, 0]) / 100), before_us=d((T[:, 2] - T[:, 1]) / 100),
                              scans_us=d((T[:, 3] - T[:, 2]) / 100), tail_us=d((T[:, 4] - T[:, 3]) / 100),
                              start_us=d((T[:, 0] - t0) / 100), end_us=d((T[:, 4] - t0) / 100))), flush=True)
