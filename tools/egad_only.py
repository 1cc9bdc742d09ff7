"""diagnostic: the adaptive EG coder alone on a C3-sized input (8 planes 16384^2, Bernoulli(0.5)):
encode, row index and device decode, 3 reps each, HIP-event timed; for rocprofv3 counter passes."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
import pybic  # noqa: E402

rows = cols = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
n = 8
ctx = pybic.Context(0)
t = ctx.torch
g = t.Generator(device=ctx.dev)
g.manual_seed(7)
wpr = (cols + 63) // 64
planes = t.randint(-2**62, 2**62, (n, rows, wpr), dtype=t.int64, device=ctx.dev, generator=g)
slot2 = ctx.slot_words(rows, cols, 2)
o2, b2 = ctx.empty_i64(n, slot2), ctx.empty_i64(n)
ai = ctx.empty_i64(n * rows * 2)
back = ctx.empty_i64(n, rows, wpr)
res = {}
for name, f in (("encode", lambda: ctx.encode_planes(planes, cols, True, 2, out=o2, plane_bits=b2)),
                ("row_index", lambda: ctx.egad_row_index(planes, cols, True, out=ai)),
                ("decode", lambda: ctx.decode_planes(2, o2, b2, n, rows, cols, True, row_index=ai, out=back))):
    f()
    ctx.sync()
    a, b = t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        f()
    b.record()
    ctx.sync()
    res[name] = round(a.elapsed_time(b) * 1e3 / 3, 1)

print(json.dumps(res), flush=True)
