"""diagnostic: per-stage times (bic_prof) of the default C3 call, 20 calls after 3 warm-up, errors of
the call ignored (for diagnostic builds whose output is wrong by design: BIC_DIAG_*). One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
import pybic  # noqa: E402

ctx = pybic.Context(0)
t = ctx.torch
g = t.Generator(device=ctx.dev)
g.manual_seed(0x5EED0000)
gray = t.randint(0, 256, (16384, 16384), dtype=t.uint8, device=ctx.dev, generator=g)


def call():
    ctx.encode_gray(gray, store_planes=False)


for _ in range(3):
    call()
try:
    ctx.sync()
except pybic.BicError:
    pass
ctx.prof_enable(True)
for _ in range(20):
    call()
try:
    ctx.sync()
except pybic.BicError:
    pass
prof = ctx.prof_collect()
print(json.dumps(dict(lib=os.path.basename(pybic.LIB_PATH),
                      us={k: round(ms * 1e3 / n, 1) for k, (n, ms) in prof.items()})), flush=True)
