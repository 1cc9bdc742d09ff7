"""diagnostic: test_single_stream_calls_match_dual's sequence (single-kernel calls, then two-pass calls
on the same context) repeated; counts the calls whose Golomb / EG bit totals differ from the oracle's.
BIC_LIB_PATH names the library."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pybic  # noqa: E402
from oracle_lib import Oracle  # noqa: E402

o = Oracle()
rows, cols = 33, 2000
P = o.gen_plane(3, 0.2, rows, cols)[None]
eg_, ee_ = o.encode_plane(P[0], cols, 1, 0)[0], o.encode_plane(P[0], cols, 1, 1)[0]
ctx = pybic.Context(0)
d = ctx.to_dev(P)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
bad = {}
for rep in range(reps):
    for mode in ("single-kernel", "two-pass"):
        ctx.set_encoder(mode)
        _, bg = ctx.encode_planes(d, cols, True, pybic.CODER_GOLOMB)
        _, be = ctx.encode_planes(d, cols, True, pybic.CODER_EG)
        (_, bg2), (_, be2) = ctx.encode_planes2(d, cols, True)
        ctx.sync()
        got = [int(pybic.as_u64(x)[0]) for x in (bg, be, bg2, be2)]
        exp = [eg_, ee_, eg_, ee_]
        for i, (g, e) in enumerate(zip(got, exp)):
            if g != e:
                k = f"{mode}/call{i}"
                bad[k] = bad.get(k, 0) + 1
print(json.dumps(dict(lib=os.path.basename(pybic.LIB_PATH), reps=reps, bad=bad)), flush=True)
