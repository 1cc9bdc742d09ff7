"""diagnostic: the first encode of a fresh process on the EG-source class-kernel
path. One encode of a 70 x 4096 image (slots pre-filled with 0xaa), then per bad Golomb row: its class
by the oracle's codeword k values (k0 / k1 / mixed), its length, the bits that differ and, per
differing 64-bit chunk of the row, whether the output there still holds the 0xaa fill. Run one
process per trial (tools/dbg_first.sh) with BIC_LIB_PATH naming the variant library."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pybic  # noqa: E402
from oracle_lib import Oracle  # noqa: E402

rows, cols = int(sys.argv[1]), int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
o = Oracle()
img = o.gen_bytes(rows * 13 + cols, rows * cols).reshape(rows, cols)
P = o.bitplanes(img, 8)
exp, ris, cls = [], [], []
for k in range(8):
    e = o.encode_plane(P[k], cols, 1, 0)
    exp.append(e)
    ris.append(list(o.row_index(P[k], cols, 1)[0::2]) + [e[0]])
    s, eo = o.plane_runs(o.med(P[k], cols), cols)
    _, _, kk, _ = o.golomb_samples(s)
    rowid = np.concatenate([[0], np.cumsum(eo)[:-1]])
    c = []
    for r in range(rows):
        u = set(kk[rowid == r].tolist())
        c.append("k0" if u == {0} else "k1" if u == {1} else "mixed")
    cls.append(c)
ctx = pybic.Context(0)
ctx.set_encoder("staged")
if os.environ.get("DBG_ONE_STREAM") == "1":  # the class kernels and k_emit_rest one after the other on one stream
    ctx.set_one_stream(True)
g = ctx.torch.from_numpy(img).to(ctx.dev)
slot = ctx.slot_words(rows, cols, pybic.CODER_GOLOMB)
og = ctx.empty_i64(8, slot)
pat = np.unpackbits(np.frombuffer(b"\xaa" * 8, np.uint8))
counts = {c: sum(x.count(c) for x in cls) for c in ("k0", "k1", "mixed")}
for rep in range(reps):
    og.fill_(-0x5555555555555556)
    _, (og_, bg), _ = ctx.encode_gray(g, store_planes=False, outs=(og, None))
    try:
        ctx.sync()
        rc = 0
    except pybic.BicError as ex:
        rc = ex.code
    bad = []
    for k in range(8):
        eb = exp[k][0]
        got = np.unpackbits(np.frombuffer(pybic.stream_bytes(og[k], eb), np.uint8))[:eb]
        ex = np.unpackbits(np.frombuffer(exp[k][1].tobytes(), np.uint8))[:eb]
        if np.array_equal(got, ex):
            continue
        for r in range(rows):
            a, b = int(ris[k][r]), int(ris[k][r + 1])
            d = np.nonzero(got[a:b] != ex[a:b])[0]
            if not len(d):
                continue
            # absolute stream words touched by the differences, and which of them still hold 0xaa
            words = sorted(set(((a + d) // 64).tolist()))
            extra = int(np.sum(got[a:b] & ~ex[a:b] & 1))  # 1s the output has and the oracle's row has not
            missing = int(np.sum(ex[a:b] & ~got[a:b] & 1))
            fill = [w for w in words if np.array_equal(got[w * 64:w * 64 + 64], pat)] if words else []
            bad.append(dict(plane=k, row=r, cls=cls[k][r], start=a, len=b - a, diffs=int(len(d)),
                            first=int(d[0]), nwords=len(words), fill_words=len(fill), extra=extra, missing=missing,
                            rel_words=[w - a // 64 for w in words][:12]))
    print(json.dumps(dict(lib=os.path.basename(pybic.LIB_PATH), rep=rep, rc=rc, classes=counts,
                          nbad=len(bad), bad_classes={c: sum(1 for x in bad if x["cls"] == c) for c in counts},
                          bad=bad[:6])), flush=True)
