"""Probe (not the bench): C3 images encoded with two images in flight -- two contexts on two HIP
streams, alternate images -- against one context on one stream; same streams checked word for word.
Usage: python tools/pipeline_probe.py [--steps N] [--streams S]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--streams", type=int, default=2)
    args = ap.parse_args()
    import torch
    import pybic
    n = args.streams
    rows = cols = 16384
    ctxs = [pybic.Context(0) for _ in range(n)]
    dev = ctxs[0].dev
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED)
    grays = [torch.randint(0, 256, (rows, cols), dtype=torch.uint8, device=dev, generator=g) for _ in range(n)]
    sg, se = ctxs[0].slot_words(rows, cols, pybic.CODER_GOLOMB), ctxs[0].slot_words(rows, cols, pybic.CODER_EG)
    outs = [(ctxs[0].empty_i64(8, sg), ctxs[0].empty_i64(8, se), ctxs[0].empty_i64(8), ctxs[0].empty_i64(8))
            for _ in range(n)]
    streams = [torch.cuda.Stream(dev) for _ in range(n)]

    def step(k, multi):
        i = k % n
        c = ctxs[i] if multi else ctxs[0]
        s = streams[i] if multi else streams[0]
        og, oe, bg, be = outs[i]
        with torch.cuda.stream(s):
            c.encode_gray(grays[i], planes=None, slots=(sg, se), outs=(og, oe), bits=(bg, be), store_planes=False)

    res = {}
    for multi in (False, True, False, True):
        for k in range(6):
            step(k, multi)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(args.steps):
            step(k, multi)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        res.setdefault("multi" if multi else "single", []).append(round(dt * 1e3, 4))
    # the streams of the last images, against one context encoding the same images alone
    ok = True
    for i in range(n):
        og, oe, bg, be = outs[i]
        ref_g, ref_e, ref_bg, ref_be = (ctxs[0].empty_i64(8, sg), ctxs[0].empty_i64(8, se), ctxs[0].empty_i64(8),
                                        ctxs[0].empty_i64(8))
        torch.cuda.synchronize()
        ctxs[0].encode_gray(grays[i], planes=None, slots=(sg, se), outs=(ref_g, ref_e), bits=(ref_bg, ref_be),
                            store_planes=False)
        ctxs[0].sync()
        ok = ok and torch.equal(bg, ref_bg) and torch.equal(be, ref_be)
        for p in range(8):
            wg = (int(pybic.as_u64(ref_bg)[p]) + 63) // 64
            we = (int(pybic.as_u64(ref_be)[p]) + 63) // 64
            ok = ok and torch.equal(og[p][:wg], ref_g[p][:wg]) and torch.equal(oe[p][:we], ref_e[p][:we])
    res["same_streams"] = bool(ok)
    res["streams"] = n
    print(json.dumps(res))


if __name__ == "__main__":
    main()
