"""Golomb decode of a C3-sized image (8 planes of 16384^2, Bernoulli(0.5) pixels) R times, for
rocprofv3 counter passes on the decoder alone: python tools/run_decode.py [--reps R] [--coder 0|1]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--coder", type=int, default=0)
    ap.add_argument("--rows", type=int, default=16384)
    args = ap.parse_args()
    import torch
    import pybic
    ctx = pybic.Context(0)
    rows = cols = args.rows
    n, wpr = 8, (cols + 63) // 64
    g = torch.Generator(device=ctx.dev)
    g.manual_seed(0x5EED)
    planes = torch.randint(0, 256, (n * rows * wpr * 8,), dtype=torch.uint8, device=ctx.dev,
                           generator=g).view(torch.int64).view(n, rows, wpr)
    idx = ctx.empty_i64(n * rows * 2)
    (og, bg, fg), (oe, be, fe) = ctx.encode_planes_packed(planes, cols, True, golomb=True, eg=True, row_index=idx)
    p00 = (planes[:, 0, 0] >> 63).to(torch.uint8) & 1
    back = ctx.empty_i64(n, rows, wpr)
    for _ in range(args.reps):
        if args.coder == 0:
            ctx.decode_planes(0, og, bg, n, rows, cols, True, word_off=fg, row_index=idx, p00=p00, out=back)
        else:
            ctx.decode_planes(1, oe, be, n, rows, cols, True, word_off=fe, p00=p00, out=back)
    ctx.sync()
    assert torch.equal(back, planes)
    print("ok")


if __name__ == "__main__":
    main()
