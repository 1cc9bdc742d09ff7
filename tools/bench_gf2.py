"""GF(2) algebra measurement (bic_gf2.hip): C = A B, A^t B and A B^t on square
n x n bit matrices resident in HBM, timed with HIP events on the launch stream (bic_prof_*), checked
bit-exactly against the oracle on a corner block, with the reference's own mul (oracle/_ref, single
thread: binmat.cpp's loops are serial) timed on a smaller sample. One JSON line per op.

  python tools/bench_gf2.py [--n 8192] [--reps 10]

Work unit: one GF(2) multiply-accumulate (bit AND + XOR), n^3 per product. k_gf2_ab is LDS-bound:
per row and 64-bit word of A it reads 16 table entries of 32 B (4 output words), i.e. 512 B of LDS
per 64 x 256 MACs; LDS peak 128 B/clk/CU x 256 CUs x 2.4 GHz = 78.6 TB/s -> 2.5e15 MAC/s."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

LDS_PEAK_TBS = 128 * 256 * 2.4e9 / 1e12
MAC_PEAK = LDS_PEAK_TBS * 1e12 / 512 * (64 * 256)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cpu-n", type=int, default=2048)
    args = ap.parse_args()
    import pybic
    from oracle_lib import Oracle, Ref, have_ref
    o = Oracle()
    ctx = pybic.Context(0)
    t = ctx.torch
    n, w = args.n, (args.n + 63) // 64
    g = t.Generator(device=ctx.dev)
    g.manual_seed(0x6F2)
    A = t.randint(-(1 << 62), 1 << 62, (n, w), dtype=t.int64, device=ctx.dev, generator=g)
    B = t.randint(-(1 << 62), 1 << 62, (n, w), dtype=t.int64, device=ctx.dev, generator=g)
    C = t.zeros((n, w), dtype=t.int64, device=ctx.dev)
    ref = Ref() if have_ref() else None
    cn = args.cpu_n
    cw = (cn + 63) // 64
    Ah, Bh = pybic.as_u64(A[:cn, :cw]).copy(), pybic.as_u64(B[:cn, :cw]).copy()
    for op, name in ((pybic.GF2_AB, "AB"), (pybic.GF2_ATB, "AtB"), (pybic.GF2_ABT, "ABt")):
        for _ in range(2):
            ctx.gf2_mul(op, A, n, B, n, C, n)
        ctx.sync()
        ctx.prof_enable(True)
        t0 = time.perf_counter()
        for _ in range(args.reps):
            ctx.gf2_mul(op, A, n, B, n, C, n)
        ctx.sync()
        wall = (time.perf_counter() - t0) / args.reps
        prof = ctx.prof_collect()
        ctx.prof_enable(False)
        kern = {k: round(1e3 * ms / max(c, 1), 2) for k, (c, ms) in prof.items()}
        mul_us = kern.get("gf2_mul", 0.0)
        # check: the top-left cn x cn block of a product of the leading blocks equals the oracle's
        Cs = t.zeros((cn, cw), dtype=t.int64, device=ctx.dev)
        Ad, Bd = ctx.to_dev(Ah), ctx.to_dev(Bh)
        ctx.gf2_mul(op, Ad, cn, Bd, cn, Cs, cn)
        ctx.sync()
        exp = o.gf2_mul(op, Ah, cn, cn, Bh, cn, cn, np.zeros((cn, cw), np.uint64), cn, cn)
        ok = bool(np.array_equal(pybic.as_u64(Cs), exp))
        cpu = None
        if ref is not None:
            # mul_ABt calls block_sum (an OpenMP region) per word pair: a smaller sample
            sn = cn if op != pybic.GF2_ABT else min(cn, 512)
            sw = (sn + 63) // 64
            As, Bs = Ah[:sn, :sw].copy(), Bh[:sn, :sw].copy()
            t0 = time.perf_counter()
            ref.gf2_mul(op, As, sn, sn, Bs, sn, sn, np.zeros((sn, sw), np.uint64), sn, sn)
            dt = time.perf_counter() - t0
            cpu = {"value": round(sn ** 3 / dt / 1e9, 3), "unit": "G MAC/s", "cores": 1, "kind": "reference",
                   "sample": f"mul() on {sn}^3 ({dt:.2f} s incl. the harness's bit-by-bit copies)"}
        macs = float(n) ** 3
        line = {"op": name, "n": n, "ms_per_product": round(wall * 1e3, 3), "kernels_us": kern,
                "value": round(macs / wall / 1e12, 2), "unit": "T MAC/s (GF(2) bit multiply-accumulates)",
                "roofline": {"bound": "lds", "kernel": "gf2_mul (k_gf2_ab)",
                             "achieved": round(macs / (mul_us * 1e-6) / 1e12, 1) if mul_us else None,
                             "peak": round(MAC_PEAK / 1e12, 1), "unit": "T MAC/s",
                             "frac": round(macs / (mul_us * 1e-6) / MAC_PEAK, 3) if mul_us else None},
                "bit_exact_check": ok, "cpu_baseline": cpu}
        print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
