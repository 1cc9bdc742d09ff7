"""Timing of the §8 rows beside the encoder (measurement for DESIGN.md §3, not a test): at configs[2]'s
size (8 planes of 16384^2, Bernoulli(0.5) pixels, device-resident) -- the packed encoder with its row
index, the device decoders (Golomb from the index, EG, both through unmed), the adaptive EG coder
(encode, its row index and its device decoder), bic_row_index from planes, PBM unpack / pack of one plane, P5 raster -> planes, planes -> gray. HIP events
around R launches of each call after a warm-up; every decode is checked against the planes.
Usage: python tools/time_aux.py [--reps R] > gpurun_out/time_aux.json"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
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
    plane_bytes = n * rows * wpr * 8
    out = {"config": f"{n} planes {rows}x{cols}, Bernoulli(0.5) pixels, device-resident", "reps": args.reps}
    stream = torch.cuda.current_stream()

    def timed(name, fn, nbytes):
        for _ in range(2):
            fn()
        ctx.sync()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(args.reps):
            fn()
        b.record(stream)
        b.synchronize()
        us = a.elapsed_time(b) * 1e3 / args.reps
        out[name] = {"us": round(us, 1), "algorithmic_bytes": int(nbytes), "GB_s": round(nbytes / us / 1e3, 1)}

    idx = ctx.empty_i64(n * rows * 2)
    enc = {}

    def encode():
        enc["r"] = ctx.encode_planes_packed(planes, cols, True, golomb=True, eg=True, row_index=idx)
    encode()
    ctx.sync()
    (og, bg, fg), (oe, be, fe) = enc["r"]
    gbytes = int(pybic.as_u64(fg)[-1]) * 8
    ebytes = int(pybic.as_u64(fe)[-1]) * 8
    timed("encode_packed_golomb_eg_index", encode, plane_bytes + gbytes + ebytes + n * rows * 16)
    p00 = (planes[:, 0, 0] >> 63).to(torch.uint8) & 1
    back = ctx.empty_i64(n, rows, wpr)

    def dec_g():
        ctx.decode_planes(0, og, bg, n, rows, cols, True, word_off=fg, row_index=idx, p00=p00, out=back)
    dec_g()
    ctx.sync()
    out["decode_golomb_ok"] = bool(torch.equal(back, planes))
    timed("decode_golomb", dec_g, gbytes + n * rows * 16 + plane_bytes)

    def dec_e():
        ctx.decode_planes(1, oe, be, n, rows, cols, True, word_off=fe, p00=p00, out=back)
    back.zero_()
    dec_e()
    ctx.sync()
    out["decode_eg_ok"] = bool(torch.equal(back, planes))
    timed("decode_eg", dec_e, ebytes + plane_bytes)

    ri = ctx.empty_i64(n * rows * 2)
    timed("row_index", lambda: ctx.row_index(planes, cols, True, out=ri), plane_bytes + n * rows * 16)
    ctx.sync()
    out["row_index_ok"] = bool(torch.equal(ri, idx))

    slot2 = ctx.slot_words(rows, cols, 2)
    o2, b2 = ctx.empty_i64(n, slot2), ctx.empty_i64(n)
    ctx.encode_planes(planes, cols, True, 2, out=o2, plane_bits=b2)
    ctx.sync()
    e2bytes = int(pybic.as_u64(b2).sum()) // 8
    timed("encode_eg_adaptive", lambda: ctx.encode_planes(planes, cols, True, 2, out=o2, plane_bits=b2),
          plane_bytes + e2bytes)
    ai = ctx.empty_i64(n * rows * 2)
    timed("egad_row_index", lambda: ctx.egad_row_index(planes, cols, True, out=ai), plane_bytes + n * rows * 16)

    def dec_a():
        ctx.decode_planes(2, o2, b2, n, rows, cols, True, row_index=ai, p00=p00, out=back)
    back.zero_()
    dec_a()
    ctx.sync()
    out["decode_eg_adaptive_ok"] = bool(torch.equal(back, planes))
    timed("decode_eg_adaptive", dec_a, e2bytes + n * rows * 16 + plane_bytes)

    p1 = planes[0]
    raster = ctx.pbm_pack(p1, cols)
    timed("pbm_pack_one_plane", lambda: ctx.pbm_pack(p1, cols, out=raster), 2 * rows * wpr * 8)
    timed("pbm_unpack_one_plane", lambda: ctx.pbm_unpack(raster, rows, cols), 2 * rows * wpr * 8)
    ctx.sync()
    out["pbm_round_trip_ok"] = bool(torch.equal(ctx.pbm_unpack(raster, rows, cols), p1))

    gray = torch.randint(0, 256, (rows * cols + 19,), dtype=torch.uint8, device=ctx.dev, generator=g)
    pl8 = ctx.empty_i64(n, rows, wpr)
    timed("pgm_bitplanes_offset19", lambda: ctx.pgm_bitplanes(gray[19:], rows, cols, 255, 8, out=pl8),
          rows * cols + plane_bytes)
    timed("bitplanes_u8", lambda: ctx.bitplanes_u8(gray[:rows * cols].view(rows, cols), out=pl8),
          rows * cols + plane_bytes)
    g8 = torch.empty(rows, cols, dtype=torch.uint8, device=ctx.dev)
    timed("planes_to_gray", lambda: ctx.planes_to_gray(pl8, cols, out=g8), rows * cols + plane_bytes)
    ctx.sync()
    out["planes_to_gray_ok"] = bool(torch.equal(g8, gray[:rows * cols].view(rows, cols)))
    ctx.sync()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
