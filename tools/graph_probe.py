"""Diagnostic (not part of the product or the bench): does replaying the C3 step's launch
sequence from a captured graph (torch.cuda.CUDAGraph over bic_encode_gray, which pybic enqueues on
torch's current stream -- the capture stream) cut the step below the eager launch sequence, and are
the streams identical? Feeds DESIGN.md §7 ("one hipGraph for the ~10 launches of a step").

    python tools/graph_probe.py [--rows 16384 --cols 16384 --steps 50]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "binary-image-compression_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=16384)
    ap.add_argument("--cols", type=int, default=16384)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--no-planes", action="store_true", help="planes NULL: the bench's default C3 call (EG source)")
    a = ap.parse_args()
    import torch
    import pybic

    ctx = pybic.Context(0)
    t, dev = torch, ctx.dev
    R, Cc, NP = a.rows, a.cols, 8
    g = t.Generator(device=dev)
    g.manual_seed(0x5EED0000)
    gray = [t.randint(0, 256, (R, Cc), dtype=t.uint8, device=dev, generator=g) for _ in range(2)]
    wpr = (Cc + 63) // 64
    planes = None if a.no_planes else ctx.empty_i64(NP, R, wpr)
    sg = ctx.slot_words(R, Cc, pybic.CODER_GOLOMB)
    se = ctx.slot_words(R, Cc, pybic.CODER_EG)
    outs = (ctx.empty_i64(NP, sg), ctx.empty_i64(NP, se))
    bits = (ctx.empty_i64(NP), ctx.empty_i64(NP))
    ctx.reserve(NP, R, Cc)

    def step(k):
        ctx.encode_gray(gray[k & 1], nplanes=NP, planes=planes, slots=(sg, se), outs=outs, bits=bits,
                        store_planes=not a.no_planes)

    for k in range(6):
        step(k)
    ctx.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        step(k)
    ctx.sync()
    torch.cuda.synchronize()
    eager_ms = (time.perf_counter() - t0) / a.steps * 1e3
    step(0)
    ctx.sync()
    ref = [x.clone() for x in outs + bits]

    graphs = []
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for k in range(2):
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=side):
                step(k)
            graphs.append(gr)
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize()
    for k in range(6):
        graphs[k & 1].replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        graphs[k & 1].replay()
    torch.cuda.synchronize()
    graph_ms = (time.perf_counter() - t0) / a.steps * 1e3
    graphs[0].replay()
    torch.cuda.synchronize()
    ctx.sync()
    same = all(bool(t.equal(x, y)) for x, y in zip(ref, list(outs + bits)))
    print({"planes": not a.no_planes, "rows": R, "cols": Cc, "eager_ms_per_step": round(eager_ms, 4), "graph_ms_per_step": round(graph_ms, 4),
           "streams_identical": same}, flush=True)


if __name__ == "__main__":
    main()
