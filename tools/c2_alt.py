"""C2 diagnostic: k_encode_rows' duration per call (bic_prof events) for a few input schedules --
two planes alternated (bench.py's C2), one plane every call, three planes in turn, and two planes
each encoded twice in a row -- to tell whether the alternation seen in the rocprofv3 trace (17 / 31
us) follows the input buffer or the call parity."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
import pybic  # noqa: E402

rows = cols = 4096
ctx = pybic.Context(0)
t = ctx.torch
g = t.Generator(device=ctx.dev)
g.manual_seed(0x5EED0000)
wpr = cols // 64
planes = [t.randint(0, 256, (rows * wpr * 8,), dtype=t.uint8, device=ctx.dev, generator=g).view(t.int64).view(1, rows, wpr)
          for _ in range(3)]
slot = ctx.slot_words(rows, cols, pybic.CODER_GOLOMB)
out = ctx.empty_i64(1, slot)
bits = ctx.empty_i64(1)
ctx.reserve(1, rows, cols)


def run(name, sched, reps=24):
    for i in range(6):
        ctx.encode_planes(planes[sched[i % len(sched)]], cols, False, pybic.CODER_GOLOMB, slot, out, bits)
    ctx.sync()
    durs = []
    for i in range(reps):
        ctx.prof_enable(True)
        ctx.prof_only("encode_rows_golomb")
        ctx.encode_planes(planes[sched[i % len(sched)]], cols, False, pybic.CODER_GOLOMB, slot, out, bits)
        ctx.sync()
        p = ctx.prof_collect()
        durs.append(round(1e3 * p["encode_rows_golomb"][1], 1))
    ctx.prof_enable(False)
    print(name, "median", float(np.median(durs)), durs, flush=True)


run("alternate 0,1", [0, 1])
run("same 0", [0])
run("same 1", [1])
run("three 0,1,2", [0, 1, 2])
run("pairs 0,0,1,1", [0, 0, 1, 1])


def run_b2b(name, sched, reps=40):
    """back to back, no sync between calls: average call time from events on the ctx stream"""
    for i in range(6):
        ctx.encode_planes(planes[sched[i % len(sched)]], cols, False, pybic.CODER_GOLOMB, slot, out, bits)
    ctx.sync()
    import time
    t0 = time.perf_counter()
    for i in range(reps):
        ctx.encode_planes(planes[sched[i % len(sched)]], cols, False, pybic.CODER_GOLOMB, slot, out, bits)
    ctx.sync()
    print(name, "back-to-back us/call", round((time.perf_counter() - t0) / reps * 1e6, 1), flush=True)


run_b2b("alternate 0,1", [0, 1])
run_b2b("same 0", [0])
run_b2b("three 0,1,2", [0, 1, 2])
