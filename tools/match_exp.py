"""Timing experiments for bic_match_encode (compress7's tile loop): workgroups per tile x input."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pybic  # noqa: E402
from oracle_lib import text_plane, pack_rows  # noqa: E402


def main():
    ctx = pybic.Context(0)
    rows = cols = int(os.environ.get("N", "512"))
    rows = int(os.environ.get("ROWS", rows))
    cols = int(os.environ.get("COLS", cols))
    W, T, R = int(os.environ.get("W", "16")), 0, int(os.environ.get("R", "128"))
    rng = np.random.default_rng(1)
    inputs = {
        "text": text_plane(1, rows, cols),
        "blank": np.zeros((rows, (cols + 63) // 64), np.uint64),
        "rand50": pack_rows(rng.random((rows, cols)) < 0.5),
    }
    e = pybic.enum_table(W)
    for name, I in inputs.items():
        d = ctx.to_dev(I)
        res = ctx.empty_i64(*I.shape)
        for parts in [int(x) for x in os.environ.get("PARTS", "0,1,4,8,16,32,64").split(",")]:
            ctx.set_match_parts(parts)
            for _ in range(2):
                ctx.match_encode(d, cols, W, T, R, e, resid=res)
            ctx.sync()
            ctx.prof_enable(True)
            for _ in range(5):
                ctx.match_encode(d, cols, W, T, R, e, resid=res)
            prof = ctx.prof_collect()
            ctx.prof_enable(False)
            n, ms = prof["match_tiles"]
            print(f"{rows}x{cols} W={W} R={R} {name:7s} parts={parts:3d} match_tiles {1e3 * ms / n:9.1f} us",
                  flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
