"""Generate tests/golden/gf2.npz + gf2.json FROM THE REFERENCE'S OWN OBJECTS: the binary_matrix
algebra over GF(2) -- mul(A, At, B, Bt, C) (binmat.cpp:516-616) and transpose_to
(binmat.cpp:199-214) run on oracle/_ref/libref.so (ref_gf2_mul / ref_gf2_transpose).

Run in the build container only (needs oracle/_ref, `make -C oracle ref`):
    python tests/golden/make_golden_gf2.py
Inputs are seeded planes (splitmix64 from oracle/liboracle.so); outputs are plain data (npz
without pickles, JSON). mul_ABt is only generated for B.cols <= B.rows: past that the reference
reads B and writes C past their buffers (binmat.cpp:584-592)."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle_lib import Oracle, Ref  # noqa: E402

# (op, a_rows, a_cols, b_rows, b_cols); C's shape follows from op
MUL_CASES = [
    (0, 1, 1, 1, 1), (0, 5, 70, 70, 3), (0, 64, 64, 64, 64), (0, 37, 130, 130, 65), (0, 100, 200, 200, 150),
    (1, 70, 5, 70, 3), (1, 130, 37, 130, 65), (1, 200, 100, 200, 150), (1, 64, 64, 64, 129),
    (2, 5, 3, 70, 3), (2, 37, 65, 130, 65), (2, 100, 150, 200, 150), (2, 20, 100, 90, 100), (2, 64, 64, 64, 64),
    (3, 7, 9, 9, 7),
]
TRANSPOSE_CASES = [(1, 1), (70, 37), (130, 200), (64, 128), (3, 65)]


def c_shape(op, ar, ac, br, bc):
    return {0: (ar, bc), 1: (ac, bc), 2: (ar, br), 3: (ac, br)}[op]


def main():
    o, r = Oracle(), Ref()
    arrays, meta = {}, {"mul": [], "transpose": []}
    for n, (op, ar, ac, br, bc) in enumerate(MUL_CASES):
        cr, cc = c_shape(op, ar, ac, br, bc)
        A = o.gen_plane(0x6F200000 + 4 * n, 0.5, ar, ac)
        B = o.gen_plane(0x6F200001 + 4 * n, 0.3, br, bc)
        C0 = o.gen_plane(0x6F200002 + 4 * n, 0.5, cr, cc)  # mul_ABt / mul_AtBt keep bits of C
        arrays[f"mul{n}_A"], arrays[f"mul{n}_B"], arrays[f"mul{n}_C0"] = A, B, C0
        arrays[f"mul{n}_C"] = r.gf2_mul(op, A, ar, ac, B, br, bc, C0, cr, cc)
        meta["mul"].append(dict(op=op, a=[ar, ac], b=[br, bc], c=[cr, cc]))
    for n, (rows, cols) in enumerate(TRANSPOSE_CASES):
        M = o.gen_plane(0x6F210000 + n, 0.5, rows, cols)
        arrays[f"tr{n}_in"] = M
        arrays[f"tr{n}_out"] = r.gf2_transpose(M, rows, cols)
        meta["transpose"].append([rows, cols])
    np.savez_compressed(os.path.join(HERE, "gf2.npz"), **arrays)
    with open(os.path.join(HERE, "gf2.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote", len(arrays), "arrays")


if __name__ == "__main__":
    main()
