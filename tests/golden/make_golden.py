"""Generate tests/golden/ fixtures FROM THE REFERENCE'S OWN OBJECTS.

Run in the build container only (needs /root/reference and oracle/_ref, built by
`make -C oracle ref`):  python tests/golden/make_golden.py

Every expected value below comes from the reference code compiled from /root/reference/src
(oracle/_ref/libref.so: binary_matrix, med, GolombCoder, EGCoder, pbm/pnm readers and
writers; oracle/_ref/bitplane_tool: the reference's own bitplane_tool main). Inputs are
seeded synthetic data (splitmix64 from oracle/liboracle.so, or numpy with a fixed seed).
The outputs are plain data (npz without pickles, JSON, PBM/PGM files).
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle_lib import Oracle, Ref  # noqa: E402
from pnm_io import write_pbm, write_pgm  # noqa: E402

REF_BITPLANE_TOOL = os.path.join(ROOT, "oracle", "_ref", "bitplane_tool")


def main():
    o, r = Oracle(), Ref()
    arrays = {}
    meta = {"generator": "tests/golden/make_golden.py", "source": "reference objects (oracle/_ref)"}

    # ---- Golomb KATs (GolombCoder.cpp:13-34) ------------------------------------------
    rng = np.random.default_rng(20241015)
    seqs = {
        "survey": np.array([0, 0, 0, 5, 3, 0, 12, 1, 100, 7, 0, 0, 1, 2, 3], np.uint32),
        "geo_small": rng.geometric(0.5, 3000).astype(np.uint32) - 1,
        "geo_large": rng.geometric(0.01, 3000).astype(np.uint32) - 1,
        "mixed": np.concatenate([np.zeros(200, np.uint32), rng.integers(0, 1 << 16, 500).astype(np.uint32),
                                 np.zeros(2000, np.uint32), rng.integers(0, 8, 500).astype(np.uint32)]),
        "big_then_dense": np.concatenate([np.array([1 << 20], np.uint32), np.zeros(4000, np.uint32),
                                          np.ones(100, np.uint32)]),
    }
    meta["golomb"] = {}
    for name, s in seqs.items():
        bits, k, ln = r.golomb(s)
        arrays[f"golomb_{name}_s"] = s
        arrays[f"golomb_{name}_k"] = k
        arrays[f"golomb_{name}_len"] = ln
        meta["golomb"][name] = bits

    # ---- EG KATs (eg.cpp:20-37, as written) ---------------------------------------------
    eg_cases = {
        "survey": (np.array([3, 0, 7, 2], np.int32), np.array([0, 0, 1, 1], np.uint8)),
        "eol_first": (np.array([4, 2, 0, 9, 1], np.int32), np.array([1, 0, 0, 1, 0], np.uint8)),
        "random": (rng.integers(0, 300, 2000).astype(np.int32), (rng.random(2000) < 0.2).astype(np.uint8)),
    }
    meta["eg"] = {}
    for name, (lens, eols) in eg_cases.items():
        bits, per = r.eg(lens, eols)
        arrays[f"eg_{name}_len"] = lens
        arrays[f"eg_{name}_eol"] = eols
        arrays[f"eg_{name}_bits"] = per
        meta["eg"][name] = bits

    # ---- adaptive EG KATs (eg.cpp:20-37 with line 25's incBlockSize enabled) --------------
    # from the reference's own EG state machine (incBlockSize / decBlockSize / EGLUT), the writes
    # of eg.cpp:24/29/32-33 as an MSB-first bit string (oracle/ref_capi.cpp ref_eg_adaptive)
    rng_ad = np.random.default_rng(777)
    Pad = o.gen_plane(0x5EED00AD, 0.1, 64, 1000)
    run_l, run_e = o.plane_runs(o.med(Pad, 1000), 1000)
    egad_cases = {
        "survey": (np.array([3, 0, 7, 2], np.int32), np.array([0, 0, 1, 1], np.uint8)),
        "short": ((rng_ad.geometric(0.5, 3000) - 1).astype(np.int32), (rng_ad.random(3000) < 0.02).astype(np.uint8)),
        "long": (rng_ad.integers(0, 20000, 500).astype(np.int32), (rng_ad.random(500) < 0.3).astype(np.uint8)),
        "plane_64x1000": (run_l.astype(np.int32), run_e.astype(np.uint8)),
    }
    meta["eg_adaptive"] = {}
    for name, (lens, eols) in egad_cases.items():
        bits, per, stream = r.eg_adaptive(lens, eols)
        arrays[f"egad_{name}_len"] = lens
        arrays[f"egad_{name}_eol"] = eols
        arrays[f"egad_{name}_bits"] = per
        arrays[f"egad_{name}_stream"] = stream
        meta["eg_adaptive"][name] = bits

    # ---- planes: med residual, weights, Golomb/EG bitcounts of the run samples -----------
    plane_cases = [
        (1, 1, 0.5, 1), (1, 64, 0.5, 2), (1, 65, 0.3, 3), (2, 1, 0.5, 4), (3, 1, 1.0, 5),
        (37, 70, 0.5, 6), (64, 64, 0.5, 7), (64, 128, 0.1, 8), (50, 200, 0.02, 9),
        (130, 130, 0.5, 10), (16, 1000, 0.3, 11), (256, 256, 0.05, 12), (20, 300, 0.0, 13),
        (20, 300, 1.0, 14), (9, 5000, 0.5, 15), (128, 4096, 0.5, 16), (40, 16384, 0.02, 17),
    ]
    meta["planes"] = []
    for (rows, cols, p, seed) in plane_cases:
        P = o.gen_plane(0x5EED0000 + seed, p, rows, cols)
        R = r.med(P, cols)
        case = dict(rows=rows, cols=cols, p=p, seed=seed, weight=r.weight(P, cols), weight_med=r.weight(R, cols))
        for pred in (0, 1):
            _, gb, eb, _ = r.baseline(P[None], rows, cols, predict=pred, do_eg=1, threads=1)
            case[f"golomb_bits_pred{pred}"] = gb
            case[f"eg_bits_pred{pred}"] = eb
        key = f"plane_{rows}x{cols}_{seed}"
        arrays[key] = P
        arrays[key + "_med"] = R
        case["key"] = key
        meta["planes"].append(case)

    # ---- tiles: compress7_test R = 0 loop (lentab from the build's enumL; GSL absent) ---
    tile_cases = [(64, 64, 32, 0.5, 21), (128, 128, 32, 0.02, 22), (96, 96, 8, 0.1, 23),
                  (50, 70, 5, 0.3, 24), (100, 100, 10, 0.05, 25), (128, 192, 64, 0.5, 26),
                  (256, 256, 32, 0.01, 27)]
    meta["tiles"] = []
    for (rows, cols, W, p, seed) in tile_cases:
        I = o.gen_plane(0x5EED0000 + seed, p, rows, cols)
        lt = o.lentab(W)
        res = r.tile_loop(I, cols, W, lt)
        key = f"tiles_{rows}x{cols}_W{W}"
        arrays[key + "_in"] = I
        arrays[key + "_lentab"] = lt
        arrays[key + "_w_nonpred"] = res["w_nonpred"]
        arrays[key + "_w_pred"] = res["w_pred"]
        arrays[key + "_resid"] = res["residual"]
        meta["tiles"].append(dict(key=key, rows=rows, cols=cols, W=W, p=p, seed=seed, bits=res["bits"],
                                  L=res["L"], modes=res["modes"]))

    # ---- get_submatrix incl. the right-edge wrap (binmat.cpp:286-291) -------------------
    I = o.gen_plane(0x5EED0031, 0.5, 6, 100)
    arrays["submat_in"] = I
    meta["submatrix"] = []
    for k, (i0, i1, j0, j1) in enumerate([(1, 3, 95, 100), (4, 6, 60, 65), (5, 6, 99, 104), (0, 6, 0, 64),
                                          (2, 5, 30, 94), (3, 6, 62, 67)]):
        arrays[f"submat_{k}"] = r.get_submatrix(I, 100, i0, i1, j0, j1)
        meta["submatrix"].append([i0, i1, j0, j1])

    # ---- PBM / PGM readers and the reference's own bitplane_tool ------------------------
    files = {}
    pbm_plane = o.gen_plane(0x5EED0041, 0.5, 37, 70)
    # first raster byte must not be a whitespace byte (SURVEY.md §4 hazard 2)
    first = int(pbm_plane[0, 0] >> np.uint64(56))
    if first in (0x09, 0x0A, 0x0B, 0x0C, 0x0D, 0x20):
        pbm_plane[0, 0] ^= np.uint64(0x8000000000000000)
    files["camera_70x37.pbm"] = write_pbm(os.path.join(HERE, "camera_70x37.pbm"), pbm_plane, 70)
    ws_plane = o.gen_plane(0x5EED0042, 0.5, 2, 32)
    ws_plane[0, 0] = np.uint64(0x200A81FF00000000)  # raster starts 20 0a: swallowed by " %d "
    files["ws_32x2.pbm"] = write_pbm(os.path.join(HERE, "ws_32x2.pbm"), ws_plane, 32)
    meta["pbm"] = {}
    with tempfile.TemporaryDirectory() as td:
        for name in ("camera_70x37.pbm", "ws_32x2.pbm"):
            path = os.path.join(HERE, name)
            rows, cols, words = r.read_pbm(path)
            arrays[f"pbm_{name}_read"] = words
            copy = os.path.join(td, "copy.pbm")
            r.pbm_roundtrip(path, copy)
            with open(copy, "rb") as f:
                arrays[f"pbm_{name}_roundtrip"] = np.frombuffer(f.read(), np.uint8).copy()
            meta["pbm"][name] = dict(rows=rows, cols=cols)

        rngi = np.random.default_rng(7)
        gray8 = rngi.integers(0, 256, (40, 48)).astype(np.uint8)
        write_pgm(os.path.join(HERE, "gray_48x40.pgm"), gray8, 255, comment="fixture")
        gray16 = rngi.integers(0, 1001, (12, 20)).astype(np.uint16)
        write_pgm(os.path.join(HERE, "gray16_20x12.pgm"), gray16, 1000)
        meta["bitplane_tool"] = {}
        for name, maxval in (("gray_48x40.pgm", 255), ("gray16_20x12.pgm", 1000)):
            wd = os.path.join(td, name)
            os.makedirs(wd)
            subprocess.run([REF_BITPLANE_TOOL, os.path.join(HERE, name)], cwd=wd, check=True,
                           stdout=subprocess.DEVNULL)
            planes = sorted(f for f in os.listdir(wd) if f.startswith("plane_"))
            meta["bitplane_tool"][name] = dict(maxval=maxval, nplanes=len(planes))
            for k, pf in enumerate(planes):
                with open(os.path.join(wd, pf), "rb") as f:
                    arrays[f"bt_{name}_{k}"] = np.frombuffer(f.read(), np.uint8).copy()

    np.savez_compressed(os.path.join(HERE, "golden.npz"), **arrays)
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote", len(arrays), "arrays")


if __name__ == "__main__":
    main()
