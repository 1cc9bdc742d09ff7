"""The CPU restatement (oracle/) against the golden vectors produced by the reference's own
objects (tests/golden/make_golden.py). CPU only."""
import os

import numpy as np
import pytest

from pnm_io import read_pbm_bytes

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_golomb_kat(oracle, golden):
    meta, A = golden
    for name, bits in meta["golomb"].items():
        s = A[f"golomb_{name}_s"]
        b, _, k, ln = oracle.golomb_samples(s, want_stream=False)
        assert b == bits, name
        assert np.array_equal(k, A[f"golomb_{name}_k"]), name
        assert np.array_equal(ln, A[f"golomb_{name}_len"]), name


def test_golomb_survey_vector(oracle):
    # SURVEY.md §8 c known answer (probe of GolombCoder.cpp:29-34)
    b, _, k, ln = oracle.golomb_samples([0, 0, 0, 5, 3, 0, 12, 1, 100, 7, 0, 0, 1, 2, 3], want_stream=False)
    assert list(k) == [1, 0, 0, 0, 1, 1, 1, 2, 2, 4, 4, 4, 4, 4, 4]
    assert list(ln) == [2, 1, 1, 6, 3, 2, 8, 3, 28, 5, 5, 5, 5, 5, 5]
    assert b == 84


def test_planes_med_weight_bits(oracle, golden):
    meta, A = golden
    for c in meta["planes"]:
        P = A[c["key"]]
        cols = c["cols"]
        assert np.array_equal(oracle.med(P, cols), A[c["key"] + "_med"]), c["key"]
        assert oracle.weight(P, cols) == c["weight"]
        assert oracle.weight(oracle.med(P, cols), cols) == c["weight_med"]
        for pred in (0, 1):
            gb, _, _ = oracle.encode_plane(P, cols, pred, 0, want_stream=False)
            eb, _, _ = oracle.encode_plane(P, cols, pred, 1, want_stream=False)
            assert gb == c[f"golomb_bits_pred{pred}"], (c["key"], pred)
            assert eb == c[f"eg_bits_pred{pred}"], (c["key"], pred)


def test_eg_closed_form(oracle, golden):
    # EG as written costs rows*(cols+1) + 1 bits on any plane with a 1
    meta, A = golden
    for c in meta["planes"]:
        P = A[c["key"]]
        R = oracle.med(P, c["cols"])
        has1 = oracle.weight(R, c["cols"]) > 0
        assert c["eg_bits_pred1"] == c["rows"] * (c["cols"] + 1) + int(has1)


def test_tiles(oracle, golden):
    meta, A = golden
    for c in meta["tiles"]:
        k = c["key"]
        res = oracle.patch_encode(A[k + "_in"], c["cols"], c["W"], A[k + "_lentab"])
        assert res["bits"] == c["bits"], k
        assert res["L"] == c["L"], k
        assert res["modes"] == c["modes"], k
        assert np.array_equal(res["w_nonpred"], A[k + "_w_nonpred"]), k
        assert np.array_equal(res["w_pred"], A[k + "_w_pred"]), k
        # residual image, pixel bits only
        rows, cols = c["rows"], c["cols"]
        for i in range(rows):
            for j in range(cols):
                w, b = j // 64, np.uint64(63 - j % 64)
                assert (res["residual"][i, w] >> b) & np.uint64(1) == (A[k + "_resid"][i, w] >> b) & np.uint64(1)


def test_submatrix_wrap(oracle, golden):
    meta, A = golden
    I = A["submat_in"]
    for k, (i0, i1, j0, j1) in enumerate(meta["submatrix"]):
        got = oracle.get_submatrix(I, 100, i0, i1, j0, j1)
        exp = A[f"submat_{k}"]
        W = j1 - j0
        mask = np.uint64(((1 << 64) - 1) ^ ((1 << (64 - W)) - 1)) if W < 64 else np.uint64((1 << 64) - 1)
        assert np.array_equal(got & mask, exp & mask), k


def test_bitplanes_vs_reference_tool(oracle, golden):
    meta, A = golden
    for name, info in meta["bitplane_tool"].items():
        data = open(os.path.join(GOLD, name), "rb").read()
        # parse our own fixture PGM (P5, maxval, optional comment)
        toks, pos = [], 2
        while len(toks) < 3:
            while data[pos:pos + 1].isspace():
                pos += 1
            if data[pos:pos + 1] == b"#":
                pos = data.index(b"\n", pos) + 1
                continue
            e = pos
            while not data[e:e + 1].isspace():
                e += 1
            toks.append(int(data[pos:e]))
            pos = e
        cols, rows, maxval = toks
        pos += 1
        dt = np.uint8 if maxval < 256 else np.dtype(">u2")
        gray = np.frombuffer(data[pos:], dt, rows * cols).reshape(rows, cols).astype(
            np.uint8 if maxval < 256 else np.uint16)
        n = oracle.lib.bo_num_planes(maxval)
        assert n == info["nplanes"]
        planes = oracle.bitplanes(gray, n)
        for b in range(n):
            r2, c2, ref_plane = read_pbm_bytes(A[f"bt_{name}_{b}"].tobytes())
            assert (r2, c2) == (rows, cols)
            assert np.array_equal(planes[b], ref_plane), (name, b)


def test_decode_roundtrip(oracle):
    for (rows, cols, p) in [(37, 70, 0.5), (64, 200, 0.05), (5, 1, 0.5), (8, 64, 0.0), (8, 64, 1.0)]:
        P = oracle.gen_plane(99, p, rows, cols)
        for pred in (0, 1):
            b, st, _ = oracle.encode_plane(P, cols, pred, 0)
            corner = int(P[0, 0] >> np.uint64(63))
            rc, Q = oracle.decode_plane_golomb(st, b, rows, cols, pred, corner)
            assert rc == 0 and np.array_equal(P, Q)


@pytest.mark.parametrize("rows,cols,p,pred", [(40, 1000, 0.5, 1), (17, 16384, 0.05, 1), (9, 65, 0.9, 0),
                                              (3, 64, 0.0, 1), (25, 300, 0.3, 0)])
def test_cpu_fast_matches_oracle(oracle, rows, cols, p, pred):
    """bench.py's strong-CPU line (oracle/cpu_fast.c, word-parallel) writes the oracle's streams"""
    P = np.stack([oracle.gen_plane(0x5EED + k, p if k else 0.5, rows, cols) for k in range(3)])
    gb, eb, G, E, _ = oracle.fast_encode(P, cols, pred)
    for k in range(3):
        for coder, bits, S in ((0, gb, G), (1, eb, E)):
            b, st, _ = oracle.encode_plane(P[k], cols, pred, coder)
            assert int(bits[k]) == b, (k, coder)
            assert S[k, :len(st) // 8].tobytes() == st.tobytes(), (k, coder)


@pytest.mark.parametrize("name", ["survey", "short", "long", "plane_64x1000"])
def test_eg_adaptive_kat(oracle, golden, name):
    """the oracle's adaptive EG (coder 2) == the reference's EG state machine with incBlockSize
    enabled (golden vectors from oracle/ref_capi.cpp ref_eg_adaptive): per-run bits and the stream"""
    meta, arr = golden
    lens, eols = arr[f"egad_{name}_len"], arr[f"egad_{name}_eol"]
    bits, per, stream = oracle.eg_runs(lens, eols, 1)
    assert bits == meta["eg_adaptive"][name]
    assert np.array_equal(per, arr[f"egad_{name}_bits"])
    assert stream.tobytes() == arr[f"egad_{name}_stream"].tobytes()


def test_gf2_algebra_golden(oracle):
    """oracle bo_gf2_mul / bo_gf2_transpose vs mul() / transpose_to run on the reference's objects
    (tests/golden/make_golden_gf2.py, binmat.cpp:199-214, 516-616)"""
    import json
    import os

    g = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    with open(os.path.join(g, "gf2.json")) as f:
        meta = json.load(f)
    A = np.load(os.path.join(g, "gf2.npz"), allow_pickle=False)
    for n, m in enumerate(meta["mul"]):
        (ar, ac), (br, bc), (cr, cc) = m["a"], m["b"], m["c"]
        got = oracle.gf2_mul(m["op"], A[f"mul{n}_A"], ar, ac, A[f"mul{n}_B"], br, bc, A[f"mul{n}_C0"], cr, cc)
        assert np.array_equal(got, A[f"mul{n}_C"]), (n, m)
    for n, (rows, cols) in enumerate(meta["transpose"]):
        assert np.array_equal(oracle.gf2_transpose(A[f"tr{n}_in"], rows, cols), A[f"tr{n}_out"]), n
