"""CPU check of the k = 1 rows' backward-parity encoder (csrc/bic_k1pi.h, used by bic_fused.hip k1_rows
under BIC_K1_PI): tests/cpp/k1pi_check.cpp composes the header's helpers as the kernel does (64 lanes,
lane-consecutive words, the nearest-right-lane parity, the lanes' offsets) and prints each row's bits;
every row whose codewords all have k = 1 (GolombCoder.cpp:13-34 over the med residual) must equal the
oracle's Golomb row bit for bit. Widths cover one, two and four words per lane, rows ending inside a
word and on a word boundary."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from oracle_lib import Oracle

SRC = os.path.join(ROOT, "tests", "cpp", "k1pi_check.cpp")
INC = os.path.join(ROOT, "binary-image-compression_amd", "csrc")


@pytest.fixture(scope="module")
def prog(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("k1pi") / "k1pi_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-I" + INC, "-o", exe, SRC], check=True)
    return exe


def _plane(rng, rows, cols, p):
    wpr = (cols + 63) // 64
    bits = rng.random((rows, wpr * 64)) < p
    bits[:, cols:] = False
    return np.packbits(bits, axis=1).view(">u8").astype(np.uint64).reshape(rows, wpr)


@pytest.mark.parametrize("layout", ["lanes", "strided"])
@pytest.mark.parametrize("cols", [4096, 16384, 8192, 4000, 1000, 130, 70, 64, 16383])
def test_k1_rows_match_oracle(prog, cols, layout):
    """layout "lanes": k1_rows (lane l holds words l WPL ..); "strided": k_emit_known's emit_known_row
    (lane l holds words t * 64 + l)"""
    o = Oracle()
    rng = np.random.default_rng(cols)
    rows = 240 if cols <= 8192 else 96
    P = np.concatenate([_plane(rng, rows // 3, cols, 0.5), _plane(rng, rows // 3, cols, 0.42),
                        _plane(rng, rows - 2 * (rows // 3), cols, 0.36)])
    R = o.med(P, cols)
    nb, st, _ = o.encode_plane(P, cols, 1, 0)
    bits = np.unpackbits(np.frombuffer(st.tobytes(), np.uint8))[:nb]
    offs = list(o.row_index(P, cols, 1)[0::2]) + [nb]
    s, eo = o.plane_runs(R, cols)
    _, _, kk, _ = o.golomb_samples(s, want_stream=False)
    rowid = np.concatenate([[0], np.cumsum(eo)[:-1]]).astype(np.int64)
    kmin = np.full(rows, 99)
    kmax = np.zeros(rows, np.int64)
    np.minimum.at(kmin, rowid, kk.astype(np.int64))
    np.maximum.at(kmax, rowid, kk.astype(np.int64))
    k1 = [r for r in range(rows) if kmin[r] == 1 and kmax[r] == 1]
    assert k1, "the input has no all-k = 1 row"
    inp = f"{cols} {len(k1)}\n" + "\n".join(" ".join(f"{int(w):x}" for w in R[r]) for r in k1) + "\n"
    p = subprocess.run([prog, layout[0]], input=inp, capture_output=True, text=True, check=True)
    got = p.stdout.split("\n")
    for i, r in enumerate(k1):
        exp = "".join(map(str, bits[offs[r]:offs[r + 1]]))
        assert got[i] == exp, (r, len(got[i]), len(exp),
                               next((j for j, (a, b) in enumerate(zip(got[i], exp)) if a != b), None))


@pytest.mark.parametrize("layout", ["lanes", "strided"])
@pytest.mark.parametrize("cols", [4096, 16384, 8192, 4000, 1000, 130, 70, 64, 16383])
def test_kmix_rows_match_oracle(prog, cols, layout):
    """rows whose codewords mix k = 0 and k = 1 (bic_k1pi.h kmix_*; "strided" composes them as
    bic_fused.hip kmix_rows does, and checks kmix_word_len against every word's string): given each codeword's k as the walk's masks (a bit at the 1 ending every k = 1 codeword, and
    the end-of-row codeword's k), the row's bits must equal the oracle's Golomb row"""
    o = Oracle()
    rng = np.random.default_rng(cols + 7)
    rows = 480 if cols <= 8192 else 192
    P = np.concatenate([_plane(rng, rows // 3, cols, 0.5), _plane(rng, rows // 3, cols, 0.45),
                        _plane(rng, rows - 2 * (rows // 3), cols, 0.55)])
    R = o.med(P, cols)
    nb, st, _ = o.encode_plane(P, cols, 1, 0)
    bits = np.unpackbits(np.frombuffer(st.tobytes(), np.uint8))[:nb]
    offs = list(o.row_index(P, cols, 1)[0::2]) + [nb]
    s, eo = o.plane_runs(R, cols)
    _, _, kk, _ = o.golomb_samples(s, want_stream=False)
    kk = kk.astype(np.int64)
    rowid = np.concatenate([[0], np.cumsum(eo)[:-1]]).astype(np.int64)  # (eo flags each row's last sample)
    start = np.searchsorted(rowid, np.arange(rows + 1))
    sel = []
    wpr = R.shape[1]
    lines = []
    for r in range(rows):
        ks = kk[start[r]:start[r + 1]]
        if ks.max() > 1 or ks.min() == ks.max():
            continue
        sel.append(r)
        # the row's 1s in column order, each ending the next sample; the last sample is the end of row
        rb = np.unpackbits(R[r].astype(">u8").view(np.uint8))[:cols]
        cols1 = np.flatnonzero(rb)
        assert len(cols1) + 1 == len(ks)
        kt = np.zeros(wpr * 64, np.uint8)
        kt[cols1[ks[:-1] == 1]] = 1
        ktw = np.packbits(kt).view(">u8").astype(np.uint64)
        lines.append(" ".join(f"{int(w):x}" for w in R[r]) + "\n" + " ".join(f"{int(w):x}" for w in ktw) +
                     f"\n{int(ks[-1])}")
    assert sel, "the input has no mixed row"
    inp = f"{cols} {len(sel)}\n" + "\n".join(lines) + "\n"
    p = subprocess.run([prog, "m" if layout == "lanes" else "n"], input=inp, capture_output=True, text=True, check=True)
    got = p.stdout.split("\n")
    for i, r in enumerate(sel):
        exp = "".join(map(str, bits[offs[r]:offs[r + 1]]))
        assert got[i] == exp, (r, len(got[i]), len(exp),
                               next((j for j, (a, b) in enumerate(zip(got[i], exp)) if a != b), None))
