"""Drop-in check of the reference's GSL drivers, SURVEY.md §8 b / §7 step 1: compress_test.cpp,
compress4_test.cpp, compress5_test.cpp, compress6_test.cpp and compress7_test.cpp compiled UNCHANGED
against this build's headers (include/) and libbicpp.so (`make -C oracle gsl_drivers`), run on PBM
inputs, with stdout and diff.pbm required byte-identical to what the reference computes.

GSL is absent from the image. The drivers' one GSL call (gsl_sf_lnchoose) is supplied to this build's
side by tests/cpp/gsl_shim; no reference-side build of the drivers is made (no stand-in headers for
reference builds). The expected bytes come from the reference's own loop objects (libref.so) and the
drivers' print statements restated with their C conversions (tests/dropin_expect.py), with the same
lnchoose. compress8_test.cpp is compiled (it builds unchanged) but not compared: its `idx_t inv;`
(compress8_test.cpp:157, 182) is read uninitialised when a window is not inverted, so its output is
whatever the compiler makes of that read; its loop is pinned with inv = false through ref_match_loop8
(tests/test_ref_crosscheck.py).

Needs /root/reference (this container only); skipped where it is absent (the GPU box).
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from pnm_io import write_pbm

REF_SRC = "/root/reference/src"
DRV = os.path.join(ROOT, "oracle", "_ref", "drv_bic")

pytestmark = pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference sources absent")


@pytest.fixture(scope="module")
def drivers():
    subprocess.run(["make", "-C", os.path.join(ROOT, "binary-image-compression_amd")], check=True,
                   stdout=subprocess.DEVNULL)
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref", "gsl_drivers"], check=True,
                   stdout=subprocess.DEVNULL)
    return DRV


def glyph_plane(seed, rows, cols, g=8, noise=0.002, blank=0.3):
    """text-like plane: g x g glyphs from a small alphabet at a jittered pitch, blank runs, sparse noise
    (so the search finds exact, near and no matches)"""
    rng = np.random.default_rng(seed)
    alphabet = rng.random((6, g, g)) < 0.45
    img = np.zeros((rows, cols), bool)
    y = 1
    while y + g <= rows:
        x = int(rng.integers(0, 3))
        while x + g <= cols:
            if rng.random() > blank:
                img[y:y + g, x:x + g] = alphabet[int(rng.integers(0, len(alphabet)))]
            x += g + int(rng.integers(0, 3))
        y += g + int(rng.integers(1, 3))
    img ^= rng.random((rows, cols)) < noise
    img[0, 0] = True  # (a first raster byte that is not whitespace: pbm.cpp:19's " %d " would eat it)
    wpr = (cols + 63) // 64
    pad = np.zeros((rows, wpr * 64), bool)
    pad[:, :cols] = img
    return np.packbits(pad, axis=1).view(">u8").astype(np.uint64).reshape(rows, wpr)


def run(drivers, tmp, name, pbm, *args, rc=0):
    d = os.path.join(str(tmp), name + "_" + "_".join(map(str, args)))
    os.makedirs(d, exist_ok=True)
    p = subprocess.run([os.path.join(drivers, name), pbm, *map(str, args)], cwd=d, capture_output=True,
                       timeout=600)
    assert p.returncode == rc, (name, p.returncode, p.stderr[-2000:])
    diff = os.path.join(d, "diff.pbm")
    return p.stdout.decode(), open(diff, "rb").read() if os.path.exists(diff) else None


def assert_same_text(got, exp, name):
    if got == exp:
        return
    a, b = got.splitlines(), exp.splitlines()
    i = next((k for k, (x, y) in enumerate(zip(a, b)) if x != y), min(len(a), len(b)))
    raise AssertionError(f"{name}: stdout differs at line {i} of {len(a)}/{len(b)}:\n  got {a[i:i + 3]}\n  exp {b[i:i + 3]}")


def _input(tmp, seed, rows, cols, g=8):
    from oracle_lib import Ref
    P = glyph_plane(seed, rows, cols, g)
    path = write_pbm(os.path.join(str(tmp), f"in_{seed}_{rows}x{cols}.pbm"), P, cols)
    r, c, words = Ref().read_pbm(path)  # the plane as the reference's reader sees the file
    assert (r, c) == (rows, cols)
    return path, words


@pytest.mark.parametrize("rows,cols,W", [(60, 200, 5), (96, 96, 8), (64, 130, 4)])
def test_compress_test(drivers, tmp_path, rows, cols, W):
    """compress_test.cpp (config C1's driver: exhaustive patch search, enumL lengths, two GolombCoders)"""
    import dropin_expect as X
    path, I = _input(tmp_path, rows + cols + W, rows, cols)
    out, _ = run(drivers, tmp_path, "compress_test", path, W)
    assert_same_text(out, X.compress_test(I, rows, cols, W), "compress_test")


def test_compress_test_c1(drivers, tmp_path):
    """config C1 itself: 512 x 512, W = 5"""
    import dropin_expect as X
    path, I = _input(tmp_path, 1, 512, 512)
    out, _ = run(drivers, tmp_path, "compress_test", path, 5)
    assert_same_text(out, X.compress_test(I, 512, 512, 5), "compress_test C1")


@pytest.mark.parametrize("rows,cols,W,T,R", [
    (64, 512, 32, 0, 0),     # the config of SURVEY §7 step 1: W = 32, T = 0, R = 0 (no search window)
    (64, 512, 32, 0, 64),    # a search window
    (48, 256, 8, 3, 16),     # near matches accepted (T > 0)
    (60, 240, 6, 0, 1000),   # the window clipped at every edge
])
def test_compress7_test(drivers, tmp_path, rows, cols, W, T, R):
    """compress7_test.cpp: search window R, threshold T, predictive / non-predictive residuals written
    back into the image (diff.pbm), two GolombCoders, MAP"""
    import dropin_expect as X
    path, I = _input(tmp_path, 7 + rows + W + R, rows, cols)
    out, diff = run(drivers, tmp_path, "compress7_test", path, W, T, R)
    exp, exp_diff = X.compress7_test(I, rows, cols, W, T, R)
    assert_same_text(out, exp, "compress7_test")
    assert diff == exp_diff


@pytest.mark.parametrize("variant", [4, 5, 6])
@pytest.mark.parametrize("rows,cols,W,T,R", [(48, 256, 8, 0, 10000), (40, 200, 8, 4, 24), (48, 256, 8, 31, 10000)])
def test_compress456_test(drivers, tmp_path, variant, rows, cols, W, T, R):
    """compress4/5/6_test.cpp: their search orders and length rules, write-back on a match only; variant 6
    also prints its predictor matrices through operator<< (binmat.cpp:624-644). Variant 5's unsigned
    comparison keeps the window nearest below W*W/2, which rarely pays: with no match at all compress4/5
    divide by zero (compress4_test.cpp:171) and die of SIGFPE, which the drop-in reproduces (same stdout up
    to the last flushed line, same signal)"""
    import dropin_expect as X
    path, I = _input(tmp_path, 40 + variant + R, rows, cols)
    exp, exp_diff, rc = X.compress456_test(I, rows, cols, W, T, R, variant)
    out, diff = run(drivers, tmp_path, f"compress{variant}_test", path, W, T, R, rc=rc)
    assert_same_text(out, exp, f"compress{variant}_test")
    assert diff == exp_diff


def test_compress8_builds(drivers):
    """compress8_test.cpp compiles and links unchanged against include/ + libbicpp.so"""
    assert os.access(os.path.join(drivers, "compress8_test"), os.X_OK)
