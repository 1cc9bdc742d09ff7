"""Oracle vs the reference objects on fresh random inputs (this container only: skipped
where oracle/_ref was not built, e.g. on the GPU box when the reference is absent)."""
import numpy as np
import pytest

from oracle_lib import have_ref

pytestmark = pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built (needs /root/reference)")


@pytest.fixture(scope="module")
def ref():
    from oracle_lib import Ref
    return Ref()


@pytest.mark.parametrize("seed", range(6))
def test_random_planes(oracle, ref, seed):
    rng = np.random.default_rng(seed)
    rows, cols = int(rng.integers(1, 90)), int(rng.integers(1, 300))
    p = float(rng.choice([0.5, 0.2, 0.03, 0.0, 1.0]))
    P = oracle.gen_plane(1000 + seed, p, rows, cols)
    assert np.array_equal(oracle.med(P, cols), ref.med(P, cols))
    for pred in (0, 1):
        _, gb, eb, _ = ref.baseline(P[None], rows, cols, predict=pred, do_eg=1, threads=1)
        assert oracle.encode_plane(P, cols, pred, 0, want_stream=False)[0] == gb
        assert oracle.encode_plane(P, cols, pred, 1, want_stream=False)[0] == eb


@pytest.mark.parametrize("W", [3, 5, 8, 16, 32])
def test_random_tiles(oracle, ref, W):
    rng = np.random.default_rng(W)
    rows, cols = int(rng.integers(W, 6 * W)), int(rng.integers(W, 7 * W))
    I = oracle.gen_plane(2000 + W, 0.2, rows, cols)
    lt = oracle.lentab(W)
    a, b = oracle.patch_encode(I, cols, W, lt), ref.tile_loop(I, cols, W, lt)
    for k in ("bits", "L", "modes"):
        assert a[k] == b[k]
    assert np.array_equal(a["w_pred"], b["w_pred"])


@pytest.mark.parametrize("W,rows,cols,p", [(5, 37, 70, 0.3), (3, 20, 33, 0.5), (8, 40, 128, 0.1), (5, 26, 64, 0.02),
                                           (4, 16, 50, 0.0)])
def test_patch_search(oracle, ref, W, rows, cols, p):
    """compress_test.cpp's patch match search: oracle restatement == the reference's own
    get_submatrix/dist loop (edge tiles wrap into the next row; sparse images hit perfect matches)"""
    I = oracle.gen_plane(3000 + W + rows, p, rows, cols)
    a, b = oracle.patch_search(I, cols, W), ref.patch_search(I, cols, W)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


MATCH_CASES = [  # W, rows, cols, T, R, input
    (8, 64, 128, 0, 32, ("periodic", 8, 8, 0.5, 0.0)),
    (8, 64, 96, 2, 24, ("periodic", 8, 24, 0.5, 0.01)),
    (5, 40, 60, 0, 12, ("periodic", 7, 11, 0.4, 0.0)),
    (4, 32, 64, 1, 4, ("random", 0.1)),
    (4, 32, 64, 0, 2, ("random", 0.3)),   # R < W: empty regions, negative search_win_size
    (16, 64, 128, 0, 40, ("periodic", 16, 32, 0.3, 0.002)),
    (6, 36, 72, 40, 12, ("random", 0.5)),  # T >= W*W+1 - ...: the first window always ends the search
    (8, 48, 64, 0, 128, ("random", 0.02)),
]


def match_input(oracle, seed, rows, cols, spec):
    from oracle_lib import periodic_plane
    if spec[0] == "periodic":
        return periodic_plane(seed, rows, cols, spec[1], spec[2], spec[3], spec[4])
    return oracle.gen_plane(seed, spec[1], rows, cols)


@pytest.mark.parametrize("case", range(len(MATCH_CASES)))
def test_match_encode(oracle, ref, case):
    """compress7_test.cpp with a search window: oracle == the driver's loop over the reference's
    own get_submatrix / dist / add / med / set_submatrix / GolombCoder"""
    W, rows, cols, T, R, spec = MATCH_CASES[case]
    I = match_input(oracle, 4000 + case, rows, cols, spec)
    e = oracle.enum_table(W)
    a = oracle.match_encode(I, cols, W, T, R, e, want_stream=False)
    b = ref.match_loop(I, cols, W, T, R, e)
    for k in ("besti", "bestj", "bestd", "weights", "residual"):
        assert np.array_equal(a[k], b[k]), k
    for k in ("modes", "matches", "bits_match", "bits_nomatch", "L"):
        assert a[k] == b[k], k
    if spec[0] == "periodic":
        assert a["matches"] > 0  # the inputs exercise the match branch


MATCH8_CASES = [  # W, rows, cols, T, R, input
    (8, 64, 128, 0, 32, ("inverted", 8, 8, 0.5, 0.0, 3)),
    (8, 64, 96, 2, 24, ("inverted", 8, 24, 0.5, 0.01, 2)),
    (5, 40, 60, 0, 12, ("inverted", 5, 10, 0.4, 0.0, 4)),
    (4, 32, 64, 1, 4, ("random", 0.9)),
    (4, 32, 64, 0, 2, ("random", 0.3)),   # R < W: empty regions
    (16, 64, 128, 3, 40, ("inverted", 16, 32, 0.3, 0.002, 1)),
    (6, 36, 72, 40, 12, ("random", 0.5)),  # T large: initial perfect matches (w <= T or w >= M - T)
    (8, 48, 64, 0, 128, ("random", 0.02)),
    (8, 64, 64, 5, 64, ("ones", 0.0)),     # all-1 tiles: bestinv from the tile weight alone
]


def match8_input(oracle, seed, rows, cols, spec):
    from oracle_lib import inverted_plane, pack_rows
    if spec[0] == "inverted":
        return inverted_plane(seed, rows, cols, *spec[1:])
    if spec[0] == "ones":
        bits = np.ones((rows, cols), bool)
        bits[rows // 2:, :] = np.random.default_rng(seed).random((rows - rows // 2, cols)) < 0.5
        return pack_rows(bits)
    return oracle.gen_plane(seed, spec[1], rows, cols)


@pytest.mark.parametrize("case", range(len(MATCH8_CASES)))
def test_match_encode_inverted(oracle, ref, case):
    """compress8_test.cpp (patch inversion): the oracle's bo_match_encode_v == the driver's loop over
    the reference's own get_submatrix / dist / flip / add / med / set_submatrix / GolombCoder"""
    W, rows, cols, T, R, spec = MATCH8_CASES[case]
    I = match8_input(oracle, 5000 + case, rows, cols, spec)
    e = oracle.enum_table(W)
    a = oracle.match_encode(I, cols, W, T, R, e, want_stream=False, invert=True)
    b = ref.match_loop8(I, cols, W, T, R, e)
    for k in ("besti", "bestj", "bestd", "weights", "residual", "inverted"):
        assert np.array_equal(a[k], b[k]), k
    for k in ("modes", "matches", "bits_match", "bits_nomatch", "L"):
        assert a[k] == b[k], k
    if spec[0] in ("inverted", "ones"):
        assert a["inverted"].any()  # the inputs exercise the inversion


VAR_CASES = MATCH_CASES + [
    (4, 32, 64, 0, 10000, ("random", 0.03)),   # the drivers' default R: the whole image above
    (8, 64, 64, 3, 10000, ("periodic", 8, 16, 0.5, 0.02)),
    (6, 36, 72, 18, 20, ("random", 0.5)),      # T = worstd: compress5's exit at its first replacement
    (6, 36, 72, 37, 20, ("random", 0.5)),      # T >= M + 1: every search ends after its first window
]


@pytest.mark.parametrize("variant", [4, 5, 6])
@pytest.mark.parametrize("case", range(len(VAR_CASES)))
def test_match_encode_variants(oracle, ref, variant, case):
    """compress4/5/6_test.cpp's loops: the oracle's bo_match_encode_var == each driver's loop over the
    reference's own get_submatrix / dist / add / weight / set_submatrix / GolombCoder"""
    from oracle_lib import match_encode_var
    W, rows, cols, T, R, spec = VAR_CASES[case]
    I = match_input(oracle, 6000 + case, rows, cols, spec)
    e = oracle.enum_table(W)
    a = match_encode_var(oracle, I, cols, W, T, R, e, variant, want_stream=False)
    b = ref.match_loop_var(I, cols, W, T, R, e, variant)
    for k in ("besti", "bestj", "bestd", "weights", "residual"):
        assert np.array_equal(a[k], b[k]), k
    for k in ("modes", "matches", "bits_match", "bits_nomatch", "L"):
        assert a[k] == b[k], k
    if spec[0] == "periodic" and variant != 5:  # (compress5 prefers windows at distance just below M / 2)
        assert a["matches"] > 0  # the inputs exercise the match branch


@pytest.mark.parametrize("seed", range(8))
def test_gf2_algebra(oracle, ref, seed):
    """bo_gf2_mul / bo_gf2_transpose vs the reference's mul() and transpose_to on fresh shapes
    (mul_ABt with B.cols <= B.rows: past that the reference reads past B's buffer)"""
    rng = np.random.default_rng(900 + seed)
    op = seed % 4
    ar, ac = int(rng.integers(1, 150)), int(rng.integers(1, 150))
    if op == 0:
        br, bc = ac, int(rng.integers(1, 150))
        cr, cc = ar, bc
    elif op == 1:
        br, bc = ar, int(rng.integers(1, 150))
        cr, cc = ac, bc
    elif op == 2:
        br, bc = int(rng.integers(ac, 200)), ac
        cr, cc = ar, br
    else:
        br, bc = int(rng.integers(1, 150)), ar
        cr, cc = ac, br
    A = oracle.gen_plane(7000 + seed, 0.5, ar, ac)
    B = oracle.gen_plane(7100 + seed, float(rng.choice([0.5, 0.1, 0.9])), br, bc)
    C0 = oracle.gen_plane(7200 + seed, 0.5, cr, cc)
    exp = ref.gf2_mul(op, A, ar, ac, B, br, bc, C0, cr, cc)
    assert np.array_equal(oracle.gf2_mul(op, A, ar, ac, B, br, bc, C0, cr, cc), exp)
    assert np.array_equal(oracle.gf2_transpose(A, ar, ac), ref.gf2_transpose(A, ar, ac))
