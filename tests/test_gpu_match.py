"""compress7_test.cpp's tile loop with a search window (bic_match_encode, csrc/bic_match.hip)
against the oracle (bo_match_encode, itself pinned to the driver's loop over the reference
objects in tests/test_ref_crosscheck.py::test_match_encode). Bit-exact: per-tile search results,
modes, coded weights, the residual image, both Golomb streams and the totals."""
import numpy as np
import pytest

from oracle_lib import periodic_plane
from pybic import as_u64, stream_bytes

pytestmark = pytest.mark.gpu

CASES = [  # W, rows, cols, T, R, input
    (8, 64, 128, 0, 32, ("periodic", 8, 8, 0.5, 0.0)),
    (8, 64, 96, 2, 24, ("periodic", 8, 24, 0.5, 0.01)),
    (5, 40, 60, 0, 12, ("periodic", 7, 11, 0.4, 0.0)),
    (4, 32, 64, 1, 4, ("random", 0.1)),
    (4, 32, 64, 0, 2, ("random", 0.3)),    # R < W: empty regions, search_win_size <= 0
    (16, 64, 128, 0, 40, ("periodic", 16, 32, 0.3, 0.002)),
    (6, 36, 72, 40, 12, ("random", 0.5)),  # large T: the first window of the scan ends the search
    (8, 48, 64, 0, 128, ("random", 0.02)),
    (16, 256, 256, 0, 128, ("periodic", 24, 40, 0.5, 0.001)),  # compress7's defaults (W 16, R 128)
    (16, 128, 512, 3, 128, ("random", 0.5)),                    # region beyond the LDS image
    (12, 96, 240, 0, 60, ("periodic", 12, 20, 0.2, 0.0)),      # tiles straddle words
    (32, 128, 256, 0, 80, ("periodic", 32, 64, 0.5, 0.003)),
    (64, 192, 320, 0, 64, ("random", 0.05)),
    (1, 8, 70, 0, 5, ("random", 0.5)),
    (16, 512, 512, 0, 128, ("random", 0.01)),                   # 1024 tiles, sparse: early exits
    (16, 48, 6400, 0, 128, ("random", 0.02)),                   # too wide for the row schedule
    (8, 96, 200, 0, 50, ("text",)),
    (16, 160, 320, 1, 96, ("text",)),
    (20, 100, 300, 0, 60, ("text",)),
]
# schedules (bic_set_match_parts): automatic, a row workgroup alone, a row workgroup with 3 helpers,
# workgroups per tile
AUTO, ROW, TEAM3, TILE = 0, 0x10000, 0x10003, 0xFFFFFFFF


def make_input(oracle, seed, rows, cols, spec):
    if spec[0] == "text":
        from oracle_lib import text_plane
        return text_plane(seed, rows, cols)
    if spec[0] == "periodic":
        return periodic_plane(seed, rows, cols, spec[1], spec[2], spec[3], spec[4])
    return oracle.gen_plane(seed, spec[1], rows, cols)


def check(ctx, oracle, I, cols, W, T, R, parts=0, invert=False):
    e = oracle.enum_table(W)
    exp = oracle.match_encode(I, cols, W, T, R, e, invert=invert)
    ctx.set_match_parts(parts)
    try:
        got = ctx.match_encode(ctx.to_dev(I), cols, W, T, R, e, invert=invert)
        ctx.sync()
    finally:
        ctx.set_match_parts(0)
    for k in ("besti", "bestj", "bestd", "weights"):
        assert np.array_equal(got[k].cpu().numpy().view(np.uint32), exp[k]), k
    if invert:
        assert np.array_equal(got["inverted"].cpu().numpy(), exp["inverted"])
    assert got["modes"].cpu().numpy().tobytes().decode() == exp["modes"]
    assert np.array_equal(as_u64(got["resid"]), exp["residual"])
    st = as_u64(got["stats"])
    assert [int(x) for x in st] == [exp["matches"], exp["bits_match"], exp["bits_nomatch"], exp["L"]]
    assert stream_bytes(got["stream_match"], st[1]) == exp["stream_match"].tobytes()
    assert stream_bytes(got["stream_nomatch"], st[2]) == exp["stream_nomatch"].tobytes()
    return exp


@pytest.mark.parametrize("sched", [AUTO, ROW, TEAM3, TILE])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_match_encode(ctx, oracle, case, sched):
    W, rows, cols, T, R, spec = CASES[case]
    I = make_input(oracle, 5000 + case, rows, cols, spec)
    exp = check(ctx, oracle, I, cols, W, T, R, sched)
    if spec[0] in ("periodic", "text"):
        assert exp["matches"] > 0


INV_CASES = [  # W, rows, cols, T, R, input (compress8_test.cpp: patch inversion)
    (8, 64, 128, 0, 32, ("inverted", 8, 8, 0.5, 0.0, 3)),
    (8, 64, 96, 2, 24, ("inverted", 8, 24, 0.5, 0.01, 2)),
    (5, 40, 60, 0, 12, ("inverted", 5, 10, 0.4, 0.0, 4)),
    (4, 32, 64, 1, 4, ("random", 0.9)),
    (4, 32, 64, 0, 2, ("random", 0.3)),
    (16, 64, 128, 3, 40, ("inverted", 16, 32, 0.3, 0.002, 1)),
    (6, 36, 72, 40, 12, ("random", 0.5)),
    (16, 256, 256, 2, 128, ("inverted", 16, 48, 0.5, 0.001, 6)),  # compress8's defaults (W 16, R 128)
    (32, 128, 256, 0, 80, ("inverted", 32, 64, 0.5, 0.003, 2)),
    (12, 96, 240, 0, 60, ("inverted", 12, 24, 0.2, 0.0, 3)),
    (16, 48, 6400, 0, 128, ("random", 0.98)),                      # too wide for the row schedule
    (16, 160, 320, 1, 96, ("text",)),
]


@pytest.mark.parametrize("sched", [AUTO, ROW, TEAM3, TILE])
@pytest.mark.parametrize("case", range(len(INV_CASES)))
def test_match_encode_inverted(ctx, oracle, case, sched):
    """bic_match_encode_inv (compress8_test.cpp's loop) against the oracle's bo_match_encode_v, itself
    pinned to the driver's loop over the reference objects (test_ref_crosscheck.py), every schedule"""
    from oracle_lib import inverted_plane
    W, rows, cols, T, R, spec = INV_CASES[case]
    if spec[0] == "inverted":
        I = inverted_plane(6000 + case, rows, cols, *spec[1:])
    else:
        I = make_input(oracle, 6000 + case, rows, cols, spec)
    exp = check(ctx, oracle, I, cols, W, T, R, sched, invert=True)
    if spec[0] == "inverted":
        assert exp["inverted"].any() and exp["matches"] > 0


@pytest.mark.parametrize("parts", [1, 3, 17])
def test_match_parts(ctx, oracle, parts):
    """the split of a tile's scan over workgroups does not change the result"""
    I = periodic_plane(77, 128, 256, 16, 40, 0.5, 0.002)
    check(ctx, oracle, I, 256, 16, 0, 100, parts)


def test_match_default_table(ctx, oracle):
    """this build's enumL table (bic_enum_codelength) equals the oracle's"""
    import pybic
    W = 16
    assert np.array_equal(pybic.enum_table(W), oracle.enum_table(W))


def test_match_repeat_and_in_place(ctx, oracle):
    """repeated calls reuse the scratch; resid may alias the plane"""
    I = periodic_plane(5, 64, 128, 8, 16, 0.5, 0.01)
    e = oracle.enum_table(8)
    exp = oracle.match_encode(I, 128, 8, 0, 32, e)
    for _ in range(3):
        d = ctx.to_dev(I)
        got = ctx.match_encode(d, 128, 8, 0, 32, e, resid=d)
        ctx.sync()
        assert np.array_equal(as_u64(d), exp["residual"])
        assert got["modes"].cpu().numpy().tobytes().decode() == exp["modes"]


VAR_CASES = CASES[:8] + [
    (4, 32, 64, 0, 10000, ("random", 0.03)),    # the drivers' default R: the whole image above
    (8, 64, 64, 3, 10000, ("periodic", 8, 16, 0.5, 0.02)),
    (6, 36, 72, 18, 20, ("random", 0.5)),       # T = worstd: compress5's exit at its first replacement
    (6, 36, 72, 37, 20, ("random", 0.5)),       # T >= M + 1: every search ends after its first window
    (16, 256, 256, 0, 10000, ("periodic", 24, 40, 0.5, 0.001)),  # region beyond the LDS image
    (8, 96, 200, 0, 10000, ("text",)),
    (8, 512, 512, 0, 64, ("text",)),             # 512^2, the drivers' W
    (4, 512, 512, 2, 32, ("random", 0.05)),
]


@pytest.mark.parametrize("parts", [0, 1, 5])
@pytest.mark.parametrize("variant", [4, 5, 6])
@pytest.mark.parametrize("case", range(len(VAR_CASES)))
def test_match_encode_variants(ctx, oracle, case, variant, parts):
    """bic_match_encode_var (the loops of compress4/5/6_test.cpp) against the oracle's
    bo_match_encode_var, itself pinned to each driver's loop over the reference objects
    (test_ref_crosscheck.py::test_match_encode_variants); automatic and fixed per-tile splits"""
    from oracle_lib import match_encode_var
    W, rows, cols, T, R, spec = VAR_CASES[case]
    I = make_input(oracle, 7000 + case, rows, cols, spec)
    e = oracle.enum_table(W)
    exp = match_encode_var(oracle, I, cols, W, T, R, e, variant)
    ctx.set_match_parts(parts)
    try:
        got = ctx.match_encode(ctx.to_dev(I), cols, W, T, R, e, variant=variant)
        ctx.sync()
    finally:
        ctx.set_match_parts(0)
    for k in ("besti", "bestj", "bestd", "weights"):
        assert np.array_equal(got[k].cpu().numpy().view(np.uint32), exp[k]), k
    assert got["modes"].cpu().numpy().tobytes().decode() == exp["modes"]
    assert np.array_equal(as_u64(got["resid"]), exp["residual"])
    st = as_u64(got["stats"])
    assert [int(x) for x in st] == [exp["matches"], exp["bits_match"], exp["bits_nomatch"], exp["L"]]
    assert stream_bytes(got["stream_match"], st[1]) == exp["stream_match"].tobytes()
    assert stream_bytes(got["stream_nomatch"], st[2]) == exp["stream_nomatch"].tobytes()
