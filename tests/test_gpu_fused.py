"""The row encoders (bic_fused.hip: the default staged one, the single kernel and the two-pass one) against the
oracle and against the multi-pass chunk kernels, with inputs built to reach each of their paths:
k = 0 copy mode, byte tables, lanes whose codewords exceed the 128-bit register string, rows whose
output exceeds the LDS window (global fallback), many short rows sharing one output word (fixup
chains), the plane's first 1 (EG's inserted bit)."""
import numpy as np
import pytest

import pybic
from pybic import CODER_EG, CODER_GOLOMB, as_u64, stream_bytes

pytestmark = pytest.mark.gpu

ONES = np.uint64(0xFFFFFFFFFFFFFFFF)
ALT = np.uint64(0xAAAAAAAAAAAAAAAA)


def check(ctx, oracle, P, cols, pred, both=True):
    P = np.asarray(P)
    if P.ndim == 2:
        P = P[None]
    (og, bg), (oe, be) = ctx.encode_planes2(ctx.to_dev(P), cols, pred)
    ctx.sync()
    for k in range(P.shape[0]):
        for coder, out, bits in ((0, og, bg), (1, oe, be)):
            eb, est, _ = oracle.encode_plane(P[k], cols, pred, coder)
            nb = int(as_u64(bits)[k])
            assert nb == eb, (k, coder)
            assert stream_bytes(out[k], nb) == est.tobytes(), (k, coder)


@pytest.fixture(params=["staged", "single-kernel", "two-pass"])
def encoder(request, ctx):
    ctx.set_encoder(request.param)
    yield request.param
    ctx.set_encoder("auto")


@pytest.mark.parametrize("rows,cols", [(1, 1), (3, 64), (7, 65), (64, 100), (50, 1000), (40, 4096), (20, 8191),
                                       (16, 16384), (130, 640)])
@pytest.mark.parametrize("p", [0.5, 0.25, 0.03, 0.0, 1.0])
def test_fused_random(ctx, oracle, encoder, rows, cols, p):
    P = np.stack([oracle.gen_plane(1000 * rows + cols + k + int(p * 97), p, rows, cols) for k in range(2)])
    for pred in (1, 0):
        check(ctx, oracle, P, cols, pred)


def test_first_one_late_in_plane(ctx, oracle, encoder):
    """EG's extra bit sits after the plane's first 1: put it deep inside the plane"""
    rows, cols = 40, 3000
    P = np.zeros((rows, (cols + 63) // 64), np.uint64)
    P[23, 17] = np.uint64(1 << 40)
    P[30:] = oracle.gen_plane(4, 0.3, 10, cols)
    for pred in (0, 1):
        check(ctx, oracle, P, cols, pred)


def test_fused_vs_multipass(ctx, oracle):
    rows, cols = 200, 3000
    P = np.stack([oracle.gen_plane(77 + k, p, rows, cols) for k, p in enumerate([0.5, 0.1, 0.01])])
    d = ctx.to_dev(P)
    res = {}
    modes = ("staged", "single-kernel", "two-pass", "multipass")
    for mode in modes:
        ctx.set_encoder(mode)
        (og, bg), (oe, be) = ctx.encode_planes2(d, cols, True)
        ctx.sync()
        res[mode] = [(as_u64(bg), [stream_bytes(og[k], as_u64(bg)[k]) for k in range(3)]),
                     (as_u64(be), [stream_bytes(oe[k], as_u64(be)[k]) for k in range(3)])]
    ctx.set_encoder("auto")
    for mode in modes[1:]:
        for c in range(2):
            assert np.array_equal(res["staged"][c][0], res[mode][c][0])
            assert res["staged"][c][1] == res[mode][c][1]


def test_long_lane_and_global_fallback(ctx, oracle, encoder):
    """zero rows drive k up (A grows, n grows by one EOL per row); then a dense word yields a
    lane string > 128 bits, and a dense row yields a row longer than the LDS window."""
    rows, cols = 160, 16384
    wpr = cols // 64
    P = np.zeros((rows, wpr), np.uint64)
    P[100, 7] = ONES                      # one dense word: long lane, row fits LDS
    P[120, :] = ONES                      # a whole dense row at large k: global fallback
    P[121, :] = ALT                       # alternating pixels: dense residual for med
    P[130:, :] = np.stack([oracle.gen_plane(5, 0.5, 30, cols)])[0]
    for pred in (0, 1):
        check(ctx, oracle, P, cols, pred)


def test_many_short_rows_share_words(ctx, oracle, encoder):
    """sparse rows of a few bits each: dozens of rows end inside one output word."""
    rows, cols = 3000, 64
    P = np.zeros((rows, 1), np.uint64)
    P[::97, 0] = np.uint64(1)
    for pred in (0, 1):
        check(ctx, oracle, P, cols, pred)


def test_copy_mode_runs_across_words(ctx, oracle, encoder):
    """p = 0.5 keeps k in {0, 1}; long stretches of k = 0 take the copy path, including runs
    that start in an earlier word."""
    rows, cols = 64, 16384
    P = oracle.gen_plane(99, 0.5, rows, cols)
    P[10, 3:9] = 0                         # a run spanning several words inside a k = 0 stretch
    check(ctx, oracle, P, cols, 0)
    check(ctx, oracle, P, cols, 1)


def test_single_stream_calls_match_dual(ctx, oracle, encoder):
    rows, cols = 33, 2000
    P = oracle.gen_plane(3, 0.2, rows, cols)[None]
    d = ctx.to_dev(P)
    og, bg = ctx.encode_planes(d, cols, True, CODER_GOLOMB)
    oe, be = ctx.encode_planes(d, cols, True, CODER_EG)
    (og2, bg2), (oe2, be2) = ctx.encode_planes2(d, cols, True)
    ctx.sync()
    assert int(as_u64(bg)[0]) == int(as_u64(bg2)[0]) and int(as_u64(be)[0]) == int(as_u64(be2)[0])
    assert stream_bytes(og[0], as_u64(bg)[0]) == stream_bytes(og2[0], as_u64(bg2)[0])
    assert stream_bytes(oe[0], as_u64(be)[0]) == stream_bytes(oe2[0], as_u64(be2)[0])


def test_fused_overflow(ctx, oracle, encoder):
    rows, cols = 64, 1024
    P = oracle.gen_plane(8, 0.5, rows, cols)
    t = ctx.torch
    slot = 100
    buf = t.full((2 * slot + 8,), 0x77, dtype=t.int64, device=ctx.dev)
    ctx.encode_planes(ctx.to_dev(np.stack([P, P])), cols, True, CODER_GOLOMB, slot_words=slot,
                      out=buf[: 2 * slot].view(2, slot))
    with pytest.raises(pybic.BicError) as e:
        ctx.sync()
    assert e.value.code == pybic.BIC_ENOSPC
    assert (as_u64(buf[2 * slot:]) == 0x77).all()
    ctx.sync()


@pytest.mark.parametrize("p", [0.5, 0.35, 0.2])
def test_k_classes_wide_rows(ctx, oracle, encoder, p):
    """hundreds of 16384-column rows: the coder state drifts far enough from the k boundaries that
    the staged encoder proves whole rows k = 0 or k = 1 (closed-form lengths, copy and k = 1 table
    rows) next to the rows that straddle a boundary (walked)."""
    rows, cols = 400, 16384
    P = oracle.gen_plane(4242 + int(100 * p), p, rows, cols)
    for pred in (0, 1):
        check(ctx, oracle, P, cols, pred)


@pytest.mark.parametrize("one_stream", [False, True])
@pytest.mark.parametrize("cols", [16384, 1000, 64])
def test_first_one_row_with_k_flags(ctx, oracle, one_stream, cols):
    """The row holding a plane's first 1 is written by both emission launches (the REST one writes
    its EG row, the main one its Golomb row when every codeword there has k = 1). Row 0's residual
    "001001..." gives codewords of k = 1 only (s = 2 from the fresh k = 1 state keeps k = 1), so
    that row is flagged k = 1 AND holds the first 1, in every plane; the two launches run side by
    side on two streams or one after the other (BIC_OPT_ONE_STREAM), and neither may depend on
    what the other does with the row's length flags."""
    ctx.set_encoder("staged")
    ctx.set_one_stream(one_stream)
    try:
        rows, n = 48, 4
        wpr = (cols + 63) // 64
        R0 = np.zeros(cols, bool)
        R0[2::3] = True
        P0 = np.cumsum(R0) % 2 == 1  # row 0's med residual is P[j] ^ P[j-1]: invert by a prefix xor
        from oracle_lib import pack_rows
        P = np.zeros((n, rows, wpr), np.uint64)
        for k in range(n):
            P[k] = oracle.gen_plane(700 + k, (0.5, 0.3, 0.1, 0.02)[k], rows, cols)
            P[k, 0] = pack_rows(P0[None])[0]
        R = oracle.med(P[0], cols)
        assert np.array_equal(R[0], pack_rows(R0[None])[0])
        check(ctx, oracle, P, cols, 1)
    finally:
        ctx.set_one_stream(False)
        ctx.set_encoder("auto")


def _gray(oracle, seed, rows, cols, kind):
    if kind == "uniform":
        return oracle.gen_bytes(seed, rows * cols).reshape(rows, cols)
    # smooth gradient + small noise: high planes have long runs (k >= 2, walked rows)
    i, j = np.mgrid[0:rows, 0:cols]
    noise = oracle.gen_bytes(seed, rows * cols).reshape(rows, cols) % 7
    return ((i * 3 + j // 5 + noise) % 256).astype(np.uint8)


@pytest.fixture
def staged(ctx):
    """the staged encoder (and bic_encode_gray's fused count pass) at test sizes, which the
    automatic choice would give to the single kernel"""
    ctx.set_encoder("staged")
    yield
    ctx.set_encoder("auto")


@pytest.mark.parametrize("rows,cols,pitch,nplanes,kind", [
    (1, 64, 64, 8, "uniform"), (17, 100, 128, 8, "uniform"), (33, 4096, 4096, 8, "uniform"),
    (40, 5000, 5120, 3, "smooth"), (24, 16384, 16384, 8, "uniform"), (70, 16384, 16384, 8, "smooth"),
    (9, 300, 300, 8, "uniform"),  # pitch < used * 64: the two-call path
    (12, 200, 208, 5, "smooth"),  # pitch < used * 64 (256): the two-call path
])
def test_encode_gray(ctx, oracle, staged, rows, cols, pitch, nplanes, kind):
    """bic_encode_gray == bitplane_tool's planes (oracle) and each plane's Golomb and EG streams"""
    t = ctx.torch
    img = np.zeros((rows, pitch), np.uint8)
    img[:, :cols] = _gray(oracle, rows * 7 + cols, rows, cols, kind)
    img[:, cols:] = 0xA5  # bytes past cols never reach a plane
    g = t.from_numpy(img).to(ctx.dev)
    for pred in (1, 0):
        planes, (og, bg), (oe, be) = ctx.encode_gray(g, cols=cols, nplanes=nplanes, predict=bool(pred))
        ctx.sync()
        exp_planes = oracle.bitplanes(np.ascontiguousarray(img[:, :cols]), nplanes)
        assert np.array_equal(as_u64(planes), exp_planes)
        for k in range(nplanes):
            for coder, out, bits in ((0, og, bg), (1, oe, be)):
                eb, est, _ = oracle.encode_plane(exp_planes[k], cols, pred, coder)
                nb = int(as_u64(bits)[k])
                assert nb == eb, (pred, k, coder)
                assert stream_bytes(out[k], nb) == est.tobytes(), (pred, k, coder)


@pytest.mark.parametrize("off,rows,cols,pitch,kind", [
    (19, 40, 4096, 4096, "uniform"),  # a P5 raster 19 bytes into its file (c3f's layout)
    (3, 33, 16384, 16384, "smooth"), (1, 17, 100, 131, "uniform"), (7, 24, 5000, 5125, "smooth"),
    (8, 9, 64, 72, "uniform"), (13, 70, 16384, 16387, "uniform"),  # pitch % 16 != 0: every row its own offset
])
def test_encode_gray_misaligned(ctx, oracle, staged, off, rows, cols, pitch, kind):
    """bic_encode_gray on gray rows at any byte alignment (the count pass reads the aligned 16-byte
    chunks that hold a lane's 64 pixels and realigns them) == the oracle's planes and streams, with
    and without the planes returned, with and without prediction"""
    t = ctx.torch
    buf = np.full(off + rows * pitch + 64, 0x5A, np.uint8)
    img = np.zeros((rows, pitch), np.uint8)
    img[:, :cols] = _gray(oracle, off * 131 + rows + cols, rows, cols, kind)
    img[:, cols:] = 0xC3  # bytes past cols never reach a plane
    buf[off:off + rows * pitch] = img.reshape(-1)
    d = t.from_numpy(buf).to(ctx.dev)
    g = d[off:off + rows * pitch].view(rows, pitch)
    assert g.data_ptr() % 16 == (d.data_ptr() + off) % 16
    exp_planes = oracle.bitplanes(np.ascontiguousarray(img[:, :cols]), 8)
    for pred, store, p0, n in ((1, True, 0, 8), (1, False, 0, 8), (0, True, 0, 8), (0, False, 0, 8), (1, False, 2, 3)):
        planes, (og, bg), (oe, be) = ctx.encode_gray(g, cols=cols, plane0=p0, nplanes=n, predict=bool(pred),
                                                     store_planes=store)
        ctx.sync()
        if store:
            assert np.array_equal(as_u64(planes), exp_planes[p0:p0 + n])
        for k in range(n):
            for coder, out, bits in ((0, og, bg), (1, oe, be)):
                eb, est, _ = oracle.encode_plane(exp_planes[p0 + k], cols, pred, coder)
                nb = int(as_u64(bits)[k])
                assert nb == eb, (pred, store, p0, k, coder)
                assert stream_bytes(out[k], nb) == est.tobytes(), (pred, store, p0, k, coder)


@pytest.mark.parametrize("rows,cols,pitch,plane0,nplanes,kind", [
    (1, 64, 64, 0, 8, "uniform"), (17, 100, 128, 0, 8, "uniform"), (33, 4096, 4096, 0, 8, "uniform"),
    (40, 5000, 5120, 2, 3, "smooth"), (24, 16384, 16384, 0, 8, "uniform"), (70, 16384, 16384, 1, 6, "smooth"),
    (9, 300, 300, 0, 8, "uniform"),  # pitch < used * 64: the two-call path into the context's buffer
    (60, 4096, 4096, 0, 8, "blank_top"),  # the planes' first residual 1 far below row 0
])
def test_encode_gray_no_planes(ctx, oracle, staged, rows, cols, pitch, plane0, nplanes, kind):
    """bic_encode_gray(_range / _packed) with planes NULL (the count pass keeps the med residual and
    the encoder codes it without prediction) == the oracle's streams of bitplane_tool's planes, and
    the packed form's row index == the oracle's"""
    t = ctx.torch
    img = np.zeros((rows, pitch), np.uint8)
    base = "smooth" if kind == "blank_top" else kind
    img[:, :cols] = _gray(oracle, rows * 5 + cols + plane0, rows, cols, base)
    if kind == "blank_top":
        img[:rows // 2, :cols] = 0x37  # constant rows: residual 0 until row rows / 2 (column 0 aside)
        img[:rows // 2, 0] = 0x37
    g = t.from_numpy(img).to(ctx.dev)
    exp_planes = oracle.bitplanes(np.ascontiguousarray(img[:, :cols]), 8)[plane0:plane0 + nplanes]
    for pred in (1, 0):
        planes, (og, bg), (oe, be) = ctx.encode_gray(g, cols=cols, nplanes=nplanes, predict=bool(pred), plane0=plane0,
                                                      store_planes=False)
        ctx.sync()
        assert planes is None
        for k in range(nplanes):
            for coder, out, bits in ((0, og, bg), (1, oe, be)):
                eb, est, _ = oracle.encode_plane(exp_planes[k], cols, pred, coder)
                nb = int(as_u64(bits)[k])
                assert nb == eb, (pred, k, coder)
                assert stream_bytes(out[k], nb) == est.tobytes(), (pred, k, coder)
    idx = ctx.empty_i64(nplanes * rows * 2)
    _, (og, bg, fg), (oe, be, fe) = ctx.encode_gray_packed(g, cols=cols, nplanes=nplanes, plane0=plane0,
                                                           store_planes=False, row_index=idx)
    ctx.sync()
    for coder, out, off in ((0, og, fg), (1, oe, fe)):
        exp, eoff = _packed_expect(oracle, exp_planes, cols, 1, coder)
        assert list(as_u64(off)) == eoff
        assert as_u64(out)[:eoff[-1]].tobytes() == exp
    ri = as_u64(idx).reshape(nplanes, 2 * rows)
    for k in range(nplanes):
        assert np.array_equal(ri[k], oracle.row_index(exp_planes[k], cols, 1)), k


def test_encode_gray_matches_two_calls(ctx, oracle, staged):
    rows, cols = 300, 16384
    img = _gray(oracle, 5, rows, cols, "uniform")
    g = ctx.torch.from_numpy(img).to(ctx.dev)
    planes, (og, bg), (oe, be) = ctx.encode_gray(g)
    p2 = ctx.bitplanes_u8(g, nplanes=8)
    (og2, bg2), (oe2, be2) = ctx.encode_planes2(p2, cols, True)
    ctx.sync()
    assert np.array_equal(as_u64(planes), as_u64(p2))
    assert np.array_equal(as_u64(bg), as_u64(bg2)) and np.array_equal(as_u64(be), as_u64(be2))
    for k in range(8):
        assert stream_bytes(og[k], as_u64(bg)[k]) == stream_bytes(og2[k], as_u64(bg2)[k])
        assert stream_bytes(oe[k], as_u64(be)[k]) == stream_bytes(oe2[k], as_u64(be2)[k])


@pytest.mark.parametrize("rows,cols,pitch,plane0,nplanes,kind", [
    (40, 4096, 4096, 1, 7, "uniform"), (33, 16384, 16384, 5, 2, "smooth"), (20, 5000, 5120, 7, 1, "smooth"),
    (9, 300, 300, 3, 4, "uniform"),  # the two-call path (bic_bitplanes_u8_range + bic_encode_planes2)
])
def test_encode_gray_range(ctx, oracle, staged, rows, cols, pitch, plane0, nplanes, kind):
    """bic_encode_gray_range (a plane-sharded rank's share): planes plane0.. of the image and their
    streams == the oracle's for bitplane_tool's planes plane0.. (the same planes as a full call)"""
    img = np.zeros((rows, pitch), np.uint8)
    img[:, :cols] = _gray(oracle, rows + plane0, rows, cols, kind)
    g = ctx.torch.from_numpy(img).to(ctx.dev)
    planes, (og, bg), (oe, be) = ctx.encode_gray(g, cols=cols, nplanes=nplanes, plane0=plane0)
    only = ctx.bitplanes_u8(g, cols=cols, nplanes=nplanes, plane0=plane0)
    ctx.sync()
    exp_planes = oracle.bitplanes(np.ascontiguousarray(img[:, :cols]), 8)[plane0:plane0 + nplanes]
    assert np.array_equal(as_u64(planes), exp_planes)
    assert np.array_equal(as_u64(only), exp_planes)
    for k in range(nplanes):
        for coder, out, bits in ((0, og, bg), (1, oe, be)):
            eb, est, _ = oracle.encode_plane(exp_planes[k], cols, 1, coder)
            nb = int(as_u64(bits)[k])
            assert nb == eb, (k, coder)
            assert stream_bytes(out[k], nb) == est.tobytes(), (k, coder)


def test_encode_gray_range_rejects(ctx):
    g = ctx.torch.zeros((4, 64), dtype=ctx.torch.uint8, device=ctx.dev)
    with pytest.raises(pybic.BicError):
        ctx.encode_gray(g, nplanes=4, plane0=5)


def _packed_expect(oracle, P, cols, pred, coder):
    """the packed buffer bic_pack_streams makes of the oracle's streams, and the word offsets"""
    words, offs = [], [0]
    for k in range(P.shape[0]):
        eb, est, _ = oracle.encode_plane(P[k], cols, pred, coder)
        words.append(est.tobytes())
        offs.append(offs[-1] + (eb + 63) // 64)
    return b"".join(words), offs


@pytest.mark.parametrize("encoder_name", ["staged", "single-kernel", "two-pass", "multipass"])
@pytest.mark.parametrize("n,rows,cols,p", [(5, 40, 1000, 0.3), (3, 17, 16384, 0.5), (4, 9, 130, 0.02)])
def test_encode_planes_packed(ctx, oracle, encoder_name, n, rows, cols, p):
    """bic_encode_planes_packed == each plane's oracle stream, word-aligned back to back"""
    P = np.stack([oracle.gen_plane(0x5EED + 31 * k + rows, (p, 0.5, 0.05)[k % 3], rows, cols) for k in range(n)])
    ctx.set_encoder(encoder_name)
    try:
        for pred in (1, 0):
            (og, bg, fg), (oe, be, fe) = ctx.encode_planes_packed(ctx.to_dev(P), cols, pred, golomb=True, eg=True)
            ctx.sync()
            for coder, out, off in ((0, og, fg), (1, oe, fe)):
                exp, eoff = _packed_expect(oracle, P, cols, pred, coder)
                O = as_u64(off)
                assert list(O) == eoff, (pred, coder)
                assert as_u64(out)[:eoff[-1]].tobytes() == exp, (pred, coder)
    finally:
        ctx.set_encoder("auto")


@pytest.mark.parametrize("plane0,nplanes", [(0, 8), (2, 3)])
def test_encode_gray_packed(ctx, oracle, staged, plane0, nplanes):
    rows, cols = 45, 4096
    img = _gray(oracle, 11 + plane0, rows, cols, "smooth")
    g = ctx.torch.from_numpy(img).to(ctx.dev)
    planes, (og, bg, fg), (oe, be, fe) = ctx.encode_gray_packed(g, nplanes=nplanes, plane0=plane0)
    ctx.sync()
    P = oracle.bitplanes(img, 8)[plane0:plane0 + nplanes]
    assert np.array_equal(as_u64(planes), P)
    for coder, out, off in ((0, og, fg), (1, oe, fe)):
        exp, eoff = _packed_expect(oracle, P, cols, 1, coder)
        assert list(as_u64(off)) == eoff
        assert as_u64(out)[:eoff[-1]].tobytes() == exp


@pytest.mark.parametrize("rows", [45, 64, 127])
@pytest.mark.parametrize("cols", [4096, 8192])
def test_encode_gray_blank_plane(ctx, oracle, staged, rows, cols):
    """a plane without a residual 1 among planes that have one: its EG stream is one bit shorter, so
    in the packed buffer the later planes start a word earlier when rows (cols + 1) % 64 == 0 --
    where the count pass's EG words (written at the offsets of planes that hold a 1) must all be
    replaced; rows >= 64 also give rows whose EG offset is word-aligned"""
    img = _gray(oracle, 3 * rows + cols, rows, cols, "uniform")
    img &= 0xEF  # one blank plane
    img[: rows // 3] &= 0x7F  # and the top plane's first 1 a third of the way down
    g = ctx.torch.from_numpy(img).to(ctx.dev)
    P = oracle.bitplanes(img, 8)
    wide = (ctx.slot_words(rows, cols, 0), ctx.slot_words(rows, cols, 1) + 5)  # EG slots longer than a stream
    for pred in (1, 0):
        for store, slots in ((False, (None, None)), (True, (None, None)), (False, wide)):
            _, (og, bg), (oe, be) = ctx.encode_gray(g, predict=bool(pred), store_planes=store, slots=slots)
            ctx.sync()
            for k in range(8):
                for coder, out, bits in ((0, og, bg), (1, oe, be)):
                    eb, est, _ = oracle.encode_plane(P[k], cols, pred, coder)
                    assert int(as_u64(bits)[k]) == eb, (pred, store, k, coder)
                    assert stream_bytes(out[k], eb) == est.tobytes(), (pred, store, k, coder)
    for store in (False, True):
        _, (og, bg, fg), (oe, be, fe) = ctx.encode_gray_packed(g, store_planes=store)
        ctx.sync()
        for coder, out, off in ((0, og, fg), (1, oe, fe)):
            exp, eoff = _packed_expect(oracle, P, cols, 1, coder)
            assert list(as_u64(off)) == eoff, (store, coder)
            assert as_u64(out)[:eoff[-1]].tobytes() == exp, (store, coder)


@pytest.mark.parametrize("rows,cols,wpr", [(37, 4096, 72), (33, 3968, 64), (19, 4000, 63), (50, 256, 4)])
@pytest.mark.parametrize("p", [0.5, 0.05])
def test_narrow_rows_pitched(ctx, oracle, rows, cols, wpr, p):
    """rows of <= 64 words through the staged encoder's four-rows-per-wave count pass: row pitches
    wider than the row (16-byte loads when the pitch and the row are multiples of 4 words, single
    words otherwise), row counts that leave partial 16-row wave blocks and 4-row groups"""
    used = (cols + 63) // 64
    P = np.stack([oracle.gen_plane(0x16 + rows + k, p, rows, cols) for k in range(3)])
    Q = np.zeros((3, rows, wpr), np.uint64)
    Q[:, :, :used] = P
    Q[:, :, used:] = ONES  # pad words past the row must not be read as pixels
    ctx.set_encoder("staged")
    try:
        (og, bg), (oe, be) = ctx.encode_planes2(ctx.to_dev(Q), cols, True)
        ctx.sync()
    finally:
        ctx.set_encoder("auto")
    for k in range(3):
        for coder, out, bits in ((0, og, bg), (1, oe, be)):
            eb, est, _ = oracle.encode_plane(P[k], cols, 1, coder)
            nb = int(as_u64(bits)[k])
            assert nb == eb, (k, coder)
            assert stream_bytes(out[k], nb) == est.tobytes(), (k, coder)


def test_look_back_records_left_zero(ctx, oracle):
    """The single-kernel and two-pass encoders skip zeroing their counters and look-back records when
    the previous call's k_fixup left them zero (bic_capi.cpp scratch_zero): calls of growing and
    shrinking row counts, with other users of the context's scratch (the staged encoder, the
    multi-pass kernels) in between, each checked against the oracle"""
    seq = [("single-kernel", 40, 1000), ("single-kernel", 12, 1000), ("single-kernel", 90, 1000),
           ("two-pass", 90, 1000), ("single-kernel", 90, 1000), ("staged", 60, 4096),
           ("single-kernel", 60, 4096), ("multipass", 30, 2000), ("two-pass", 30, 2000), ("single-kernel", 30, 2000)]
    try:
        for i, (mode, rows, cols) in enumerate(seq):
            ctx.set_encoder(mode)
            P = np.stack([oracle.gen_plane(0xAB + 7 * i + k, (0.5, 0.1)[k], rows, cols) for k in range(2)])
            check(ctx, oracle, P, cols, i & 1)
    finally:
        ctx.set_encoder("auto")


@pytest.mark.parametrize("encoder_name", ["single-kernel", "two-pass"])
def test_capture_replay_between_other_work(ctx, oracle, encoder_name):
    """the single and two-pass encoders skip their record / counter memset when the previous
    call's k_fixup left them zero (host bookkeeping, bic_capi.cpp scratch_zero). A call captured into a
    graph, and replays of it between other calls of the context, are work that bookkeeping never sees: a
    graph captured while the arena was clean must still clear it on every replay. Capture an encode, then
    replay it right after a staged encode (which leaves its counters dirty) and between eager calls;
    every stream must equal the oracle's."""
    torch = ctx.torch
    rows, cols = 64, 2000
    P1 = oracle.gen_plane(41, 0.3, rows, cols)[None]
    P2 = oracle.gen_plane(42, 0.45, 3 * rows, cols)[None]
    d1, d2 = ctx.to_dev(P1), ctx.to_dev(P2)
    slot = ctx.slot_words(rows, cols, CODER_GOLOMB)
    og, bg = ctx.empty_i64(1, slot), ctx.empty_i64(1)
    ctx.reserve(1, 3 * rows, cols)

    def same(out, bits, P):
        eb, est, _ = oracle.encode_plane(P[0], cols, 1, 0)
        nb = int(as_u64(bits)[0])
        return nb == eb and stream_bytes(out[0], nb) == est.tobytes()

    ctx.set_encoder(encoder_name)
    try:
        ctx.encode_planes(d1, cols, True, CODER_GOLOMB, out=og, plane_bits=bg)  # eager: leaves the records zero
        ctx.sync()
        torch.cuda.synchronize()
        assert same(og, bg, P1)
        side = torch.cuda.Stream(ctx.dev)
        side.wait_stream(torch.cuda.current_stream(ctx.dev))
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            with torch.cuda.graph(gr, stream=side):
                ctx.encode_planes(d1, cols, True, CODER_GOLOMB, out=og, plane_bits=bg)
        torch.cuda.current_stream(ctx.dev).wait_stream(side)
        torch.cuda.synchronize()
        for rep in range(3):
            ctx.set_encoder("staged")  # counters left dirty for the replay that follows
            o2, b2 = ctx.encode_planes(d2, cols, True, CODER_GOLOMB)
            ctx.set_encoder(encoder_name)
            og.zero_()
            gr.replay()
            torch.cuda.synchronize()
            assert same(og, bg, P1), rep
            assert same(o2, b2, P2), rep
            o3, b3 = ctx.encode_planes(d2, cols, True, CODER_GOLOMB)  # eager, after a replay
            ctx.sync()
            torch.cuda.synchronize()
            assert same(o3, b3, P2), rep
    finally:
        ctx.set_encoder("auto")
