"""HIP path (libbic.so, through the C ABI) against the CPU oracle and the golden vectors
produced by the reference's own objects. Bit-exact everywhere (integer/bit work)."""
import ctypes as C

import numpy as np
import pytest

import pybic
from pybic import CODER_EG, CODER_GOLOMB, as_u64, stream_bytes

pytestmark = pytest.mark.gpu

SHAPES = [(1, 1), (1, 64), (1, 65), (2, 1), (3, 130), (37, 70), (64, 64), (100, 4096), (33, 8192),
          (17, 16384), (6, 20000), (5, 40000)]


def planes_of(oracle, n, rows, cols, p, seed, wpr=None):
    return np.stack([oracle.gen_plane(seed + k, p, rows, cols, wpr) for k in range(n)])


def mask_pixels(words, cols):
    """zero the pad bits/words past `cols` (they are unspecified on input)."""
    w = np.array(words, copy=True)
    used = (cols + 63) // 64
    w[..., used:] = 0
    if cols % 64:
        w[..., used - 1] &= np.uint64(((1 << 64) - 1) ^ ((1 << (64 - cols % 64)) - 1))
    return w


# ------------------------------------------------------------------------------------------
def test_bitplanes_u8(ctx, oracle):
    t = ctx.torch
    for (rows, cols, pitch) in [(1, 1, 1), (3, 70, 70), (40, 48, 48), (17, 1000, 1024), (64, 4096, 4096),
                                (5, 16384, 16384), (9, 129, 133)]:
        gray = oracle.gen_bytes(77 + rows, rows * pitch).reshape(rows, pitch)
        exp = oracle.bitplanes(np.ascontiguousarray(gray[:, :cols]), 8)
        g = t.from_numpy(gray).to(ctx.dev)
        for n in (8, 3):
            got = as_u64(ctx.bitplanes_u8(g, cols=cols, nplanes=n))
            ctx.sync()
            assert np.array_equal(got, exp[:n]), (rows, cols, pitch, n)


def test_bitplanes_golden_pgm(ctx, golden):
    """the reference's own bitplane_tool output (tests/golden) for an 8-bit PGM"""
    from pnm_io import read_pbm_bytes
    meta, A = golden
    import os
    data = open(os.path.join(os.path.dirname(__file__), "golden", "gray_48x40.pgm"), "rb").read()
    gray = np.frombuffer(data[-48 * 40:], np.uint8).reshape(40, 48)
    got = as_u64(ctx.bitplanes_u8(ctx.torch.from_numpy(gray.copy()).to(ctx.dev), nplanes=8))
    ctx.sync()
    for b in range(8):
        _, _, ref = read_pbm_bytes(A[f"bt_gray_48x40.pgm_{b}"].tobytes())
        assert np.array_equal(got[b], ref), b


@pytest.mark.parametrize("rows,cols", SHAPES)
def test_med_residual_and_weight(ctx, oracle, rows, cols):
    for p in (0.5, 0.05):
        P = planes_of(oracle, 2, rows, cols, p, 10 * rows + cols)
        resid, w = ctx.med_residual(ctx.to_dev(P), cols, predict=True)
        rawr, w0 = ctx.med_residual(ctx.to_dev(P), cols, predict=False)
        ctx.sync()
        R = as_u64(resid)
        for k in range(2):
            exp = oracle.med(P[k], cols)
            assert np.array_equal(R[k], exp), (rows, cols, p, k)
            assert int(as_u64(w)[k]) == oracle.weight(exp, cols)
            assert int(as_u64(w0)[k]) == oracle.weight(P[k], cols)
            assert np.array_equal(as_u64(rawr)[k], mask_pixels(P[k], cols))


def test_med_golden(ctx, golden):
    meta, A = golden
    for c in meta["planes"]:
        P = A[c["key"]]
        resid, w = ctx.med_residual(ctx.to_dev(P[None]), c["cols"])
        ctx.sync()
        assert np.array_equal(as_u64(resid)[0], A[c["key"] + "_med"]), c["key"]
        assert int(as_u64(w)[0]) == c["weight_med"]


def test_pad_words_and_garbage_pad_bits(ctx, oracle):
    rows, cols, wpr = 20, 100, 5  # 2 used words + 3 pad words per row
    P = oracle.gen_plane(5, 0.4, rows, cols, wpr)
    dirty = P.copy()
    dirty[:, 1] |= np.uint64((1 << (64 - 36)) - 1)  # garbage in the pad bits of word 1
    dirty[:, 2:] = np.uint64(0xDEADBEEFDEADBEEF)  # garbage pad words
    for coder in (CODER_GOLOMB, CODER_EG):
        out, bits = ctx.encode_planes(ctx.to_dev(dirty[None]), cols, True, coder)
        ctx.sync()
        eb, est, _ = oracle.encode_plane(P[:, :2].copy(), cols, 1, coder)
        assert int(as_u64(bits)[0]) == eb
        assert stream_bytes(out[0], eb) == est.tobytes()


# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("rows,cols", SHAPES)
@pytest.mark.parametrize("coder", [CODER_GOLOMB, CODER_EG])
def test_encode_planes(ctx, oracle, rows, cols, coder):
    ps = [0.5, 0.02] if rows * cols > 100000 else [0.5, 0.1, 0.0, 1.0]
    for p in ps:
        n = 3
        P = planes_of(oracle, n, rows, cols, p, 7 * rows + cols + int(100 * p))
        for pred in (1, 0):
            out, bits = ctx.encode_planes(ctx.to_dev(P), cols, pred, coder)
            ctx.sync()
            B = as_u64(bits)
            for k in range(n):
                eb, est, _ = oracle.encode_plane(P[k], cols, pred, coder)
                assert int(B[k]) == eb, (rows, cols, p, pred, k)
                assert stream_bytes(out[k], eb) == est.tobytes(), (rows, cols, p, pred, k)


def test_encode_golden_bitcounts(ctx, golden):
    meta, A = golden
    for c in meta["planes"]:
        P = A[c["key"]][None]
        for pred in (0, 1):
            for coder, key in ((CODER_GOLOMB, "golomb"), (CODER_EG, "eg")):
                _, bits = ctx.encode_planes(ctx.to_dev(P), c["cols"], pred, coder)
                ctx.sync()
                assert int(as_u64(bits)[0]) == c[f"{key}_bits_pred{pred}"], (c["key"], pred, key)


def test_structured_long_runs(ctx, oracle):
    """sparse rows with runs longer than a chunk's LDS window (global-emitter path) and
    rows split over several chunks"""
    rows, cols = 12, 70000
    P = np.zeros((rows, (cols + 63) // 64), np.uint64)
    P[3, 500] = np.uint64(1)
    P[7, -1] = np.uint64(1 << 16)  # near the right edge
    P[9, 0] = np.uint64(0x8000000000000000)
    for pred in (0, 1):
        out, bits = ctx.encode_planes(ctx.to_dev(P[None]), cols, pred, CODER_GOLOMB)
        ctx.sync()
        eb, est, _ = oracle.encode_plane(P, cols, pred, 0)
        assert int(as_u64(bits)[0]) == eb
        assert stream_bytes(out[0], eb) == est.tobytes()


def test_decode_roundtrip_gpu_stream(ctx, oracle):
    rows, cols = 64, 1000
    P = oracle.gen_plane(4242, 0.3, rows, cols)
    out, bits = ctx.encode_planes(ctx.to_dev(P[None]), cols, True, CODER_GOLOMB)
    ctx.sync()
    nb = int(as_u64(bits)[0])
    st = np.frombuffer(stream_bytes(out[0], nb), np.uint8)
    rc, Q = oracle.decode_plane_golomb(st, nb, rows, cols, 1, corner=int(P[0, 0] >> np.uint64(63)))
    assert rc == 0 and np.array_equal(Q, P)


def test_overflow_reports_enospc(ctx, oracle):
    rows, cols = 64, 256
    P = oracle.gen_plane(9, 0.5, rows, cols)
    slot = 40  # far too small (a plane needs ~260 words)
    t = ctx.torch
    small = t.full((3 * slot + 8,), 0x5A5A, dtype=t.int64, device=ctx.dev)
    _, bits = ctx.encode_planes(ctx.to_dev(np.stack([P, P, P])), cols, True, CODER_GOLOMB, slot_words=slot,
                                out=small[: 3 * slot].view(3, slot))
    with pytest.raises(pybic.BicError) as e:
        ctx.sync()
    assert e.value.code == pybic.BIC_ENOSPC
    assert (as_u64(small[3 * slot:]) == 0x5A5A).all()  # nothing written past the slots
    ctx.sync()  # flag cleared


def test_invalid_args(ctx):
    t = ctx.torch
    P = t.zeros((1, 4, 1), dtype=t.int64, device=ctx.dev)
    with pytest.raises(pybic.BicError) as e:
        ctx.encode_planes(P, 0, True, CODER_GOLOMB)  # cols = 0
    assert e.value.code == pybic.BIC_EINVAL
    with pytest.raises(pybic.BicError):
        ctx.encode_planes(P, 65, True, CODER_GOLOMB)  # wpr too small for cols
    with pytest.raises(pybic.BicError):
        ctx.encode_planes(P, 64, True, 7)  # unknown coder


def test_empty_rows(ctx):
    t = ctx.torch
    P = t.zeros((2, 0, 1), dtype=t.int64, device=ctx.dev)
    out, bits = ctx.encode_planes(P, 64, True, CODER_GOLOMB, slot_words=4)
    ctx.sync()
    assert (as_u64(bits) == 0).all()


# ------------------------------------------------------------------------------------------
def test_golomb_samples_kat(ctx, golden):
    meta, A = golden
    for name, bits in meta["golomb"].items():
        s = A[f"golomb_{name}_s"]
        out, b = ctx.golomb_encode_samples(ctx.to_dev(s))
        ctx.sync()
        assert int(as_u64(b)[0]) == bits, name
        assert int(as_u64(b)[1]) == int(s.astype(np.uint64).sum())


def test_golomb_samples_stream_and_shards(ctx, oracle):
    rng = np.random.default_rng(3)
    s = (rng.geometric(0.05, 20000) - 1).astype(np.uint32)
    eb, est, _, ln = oracle.golomb_samples(s)
    out, b = ctx.golomb_encode_samples(ctx.to_dev(s))
    ctx.sync()
    assert int(as_u64(b)[0]) == eb
    assert stream_bytes(out, eb) == est.tobytes()
    # continue from a coder state and a bit offset (the multi-GPU shard path)
    cut = 7777
    n0, a0 = cut, int(s[:cut].astype(np.uint64).sum())
    bit0 = int(ln[:cut].astype(np.uint64).sum())
    out2, b2 = ctx.golomb_encode_samples(ctx.to_dev(s[cut:]), n0=n0, a0=a0, bit0=bit0 % 64)
    ctx.sync()
    tail = int(as_u64(b2)[0])
    assert bit0 + tail == eb
    # the shard's words, OR'd into the prefix's stream at word bit0//64, rebuild the whole
    whole = np.frombuffer(est.tobytes(), ">u8").astype(np.uint64)
    mine = as_u64(out2)[: (bit0 % 64 + tail + 63) // 64].byteswap()
    pre = whole.copy()
    w0 = bit0 // 64
    keep = np.uint64(((1 << 64) - 1) ^ ((1 << (64 - bit0 % 64)) - 1)) if bit0 % 64 else np.uint64(0)
    pre[w0] &= keep
    pre[w0 + 1:] = 0
    pre[w0:w0 + len(mine)] |= mine
    assert np.array_equal(pre, whole)
    # the lengths-only call (no output) gives the same counts from the same coder state
    b3 = ctx.golomb_lengths(ctx.to_dev(s[cut:]), n0=n0, a0=a0)
    ctx.sync()
    assert [int(x) for x in as_u64(b3)] == [int(x) for x in as_u64(b2)]
    with pytest.raises(pybic.BicError):
        ctx._chk(ctx.lib.bic_golomb_encode_samples(ctx.h, C.c_void_p(s.ctypes.data), 4, 0, 0, 0, None, 5,
                                                   C.c_void_p(b3.data_ptr())), "no output with a capacity")


# ------------------------------------------------------------------------------------------
def test_tiles_golden(ctx, golden):
    meta, A = golden
    for c in meta["tiles"]:
        k, W, rows, cols = c["key"], c["W"], c["rows"], c["cols"]
        if rows % W or cols % W:
            continue  # the edge-wrap case is CPU-only
        res = ctx.patch_encode(ctx.to_dev(A[k + "_in"]), cols, W, A[k + "_lentab"])
        ctx.sync()
        stats = as_u64(res["stats"])
        assert int(stats[0]) == c["bits"], k
        assert int(stats[2]) == c["L"], k
        assert bytes(res["modes"].cpu().numpy()).decode() == c["modes"], k
        assert np.array_equal(res["w_nonpred"].cpu().numpy().view(np.uint32), A[k + "_w_nonpred"])
        assert np.array_equal(res["w_pred"].cpu().numpy().view(np.uint32), A[k + "_w_pred"])
        assert np.array_equal(as_u64(res["resid"]), mask_pixels(A[k + "_resid"], cols)), k


@pytest.mark.parametrize("W,rows,cols,p,wpr", [(32, 1024, 1024, 0.5, None), (32, 512, 2048, 0.02, None),
                                               (8, 256, 512, 0.1, None), (5, 100, 200, 0.3, None),
                                               (64, 256, 320, 0.01, None), (16, 96, 208, 0.4, None),
                                               (8, 64, 72, 0.5, None), (32, 64, 96, 0.3, 4), (16, 48, 4160, 0.2, None),
                                               (32, 512, 4096, 0.5, None), (8, 64, 4096, 0.3, None),
                                               (16, 96, 8192, 0.05, None), (64, 128, 4096, 0.5, None),
                                               (32, 2048, 8192, 0.02, None)])
def test_tiles_stream(ctx, oracle, W, rows, cols, p, wpr):
    """aligned tiles (W in 8..64, one word holds 64/W tiles) and the generic path (W = 5); partial
    last words, rows with words past the pixels (wpr > ceil(cols/64)); rows of whole 64-word groups
    (cols % 4096 == 0) take the tile kernel that also scans the sample coder"""
    I = oracle.gen_plane(31 + W, p, rows, cols, wpr=wpr)
    lt = oracle.lentab(W)
    exp = oracle.patch_encode(I, cols, W, lt)
    res = ctx.patch_encode(ctx.to_dev(I), cols, W, lt)
    ctx.sync()
    stats = as_u64(res["stats"])
    assert int(stats[0]) == exp["bits"]
    assert int(stats[2]) == exp["L"]
    assert stream_bytes(res["stream"], exp["bits"]) == exp["stream"].tobytes()
    assert np.array_equal(as_u64(res["resid"]), mask_pixels(exp["residual"], cols))
    for key in ("w_nonpred", "w_pred", "weights"):
        if key in exp:
            assert np.array_equal(res[key].cpu().numpy().view(np.uint32), np.asarray(exp[key], np.uint32)), key
    if "modes" in exp:
        assert bytes(res["modes"].cpu().numpy()).decode() == exp["modes"], "modes"


def test_tiles_stream_reused_buffers(ctx, oracle):
    """patch_encode(bufs=...) writes the same buffers again: a second plane through the first call's
    buffers (stream words of the first, longer stream left behind) == the oracle's"""
    W, rows, cols = 32, 512, 1024
    lt = oracle.lentab(W)
    I1 = oracle.gen_plane(7, 0.5, rows, cols)
    I2 = oracle.gen_plane(8, 0.05, rows, cols)
    res = ctx.patch_encode(ctx.to_dev(I1), cols, W, lt)
    res2 = ctx.patch_encode(ctx.to_dev(I2), cols, W, lt, bufs=res)
    ctx.sync()
    assert res2["stream"].data_ptr() == res["stream"].data_ptr()
    exp = oracle.patch_encode(I2, cols, W, lt)
    assert int(as_u64(res2["stats"])[0]) == exp["bits"]
    assert stream_bytes(res2["stream"], exp["bits"]) == exp["stream"].tobytes()
    assert np.array_equal(as_u64(res2["resid"]), mask_pixels(exp["residual"], cols))


def test_pack_streams(ctx, oracle):
    rows, cols = 50, 700
    P = planes_of(oracle, 4, rows, cols, 0.2, 600)
    out, bits = ctx.encode_planes(ctx.to_dev(P), cols, True, CODER_GOLOMB)
    dst, off = ctx.pack_streams(out, bits)
    ctx.sync()
    O = as_u64(off)
    D = as_u64(dst)
    for k in range(4):
        eb, est, _ = oracle.encode_plane(P[k], cols, 1, 0)
        nw = (eb + 63) // 64
        assert O[k + 1] - O[k] == nw
        assert D[O[k]:O[k] + nw].tobytes() == est.tobytes()


@pytest.mark.parametrize("rows,cols", [(1, 1), (3, 7), (5, 64), (9, 65), (37, 70), (20, 1000), (4, 16384)])
def test_pbm_raster_pack_unpack(ctx, oracle, rows, cols):
    """device P4 rasters (pbm.cpp:29-77) against the host writer, both directions"""
    from pnm_io import plane_to_p4_rows
    P = oracle.gen_plane(rows * 7 + cols, 0.4, rows, cols)
    raster = plane_to_p4_rows(P, cols)
    d = ctx.torch.from_numpy(raster.reshape(-1).copy()).to(ctx.dev)
    back = ctx.pbm_unpack(d, rows, cols)
    ras2 = ctx.pbm_pack(ctx.to_dev(P), cols)
    ctx.sync()
    assert np.array_equal(as_u64(back), mask_pixels(P, cols))
    assert ras2.cpu().numpy().tobytes() == raster.tobytes()


@pytest.mark.parametrize("W,rows,cols,p", [(5, 37, 70, 0.3), (3, 20, 33, 0.5), (8, 40, 128, 0.1), (5, 26, 64, 0.02),
                                           (4, 16, 50, 0.0), (32, 96, 200, 0.2), (5, 120, 300, 0.05),
                                           (1, 9, 40, 0.5), (2, 17, 65, 0.3), (6, 31, 100, 0.4), (7, 50, 90, 0.1),
                                           (9, 45, 130, 0.2)])
def test_patch_search(ctx, oracle, W, rows, cols, p):
    """compress_test.cpp's search (tiles past the edges wrap into the next row; sparse images give
    perfect matches; p = 0 gives ties everywhere)"""
    I = oracle.gen_plane(3000 + W + rows, p, rows, cols)
    exp = oracle.patch_search(I, cols, W)
    got = ctx.patch_search(ctx.to_dev(I), cols, W)
    ctx.sync()
    for name, e, g in zip(("besti", "bestj", "bestd"), exp, got):
        assert np.array_equal(g.cpu().numpy().view(np.uint32), e), name
