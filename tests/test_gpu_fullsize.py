"""Parity at the BASELINE.json configs' own sizes (configs[0..4] = C1..C5), through the C ABI,
against the CPU oracle run on host threads (tests/oracle_lib.py pool_map). Every plane, frame,
tile and stream of each config's workload is compared bit for bit -- the bench itself only
checks one plane.

  C1  512x512 plane, compress_test patch search W = 5 (and compress7's loop, W = 16, R = 128)
  C2  4096x4096 plane, Golomb on the raw plane, the default (auto) encoder
  C3  16384x16384 8-bit gray -> 8 planes -> med -> Golomb + EG (bic_encode_gray), uniform bytes
      and a smooth gradient (long runs, k >= 2, rows whose Golomb codewords mix k); both with the
      staged encoder's emission launches side by side (two streams) and one after the other
  C4  64 frames of 4096x4096 -> med -> Golomb, streams packed (bic_pack_streams)
  C5  8192x8192 plane, 32x32 tiles: weights, modes, residual, L and the Golomb stream
"""
import numpy as np
import pytest

from oracle_lib import pool_map, text_plane
from pybic import CODER_GOLOMB, as_u64, stream_bytes

pytestmark = pytest.mark.gpu


def _gray(oracle, seed, rows, cols, kind):
    if kind == "uniform":
        return oracle.gen_bytes(seed, rows * cols).reshape(rows, cols)
    # smooth gradient + small noise: high planes hold long runs, low planes are near random
    i = np.arange(rows, dtype=np.int64)[:, None]
    j = np.arange(cols, dtype=np.int64)[None, :]
    noise = oracle.gen_bytes(seed, rows * cols).reshape(rows, cols) % 7
    return ((i * 3 + j // 5 + noise) % 256).astype(np.uint8)


def _check_streams(ctx, exp, nplanes, outs):
    """exp: {(plane, coder): (bits, bytes)}; outs: ((out_g, bits_g), (out_e, bits_e))"""
    for coder, (out, bits) in enumerate(outs):
        B = as_u64(bits)
        for k in range(nplanes):
            eb, est = exp[(k, coder)]
            assert int(B[k]) == eb, (k, coder)
            assert stream_bytes(out[k], eb) == est.tobytes(), (k, coder)


@pytest.mark.parametrize("kind", ["uniform", "smooth"])
def test_c3_full(ctx, oracle, kind):
    """configs[2]: 16384^2 gray, all 8 planes, Golomb and EG, predictor on (the bench's call)"""
    rows = cols = 16384
    img = _gray(oracle, 0x5EED0000 + (kind == "smooth"), rows, cols, kind)
    g = ctx.torch.from_numpy(img).to(ctx.dev)
    planes, og, oe = ctx.encode_gray(g, nplanes=8)
    ctx.sync()
    exp_planes = oracle.bitplanes_par(img, 8)
    assert np.array_equal(as_u64(planes), exp_planes)
    exp = oracle.encode_planes_par(exp_planes, cols, 1)
    _check_streams(ctx, exp, 8, (og, oe))
    # the same call with the REST emission launch ordered before the main one on one stream
    ctx.set_one_stream(True)
    try:
        for t in (og[0], og[1], oe[0], oe[1]):
            t.fill_(-1)
        ctx.encode_gray(g, nplanes=8, planes=planes, outs=(og[0], oe[0]), bits=(og[1], oe[1]))
        ctx.sync()
    finally:
        ctx.set_one_stream(False)
    _check_streams(ctx, exp, 8, (og, oe))
    # planes NULL (the bench's default): the count pass keeps the residual, the encoder codes it as is
    for t in (og[0], og[1], oe[0], oe[1]):
        t.fill_(-1)
    none, _, _ = ctx.encode_gray(g, nplanes=8, outs=(og[0], oe[0]), bits=(og[1], oe[1]), store_planes=False)
    ctx.sync()
    assert none is None
    _check_streams(ctx, exp, 8, (og, oe))


@pytest.mark.parametrize("p,pred", [(0.5, 0), (0.05, 0), (0.5, 1)])
def test_c2_full(ctx, oracle, p, pred):
    """configs[1]: one 4096^2 plane, Golomb, the default encoder choice for that batch"""
    rows = cols = 4096
    P = oracle.gen_plane(0x5EED0000 + int(p * 100), p, rows, cols)
    out, bits = ctx.encode_planes(ctx.to_dev(P[None]), cols, pred, CODER_GOLOMB)
    ctx.sync()
    eb, est, _ = oracle.encode_plane(P, cols, pred, 0)
    assert int(as_u64(bits)[0]) == eb
    assert stream_bytes(out[0], eb) == est.tobytes()


def test_c4_full(ctx, oracle):
    """configs[3]: 64 frames of 4096^2 (one rank's share at N = 1), med + Golomb, then the packed
    buffer the gather sends: every frame's stream at its word offset"""
    n, rows, cols = 64, 4096, 4096
    P = np.stack(pool_map(lambda k: oracle.gen_plane(0x5EED0000 + k, (0.5, 0.2, 0.05, 0.01)[k % 4], rows, cols),
                          list(range(n))))
    out, bits = ctx.encode_planes(ctx.to_dev(P), cols, True, CODER_GOLOMB)
    dst, off = ctx.pack_streams(out, bits)
    ctx.sync()
    exp = oracle.encode_planes_par(P, cols, 1, coders=(0,))
    B, O, D = as_u64(bits), as_u64(off), as_u64(dst)
    assert O[0] == 0
    for k in range(n):
        eb, est = exp[(k, 0)]
        assert int(B[k]) == eb, k
        nw = (eb + 63) // 64
        assert O[k + 1] - O[k] == nw, k
        assert stream_bytes(out[k], eb) == est.tobytes(), k
        assert D[O[k]:O[k] + nw].tobytes() == est.tobytes(), k


@pytest.mark.parametrize("p", [0.5, 0.03])
def test_c5_full(ctx, oracle, p):
    """configs[4]: 8192^2, 32x32 tiles (compress7 with R = 0), adaptive Golomb over the tiles"""
    rows = cols = 8192
    W = 32
    I = oracle.gen_plane(0x5EED0000 + int(p * 100), p, rows, cols)
    lt = oracle.lentab(W)
    exp = oracle.patch_encode(I, cols, W, lt)
    res = ctx.patch_encode(ctx.to_dev(I), cols, W, lt)
    ctx.sync()
    st = as_u64(res["stats"])
    assert int(st[0]) == exp["bits"] and int(st[2]) == exp["L"]
    assert stream_bytes(res["stream"], exp["bits"]) == exp["stream"].tobytes()
    assert bytes(res["modes"].cpu().numpy()).decode() == exp["modes"]
    assert np.array_equal(res["w_nonpred"].cpu().numpy().view(np.uint32), exp["w_nonpred"])
    assert np.array_equal(res["w_pred"].cpu().numpy().view(np.uint32), exp["w_pred"])
    assert np.array_equal(as_u64(res["resid"]), exp["residual"])


def test_c1_search_full(ctx, oracle):
    """configs[0]: compress_test's patch search over the whole 512^2 plane, W = 5 (512 is not a
    multiple of 5: the last tile column wraps into the next row)"""
    rows = cols = 512
    W = 5
    I = oracle.gen_plane(0x5EED0000, 0.5, rows, cols)
    exp = oracle.patch_search_par(I, cols, W)
    got = ctx.patch_search(ctx.to_dev(I), cols, W)
    ctx.sync()
    for name, e, g in zip(("besti", "bestj", "bestd"), exp, got):
        assert np.array_equal(g.cpu().numpy().view(np.uint32), e), name


def test_c1_match_loop_full(ctx, oracle):
    """compress7_test's whole tile loop on a 512^2 text-like page, W = 16, T = 0, R = 128"""
    rows = cols = 512
    W, T, R = 16, 0, 128
    I = text_plane(0x5EED, rows, cols)
    exp = oracle.match_encode(I, cols, W, T, R)
    res = ctx.match_encode(ctx.to_dev(I), cols, W, T, R)
    ctx.sync()
    st = [int(x) for x in as_u64(res["stats"])]
    assert st == [exp["matches"], exp["bits_match"], exp["bits_nomatch"], exp["L"]]
    assert np.array_equal(as_u64(res["resid"]), exp["residual"])
    assert bytes(res["modes"].cpu().numpy()).decode() == exp["modes"]
    assert stream_bytes(res["stream_match"], exp["bits_match"]) == exp["stream_match"].tobytes()
    assert stream_bytes(res["stream_nomatch"], exp["bits_nomatch"]) == exp["stream_nomatch"].tobytes()


def test_c3_full_round_trip(ctx, oracle):
    """§8 f1 at configs[2]'s size: the 8 planes of a 16384^2 gray image -> Golomb and EG streams
    (packed, with the row index) -> decoded on the device (med inverted there) == the planes ->
    reassembled on the device (bic_planes_to_gray) == the gray image"""
    rows = cols = 16384
    img = _gray(oracle, 0x5EED0002, rows, cols, "smooth")
    g = ctx.torch.from_numpy(img).to(ctx.dev)
    idx = ctx.empty_i64(8 * rows * 2)
    planes, (og, bg, fg), (oe, be, fe) = ctx.encode_gray_packed(g, nplanes=8, row_index=idx)
    p00 = ctx.torch.from_numpy(((img[0, 0] >> np.arange(8)) & 1).astype(np.uint8)).to(ctx.dev)
    back = ctx.decode_planes(0, og, bg, 8, rows, cols, True, word_off=fg, row_index=idx, p00=p00)
    ctx.sync()
    assert ctx.torch.equal(back, planes)
    back = ctx.decode_planes(1, oe, be, 8, rows, cols, True, word_off=fe, p00=p00, out=back)
    ctx.sync()
    assert ctx.torch.equal(back, planes)
    exp_planes = oracle.bitplanes_par(img, 8)
    assert np.array_equal(as_u64(planes), exp_planes)
    # ... and the last leg (plane2pgm_tool.cpp:33-52 on the device): the decoded planes -> the gray image
    gray_back = ctx.planes_to_gray(back, cols)
    ctx.sync()
    assert ctx.torch.equal(gray_back, g)


@pytest.mark.parametrize("p", [0.5, 0.05])
def test_c2_full_eg_adaptive(ctx, oracle, p):
    """configs[1]'s 4096^2 plane through the adaptive EG coder (BIC_CODER_EG_ADAPTIVE), med on"""
    rows = cols = 4096
    P = oracle.gen_plane(0x5EED00E0 + int(p * 100), p, rows, cols)
    out, bits = ctx.encode_planes(ctx.to_dev(P[None]), cols, True, 2)
    ctx.sync()
    eb, est, _ = oracle.encode_plane(P, cols, 1, 2)
    assert int(as_u64(bits)[0]) == eb
    assert stream_bytes(out[0], eb) == est.tobytes()


def test_c3_full_eg_adaptive_round_trip(ctx, oracle):
    """the adaptive EG coder at configs[2]'s size: the 8 planes of a 16384^2 gray image -> adaptive EG
    streams -> the row index (coder state per row) -> decoded on the device == the planes; one plane's
    stream and index against the oracle"""
    import pybic
    rows = cols = 16384
    img = _gray(oracle, 0x5EED0006, rows, cols, "smooth")
    g = ctx.torch.from_numpy(img).to(ctx.dev)
    planes = ctx.bitplanes_u8(g, nplanes=8)
    out, bits = ctx.encode_planes(planes, cols, True, pybic.CODER_EG_ADAPTIVE)
    idx = ctx.egad_row_index(planes, cols, True)
    p00 = ctx.torch.from_numpy(((img[0, 0] >> np.arange(8)) & 1).astype(np.uint8)).to(ctx.dev)
    back = ctx.decode_planes(pybic.CODER_EG_ADAPTIVE, out, bits, 8, rows, cols, True, row_index=idx, p00=p00)
    ctx.sync()
    assert ctx.torch.equal(back, planes)
    P6 = pybic.as_u64(planes[6])
    eb, est, _ = oracle.encode_plane(P6, cols, 1, 2)
    assert int(as_u64(bits)[6]) == eb and stream_bytes(out[6], eb) == est.tobytes()
    assert np.array_equal(as_u64(idx).reshape(8, 2 * rows)[6], oracle.egad_row_index(P6, cols, 1))


def test_c3_p5_file_full(ctx, oracle):
    """configs[2] from a P5 file's bytes on the device: header parsed on the host, the planes of the
    raster in place (it starts 19 bytes into the file), both streams of every plane"""
    import pybic
    rows = cols = 16384
    img = _gray(oracle, 0x5EED0004, rows, cols, "uniform")
    hdr = f"P5\n{cols} {rows}\n255\n".encode()
    data = np.frombuffer(hdr + img.tobytes(), np.uint8)
    h = pybic.pnm_header(data[:64].tobytes())
    dev = ctx.torch.from_numpy(data.copy()).to(ctx.dev)
    planes = ctx.pgm_bitplanes(dev[h.data_offset:], h.rows, h.cols, h.maxval, 8)
    (og, bg), (oe, be) = ctx.encode_planes2(planes, cols, True)
    ctx.sync()
    exp_planes = oracle.bitplanes_par(img, 8)
    assert np.array_equal(as_u64(planes), exp_planes)
    exp = oracle.encode_planes_par(exp_planes, cols, 1)
    _check_streams(ctx, exp, 8, ((og, bg), (oe, be)))
    # the bench's c3f step: ONE bic_encode_gray call on the raster where it lies (misaligned count pass)
    raster = dev[h.data_offset:h.data_offset + rows * cols].view(rows, cols)
    assert raster.data_ptr() % 16 == 3
    _, (og2, bg2), (oe2, be2) = ctx.encode_gray(raster, cols=cols, nplanes=8, store_planes=False)
    ctx.sync()
    _check_streams(ctx, exp, 8, ((og2, bg2), (oe2, be2)))
