"""f1: the device decoders (bic_decode_planes; bic_row_index) -- streams back to planes on the GPU,
med inverted on the device. Checked by round trips (GPU encode -> GPU decode == the input planes),
by decoding the oracle's own streams, and by the row index against the oracle's coder states
(GolombDecoder.cpp:15-23 read order; eg.cpp:20-37 as written)."""
import numpy as np
import pytest

import pybic
from pybic import CODER_EG, CODER_GOLOMB, as_u64

pytestmark = pytest.mark.gpu


def _planes(oracle, n, rows, cols, ps, seed=0x5EED):
    return np.stack([oracle.gen_plane(seed + 17 * k + rows + cols, ps[k % len(ps)], rows, cols) for k in range(n)])


def _p00(ctx, P):
    return ctx.torch.tensor([int(P[k, 0, 0] >> np.uint64(63)) for k in range(P.shape[0])], dtype=ctx.torch.uint8,
                            device=ctx.dev)


@pytest.fixture(params=["staged", "auto"])
def enc(request, ctx):
    ctx.set_encoder(request.param)
    yield request.param
    ctx.set_encoder("auto")


@pytest.mark.parametrize("n,rows,cols,ps", [
    (3, 40, 1000, (0.5, 0.2, 0.02)), (2, 17, 16384, (0.5, 0.05)), (4, 1, 64, (0.5, 0.0, 1.0, 0.3)),
    (3, 70, 65, (0.5, 0.01, 0.9)), (2, 33, 4096, (0.0, 0.001)),
])
@pytest.mark.parametrize("pred", [1, 0])
def test_round_trip_packed(ctx, oracle, enc, n, rows, cols, ps, pred):
    """GPU encode (packed, with the row index) -> GPU decode == the planes, both coders"""
    P = _planes(oracle, n, rows, cols, ps)
    d = ctx.to_dev(P)
    idx = ctx.empty_i64(n * rows * 2)
    (og, bg, fg), (oe, be, fe) = ctx.encode_planes_packed(d, cols, pred, golomb=True, eg=True, row_index=idx)
    p00 = _p00(ctx, P) if pred else None
    back_g = ctx.decode_planes(CODER_GOLOMB, og, bg, n, rows, cols, pred, word_off=fg, row_index=idx, p00=p00)
    back_e = ctx.decode_planes(CODER_EG, oe, be, n, rows, cols, pred, word_off=fe, p00=p00)
    ctx.sync()
    ri = as_u64(idx).reshape(n, 2 * rows)
    for k in range(n):
        assert np.array_equal(ri[k], oracle.row_index(P[k], cols, pred)), k
    assert np.array_equal(as_u64(back_g), P)
    assert np.array_equal(as_u64(back_e), P)


@pytest.mark.parametrize("rows,cols", [(50, 300), (20, 16384)])
def test_decode_oracle_streams(ctx, oracle, rows, cols):
    """the oracle's streams in slots, the index from bic_row_index"""
    n = 3
    P = _planes(oracle, n, rows, cols, (0.5, 0.1, 0.02), seed=99)
    for coder in (CODER_GOLOMB, CODER_EG):
        slot = ctx.slot_words(rows, cols, coder)
        S = np.zeros((n, slot), np.uint64)
        bits = np.zeros(n, np.uint64)
        for k in range(n):
            b, st, _ = oracle.encode_plane(P[k], cols, 1, coder)
            S[k, :len(st) // 8] = np.frombuffer(st.tobytes(), np.uint64)  # slot bytes = the bit stream
            bits[k] = b
        idx = ctx.row_index(ctx.to_dev(P), cols, True) if coder == CODER_GOLOMB else None
        back = ctx.decode_planes(coder, ctx.to_dev(S), ctx.to_dev(bits), n, rows, cols, True, row_index=idx,
                                 p00=_p00(ctx, P))
        ctx.sync()
        assert np.array_equal(as_u64(back), P), coder


@pytest.mark.parametrize("coder", [CODER_GOLOMB, CODER_EG])
def test_malformed_stream(ctx, oracle, coder):
    rows, cols = 30, 500
    P = _planes(oracle, 1, rows, cols, (0.3,))
    d = ctx.to_dev(P)
    idx = ctx.empty_i64(rows * 2)
    outs = ctx.encode_planes_packed(d, cols, True, golomb=coder == CODER_GOLOMB, eg=coder == CODER_EG, row_index=idx)
    out, bits, off = outs[0] if coder == CODER_GOLOMB else outs[1]
    ctx.sync()
    bad_bits = bits.clone()
    bad_bits[0] -= 1  # the stream is one bit longer than claimed
    ctx.decode_planes(coder, out, bad_bits, 1, rows, cols, True, word_off=off, row_index=idx)
    with pytest.raises(pybic.BicError) as e:
        ctx.sync()
    assert e.value.code == pybic.BIC_EDATA
    ctx.decode_planes(coder, out, bits, 1, rows, cols, True, word_off=off, row_index=idx)
    ctx.sync()  # the good stream decodes cleanly afterwards


@pytest.mark.parametrize("coder", [CODER_GOLOMB, CODER_EG])
@pytest.mark.parametrize("packed", [True, False])
def test_inflated_length(ctx, oracle, coder, packed):
    """a stated length past the plane's own words (its slot, or its packed words) is BIC_EDATA, and
    nothing past them is read: plane 0's inflated length must not reach into plane 1's stream"""
    rows, cols, n = 30, 500, 2
    P = _planes(oracle, n, rows, cols, (0.3, 0.5))
    d = ctx.to_dev(P)
    idx = ctx.empty_i64(n * rows * 2)
    if packed:
        outs = ctx.encode_planes_packed(d, cols, True, golomb=coder == CODER_GOLOMB, eg=coder == CODER_EG,
                                        row_index=idx)
        out, bits, off = outs[0] if coder == CODER_GOLOMB else outs[1]
        ctx.sync()
        cap = int(as_u64(off)[1] - as_u64(off)[0])
    else:
        out, bits = ctx.encode_planes(d, cols, True, coder)
        off = None
        if coder == CODER_GOLOMB:
            idx = ctx.row_index(d, cols, True)
        ctx.sync()
        cap = out.shape[1]
    bad_bits = bits.clone()
    bad_bits[0] = 64 * cap + 64 * 1000  # far past the plane's capacity
    ctx.decode_planes(coder, out, bad_bits, n, rows, cols, True, word_off=off, row_index=idx)
    with pytest.raises(pybic.BicError) as e:
        ctx.sync()
    assert e.value.code == pybic.BIC_EDATA
    back = ctx.decode_planes(coder, out, bits, n, rows, cols, True, word_off=off, row_index=idx, p00=_p00(ctx, P))
    ctx.sync()
    assert np.array_equal(as_u64(back), P)


def test_decode_rejects(ctx):
    t = ctx.empty_i64(4, 8)
    b = ctx.empty_i64(4)
    with pytest.raises(pybic.BicError):
        ctx.decode_planes(CODER_GOLOMB, t, b, 4, 10, 64, True)  # Golomb without a row index
    with pytest.raises(pybic.BicError):
        ctx.decode_planes(CODER_EG, t, b, 4, 10, 20000, True)  # rows wider than 16384 columns


@pytest.mark.parametrize("n,rows,cols,ps", [
    (3, 40, 1000, (0.5, 0.2, 0.02)), (2, 17, 16384, (0.5, 0.05)), (4, 1, 64, (0.5, 0.0, 1.0, 0.3)),
    (3, 70, 65, (0.5, 0.01, 0.9)), (2, 33, 4096, (0.0, 0.001)), (2, 9, 20000, (0.5, 0.03)),
])
@pytest.mark.parametrize("pred", [1, 0])
def test_round_trip_eg_adaptive(ctx, oracle, n, rows, cols, ps, pred):
    """BIC_CODER_EG_ADAPTIVE: GPU encode -> bic_egad_row_index (== the oracle's coder states at every
    row start) -> GPU decode in eg.cpp:41-55's read order == the planes"""
    P = _planes(oracle, n, rows, cols, ps, seed=0xEAD)
    d = ctx.to_dev(P)
    out, bits = ctx.encode_planes(d, cols, pred, pybic.CODER_EG_ADAPTIVE)
    idx = ctx.egad_row_index(d, cols, pred)
    ctx.sync()
    ri = as_u64(idx).reshape(n, 2 * rows)
    for k in range(n):
        assert np.array_equal(ri[k], oracle.egad_row_index(P[k], cols, pred)), k
    if cols > 16384:
        return  # (the decoders take rows of up to 16384 columns)
    back = ctx.decode_planes(pybic.CODER_EG_ADAPTIVE, out, bits, n, rows, cols, pred, row_index=idx,
                             p00=_p00(ctx, P) if pred else None)
    ctx.sync()
    assert np.array_equal(as_u64(back), P)


def test_malformed_eg_adaptive(ctx, oracle):
    rows, cols = 30, 500
    P = _planes(oracle, 1, rows, cols, (0.3,))
    d = ctx.to_dev(P)
    out, bits = ctx.encode_planes(d, cols, True, pybic.CODER_EG_ADAPTIVE)
    idx = ctx.egad_row_index(d, cols, True)
    ctx.sync()
    bad_bits = bits.clone()
    bad_bits[0] -= 1
    ctx.decode_planes(pybic.CODER_EG_ADAPTIVE, out, bad_bits, 1, rows, cols, True, row_index=idx)
    with pytest.raises(pybic.BicError) as e:
        ctx.sync()
    assert e.value.code == pybic.BIC_EDATA
    back = ctx.decode_planes(pybic.CODER_EG_ADAPTIVE, out, bits, 1, rows, cols, True, row_index=idx, p00=_p00(ctx, P))
    ctx.sync()
    assert np.array_equal(as_u64(back), P)
