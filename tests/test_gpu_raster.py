"""f3: PBM / PGM rasters on the device straight out of a file's bytes (bic_raster.hip): P4 rows
(pbm.cpp:29-77) and P5 samples of 1 or 2 bytes (pnm.cpp:54-89) at every misalignment a header can
leave, against the host readers / the oracle's bitplanes, and a whole P5 file -> header on the host
-> planes -> streams chain against the oracle."""
import numpy as np
import pytest

import pybic
from pnm_io import p4_rows_to_plane, plane_to_p4_rows
from pybic import CODER_GOLOMB, as_u64, stream_bytes

pytestmark = pytest.mark.gpu


def _dev_bytes(ctx, b):
    return ctx.torch.from_numpy(np.frombuffer(bytes(b), np.uint8).copy()).to(ctx.dev)


@pytest.mark.parametrize("rows,cols", [(1, 1), (3, 7), (5, 64), (9, 65), (17, 200), (33, 4096), (4, 16383)])
@pytest.mark.parametrize("off", [0, 1, 3, 7, 12])
def test_pbm_unpack_any_offset(ctx, oracle, rows, cols, off):
    P = oracle.gen_plane(rows * 131 + cols + off, 0.4, rows, cols)
    ras = plane_to_p4_rows(P, cols).tobytes()
    buf = _dev_bytes(ctx, b"\xa5" * off + ras)  # the raster after `off` header bytes
    got = ctx.pbm_unpack(buf[off:], rows, cols)
    ctx.sync()
    assert np.array_equal(as_u64(got), p4_rows_to_plane(ras, rows, cols))


@pytest.mark.parametrize("rows,cols", [(3, 7), (9, 65), (8, 128), (5, 4096)])
@pytest.mark.parametrize("off", [0, 5])
def test_pbm_pack(ctx, oracle, rows, cols, off):
    P = oracle.gen_plane(rows + cols, 0.5, rows, cols)
    nb = (cols + 7) // 8
    out = ctx.torch.zeros(off + rows * nb + 8, dtype=ctx.torch.uint8, device=ctx.dev)
    ctx.pbm_pack(ctx.to_dev(P), cols, out=out[off:])
    ctx.sync()
    assert out[off:off + rows * nb].cpu().numpy().tobytes() == plane_to_p4_rows(P, cols).tobytes()


@pytest.mark.parametrize("rows,cols", [(1, 1), (3, 70), (17, 1000), (5, 4096), (3, 16384), (2, 4099)])
@pytest.mark.parametrize("maxval", [255, 100, 1023, 65535])
@pytest.mark.parametrize("off", [0, 1, 6, 15])
def test_pgm_bitplanes(ctx, oracle, rows, cols, maxval, off):
    rng = np.random.default_rng(rows * cols + maxval + off)
    g = rng.integers(0, maxval + 1, (rows, cols)).astype(np.uint16 if maxval > 255 else np.uint8)
    ras = g.astype(">u2").tobytes() if maxval > 255 else g.tobytes()
    buf = _dev_bytes(ctx, b"#" * off + ras)
    nplanes = 16 if maxval > 255 else 8
    got = ctx.pgm_bitplanes(buf[off:], rows, cols, maxval, nplanes)
    part = ctx.pgm_bitplanes(buf[off:], rows, cols, maxval, 3, plane0=nplanes - 4)
    ctx.sync()
    exp = oracle.bitplanes(g, nplanes)
    assert np.array_equal(as_u64(got), exp)
    assert np.array_equal(as_u64(part), exp[nplanes - 4:nplanes - 1])


def test_pgm_rejects(ctx):
    b = ctx.torch.zeros(64, dtype=ctx.torch.uint8, device=ctx.dev)
    with pytest.raises(pybic.BicError):
        ctx.pgm_bitplanes(b, 2, 4, 255, 9)  # 8-bit samples have 8 planes
    with pytest.raises(pybic.BicError):
        ctx.pgm_bitplanes(b, 2, 4, 0, 1)


@pytest.mark.parametrize("rows,cols,maxval,comment", [(40, 1000, 255, None), (21, 4096, 4095, "made by a test"),
                                                       (64, 16384, 255, "x")])
def test_p5_file_to_streams(ctx, oracle, tmp_path, rows, cols, maxval, comment):
    """a P5 file's bytes on the device: header parsed on the host (bic_pnm_parse_header), planes
    from the raster in place (bic_pgm_bitplanes), Golomb streams (bic_encode_planes) == the oracle"""
    from pnm_io import write_pgm
    rng = np.random.default_rng(rows)
    g = rng.integers(0, maxval + 1, (rows, cols)).astype(np.uint16 if maxval > 255 else np.uint8)
    path = write_pgm(str(tmp_path / "in.pgm"), g, maxval, comment=comment)
    data = open(path, "rb").read()
    h = pybic.pnm_header(data[:1024])
    assert (h.type, h.rows, h.cols, h.maxval) == (5, rows, cols, maxval)
    nplanes = oracle.lib.bo_num_planes(maxval)
    dev = _dev_bytes(ctx, data)
    planes = ctx.pgm_bitplanes(dev[h.data_offset:], rows, cols, maxval, nplanes)
    out, bits = ctx.encode_planes(planes, cols, True, CODER_GOLOMB)
    ctx.sync()
    exp = oracle.bitplanes(g, nplanes)
    assert np.array_equal(as_u64(planes), exp)
    for k in range(nplanes):
        eb, est, _ = oracle.encode_plane(exp[k], cols, 1, 0)
        assert int(as_u64(bits)[k]) == eb and stream_bytes(out[k], eb) == est.tobytes(), k


@pytest.mark.parametrize("rows,cols", [(1, 1), (3, 70), (17, 1000), (5, 4096), (3, 16384), (2, 4099)])
@pytest.mark.parametrize("bps,nplanes,plane0", [(1, 8, 0), (1, 3, 2), (2, 16, 0), (2, 10, 0), (2, 5, 9)])
@pytest.mark.parametrize("off", [0, 3])
def test_planes_to_gray(ctx, oracle, rows, cols, bps, nplanes, plane0, off):
    """bic_planes_to_gray (plane2pgm_tool.cpp:33-52) == the oracle's reassembly (bo_planes_to_gray, pinned to
    the reference tool by test_dropin), as 8-bit samples or big-endian 16-bit ones, at any byte offset"""
    rng = np.random.default_rng(rows * cols + 7 * nplanes + off)
    P = np.stack([oracle.gen_plane(int(rng.integers(1 << 30)), (0.5, 0.1, 0.9)[k % 3], rows, cols)
                  for k in range(nplanes)])
    exp = oracle.planes_to_gray(P, cols).astype(np.uint64) << np.uint64(plane0)
    pitch = cols * bps + 5
    buf = ctx.torch.full((off + rows * pitch,), 0xA5, dtype=ctx.torch.uint8, device=ctx.dev)
    ctx.planes_to_gray(ctx.to_dev(P), cols, plane0=plane0, sample_bytes=bps, out=buf[off:], pitch=pitch)
    ctx.sync()
    got = buf[off:].cpu().numpy().reshape(rows, pitch)
    samples = got[:, :cols * bps].copy().view(">u2" if bps == 2 else np.uint8).astype(np.uint64)
    assert np.array_equal(samples, exp)
    assert (got[:, cols * bps:] == 0xA5).all()  # nothing past a row's samples is written
    assert (buf[:off].cpu().numpy() == 0xA5).all()


def test_planes_to_gray_rejects(ctx):
    P = ctx.empty_i64(9, 2, 1)
    with pytest.raises(pybic.BicError):
        ctx.planes_to_gray(P, 64)  # 9 planes do not fit 8-bit samples
    with pytest.raises(pybic.BicError):
        ctx.planes_to_gray(P[:4], 64, plane0=6)


def test_gray_round_trip(ctx, oracle):
    """gray -> bitplanes -> bic_planes_to_gray == gray (8-bit), on the device"""
    rows, cols = 37, 5000
    g = oracle.gen_bytes(0x5EED0077, rows * cols).reshape(rows, cols)
    planes = ctx.bitplanes_u8(ctx.torch.from_numpy(g).to(ctx.dev), nplanes=8)
    back = ctx.planes_to_gray(planes, cols)
    ctx.sync()
    assert np.array_equal(back.cpu().numpy(), g)
