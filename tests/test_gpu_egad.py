"""a9 as intended: the adaptive EG coder (BIC_CODER_EG_ADAPTIVE: eg.cpp:20-37 with incBlockSize
enabled, JPEG-LS run mode) on the GPU (bic_egad.hip) against the oracle's coder 2, which is pinned to
the reference's own EG state machine (tests/test_oracle_golden.py::test_eg_adaptive_kat). Inputs
reach every part of the row-parallel schedule: dense rows (the state trajectories from 0 and 31
meet), sparse rows (they do not: the resolve walks the row), all-zero planes (the index climbs to its
saturation at 31), the fresh coder's g = 1 on the plane's first run."""
import numpy as np
import pytest

from pybic import CODER_EG_ADAPTIVE, as_u64, stream_bytes

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,cols", [(1, 1), (1, 64), (3, 65), (40, 1000), (17, 4096), (8, 16384), (130, 640),
                                       (5, 20000)])
@pytest.mark.parametrize("pred", [1, 0])
def test_egad_planes(ctx, oracle, rows, cols, pred):
    ps = (0.5, 0.1, 0.01, 0.0, 0.9, 0.001)
    P = np.stack([oracle.gen_plane(0xEAD + 7 * k + rows + cols, ps[k], rows, cols) for k in range(len(ps))])
    out, bits = ctx.encode_planes(ctx.to_dev(P), cols, pred, CODER_EG_ADAPTIVE)
    ctx.sync()
    for k in range(len(ps)):
        eb, est, _ = oracle.encode_plane(P[k], cols, pred, 2)
        nb = int(as_u64(bits)[k])
        assert nb == eb, (k, ps[k])
        assert stream_bytes(out[k], nb) == est.tobytes(), (k, ps[k])


def test_egad_structured(ctx, oracle):
    """a smooth gray image's planes: long runs on the high planes, noise on the low ones"""
    rows, cols = 64, 4096
    i = np.arange(rows)[:, None]
    j = np.arange(cols)[None, :]
    img = ((i * 3 + j // 5 + oracle.gen_bytes(3, rows * cols).reshape(rows, cols) % 7) % 256).astype(np.uint8)
    P = oracle.bitplanes(img, 8)
    out, bits = ctx.encode_planes(ctx.to_dev(P), cols, True, CODER_EG_ADAPTIVE)
    ctx.sync()
    for k in range(8):
        eb, est, _ = oracle.encode_plane(P[k], cols, 1, 2)
        assert int(as_u64(bits)[k]) == eb and stream_bytes(out[k], eb) == est.tobytes(), k
