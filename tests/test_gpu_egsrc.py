"""The EG source path of bic_encode_gray without planes (BIC_OPT_EG_SOURCE, the default C3 step):
the count pass writes each plane's EG stream (eg.cpp:20-37 with the block size fixed at 1) in its
uniform layout -- row r at bit r (cols + 1) + 1 -- and the Golomb kernels read the residual rows
back from it; the ONES scan assembles the words across strip edges and one bit per plane is
cleared after the emission (bic_fused.hip eg_src_junctions / eg_fix_bit). Against the oracle and
against the round-3 path (residual planes in a context buffer), at every row-offset phase (rows
>= 64: offsets whose bit is 0 and 63 in their word), 1 to 4 strips per row, the plane's first 1 at
column 0 of a later row, on a strip edge, far down the plane, and planes without a residual 1."""
import numpy as np
import pytest

from pybic import as_u64, stream_bytes  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture
def staged(ctx):
    ctx.set_encoder("staged")
    yield
    ctx.set_encoder("auto")
    ctx.set_eg_source(True)


def _img(oracle, seed, rows, cols, kind):
    u = oracle.gen_bytes(seed, rows * cols).reshape(rows, cols)
    if kind == "uniform":
        return u
    if kind == "smooth":
        i, j = np.mgrid[0:rows, 0:cols]
        return ((i * 3 + j // 5 + u % 7) % 256).astype(np.uint8)
    if kind == "constant":  # no residual 1 in any plane
        return np.full((rows, cols), 0x5C, np.uint8)
    img = u.copy()
    if kind == "first_col0":  # every plane's first 1 at column 0 of row rows // 2
        img[: rows // 2] = 0
        img[rows // 2:, 0] = 0xFF
        img[rows // 2, 1:] = 0xFF
        return img
    if kind == "first_edge":  # first 1 on the second strip's first column
        img[: rows // 3] = 0
        img[rows // 3, :4096] = 0
        return img
    if kind == "sparse":  # high planes blank, low planes rare
        return (u > 250).astype(np.uint8) * (u & 3)
    raise ValueError(kind)


def _check(ctx, oracle, g, img, nplanes, plane0, golomb, eg):
    cols = img.shape[1]
    P = oracle.bitplanes(np.ascontiguousarray(img), 8)[plane0:plane0 + nplanes]
    _, rg, re = ctx.encode_gray(g, cols=cols, nplanes=nplanes, plane0=plane0, store_planes=False, golomb=golomb, eg=eg)
    ctx.sync()
    for k in range(nplanes):
        for coder, res in ((0, rg), (1, re)):
            if res is None:
                continue
            out, bits = res
            eb, est, _ = oracle.encode_plane(P[k], cols, 1, coder)
            assert int(as_u64(bits)[k]) == eb, (k, coder)
            assert stream_bytes(out[k], eb) == est.tobytes(), (k, coder)


@pytest.mark.parametrize("rows,cols,kind", [
    (70, 4096, "uniform"), (130, 4096, "smooth"), (66, 8192, "uniform"), (65, 12288, "smooth"),
    (64, 16384, "uniform"), (33, 16384, "smooth"), (90, 4096, "first_col0"), (40, 8192, "first_edge"),
    (40, 16384, "first_edge"),
    (70, 4096, "constant"), (70, 8192, "sparse"), (1, 4096, "uniform"), (2, 16384, "smooth"),
])
def test_eg_source(ctx, oracle, staged, rows, cols, kind):
    img = _img(oracle, rows * 13 + cols, rows, cols, kind)
    g = ctx.torch.from_numpy(img).to(ctx.dev)
    for golomb, eg in ((True, True), (False, True), (True, False)):
        _check(ctx, oracle, g, img, 8, 0, golomb, eg)
    _check(ctx, oracle, g, img, 3, 4, True, True)


@pytest.mark.parametrize("rows,cols", [(40, 16384), (24, 16384), (40, 12288)])
def test_eg_source_first1_slow_row(ctx, oracle, staged, rows, cols):
    """The row holding a plane's first residual 1 at column j1 > 0 whose Golomb image exceeds the LDS
    window (a dense row after long zero runs: high k), so k_rows_global re-reads it from the EG slot.
    The EG stream's one fixed bit per plane (at that row's layout bit of pixel j1 - 1) must be cleared
    only after that read (it was cleared by k_rows_global's block 0 before its row loop).
    One plane per call, so the first-1 row is the slow list's first entry, the one block 0's wave 0
    takes."""
    img = _img(oracle, rows * 7 + cols, rows, cols, "first_edge")
    g = ctx.torch.from_numpy(img).to(ctx.dev)
    for p in range(8):
        _check(ctx, oracle, g, img, 1, p, True, True)
    _check(ctx, oracle, g, img, 8, 0, True, True)


def test_eg_source_matches_resid_path(ctx, oracle, staged):
    """both paths of planes = NULL give the same streams (every word of every slot compared, so the
    words past each stream's end too)"""
    rows, cols = 200, 8192
    img = _img(oracle, 77, rows, cols, "smooth")
    g = ctx.torch.from_numpy(img).to(ctx.dev)
    res = []
    for on in (True, False):
        ctx.set_eg_source(on)
        _, (og, bg), (oe, be) = ctx.encode_gray(g, store_planes=False)
        ctx.sync()
        res.append((as_u64(og).copy(), as_u64(bg).copy(), as_u64(oe).copy(), as_u64(be).copy()))
    for k in range(8):
        assert np.array_equal(res[0][1], res[1][1]) and np.array_equal(res[0][3], res[1][3])
        nw = (int(res[0][1][k]) + 63) // 64
        assert np.array_equal(res[0][0][k][:nw], res[1][0][k][:nw])
    assert np.array_equal(res[0][2], res[1][2])


_FRESH = r"""
import sys
sys.path.insert(0, {pkg!r}); sys.path.insert(0, {tests!r})
import numpy as np
import pybic
from oracle_lib import Oracle
o = Oracle()
rows, cols = 70, 4096
img = o.gen_bytes(rows * 13 + cols, rows * cols).reshape(rows, cols)
P = o.bitplanes(img, 8)
ctx = pybic.Context(0)
ctx.set_encoder("staged")
g = ctx.torch.from_numpy(img).to(ctx.dev)
_, (og, bg), _ = ctx.encode_gray(g, store_planes=False)  # the process's first encode
ctx.sync()
bad = [k for k in range(8) if pybic.stream_bytes(og[k], o.encode_plane(P[k], cols, 1, 0)[0])
       != o.encode_plane(P[k], cols, 1, 0)[1].tobytes()]
print("BAD", bad)
sys.exit(1 if bad else 0)
"""


_FRESH_C3 = r"""
import sys
sys.path.insert(0, {pkg!r}); sys.path.insert(0, {tests!r})
import numpy as np
import pybic
from oracle_lib import Oracle
o = Oracle()
rows = cols = 16384
ctx = pybic.Context(0)
t = ctx.torch
gen = t.Generator(device=ctx.dev)
gen.manual_seed(0x5EED0000)
g = t.randint(0, 256, (rows, cols), dtype=t.uint8, device=ctx.dev, generator=gen)  # (bench.py's C3 input)
_, (og, bg), (oe, be) = ctx.encode_gray(g, store_planes=False)  # the process's first encode: the bench's C3 call
ctx.sync()
P = o.bitplanes_par(g.cpu().numpy(), 8)
exp = o.encode_planes_par(P, cols, 1)
bad = []
for k in range(8):
    for coder, out, bits in ((0, og, bg), (1, oe, be)):
        eb, est = exp[(k, coder)]
        if int(pybic.as_u64(bits)[k]) != eb or pybic.stream_bytes(out[k], eb) != est.tobytes():
            bad.append((k, coder))
print("BAD", bad)
sys.exit(1 if bad else 0)
"""


def test_first_encode_of_a_process():
    """The first encode of a fresh process: in round 4 (kernels of commit 67ba6e6, device-scope fork /
    join events) class-kernel rows came out wrong in 15 of 16 fresh processes on the pool's boxes
    (DESIGN.md §3). Two fresh processes at 70 x 4096, and one running exactly the bench's default C3 call
    (16384^2 gray, planes not returned) as its first encode, each checked against the oracle."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    kw = dict(pkg=os.path.join(root, "binary-image-compression_amd"), tests=os.path.join(root, "tests"))
    for code in (_FRESH.format(**kw), _FRESH.format(**kw), _FRESH_C3.format(**kw)):
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


def test_images_in_flight(ctx, oracle, staged):
    """bench.py --inflight: two contexts, each on its own HIP stream, encode alternate images with no
    synchronisation between launches (one image's emission overlapping the next one's count pass);
    every image's streams == the oracle's"""
    import pybic
    t = ctx.torch
    rows, cols = 96, 8192
    imgs = [_img(oracle, 900 + i, rows, cols, ("uniform", "smooth", "sparse", "uniform")[i]) for i in range(4)]
    ctxs = [ctx, pybic.Context(ctx.dev.index)]
    ctxs[1].set_encoder("staged")
    streams = [t.cuda.Stream(ctx.dev) for _ in range(2)]
    gs = [t.from_numpy(im).to(ctx.dev) for im in imgs]
    t.cuda.synchronize()
    outs = []
    for rnd in range(3):
        for i, g in enumerate(gs):
            with t.cuda.stream(streams[i & 1]):
                outs.append((i, ctxs[i & 1].encode_gray(g, store_planes=False)))
    t.cuda.synchronize()
    for i, (_, (og, bg), (oe, be)) in outs:
        P = oracle.bitplanes(imgs[i], 8)
        for k in range(8):
            for coder, out, bits in ((0, og, bg), (1, oe, be)):
                eb, est, _ = oracle.encode_plane(P[k], cols, 1, coder)
                assert int(as_u64(bits)[k]) == eb, (i, k, coder)
                assert stream_bytes(out[k], eb) == est.tobytes(), (i, k, coder)
