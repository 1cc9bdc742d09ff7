"""f4: the binary_matrix algebra over GF(2) on the device (bic_gf2.hip, include/bic.h bic_gf2_mul /
bic_gf2_transpose) against the oracle's restatement of mul_AB / mul_AtB / mul_ABt / mul_AtBt and
transpose_to (binmat.cpp:199-214, 516-616; the oracle is pinned to the reference's own objects by
tests/golden/gf2.npz). Bit-exact, padding bits included: ragged shapes, K = 1 and K on word
boundaries, operands with nonzero padding bits, mul_ABt's as-written j < B.cols (B.cols above and
below B.rows), pitched rows, and a 4096-class product."""
import numpy as np
import pytest

import pybic
from pybic import GF2_AB, GF2_ABT, GF2_ATB, GF2_ATBT, as_u64

pytestmark = pytest.mark.gpu


def c_shape(op, ar, ac, br, bc):
    return {GF2_AB: (ar, bc), GF2_ATB: (ac, bc), GF2_ABT: (ar, br), GF2_ATBT: (ac, br)}[op]


def shapes(op, m, k, n):
    """(a_rows, a_cols, b_rows, b_cols) for C = m x n with inner dimension k"""
    return {GF2_AB: (m, k, k, n), GF2_ATB: (k, m, k, n), GF2_ABT: (m, k, n, k), GF2_ATBT: (k, m, n, k)}[op]


def dirty_padding(rng, M, cols):
    """set random bits past `cols` in every row's last word (the reference's loops read whole words)"""
    M = M.copy()
    if cols % 64:
        pad = np.uint64((1 << (64 - cols % 64)) - 1)
        M[:, (cols - 1) // 64] |= rng.integers(0, 1 << 63, M.shape[0], dtype=np.uint64) & pad
    return M


def run(ctx, oracle, op, ar, ac, br, bc, seed, dirty=False, pitch=0):
    rng = np.random.default_rng(seed)
    cr, cc = c_shape(op, ar, ac, br, bc)
    A = oracle.gen_plane(seed, 0.5, ar, ac)
    B = oracle.gen_plane(seed + 1, 0.4, br, bc)
    C0 = oracle.gen_plane(seed + 2, 0.5, cr, cc)
    if dirty:
        A, B, C0 = dirty_padding(rng, A, ac), dirty_padding(rng, B, bc), dirty_padding(rng, C0, cc)
    exp = oracle.gf2_mul(op, A, ar, ac, B, br, bc, C0, cr, cc)

    def dev(M):
        if pitch:
            M = np.concatenate([M, rng.integers(0, 1 << 63, (M.shape[0], pitch), dtype=np.uint64)], axis=1)
        return ctx.to_dev(M), M

    (dA, _), (dB, _), (dC, C0p) = dev(A), dev(B), dev(C0)
    ctx.gf2_mul(op, dA, ac, dB, bc, dC, cc)
    ctx.sync()
    got = as_u64(dC)
    cw = (cc + 63) // 64
    assert np.array_equal(got[:, :cw], exp), (op, ar, ac, br, bc)
    if pitch:
        assert np.array_equal(got[:, cw:], C0p[:, cw:])  # words past the row's own are not touched


OPS = [GF2_AB, GF2_ATB, GF2_ABT, GF2_ATBT]


@pytest.mark.parametrize("op", OPS)
@pytest.mark.parametrize("m,k,n", [(1, 1, 1), (3, 5, 7), (64, 64, 64), (65, 63, 129), (257, 130, 300),
                                   (100, 1, 70), (5, 640, 9), (300, 256, 257)])
def test_mul_shapes(ctx, oracle, op, m, k, n):
    run(ctx, oracle, op, *shapes(op, m, k, n), seed=1000 * op + m + 7 * k + 31 * n)


@pytest.mark.parametrize("op", OPS)
@pytest.mark.parametrize("m,k,n", [(37, 70, 45), (129, 200, 65)])
def test_mul_dirty_padding(ctx, oracle, op, m, k, n):
    run(ctx, oracle, op, *shapes(op, m, k, n), seed=5000 + op, dirty=True)


@pytest.mark.parametrize("ar,ac,br,bc", [(20, 100, 90, 100), (20, 100, 130, 100), (33, 70, 64, 70),
                                         (9, 65, 1, 65), (70, 200, 120, 200)])
def test_mul_abt_as_written(ctx, oracle, ar, ac, br, bc):
    """j runs over B.cols (binmat.cpp:584): below B.rows the bits past B.cols keep their value,
    above it the extra bits are written 0 and the writes past the row spill (and are dropped)"""
    run(ctx, oracle, GF2_ABT, ar, ac, br, bc, seed=ar * 7 + br, dirty=True)


@pytest.mark.parametrize("op", OPS)
def test_mul_pitched(ctx, oracle, op):
    run(ctx, oracle, op, *shapes(op, 70, 130, 90), seed=6000 + op, pitch=3)


@pytest.mark.parametrize("op", [GF2_AB, GF2_ATB, GF2_ABT])
def test_mul_large(ctx, oracle, op):
    run(ctx, oracle, op, *shapes(op, 1024, 700, 2048), seed=7000 + op)


def test_mul_bad_shapes(ctx, oracle):
    A = ctx.to_dev(oracle.gen_plane(1, 0.5, 4, 5))
    B = ctx.to_dev(oracle.gen_plane(2, 0.5, 6, 7))
    C = ctx.to_dev(oracle.gen_plane(3, 0.5, 4, 7))
    for op in OPS:
        with pytest.raises(pybic.BicError):
            ctx.gf2_mul(op, A, 5, B, 7, C, 7)  # A.cols != B.rows etc.: the reference asserts
    with pytest.raises(pybic.BicError):
        ctx.gf2_mul(9, A, 5, B, 7, C, 7)


@pytest.mark.parametrize("rows,cols", [(1, 1), (3, 65), (64, 64), (70, 37), (130, 200), (1000, 333), (4096, 64)])
def test_transpose(ctx, oracle, rows, cols):
    M = oracle.gen_plane(rows * 3 + cols, 0.5, rows, cols)
    got = as_u64(ctx.gf2_transpose(ctx.to_dev(M), cols))
    ctx.sync()
    assert np.array_equal(got, oracle.gf2_transpose(M, rows, cols))
