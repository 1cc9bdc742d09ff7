"""Expected stdout of the reference's GSL drivers (compress_test, compress4/5/6/7_test) -- TEST
INFRASTRUCTURE ONLY (tests/test_dropin_compress.py).

The drivers need GSL (gsl_sf_lnchoose), which this image lacks, so no reference-side build of them is
made. Their expected output is assembled here instead:
* every value that comes out of the tile loops -- the search results, the tile weights the drivers print,
  the modes, the Golomb bit counts, the final image -- from the reference's OWN objects, run through
  oracle/_ref/libref.so (ref_patch_search_w, ref_match_loop_w4, ref_match_loop_var_w2: the drivers'
  loops over binmat.cpp / GolombCoder.cpp compiled from /root/reference, enumL passed in);
* the printed arithmetic restated from the drivers' statements, with the C conversions they perform
  (double -> idx_t as gcc's x86-64 code does it, unsigned 64-bit wrap-around);
* enumL through the same lnchoose as tests/cpp/gsl_shim (a sum of libm logs, which math.log is).
Each function cites the driver lines it restates.
"""
import ctypes as C
import math

import numpy as np

from oracle_lib import Ref, dp, ptr, sz, u32p, u64p

LOG2E = float("1.442695040888963387004650940070860087872")  # COSMOS_LOG2E (compress7_test.cpp:22)
SEP = "\n" + "=" * 75 + "\n\n"  # "\n===...===\n" << std::endl
U64 = (1 << 64) - 1
TWO63 = float(1 << 63)


def lnchoose(n, m):
    """tests/cpp/gsl_shim/gsl/gsl_sf_gamma.h, operation for operation"""
    if 2 * m > n:
        m = n - m
    s = 0.0
    for i in range(1, m + 1):
        s += math.log(float(n - m + i) / float(i))
    return s


def enumL(n, r):
    """compress7_test.cpp:25-28 (and the same function in every GSL driver)"""
    return lnchoose(n, r) * LOG2E if r > 0 else 0.0


def _cvtt(d):
    """cvttsd2si: truncation, 0x8000000000000000 for NaN / infinities / out of range"""
    if math.isnan(d) or math.isinf(d) or d >= TWO63 or d < -TWO63:
        return -(1 << 63)
    return int(d)


def d2u(d):
    """double -> unsigned long (idx_t) as gcc emits it on x86-64: below 2^63 (or unordered) one
    cvttsd2si, else cvttsd2si(d - 2^63) with the top bit flipped"""
    if not d >= TWO63:
        return _cvtt(d) & U64
    return (_cvtt(d - TWO63) ^ (1 << 63)) & U64


def u2d(u):
    """unsigned long -> double (correctly rounded)"""
    return float(u & U64)


def ceil_log2(x):
    """idx_t(ceil(log2(x))) for an integer argument (log2 of 0 is -inf, of a negative NaN)"""
    if x > 0:
        return d2u(math.ceil(math.log2(float(x))))
    return d2u(float("-inf") if x == 0 else float("nan"))


def g(x):
    """std::cout << double (precision 6, %g)"""
    return "%g" % x


def print_hist(hist, n, logscale):
    """compress7_test.cpp:31-41 (print_hist)"""
    out = []
    for i in range(n):
        top = d2u(math.ceil(math.log2(hist[i] + 1.0))) if logscale else hist[i]
        out.append(f"{i}:" + "#" * top + "\n")
    return "".join(out)


def golomb_bits(samples):
    """bitcount of a fresh GolombCoder after codeSample over samples (GolombCoder.cpp:13-34), by the
    reference's own coder"""
    if not samples:
        return 0
    b, _, _ = Ref().golomb(np.asarray(samples, np.uint32))
    return b


def _tiles(rows, cols, W):
    return (W - 1 + rows) // W, (W - 1 + cols) // W


# ---------------------------------------------------------------------------------------------------
def compress_test(I, rows, cols, W):
    """compress_test.cpp:41-164 for input plane I (words) and tile width W -> stdout"""
    ref = Ref()
    Ny, Nx = _tiles(rows, cols, W)
    n = Ny * Nx
    bi, bj, bd, wP = (np.zeros(n, np.uint32) for _ in range(4))
    I = np.ascontiguousarray(I)
    ref.lib.ref_patch_search_w.restype = C.c_int
    ref.lib.ref_patch_search_w.argtypes = [u64p, sz, sz, sz, C.c_uint, u32p, u32p, u32p, u32p]
    ref.lib.ref_patch_search_w(ptr(I, u64p), rows, cols, I.shape[1], W, ptr(bi, u32p), ptr(bj, u32p),
                               ptr(bd, u32p), ptr(wP, u32p))
    out = [f"rows={rows} cols={cols}\n"]
    hist = [0] * (W * W)
    L = 0.0
    avg = 0
    matches = 0
    sm, sn = [], []
    li = 0
    for i in range(Ny):
        for j in range(Nx):
            b_i, b_j, b_d, w = int(bi[li]), int(bj[li]), int(bd[li]), int(wP[li])
            out.append(SEP)
            out.append(f"i={i * W} j={j * W} besti={b_i} bestj={b_j} bestd={b_d}\n")
            idx_len = ceil_log2(li)  # :117
            nomatch_len = d2u(1 + enumL(W * W, w))  # :123
            match_len = d2u(u2d((1 + idx_len) & U64) + enumL(W * W, b_d))  # :124
            out.append(f"nomatch len={nomatch_len} match_len={match_len}")
            if nomatch_len > match_len:
                sm.append(b_d)
                out.append(" USE MATCH!\n")
                hist[b_d] += 1
                avg += b_d
                matches += 1
                L += u2d(match_len)
            else:
                sn.append(w)
                L += u2d(nomatch_len)
            li += 1
    bm, bn = golomb_bits(sm), golomb_bits(sn)
    avg //= matches  # (the driver divides by zero without a match: callers pick inputs with one)
    out.append(f"MATCHES: {matches}\n")
    out.append(f"\nAVG. WEIGHT: {avg}\n")
    out.append(f"Avg. Golomb/Match: {bm // matches}\n")
    out.append(f"Avg. Golomb/NoMatch: {bn // (Nx * Ny - matches)}\n")
    out.append(f"AVG. WEIGHT: {avg}\n")
    out.append(f"COMP CODELENGTH (bytes): {g((L + bm + bn) / 8)}\n")
    out.append(f"RAW CODELENGTH (bytes): {(rows * cols) // 8}\n")
    out.append(f"RATIO: {g(100.0 * L / (rows * cols))}\n")
    out.append(print_hist(hist, W * W, True))
    return "".join(out)


# ---------------------------------------------------------------------------------------------------
def _window(i0, j0, W, R, cols):
    """compress7_test.cpp:127-132 (and compress4/5/6's subset)"""
    mini = i0 - R if i0 > R else 0
    minj = j0 - R if j0 > R else 0
    maxj = (cols - W) if (j0 + R) > (cols - W) else (j0 + R)
    mini2 = i0 - W if i0 > W else 0
    maxj2 = j0 - W if j0 > W else 0
    swin = (i0 - mini2) * (maxj2 - minj) + (mini2 - mini) * (maxj - minj)
    return mini, minj, maxj, mini2, maxj2, swin


def _write_pbm(ref, I, rows, cols):
    import os
    import tempfile
    fd, path = tempfile.mkstemp(suffix=".pbm")
    os.close(fd)
    try:
        ref.lib.ref_write_pbm.restype = C.c_int
        ref.lib.ref_write_pbm.argtypes = [u64p, sz, sz, sz, C.c_char_p]
        I = np.ascontiguousarray(I)
        assert ref.lib.ref_write_pbm(ptr(I, u64p), rows, cols, I.shape[1], path.encode()) == 0
        with open(path, "rb") as f:
            return f.read()
    finally:
        os.unlink(path)


def _enum_table(M):
    return np.array([enumL(M, w) for w in range(M + 1)], np.float64)


def compress7_test(I, rows, cols, W, T, R):
    """compress7_test.cpp:58-311 -> (stdout, diff.pbm bytes)"""
    ref = Ref()
    M = W * W
    Ny, Nx = _tiles(rows, cols, W)
    n = Ny * Nx
    Iw = np.array(I, np.uint64, copy=True)
    bi, bj, bd, wt = (np.zeros(n, np.uint32) for _ in range(4))
    w4 = np.zeros(4 * n, np.uint32)
    modes = C.create_string_buffer(n + 1)
    stats = np.zeros(4, np.uint64)
    en = _enum_table(M)
    f = ref.lib.ref_match_loop_w4
    f.restype = C.c_int
    f.argtypes = [u64p, sz, sz, sz, C.c_uint, C.c_uint, C.c_uint, dp, u32p, u32p, u32p, u32p, C.c_char_p, u64p,
                  u32p]
    assert f(ptr(Iw, u64p), rows, cols, Iw.shape[1], W, T, R, ptr(en, dp), ptr(bi, u32p), ptr(bj, u32p),
             ptr(bd, u32p), ptr(wt, u32p), modes, ptr(stats, u64p), ptr(w4, u32p)) == 0
    md = modes.raw[:n].decode()
    out = [f"rows={rows} cols={cols}\n"]
    hist = [0] * M
    L = 0.0
    avg = 0
    matches = 0
    li = 0
    mp = []
    for i in range(Ny):
        row = []
        for j in range(Nx):
            i0, j0 = i * W, j * W
            mini, minj, maxj, mini2, maxj2, swin = _window(i0, j0, W, R, cols)
            out.append(f"\n{mini2} {i0} {minj} {maxj2} \n{mini} {mini2} {minj} {maxj} ")
            b_i, b_j, b_d = int(bi[li]), int(bj[li]), int(bd[li])
            out.append(SEP)
            out.append(f"i={i0} j={j0} besti={b_i} bestj={b_j} bestd={b_d}\n")
            w_nn, w_np, w_mn, w_mp = (int(x) for x in w4[4 * li:4 * li + 4])
            idx_len = ceil_log2(swin)  # :211
            out.append(f"Search cost: size={swin} len={idx_len}\n")
            out.append(f"weight: nonmatch/nonpred={w_nn}\tnonmatch/pred={w_np}\tmatch/nonpred={w_mn}\t"
                       f"match/pred={w_mp}\n")
            nn = d2u(2 + enumL(M, w_nn))  # :220-223
            np_ = d2u(2 + enumL(M, w_np))
            mn = d2u(u2d((2 + idx_len) & U64) + enumL(M, w_mn))
            mpl = d2u(u2d((2 + idx_len) & U64) + enumL(M, w_mp))
            out.append(f"len: nonmatch/nonpred={nn}\tnonmatch/pred={np_}\tmatch/nonpred={mn}\tmatch/pred={mpl}\n")
            m_len, m_w, m_mode = (mpl, w_mp, "X") if mn > mpl else (mn, w_mn, "x")  # :236-246
            n_len, n_w, n_mode = (np_, w_np, "O") if nn > np_ else (nn, w_nn, "o")  # :248-258
            if n_len > m_len:
                hist[b_d] += 1
                avg += m_w
                matches += 1
                L += u2d(m_len)
                mode = m_mode
            else:
                L += u2d(n_len)
                mode = n_mode
            assert mode == md[li], (li, mode, md[li])  # the reference loop took the same decision
            out.append(f"mode={mode}\n")
            row.append(mode)
            li += 1
        mp.append("".join(row))
    if matches == 0:
        matches += 1
    avg //= matches
    bm, bn = int(stats[1]), int(stats[2])
    out.append(f"\nMATCHES: {matches}\n")
    out.append(f"AVG. WEIGHT: {avg}\n")
    out.append(f"Avg. Golomb/Match: {bm // matches}\n")
    out.append(f"Avg. Golomb/NoMatch: {bn // (Nx * Ny - matches)}\n")
    out.append(f"AVG. WEIGHT: {avg}\n")
    L = L + bm + bn
    out.append(f"COMP CODELENGTH (bytes): {g(L / 8)}\n")
    out.append(f"RAW CODELENGTH (bytes): {(rows * cols) // 8}\n")
    out.append(f"RATIO: {g(100.0 * L / (rows * cols))}\n")
    out.append(print_hist(hist, M // 4, True))
    out.append("MAP:\n" + "".join(r + "\n" for r in mp))
    return "".join(out), _write_pbm(ref, Iw, rows, cols)


def compress456_test(I, rows, cols, W, T, R, variant):
    """compress4_test.cpp:52-193 (variant 4), compress5_test.cpp (5: the unsigned `(d - worstd) >
    (bestd - worstd)` comparison) and compress6_test.cpp:53-233 (6) -> (stdout, diff.pbm bytes or None,
    exit status: -8 where the driver divides by zero)"""
    ref = Ref()
    M = W * W
    Ny, Nx = _tiles(rows, cols, W)
    n = Ny * Nx
    Iw = np.array(I, np.uint64, copy=True)
    bi, bj, bd, wt = (np.zeros(n, np.uint32) for _ in range(4))
    w2 = np.zeros(2 * n, np.uint32)
    modes = C.create_string_buffer(n + 1)
    stats = np.zeros(4, np.uint64)
    en = _enum_table(M)
    f = ref.lib.ref_match_loop_var_w2
    f.restype = C.c_int
    f.argtypes = [u64p, sz, sz, sz, C.c_uint, C.c_uint, C.c_uint, dp, u32p, u32p, u32p, u32p, C.c_char_p, u64p,
                  C.c_int, u32p]
    assert f(ptr(Iw, u64p), rows, cols, Iw.shape[1], W, T, R, ptr(en, dp), ptr(bi, u32p), ptr(bj, u32p),
             ptr(bd, u32p), ptr(wt, u32p), modes, ptr(stats, u64p), variant, ptr(w2, u32p)) == 0
    md = modes.raw[:n].decode()
    out = []
    if variant == 6:  # compress6_test.cpp:77-78, before set_grid_width
        buf = C.create_string_buffer(64 * (M + 8) * (2 * M + 16))
        ref.lib.ref_print_pred_matrices.restype = C.c_long
        ref.lib.ref_print_pred_matrices.argtypes = [C.c_uint, C.c_char_p, sz]
        k = ref.lib.ref_print_pred_matrices(M, buf, len(buf))
        assert k >= 0
        out.append(buf.raw[:k].decode())
    out.append(f"rows={rows} cols={cols}\n")
    ninf = rows if cols < rows else cols
    hist = [0] * M
    histi, histj, histr = [0] * rows, [0] * cols, [0] * ninf
    L = 0.0
    avg = 0
    matches = 0
    li = 0
    for i in range(Ny):
        for j in range(Nx):
            i0, j0 = i * W, j * W
            mini, minj, maxj, mini2, maxj2, swin = _window(i0, j0, W, R, cols)
            out.append(f"\n{mini2} {i0} {minj} {j0 - W} ")
            b_i, b_j, b_d = int(bi[li]), int(bj[li]), int(bd[li])
            out.append(SEP)
            out.append(f"i={i0} j={j0} besti={b_i} bestj={b_j} bestd={b_d}\n")
            histi[b_i] += 1
            histj[b_j] += 1
            r = int(math.sqrt(float((b_i * b_i + b_j * b_j) & U64)))
            assert r < ninf, "input whose best match lies outside the driver's histr (out of bounds there)"
            histr[r] += 1
            wP, mw = int(w2[2 * li]), int(w2[2 * li + 1])
            idx_len = ceil_log2(li)
            if variant == 6:  # compress6_test.cpp:186-194
                out.append(f"nmweight={wP} mweight={mw}\n")
                nomatch_len = d2u(1 + enumL(M, wP))
                match_len = d2u(u2d((1 + idx_len) & U64) + enumL(M, mw))
                sample = mw
            else:  # compress4_test.cpp:143-155
                nomatch_len = d2u(1 + enumL(M, wP))
                match_len = d2u(u2d((1 + idx_len) & U64) + enumL(M, b_d)) if b_d <= M else 100000
                sample = b_d
            out.append(f"nomatch len={nomatch_len} match_len={match_len}")
            take = nomatch_len > match_len
            assert ("x" if take else "o") == md[li], (li, take, md[li])
            if take:
                out.append(" USE MATCH!\n")
                hist[b_d] += 1
                avg += sample
                matches += 1
                L += u2d(match_len)
            else:
                L += u2d(nomatch_len)
            li += 1
    bm, bn = int(stats[1]), int(stats[2])
    if variant == 6:
        if matches == 0:
            matches += 1
        avg //= matches
        out.append(f"\nMATCHES: {matches}\n")
        out.append(f"AVG. WEIGHT: {avg}\n")
    else:
        if matches == 0:
            # compress4/5 have no guard: `average_weight /= matches` (compress4_test.cpp:171) divides by
            # zero. The process dies of SIGFPE there, with stdout flushed up to its last std::endl.
            text = "".join(out)
            return text[:text.rfind("\n") + 1], None, -8
        avg //= matches
        out.append(f"MATCHES: {matches}\n")
        out.append(f"\nAVG. WEIGHT: {avg}\n")
    out.append(f"Avg. Golomb/Match: {bm // matches}\n")
    out.append(f"Avg. Golomb/NoMatch: {bn // (Nx * Ny - matches)}\n")
    out.append(f"AVG. WEIGHT: {avg}\n")
    L = L + bm + bn
    out.append(f"COMP CODELENGTH (bytes): {g(L / 8)}\n")
    out.append(f"RAW CODELENGTH (bytes): {(rows * cols) // 8}\n")
    out.append(f"RATIO: {g(100.0 * L / (rows * cols))}\n")
    out.append(print_hist(hist, M, True))
    out.append(print_hist(histi, rows, False))
    out.append(print_hist(histj, cols, False))
    out.append(print_hist(histr, ninf, False))
    return "".join(out), _write_pbm(ref, Iw, rows, cols), 0
