"""ctypes bindings for the TEST-ONLY oracle (oracle/liboracle.so) and, where present,
the reference-object harness (oracle/_ref/libref.so). Test infrastructure: the product
path (binary-image-compression_amd/) never imports this module."""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref.so")

u64p = C.POINTER(C.c_uint64)
u32p = C.POINTER(C.c_uint32)
i32p = C.POINTER(C.c_int32)
u8p = C.POINTER(C.c_uint8)
dp = C.POINTER(C.c_double)
sz = C.c_size_t


def ptr(a, t):
    return a.ctypes.data_as(t) if a is not None else None


def _sig(lib, name, res, args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = args
    return f


class Oracle:
    def __init__(self, path=ORACLE_SO):
        self.lib = L = C.CDLL(path)
        _sig(L, "bo_gen_plane", None, [C.c_uint64, C.c_double, sz, sz, sz, u64p])
        _sig(L, "bo_gen_bytes", None, [C.c_uint64, sz, u8p])
        _sig(L, "bo_bitplanes", None, [C.c_void_p, C.c_int, sz, sz, C.c_int, u64p, sz])
        _sig(L, "bo_planes_to_gray", None, [u64p, C.c_int, sz, sz, sz, u32p])
        _sig(L, "bo_num_planes", C.c_int, [C.c_int])
        _sig(L, "bo_med", None, [u64p, u64p, sz, sz, sz])
        _sig(L, "bo_weight", C.c_uint64, [u64p, sz, sz, sz])
        _sig(L, "bo_encode_plane", C.c_int64, [u64p, sz, sz, sz, C.c_int, C.c_int, u8p, sz, u64p])
        _sig(L, "bo_plane_runs", sz, [u64p, sz, sz, sz, u32p, u8p, sz])
        _sig(L, "bo_golomb_samples", C.c_int64, [u32p, sz, u8p, sz, u32p, u32p])
        _sig(L, "bo_decode_plane_golomb", C.c_int, [u8p, C.c_uint64, sz, sz, sz, C.c_int, C.c_int, u64p])
        _sig(L, "bo_unmed", None, [u64p, u64p, sz, sz, sz, C.c_int])
        _sig(L, "bo_row_index", None, [u64p, sz, sz, sz, C.c_int, u64p])
        _sig(L, "bo_egad_row_index", None, [u64p, sz, sz, sz, C.c_int, u64p])
        _sig(L, "bo_eg_runs", C.c_int64, [i32p, u8p, sz, C.c_int, u8p, sz, u32p])
        _sig(L, "cf_encode_planes", C.c_uint64, [u64p, C.c_int, sz, sz, sz, C.c_int, C.c_int, u64p, C.c_uint64, u64p,
                                                  C.c_uint64, u64p, u64p, C.POINTER(C.c_int)])
        _sig(L, "bo_get_submatrix", None, [u64p, sz, sz, sz, sz, sz, sz, sz, u64p, sz])
        _sig(L, "bo_set_submatrix", None, [u64p, sz, sz, sz, sz, sz, u64p, sz, sz, sz])
        _sig(L, "bo_enumL", C.c_double, [C.c_uint, C.c_uint])
        _sig(L, "bo_patch_encode", C.c_int64,
             [u64p, sz, sz, sz, C.c_uint, u64p, u32p, u32p, C.c_char_p, u64p, u8p, sz])
        _sig(L, "bo_baseline_planes", C.c_uint64, [u64p, C.c_int, sz, sz, sz, C.c_int, C.c_int, C.POINTER(C.c_int)])
        _sig(L, "bo_patch_search", None, [u64p, sz, sz, sz, C.c_uint, u32p, u32p, u32p])
        _sig(L, "bo_patch_search_rows", None, [u64p, sz, sz, sz, C.c_uint, sz, sz, u32p, u32p, u32p])
        _sig(L, "bo_gf2_transpose", None, [u64p, sz, sz, u64p])
        _sig(L, "bo_gf2_mul", C.c_int, [C.c_int, u64p, sz, sz, u64p, sz, sz, u64p, sz, sz])
        _sig(L, "bo_match_encode", C.c_int,
             [u64p, sz, sz, sz, C.c_uint, C.c_uint, C.c_uint, dp, u32p, u32p, u32p, u32p, C.c_char_p, u64p,
              u8p, u8p, sz])
        _sig(L, "bo_match_encode_v", C.c_int,
             [u64p, sz, sz, sz, C.c_uint, C.c_uint, C.c_uint, dp, u32p, u32p, u32p, u32p, C.c_char_p, u64p,
              u8p, u8p, sz, C.c_int, u8p])
        _sig(L, "bo_match_encode_var", C.c_int,
             [u64p, sz, sz, sz, C.c_uint, C.c_uint, C.c_uint, dp, u32p, u32p, u32p, u32p, C.c_char_p, u64p,
              u8p, u8p, sz, C.c_int])

    # -- inputs ----------------------------------------------------------
    def gen_plane(self, seed, p, rows, cols, wpr=None):
        wpr = wpr or (cols + 63) // 64
        P = np.zeros((rows, wpr), np.uint64)
        self.lib.bo_gen_plane(seed, p, rows, cols, wpr, ptr(P, u64p))
        return P

    def gen_bytes(self, seed, n):
        out = np.zeros(n, np.uint8)
        self.lib.bo_gen_bytes(seed, n, ptr(out, u8p))
        return out

    # -- ops ---------------------------------------------------------------
    def bitplanes(self, gray, nplanes, wpr=None):
        rows, cols = gray.shape
        wpr = wpr or (cols + 63) // 64
        gray = np.ascontiguousarray(gray)
        out = np.zeros((nplanes, rows, wpr), np.uint64)
        self.lib.bo_bitplanes(gray.ctypes.data, gray.dtype.itemsize, rows, cols, nplanes, ptr(out, u64p), wpr)
        return out

    def planes_to_gray(self, planes, cols):
        """plane2pgm_tool.cpp:26-41: planes [n, rows, wpr] -> uint32 samples [rows, cols]"""
        planes = np.ascontiguousarray(planes, np.uint64)
        n, rows, wpr = planes.shape
        out = np.zeros((rows, cols), np.uint32)
        self.lib.bo_planes_to_gray(ptr(planes, u64p), n, rows, cols, wpr, ptr(out, u32p))
        return out

    def med(self, P, cols):
        P = np.ascontiguousarray(P)
        R = np.zeros_like(P)
        self.lib.bo_med(ptr(P, u64p), ptr(R, u64p), P.shape[0], cols, P.shape[1])
        return R

    def weight(self, P, cols):
        P = np.ascontiguousarray(P)
        return int(self.lib.bo_weight(ptr(P, u64p), P.shape[0], cols, P.shape[1]))

    def encode_plane(self, P, cols, predict, coder, want_stream=True):
        """returns (nbits, stream bytes (len = ceil(bits/64)*8), nsamples)"""
        P = np.ascontiguousarray(P)
        rows, wpr = P.shape
        ns = C.c_uint64(0)
        if not want_stream:
            b = self.lib.bo_encode_plane(ptr(P, u64p), rows, cols, wpr, predict, coder, None, 0, C.byref(ns))
            return int(b), None, ns.value
        cap = rows * (cols + 1) // 2 + 4096
        while True:
            buf = np.zeros(cap, np.uint8)
            b = self.lib.bo_encode_plane(ptr(P, u64p), rows, cols, wpr, predict, coder, ptr(buf, u8p), cap, C.byref(ns))
            if b >= 0:
                return int(b), buf[: ((b + 63) // 64) * 8].copy(), ns.value
            cap *= 4

    def plane_runs(self, P, cols):
        P = np.ascontiguousarray(P)
        rows, wpr = P.shape
        cap = rows * (cols + 1)
        runs = np.zeros(cap, np.uint32)
        eols = np.zeros(cap, np.uint8)
        n = self.lib.bo_plane_runs(ptr(P, u64p), rows, cols, wpr, ptr(runs, u32p), ptr(eols, u8p), cap)
        return runs[:n].copy(), eols[:n].copy()

    def golomb_samples(self, s, want_stream=True):
        s = np.ascontiguousarray(s, np.uint32)
        n = len(s)
        k = np.zeros(n, np.uint32)
        ln = np.zeros(n, np.uint32)
        if not want_stream:
            b = self.lib.bo_golomb_samples(ptr(s, u32p), n, None, 0, ptr(k, u32p), ptr(ln, u32p))
            return int(b), None, k, ln
        cap = int(ln.size * 8 + 64)
        b = -1
        while b < 0:
            buf = np.zeros(cap, np.uint8)
            b = self.lib.bo_golomb_samples(ptr(s, u32p), n, ptr(buf, u8p), cap, ptr(k, u32p), ptr(ln, u32p))
            cap *= 4
        return int(b), buf[: ((b + 63) // 64) * 8].copy(), k, ln

    def decode_plane_golomb(self, stream, nbits, rows, cols, predict, corner=0, wpr=None):
        wpr = wpr or (cols + 63) // 64
        P = np.zeros((rows, wpr), np.uint64)
        stream = np.ascontiguousarray(stream, np.uint8)
        rc = self.lib.bo_decode_plane_golomb(ptr(stream, u8p), nbits, rows, cols, wpr, predict, corner, ptr(P, u64p))
        return rc, P

    def fast_encode(self, planes, cols, predict, do_eg=1, want_streams=True):
        """the word-parallel strong-CPU encoder (oracle/cpu_fast.c): (gbits, ebits, G slots, E slots, threads)"""
        planes = np.ascontiguousarray(planes)
        n, rows, wpr = planes.shape
        gslot = 2 * rows * (cols + 1) // 64 + 64
        eslot = (rows * (cols + 1) + 1 + 63) // 64 + 1
        G = np.zeros((n, gslot), np.uint64) if want_streams else None
        E = np.zeros((n, eslot), np.uint64) if want_streams and do_eg else None
        gb, eb = np.zeros(n, np.uint64), np.zeros(n, np.uint64)
        used = C.c_int(0)
        self.lib.cf_encode_planes(ptr(planes, u64p), n, rows, cols, wpr, predict, do_eg, ptr(G, u64p), gslot,
                                  ptr(E, u64p), eslot, ptr(gb, u64p), ptr(eb, u64p), C.byref(used))
        return gb, eb, G, E, used.value

    def eg_runs(self, lens, eols, adaptive):
        """EG over a run list: (total bits, per-run bits, MSB-first stream bytes padded to 64 bits)"""
        lens = np.ascontiguousarray(lens, np.int32)
        eols = np.ascontiguousarray(eols, np.uint8)
        n = len(lens)
        per = np.zeros(n, np.uint32)
        cap = int(np.sum(lens.astype(np.int64))) // 2 + 32 * n + 64
        buf = np.zeros(cap, np.uint8)
        b = self.lib.bo_eg_runs(ptr(lens, i32p), ptr(eols, u8p), n, adaptive, ptr(buf, u8p), cap, ptr(per, u32p))
        return int(b), per, buf[: ((b + 63) // 64) * 8].copy()

    def row_index(self, P, cols, predict):
        """per row: (Golomb bit offset of its first codeword, residual 1s before it), flat u64"""
        P = np.ascontiguousarray(P)
        rows, wpr = P.shape
        out = np.zeros(2 * rows, np.uint64)
        self.lib.bo_row_index(ptr(P, u64p), rows, cols, wpr, predict, ptr(out, u64p))
        return out

    def egad_row_index(self, P, cols, predict):
        """per row: (adaptive EG bit offset of its first codeword, coder state there: lutIndex, 32 fresh)"""
        P = np.ascontiguousarray(P)
        rows, wpr = P.shape
        out = np.zeros(2 * rows, np.uint64)
        self.lib.bo_egad_row_index(ptr(P, u64p), rows, cols, wpr, predict, ptr(out, u64p))
        return out

    def get_submatrix(self, I, cols, i0, i1, j0, j1):
        I = np.ascontiguousarray(I)
        bw = (j1 - j0 + 63) // 64
        B = np.zeros((i1 - i0, bw), np.uint64)
        self.lib.bo_get_submatrix(ptr(I, u64p), I.shape[0], cols, I.shape[1], i0, i1, j0, j1, ptr(B, u64p), bw)
        return B

    def enumL(self, n, r):
        return float(self.lib.bo_enumL(n, r))

    def lentab(self, W):
        M = W * W
        return np.array([int(2.0 + self.enumL(M, w)) for w in range(M + 1)], np.uint64)

    def patch_encode(self, I, cols, W, lentab=None, want_stream=True):
        I = np.array(I, copy=True)
        rows, wpr = I.shape
        lentab = self.lentab(W) if lentab is None else np.ascontiguousarray(lentab, np.uint64)
        ny, nx = (rows + W - 1) // W, (cols + W - 1) // W
        n = ny * nx
        wo = np.zeros(n, np.uint32)
        wO = np.zeros(n, np.uint32)
        modes = C.create_string_buffer(n + 1)
        L = C.c_uint64(0)
        cap = n * 8 + 4096
        buf = np.zeros(cap, np.uint8) if want_stream else None
        bits = self.lib.bo_patch_encode(ptr(I, u64p), rows, cols, wpr, W, ptr(lentab, u64p), ptr(wo, u32p),
                                        ptr(wO, u32p), modes, C.byref(L), ptr(buf, u8p), cap if want_stream else 0)
        stream = buf[: ((bits + 63) // 64) * 8].copy() if want_stream else None
        return dict(bits=int(bits), L=L.value, w_nonpred=wo, w_pred=wO,
                    modes=modes.raw[:n].decode(), residual=I, stream=stream)


    def gf2_transpose(self, M, rows, cols):
        """binmat.cpp:199-214 on reference-layout words [rows, ceil(cols/64)]"""
        M = np.ascontiguousarray(M, np.uint64)
        out = np.zeros((cols, (rows + 63) // 64), np.uint64)
        self.lib.bo_gf2_transpose(ptr(M, u64p), rows, cols, ptr(out, u64p))
        return out

    def gf2_mul(self, op, A, a_rows, a_cols, B, b_rows, b_cols, C0, c_rows, c_cols):
        """mul(A, At, B, Bt, C) (binmat.cpp:516-616) on reference-layout words; C0 = C's contents before"""
        A, B = (np.ascontiguousarray(x, np.uint64) for x in (A, B))
        Cm = np.array(C0, np.uint64, copy=True)
        rc = self.lib.bo_gf2_mul(op, ptr(A, u64p), a_rows, a_cols, ptr(B, u64p), b_rows, b_cols, ptr(Cm, u64p),
                                 c_rows, c_cols)
        assert rc == 0
        return Cm

    def patch_search(self, I, cols, W):
        """compress_test.cpp:73-111 search: (besti, bestj, bestd) per tile, raster order."""
        I = np.ascontiguousarray(I)
        rows, wpr = I.shape
        n = ((rows + W - 1) // W) * ((cols + W - 1) // W)
        bi, bj, bd = (np.zeros(n, np.uint32) for _ in range(3))
        self.lib.bo_patch_search(ptr(I, u64p), rows, cols, wpr, W, ptr(bi, u32p), ptr(bj, u32p), ptr(bd, u32p))
        return bi, bj, bd

    def patch_search_par(self, I, cols, W, threads=None):
        """patch_search split by tile rows over host threads (ctypes drops the GIL); the later
        tile rows search more windows, so the rows are dealt out round-robin"""
        I = np.ascontiguousarray(I)
        rows, wpr = I.shape
        ny, nx = (rows + W - 1) // W, (cols + W - 1) // W
        bi, bj, bd = (np.zeros(ny * nx, np.uint32) for _ in range(3))

        def one(tr):
            self.lib.bo_patch_search_rows(ptr(I, u64p), rows, cols, wpr, W, tr, tr + 1, ptr(bi, u32p),
                                          ptr(bj, u32p), ptr(bd, u32p))
        pool_map(one, list(range(ny - 1, -1, -1)), threads)
        return bi, bj, bd

    def bitplanes_par(self, gray, nplanes, threads=None, band=512):
        """bitplanes over bands of rows on host threads"""
        gray = np.ascontiguousarray(gray)
        rows, cols = gray.shape
        out = np.zeros((nplanes, rows, (cols + 63) // 64), np.uint64)

        def one(r0):
            out[:, r0:r0 + band] = self.bitplanes(gray[r0:r0 + band], nplanes)
        pool_map(one, list(range(0, rows, band)), threads)
        return out

    def encode_planes_par(self, planes, cols, predict, coders=(0, 1), threads=None):
        """{(plane, coder): (nbits, stream bytes)} for every plane and coder, on host threads"""
        jobs = [(k, c) for k in range(planes.shape[0]) for c in coders]

        def one(job):
            k, c = job
            b, st, _ = self.encode_plane(planes[k], cols, predict, c)
            return job, (b, st)
        return dict(pool_map(one, jobs, threads))

    def enum_table(self, W):
        """enumL(W*W, w) for w = 0..W*W (the double table the match loop takes)."""
        M = W * W
        return np.array([self.enumL(M, w) for w in range(M + 1)], np.float64)

    def match_encode(self, I, cols, W, T=0, R=128, enuml=None, want_stream=True, invert=False):
        """compress7_test.cpp:117-275 with search window R, threshold T (bo_match_encode); invert:
        compress8_test.cpp's patch-inversion variant (bo_match_encode_v), with `inverted` per tile."""
        I = np.array(I, copy=True)
        rows, wpr = I.shape
        enuml = self.enum_table(W) if enuml is None else np.ascontiguousarray(enuml, np.float64)
        n = (rows // W) * (cols // W)
        bi, bj, bd, wt = (np.zeros(n, np.uint32) for _ in range(4))
        modes = C.create_string_buffer(n + 1)
        stats = np.zeros(4, np.uint64)
        cap = n * 8 + 4096
        bm = np.zeros(cap, np.uint8) if want_stream else None
        bn = np.zeros(cap, np.uint8) if want_stream else None
        inv = np.zeros(n, np.uint8)
        rc = self.lib.bo_match_encode_v(ptr(I, u64p), rows, cols, wpr, W, T, R, ptr(enuml, dp), ptr(bi, u32p),
                                        ptr(bj, u32p), ptr(bd, u32p), ptr(wt, u32p), modes, ptr(stats, u64p),
                                        ptr(bm, u8p), ptr(bn, u8p), cap if want_stream else 0, int(invert),
                                        ptr(inv, u8p))
        assert rc == 0, rc
        out = dict(besti=bi, bestj=bj, bestd=bd, weights=wt, modes=modes.raw[:n].decode(), residual=I,
                   matches=int(stats[0]), bits_match=int(stats[1]), bits_nomatch=int(stats[2]), L=int(stats[3]),
                   inverted=inv)
        if want_stream:
            out["stream_match"] = bm[: ((out["bits_match"] + 63) // 64) * 8].copy()
            out["stream_nomatch"] = bn[: ((out["bits_nomatch"] + 63) // 64) * 8].copy()
        return out


def _match_var(lib_fn, I, cols, W, T, R, enuml, variant, cap):
    I = np.array(I, copy=True)
    rows, wpr = I.shape
    n = (rows // W) * (cols // W)
    bi, bj, bd, wt = (np.zeros(n, np.uint32) for _ in range(4))
    modes = C.create_string_buffer(n + 1)
    stats = np.zeros(4, np.uint64)
    streams = [np.zeros(cap, np.uint8), np.zeros(cap, np.uint8)] if cap else [None, None]
    rc = lib_fn(I, rows, wpr, bi, bj, bd, wt, modes, stats, streams, n)
    assert rc == 0, rc
    out = dict(besti=bi, bestj=bj, bestd=bd, weights=wt, modes=modes.raw[:n].decode(), residual=I,
               matches=int(stats[0]), bits_match=int(stats[1]), bits_nomatch=int(stats[2]), L=int(stats[3]))
    if cap:
        out["stream_match"] = streams[0][: ((out["bits_match"] + 63) // 64) * 8].copy()
        out["stream_nomatch"] = streams[1][: ((out["bits_nomatch"] + 63) // 64) * 8].copy()
    return out


def match_encode_var(oracle, I, cols, W, T, R, enuml, variant, want_stream=True):
    """compress4/5/6_test.cpp's loops (bo_match_encode_var: variant 4, 5 or 6)"""
    enuml = np.ascontiguousarray(enuml, np.float64)

    def call(I, rows, wpr, bi, bj, bd, wt, modes, stats, streams, n):
        cap = len(streams[0]) if streams[0] is not None else 0
        return oracle.lib.bo_match_encode_var(ptr(I, u64p), rows, cols, wpr, W, T, R, ptr(enuml, dp), ptr(bi, u32p),
                                              ptr(bj, u32p), ptr(bd, u32p), ptr(wt, u32p), modes, ptr(stats, u64p),
                                              ptr(streams[0], u8p), ptr(streams[1], u8p), cap, variant)
    n = (I.shape[0] // W) * (cols // W)
    return _match_var(call, I, cols, W, T, R, enuml, variant, n * 8 + 4096 if want_stream else 0)


class Ref:
    """The reference's own objects (oracle/_ref/libref.so): compiled in the build container from the
    reference's sources (oracle/Makefile ref; git-ignored, never committed, and kept off the GPU box
    by .gpurunignore). Test-side only."""

    def __init__(self, path=REF_SO):
        self.lib = L = C.CDLL(path)
        _sig(L, "ref_med", C.c_int, [u64p, u64p, sz, sz, sz])
        _sig(L, "ref_weight", C.c_uint64, [u64p, sz, sz, sz])
        _sig(L, "ref_golomb", C.c_int64, [u32p, sz, u32p, u32p])
        _sig(L, "ref_eg", C.c_uint64, [i32p, u8p, sz, u32p])
        _sig(L, "ref_get_submatrix", C.c_int, [u64p, sz, sz, sz, sz, sz, sz, sz, u64p, sz])
        _sig(L, "ref_set_submatrix", C.c_int, [u64p, sz, sz, sz, sz, sz, u64p, sz, sz, sz])
        _sig(L, "ref_tile_loop", C.c_int64, [u64p, sz, sz, sz, C.c_uint, u64p, u32p, u32p, C.c_char_p, u64p])
        _sig(L, "ref_pbm_roundtrip", C.c_int, [C.c_char_p, C.c_char_p, u64p])
        _sig(L, "ref_read_pbm", C.c_int, [C.c_char_p, u64p, sz, u64p])
        _sig(L, "ref_read_pgm", C.c_int, [C.c_char_p, C.POINTER(C.c_int), u32p])
        _sig(L, "ref_patch_search", C.c_int, [u64p, sz, sz, sz, C.c_uint, u32p, u32p, u32p])
        _sig(L, "ref_match_loop", C.c_int,
             [u64p, sz, sz, sz, C.c_uint, C.c_uint, C.c_uint, dp, u32p, u32p, u32p, u32p, C.c_char_p, u64p])
        _sig(L, "ref_match_loop8", C.c_int,
             [u64p, sz, sz, sz, C.c_uint, C.c_uint, C.c_uint, dp, u32p, u32p, u32p, u32p, C.c_char_p, u8p, u64p])
        _sig(L, "ref_match_loop_var", C.c_int,
             [u64p, sz, sz, sz, C.c_uint, C.c_uint, C.c_uint, dp, u32p, u32p, u32p, u32p, C.c_char_p, u64p, C.c_int])
        _sig(L, "ref_gf2_mul", C.c_int, [C.c_int, u64p, sz, sz, u64p, sz, sz, u64p, sz, sz])
        _sig(L, "ref_gf2_transpose", C.c_int, [u64p, sz, sz, u64p])
        _sig(L, "ref_baseline_planes", C.c_double,
             [u64p, C.c_int, sz, sz, sz, C.c_int, C.c_int, C.c_int, u64p, C.POINTER(C.c_int)])

    def planes_to_gray(self, planes, cols):
        """plane2pgm_tool.cpp:26-41: planes [n, rows, wpr] -> uint32 samples [rows, cols]"""
        planes = np.ascontiguousarray(planes, np.uint64)
        n, rows, wpr = planes.shape
        out = np.zeros((rows, cols), np.uint32)
        self.lib.bo_planes_to_gray(ptr(planes, u64p), n, rows, cols, wpr, ptr(out, u32p))
        return out

    def med(self, P, cols):
        P = np.ascontiguousarray(P)
        R = np.zeros_like(P)
        self.lib.ref_med(ptr(P, u64p), ptr(R, u64p), P.shape[0], cols, P.shape[1])
        return R

    def weight(self, P, cols):
        P = np.ascontiguousarray(P)
        return int(self.lib.ref_weight(ptr(P, u64p), P.shape[0], cols, P.shape[1]))

    def golomb(self, s):
        s = np.ascontiguousarray(s, np.uint32)
        k = np.zeros(len(s), np.uint32)
        ln = np.zeros(len(s), np.uint32)
        b = self.lib.ref_golomb(ptr(s, u32p), len(s), ptr(k, u32p), ptr(ln, u32p))
        return int(b), k, ln

    def eg(self, lens, eols):
        lens = np.ascontiguousarray(lens, np.int32)
        eols = np.ascontiguousarray(eols, np.uint8)
        bits = np.zeros(len(lens), np.uint32)
        b = self.lib.ref_eg(ptr(lens, i32p), ptr(eols, u8p), len(lens), ptr(bits, u32p))
        return int(b), bits

    def eg_adaptive(self, lens, eols):
        """the reference's EG state machine with incBlockSize enabled: (bits, per-run bits, stream bytes)"""
        lens = np.ascontiguousarray(lens, np.int32)
        eols = np.ascontiguousarray(eols, np.uint8)
        n = len(lens)
        per = np.zeros(n, np.uint32)
        cap = int(np.sum(lens.astype(np.int64))) // 2 + 32 * n + 64
        buf = np.zeros(cap, np.uint8)
        f = self.lib.ref_eg_adaptive
        f.restype = C.c_uint64
        f.argtypes = [i32p, u8p, sz, u32p, u8p, sz]
        b = f(ptr(lens, i32p), ptr(eols, u8p), n, ptr(per, u32p), ptr(buf, u8p), cap)
        return int(b), per, buf[: ((b + 63) // 64) * 8].copy()

    def get_submatrix(self, I, cols, i0, i1, j0, j1):
        I = np.ascontiguousarray(I)
        bw = (j1 - j0 + 63) // 64
        B = np.zeros((i1 - i0, bw), np.uint64)
        self.lib.ref_get_submatrix(ptr(I, u64p), I.shape[0], cols, I.shape[1], i0, i1, j0, j1, ptr(B, u64p), bw)
        return B

    def tile_loop(self, I, cols, W, lentab):
        I = np.array(I, copy=True)
        rows, wpr = I.shape
        lentab = np.ascontiguousarray(lentab, np.uint64)
        n = ((rows + W - 1) // W) * ((cols + W - 1) // W)
        wo = np.zeros(n, np.uint32)
        wO = np.zeros(n, np.uint32)
        modes = C.create_string_buffer(n + 1)
        L = C.c_uint64(0)
        bits = self.lib.ref_tile_loop(ptr(I, u64p), rows, cols, wpr, W, ptr(lentab, u64p), ptr(wo, u32p),
                                      ptr(wO, u32p), modes, C.byref(L))
        return dict(bits=int(bits), L=L.value, w_nonpred=wo, w_pred=wO, modes=modes.raw[:n].decode(), residual=I)

    def read_pbm(self, path):
        rc = np.zeros(2, np.uint64)
        self.lib.ref_read_pbm(path.encode(), None, 0, ptr(rc, u64p))
        rows, cols = int(rc[0]), int(rc[1])
        wpr = (cols + 63) // 64
        out = np.zeros((rows, wpr), np.uint64)
        self.lib.ref_read_pbm(path.encode(), ptr(out, u64p), wpr, ptr(rc, u64p))
        return rows, cols, out

    def pbm_roundtrip(self, path, out_path):
        rc = np.zeros(2, np.uint64)
        return self.lib.ref_pbm_roundtrip(path.encode(), out_path.encode(), ptr(rc, u64p))

    def gf2_transpose(self, M, rows, cols):
        M = np.ascontiguousarray(M, np.uint64)
        out = np.zeros((cols, (rows + 63) // 64), np.uint64)
        self.lib.ref_gf2_transpose(ptr(M, u64p), rows, cols, ptr(out, u64p))
        return out

    def gf2_mul(self, op, A, a_rows, a_cols, B, b_rows, b_cols, C0, c_rows, c_cols):
        A, B = (np.ascontiguousarray(x, np.uint64) for x in (A, B))
        Cm = np.array(C0, np.uint64, copy=True)
        self.lib.ref_gf2_mul(op, ptr(A, u64p), a_rows, a_cols, ptr(B, u64p), b_rows, b_cols, ptr(Cm, u64p),
                             c_rows, c_cols)
        return Cm

    def patch_search(self, I, cols, W):
        I = np.ascontiguousarray(I)
        rows, wpr = I.shape
        n = ((rows + W - 1) // W) * ((cols + W - 1) // W)
        bi, bj, bd = (np.zeros(n, np.uint32) for _ in range(3))
        self.lib.ref_patch_search(ptr(I, u64p), rows, cols, wpr, W, ptr(bi, u32p), ptr(bj, u32p), ptr(bd, u32p))
        return bi, bj, bd

    def match_loop(self, I, cols, W, T, R, enuml):
        I = np.array(I, copy=True)
        rows, wpr = I.shape
        enuml = np.ascontiguousarray(enuml, np.float64)
        n = (rows // W) * (cols // W)
        bi, bj, bd, wt = (np.zeros(n, np.uint32) for _ in range(4))
        modes = C.create_string_buffer(n + 1)
        stats = np.zeros(4, np.uint64)
        self.lib.ref_match_loop(ptr(I, u64p), rows, cols, wpr, W, T, R, ptr(enuml, dp), ptr(bi, u32p),
                                ptr(bj, u32p), ptr(bd, u32p), ptr(wt, u32p), modes, ptr(stats, u64p))
        return dict(besti=bi, bestj=bj, bestd=bd, weights=wt, modes=modes.raw[:n].decode(), residual=I,
                    matches=int(stats[0]), bits_match=int(stats[1]), bits_nomatch=int(stats[2]), L=int(stats[3]))

    def match_loop_var(self, I, cols, W, T, R, enuml, variant):
        """compress4/5/6_test.cpp's loops over the reference's objects (ref_match_loop_var)"""
        enuml = np.ascontiguousarray(enuml, np.float64)

        def call(I, rows, wpr, bi, bj, bd, wt, modes, stats, streams, n):
            return self.lib.ref_match_loop_var(ptr(I, u64p), rows, cols, wpr, W, T, R, ptr(enuml, dp), ptr(bi, u32p),
                                               ptr(bj, u32p), ptr(bd, u32p), ptr(wt, u32p), modes, ptr(stats, u64p),
                                               variant)
        return _match_var(call, I, cols, W, T, R, enuml, variant, 0)

    def match_loop8(self, I, cols, W, T, R, enuml):
        """compress8_test.cpp:126-272 over the reference's objects (ref_match_loop8)"""
        I = np.array(I, copy=True)
        rows, wpr = I.shape
        enuml = np.ascontiguousarray(enuml, np.float64)
        n = (rows // W) * (cols // W)
        bi, bj, bd, wt = (np.zeros(n, np.uint32) for _ in range(4))
        inv = np.zeros(n, np.uint8)
        modes = C.create_string_buffer(n + 1)
        stats = np.zeros(4, np.uint64)
        self.lib.ref_match_loop8(ptr(I, u64p), rows, cols, wpr, W, T, R, ptr(enuml, dp), ptr(bi, u32p),
                                 ptr(bj, u32p), ptr(bd, u32p), ptr(wt, u32p), modes, ptr(inv, u8p), ptr(stats, u64p))
        return dict(besti=bi, bestj=bj, bestd=bd, weights=wt, modes=modes.raw[:n].decode(), residual=I,
                    matches=int(stats[0]), bits_match=int(stats[1]), bits_nomatch=int(stats[2]), L=int(stats[3]),
                    inverted=inv)

    def baseline(self, planes, rows, cols, predict=1, do_eg=1, threads=0):
        planes = np.ascontiguousarray(planes)
        nplanes = planes.shape[0]
        wpr = planes.shape[-1]
        bits = np.zeros(2, np.uint64)
        used = C.c_int(0)
        dt = self.lib.ref_baseline_planes(ptr(planes, u64p), nplanes, rows, cols, wpr, predict, do_eg,
                                          threads, ptr(bits, u64p), C.byref(used))
        return dt, int(bits[0]), int(bits[1]), used.value


def have_ref():
    return os.path.exists(REF_SO)


def host_threads():
    """worker threads for the checker: the box's CPU share (OMP_NUM_THREADS is set to it there;
    os.cpu_count() reports the whole machine)"""
    try:
        n = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        n = 0
    return max(1, min(16, n or os.cpu_count() or 1))


def pool_map(fn, items, threads=None):
    """fn over items on a thread pool, results in order (the oracle's ctypes calls drop the GIL)"""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=threads or host_threads()) as ex:
        return list(ex.map(fn, items))


def pack_rows(bits):
    """bool (rows, cols) -> plane words (rows, ceil(cols/64)), MSB = leftmost pixel."""
    rows, cols = bits.shape
    wpr = max(1, (cols + 63) // 64)
    pad = np.zeros((rows, wpr * 64), bool)
    pad[:, :cols] = bits
    return np.packbits(pad, axis=1).view(">u8").astype(np.uint64).reshape(rows, wpr)


def periodic_plane(seed, rows, cols, ph, pw, p=0.5, flip=0.0):
    """A random ph x pw block repeated over the plane, then bits flipped with probability
    `flip`: inputs on which compress7's match search finds exact and near matches."""
    rng = np.random.default_rng(seed)
    blk = rng.random((ph, pw)) < p
    bits = np.tile(blk, (rows // ph + 1, cols // pw + 1))[:rows, :cols]
    if flip:
        bits ^= rng.random((rows, cols)) < flip
    return pack_rows(bits)


def inverted_plane(seed, rows, cols, ph, pw, p=0.5, flip=0.0, ones_tiles=0):
    """periodic_plane with every other period block (checkerboard) complemented, plus `ones_tiles`
    all-1 blocks of ph x pw: inputs on which compress8's search prefers inverted windows and meets
    tiles whose weight is M (its initial bestinv)."""
    rng = np.random.default_rng(seed)
    blk = rng.random((ph, pw)) < p
    bits = np.tile(blk, (rows // ph + 1, cols // pw + 1))[:rows, :cols]
    ii, jj = np.meshgrid(np.arange(rows) // ph, np.arange(cols) // pw, indexing="ij")
    bits ^= ((ii + jj) & 1).astype(bool)
    if flip:
        bits ^= rng.random((rows, cols)) < flip
    for _ in range(ones_tiles):
        i0, j0 = int(rng.integers(0, rows // ph)) * ph, int(rng.integers(0, cols // pw)) * pw
        bits[i0:i0 + ph, j0:j0 + pw] = True
    return pack_rows(bits)


def text_plane(seed, rows, cols, glyph_h=11, glyph_w=7, advance=8, line=16, nglyphs=40, p=0.45, space=0.15):
    """A synthetic bilevel 'text' page: lines of glyphs drawn from a small random alphabet at a
    fixed advance, with word gaps -- repeated shapes at offsets unrelated to the tile grid, the
    kind of input compress7's match search is for."""
    rng = np.random.default_rng(seed)
    alpha = rng.random((nglyphs, glyph_h, glyph_w)) < p
    bits = np.zeros((rows, cols), bool)
    top = 2
    while top + glyph_h <= rows:
        x = 3 + int(rng.integers(0, advance))
        while x + glyph_w <= cols:
            if rng.random() >= space:
                bits[top:top + glyph_h, x:x + glyph_w] = alpha[int(rng.integers(0, nglyphs))]
            x += advance
        top += line
    return pack_rows(bits)
