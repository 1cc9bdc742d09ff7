"""pybic -- thin ctypes binding of lib/libbic.so (include/bic.h) for tests, bench and tools.

torch supplies device memory and the stream (plumbing only); every computation runs in the
HIP kernels behind the C ABI. There is no fallback: if libbic.so or a gfx950 device is
missing, construction of `Context` raises.

uint64 planes/streams are carried in torch.int64 tensors (same bits); use `as_u64()` to view
them as numpy uint64 on the host.
"""
import ctypes as C
import os

import numpy as np

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("BIC_LIB_PATH") or os.path.join(PKG, "lib", "libbic.so")

BIC_OK, BIC_EINVAL, BIC_ENOMEM, BIC_EDEVICE, BIC_ENOSPC, BIC_ENODEV, BIC_EDATA = range(7)
CODER_GOLOMB, CODER_EG, CODER_EG_ADAPTIVE = 0, 1, 2

# every symbol include/bic.h declares (tests check the library exports all of them)
EXPORTS = [
    "bic_ctx_create", "bic_ctx_destroy", "bic_ctx_set_stream", "bic_ctx_get_stream", "bic_ctx_own_stream",
    "bic_sync",
    "bic_strerror", "bic_device_count", "bic_reserve", "bic_bitplanes_u8", "bic_med_residual",
    "bic_encode_planes", "bic_encode_planes2", "bic_ctx_set_option", "bic_encode_slot_words", "bic_golomb_encode_samples", "bic_patch_encode",
    "bic_pack_streams", "bic_prof_enable", "bic_prof_collect", "bic_prof_only", "bic_enum_codelength", "bic_tile_lentab",
    "bic_malloc", "bic_free", "bic_memcpy_h2d", "bic_memcpy_d2h", "bic_memset", "bic_pbm_unpack", "bic_pbm_pack",
    "bic_patch_search", "bic_match_encode", "bic_set_match_parts", "bic_encode_gray",
    "bic_bitplanes_u8_range", "bic_encode_gray_range", "bic_encode_planes_packed", "bic_encode_gray_packed",
    "bic_row_index", "bic_decode_planes", "bic_pgm_bitplanes", "bic_pnm_parse_header",
    "bic_gf2_transpose", "bic_gf2_mul", "bic_planes_to_gray", "bic_match_encode_inv", "bic_match_encode_var", "bic_egad_row_index",
]

# bic_gf2_mul ops (include/bic.h)
GF2_AB, GF2_ATB, GF2_ABT, GF2_ATBT = 0, 1, 2, 3


class PnmInfo(C.Structure):
    """include/bic.h bic_pnm_info"""
    _fields_ = [("type", C.c_int), ("rows", C.c_size_t), ("cols", C.c_size_t), ("maxval", C.c_int),
                ("data_offset", C.c_size_t)]


class BicError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        super().__init__(f"{what}: bic error {code} ({_strerror(code)})")


_lib = None


def _strerror(code):
    try:
        return load().bic_strerror(code).decode()
    except Exception:  # pragma: no cover
        return "?"


def load(path=LIB_PATH):
    """Load libbic.so (raises OSError if it is missing: build it with `make` in the package)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OSError(f"{path} not built; run make -C binary-image-compression_amd")
    L = C.CDLL(path)
    vp, sz, u64, i32, u32 = C.c_void_p, C.c_size_t, C.c_uint64, C.c_int, C.c_uint

    def sig(name, res, args):
        f = getattr(L, name)
        f.restype, f.argtypes = res, args

    sig("bic_ctx_create", i32, [i32, C.POINTER(vp)])
    sig("bic_ctx_destroy", i32, [vp])
    sig("bic_ctx_set_stream", i32, [vp, vp])
    sig("bic_ctx_get_stream", vp, [vp])
    sig("bic_ctx_own_stream", vp, [vp])
    sig("bic_sync", i32, [vp])
    sig("bic_strerror", C.c_char_p, [i32])
    sig("bic_device_count", i32, [C.POINTER(i32)])
    sig("bic_reserve", i32, [vp, i32, sz, sz])
    sig("bic_bitplanes_u8", i32, [vp, vp, sz, sz, sz, i32, vp, sz])
    sig("bic_med_residual", i32, [vp, vp, i32, sz, sz, sz, i32, vp, vp])
    sig("bic_encode_planes", i32, [vp, vp, i32, sz, sz, sz, i32, i32, vp, sz, vp])
    sig("bic_encode_slot_words", sz, [sz, sz, i32])
    sig("bic_encode_planes2", i32, [vp, vp, i32, sz, sz, sz, i32, vp, sz, vp, vp, sz, vp])
    sig("bic_ctx_set_option", i32, [vp, i32, C.c_long])
    sig("bic_golomb_encode_samples", i32, [vp, vp, sz, u64, u64, u32, vp, sz, vp])
    sig("bic_patch_encode", i32, [vp, vp, sz, sz, sz, u32, vp, vp, vp, vp, vp, vp, vp, sz, vp])
    sig("bic_pack_streams", i32, [vp, vp, i32, sz, vp, vp, vp])
    sig("bic_prof_enable", i32, [vp, i32])
    sig("bic_prof_collect", i32, [vp, C.c_char_p, sz])
    sig("bic_prof_only", i32, [vp, C.c_char_p])
    sig("bic_enum_codelength", C.c_double, [u32, u32])
    sig("bic_tile_lentab", i32, [u32, vp])
    sig("bic_malloc", i32, [vp, sz, C.POINTER(vp)])
    sig("bic_free", i32, [vp, vp])
    sig("bic_memcpy_h2d", i32, [vp, vp, vp, sz])
    sig("bic_memcpy_d2h", i32, [vp, vp, vp, sz])
    sig("bic_memset", i32, [vp, vp, i32, sz])
    sig("bic_pbm_unpack", i32, [vp, vp, sz, sz, vp, sz])
    sig("bic_pbm_pack", i32, [vp, vp, sz, sz, sz, vp])
    sig("bic_patch_search", i32, [vp, vp, sz, sz, sz, u32, vp, vp, vp])
    sig("bic_match_encode", i32, [vp, vp, sz, sz, sz, u32, u32, u32, vp, vp, vp, vp, vp, vp, vp, vp, vp, sz, vp])
    sig("bic_set_match_parts", i32, [vp, u32])
    sig("bic_match_encode_inv", i32, [vp, vp, sz, sz, sz, u32, u32, u32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, sz, vp])
    sig("bic_egad_row_index", i32, [vp, vp, i32, sz, sz, sz, i32, vp])
    sig("bic_match_encode_var", i32, [vp, i32, vp, sz, sz, sz, u32, u32, u32, vp, vp, vp, vp, vp, vp, vp, vp, vp, sz, vp])
    sig("bic_encode_gray", i32, [vp, vp, sz, sz, sz, i32, vp, sz, i32, vp, sz, vp, vp, sz, vp])
    sig("bic_bitplanes_u8_range", i32, [vp, vp, sz, sz, sz, i32, i32, vp, sz])
    sig("bic_encode_gray_range", i32, [vp, vp, sz, sz, sz, i32, i32, vp, sz, i32, vp, sz, vp, vp, sz, vp])
    sig("bic_encode_planes_packed", i32, [vp, vp, i32, sz, sz, sz, i32, vp, sz, vp, vp, vp, sz, vp, vp, vp])
    sig("bic_encode_gray_packed", i32, [vp, vp, sz, sz, sz, i32, i32, vp, sz, i32, vp, sz, vp, vp, vp, sz, vp, vp, vp])
    sig("bic_row_index", i32, [vp, vp, i32, sz, sz, sz, i32, vp])
    sig("bic_decode_planes", i32, [vp, i32, vp, sz, vp, vp, vp, i32, sz, sz, sz, i32, vp, vp])
    sig("bic_pgm_bitplanes", i32, [vp, vp, sz, sz, i32, i32, i32, vp, sz])
    sig("bic_pnm_parse_header", i32, [C.c_char_p, sz, C.POINTER(PnmInfo)])
    sig("bic_gf2_transpose", i32, [vp, vp, sz, sz, sz, vp, sz])
    sig("bic_gf2_mul", i32, [vp, i32, vp, sz, sz, sz, vp, sz, sz, sz, vp, sz, sz, sz])
    sig("bic_planes_to_gray", i32, [vp, vp, i32, i32, sz, sz, sz, i32, vp, sz])
    _lib = L
    return L


def as_u64(t):
    """torch int64 tensor (any device) -> numpy uint64 copy."""
    return t.detach().cpu().numpy().view(np.uint64)


def stream_bytes(words_i64, nbits):
    """First ceil(nbits/64) big-endian words of a stream slot as the MSB-first byte string."""
    nw = (int(nbits) + 63) // 64
    return as_u64(words_i64[:nw]).tobytes()


def _p(t):
    return None if t is None else C.c_void_p(t.data_ptr())


class Context:
    """One device context (include/bic.h bic_ctx). Calls are enqueued on torch's current
    stream of the device, so they order with torch allocations and copies."""

    def __init__(self, device=0):
        import torch

        self.torch = torch
        self.lib = load()
        self.device = device
        h = C.c_void_p()
        rc = self.lib.bic_ctx_create(device, C.byref(h))
        if rc != BIC_OK:
            raise BicError(rc, f"bic_ctx_create({device})")
        self.h = h
        self.dev = torch.device("cuda", device)

    def close(self):
        if getattr(self, "h", None):
            self.lib.bic_ctx_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # -- plumbing ---------------------------------------------------------------------
    def _bind_stream(self):
        # torch's current stream of the device (handle 0 = the null stream, which is what
        # bic_ctx_set_stream(NULL) selects), so kernels order with torch's copies/allocations
        s = self.torch.cuda.current_stream(self.dev).cuda_stream
        self.lib.bic_ctx_set_stream(self.h, C.c_void_p(s) if s else None)

    def _chk(self, rc, what):
        if rc != BIC_OK:
            raise BicError(rc, what)

    def sync(self):
        rc = self.lib.bic_sync(self.h)
        self._chk(rc, "bic_sync")

    def empty_i64(self, *shape):
        return self.torch.empty(*shape, dtype=self.torch.int64, device=self.dev)

    def to_dev(self, a):
        """numpy array -> device tensor (uint64 carried as int64, uint32 as int32)."""
        a = np.ascontiguousarray(a)
        if a.dtype == np.uint64:
            a = a.view(np.int64)
        elif a.dtype == np.uint32:
            a = a.view(np.int32)
        return self.torch.from_numpy(a).to(self.dev)

    def reserve(self, nplanes, rows, cols):
        self._chk(self.lib.bic_reserve(self.h, nplanes, rows, cols), "bic_reserve")

    def prof_enable(self, on=True):
        self._chk(self.lib.bic_prof_enable(self.h, int(on)), "bic_prof_enable")

    def prof_only(self, name=None):
        """bracket only launches recorded as `name` (None = all; bic_prof_only)"""
        self._chk(self.lib.bic_prof_only(self.h, name.encode() if name else None), "bic_prof_only")

    def prof_collect(self):
        """-> {kernel name: (launches, total_ms)} since the last collect (syncs)."""
        buf = C.create_string_buffer(1 << 16)
        self._chk(self.lib.bic_prof_collect(self.h, buf, len(buf)), "bic_prof_collect")
        out = {}
        for line in buf.value.decode().splitlines():
            name, n, ms = line.split()
            out[name] = (int(n), float(ms))
        return out

    # -- ops --------------------------------------------------------------------------
    def bitplanes_u8(self, gray, cols=None, nplanes=8, wpr=None, out=None, plane0=0):
        """gray: uint8 device tensor [rows, pitch] -> int64 tensor [nplanes, rows, wpr] (planes
        plane0 .. plane0 + nplanes - 1: bic_bitplanes_u8_range)."""
        rows, pitch = gray.shape
        cols = pitch if cols is None else cols
        wpr = wpr or (cols + 63) // 64
        if out is None:
            out = self.empty_i64(nplanes, rows, wpr)
        self._bind_stream()
        if plane0:
            self._chk(self.lib.bic_bitplanes_u8_range(self.h, _p(gray), pitch, rows, cols, plane0, nplanes, _p(out),
                                                      wpr), "bic_bitplanes_u8_range")
        else:
            self._chk(self.lib.bic_bitplanes_u8(self.h, _p(gray), pitch, rows, cols, nplanes, _p(out), wpr),
                      "bic_bitplanes_u8")
        return out

    def med_residual(self, planes, cols, predict=True, want_resid=True, want_weight=True):
        planes = planes if planes.dim() == 3 else planes.unsqueeze(0)
        n, rows, wpr = planes.shape
        resid = self.empty_i64(n, rows, wpr) if want_resid else None
        w = self.torch.zeros(n, dtype=self.torch.int64, device=self.dev) if want_weight else None
        self._bind_stream()
        self._chk(self.lib.bic_med_residual(self.h, _p(planes), n, rows, cols, wpr, int(predict),
                                            _p(resid), _p(w)), "bic_med_residual")
        return resid, w

    def slot_words(self, rows, cols, coder):
        return int(self.lib.bic_encode_slot_words(rows, cols, coder))

    def encode_planes(self, planes, cols, predict=True, coder=CODER_GOLOMB, slot_words=None,
                      out=None, plane_bits=None):
        """-> (out int64 [nplanes, slot_words], plane_bits int64 [nplanes]) (async)."""
        planes = planes if planes.dim() == 3 else planes.unsqueeze(0)
        n, rows, wpr = planes.shape
        slot_words = slot_words or self.slot_words(rows, cols, coder)
        if out is None:
            out = self.empty_i64(n, slot_words)
        if plane_bits is None:
            plane_bits = self.empty_i64(n)
        self._bind_stream()
        self._chk(self.lib.bic_encode_planes(self.h, _p(planes), n, rows, cols, wpr, int(predict), coder,
                                             _p(out), slot_words, _p(plane_bits)), "bic_encode_planes")
        return out, plane_bits

    def encode_planes2(self, planes, cols, predict=True, golomb=True, eg=True, slots=(None, None),
                       outs=(None, None), bits=(None, None)):
        """both streams in one pass -> ((out_g, bits_g) or None, (out_e, bits_e) or None)."""
        planes = planes if planes.dim() == 3 else planes.unsqueeze(0)
        n, rows, wpr = planes.shape
        res = []
        for on, coder, slot, out, b in ((golomb, CODER_GOLOMB, slots[0], outs[0], bits[0]),
                                        (eg, CODER_EG, slots[1], outs[1], bits[1])):
            if not on:
                res.append((None, 0, None))
                continue
            slot = slot or self.slot_words(rows, cols, coder)
            out = self.empty_i64(n, slot) if out is None else out
            b = self.empty_i64(n) if b is None else b
            res.append((out, slot, b))
        (og, sg, bg), (oe, se, be) = res
        self._bind_stream()
        self._chk(self.lib.bic_encode_planes2(self.h, _p(planes), n, rows, cols, wpr, int(predict), _p(og), sg,
                                              _p(bg), _p(oe), se, _p(be)), "bic_encode_planes2")
        return (og, bg) if golomb else None, (oe, be) if eg else None

    def encode_gray(self, gray, cols=None, nplanes=8, predict=True, planes=None, slots=(None, None),
                    outs=(None, None), bits=(None, None), golomb=True, eg=True, plane0=0, store_planes=True):
        """gray uint8 [rows, pitch] -> (planes, (out_g, bits_g) or None, (out_e, bits_e) or None):
        the bitplanes and both streams of every plane in one call (bic_encode_gray; planes plane0 ..
        plane0 + nplanes - 1 with bic_encode_gray_range). store_planes=False: planes NULL (not
        returned: None), the count pass keeps the residual planes in the context instead."""
        rows, pitch = gray.shape
        cols = pitch if cols is None else cols
        wpr = (cols + 63) // 64
        if planes is None and store_planes:
            planes = self.empty_i64(nplanes, rows, wpr)
        wpr = planes.shape[-1] if planes is not None else wpr
        res = []
        for on, coder, slot, out, b in ((golomb, CODER_GOLOMB, slots[0], outs[0], bits[0]),
                                        (eg, CODER_EG, slots[1], outs[1], bits[1])):
            if not on:
                res.append((None, 0, None))
                continue
            slot = slot or self.slot_words(rows, cols, coder)
            out = self.empty_i64(nplanes, slot) if out is None else out
            b = self.empty_i64(nplanes) if b is None else b
            res.append((out, slot, b))
        (og, sg, bg), (oe, se, be) = res
        self._bind_stream()
        if plane0:
            self._chk(self.lib.bic_encode_gray_range(self.h, _p(gray), pitch, rows, cols, plane0, nplanes, _p(planes),
                                                     wpr, int(predict), _p(og), sg, _p(bg), _p(oe), se, _p(be)),
                      "bic_encode_gray_range")
        else:
            self._chk(self.lib.bic_encode_gray(self.h, _p(gray), pitch, rows, cols, nplanes, _p(planes), wpr,
                                               int(predict), _p(og), sg, _p(bg), _p(oe), se, _p(be)), "bic_encode_gray")
        return planes, ((og, bg) if golomb else None), ((oe, be) if eg else None)

    def encode_planes_packed(self, planes, cols, predict=True, golomb=True, eg=False, slots=(None, None),
                             outs=(None, None), bits=(None, None), offs=(None, None), row_index=None):
        """-> ((out_g, bits_g, off_g) or None, (out_e, bits_e, off_e) or None): each coder's streams
        packed word-aligned in plane order, off = start words + total (bic_encode_planes_packed)."""
        planes = planes if planes.dim() == 3 else planes.unsqueeze(0)
        n, rows, wpr = planes.shape
        res = self._packed_bufs(n, rows, cols, golomb, eg, slots, outs, bits, offs)
        (og, sg, bg, fg), (oe, se, be, fe) = res
        self._bind_stream()
        self._chk(self.lib.bic_encode_planes_packed(self.h, _p(planes), n, rows, cols, wpr, int(predict), _p(og), sg,
                                                    _p(bg), _p(fg), _p(oe), se, _p(be), _p(fe), _p(row_index)),
                  "bic_encode_planes_packed")
        return ((og, bg, fg) if golomb else None), ((oe, be, fe) if eg else None)

    def encode_gray_packed(self, gray, cols=None, nplanes=8, plane0=0, predict=True, planes=None, golomb=True,
                           eg=True, slots=(None, None), outs=(None, None), bits=(None, None), offs=(None, None),
                           row_index=None, store_planes=True):
        """bic_encode_gray_packed -> (planes, (out_g, bits_g, off_g) or None, (out_e, bits_e, off_e) or None)
        (store_planes=False: planes NULL, returned as None)"""
        rows, pitch = gray.shape
        cols = pitch if cols is None else cols
        if planes is None and store_planes:
            planes = self.empty_i64(nplanes, rows, (cols + 63) // 64)
        wpr = planes.shape[-1] if planes is not None else (cols + 63) // 64
        (og, sg, bg, fg), (oe, se, be, fe) = self._packed_bufs(nplanes, rows, cols, golomb, eg, slots, outs, bits, offs)
        self._bind_stream()
        self._chk(self.lib.bic_encode_gray_packed(self.h, _p(gray), pitch, rows, cols, plane0, nplanes, _p(planes), wpr,
                                                  int(predict), _p(og), sg, _p(bg), _p(fg), _p(oe), se, _p(be),
                                                  _p(fe), _p(row_index)), "bic_encode_gray_packed")
        return planes, ((og, bg, fg) if golomb else None), ((oe, be, fe) if eg else None)

    def row_index(self, planes, cols, predict=True, out=None):
        """bic_row_index: int64 [nplanes * rows * 2] (per row: Golomb bit offset, residual 1s before)"""
        planes = planes if planes.dim() == 3 else planes.unsqueeze(0)
        n, rows, wpr = planes.shape
        out = self.empty_i64(n * rows * 2) if out is None else out
        self._bind_stream()
        self._chk(self.lib.bic_row_index(self.h, _p(planes), n, rows, cols, wpr, int(predict), _p(out)), "bic_row_index")
        return out

    def egad_row_index(self, planes, cols, predict=True, out=None):
        """bic_egad_row_index: int64 [nplanes * rows * 2] (per row: bit offset in the adaptive EG stream,
        the coder state there)"""
        planes = planes if planes.dim() == 3 else planes.unsqueeze(0)
        n, rows, wpr = planes.shape
        out = self.empty_i64(n * rows * 2) if out is None else out
        self._bind_stream()
        self._chk(self.lib.bic_egad_row_index(self.h, _p(planes), n, rows, cols, wpr, int(predict), _p(out)),
                  "bic_egad_row_index")
        return out

    def decode_planes(self, coder, streams, plane_bits, nplanes, rows, cols, predict=True, word_off=None,
                      row_index=None, p00=None, out=None, wpr=None):
        """bic_decode_planes: streams int64 [nplanes, slot] (slots) or [words] with word_off (packed)
        -> planes int64 [nplanes, rows, wpr]. p00: uint8 device tensor [nplanes] or None."""
        wpr = wpr or (cols + 63) // 64
        out = self.empty_i64(nplanes, rows, wpr) if out is None else out
        slot = streams.shape[-1] if (word_off is None and streams.dim() == 2) else 0
        self._bind_stream()
        self._chk(self.lib.bic_decode_planes(self.h, coder, _p(streams), slot, _p(word_off), _p(plane_bits),
                                             _p(row_index), nplanes, rows, cols, wpr, int(predict), _p(p00), _p(out)),
                  "bic_decode_planes")
        return out

    def _packed_bufs(self, n, rows, cols, golomb, eg, slots, outs, bits, offs):
        res = []
        for i, (on, coder) in enumerate(((golomb, CODER_GOLOMB), (eg, CODER_EG))):
            if not on:
                res.append((None, 0, None, None))
                continue
            slot = slots[i] or self.slot_words(rows, cols, coder)
            res.append((self.empty_i64(n * slot) if outs[i] is None else outs[i], slot,
                        self.empty_i64(n) if bits[i] is None else bits[i],
                        self.empty_i64(n + 1) if offs[i] is None else offs[i]))
        return res

    def set_encoder(self, name):
        """row encoder for rows <= 16384 columns: "auto" (default: staged from 32768 rows on, the
        single kernel below), "staged" (forced), "single-kernel", "two-pass", "multipass"
        (bic_ctx_set_option)"""
        assert name in ("auto", "staged", "single-kernel", "two-pass", "multipass"), name
        self.set_multipass(name == "multipass")
        self._chk(self.lib.bic_ctx_set_option(self.h, 4, int(name == "staged")), "bic_ctx_set_option")
        self._chk(self.lib.bic_ctx_set_option(self.h, 2, int(name == "two-pass")), "bic_ctx_set_option")
        self._chk(self.lib.bic_ctx_set_option(self.h, 3, int(name == "single-kernel")), "bic_ctx_set_option")

    def set_one_stream(self, on=True):
        """the staged encoder's two emission launches one after the other on the ctx stream
        (BIC_OPT_ONE_STREAM) instead of side by side on a second stream"""
        self._chk(self.lib.bic_ctx_set_option(self.h, 5, int(on)), "bic_ctx_set_option")

    def set_eg_source(self, on=True):
        """bic_encode_gray* without planes: the count pass writes the EG stream and the Golomb kernels
        read the residual rows back from it (BIC_OPT_EG_SOURCE, default on) -- off: the residual
        planes in a context buffer; 2: the EG source with one emission kernel for every row class"""
        self._chk(self.lib.bic_ctx_set_option(self.h, 6, int(on)), "bic_ctx_set_option")

    def set_multipass(self, on=True):
        self._chk(self.lib.bic_ctx_set_option(self.h, 1, int(on)), "bic_ctx_set_option")

    def set_two_pass(self, on=True):
        """the two-pass row encoder instead of the default staged one"""
        self._chk(self.lib.bic_ctx_set_option(self.h, 2, int(on)), "bic_ctx_set_option")

    def golomb_lengths(self, samples, n0=0, a0=0):
        """bic_golomb_encode_samples without an output: -> bits int64[2] (codeword bits, sum of samples)"""
        bits = self.empty_i64(2)
        self._bind_stream()
        self._chk(self.lib.bic_golomb_encode_samples(self.h, _p(samples), samples.numel(), n0, a0, 0, None, 0,
                                                     _p(bits)), "bic_golomb_encode_samples")
        return bits

    def golomb_encode_samples(self, samples, n0=0, a0=0, bit0=0, cap_words=None, out=None):
        """samples: int32 device tensor (uint32 values) -> (stream int64 [cap], bits int64[2])."""
        n = samples.numel()
        if cap_words is None:  # always enough: sum(s >> k) <= sum(s), k + 1 <= 32 per sample
            tot = int(samples.to(self.torch.int64).bitwise_and(0xFFFFFFFF).sum().item()) if n else 0
            cap_words = max(1, (tot + 32 * n + bit0 + 63) // 64 + 1)
        if out is None:
            out = self.empty_i64(cap_words)
        bits = self.empty_i64(2)
        self._bind_stream()
        self._chk(self.lib.bic_golomb_encode_samples(self.h, _p(samples), n, n0, a0, bit0, _p(out),
                                                     cap_words, _p(bits)), "bic_golomb_encode_samples")
        return out, bits

    def patch_encode(self, plane, cols, W, lentab, cap_words=None, want_resid=True, bufs=None):
        """plane: int64 [rows, wpr]; lentab: numpy uint64 [W*W+1] (host). bufs: the dict an earlier
        call returned, whose device buffers are written again (same shapes; no allocation)."""
        rows, wpr = plane.shape
        nt = (rows // W) * (cols // W)
        t = self.torch
        # sum of tile weights <= rows*cols, and k + 1 <= 32 per tile: always enough
        cap_words = cap_words or max(1, (rows * cols + 32 * nt + 63) // 64 + 1)
        if bufs is not None and bufs["weights"].numel() == nt and bufs["stream"].numel() >= cap_words and \
                (bufs["resid"] is not None) == bool(want_resid):
            weights, wo, wO, modes = bufs["weights"], bufs["w_nonpred"], bufs["w_pred"], bufs["modes"]
            resid, stream, stats = bufs["resid"], bufs["stream"], bufs["stats"]
            cap_words = stream.numel()
        else:
            weights = t.empty(nt, dtype=t.int32, device=self.dev)
            wo = t.empty(nt, dtype=t.int32, device=self.dev)
            wO = t.empty(nt, dtype=t.int32, device=self.dev)
            modes = t.empty(nt, dtype=t.uint8, device=self.dev)
            resid = self.empty_i64(rows, wpr) if want_resid else None
            stream = self.empty_i64(cap_words)
            stats = self.empty_i64(3)
        lt = lentab if isinstance(lentab, np.ndarray) and lentab.dtype == np.uint64 and lentab.flags.c_contiguous \
            else np.ascontiguousarray(lentab, np.uint64)
        self._bind_stream()
        self._chk(self.lib.bic_patch_encode(self.h, _p(plane), rows, cols, wpr, W, lt.ctypes.data_as(C.c_void_p),
                                            _p(weights), _p(wo), _p(wO), _p(modes), _p(resid), _p(stream),
                                            cap_words, _p(stats)), "bic_patch_encode")
        return dict(weights=weights, w_nonpred=wo, w_pred=wO, modes=modes, resid=resid, stream=stream,
                    stats=stats)

    def patch_search(self, plane, cols, W):
        """compress_test.cpp's patch search -> (besti, bestj, bestd) int32 device tensors per tile."""
        rows, wpr = plane.shape
        n = ((rows + W - 1) // W) * ((cols + W - 1) // W)
        t = self.torch
        out = [t.empty(n, dtype=t.int32, device=self.dev) for _ in range(3)]
        self._bind_stream()
        self._chk(self.lib.bic_patch_search(self.h, _p(plane), rows, cols, wpr, W, *(_p(o) for o in out)),
                  "bic_patch_search")
        return tuple(out)

    def match_encode(self, plane, cols, W, T=0, R=128, enuml=None, cap_words=None, resid=None, invert=False,
                     variant=7):
        """compress7_test.cpp's tile loop with search window R and threshold T (bic_match_encode);
        invert: compress8_test.cpp's patch-inversion variant (bic_match_encode_inv, `inverted` per tile);
        variant 4 / 5 / 6: the loops of compress4/5/6_test.cpp (bic_match_encode_var).
        plane: int64 [rows, wpr] device tensor (not modified); enuml: numpy float64 [W*W+1] (host),
        default enumL from this build. Returns device tensors per tile and the two streams."""
        rows, wpr = plane.shape
        nt = (rows // W) * (cols // W)
        t = self.torch
        bi, bj, bd, wt = (t.empty(nt, dtype=t.int32, device=self.dev) for _ in range(4))
        modes = t.empty(nt, dtype=t.uint8, device=self.dev)
        resid = self.empty_i64(rows, wpr) if resid is None else resid
        cap_words = cap_words or max(1, (rows * cols + 33 * nt + 63) // 64 + 1)
        sm, sn = self.empty_i64(cap_words), self.empty_i64(cap_words)
        stats = self.empty_i64(4)
        e = enum_table(W) if enuml is None else np.ascontiguousarray(enuml, np.float64)
        inv = t.empty(nt, dtype=t.uint8, device=self.dev) if invert else None
        self._bind_stream()
        if variant in (4, 5, 6):
            self._chk(self.lib.bic_match_encode_var(self.h, variant, _p(plane), rows, cols, wpr, W, T, R,
                                                    e.ctypes.data_as(C.c_void_p), _p(bi), _p(bj), _p(bd), _p(wt),
                                                    _p(modes), _p(resid), _p(sm), _p(sn), cap_words, _p(stats)),
                      "bic_match_encode_var")
        elif invert:
            self._chk(self.lib.bic_match_encode_inv(self.h, _p(plane), rows, cols, wpr, W, T, R,
                                                    e.ctypes.data_as(C.c_void_p), _p(bi), _p(bj), _p(bd), _p(wt),
                                                    _p(modes), _p(inv), _p(resid), _p(sm), _p(sn), cap_words,
                                                    _p(stats)), "bic_match_encode_inv")
        else:
            self._chk(self.lib.bic_match_encode(self.h, _p(plane), rows, cols, wpr, W, T, R,
                                                e.ctypes.data_as(C.c_void_p), _p(bi), _p(bj), _p(bd), _p(wt),
                                                _p(modes), _p(resid), _p(sm), _p(sn), cap_words, _p(stats)),
                      "bic_match_encode")
        return dict(besti=bi, bestj=bj, bestd=bd, weights=wt, modes=modes, resid=resid, stream_match=sm,
                    stream_nomatch=sn, stats=stats, inverted=inv)

    def set_match_parts(self, parts):
        self._chk(self.lib.bic_set_match_parts(self.h, parts), "bic_set_match_parts")

    def pgm_bitplanes(self, raster, rows, cols, maxval, nplanes, plane0=0, wpr=None, out=None):
        """P5 samples (uint8 device tensor view starting at the first sample, any alignment) -> planes"""
        wpr = wpr or (cols + 63) // 64
        out = self.empty_i64(nplanes, rows, wpr) if out is None else out
        self._bind_stream()
        self._chk(self.lib.bic_pgm_bitplanes(self.h, _p(raster), rows, cols, maxval, plane0, nplanes, _p(out), wpr),
                  "bic_pgm_bitplanes")
        return out

    def planes_to_gray(self, planes, cols, plane0=0, sample_bytes=1, out=None, pitch=None):
        """bic_planes_to_gray: planes int64 [n, rows, wpr] -> uint8 device tensor [rows, pitch] of samples
        (sample_bytes 2: big-endian 16-bit, as a P5 raster with maxval >= 256)"""
        planes = planes if planes.dim() == 3 else planes.unsqueeze(0)
        n, rows, wpr = planes.shape
        pitch = pitch or cols * sample_bytes
        out = self.torch.zeros(rows, pitch, dtype=self.torch.uint8, device=self.dev) if out is None else out
        self._bind_stream()
        self._chk(self.lib.bic_planes_to_gray(self.h, _p(planes), plane0, n, rows, cols, wpr, sample_bytes, _p(out),
                                              pitch), "bic_planes_to_gray")
        return out

    def pbm_unpack(self, raster, rows, cols, wpr=None):
        """P4 raster bytes (uint8 device tensor, rows x ceil(cols/8)) -> int64 plane [rows, wpr]."""
        wpr = wpr or (cols + 63) // 64
        plane = self.empty_i64(rows, wpr)
        self._bind_stream()
        self._chk(self.lib.bic_pbm_unpack(self.h, _p(raster), rows, cols, _p(plane), wpr), "bic_pbm_unpack")
        return plane

    def pbm_pack(self, plane, cols, out=None):
        """int64 plane [rows, wpr] -> P4 raster bytes (uint8 device tensor; `out`: any alignment)."""
        rows, wpr = plane.shape
        raster = self.torch.empty(rows * ((cols + 7) // 8), dtype=self.torch.uint8, device=self.dev) if out is None else out
        self._bind_stream()
        self._chk(self.lib.bic_pbm_pack(self.h, _p(plane), rows, cols, wpr, _p(raster)), "bic_pbm_pack")
        return raster

    def gf2_transpose(self, M, cols, out=None):
        """int64 matrix [rows, wpr] of `cols` bits -> its transpose [cols, ceil(rows/64)] (or `out`)."""
        rows, wpr = M.shape
        out = self.empty_i64(cols, (rows + 63) // 64) if out is None else out
        self._bind_stream()
        self._chk(self.lib.bic_gf2_transpose(self.h, _p(M), rows, cols, wpr, _p(out), out.shape[1]),
                  "bic_gf2_transpose")
        return out

    def gf2_mul(self, op, A, a_cols, B, b_cols, C, c_cols):
        """mul(A, At, B, Bt, C) over GF(2) in place on C (int64 [rows, wpr] device tensors)."""
        self._bind_stream()
        self._chk(self.lib.bic_gf2_mul(self.h, op, _p(A), A.shape[0], a_cols, A.shape[1], _p(B), B.shape[0], b_cols,
                                       B.shape[1], _p(C), C.shape[0], c_cols, C.shape[1]), "bic_gf2_mul")
        return C

    def pack_streams(self, slots, plane_bits, dst_words=None):
        n, slot_words = slots.shape
        dst = self.empty_i64(dst_words or n * slot_words)
        off = self.empty_i64(n + 1)
        self._bind_stream()
        self._chk(self.lib.bic_pack_streams(self.h, _p(slots), n, slot_words, _p(plane_bits), _p(dst), _p(off)),
                  "bic_pack_streams")
        return dst, off


def pnm_header(data):
    """bic_pnm_parse_header on host bytes -> PnmInfo (raises BicError on a malformed header)"""
    info = PnmInfo()
    rc = load().bic_pnm_parse_header(bytes(data), len(data), C.byref(info))
    if rc != BIC_OK:
        raise BicError(rc, "bic_pnm_parse_header")
    return info


def enum_codelength(n, r):
    """log2 C(n, r) (coding.h enumerative_codelength), host-side, from libbic.so."""
    return float(load().bic_enum_codelength(n, r))


def enum_table(W):
    """enumL(W*W, w) for w = 0..W*W (float64), the table bic_match_encode takes."""
    f = load().bic_enum_codelength
    return np.array([f(W * W, w) for w in range(W * W + 1)], np.float64)


def lentab(W):
    """tile length table for bic_patch_encode: (uint64)(2 + log2 C(W*W, w)), w = 0..W*W."""
    out = np.zeros(W * W + 1, np.uint64)
    rc = load().bic_tile_lentab(W, out.ctypes.data_as(C.c_void_p))
    if rc != BIC_OK:
        raise BicError(rc, "bic_tile_lentab")
    return out


def sources_hash():
    """sha256 of the HIP/C++ sources libbic.so is built from (csrc/*): PMC summaries under profiles/
    carry the hash of the sources they profiled, so bench.py can tell whether they describe the
    kernels it is running."""
    import hashlib
    h = hashlib.sha256()
    d = os.path.join(PKG, "csrc")
    for name in sorted(os.listdir(d)):
        if name.endswith((".hip", ".cpp", ".h")):
            h.update(name.encode())
            with open(os.path.join(d, name), "rb") as f:
                h.update(f.read())
    return h.hexdigest()


def device_count():
    n = C.c_int(0)
    load().bic_device_count(C.byref(n))
    return n.value
