"""bic_pnm_parse_header (host, C ABI) against the reference's header grammar (pnm.cpp:5-42,
pbm.cpp:4-27) -- and against the reference's own readers where they are built (oracle/_ref)."""
import numpy as np
import pytest

import pybic


@pytest.mark.parametrize("data,exp", [
    (b"P5\n16 9\n255\nXYZ", (5, 9, 16, 255, 12)),
    (b"P5\n# a comment\n16 9\n255\n\x00", (5, 9, 16, 255, 24)),
    (b"P2 # c1\n# c2\n3\n# c3\n2 15\n1 2 3", (2, 2, 3, 15, 25)),
    (b"P5\n300 1\n1023\n\x00\x01", (5, 1, 300, 1023, 14)),
    (b"P6\n4 4\n255\n", (6, 4, 4, 255, 11)),
    (b"P4\n64 2\n\x00\x00", (4, 2, 64, 1, 8)),
    (b"P4\n64 2\n \x0a\xff", (4, 2, 64, 1, 10)),   # " %d " eats whitespace-valued raster bytes (pbm.cpp:19)
    (b"P4 5\t7 \x01", (4, 7, 5, 1, 7)),
])
def test_headers(data, exp):
    h = pybic.pnm_header(data)
    assert (h.type, h.rows, h.cols, h.maxval, h.data_offset) == exp


def test_long_comment_line():
    # skip_comments reads a '#' line with fgets into 100 bytes: 99 at most, the rest is read as data
    data = b"P5\n#" + b"x" * 98 + b"\n12 3\n255\n"
    h = pybic.pnm_header(data)
    assert (h.cols, h.rows) == (12, 3)
    bad = b"P5\n#" + b"x" * 120 + b"\n12 3\n255\n"
    with pytest.raises(pybic.BicError):
        pybic.pnm_header(bad)


@pytest.mark.parametrize("data", [b"", b"P", b"Q5\n1 1\n255\n", b"P3\n1 1\n255\n", b"P5\n0 4\n255\n",
                                  b"P5\n4\n", b"P4\n0 5\n", b"P5\n4 4\n70000\n"])
def test_rejects(data):
    with pytest.raises(pybic.BicError):
        pybic.pnm_header(data)


def test_against_reference_readers(tmp_path):
    """the offsets, sizes and maxvals the reference's own read_pnm_header / read_pbm_header leave
    (oracle/_ref ref_pnm_header: ftell after the call), on headers with comments and odd spacing"""
    import ctypes as C
    import os
    from oracle_lib import REF_SO, have_ref
    if not have_ref():
        pytest.skip("oracle/_ref not built")
    f = C.CDLL(REF_SO).ref_pnm_header
    rng = np.random.default_rng(5)
    ws = [b" ", b"\n", b"\t", b"\r\n", b"  \n "]
    for k in range(200):
        t = int(rng.choice([2, 4, 5, 6]))
        cols, rows, mv = int(rng.integers(1, 5000)), int(rng.integers(1, 5000)), int(rng.integers(1, 65536))
        def sep():
            s = ws[rng.integers(len(ws))]
            if t != 4 and rng.random() < 0.4:
                s += b"# " + bytes(rng.integers(32, 127, int(rng.integers(0, 130))).astype(np.uint8)) + b"\n"
            return s
        hdr = b"P%d" % t + sep() + b"%d" % cols + sep() + b"%d" % rows
        if t != 4:
            hdr += sep() + b"%d" % mv
        hdr += ws[rng.integers(len(ws))][:1]  # the one whitespace byte that ends a header
        data = hdr + bytes([int(x) for x in rng.integers(0, 256, 8)])
        p = tmp_path / f"h{k}"
        p.write_bytes(data)
        ti, r, c, m, o = C.c_int(), C.c_long(), C.c_long(), C.c_int(), C.c_long()
        rc = f(str(p).encode(), C.byref(ti), C.byref(r), C.byref(c), C.byref(m), C.byref(o))
        try:
            h = pybic.pnm_header(data)
            got = (0, h.type, h.rows, h.cols, h.maxval, h.data_offset)
        except pybic.BicError:
            got = None
        if rc == 0 and c.value > 0 and r.value > 0:
            assert got == (0, ti.value, r.value, c.value, m.value, o.value), data
        else:
            assert got is None, data
