"""The C++ reference API (include/*.h, libbicpp.so) through tests/cpp/host_api_check.cpp:
coder known answers, stream decoders against the oracle's streams, the inverse predictor, and
(GPU) the bitplane / med / encode / tile bridge against the reference-API coders and the oracle."""
import os
import subprocess

import numpy as np
import pytest

from conftest import PKG, ROOT
from pnm_io import read_pbm_bytes, write_pbm, write_pgm

SRC = os.path.join(ROOT, "tests", "cpp", "host_api_check.cpp")
EXE = os.path.join(PKG, "build", "host_api_check")


@pytest.fixture(scope="module")
def exe():
    lib = os.path.join(PKG, "lib", "libbicpp.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", PKG], check=True, stdout=subprocess.DEVNULL)
    if not os.path.exists(EXE) or os.path.getmtime(EXE) < max(os.path.getmtime(SRC), os.path.getmtime(lib)):
        os.makedirs(os.path.dirname(EXE), exist_ok=True)
        subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-o", EXE, SRC,
                        "-L", os.path.join(PKG, "lib"), "-lbicpp", "-lbic",
                        "-Wl,-rpath," + os.path.join(PKG, "lib")], check=True)
    return EXE


def run(exe, *args, timeout=300):
    p = subprocess.run([exe] + [str(a) for a in args], capture_output=True, text=True, timeout=timeout)
    return p.returncode, p.stdout + p.stderr


def test_coder_known_answers(exe):
    rc, out = run(exe, "kat")
    assert rc == 0, out


@pytest.mark.parametrize("rows,cols,p", [(1, 1, 0.5), (5, 64, 0.5), (17, 100, 0.1), (40, 333, 0.02),
                                         (64, 1024, 0.5), (9, 130, 0.0), (7, 65, 1.0)])
@pytest.mark.parametrize("predict", [0, 1])
def test_decoders_read_oracle_streams(exe, oracle, tmp_path, rows, cols, p, predict):
    """oracle stream -> C++ decoder -> the residual the oracle coded (Golomb, EG as written, EG adaptive)"""
    P = oracle.gen_plane(7 * rows + cols, p, rows, cols)
    R = oracle.med(P, cols) if predict else P
    for coder in (0, 1, 2):
        bits, stream, _ = oracle.encode_plane(P, cols, predict, coder)
        sp = tmp_path / f"s{coder}.bin"
        sp.write_bytes(stream.tobytes())
        op = tmp_path / f"d{coder}.pbm"
        rc, out = run(exe, "decode", coder, rows, cols, bits, sp, op)
        assert rc == 0, out
        r, c, D = read_pbm_bytes(op.read_bytes())
        assert (r, c) == (rows, cols)
        assert np.array_equal(D, R), (coder, predict)
        # a truncated stream is rejected
        if bits > 1:
            rc, _ = run(exe, "decode", coder, rows, cols, bits - 1, sp, op)
            assert rc != 0


@pytest.mark.parametrize("rows,cols", [(1, 70), (33, 64), (20, 129), (64, 1000)])
def test_unmed_inverts_med(exe, oracle, tmp_path, rows, cols):
    P = oracle.gen_plane(rows + 3 * cols, 0.3, rows, cols)
    R = oracle.med(P, cols)
    write_pbm(str(tmp_path / "r.pbm"), R, cols)
    p00 = int(P[0, 0] >> np.uint64(63))
    rc, out = run(exe, "unmed", tmp_path / "r.pbm", p00, tmp_path / "p.pbm")
    assert rc == 0, out
    _, _, Q = read_pbm_bytes((tmp_path / "p.pbm").read_bytes())
    assert np.array_equal(Q, P)


@pytest.mark.gpu
@pytest.mark.parametrize("shape,maxval", [((48, 40), 255), ((64, 128), 255), ((37, 200), 1023), ((1, 1), 255),
                                          ((256, 640), 200)])
def test_gpu_bridge(exe, oracle, tmp_path, shape, maxval):
    """bic::Device and med() on the GPU: self-checked in C++ against the per-pixel bitplane loop, the
    reference-API coders and the decoders; the streams it wrote are compared with the oracle here."""
    rows, cols = shape
    rng = np.random.default_rng(rows * cols + maxval)
    gray = rng.integers(0, maxval + 1, shape, dtype=np.uint16)
    write_pgm(str(tmp_path / "in.pgm"), gray, maxval)
    out = tmp_path / "out"
    out.mkdir()
    rc, log = run(exe, "gpu", tmp_path / "in.pgm", out)
    assert rc == 0, log
    nplanes = int(np.ceil(np.log2(maxval))) if maxval > 1 else 0
    planes = oracle.bitplanes(gray, nplanes)
    for p in range(nplanes):
        _, _, W = read_pbm_bytes((out / f"plane_{p:02d}.pbm").read_bytes())
        assert np.array_equal(W, planes[p]), p
        for predict in (0, 1):
            for c, tag in ((0, "g"), (1, "e")):
                bits, stream, _ = oracle.encode_plane(planes[p], cols, predict, c)
                got = (out / f"stream_{tag}{predict}_{p:02d}.bin").read_bytes()
                assert got == stream.tobytes()[: (bits + 7) // 8], (p, predict, c)


REFERENCE_API = [
    "binary_matrix::binary_matrix(unsigned long, unsigned long)", "binary_matrix::weight() const",
    "binary_matrix::get_submatrix(unsigned long, unsigned long, unsigned long, unsigned long) const",
    "binary_matrix::set_submatrix(unsigned long, unsigned long, binary_matrix const&)",
    "binary_matrix::copy_submatrix_to(unsigned long, unsigned long, unsigned long, unsigned long, binary_matrix&) const",
    "binary_matrix::get_vectorized() const", "binary_matrix::set_vectorized(binary_matrix const&)",
    "binary_matrix::get_copy() const", "binary_matrix::operator=(binary_matrix const&)",
    "binary_matrix::add_rows(unsigned long)", "binary_matrix::remove_rows(unsigned long)",
    "add(binary_matrix const&, binary_matrix const&, binary_matrix&)",
    "bool_and(binary_matrix const&, binary_matrix const&, binary_matrix&)",
    "mul(binary_matrix const&, bool, binary_matrix const&, bool, binary_matrix&)",
    "dist(binary_matrix const&, binary_matrix const&)", "operator<<(std::ostream&, binary_matrix const&)",
    "set_grid_width(unsigned long)", "med(binary_matrix const&, binary_matrix&)",
    "read_pbm_header(_IO_FILE*, unsigned long&, unsigned long&)", "read_pbm_data(_IO_FILE*, binary_matrix&)",
    "write_pbm(binary_matrix&, _IO_FILE*)", "write_pbm(binary_matrix&, char const*)",
    "read_pnm_header(_IO_FILE*, int&, int&, int&, int&)", "read_pgm_data(_IO_FILE*, int, int, int, int, unsigned int*)",
    "write_pgm(unsigned int const*, int, int, int, int, char const*)",
    "write_ppm(unsigned int const*, int, int, int, int, char const*)",
    "read_ppm_data(_IO_FILE*, int, int, int, int, unsigned int*)",
    "write_ppm_header(int, int, int, int, _IO_FILE*)", "write_p2_data(unsigned int const*, int, int, _IO_FILE*)",
    "write_p5_data(unsigned int const*, int, int, _IO_FILE*)",
    "render_mosaic(binary_matrix const&, char const*)", "counting_sort(std::pair<unsigned long, unsigned long>*, unsigned long)",
    "enumerative_codelength(unsigned int, unsigned int)", "universal_codelength(unsigned int, unsigned int)",
    "GolombCoder::codeSample(unsigned int)", "EGCoder::codeRun(int, bool)", "EG::incBlockSize()", "EG::decBlockSize()",
]


def test_library_exports_reference_api():
    """libbicpp.so defines every function of the reference headers (binmat.h, pbm.h, pnm.h, util.h,
    coding.h, GolombCoder.h, eg.h) plus med (pred.cpp)"""
    lib = os.path.join(PKG, "lib", "libbicpp.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", PKG], check=True, stdout=subprocess.DEVNULL)
    syms = subprocess.run(["nm", "-DC", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    defined = {line.split(" ", 2)[2] for line in syms.splitlines() if line.count(" ") >= 2}
    missing = [s for s in REFERENCE_API if s not in defined]
    assert not missing, missing


@pytest.mark.gpu
def test_med_call_pattern(exe):
    """compress7_test.cpp:205-206's pattern through the drop-in med(): 65,536 separate 32x32 calls (one
    8192^2 plane's tiles), each a device round trip; the time per call goes to INTEGRATION.md"""
    rc, out = run(exe, "medcalls", 65536, 32, timeout=600)
    assert rc == 0, out
    print(out.strip())
    from oracle_lib import REF_SO, have_ref
    if have_ref():  # the reference's own med, same pattern, on this host (tile fill included)
        import ctypes as C
        f = C.CDLL(REF_SO).ref_med_calls
        f.restype = C.c_double
        f.argtypes = [C.c_int, C.c_int]
        print(f"reference med (oracle/_ref) us_per_call={f(65536, 32) * 1e6:.2f}")
