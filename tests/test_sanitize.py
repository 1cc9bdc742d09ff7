"""the host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only, any
report fatal). oracle/Makefile `san` builds (1) the reference's own GSL-free drivers against this
build's headers with the host library's CPU sources (host/*.cpp but the GPU bridge, med and enumL,
which need the device) and (2) the oracle + the strong-CPU encoder under a C driver
(tests/cpp/oracle_san.c). The drivers must behave exactly like the reference build on the drop-in
test's inputs, sanitized."""
import os
import shutil
import subprocess

import pytest

from test_dropin import GOLDEN, assert_same, gray_inputs, pbm_inputs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/src"
SAN_ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=99",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1:exitcode=98")


@pytest.fixture(scope="module")
def san():
    if not os.path.isdir(REF):
        pytest.skip("reference sources absent (the GPU box): nothing to build the drivers from")
    subprocess.run(["make", "-C", os.path.join(ROOT, "binary-image-compression_amd")], check=True,
                   stdout=subprocess.DEVNULL)
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "drivers", "san"], check=True,
                   stdout=subprocess.DEVNULL)
    return os.path.join(ROOT, "oracle", "_ref")


def test_oracle_sanitized(san):
    p = subprocess.run([os.path.join(san, "oracle_san")], capture_output=True, text=True, timeout=600, env=SAN_ENV)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]


def _run(san, side, tmp, name, args, setup):
    d = os.path.join(tmp, side)
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(os.path.join(d, "data"))
    setup(d)
    before = set(os.listdir(d))
    p = subprocess.run([os.path.join(san, side, name)] + args, cwd=d, capture_output=True, timeout=300, env=SAN_ENV)
    files = {}
    for root, _, names in os.walk(d):
        for n in names:
            path = os.path.join(root, n)
            rel = os.path.relpath(path, d)
            if rel not in before and not rel.startswith("data"):
                with open(path, "rb") as f:
                    files[rel] = f.read()
    assert b"runtime error" not in p.stderr and b"AddressSanitizer" not in p.stderr, p.stderr.decode()[-4000:]
    return p.returncode, p.stdout, files


def _both(san, tmp, name, args, setup):
    return {"drv_ref": _run(san, "drv_ref", tmp, name, args, setup),
            "drv_bic": _run(san, "drv_san", tmp, name, args, setup)}


@pytest.mark.parametrize("driver,args", [("binmat_test", []), ("pbm_test", []), ("patch_test", ["5"]),
                                         ("patch_test", ["32"])])
def test_drivers_sanitized(san, tmp_path, driver, args):
    for key, src in pbm_inputs(str(tmp_path)).items():
        name = "in.pbm" if driver == "patch_test" else "camera.pbm"
        a = ["data/in.pbm"] + args if driver == "patch_test" else args
        res = _both(san, str(tmp_path), driver, a, lambda d, s=src, n=name: shutil.copy(s, os.path.join(d, "data", n)))
        assert_same(res, f"{driver}/{key}")


def test_bitplane_tools_sanitized(san, tmp_path):
    for key, src in gray_inputs(str(tmp_path)).items():
        res = _both(san, str(tmp_path), "bitplane_tool", ["data/in.pgm"],
                    lambda d, s=src: shutil.copy(s, os.path.join(d, "data", "in.pgm")))
        assert_same(res, f"bitplane_tool/{key}")
        planes = res["drv_ref"][2]

        def setup(d, planes=planes):
            for n, b in planes.items():
                with open(os.path.join(d, "data", n), "wb") as f:
                    f.write(b)
        assert_same(_both(san, str(tmp_path), "plane2pgm_tool", ["data/plane_%02d.pbm", "rec.pgm"], setup),
                    f"plane2pgm_tool/{key}")
