"""The C-ABI library loads and exports every entry point include/bic.h declares (CPU only:
no compute is called without a GPU), and the host-side helpers behave."""
import os
import re

import numpy as np
import pytest

import pybic

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "bic.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(bic_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_declared_symbol():
    lib = pybic.load()
    syms = header_symbols()
    assert len(syms) >= 15
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(pybic.EXPORTS) == syms


def test_no_cpu_fallback_without_device():
    n = pybic.device_count()
    if n == 0:
        with pytest.raises(pybic.BicError) as e:
            pybic.Context(0)
        assert e.value.code == pybic.BIC_ENODEV


def test_strerror_and_slot_words():
    lib = pybic.load()
    assert lib.bic_strerror(pybic.BIC_ENOSPC) == b"output slot too small"
    # EG as written: rows*(cols+1)+1 bits, exactly
    assert lib.bic_encode_slot_words(16384, 16384, pybic.CODER_EG) == (16384 * 16385 + 1 + 63) // 64
    assert lib.bic_encode_slot_words(16384, 16384, pybic.CODER_GOLOMB) >= 2 * 16384 * 16385 // 64


def test_lentab_matches_oracle(oracle):
    for W in (2, 5, 16, 32, 64):
        assert np.array_equal(pybic.lentab(W), oracle.lentab(W))


def test_enum_codelength_exact_points():
    # log2 C(1024, 1) = 10 exactly: the value GSL rounds by an ulp (parity unpinned)
    assert pybic.enum_codelength(1024, 1) == 10.0
    assert pybic.enum_codelength(1024, 1023) == 10.0
    assert pybic.enum_codelength(1024, 0) == 0.0
    assert pybic.enum_codelength(1024, 1024) == 0.0
    assert abs(pybic.enum_codelength(25, 12) - np.log2(5200300)) < 1e-9
