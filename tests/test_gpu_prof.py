"""Kernel timing API (include/bic.h bic_prof_enable / bic_prof_only / bic_prof_collect): what
bench.py's roofline timing relies on."""
import pytest

pytestmark = pytest.mark.gpu


def test_prof_only_brackets_named_launches(ctx):
    t = ctx.torch
    gray = t.randint(0, 256, (64, 200), dtype=t.uint8, device=ctx.dev)
    ctx.sync()
    ctx.prof_collect()  # drop anything earlier tests left
    ctx.prof_enable(True)
    try:
        ctx.prof_only(None)
        ctx.bitplanes_u8(gray, nplanes=8)
        ctx.bitplanes_u8(gray, nplanes=8)
        allp = ctx.prof_collect()
        assert allp["bitplanes_u8"][0] == 2 and allp["bitplanes_u8"][1] >= 0
        ctx.prof_only("no_such_kernel")
        ctx.bitplanes_u8(gray, nplanes=8)
        assert ctx.prof_collect() == {}
        ctx.prof_only("bitplanes_u8")
        ctx.bitplanes_u8(gray, nplanes=8)
        assert ctx.prof_collect()["bitplanes_u8"][0] == 1
    finally:
        ctx.prof_only(None)
        ctx.prof_enable(False)
