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


@pytest.mark.parametrize("encoder", ["auto", "staged", "single-kernel", "two-pass"])
def test_prof_rows_timing_every_encoder(ctx, encoder):
    """the emission's kernel timing (bic_capi.cpp timed_rows) on every row encoder: the single and
    two-pass encoders have no separate main kernel, and their end event must still be recorded --
    an event left unrecorded fails the elapsed-time query, and that HIP error used to stay pending and
    fail the NEXT call (bench.py --gpus 2 --shard planes: bic error 3)"""
    t = ctx.torch
    g = t.Generator(device=ctx.dev)
    g.manual_seed(7)
    planes = t.randint(-2**62, 2**62, (2, 96, 64), dtype=t.int64, device=ctx.dev, generator=g)
    ctx.sync()
    ctx.prof_collect()
    ref, ref_bits = ctx.encode_planes(planes, 4096)
    ctx.sync()
    ref, ref_bits = ref.clone(), ref_bits.clone()
    ctx.set_encoder(encoder)
    ctx.prof_enable(True)
    try:
        ctx.prof_only(None)
        out, bits = ctx.encode_planes(planes, 4096)
        got = ctx.prof_collect()
        rows = [k for k in got if k.startswith("encode_rows")]
        assert rows and all(got[k][1] >= 0 for k in rows), got
        out2, bits2 = ctx.encode_planes(planes, 4096)  # the next call must not inherit an error
        ctx.sync()
        assert t.equal(bits, ref_bits) and t.equal(bits2, ref_bits)
        for p in range(2):
            nw = (int(ref_bits[p]) + 63) // 64
            assert t.equal(out[p, :nw], ref[p, :nw]) and t.equal(out2[p, :nw], ref[p, :nw])
    finally:
        ctx.prof_only(None)
        ctx.prof_enable(False)
        ctx.set_encoder("auto")
