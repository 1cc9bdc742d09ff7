"""One rank of torch.distributed over backend "nccl" (RCCL) at world size 1, on the one GPU of the test box
(tests/test_gpu_gather_nccl.py): the overlapped gather pybic.parallel.ChunkedGather on its DEVICE path --
the communication stream, the per-chunk events recorded on the compute stream, comm.wait_event and the
final wait_stream -- which gloo (host tensors, no streams) never takes. Two jobs, each as bench.py runs it
at N > 1:
* c4: frames encoded in chunks with bic_encode_planes_packed, each chunk's packed Golomb streams added
  right after its encode is enqueued;
* c3planes: one gray image's planes encoded in chunks with bic_encode_gray_packed (the EG source path,
  planes not stored), both coders' packed streams through two gathers.
Rank 0's gathered words are checked against the oracle, word for word. Prints "OK <job>" per job."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import pybic  # noqa: E402
from oracle_lib import Oracle  # noqa: E402
from pybic.parallel import ChunkedGather, plan_chunks  # noqa: E402


def packed_expect(o, planes, cols, coder):
    """the oracle's streams of planes, word-aligned back to back (bic_pack_streams' layout)"""
    words = []
    for P in planes:
        nb, st, _ = o.encode_plane(P, cols, 1, coder)
        w = np.zeros((nb + 63) // 64, np.uint64)
        b = np.frombuffer(st.tobytes(), np.uint8)[: len(w) * 8]
        w.view(np.uint8)[: len(b)] = b
        words.append(w)  # (memory order: the slots' words are big-endian, their bytes are the stream)
    return np.concatenate(words) if words else np.zeros(0, np.uint64)


def check(got, offs, exp, what):
    g = pybic.as_u64(got.cpu())
    assert offs == [0, len(exp)], (what, offs, len(exp))
    assert np.array_equal(g[: len(exp)], exp), (what, int(np.nonzero(g[: len(exp)] != exp)[0][0]))


def job_c4(ctx, o):
    rows, cols, nf = 256, 4096, 6
    rng = np.random.default_rng(404)
    frames = rng.integers(0, 2 ** 63, size=(nf, rows, cols // 64), dtype=np.uint64)
    frames |= rng.integers(0, 2, size=frames.shape, dtype=np.uint64) << np.uint64(63)
    planes = ctx.to_dev(frames)
    slot = ctx.slot_words(rows, cols, pybic.CODER_GOLOMB)
    packed = ctx.empty_i64(nf * slot)
    bits = ctx.torch.zeros(nf, dtype=torch.int64, device=ctx.dev)
    chunks = plan_chunks(nf, nf, 1, 3)
    offs = [ctx.torch.zeros(b - a + 1, dtype=torch.int64, device=ctx.dev) for a, b in chunks]
    cg = ChunkedGather(ctx.dev, 1, 0)
    assert cg.comm is not None, "the device path (comm stream) is what this test is for"
    for (a, b), off in zip(chunks, offs):
        region = packed[a * slot:b * slot]
        ctx.encode_planes_packed(planes[a:b], cols, True, golomb=True, eg=False, slots=(slot, None),
                                 outs=(region, None), bits=(bits[a:b], None), offs=(off, None))
        cg.add(region, off[-1:])
    out, goffs = cg.finish()
    torch.cuda.synchronize()
    ctx.sync()
    check(out, goffs, packed_expect(o, frames, cols, 0), "c4")


def job_c3planes(ctx, o):
    rows, cols = 192, 8192
    ctx.set_encoder("staged")  # the C3 step's encoder (the EG source: planes not stored)
    gray = o.gen_bytes(0xC3, rows * cols).reshape(rows, cols)
    P = o.bitplanes(gray, 8)
    g = ctx.torch.from_numpy(gray).to(ctx.dev)
    sg, se = ctx.slot_words(rows, cols, pybic.CODER_GOLOMB), ctx.slot_words(rows, cols, pybic.CODER_EG)
    out_g, out_e = ctx.empty_i64(8 * sg), ctx.empty_i64(8 * se)
    bg, be = (ctx.torch.zeros(8, dtype=torch.int64, device=ctx.dev) for _ in range(2))
    chunks = plan_chunks(8, 8, 1, 8)  # one chunk per plane, as bench.py c3 --shard planes
    cgs = (ChunkedGather(ctx.dev, 1, 0), ChunkedGather(ctx.dev, 1, 0))
    for a, b in chunks:
        fg = ctx.torch.zeros(b - a + 1, dtype=torch.int64, device=ctx.dev)
        fe = ctx.torch.zeros(b - a + 1, dtype=torch.int64, device=ctx.dev)
        rg, re = out_g[a * sg:b * sg], out_e[a * se:b * se]
        ctx.encode_gray_packed(g, nplanes=b - a, plane0=a, planes=None, slots=(sg, se), outs=(rg, re),
                               bits=(bg[a:b], be[a:b]), offs=(fg, fe), store_planes=False)
        cgs[0].add(rg, fg[-1:])
        cgs[1].add(re, fe[-1:])
    (og, offg), (oe, offe) = cgs[0].finish(), cgs[1].finish()
    torch.cuda.synchronize()
    ctx.sync()
    check(og, offg, packed_expect(o, P, cols, 0), "c3planes golomb")
    check(oe, offe, packed_expect(o, P, cols, 1), "c3planes eg")
    ctx.set_encoder("auto")


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        ctx = pybic.Context(0)
        o = Oracle()
        for name in sys.argv[1:]:
            {"c4": job_c4, "c3planes": job_c3planes}[name](ctx, o)
            print("OK", name, flush=True)
        ctx.close()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
