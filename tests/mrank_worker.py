"""One rank of the multi-rank GPU test (tests/test_gpu_multirank.py): several processes share the
one GPU of the box, talk over gloo (host tensors; RCCL needs one GPU per rank), and run the real
sharded chains through libbic.so -- the same code bench.py runs at N GPUs over RCCL:

  frames  C4: frames split over the ranks -> med + Golomb, written packed by the encoder
          (bic_encode_planes_packed; odd ranks: slots + bic_pack_streams) -> gather_streams to rank 0
  planes  C3: the 8 planes of one gray image split over the ranks -> bic_encode_gray_packed (planes
          plane0.., Golomb and EG written packed) -> gather_streams
  tiles   C5: bands of tile rows -> bic_patch_encode per band -> one adaptive Golomb coder over the
          whole tile sequence continued across ranks (sharded_golomb + bic_golomb_encode_samples)

Rank 0 compares what it received with the oracle over the whole input and exits non-zero on any
difference. Env: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT (set by the test)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binary-image-compression_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import pybic  # noqa: E402
from pybic import CODER_EG, CODER_GOLOMB, as_u64  # noqa: E402
from pybic.parallel import gather_streams, sharded_golomb  # noqa: E402


def share(n, world, rank):
    return rank * n // world, (rank + 1) * n // world


def gray_image(oracle, rows, cols):
    i = np.arange(rows, dtype=np.int64)[:, None]
    j = np.arange(cols, dtype=np.int64)[None, :]
    noise = oracle.gen_bytes(0x5EED, rows * cols).reshape(rows, cols) % 7
    return ((i * 3 + j // 5 + noise) % 256).astype(np.uint8)


def split_packed(words, bits):
    """a rank's packed buffer (bic_pack_streams: streams word-aligned, back to back) -> per-plane bytes"""
    out, o = [], 0
    for b in bits:
        nw = (int(b) + 63) // 64
        out.append(words[o:o + nw].tobytes())
        o += nw
    return out, o


def gather_bits(bits, n_total, world, rank):
    """every rank's per-plane bit counts, in rank order (all_gather of a padded host tensor)"""
    t = torch.zeros(n_total, dtype=torch.int64)
    t[:bits.numel()] = bits.cpu()
    outs = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    return [o.numpy().view(np.uint64) for o in outs]


def frames(ctx, oracle, world, rank):
    F, rows, cols = 6, 130, 640
    P = np.stack([oracle.gen_plane(0x5EED0000 + k, (0.5, 0.2, 0.05)[k % 3], rows, cols) for k in range(F)])
    lo, hi = share(F, world, rank)
    if rank % 2:  # slots + bic_pack_streams on odd ranks, the encoder's packed output on even ones
        out, bits = ctx.encode_planes(ctx.to_dev(P[lo:hi]), cols, True, CODER_GOLOMB)
        packed, off = ctx.pack_streams(out, bits)
    else:
        (packed, bits, off), _ = ctx.encode_planes_packed(ctx.to_dev(P[lo:hi]), cols, True, golomb=True, eg=False)
    allbits = gather_bits(bits, F, world, rank)
    words, offs = gather_streams(packed, off[-1:], world, rank)
    if rank:
        return True
    W = as_u64(words)
    ok = True
    k = 0
    for r in range(world):
        a, b = share(F, world, r)
        parts, nw = split_packed(W[offs[r]:offs[r + 1]], allbits[r][:b - a])
        ok &= nw == offs[r + 1] - offs[r]
        for st in parts:
            eb, est, _ = oracle.encode_plane(P[k], cols, 1, 0)
            ok &= int(allbits[r][k - a]) == eb and st == est.tobytes()
            k += 1
    return bool(ok and k == F)


def planes(ctx, oracle, world, rank):
    rows, cols = 70, 16384
    img = gray_image(oracle, rows, cols)
    g = torch.from_numpy(img).to(ctx.dev)
    lo, hi = share(8, world, rank)
    _, (og, bg, fg), (oe, be, fe) = ctx.encode_gray_packed(g, nplanes=hi - lo, plane0=lo)
    res = {}
    for coder, packed, bits, off in ((0, og, bg, fg), (1, oe, be, fe)):
        allbits = gather_bits(bits, 8, world, rank)
        words, offs = gather_streams(packed, off[-1:], world, rank)
        res[coder] = (allbits, words, offs)
    if rank:
        return True
    exp = oracle.bitplanes(img, 8)
    ok = True
    for coder in (0, 1):
        allbits, words, offs = res[coder]
        W = as_u64(words)
        k = 0
        for r in range(world):
            a, b = share(8, world, r)
            parts, _ = split_packed(W[offs[r]:offs[r + 1]], allbits[r][:b - a])
            for st in parts:
                eb, est, _ = oracle.encode_plane(exp[k], cols, 1, coder)
                ok &= int(allbits[r][k - a]) == eb and st == est.tobytes()
                k += 1
        ok &= k == 8
    return bool(ok)


def tiles(ctx, oracle, world, rank):
    rows, cols, W = 512, 1024, 32
    I = oracle.gen_plane(0x5EED0003, 0.03, rows, cols)
    lt = oracle.lentab(W)
    ny = rows // W
    lo, hi = share(ny, world, rank)
    res = ctx.patch_encode(ctx.to_dev(I[lo * W:hi * W]), cols, W, lt)
    wts = res["weights"]
    total = int(as_u64(res["stats"])[1])

    def enc(n0, a0, bit0):
        out, bits = ctx.golomb_encode_samples(wts, n0=n0, a0=a0, bit0=bit0)
        return out, int(as_u64(bits)[0])

    def lengths(n0, a0):
        return int(as_u64(ctx.golomb_lengths(wts, n0=n0, a0=a0))[0])

    merged, total_bits = sharded_golomb(enc, wts.numel(), total, ctx.dev, lengths=lengths)
    if rank:
        return True
    exp = oracle.patch_encode(I, cols, W, lt)
    return bool(total_bits == exp["bits"] and
                pybic.stream_bytes(merged, total_bits) == exp["stream"].tobytes())


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    from oracle_lib import Oracle
    oracle = Oracle()
    ctx = pybic.Context(0)
    ctx.set_encoder(os.environ.get("BIC_MR_ENCODER", "auto"))
    results = {}
    for name in sys.argv[1:] or ["frames", "planes", "tiles"]:
        results[name] = {"frames": frames, "planes": planes, "tiles": tiles}[name](ctx, oracle, world, rank)
        ctx.sync()
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()
    if rank == 0:
        print("results", results, flush=True)
    sys.exit(0 if all(results.values()) else 1)


if __name__ == "__main__":
    main()
