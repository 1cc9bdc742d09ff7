"""Multi-GPU plumbing over torch.distributed (backend "nccl" = RCCL over xGMI on ROCm; "gloo"
for CPU tests). The encode itself never exchanges data: planes/frames are independent units
(SURVEY.md §8 e). Two real exchange steps exist:

* gather_streams: the final stream concatenation -- every rank's packed stream goes to rank 0
  by direct point-to-point transfers (xGMI is point-to-point; a ring would be per-link bound).
* shard_state / shard_offsets: one adaptive Golomb coder split across ranks (the C5 tile
  sequence): each rank needs the coder state (samples, accumulated error) and the bit offset of
  everything before it -- an all-gather of two u64 per rank each.
"""
import torch
import torch.distributed as dist


def _host_only():
    """gloo (CPU tests, one-GPU rehearsals) moves host tensors only"""
    return dist.get_backend() == "gloo"


def _allgather_i64(vals, device):
    t = torch.tensor(vals, dtype=torch.int64, device="cpu" if _host_only() else device)
    outs = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(outs, t)
    return [o.tolist() for o in outs]


def gather_streams(packed, nwords, world=None, rank=None, dst=0):
    """packed: int64 tensor whose first nwords entries are this rank's stream words; nwords:
    int (or 1-element tensor). Returns (words, offsets) on `dst` -- all ranks' words back to
    back in rank order and each rank's start -- and (None, None) elsewhere."""
    world = world or dist.get_world_size()
    rank = dist.get_rank() if rank is None else rank
    n = int(nwords.reshape(-1)[0].item()) if torch.is_tensor(nwords) else int(nwords)
    sizes = [s[0] for s in _allgather_i64([n], packed.device)]
    dev = packed.device
    if _host_only():
        packed = packed.cpu()
    if rank == dst:
        offs = [0]
        for s in sizes:
            offs.append(offs[-1] + s)
        out = torch.empty(offs[-1], dtype=packed.dtype, device=packed.device)
        out[offs[rank]:offs[rank] + n].copy_(packed[:n])
        ops = [dist.P2POp(dist.irecv, out[offs[r]:offs[r + 1]], r) for r in range(world) if r != dst and sizes[r]]
        for req in (dist.batch_isend_irecv(ops) if ops else []):
            req.wait()
        return out.to(dev), offs
    if n:
        for req in dist.batch_isend_irecv([dist.P2POp(dist.isend, packed[:n].contiguous(), dst)]):
            req.wait()
    return None, None


def shard_state(count, total, device):
    """Exclusive prefix over ranks of (samples, accumulated error): the GolombCoder state a
    rank's first sample sees (Golomb.h:21-24) when the sequence is split in rank order."""
    rows = _allgather_i64([int(count), int(total)], device)
    r = dist.get_rank()
    n0 = sum(x[0] for x in rows[:r])
    a0 = sum(x[1] for x in rows[:r])
    return n0, a0


def shard_offsets(bits, device):
    """Exclusive prefix over ranks of stream bit lengths, and the total."""
    rows = _allgather_i64([int(bits)], device)
    r = dist.get_rank()
    return sum(x[0] for x in rows[:r]), sum(x[0] for x in rows)


def merge_bit_streams(parts, bit_offsets, total_bits, device):
    """parts[r]: int64 words of rank r's stream, written at bit alignment bit_offsets[r] % 64 so its
    word 0 is global word bit_offsets[r] // 64. A word two neighbours share is the OR of both."""
    out = torch.zeros((int(total_bits) + 63) // 64, dtype=torch.int64, device=device)
    for p, b0 in zip(parts, bit_offsets):
        w0 = int(b0) // 64
        n = min(p.numel(), out.numel() - w0)
        if n > 0:
            out[w0:w0 + n] |= p[:n]
    return out


def sharded_golomb(encode, count, total, device, dst=0, lengths=None):
    """One adaptive Golomb coder over a sample sequence split across the ranks in rank order
    (C5: each rank holds a band of tile rows). encode(n0, a0, bit0) -> (words, bits) codes this
    rank's samples from coder state (n0 samples, accumulated error a0) with its first codeword at
    bit bit0 of words[0]; lengths(n0, a0) -> bits gives the same bit count without writing a
    stream. Exchanges: all-gather of (count, total), all-gather of the bit lengths, point-to-point
    gather of the words. Each rank's stream is written ONCE, at its global bit alignment: the
    length comes first (`lengths`, a scan without the emission; without it, the words are written
    at alignment 0 and written again only when the rank's offset is not a multiple of 64).
    Returns (words, total_bits) on `dst`, (None, total_bits) elsewhere."""
    world, rank = dist.get_world_size(), dist.get_rank()
    n0, a0 = shard_state(count, total, device)
    words = None
    if lengths is not None:
        bits = int(lengths(n0, a0))
    else:
        words, bits = encode(n0, a0, 0)
    lens = [x[0] for x in _allgather_i64([int(bits)], device)]
    b0s = [sum(lens[:r]) for r in range(world)]
    total_bits = sum(lens)
    if words is None or b0s[rank] % 64:
        words, _ = encode(n0, a0, b0s[rank] % 64)
    nwords = (b0s[rank] % 64 + int(bits) + 63) // 64
    gathered, offs = gather_streams(words, nwords, world, rank, dst)
    if rank != dst:
        return None, total_bits
    parts = [gathered[offs[r]:offs[r + 1]] for r in range(world)]
    return merge_bit_streams(parts, b0s, total_bits, device), total_bits
