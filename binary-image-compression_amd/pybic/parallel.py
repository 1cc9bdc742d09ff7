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


def plan_chunks(n_units, total_units, world, chunks=None):
    """Chunk boundaries [(a, b), ...] over a rank's n_units units, for ChunkedGather. The count is the
    same on every rank -- min(chunks or ceil(total/world), ceil(total/world)), a function of the job alone
    -- because every chunk is one collective step (one all-gather of sizes); a rank with fewer units gets
    empty chunks (a == b), which it still adds (with 0 words)."""
    per = -(-int(total_units) // int(world))
    nch = max(1, min(int(chunks) if chunks else per, per))
    return [(i * n_units // nch, (i + 1) * n_units // nch) for i in range(nch)]


class ChunkedGather:
    """gather_streams overlapped with the encode: a rank encodes its units (frames, planes) in chunks
    and hands each chunk's packed words here right after enqueueing its encode (add). finish() then
    walks the chunks in order: a communication stream waits for the chunk's encode only (an event on
    the compute stream), exchanges the chunk's size (one small all-gather) and sends it to `dst` --
    while the compute stream is already encoding the next chunks, so only the last chunk's transfer
    is exposed. The host blocks on one chunk's size at a time (the receiver must post exact counts).
    dst receives every (rank, chunk) into its own buffer and concatenates them in rank order, chunk
    order: (words, offsets per rank) as gather_streams returns them. gloo (CPU tests) runs the same
    protocol on host tensors, without streams.

    Every rank must add() the same number of chunks (plan_chunks gives such a plan; empty chunks are
    allowed): each chunk is one all-gather, so unequal counts would leave ranks waiting on each other."""

    def __init__(self, device, world=None, rank=None, dst=0):
        self.world = world or dist.get_world_size()
        self.rank = dist.get_rank() if rank is None else rank
        self.dst, self.device = dst, device
        self.host = _host_only()
        self.comm = None if self.host or device.type != "cuda" else torch.cuda.Stream(device)
        self.parts = []

    def add(self, packed, nwords):
        """packed: this chunk's words (int64, first nwords used); nwords: 1-element int64 tensor (device)
        or int, final once the encode enqueued on the current stream completes"""
        ev = None
        if self.comm is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
        self.parts.append((packed, nwords, ev))

    def _sizes(self, nwords):
        t = nwords.reshape(-1)[:1].to(torch.int64) if torch.is_tensor(nwords) else torch.tensor([int(nwords)])
        t = t.cpu() if self.host else t.to(self.device)
        outs = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(outs, t)
        return [int(x) for x in torch.cat(outs).cpu()]  # (host sync: this chunk's size exchange only)

    def finish(self):
        got = {r: [] for r in range(self.world)}  # dst: per rank its chunks' words
        reqs = []
        cur = torch.cuda.current_stream(self.device) if self.comm is not None else None
        for packed, nwords, ev in self.parts:
            ctx = torch.cuda.stream(self.comm) if self.comm is not None else _null()
            with ctx:
                if ev is not None:
                    self.comm.wait_event(ev)
                sizes = self._sizes(nwords)
                n = sizes[self.rank]
                src = packed.cpu() if self.host else packed
                if self.rank == self.dst:
                    ops = []
                    for r in range(self.world):
                        if r == self.rank:
                            got[r].append(src[:n])
                        elif sizes[r]:
                            buf = torch.empty(sizes[r], dtype=packed.dtype, device=src.device)
                            got[r].append(buf)
                            ops.append(dist.P2POp(dist.irecv, buf, r))
                    if ops:
                        reqs += dist.batch_isend_irecv(ops)
                elif n:
                    reqs += dist.batch_isend_irecv([dist.P2POp(dist.isend, src[:n].contiguous(), self.dst)])
        with (torch.cuda.stream(self.comm) if self.comm is not None else _null()):
            for q in reqs:
                q.wait()
            if self.rank != self.dst:
                out = None
            else:
                offs = [0]
                for r in range(self.world):
                    offs.append(offs[-1] + sum(int(x.numel()) for x in got[r]))
                chunks = [x for r in range(self.world) for x in got[r]]
                out = torch.cat(chunks) if chunks else torch.empty(0, dtype=torch.int64)
        if cur is not None:
            cur.wait_stream(self.comm)  # the step ends with the streams on dst (and the sends done)
        self.parts = []
        if out is None:
            return None, None
        return out.to(self.device), offs


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


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
