"""Multi-rank plumbing (pybic.parallel) on CPU with gloo, world_size 2."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "binary-image-compression_amd"))
    import torch.distributed as dist

    from pybic.parallel import gather_streams, shard_offsets, shard_state
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 3 + 4 * rank
        packed = torch.arange(100, dtype=torch.int64) + 1000 * rank
        out, offs = gather_streams(packed, n)
        n0, a0 = shard_state(10 + rank, 100 * (rank + 1), torch.device("cpu"))
        b0, tot = shard_offsets(7 * (rank + 1), torch.device("cpu"))
        q.put((rank, None if out is None else out.tolist(), offs, n0, a0, b0, tot))
    finally:
        dist.destroy_process_group()


def test_gather_and_shard_prefix():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    out, offs = res[0][1], res[0][2]
    assert offs == [0, 3, 10]
    assert out == [0, 1, 2] + [1000 + i for i in range(7)]
    assert res[1][1] is None
    assert (res[0][3], res[0][4]) == (0, 0) and (res[1][3], res[1][4]) == (10, 100)
    assert (res[0][5], res[1][5], res[0][6]) == (0, 7, 21)


def _golomb_py(samples, n0, a0, bit0):
    """GolombCoder::codeSample (GolombCoder.cpp:29-34) from state (n0, a0), first bit at bit0: small
    pure-Python encoder for the sharding test (the GPU coder is checked in test_gpu_parity)."""
    bits = [0] * bit0
    n, A, k = n0, a0, 1
    if n0:
        k = 0
        while (n0 << k) < a0:
            k += 1
    for s in samples:
        bits += [(s >> (k - 1 - i)) & 1 for i in range(k)] + [0] * (s >> k) + [1]
        n += 1
        A += s
        k = 0
        while (n << k) < A:
            k += 1
    nbits = len(bits) - bit0
    bits += [0] * (-len(bits) % 64)
    words = []
    for w in range(len(bits) // 64):
        v = 0
        for b in bits[64 * w:64 * w + 64]:
            v = (v << 1) | b
        words.append(v - (1 << 64) if v >= 1 << 63 else v)
    return torch.tensor(words, dtype=torch.int64), nbits


def _sharded_worker(rank, world, port, q, samples, use_lengths=False):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "binary-image-compression_amd"))
    import torch.distributed as dist

    from pybic.parallel import sharded_golomb
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = rank * len(samples) // world, (rank + 1) * len(samples) // world
        mine = samples[lo:hi]
        calls = []

        def enc(n0, a0, b0):
            calls.append(b0)
            return _golomb_py(mine, n0, a0, b0)
        lengths = (lambda n0, a0: _golomb_py(mine, n0, a0, 0)[1]) if use_lengths else None
        words, total = sharded_golomb(enc, len(mine), sum(mine), torch.device("cpu"), lengths=lengths)
        q.put((rank, None if words is None else words.tolist(), total, calls))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("use_lengths", [False, True])
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_golomb_matches_one_coder(world, use_lengths):
    """C5's exchange: the tile-weight sequence split over ranks, coded with the exchanged coder state
    and bit offsets, reassembled on rank 0 == one coder over the whole sequence"""
    import random
    rnd = random.Random(5)
    samples = [rnd.choice([0, 1, 2, 3, 7, 40, 300]) for _ in range(301)]
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_sharded_worker, args=(r, world, port, q, samples, use_lengths)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp, nbits = _golomb_py(samples, 0, 0, 0)
    assert res[0][2] == nbits and all(res[r][1] is None for r in range(1, world))
    assert res[0][1] == exp.tolist()
    if use_lengths:  # with a lengths-only call, each rank writes its stream exactly once, at its alignment
        offs = [0]
        for r in range(world):
            lo, hi = r * len(samples) // world, (r + 1) * len(samples) // world
            n0, a0 = lo, sum(samples[:lo])
            offs.append(offs[-1] + _golomb_py(samples[lo:hi], n0, a0, 0)[1])
        assert all(res[r][3] == [offs[r] % 64] for r in range(world)), [res[r][3] for r in range(world)]


def _chunked_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "binary-image-compression_amd"))
    import torch.distributed as dist

    from pybic.parallel import ChunkedGather
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cg = ChunkedGather(torch.device("cpu"), world, rank)
        for c in range(3):  # three chunks per rank, one of them empty on rank 1
            n = 0 if (rank == 1 and c == 1) else 2 + rank + 3 * c
            buf = torch.arange(64, dtype=torch.int64) + 10000 * rank + 100 * c
            cg.add(buf, torch.tensor([n, 99], dtype=torch.int64))
        out, offs = cg.finish()
        q.put((rank, None if out is None else out.tolist(), offs))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_chunked_gather(world):
    """pybic.parallel.ChunkedGather (the overlapped gather of bench.py c4 / c3 --shard planes): the
    chunks of every rank land on rank 0 back to back in rank order, chunk order, as gather_streams
    lays out one stream per rank"""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_chunked_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp, offs = [], [0]
    for r in range(world):
        for c in range(3):
            n = 0 if (r == 1 and c == 1) else 2 + r + 3 * c
            exp += [10000 * r + 100 * c + i for i in range(n)]
        offs.append(len(exp))
    assert res[0][1] == exp and res[0][2] == offs
    assert all(res[r][1] is None for r in range(1, world))


def test_plan_chunks_uniform():
    """pybic.parallel.plan_chunks: the same chunk count on every rank for any split of the units, the
    chunks of a rank cover its units in order (8 planes over 3, 5, 6 or 7 ranks gave the ranks
    different chunk counts, i.e. different numbers of collectives)"""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "binary-image-compression_amd"))
    from pybic.parallel import plan_chunks
    for total in (8, 64, 3):
        for world in range(2, 10):
            for chunks in (None, 1, 2, 3, 16):
                plans = []
                for r in range(world):
                    n = (r + 1) * total // world - r * total // world
                    p = plan_chunks(n, total, world, chunks)
                    assert p[0][0] == 0 and p[-1][1] == n
                    assert all(p[i][1] == p[i + 1][0] and p[i][0] <= p[i][1] for i in range(len(p) - 1))
                    plans.append(p)
                assert len({len(p) for p in plans}) == 1, (total, world, chunks, plans)


def _uneven_worker(rank, world, port, q, total):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "binary-image-compression_amd"))
    import torch.distributed as dist

    from pybic.parallel import ChunkedGather, plan_chunks
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = rank * total // world, (rank + 1) * total // world  # bench.py C3Planes' split
        cg = ChunkedGather(torch.device("cpu"), world, rank)
        for a, b in plan_chunks(hi - lo, total, world):
            # a chunk's packed words: unit u contributes 3 + u words valued 1000 u + i
            words = [1000 * (lo + u) + i for u in range(a, b) for i in range(3 + lo + u)]
            cg.add(torch.tensor(words + [7] * 5, dtype=torch.int64), len(words))
        out, offs = cg.finish()
        q.put((rank, None if out is None else out.tolist(), offs))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [3, 5])
def test_chunked_gather_uneven_units(world):
    """8 planes over 3 or 5 ranks (2-3 / 1-2 planes per rank) through plan_chunks + ChunkedGather, as bench.py
    c3 --shard planes runs them: no rank waits on a collective the others never post, and rank 0 ends with
    every unit's words in unit order"""
    total = 8
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_uneven_worker, args=(r, world, port, q, total)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = [1000 * u + i for u in range(total) for i in range(3 + u)]
    assert res[0][1] == exp
    assert all(res[r][1] is None for r in range(1, world))
