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
