"""The N > 1 chains on the one GPU of the test box: several ranks (separate processes, gloo between
them) run the real sharded paths through libbic.so -- frames (C4) and planes (C3) packed and
gathered to rank 0, tiles (C5) with one adaptive coder continued across ranks -- and rank 0
checks every byte it received against the oracle (tests/mrank_worker.py). The same code runs over
RCCL at one rank per GPU in bench.py; only the transport differs."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, jobs, encoder="auto", timeout=240):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), BIC_MR_ENCODER=encoder, OMP_NUM_THREADS="2")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mrank_worker.py"), *jobs],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append(out)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, f"rank {r} exit {p.returncode}:\n{out[-3000:]}"
    return outs[0]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_chains(world):
    out = _run(world, ["frames", "planes", "tiles"])
    assert "'frames': True" in out and "'planes': True" in out and "'tiles': True" in out, out


def test_sharded_staged_encoder():
    out = _run(2, ["frames", "planes"], encoder="staged")
    assert "'frames': True" in out and "'planes': True" in out, out


@pytest.mark.parametrize("workload", [
    ["--workload", "c3", "--shard", "planes", "--rows", "512", "--cols", "4096"],
    ["--workload", "c4", "--rows", "256", "--cols", "1024"],
    ["--workload", "c5", "--rows", "1024", "--cols", "2048"],
], ids=["c3-planes", "c4", "c5"])
def test_bench_gpus2_spawns_ranks(workload):
    """the plain command `bench.py --gpus 2 ...` (no launcher in the command: bench.py starts the two
    ranks itself, as a child torch.distributed.run) on the one GPU over gloo: rank 0 prints one line
    with n_gpus 2, and its bit_exact_check covers what rank 0 RECEIVED -- the gathered C3 plane
    streams / all 64 C4 frames' streams, the merged C5 stream of the whole plane"""
    import json
    env = dict(os.environ, BIC_BENCH_BACKEND="gloo", OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *workload, "--steps", "2", "--warmup", "1"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    j = json.loads(lines[0])
    assert j["bit_exact_check"] is True and j["n_gpus"] == 2 and j["scaling"] == "strong", j


def test_bench_plane_count_one_rank():
    """--plane-count 1 at N = 1: the per-rank step of an 8-GPU plane-sharded run, bit-exact"""
    import json
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "c3", "--shard", "planes", "--plane-count",
           "1", "--rows", "512", "--cols", "4096", "--steps", "2", "--warmup", "1", "--no-cpu"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    j = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
    assert j["bit_exact_check"] is True and j["config"]["planes_per_gpu"] == 1, j
