"""ChunkedGather's device path over RCCL: backend "nccl" at world size 1 on the one GPU
of the test box, in a fresh process (tests/nccl1_worker.py). The gloo tests never take this path (gloo
moves host tensors, so ChunkedGather runs without its communication stream); here the comm stream, the
per-chunk events on the compute stream, comm.wait_event and the closing wait_stream all run, for bench.py's
c4 chunks and c3 --shard planes chunks, and rank 0's gathered words are checked against the oracle."""
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


def test_chunked_gather_rccl_world1():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "nccl1_worker.py"), "c4", "c3planes"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "OK c4" in p.stdout and "OK c3planes" in p.stdout, p.stdout
