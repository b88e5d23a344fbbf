"""RCCL with more than one rank: the sharded engines' collectives --
the count all-gather and picks all-reduce MAX of column shards, the grouped ncclSend /
ncclRecv of row shards (full view and partial view), the count broadcasts and node 0's row
broadcast -- run between real ranks, and the job's results are checked against the oracle
(the behaviour is EmulNet::ENsend / ENrecv across shards, EmulNet.cpp:87-177).

Each case launches tests/rccl_ranks.py under torch.distributed.run, one fresh child process
per GPU (this process makes no GPU call for it: the device count comes from torch, which does
not initialise the GPU to count).  Skips where fewer than two GPUs are visible -- the
one-GPU boxes this build is developed on; the driver's 8-GPU node runs it.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gpus():
    import torch
    return torch.cuda.device_count()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(case, world):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
           str(world), "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "rccl_ranks.py"), case]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0 and lines, "rc %d\n%s\n%s" % (p.returncode, p.stdout[-3000:],
                                                          p.stderr[-3000:])
    res = json.loads(lines[-1])
    assert res["world"] == world
    return res["ranks"]


@pytest.mark.parametrize("case", ["columns_tiled", "rows", "pview_rows", "pview_capacity",
                                  "rows_capacity", "pview_burst", "rows_burst"])
def test_two_ranks_match_the_oracle(case):
    if _gpus() < 2:
        pytest.skip("needs two GPUs (%d visible)" % _gpus())
    for r in _launch(case, 2):
        assert r["bad"] == [] and ("capacity" in case or r["xgmi"] > 0), r


def test_rank_program_one_rank():
    """The same child program with one rank (the one-GPU boxes): every check but the xGMI
    bytes, so the multi-GPU test's own logic is exercised wherever a GPU exists."""
    for case in ("columns_tiled", "rows", "pview_rows", "pview_capacity", "rows_capacity",
                 "pview_burst", "rows_burst"):
        for r in _launch(case, 1):
            assert r["bad"] == [], (case, r)
