"""The RCCL leg of the multi-GPU path, on the one GPU a test box has: torch.distributed "nccl" with a
world of one drives routed windows (all_to_all_single with uneven splits) and general windows
(all_reduce) through tigerbeetle_amd.sharding, against the unsharded engine (tests/rccl_one_rank.py,
in its own process so that its process group cannot leak into other tests)."""
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.gpu
def test_rccl_one_rank_routed_and_general():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run([sys.executable, os.path.join(HERE, "rccl_one_rank.py"), str(port)], env=env,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    assert "rccl one-rank ok" in p.stdout
