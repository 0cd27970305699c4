"""The N>1 bench path end to end: `bench.py` under torch.distributed.run with two ranks sharing one
GPU (gloo exchanges), on a small cfg5 stream with --verify (every account and transfer ok, failures
summed over the ranks' home batches). Guards the code the driver runs at N = 2/4/8 (there with RCCL)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_two_ranks_gloo():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--backend", "gloo", "--accounts", "100000", "--transfers", "1000000",
           "--window", "16", "--warmup", "16", "--verify", "--no-cpu-baseline"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [x for x in out.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["results"]["failed_events_timed"] == 0
    assert d["config"]["workload"].startswith("cfg5")
    assert d["value"] > 0
