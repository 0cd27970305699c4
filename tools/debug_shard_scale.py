"""Diagnostic: bench-scale sharded create_accounts window (one window of 49 batches), in-process."""
import sys

import numpy as np
import torch

sys.path.insert(0, "tests")
from test_gpu_shard import LocalShards  # noqa: E402

from tigerbeetle_amd import workload  # noqa: E402
from tigerbeetle_amd.sharding import shard_of  # noqa: E402
from tigerbeetle_amd.types import Operation  # noqa: E402

G, n = 2, 400_000
sh = LocalShards(G, 8190, int(n / G * 1.02) + 65536, 1 << 16, 64 * 8190)
acc = workload.accounts(0, n, seed=47)
batches = [acc[i:i + 8190] for i in range(0, n, 8190)]
rep = sh.commit_window(Operation.create_accounts, batches)
print("replies empty:", all(r == b"" for r in rep), flush=True)
own = shard_of(acc["id_lo"], acc["id_hi"], G)
for r, s in enumerate(sh.shards):
    print(f"shard {r}: accounts {s.stats()['accounts']} expected {int((own == r).sum())}", flush=True)
