"""Reproducer: fresh single-shard engines, one create_accounts window each; checks the engine's
globals right after creation and the stored count after the window. Stops at the first anomaly."""
import sys

import numpy as np
import torch

sys.path.insert(0, "tests")
from test_gpu_shard import LocalShards  # noqa: E402

from tigerbeetle_amd import workload  # noqa: E402
from tigerbeetle_amd.types import Operation  # noqa: E402

n = 30_000
acc = workload.accounts(0, n, seed=9)
batches = [acc[i:i + 8190] for i in range(0, n, 8190)]
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    sh = LocalShards(1, 8190, n + 4096, 250_000 + 16384, 8 * 8190)
    st0 = sh.shards[0].stats()
    if st0["accounts"] or st0["transfers"] or st0["events_total"]:
        print(f"iter {it}: fresh engine globals not zero: {st0}", flush=True)
        break
    try:
        sh.commit_window(Operation.create_accounts, batches)
    except Exception as e:  # noqa: BLE001
        print(f"iter {it}: {e}", flush=True)
        break
    st = sh.shards[0].stats()
    if st["accounts"] != n:
        print(f"iter {it}: accounts {st['accounts']}", flush=True)
        break
    sh.close()
else:
    print("no anomaly", flush=True)
