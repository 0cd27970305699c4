"""Diagnostic: G-shard create_accounts window; per-shard records vs the expected owned set."""
import sys

import numpy as np
import torch

sys.path.insert(0, "tests")
from test_gpu_shard import LocalShards  # noqa: E402

from tigerbeetle_amd import workload  # noqa: E402
from tigerbeetle_amd.sharding import shard_of  # noqa: E402
from tigerbeetle_amd.types import Operation  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n = 30_000
sh = LocalShards(G, 8190, n // G + 4096, 1 << 16, 8 * 8190)
acc = workload.accounts(0, n, seed=9)
batches = [acc[i:i + 8190] for i in range(0, n, 8190)]
rep = sh.commit_window(Operation.create_accounts, batches)
print("replies empty:", all(r == b"" for r in rep))
own = shard_of(acc["id_lo"], acc["id_hi"], G)
for r, s in enumerate(sh.shards):
    a = s.sm.dump_accounts()
    exp = set(acc["id_lo"][own == r].tolist())
    got = a["id_lo"].tolist()
    zeros = int((a["id_lo"] == 0).sum())
    st = s.stats()
    cls = np.zeros(n, np.uint32)
    code = np.zeros(n, np.uint32)
    from tigerbeetle_amd import _lib
    _lib.lib().tbg_debug_last_batch(s.h, cls.ctypes.data, code.ctypes.data, n)
    C_OWN, C_INSERTED, C_COMMIT = 1 << 18, 1 << 14, 1 << 13
    print(f"shard {r}: count {len(a)} expected {len(exp)} zeros {zeros} missing {len(exp - set(got))} "
          f"extra {len(set(got) - exp)} own_bits {int(((cls & C_OWN) != 0).sum())} "
          f"inserted_bits {int(((cls & C_INSERTED) != 0).sum())} commit {int(((cls & C_COMMIT) != 0).sum())} "
          f"codes!=0 {int((code != 0).sum())} stats {st['accounts']}")
    if zeros:
        zi = np.nonzero(a["id_lo"] == 0)[0]
        print("   zero slots:", zi[:10].tolist())
sh.close()
