"""Debug probe: one cfg4 window (test_geometry_cfg4_mixed_windows' first) on the engine and the CPU
restatement; prints the first differing results with each event's flags."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

from oracle_sm import OracleStateMachine  # noqa: E402
from test_gpu_geometry import BM, N_ACC, _accounts, _batches  # noqa: E402
from test_gpu_window import commit_window, oracle_batches  # noqa: E402
from tigerbeetle_amd import StateMachine, workload  # noqa: E402
from tigerbeetle_amd.types import Operation  # noqa: E402

seed = 46
n_x = 128 * BM
gpu = StateMachine(batch_max=BM, accounts_max=N_ACC, transfers_max=n_x, window_events_max=128 * BM)
ref = OracleStateMachine(batch_max=BM)
_accounts(gpu, ref, seed)
host = workload.transfers_cfg4(0, n_x, seed, N_ACC, BM)
xb = _batches(host, 0, 128 * BM)
g = commit_window(gpu, Operation.create_transfers, xb)
r = oracle_batches(ref, Operation.create_transfers, xb)
out = []
for b in range(128):
    if g[b] == r[b]:
        continue
    gd = {int(x[0]): int(x[1]) for x in np.frombuffer(g[b], dtype=np.uint32).reshape(-1, 2)}
    rd = {int(x[0]): int(x[1]) for x in np.frombuffer(r[b], dtype=np.uint32).reshape(-1, 2)}
    for k in sorted(set(gd) | set(rd)):
        if gd.get(k, 0) != rd.get(k, 0):
            ev = xb[b][k]
            out.append({"b": b, "k": k, "i": b * BM + k, "gpu": gd.get(k, 0), "ref": rd.get(k, 0),
                        "flags": int(ev["flags"]), "pid": int(ev["pending_id_lo"]), "id": int(ev["id_lo"])})
            if len(out) >= 40:
                break
    if len(out) >= 40:
        break
print(json.dumps({"n_bad_batches": sum(g[b] != r[b] for b in range(128)), "first": out}))
