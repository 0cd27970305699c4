"""Probe: bench.py's cfg4 stream window by window (+1 s per batch, 128-batch windows): per window the
component walkers' counters (tbg_debug_counters [5] longest component so far, [6] components,
[7] events walked) and the window's synchronized wall time."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tigerbeetle_amd import StateMachine, _lib, workload  # noqa: E402
from tigerbeetle_amd.types import NS_PER_S, Operation  # noqa: E402

BM, N_ACC, W = 8190, 1_000_000, 128
n_win = int(sys.argv[1]) if len(sys.argv) > 1 else 10
L = _lib.lib()
sm = StateMachine(batch_max=BM, accounts_max=N_ACC, transfers_max=n_win * W * BM + 1, window_events_max=W * BM)
d_acc = torch.empty(N_ACC * 128, dtype=torch.uint8, device="cuda")
d_x = torch.empty(n_win * W * BM * 128, dtype=torch.uint8, device="cuda")
st = sm.stream
_lib.check(L.tbg_gen_accounts(d_acc.data_ptr(), 0, N_ACC, 46, 2, 1, 0, st), "gen")
_lib.check(L.tbg_gen_transfers_cfg4(d_x.data_ptr(), 0, n_win * W * BM, 46, N_ACC, BM, 0, st), "gen")
torch.cuda.synchronize()
d_res = torch.empty(W * BM * 8, dtype=torch.uint8, device="cuda")
d_base = torch.zeros(W + 1, dtype=torch.int32, device="cuda")
ts = [0]


def window(op, ptr, n_total, tick):
    ns, tss = [], []
    for b in range(0, n_total, BM):
        n = min(BM, n_total - b)
        ts[0] += tick + 1 + n
        ns.append(n)
        tss.append(ts[0])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sm.commit_window(op, ptr, ns, tss, d_res.data_ptr(), d_base.data_ptr(), True, tss[0])
    sm.sync()
    return time.perf_counter() - t0


for a in range(0, N_ACC, W * BM):
    window(Operation.create_accounts, d_acc.data_ptr() + a * 128, min(W * BM, N_ACC - a), 0)
rows = []
prev = np.zeros(8, np.uint64)
for w in range(n_win):
    dt = window(Operation.create_transfers, d_x.data_ptr() + w * W * BM * 128, W * BM, NS_PER_S)
    dbg = (ctypes.c_uint64 * 8)()
    _lib.check(L.tbg_debug_counters(sm.h, dbg, 8), "dbg")
    v = np.array(list(dbg), np.uint64)
    rows.append({"w": w, "ms": round(dt * 1e3, 3), "longest_so_far": int(v[5]), "components": int(v[6] - prev[6]),
                 "events": int(v[7] - prev[7])})
    prev = v
    print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
print(json.dumps(rows))
