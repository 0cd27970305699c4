"""cfg4 window anatomy (GPU box): commits the first windows of bench.py's cfg4 stream (+1 s per
batch, 128-batch windows) and prints, per window, the component-walker counters (tbg_debug_counters:
[5] longest component, [6] components, [7] W events walked) and the phase times.
usage: python tools/cfg4_probe.py [windows] [window_batches]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tigerbeetle_amd import StateMachine, _lib  # noqa: E402
from tigerbeetle_amd.types import NS_PER_S, Operation  # noqa: E402

BM = 8190
PHASES = ["prep", "resolve", "classify", "wcount", "wlist", "walk", "final", "pulse", "cpw"]


def main():
    n_win = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    win = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    n_acc, seed = 1_000_000, 46
    n_x = n_win * win * BM
    L = _lib.lib()
    sm = StateMachine(batch_max=BM, accounts_max=n_acc, transfers_max=n_x, window_events_max=win * BM)
    d_acc = torch.empty(n_acc * 128, dtype=torch.uint8, device="cuda")
    d_x = torch.empty(n_x * 128, dtype=torch.uint8, device="cuda")
    d_res = torch.empty(win * BM * 8, dtype=torch.uint8, device="cuda")
    d_base = torch.empty(win + 1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    _lib.check(L.tbg_gen_accounts(d_acc.data_ptr(), 0, n_acc, seed, 2, 1, 0, sm.stream), "gen")
    _lib.check(L.tbg_gen_transfers_cfg4(d_x.data_ptr(), 0, n_x, seed, n_acc, BM, 0, sm.stream), "gen")

    def commit(op, d, first_batch, nb, n_total, tick):
        ns, ts = [], []
        for b in range(first_batch, first_batch + nb):
            n = min(BM, n_total - b * BM)
            sm.prepare_timestamp += tick + 1 + n
            ns.append(n)
            ts.append(sm.prepare_timestamp)
        sm.commit_window(op, d.data_ptr() + first_batch * BM * 128, ns, ts, d_res.data_ptr(), d_base.data_ptr(),
                         True, ts[0])
        sm.sync()

    nb_acc = (n_acc + BM - 1) // BM
    for b0 in range(0, nb_acc, 128):
        commit(Operation.create_accounts, d_acc, b0, min(128, nb_acc - b0), n_acc, 0)
    dbg = (ctypes.c_uint64 * 8)()
    ms = (ctypes.c_double * len(PHASES))()
    cnt = (ctypes.c_uint64 * len(PHASES))()
    L.tbg_timing_enable(sm.h, -1)
    L.tbg_timing_collect(sm.h, ms, cnt, len(PHASES))
    prev = [0] * 8
    for w in range(n_win):
        commit(Operation.create_transfers, d_x, w * win, win, n_x, NS_PER_S)
        L.tbg_debug_counters(sm.h, dbg, 8)
        L.tbg_timing_collect(sm.h, ms, cnt, len(PHASES))
        cur = list(dbg)
        print(f"window {w}: longest component {cur[5]}, components {cur[6] - prev[6]}, W events {cur[7] - prev[7]}, "
              f"failed {int(d_base[win].item())}")
        print("   phases us: " + ", ".join(f"{p} {ms[k] * 1000:.0f}" for k, p in enumerate(PHASES) if cnt[k]))
        prev = cur
    st = sm.stats()
    print("stats", st)
    sm.close()


if __name__ == "__main__":
    main()
