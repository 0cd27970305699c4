"""cfg3 window anatomy (GPU box): bench.py's cfg3 stream (Zipf(1.2) debits over accounts with
debits_must_not_exceed_credits, pre-funded) in 32-batch windows; per window the relaxation
iterations (tbg_debug_counters [0], [1] change-free ones) and the phase times.
usage: python tools/cfg3_probe.py [windows] [window_batches]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tigerbeetle_amd import StateMachine, _lib, workload  # noqa: E402
from tigerbeetle_amd.types import Operation  # noqa: E402

BM = 8190
PHASES = ["prep", "resolve", "classify", "wcount", "wlist", "walk", "final", "pulse", "cpw"]


def main():
    n_win = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    win = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    n_acc, seed, top, treasury, fund, fund_id = 1_000_000, 45, 1000, 1000, 1_000_000, 10**15
    n_x = n_win * win * BM
    L = _lib.lib()
    sm = StateMachine(batch_max=BM, accounts_max=n_acc + treasury, transfers_max=n_x + n_acc,
                      window_events_max=128 * BM)
    d_acc = torch.empty((n_acc + treasury) * 128, dtype=torch.uint8, device="cuda")
    d_f = torch.empty(n_acc * 128, dtype=torch.uint8, device="cuda")
    d_x = torch.empty(n_x * 128, dtype=torch.uint8, device="cuda")
    cdf = torch.from_numpy(workload.zipf_cdf(n_acc)).cuda()
    d_res = torch.empty(128 * BM * 8, dtype=torch.uint8, device="cuda")
    d_base = torch.empty(129, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    _lib.check(L.tbg_gen_accounts_cfg3(d_acc.data_ptr(), 0, n_acc + treasury, seed, n_acc, top, sm.stream), "gen")
    _lib.check(L.tbg_gen_funding_cfg3(d_f.data_ptr(), 0, n_acc, seed, n_acc, treasury, fund, fund_id, sm.stream), "gen")
    _lib.check(L.tbg_gen_transfers_zipf(d_x.data_ptr(), 0, n_x, seed, n_acc, cdf.data_ptr(), 0, sm.stream), "gen")

    def commit(op, d, first_batch, nb, n_total):
        ns, ts = [], []
        for b in range(first_batch, first_batch + nb):
            n = min(BM, n_total - b * BM)
            sm.prepare_timestamp += 1 + n
            ns.append(n)
            ts.append(sm.prepare_timestamp)
        sm.commit_window(op, d.data_ptr() + first_batch * BM * 128, ns, ts, d_res.data_ptr(), d_base.data_ptr(),
                         True, ts[0])
        sm.sync()
        return int(d_base[nb].item())

    for data, n_total, op in ((d_acc, n_acc + treasury, Operation.create_accounts), (d_f, n_acc, Operation.create_transfers)):
        nb = (n_total + BM - 1) // BM
        for b0 in range(0, nb, 128):
            commit(op, data, b0, min(128, nb - b0), n_total)
    dbg = (ctypes.c_uint64 * 8)()
    ms = (ctypes.c_double * len(PHASES))()
    cnt = (ctypes.c_uint64 * len(PHASES))()
    L.tbg_timing_enable(sm.h, -1)
    L.tbg_timing_collect(sm.h, ms, cnt, len(PHASES))
    L.tbg_debug_counters(sm.h, dbg, 8)
    prev = list(dbg)
    for w in range(n_win):
        fails = commit(Operation.create_transfers, d_x, w * win, win, n_x)
        L.tbg_debug_counters(sm.h, dbg, 8)
        L.tbg_timing_collect(sm.h, ms, cnt, len(PHASES))
        cur = list(dbg)
        print(f"window {w}: iterations {cur[0] - prev[0]}, change-free {cur[1] - prev[1]}, failed {fails}, "
              f"dbg[2:8] {[cur[k] - prev[k] for k in range(2, 8)]}")
        print("   phases us: " + ", ".join(f"{p} {ms[k] * 1000:.0f}" for k, p in enumerate(PHASES) if cnt[k]))
        prev = cur
    print("stats", sm.stats())
    sm.close()


if __name__ == "__main__":
    main()
