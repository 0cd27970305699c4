"""Write-back stream (TBG_FLAG_CHANGE_LOG, tbg_window_changes) vs the CPU restatement's store diffs.

After every window: the logged transfers are exactly the records the window inserted; the logged
accounts are the new accounts (create_accounts) or a superset of the accounts whose record changed
(create_transfers: every account a committed event touched), each equal to the oracle's record now;
the TransferPending rows cover every new pending transfer and every earlier one the window posted,
voided or expired, each with the oracle's status now. A 1 s tick before every transfer window makes
the window's pulse expire pending transfers: the log of a window covers its pulse too."""
import numpy as np
import pytest

from chaos import Chaos
from oracle_sm import OracleStateMachine, lib
from test_gpu_window import commit_window, oracle_batches
from tigerbeetle_amd.types import NS_PER_S, Operation


def _by_id(arr):
    return {(int(r["id_lo"]), int(r["id_hi"])): r.tobytes() for r in arr}


def _statuses(ref, xfers):
    pend = xfers[(xfers["flags"] & 2) != 0]
    return {int(ts): int(lib().tbo_pending_status(ref.h, int(ts))) for ts in pend["timestamp"]}


def _check_log(gpu, ref, op, acc0, x0, st0, w):
    """The engine's log of the last window vs the restatement's store diff across it."""
    acc1, x1 = ref.dump_accounts(), ref.dump_transfers()
    la, lx, rows = gpu.window_changes()
    # inserted records, in commit order
    assert lx.tobytes() == x1[len(x0):].tobytes()
    after, before = _by_id(acc1), _by_id(acc0)
    logged = _by_id(la)
    for k, v in logged.items():
        assert after[k] == v, f"window {w}: logged account {k} differs from the oracle's"
    changed = {k for k, v in after.items() if before.get(k) != v}
    assert changed <= set(logged), f"window {w}: {sorted(changed - set(logged))[:5]} not logged"
    if op == Operation.create_accounts:
        # the new accounts, after the accounts the window's pulse changed
        new = acc1[len(acc0):]
        assert la[len(la) - len(new):].tobytes() == new.tobytes()
    # TransferPending rows
    st1 = _statuses(ref, x1)
    got = {int(r["timestamp"]): int(r["status"]) for r in rows}
    assert len(got) == len(rows) and list(rows["timestamp"]) == sorted(rows["timestamp"])
    expect = {ts: s for ts, s in st1.items() if ts not in st0 or st0[ts] != s}
    assert set(expect) <= set(got), f"window {w}: rows missing {sorted(set(expect) - set(got))[:5]}"
    for ts, s in got.items():
        assert st1[ts] == s, f"window {w}: row {ts} status {s} vs oracle {st1[ts]}"
    return rows


@pytest.mark.gpu
@pytest.mark.parametrize("seed,win,bm", [(0, 4, 64), (1, 2, 512), (2, 8, 32)])
def test_change_log_matches_oracle_diffs(seed, win, bm):
    from tigerbeetle_amd import StateMachine

    gpu = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 17, window_events_max=win * bm,
                       change_log=True)
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(500 + seed, n_accounts=60, id_space=3000)
    rows_seen = expired = 0
    try:
        for w in range(10):
            acc0, x0 = ref.dump_accounts(), ref.dump_transfers()
            st0 = _statuses(ref, x0)
            tick = NS_PER_S if w >= 3 else 0
            if w < 2 or w == 6:
                op = Operation.create_accounts
                batches = [ch.accounts_batch(ch.rng.randint(1, bm)) for _ in range(win)]
            else:
                op = Operation.create_transfers
                batches = [ch.transfers_batch(ch.rng.randint(1, bm)) for _ in range(win)]
            assert commit_window(gpu, op, batches, tick) == oracle_batches(ref, op, batches, tick)
            rows = _check_log(gpu, ref, op, acc0, x0, st0, w)
            rows_seen += len(rows)
            expired += int((rows["status"] == 4).sum())
        assert rows_seen > 0
        print(f"rows {rows_seen}, expired {expired}")
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("queued", [False, True])
def test_change_log_fused_windows_and_replays(queued):
    """The change log through the fused pass (fused.h marks its accounts in ChgLog::fmark, counted only
    when it commits the window): uniform windows in the class, windows that leave it (one pending or
    limit event: the speculation is undone and the general path logs), and a fused-only window whose
    pulse expired transfers before it left the class: its replay keeps that log (host.inc settle,
    keep_chg). `queued`: the windows before the last are queued without syncs."""
    import torch

    from test_gpu_fused import BM as FBM, WIN, _queue, _replies
    from tigerbeetle_amd import StateMachine, workload

    n_acc = 3000
    gpu = StateMachine(batch_max=FBM, accounts_max=n_acc + 8, transfers_max=1 << 19,
                       window_events_max=WIN * FBM, change_log=True)
    ref = OracleStateMachine(batch_max=FBM)
    try:
        acc = workload.accounts(0, n_acc + 1, seed=11)
        acc["flags"][n_acc] = 2  # debits_must_not_exceed_credits
        batches = [acc[f:f + FBM] for f in range(0, n_acc + 1, FBM)]
        assert commit_window(gpu, Operation.create_accounts, batches) == \
            oracle_batches(ref, Operation.create_accounts, batches)
        first = 0

        def window(kind):
            nonlocal first
            t = workload.transfers_uniform(first, WIN * FBM, seed=12, n_accounts=n_acc)
            first += WIN * FBM
            if kind == "pending":  # pending transfers with a 1 s timeout (out of class)
                t["flags"][::97] = 2
                t["timeout"][::97] = 1
            elif kind == "limit":  # one event reads a balance, near the end (out of class)
                t["debit_account_id_lo"][-10] = n_acc + 1
            return [t[k * FBM:(k + 1) * FBM].copy() for k in range(WIN)]

        # after a window outside the class the speculation backs off (two general-path windows, then a
        # fused attempt that commits re-enables fused-only windows at the next sync)
        plan = ([("plain", 0), ("pending", 0)] + [("plain", 0)] * 4 + [("limit", 2 * NS_PER_S)] +
                [("plain", 0)] * 4 + [("pending", 0)] + [("plain", 0)] * 4 + [("plain", 2 * NS_PER_S), ("limit", 0),
                                                                            ("plain", 0)])
        outs = []
        for w, (kind, tick) in enumerate(plan):
            acc0, x0 = ref.dump_accounts(), ref.dump_transfers()
            st0 = _statuses(ref, x0)
            b = window(kind)
            h = _queue(gpu, b, tick)
            r = oracle_batches(ref, Operation.create_transfers, b, tick)
            outs.append((h, r))
            if queued and w + 1 < len(plan):
                continue
            gpu.sync()
            _check_log(gpu, ref, Operation.create_transfers, acc0, x0, st0, w)
        for h, r in outs:
            assert _replies(h) == r
        st = gpu.stats()
        assert st["fused_windows"] >= 3
        assert (gpu.dump_transfer_status() == 4).sum() > 0  # the pulses expired transfers
    finally:
        gpu.close()
        ref.close()
