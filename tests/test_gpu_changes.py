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
            rows_seen += len(rows)
            expired += int((rows["status"] == 4).sum())
        assert rows_seen > 0
        print(f"rows {rows_seen}, expired {expired}")
    finally:
        gpu.close()
        ref.close()
