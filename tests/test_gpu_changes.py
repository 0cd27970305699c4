"""Write-back stream (TBG_FLAG_CHANGE_LOG, tbg_window_changes) vs the CPU restatement's store diffs.

After every window: the logged transfers are exactly the records the window inserted; the logged
accounts are the new accounts (create_accounts) or a superset of the accounts whose record changed
(create_transfers: every account a committed event touched), each equal to the oracle's record now;
the TransferPending rows cover every new pending transfer and every earlier one the window posted or
voided, each with the oracle's status now. No clock ticks, so no pulse expires anything (pulse
changes are not logged)."""
import numpy as np
import pytest

from chaos import Chaos
from oracle_sm import OracleStateMachine, lib
from test_gpu_window import commit_window, oracle_batches
from tigerbeetle_amd.types import Operation


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
    rows_seen = 0
    try:
        for w in range(10):
            acc0, x0 = ref.dump_accounts(), ref.dump_transfers()
            st0 = _statuses(ref, x0)
            if w < 2:
                op = Operation.create_accounts
                batches = [ch.accounts_batch(ch.rng.randint(1, bm)) for _ in range(win)]
            else:
                op = Operation.create_transfers
                batches = [ch.transfers_batch(ch.rng.randint(1, bm)) for _ in range(win)]
            assert commit_window(gpu, op, batches) == oracle_batches(ref, op, batches)
            acc1, x1 = ref.dump_accounts(), ref.dump_transfers()
            la, lx, rows = gpu.window_changes()
            # inserted records, in commit order
            assert lx.tobytes() == x1[len(x0):].tobytes()
            after, before = _by_id(acc1), _by_id(acc0)
            logged = _by_id(la)
            for k, v in logged.items():
                assert after[k] == v, f"window {w}: logged account {k} differs from the oracle's"
            changed = {k for k, v in after.items() if before.get(k) != v}
            if op == Operation.create_accounts:
                assert set(logged) == changed and la.tobytes() == acc1[len(acc0):].tobytes()
            else:
                assert changed <= set(logged), f"window {w}: {sorted(changed - set(logged))[:5]} not logged"
            # TransferPending rows
            st1 = _statuses(ref, x1)
            got = {int(r["timestamp"]): int(r["status"]) for r in rows}
            assert len(got) == len(rows) and list(rows["timestamp"]) == sorted(rows["timestamp"])
            expect = {ts: s for ts, s in st1.items() if ts not in st0 or st0[ts] != s}
            assert set(expect) <= set(got), f"window {w}: rows missing {sorted(set(expect) - set(got))[:5]}"
            for ts, s in got.items():
                assert st1[ts] == s, f"window {w}: row {ts} status {s} vs oracle {st1[ts]}"
            rows_seen += len(rows)
        assert rows_seen > 0
    finally:
        gpu.close()
        ref.close()
