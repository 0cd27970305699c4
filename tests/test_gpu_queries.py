"""get_account_transfers / get_account_balances (state_machine.zig:786-996, 1346-1419) and the
history rows behind them (historical_balance, :1806-1841) on the GPU engine vs the CPU restatement.
The reference's own query tables run in test_gpu_kat.py; here: random filters (valid and invalid,
both directions, timestamp bounds, limits below and above batch_max) over chaos streams whose
accounts carry flags.history, in single-batch and multi-batch windows, and after a restart from the
forest's objects (tbg_open with the account_balances rows)."""
import numpy as np
import pytest

from chaos import Chaos, run_protocol
from oracle_sm import OracleStateMachine
from test_gpu_parity import _compare_final
from test_gpu_window import commit_window, oracle_batches
from tigerbeetle_amd.types import (
    FILTER_CREDITS,
    FILTER_DEBITS,
    FILTER_DTYPE,
    FILTER_REVERSED,
    NS_PER_S,
    Operation,
    set_u128,
)

QUERIES = (Operation.get_account_transfers, Operation.get_account_balances)


def _filter(rng, n_accounts, timestamps, bm):
    f = np.zeros(1, FILTER_DTYPE)
    set_u128(f[0], "account_id", rng.choice([rng.randint(1, n_accounts + 2), rng.randint(1, n_accounts)]))
    if timestamps and rng.random() < 0.25:
        f[0]["timestamp_min"] = rng.choice(timestamps)
    if timestamps and rng.random() < 0.25:
        f[0]["timestamp_max"] = rng.choice(timestamps)
    f[0]["limit"] = rng.choice([0, 1, 2, 5, bm - 1, bm, bm + 7, 100000])
    both = FILTER_DEBITS | FILTER_CREDITS
    flags = rng.choice([FILTER_DEBITS, FILTER_CREDITS, both, both, both, 0])
    if rng.random() < 0.5:
        flags |= FILTER_REVERSED
    if rng.random() < 0.03:
        flags |= 8  # padding: invalid
    f[0]["flags"] = flags
    if rng.random() < 0.03:
        f[0]["reserved"][5] = 1  # invalid
    return f.tobytes()


def _queries(gpu, ref, rng, n_accounts, bm, k):
    ts = [int(t) for t in ref.dump_transfers()["timestamp"]]
    nonempty = 0
    for _ in range(k):
        q = _filter(rng, n_accounts, ts, bm)
        for op in QUERIES:
            a = gpu.commit(0, 1, gpu.prepare_timestamp, op, q)
            b = ref.commit(0, 1, ref.prepare_timestamp, op, q)
            assert a == b, f"{op.name}: {len(a)} vs {len(b)} bytes, filter {np.frombuffer(q, FILTER_DTYPE)}"
            nonempty += int(len(b) > 0)
    return nonempty


@pytest.mark.gpu
@pytest.mark.parametrize("seed,bm", [(0, 16), (1, 64), (2, 256)])
def test_queries_chaos(seed, bm):
    from tigerbeetle_amd import StateMachine

    gpu = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 16)
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(5100 + seed, n_accounts=30, history=0.5)
    nonempty = 0
    try:
        for b in range(36):
            if b < 3:
                ev, op = ch.accounts_batch(ch.rng.randint(1, bm)), Operation.create_accounts
            else:
                ev, op = ch.transfers_batch(ch.rng.choice([1, 3, bm // 2, bm])), Operation.create_transfers
            tick = NS_PER_S if b % 3 == 0 else 0
            assert run_protocol(gpu, op, ev, tick) == run_protocol(ref, op, ev, tick)
            if b % 4 == 3:
                nonempty += _queries(gpu, ref, ch.rng, 30, bm, 12)
        _compare_final(gpu, ref)
        assert nonempty > 10
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,win,bm", [(0, 4, 32), (1, 8, 16)])
def test_queries_after_windows(seed, win, bm):
    """History rows written by multi-batch windows (the sequential walker decides every event that
    touches a history account, in order)."""
    from tigerbeetle_amd import StateMachine

    gpu = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 16, window_events_max=win * bm)
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(5200 + seed, n_accounts=25, history=0.6, limits=0.2)
    try:
        for w in range(14):
            if w < 2:
                op = Operation.create_accounts
                batches = [ch.accounts_batch(ch.rng.randint(1, bm)) for _ in range(win)]
            else:
                op = Operation.create_transfers
                batches = [ch.transfers_batch(ch.rng.choice([1, 3, bm // 2, bm])) for _ in range(win)]
            assert commit_window(gpu, op, batches, NS_PER_S) == oracle_batches(ref, op, batches, NS_PER_S)
            if w % 3 == 2:
                _queries(gpu, ref, ch.rng, 25, bm, 10)
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_queries_after_open_with_history_rows():
    """A restart: open from the objects and the account_balances rows; every query answers as
    before the restart."""
    from test_gpu_restore import _oracle_status
    from tigerbeetle_amd import StateMachine

    bm = 32
    gpu = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 15)
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(5300, n_accounts=20, history=0.7)
    try:
        for b in range(45):
            if b < 3:
                ev, op = ch.accounts_batch(bm), Operation.create_accounts
            else:
                ev, op = ch.transfers_batch(ch.rng.choice([1, 3, bm])), Operation.create_transfers
            run_protocol(ref, op, ev, NS_PER_S if b % 3 == 0 else 0)
        rx = ref.dump_transfers()
        rows = ref.dump_account_balances()
        assert len(rows) > 0
        gpu.open(ref.dump_accounts(), rx, _oracle_status(ref, rx), rows)
        gpu.prepare_timestamp = ref.prepare_timestamp
        _queries(gpu, ref, ch.rng, 20, bm, 40)
        nonempty = 0
        for acc in range(1, 21):  # every account, both sides, both directions
            for flags in (FILTER_DEBITS | FILTER_CREDITS, FILTER_DEBITS | FILTER_CREDITS | FILTER_REVERSED):
                f = np.zeros(1, FILTER_DTYPE)
                set_u128(f[0], "account_id", acc)
                f[0]["limit"] = bm
                f[0]["flags"] = flags
                for op in QUERIES:
                    a = gpu.commit(0, 1, 0, op, f.tobytes())
                    assert a == ref.commit(0, 1, 0, op, f.tobytes()), (acc, flags, op.name)
                    nonempty += int(len(a) > 0)
        assert nonempty > 10
    finally:
        gpu.close()
        ref.close()
