"""The pulse decision (state_machine.zig:589-596) on the GPU engine is the reference's, batch for
batch: pulse_next_timestamp is lowered by every timeout creation that ran ok, also when its chain
is rolled back later (:1576-1581), reset to timestamp_min by a post/void of the transfer whose
expiry it holds (:1704-1708), and set by each pulse's finish (:2112-2145).

- lockstep runs (tests/lockstep.py): every pulse() decision, reply and pulse_next_timestamp equal
  the CPU restatement's, over the reference KAT tables, chaos streams and the cfg4 stream;
- a replica-protocol run in which a pulse is its own prepare (vsr/replica.zig:5763-5771,
  9459-9487), so a different decision would shift every later stored timestamp;
- super-batched windows: a reset inside a window (then an empty pulse at the next batch) is
  replayed exactly, and a window that spans a due pulse is rejected whole, then resubmitted.
"""
import glob
import os

import numpy as np
import pytest

from chaos import Chaos, run_protocol
from kat import check
from lockstep import Lockstep, replica_commit
from oracle_sm import OracleStateMachine
from test_gpu_parity import _compare_final
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import NS_PER_S, Operation

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KATS = sorted(glob.glob(os.path.join(GOLDEN, "kat_*.tbl")))


@pytest.mark.gpu
def test_pulse_lockstep_kat_tables():
    from tigerbeetle_amd import StateMachine

    decisions = pulses = 0
    for path in KATS:
        gpu = StateMachine(batch_max=64, accounts_max=1024, transfers_max=4096)
        ref = OracleStateMachine(batch_max=64)
        try:
            ls = Lockstep(gpu, ref)
            check(ls, open(path).read())
            decisions += ls.decisions
            pulses += ls.pulses
        finally:
            gpu.close()
            ref.close()
    assert decisions > 50 and pulses > 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed,bm,tick_every", [(0, 16, 2), (1, 16, 3), (2, 64, 2), (3, 256, 4), (4, 8, 1)])
def test_pulse_lockstep_chaos(seed, bm, tick_every):
    """Chaos streams with timeouts, posts/voids of pending transfers (resets), chain rollbacks of
    pending creations (rolled-back lowerings) and the pulse cap."""
    from tigerbeetle_amd import StateMachine

    gpu = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 16)
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(500 + seed, pending=0.5, postvoid=0.35, linked=0.2)
    try:
        ls = Lockstep(gpu, ref)
        for b in range(60):
            if b < 3:
                ev, op = ch.accounts_batch(ch.rng.randint(1, bm)), Operation.create_accounts
            else:
                ev, op = ch.transfers_batch(ch.rng.choice([1, 2, bm // 2, bm])), Operation.create_transfers
            run_protocol(ls, op, ev, NS_PER_S if b % tick_every == 0 else 0)
        _compare_final(gpu, ref)
        assert ls.pulses > 0
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_pulse_lockstep_resets_happen():
    """Streams built to post/void the transfer with the earliest expiry: the reset path runs."""
    from tigerbeetle_amd import StateMachine

    resets = 0
    for seed in range(6):
        gpu = StateMachine(batch_max=16, accounts_max=1 << 10, transfers_max=1 << 14)
        ref = OracleStateMachine(batch_max=16)
        ch = Chaos(900 + seed, n_accounts=8, id_space=60, pending=0.7, postvoid=0.5, linked=0.1, invalid=0.0,
                   balancing=0.0, limits=0.0)
        try:
            ls = Lockstep(gpu, ref)
            for b in range(40):
                if b < 2:
                    ev, op = ch.accounts_batch(16), Operation.create_accounts
                else:
                    ev, op = ch.transfers_batch(ch.rng.choice([1, 2, 4])), Operation.create_transfers
                run_protocol(ls, op, ev, NS_PER_S if b % 5 == 0 else 0)
            resets += ls.resets
        finally:
            gpu.close()
            ref.close()
    assert resets > 0


@pytest.mark.gpu
def test_pulse_lockstep_cfg4_stream():
    """The cfg4 generator (30 % pending with 1-60 s timeouts, posts/voids, chains with injected
    failures), +1 s per batch: a pulse is due before nearly every batch."""
    from tigerbeetle_amd import StateMachine

    n_acc, bm, nb = 3000, 8190, 20
    gpu = StateMachine(batch_max=bm, accounts_max=n_acc, transfers_max=nb * bm)
    ref = OracleStateMachine(batch_max=bm)
    try:
        ls = Lockstep(gpu, ref)
        run_protocol(ls, Operation.create_accounts, workload.accounts(0, n_acc, seed=46), 0)
        for b in range(nb):
            ev = workload.transfers_cfg4(b * bm, bm, 46, n_acc, bm)
            run_protocol(ls, Operation.create_transfers, ev, NS_PER_S)
        assert ls.pulses >= nb - 2
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


def _replica_run(sm, ch_seed, bm, batches):
    ch = Chaos(ch_seed, pending=0.6, postvoid=0.4, linked=0.15)
    replies, pulses, op = [], 0, 1
    for b in range(batches):
        if b < 3:
            ev, operation = ch.accounts_batch(ch.rng.randint(1, bm)), Operation.create_accounts
        else:
            ev, operation = ch.transfers_batch(ch.rng.choice([1, 3, bm // 2, bm])), Operation.create_transfers
        # a stale wall clock most of the time (timestamps advance by the prepares alone, so every
        # pulse prepare shifts the later ones by one), a 1.5 s jump every fourth request
        realtime = sm.prepare_timestamp + NS_PER_S * 3 // 2 if b % 4 == 0 else 0
        r, op, pulsed = replica_commit(sm, op, operation, ev, realtime)
        replies.append(r)
        pulses += int(pulsed)
    return replies, pulses


@pytest.mark.gpu
@pytest.mark.parametrize("seed,bm", [(0, 16), (1, 64), (2, 8)])
def test_pulse_replica_protocol(seed, bm):
    """Independent runs (not lockstep) under the replica's protocol: identical replies and stores,
    stored timestamps included, and the same number of pulse prepares."""
    from tigerbeetle_amd import StateMachine

    gpu = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 16)
    ref = OracleStateMachine(batch_max=bm)
    try:
        g, gp = _replica_run(gpu, 700 + seed, bm, 50)
        r, rp = _replica_run(ref, 700 + seed, bm, 50)
        assert gp == rp and gp > 0
        for k, (a, b) in enumerate(zip(g, r)):
            assert a == b, f"request {k}"
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


def _window(gpu, op, batches, tick_ns):
    """Harness timestamps for the window's batches; commits them as one window. On a rejected
    window (TBG_E_WINDOW) nothing may have changed: checks that, then resubmits the batches one
    window each. Returns (per-batch replies, rejected)."""
    import torch

    from test_gpu_window import commit_window
    from tigerbeetle_amd._lib import RejectedWindow
    from tigerbeetle_amd.state_machine import to_host

    ts0 = gpu.prepare_timestamp
    before = (gpu.dump_accounts().tobytes(), gpu.dump_transfers().tobytes(), gpu.dump_transfer_status().tobytes(),
              gpu.pulse_next_timestamp(), gpu.windows_committed())
    try:
        return commit_window(gpu, op, batches, tick_ns), False
    except RejectedWindow:
        pass
    after = (gpu.dump_accounts().tobytes(), gpu.dump_transfers().tobytes(), gpu.dump_transfer_status().tobytes(),
             gpu.pulse_next_timestamp())
    assert after == before[:4], "a rejected window changed the state"
    applied, submitted = gpu.windows_committed()
    assert applied == before[4][0] and submitted == before[4][1] + 1
    # resubmit with the same timestamps, one batch per window (each with its own pulse check)
    gpu.prepare_timestamp = ts0 + tick_ns
    out = []
    for ev in batches:
        gpu.prepare_timestamp += 1 + len(ev)
        T = gpu.prepare_timestamp
        d_ev = torch.from_numpy(np.frombuffer(ev.tobytes(), np.uint8).copy()).cuda() if len(ev) else \
            torch.zeros(128, dtype=torch.uint8).cuda()
        d_res = torch.zeros(max(len(ev), 1) * 8, dtype=torch.uint8).cuda()
        d_base = torch.zeros(2, dtype=torch.int32).cuda()
        torch.cuda.synchronize()
        gpu.commit_window(op, d_ev.data_ptr(), [len(ev)], [T], d_res.data_ptr(), d_base.data_ptr(), True, T)
        gpu.sync()
        base = to_host(d_base)
        out.append(to_host(d_res).tobytes()[base[0] * 8: base[1] * 8])
    return out, True


def _run_windows(seed, win, bm):
    """Multi-batch windows on chaos streams with timeouts: pulse_next after every window equals the
    oracle's after the same batches one by one; resets inside windows (pulse_next == timestamp_min
    after a batch that is not the window's last) are replayed, due pulses inside a window reject it.
    Returns (resets inside windows, rejected windows)."""
    from tigerbeetle_amd import StateMachine

    gpu = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 17, window_events_max=win * bm)
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(4000 + seed, n_accounts=20, id_space=300, pending=0.6, postvoid=0.45, linked=0.12)
    mid_resets = rejected = 0
    try:
        for w in range(30):
            if w < 2:
                op = Operation.create_accounts
                batches = [ch.accounts_batch(ch.rng.randint(1, bm)) for _ in range(win)]
            else:
                op = Operation.create_transfers
                batches = [ch.transfers_batch(ch.rng.choice([1, 2, bm // 2, bm])) for _ in range(win)]
            # mostly no tick (pulses come from resets only); sometimes 1 s before the window, and
            # sometimes just short of an expiry so a pulse falls due inside the window
            tick = ch.rng.choice([0, 0, 0, NS_PER_S, NS_PER_S - 3])
            g, rej = _window(gpu, op, batches, tick)
            rejected += int(rej)
            r = []
            for k, ev in enumerate(batches):
                r.append(run_protocol(ref, op, ev, tick if k == 0 else 0))
                if k < len(batches) - 1 and ref.pulse_next_timestamp() == 1:
                    mid_resets += 1
            assert g == r, f"window {w}"
            assert gpu.pulse_next_timestamp() == ref.pulse_next_timestamp(), f"window {w}"
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()
    return mid_resets, rejected


@pytest.mark.gpu
@pytest.mark.parametrize("seed,win,bm", [(0, 4, 16), (1, 8, 8), (2, 3, 64), (3, 16, 16)])
def test_pulse_windows(seed, win, bm):
    _run_windows(seed, win, bm)


@pytest.mark.gpu
def test_pulse_windows_cover_resets_and_rejections():
    mid = rej = 0
    for seed, win, bm in [(10, 8, 8), (11, 16, 4), (12, 6, 16), (13, 12, 8)]:
        m, r = _run_windows(seed, win, bm)
        mid += m
        rej += r
    assert mid > 0 and rej > 0, (mid, rej)


@pytest.mark.gpu
@pytest.mark.parametrize("n_due", [3, 4, 5, 8])
def test_pulse_exactly_cap_due(n_due):
    """batch_max = 4 and 3, 4, 5 or 8 pending transfers due at one pulse. The scan's buffer-full
    check precedes each next() (lsm/scan_lookup.zig:151-156): with exactly 4 due the buffer fills
    before the scan sees the next entry, so the pulse ends buffer_finished, pulse_next_timestamp is
    the last expired one's expires_at (state_machine.zig:2112-2145) and another pulse follows."""
    from tigerbeetle_amd import StateMachine
    from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE, set_u128

    bm = 4
    gpu = StateMachine(batch_max=bm, accounts_max=64, transfers_max=1024)
    ref = OracleStateMachine(batch_max=bm)
    try:
        ls = Lockstep(gpu, ref)
        a = np.zeros(2, ACCOUNT_DTYPE)
        for k in range(2):
            set_u128(a[k], "id", k + 1)
            a[k]["ledger"], a[k]["code"] = 1, 1
        run_protocol(ls, Operation.create_accounts, a, 0)
        ids = iter(range(100, 1000))

        def xfers(n, timeout, pending=True):
            t = np.zeros(n, TRANSFER_DTYPE)
            for k in range(n):
                set_u128(t[k], "id", next(ids))
                set_u128(t[k], "debit_account_id", 1)
                set_u128(t[k], "credit_account_id", 2)
                set_u128(t[k], "amount", 10)
                t[k]["ledger"], t[k]["code"] = 1, 1
                t[k]["flags"] = 2 if pending else 0
                t[k]["timeout"] = timeout
            return t

        left = n_due
        while left:
            run_protocol(ls, Operation.create_transfers, xfers(min(bm, left), 1), 0)
            left -= min(bm, left)
        run_protocol(ls, Operation.create_transfers, xfers(1, 30), 0)  # a later live entry
        for k in range(4):  # past the timeouts, then a few batches: one or more pulses
            run_protocol(ls, Operation.create_transfers, xfers(1, 0, pending=False), 2 * NS_PER_S if k == 0 else 0)
        assert ls.pulses >= 2
        _compare_final(gpu, ref)
        assert (ref.dump_transfer_status() == 4).sum() == n_due
    finally:
        gpu.close()
        ref.close()
