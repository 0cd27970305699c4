"""Windows with pulses inside them (csrc/xwin.h): a window whose batches span a second or more has
pulses due before some of its batches (the harness runs a pulse check before every batch,
state_machine.zig:2719-2739). The GPU engine models them: post/voids find a transfer expired from
its due batch on, the expiries land after the window, and pulse_next_timestamp is replayed batch by
batch. Checked against the CPU restatement run batch by batch with a pulse before each: replies,
pulse_next_timestamp after every window, and the final stores (balances, statuses, records).

Windows the model does not cover (a balance read by a decision, history rows, a pulse that would hit
the scan cap) are rejected (TBG_E_WINDOW) after the window's first pulse; resubmitting the batches
one by one gives the reference's result (that pulse is not run twice)."""
import numpy as np
import pytest

from chaos import Chaos, run_protocol
from oracle_sm import OracleStateMachine
from test_gpu_parity import _compare_final
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import NS_PER_S, Operation


def _stamps(sm, batches, ticks):
    ns, ts = [], []
    for ev, tick in zip(batches, ticks):
        sm.prepare_timestamp += tick + 1 + len(ev)
        ns.append(len(ev))
        ts.append(sm.prepare_timestamp)
    return ns, ts


def commit_ticked(gpu, op, batches, ticks):
    """One window whose batch b is preceded by ticks[b] ns of wall clock. Returns (replies,
    rejected); a rejected window is resubmitted one batch per window with the same timestamps."""
    import torch

    from tigerbeetle_amd._lib import RejectedWindow
    from tigerbeetle_amd.state_machine import to_host

    ts0 = gpu.prepare_timestamp
    ns, ts = _stamps(gpu, batches, ticks)
    data = np.concatenate([np.frombuffer(ev.tobytes(), np.uint8) for ev in batches])
    d_ev = torch.from_numpy(data.copy()).cuda() if len(data) else torch.zeros(128, dtype=torch.uint8).cuda()
    d_res = torch.zeros(max(sum(ns), 1) * 8, dtype=torch.uint8).cuda()
    d_base = torch.zeros(len(ns) + 1, dtype=torch.int32).cuda()
    torch.cuda.synchronize()
    try:
        gpu.commit_window(op, d_ev.data_ptr(), ns, ts, d_res.data_ptr(), d_base.data_ptr(), True, ts[0])
        gpu.sync()
        res = to_host(d_res).tobytes()
        base = to_host(d_base)
        return [res[base[b] * 8: base[b + 1] * 8] for b in range(len(ns))], False
    except RejectedWindow:
        pass
    gpu.prepare_timestamp = ts0
    out = []
    for ev, tick in zip(batches, ticks):
        (n,), (T,) = _stamps(gpu, [ev], [tick])
        d_ev = torch.from_numpy(np.frombuffer(ev.tobytes(), np.uint8).copy()).cuda() if n else \
            torch.zeros(128, dtype=torch.uint8).cuda()
        d_res = torch.zeros(max(n, 1) * 8, dtype=torch.uint8).cuda()
        d_base = torch.zeros(2, dtype=torch.int32).cuda()
        torch.cuda.synchronize()
        gpu.commit_window(op, d_ev.data_ptr(), [n], [T], d_res.data_ptr(), d_base.data_ptr(), True, T)
        gpu.sync()
        base = to_host(d_base)
        out.append(to_host(d_res).tobytes()[base[0] * 8: base[1] * 8])
    return out, True


def oracle_ticked(ref, op, batches, ticks):
    """The same batches through the restatement, a pulse check before each; counts the pulses that
    ran before a batch other than the window's first."""
    out, inner = [], 0
    for k, (ev, tick) in enumerate(zip(batches, ticks)):
        ref.prepare_timestamp += tick + 1
        ref.prepare(Operation(op), ev.tobytes())
        T = ref.prepare_timestamp
        if ref.pulse():
            ref.prefetch_timestamp = T
            ref.prefetch(1, Operation.pulse, b"")
            ref.commit(0, 1, T, Operation.pulse, b"")
            inner += int(k > 0)
        ref.prefetch_timestamp = T
        ref.prefetch(2, op, ev.tobytes())
        out.append(ref.commit(0, 2, T, op, ev.tobytes()))
    return out, inner


def _chaos_run(seed, win, bm, windows, tick_mode, **chaos):
    from tigerbeetle_amd import StateMachine

    gpu = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 17, window_events_max=win * bm)
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(6000 + seed, **chaos)
    inner = rejected = accepted = 0
    try:
        for w in range(windows):
            if w < 2:
                op = Operation.create_accounts
                batches = [ch.accounts_batch(ch.rng.randint(1, bm)) for _ in range(win)]
                ticks = [0] * win
            else:
                op = Operation.create_transfers
                batches = [ch.transfers_batch(ch.rng.choice([1, 2, bm // 2, bm])) for _ in range(win)]
                if tick_mode == "each":
                    ticks = [NS_PER_S] * win
                else:  # ragged: some batches a second apart, some a few ns short of a second
                    ticks = [ch.rng.choice([0, 0, NS_PER_S, NS_PER_S - 2, 2 * NS_PER_S]) for _ in range(win)]
            g, rej = commit_ticked(gpu, op, batches, ticks)
            r, n_inner = oracle_ticked(ref, op, batches, ticks)
            assert g == r, f"window {w} (rejected={rej})"
            assert gpu.pulse_next_timestamp() == ref.pulse_next_timestamp(), f"window {w}"
            if op == Operation.create_transfers:
                rejected += int(rej)
                if not rej:
                    accepted += 1
                    inner += n_inner
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()
    return inner, accepted, rejected


@pytest.mark.gpu
@pytest.mark.parametrize("seed,win,bm,mode", [(0, 4, 16, "each"), (1, 8, 8, "each"), (2, 16, 16, "ragged"),
                                              (3, 6, 64, "ragged"), (4, 32, 4, "each")])
def test_xwin_chaos(seed, win, bm, mode):
    """Two-phase chaos (1-9 s timeouts, posts/voids of in-window and earlier pending transfers,
    chain rollbacks, duplicate ids) with no balance reads: the windows are modelled, not rejected,
    and pulses with expiries run inside them."""
    inner, accepted, rejected = _chaos_run(seed, win, bm, 24, mode, n_accounts=20, id_space=300, pending=0.6,
                                           postvoid=0.45, linked=0.12, limits=0.0, balancing=0.0)
    assert accepted > 0 and inner > 0, (inner, accepted, rejected)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1])
def test_xwin_rejected_when_balances_are_read(seed):
    """Accounts with limits and balancing transfers make the windows' decisions read balances: those
    windows are rejected after their first pulse and resubmitted batch by batch."""
    inner, accepted, rejected = _chaos_run(20 + seed, 6, 16, 20, "each", n_accounts=10, pending=0.5, postvoid=0.4,
                                           limits=0.6, balancing=0.2)
    assert rejected > 0


@pytest.mark.gpu
def test_xwin_cfg4_stream():
    """The cfg4 generator in 8-batch windows, +1 s per batch: a pulse with expiries is due before
    nearly every batch of every window."""
    from tigerbeetle_amd import StateMachine

    n_acc, bm, win, nw = 3000, 8190, 8, 4
    gpu = StateMachine(batch_max=bm, accounts_max=n_acc, transfers_max=win * nw * bm, window_events_max=win * bm)
    ref = OracleStateMachine(batch_max=bm)
    try:
        acc = [workload.accounts(0, n_acc, seed=46)]
        assert commit_ticked(gpu, Operation.create_accounts, acc, [0])[0] == \
            oracle_ticked(ref, Operation.create_accounts, acc, [0])[0]
        inner = 0
        for w in range(nw):
            batches = [workload.transfers_cfg4((w * win + k) * bm, bm, 46, n_acc, bm) for k in range(win)]
            g, rej = commit_ticked(gpu, Operation.create_transfers, batches, [NS_PER_S] * win)
            r, n_inner = oracle_ticked(ref, Operation.create_transfers, batches, [NS_PER_S] * win)
            assert not rej
            assert g == r, f"window {w}"
            assert gpu.pulse_next_timestamp() == ref.pulse_next_timestamp(), f"window {w}"
            inner += n_inner
        assert inner >= nw * (win - 1) - 2
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()
