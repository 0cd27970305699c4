"""The wave-decided long components (csrc/cps.h) against the restatement and against the component
walkers alone. TBG_CPS_MIN (read when an engine is created) sets the length above which a component
of a component-walked window is decided by one wave as a fixed point; 0 leaves every component to
the per-component walkers (cpw.h). Small thresholds push the chaos streams' short components (chains
with rollbacks, duplicate ids, posts/voids of in-window and stored pending transfers, expiry inside
the window) through the solver too."""
import ctypes

import numpy as np
import pytest

from chaos import Chaos
from oracle_sm import OracleStateMachine
from test_gpu_parity import _compare_final
from test_gpu_window import commit_window, oracle_batches
from test_gpu_xwin import commit_ticked, oracle_ticked
from tigerbeetle_amd import _lib, workload
from tigerbeetle_amd.types import NS_PER_S, Operation


def _solver_counters(sm):
    """tbg_debug_counters in component windows: [1] wave-decided components, [2] their events,
    [3] their passes, [4] the most passes one component took."""
    d = (ctypes.c_uint64 * 8)()
    _lib.check(_lib.lib().tbg_debug_counters(sm.h, d, 8), "debug counters")
    return list(d)


def _chaos_windows(seed, win, bm, windows, ticks_mode, **chaos):
    """Chaos windows with no balance reads (limits / balancing stripped): GPU vs the restatement,
    replies and pulse_next_timestamp per window, the stores at the end. Returns the GPU engine's
    solver counters."""
    from tigerbeetle_amd import StateMachine

    gpu = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 17, window_events_max=win * bm)
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(7100 + seed, **chaos)
    try:
        for w in range(windows):
            if w < 2:
                op = Operation.create_accounts
                batches = [ch.accounts_batch(ch.rng.randint(1, bm)) for _ in range(win)]
                for b in batches:
                    b["flags"] &= ~np.uint16(6)  # no balance limits
                ticks = [0] * win
            else:
                op = Operation.create_transfers
                batches = [ch.transfers_batch(ch.rng.choice([1, 3, bm // 2, bm])) for _ in range(win)]
                for b in batches:
                    b["flags"] &= ~np.uint16(0x30)  # no balancing
                ticks = [NS_PER_S if ticks_mode == "each" else ch.rng.choice([0, 0, NS_PER_S]) for _ in range(win)]
            g, _ = commit_ticked(gpu, op, batches, ticks)
            r, _ = oracle_ticked(ref, op, batches, ticks)
            assert g == r, f"window {w}"
            assert gpu.pulse_next_timestamp() == ref.pulse_next_timestamp(), f"window {w}"
        _compare_final(gpu, ref)
        return _solver_counters(gpu)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cps_min", [1, 3])
@pytest.mark.parametrize("seed,win,bm,mode", [(0, 4, 64, "each"), (1, 8, 128, "ragged"), (2, 2, 1024, "each")])
def test_cps_chaos_vs_restatement(monkeypatch, cps_min, seed, win, bm, mode):
    monkeypatch.setenv("TBG_CPS_MIN", str(cps_min))
    dbg = _chaos_windows(seed, win, bm, 16, mode, n_accounts=30, id_space=600, pending=0.5, postvoid=0.45,
                         linked=0.2, limits=0.0, balancing=0.0)
    assert dbg[1] > 0 and dbg[2] > dbg[1], dbg  # the solver decided components


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [3, 4])
def test_cps_matches_component_walkers(monkeypatch, seed):
    """Same chaos stream (duplicate ids, retries, chain rollbacks) with the solver taking every
    component of two events or more, and with the walkers alone: identical replies and stores."""
    from tigerbeetle_amd import StateMachine

    out = []
    for cps_min in ("1", "0"):
        monkeypatch.setenv("TBG_CPS_MIN", cps_min)
        gpu = StateMachine(batch_max=256, accounts_max=1 << 12, transfers_max=1 << 17, window_events_max=4 * 256)
        ch = Chaos(8300 + seed, n_accounts=40, id_space=800, limits=0.0, balancing=0.0, pending=0.4,
                   postvoid=0.35, linked=0.25)
        replies = []
        try:
            for w in range(14):
                if w < 2:
                    op = Operation.create_accounts
                    batches = [ch.accounts_batch(ch.rng.randint(1, 256)) for _ in range(4)]
                    for b in batches:
                        b["flags"] &= ~np.uint16(6)
                else:
                    op = Operation.create_transfers
                    batches = [ch.transfers_batch(ch.rng.choice([1, 3, 128, 256])) for _ in range(4)]
                    for b in batches:
                        b["flags"] &= ~np.uint16(0x30)
                replies.append(commit_window(gpu, op, batches, NS_PER_S))
            out.append((replies, gpu.dump_accounts().tobytes(), gpu.dump_transfers().tobytes(),
                        gpu.dump_transfer_status().tobytes(), _solver_counters(gpu)))
        finally:
            gpu.close()
    assert out[0][0] == out[1][0]
    assert out[0][1:4] == out[1][1:4]
    assert out[0][4][1] > 0 and out[1][4][1] == 0, (out[0][4], out[1][4])


@pytest.mark.gpu
@pytest.mark.parametrize("cps_min", [1, 16, 100])
def test_cps_cfg4_window(monkeypatch, cps_min):
    """cfg4's generator in 32-batch windows with pulses inside (+1 s per batch), the solver taking
    every component longer than cps_min (100: the walkers order segments of 17-100 events in
    memory, cpw.h cc_order)."""
    from tigerbeetle_amd import StateMachine

    monkeypatch.setenv("TBG_CPS_MIN", str(cps_min))
    n_acc, bm, win = 50_000, 8190, 32
    gpu = StateMachine(batch_max=bm, accounts_max=n_acc, transfers_max=2 * win * bm, window_events_max=win * bm)
    ref = OracleStateMachine(batch_max=bm)
    try:
        acc = [workload.accounts(f, min(bm, n_acc - f), seed=46) for f in range(0, n_acc, bm)]
        assert commit_window(gpu, Operation.create_accounts, acc) == oracle_batches(ref, Operation.create_accounts, acc)
        for w in range(2):
            batches = [workload.transfers_cfg4((w * win + k) * bm, bm, 46, n_acc, bm) for k in range(win)]
            g, rej = commit_ticked(gpu, Operation.create_transfers, batches, [NS_PER_S] * win)
            r, _ = oracle_ticked(ref, Operation.create_transfers, batches, [NS_PER_S] * win)
            assert not rej
            assert g == r, f"window {w}"
            assert gpu.pulse_next_timestamp() == ref.pulse_next_timestamp()
        dbg = _solver_counters(gpu)
        assert dbg[1] > 0 or cps_min >= 100, dbg
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_cps_component_above_the_solver():
    """A linked chain of 700 events (one component above CPS_NMAX = 512) in every window: the grouped
    window walks it after cc_order's in-place sort, and the window after it is grouped by the sort
    (cpw.h); replies and stores against the restatement."""
    from tigerbeetle_amd import StateMachine

    bm, n_acc = 2048, 2000
    gpu = StateMachine(batch_max=bm, accounts_max=n_acc, transfers_max=1 << 16, window_events_max=2 * bm)
    ref = OracleStateMachine(batch_max=bm)
    try:
        acc = [workload.accounts(0, n_acc, seed=5)]
        assert commit_window(gpu, Operation.create_accounts, acc) == oracle_batches(ref, Operation.create_accounts, acc)
        for w in range(4):
            batches = [workload.transfers_cfg4((w * 2 + k) * bm, bm, 5, n_acc, bm) for k in range(2)]
            b = batches[0]
            b["flags"][:699] |= np.uint16(1)   # linked: events 0..698 chain into 699
            b["flags"][699] &= ~np.uint16(1)
            g = commit_window(gpu, Operation.create_transfers, batches)
            r = oracle_batches(ref, Operation.create_transfers, batches)
            assert g == r, f"window {w}"
            assert gpu.pulse_next_timestamp() == ref.pulse_next_timestamp()
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()
