"""GPU engine vs CPU restatement on identical seeded streams: per-batch reply bytes and the final
stores (every account record, every transfer record, every pending status) must be identical."""
import numpy as np
import pytest

from chaos import Chaos, run_protocol
from oracle_sm import OracleStateMachine
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import NS_PER_S, Operation


def _compare_final(gpu, ref):
    ga, ra = gpu.dump_accounts(), ref.dump_accounts()
    assert len(ga) == len(ra)
    assert ga.tobytes() == ra.tobytes()
    gt, rt = gpu.dump_transfers(), ref.dump_transfers()
    assert len(gt) == len(rt)
    assert gt.tobytes() == rt.tobytes()
    assert np.array_equal(gpu.dump_transfer_status(), ref.dump_transfer_status())


def _chaos_run(seed, batches, batch_max, tick_every=3, **kw):
    from tigerbeetle_amd import StateMachine

    gpu = StateMachine(batch_max=batch_max, accounts_max=1 << 12, transfers_max=1 << 16)
    ref = OracleStateMachine(batch_max=batch_max)
    ch = Chaos(seed, **kw)
    try:
        for b in range(batches):
            if b < 3:
                ev, op = ch.accounts_batch(ch.rng.randint(1, batch_max)), Operation.create_accounts
            else:
                n = ch.rng.choice([1, 2, 5, batch_max // 2, batch_max])
                ev, op = ch.transfers_batch(n), Operation.create_transfers
            tick = NS_PER_S if (b % tick_every == 0) else 0
            r1 = run_protocol(gpu, op, ev, tick)
            r2 = run_protocol(ref, op, ev, tick)
            assert r1 == r2, f"seed {seed} batch {b}: gpu {np.frombuffer(r1, '<u4')} ref {np.frombuffer(r2, '<u4')}"
            # the next pulse() decision (state_machine.zig:589-596) reads this value
            assert gpu.pulse_next_timestamp() == ref.pulse_next_timestamp(), f"seed {seed} batch {b}"
        _compare_final(gpu, ref)
        return gpu.stats()
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_chaos_small_batches(seed):
    _chaos_run(seed, batches=40, batch_max=16)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_chaos_large_batches(seed):
    _chaos_run(100 + seed, batches=30, batch_max=512, n_accounts=300, id_space=4000)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_chaos_overflow_amounts(seed):
    _chaos_run(200 + seed, batches=30, batch_max=64, huge=True)


@pytest.mark.gpu
def test_chaos_expiry_cap():
    # batch_max 8 makes the pulse cap (8 expiries) bind: exercises buffer_finished and the
    # expired-post-still-inserts quirk (state_machine.zig:1689-1696).
    _chaos_run(300, batches=80, batch_max=8, tick_every=2, pending=0.7, postvoid=0.3, linked=0.05)


@pytest.mark.gpu
def test_uniform_stream_config1_shape():
    """Config-1 shape at reduced size: 10k accounts, 200k uniform transfers in 8190-event batches."""
    from tigerbeetle_amd import StateMachine

    n_acc, n_xfer, bm = 10_000, 200_000, 8190
    gpu = StateMachine(batch_max=bm, accounts_max=n_acc, transfers_max=n_xfer)
    ref = OracleStateMachine(batch_max=bm)
    try:
        for first in range(0, n_acc, bm):
            ev = workload.accounts(first, min(bm, n_acc - first), seed=42)
            assert run_protocol(gpu, Operation.create_accounts, ev) == run_protocol(ref, Operation.create_accounts, ev)
        for first in range(0, n_xfer, bm):
            ev = workload.transfers_uniform(first, min(bm, n_xfer - first), seed=42, n_accounts=n_acc)
            r1 = run_protocol(gpu, Operation.create_transfers, ev)
            r2 = run_protocol(ref, Operation.create_transfers, ev)
            assert r1 == r2 == b""
        _compare_final(gpu, ref)
        st = gpu.stats()
        assert st["walker_events"] == 0  # pure balance-apply stream: fully parallel path
    finally:
        gpu.close()
        ref.close()
