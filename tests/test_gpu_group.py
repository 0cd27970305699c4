"""The sharded group behind the StateMachine interface (include/tbg.h tbg_group_*, csrc/group.inc),
driven through the C ABI only (ctypes; no torch.distributed, no Python dispatch): G shards on one GPU
with the group's copy exchange. Replies, every pulse() decision and pulse_next_timestamp, the merged
stores and statuses, and lookups must equal the CPU restatement's on chaos streams (two-phase with
timeouts and the expiry cap, limits, balancing, chains, duplicates) and on the cfg4 / uniform shapes."""
import numpy as np
import pytest

from chaos import Chaos, run_protocol
from oracle_sm import OracleStateMachine
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import NS_PER_S, Operation


def _group(G, batch_max, accounts_max=1 << 12, transfers_max=1 << 16, window_events_max=0):
    from tigerbeetle_amd.group import GroupStateMachine

    return GroupStateMachine(G, batch_max=batch_max, accounts_max=accounts_max, transfers_max=transfers_max,
                             window_events_max=window_events_max)


def _compare_final(gpu, ref):
    ga, ra = gpu.dump_accounts(), ref.dump_accounts()
    assert ga.tobytes() == ra.tobytes()
    gt, rt = gpu.dump_transfers(), ref.dump_transfers()
    assert gt.tobytes() == rt.tobytes()
    assert np.array_equal(gpu.dump_transfer_status(), ref.dump_transfer_status())


def _lookups(gpu, ref, rng, batch_max):
    acc = ref.dump_accounts()
    xf = ref.dump_transfers()
    for op, recs in ((Operation.lookup_accounts, acc), (Operation.lookup_transfers, xf)):
        if not len(recs):
            continue
        k = rng.choice(len(recs), min(40, len(recs), batch_max - 3), replace=False)  # (input_valid: <= batch_max)
        ids = np.zeros((len(k) + 3, 2), np.uint64)
        ids[: len(k), 0], ids[: len(k), 1] = recs["id_lo"][k], recs["id_hi"][k]
        ids[len(k):, 0] = [987654321, 0, 5]  # missing ids, a zero id
        data = ids.tobytes()
        assert gpu.commit(0, 9, gpu.prepare_timestamp, op, data) == ref.commit(0, 9, ref.prepare_timestamp, op, data)


def _chaos_group(G, seed, batches, batch_max, tick_every=3, **kw):
    gpu = _group(G, batch_max)
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
            assert r1 == r2, f"G {G} seed {seed} batch {b}"
            # the next pulse() decision (state_machine.zig:589-596) reads this value
            assert gpu.pulse_next_timestamp() == ref.pulse_next_timestamp(), f"G {G} seed {seed} batch {b}"
        _compare_final(gpu, ref)
        _lookups(gpu, ref, np.random.default_rng(seed), batch_max)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("G,seed", [(2, 1), (4, 2), (8, 3)])
def test_group_chaos(G, seed):
    _chaos_group(G, seed, batches=30, batch_max=32)


@pytest.mark.gpu
def test_group_chaos_expiry_cap():
    # batch_max 8: the pulse cap binds across shards (every shard offers its cap + 1 smallest entries)
    _chaos_group(3, 300, batches=60, batch_max=8, tick_every=2, pending=0.7, postvoid=0.3, linked=0.05)


@pytest.mark.gpu
@pytest.mark.parametrize("G", [2, 4])
def test_group_cfg4_shape(G):
    """cfg4 at reduced size: two-phase with 1-60 s timeouts, posts / voids, linked chains with injected
    failures, +1 s per batch (pulses expire transfers)."""
    bm, n_acc, n_x = 512, 2000, 12 * 512
    gpu = _group(G, bm, accounts_max=4096, transfers_max=1 << 15)
    ref = OracleStateMachine(batch_max=bm)
    try:
        for first in range(0, n_acc, bm):
            ev = workload.accounts(first, min(bm, n_acc - first), seed=46)
            assert run_protocol(gpu, Operation.create_accounts, ev) == run_protocol(ref, Operation.create_accounts, ev)
        x = workload.transfers_cfg4(0, n_x, 46, n_acc, bm)
        for k, first in enumerate(range(0, n_x, bm)):
            ev = x[first: first + bm]
            p1 = gpu.prepare_timestamp
            r1 = run_protocol(gpu, Operation.create_transfers, ev, NS_PER_S)
            r2 = run_protocol(ref, Operation.create_transfers, ev, NS_PER_S)
            assert r1 == r2, f"batch {k}"
            assert gpu.prepare_timestamp == ref.prepare_timestamp != p1
            assert gpu.pulse_next_timestamp() == ref.pulse_next_timestamp(), f"batch {k}"
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("G", [2, 8])
def test_group_routed_windows(G):
    """Uniform windows through tbg_group_commit_window: the routed path (partitioned ingestion)."""
    bm, n_acc, n_x, win = 4096, 20_000, 120_000, 6
    gpu = _group(G, bm, accounts_max=n_acc // G + 4096, transfers_max=n_x // G + 16384, window_events_max=win * bm)
    ref = OracleStateMachine(batch_max=bm)
    try:
        acc = workload.accounts(0, n_acc, seed=5)
        batches = [acc[i:i + bm] for i in range(0, n_acc, bm)]
        for w0 in range(0, len(batches), win):
            got = gpu.commit_window(Operation.create_accounts, batches[w0:w0 + win])
            assert got == [run_protocol(ref, Operation.create_accounts, b) for b in batches[w0:w0 + win]]
        x = workload.transfers_uniform(0, n_x, seed=5, n_accounts=n_acc)
        batches = [x[i:i + bm] for i in range(0, n_x, bm)]
        for w0 in range(0, len(batches), win):
            got = gpu.commit_window(Operation.create_transfers, batches[w0:w0 + win])
            assert got == [run_protocol(ref, Operation.create_transfers, b) for b in batches[w0:w0 + win]]
        _compare_final(gpu, ref)
        assert all(s.stats()["sorted_transfers"] == s.stats()["transfers"] for s in gpu.shards)
    finally:
        gpu.close()
        ref.close()
