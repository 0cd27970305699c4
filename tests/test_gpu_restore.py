"""The rest of the StateMachine surface a replica drives: open from the forest's objects
(state_machine.zig:527-541), reset (:486-501), prefetch completion (:598-648), compact/checkpoint
barriers (:1148-1188), the static input_valid (:543-572, called as StateMachine.input_valid at
vsr/replica.zig:4855), and the whole-state digest checked against the CPU restatement's dumps."""
import ctypes

import numpy as np
import pytest

from chaos import Chaos, run_protocol
from oracle_sm import OracleStateMachine, lib as olib
from test_gpu_parity import _compare_final
from tigerbeetle_amd import _lib
from tigerbeetle_amd.digest import digest
from tigerbeetle_amd.types import NS_PER_S, Operation


def _oracle_status(ref, xfers):
    return np.array([olib().tbo_pending_status(ref.h, int(ts)) for ts in xfers["timestamp"]], np.uint8)


def _stream(ch, b, bm):
    if b < 3:
        return ch.accounts_batch(ch.rng.randint(1, bm)), Operation.create_accounts
    return ch.transfers_batch(ch.rng.choice([1, 3, bm // 2, bm])), Operation.create_transfers


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_digest_matches_oracle_dumps(seed):
    from tigerbeetle_amd import StateMachine

    bm = 32
    gpu = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 15)
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(3100 + seed)
    try:
        for b in range(30):
            ev, op = _stream(ch, b, bm)
            tick = NS_PER_S if b % 3 == 0 else 0
            assert run_protocol(gpu, op, ev, tick) == run_protocol(ref, op, ev, tick)
            if b % 10 == 9:
                rx = ref.dump_transfers()
                want = digest(ref.dump_accounts(), rx, _oracle_status(ref, rx), ref.pulse_next_timestamp())
                assert gpu.digest() == want, b
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_open_from_forest_objects(seed):
    """A replica restarts: a new engine opens from the objects (records + TransferPending statuses)
    and then commits the same stream as the engine that kept running: identical replies, stores and
    digests."""
    from tigerbeetle_amd import StateMachine

    bm = 32
    a = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 15)
    b_ = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 15)
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(3200 + seed)
    try:
        for b in range(20):
            ev, op = _stream(ch, b, bm)
            tick = NS_PER_S if b % 3 == 0 else 0
            assert run_protocol(a, op, ev, tick) == run_protocol(ref, op, ev, tick)
        rx = ref.dump_transfers()
        b_.open(ref.dump_accounts(), rx, _oracle_status(ref, rx))
        b_.prepare_timestamp = a.prepare_timestamp
        b_.commit_timestamp = a.commit_timestamp
        da, db = a.digest(), b_.digest()
        assert da[:3] == db[:3] and db[3] == 1  # pulse_next_timestamp restarts at timestamp_min
        st = b_.stats()
        assert st["accounts"] == len(ref.dump_accounts()) and st["transfers"] == len(rx)
        # the harness pulses at the same T as the batch, so the restarted engine's first (extra)
        # pulse changes nothing but pulse_next; the stores stay identical
        for b in range(20, 45):
            ev, op = _stream(ch, b, bm)
            tick = NS_PER_S if b % 3 == 0 else 0
            r = run_protocol(ref, op, ev, tick)
            assert run_protocol(a, op, ev, tick) == r
            assert run_protocol(b_, op, ev, tick) == r
        assert a.digest() == b_.digest()
        _compare_final(b_, ref)
    finally:
        a.close()
        b_.close()
        ref.close()


@pytest.mark.gpu
def test_reset_then_replay():
    from tigerbeetle_amd import StateMachine

    bm = 32
    gpu = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 15)
    try:
        runs = []
        for _ in range(2):
            ch = Chaos(3300)
            replies = []
            for b in range(25):
                ev, op = _stream(ch, b, bm)
                replies.append(run_protocol(gpu, op, ev, NS_PER_S if b % 3 == 0 else 0))
            runs.append((replies, gpu.digest()))
            gpu.reset()
            st = gpu.stats()
            assert st["accounts"] == 0 and st["transfers"] == 0 and st["pulse_next_timestamp"] == 1
        assert runs[0] == runs[1]
    finally:
        gpu.close()


@pytest.mark.gpu
def test_prefetch_poll_compact_checkpoint():
    from tigerbeetle_amd import StateMachine

    bm = 64
    gpu = StateMachine(batch_max=bm, accounts_max=1 << 10, transfers_max=1 << 12)
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(3400)
    try:
        assert gpu.prefetch_done()  # nothing in flight
        for b in range(8):
            ev, op = _stream(ch, b, bm)
            data = ev.tobytes()
            for sm in (gpu, ref):
                sm.prepare_timestamp += 1
                sm.prepare(op, data)
                sm.prefetch_timestamp = sm.prepare_timestamp
                sm.prefetch(b + 1, op, data)
            while not gpu.prefetch_done():  # the replica fires the callback on a later tick
                pass
            T = gpu.prepare_timestamp
            assert gpu.commit(0, b + 1, T, op, data) == ref.commit(0, b + 1, T, op, data)
            gpu.compact(b + 1)
        gpu.checkpoint()
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


def test_input_valid_is_static():
    """No engine needed, as the replica calls it (batch_max 8190)."""
    L = _lib.lib()
    assert L.tbg_input_valid(None, int(Operation.create_transfers), 8190 * 128) == 1
    assert L.tbg_input_valid(None, int(Operation.create_transfers), 8191 * 128) == 0
    assert L.tbg_input_valid(None, int(Operation.create_accounts), 0) == 1
    assert L.tbg_input_valid(None, int(Operation.pulse), 0) == 1
    assert L.tbg_input_valid(None, int(Operation.pulse), 128) == 0
    assert L.tbg_input_valid(None, int(Operation.lookup_accounts), 17) == 0


def test_digest_twin_is_position_sensitive():
    from tigerbeetle_amd.types import ACCOUNT_DTYPE

    a = np.zeros(3, ACCOUNT_DTYPE)
    a["ledger"] = [1, 2, 3]
    d1 = digest(a, a[:0], np.zeros(0, np.uint8), 5)
    d2 = digest(a[::-1].copy(), a[:0], np.zeros(0, np.uint8), 5)
    assert d1[0] != d2[0] and d1[1:] == d2[1:]
    assert ctypes.sizeof(ctypes.c_uint64) == 8
