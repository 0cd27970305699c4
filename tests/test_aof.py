"""The wire steps either side of the commit path:

- the client's reply Demuxer (state_machine.zig:133-176) over the C ABI, with the reference's own
  property test (:3667-3709: random result sets, requests of random strides; every decoded result
  lies inside its request) plus exact reconstruction of the reply;
- AOF replay (aof.zig:23-55, Iterator.next :176-228): logs written in the reference's on-disk format
  by running the CPU restatement under the replica protocol (pulses are prepares of their own), then
  replayed into the GPU engine (checksums verified on the GPU, windows in log mode): the stores,
  statuses, pulse_next_timestamp and digest equal the restatement's; every iterator error (short
  read, magic, header checksum, body checksum, hash chain) stops the replay at the right entry with
  exactly the entries before it applied."""
import random
import struct

import numpy as np
import pytest

from aof_writer import MAGIC, SECTOR, VSR_PULSE, AofLog, prepare_header, record
from chaos import Chaos
from oracle_sm import OracleStateMachine
from test_checksum import oracle_checksum
from test_gpu_parity import _compare_final
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import NS_PER_S, Operation

RESULT = np.dtype([("index", "<u4"), ("result", "<u4")])


def test_demuxer_reference_property():
    from tigerbeetle_amd.demux import Demuxer

    rng = random.Random(42)
    for operation in (Operation.create_accounts, Operation.create_transfers):
        for _ in range(100):
            n_max = 8190
            idx = [i for i in range(n_max) if rng.random() < 0.5]
            res = np.zeros(len(idx), RESULT)
            res["index"] = idx
            dm = Demuxer(operation, res.tobytes())
            event_count = max(1, rng.randint(0, n_max))
            off, got = 0, []
            while off < event_count:
                size = max(1, rng.randint(0, event_count - off))
                r = np.frombuffer(dm.decode(off, size), RESULT)
                assert (r["index"] < size).all() and (r["result"] == 0).all()
                got += [off + int(i) for i in r["index"]]
                off += size
            assert got == [i for i in idx if i < event_count]


def test_demuxer_unbatched_operations():
    from tigerbeetle_amd.demux import Demuxer

    body = bytes(range(256)) * 2  # two 128-byte results
    dm = Demuxer(Operation.lookup_accounts, body)
    assert dm.decode(0, 5) == body
    with pytest.raises(RuntimeError):
        Demuxer(Operation.lookup_transfers, body).decode(1, 1)
    with pytest.raises(RuntimeError):
        Demuxer(Operation.pulse, b"")


def _iterate(data, validate_chain=True):
    """The reference iterator restated (test infrastructure): yields (header, body), raises the
    iterator's error name."""
    off, last = 0, None
    while off < len(data):
        buf = data[off: off + 4096 + (1 << 20)]
        size = struct.unpack_from("<I", buf, 4096 + 96)[0] if len(buf) >= 4096 + 256 else 0
        disk = (4096 + size + SECTOR - 1) // SECTOR * SECTOR
        if len(buf) < 4096 + 256 or len(buf) < disk:
            raise ValueError("AOFShortRead")
        if int.from_bytes(buf[:16], "little") != MAGIC:
            raise ValueError("AOFMagicNumberMismatch")
        h, body = buf[4096: 4096 + 256], buf[4096 + 256: 4096 + size]
        if oracle_checksum(h[16:]) != int.from_bytes(h[:16], "little"):
            raise ValueError("AOFChecksumMismatch")
        if oracle_checksum(body) != int.from_bytes(h[32:48], "little"):
            raise ValueError("AOFBodyChecksumMismatch")
        if validate_chain and last is not None and int.from_bytes(h[128:144], "little") != last:
            raise ValueError("AOFChecksumChainMismatch")
        last = int.from_bytes(h[:16], "little")
        yield h, body
        off += disk


def _requests(seed, n, bm):
    ch = Chaos(seed, pending=0.5, postvoid=0.4, linked=0.15)
    out = []
    for b in range(n):
        if b < 3:
            out.append((Operation.create_accounts, ch.accounts_batch(ch.rng.randint(1, bm))))
        else:
            out.append((Operation.create_transfers, ch.transfers_batch(ch.rng.choice([1, 3, bm // 2, bm]))))
    return out


def _realtime(k, ts):
    return ts + NS_PER_S * 3 // 2 if k % 4 == 0 else 0  # a 1.5 s clock jump every fourth request


def test_aof_writer_matches_the_iterator():
    ref = OracleStateMachine(batch_max=16)
    try:
        log, _ = record(ref, _requests(1, 20, 16), _realtime)
    finally:
        ref.close()
    entries = list(_iterate(bytes(log.data)))
    assert len(entries) == len(log.entries)
    assert any(h[252] == VSR_PULSE for h, _ in entries)


def apply_log(ref, entries):
    """The restatement applying log entries [(header, body)] as a replica commits its journal."""
    for h, body in entries:
        operation, T = h[252], struct.unpack_from("<Q", h, 240)[0]
        if operation == VSR_PULSE:
            ref.commit(0, 0, T, Operation.pulse, b"")
        elif operation in (Operation.create_accounts, Operation.create_transfers):
            ref.prepare_timestamp = T
            ref.commit(0, 0, T, Operation(operation), body)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,bm,n", [(0, 16, 60), (1, 64, 50), (2, 8, 80)])
def test_aof_replay_matches_restatement(seed, bm, n):
    from tigerbeetle_amd import StateMachine

    ref = OracleStateMachine(batch_max=bm)
    gpu = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 16, window_events_max=32 * bm)
    try:
        log, _ = record(ref, _requests(300 + seed, n, bm), _realtime)
        st = gpu.aof_replay(bytes(log.data))
        assert st["error"] is None, st
        n_pulse = sum(1 for _, h in log.entries if h[252] == VSR_PULSE)
        assert st["pulses"] == n_pulse > 0 and st["prepares"] == n and st["entries"] == len(log.entries)
        assert st["windows"] < n  # runs of prepares between pulses went as windows
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_aof_replay_cfg4_stream():
    """cfg4 batches (two-phase, 1-60 s timeouts, chains) a second apart: a pulse prepare before most
    batches of the log, windows of one batch between them."""
    from tigerbeetle_amd import StateMachine

    n_acc, bm, nb = 2000, 8190, 12
    ref = OracleStateMachine(batch_max=bm)
    gpu = StateMachine(batch_max=bm, accounts_max=n_acc, transfers_max=nb * bm, window_events_max=8 * bm)
    try:
        reqs = [(Operation.create_accounts, workload.accounts(0, n_acc, seed=46))]
        reqs += [(Operation.create_transfers, workload.transfers_cfg4(b * bm, bm, 46, n_acc, bm)) for b in range(nb)]
        log, _ = record(ref, reqs, lambda k, ts: ts + NS_PER_S)
        st = gpu.aof_replay(bytes(log.data))
        assert st["error"] is None and st["pulses"] >= 3, st
        assert st["events"] == n_acc + nb * bm
        _compare_final(gpu, ref)
        assert gpu.digest()[3] == ref.pulse_next_timestamp()
    finally:
        gpu.close()
        ref.close()


def _corrupt(kind, log, m):
    data = bytearray(log.data)
    off, h = log.entries[m]
    if kind == "body":
        size = struct.unpack_from("<I", h, 96)[0]
        assert size > 256
        data[off + 4096 + 256 + (size - 256) // 2] ^= 0x40
    elif kind == "header":
        data[off + 4096 + 248] ^= 1  # request
    elif kind == "magic":
        data[off + 3] ^= 1
    elif kind == "chain":
        h2 = bytearray(h)
        h2[128] ^= 1  # parent, then a valid checksum over the edited header
        h2[:16] = oracle_checksum(bytes(h2[16:])).to_bytes(16, "little")
        data[off + 4096: off + 4096 + 256] = h2
    elif kind == "short":
        data = data[: off + 4096 + 200]
    return bytes(data)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,error", [("body", "AOFBodyChecksumMismatch"), ("header", "AOFChecksumMismatch"),
                                        ("magic", "AOFMagicNumberMismatch"), ("chain", "AOFChecksumChainMismatch"),
                                        ("short", "AOFShortRead")])
def test_aof_replay_stops_at_the_bad_entry(kind, error):
    from tigerbeetle_amd import StateMachine

    bm = 16
    ref = OracleStateMachine(batch_max=bm)
    try:
        log, _ = record(ref, _requests(77, 40, bm), _realtime)
    finally:
        ref.close()
    # a create_transfers entry past the accounts (its body is not empty)
    m = next(k for k, (_, h) in enumerate(log.entries) if k > 20 and h[252] == Operation.create_transfers)
    data = _corrupt(kind, log, m)
    gpu = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 16, window_events_max=16 * bm)
    want = OracleStateMachine(batch_max=bm)
    try:
        st = gpu.aof_replay(data)
        assert st["error"] == error and st["error_entry"] == m, st
        assert st["entries"] == m
        prefix = [(bytes(log.data[o + 4096: o + 4096 + 256]),
                   bytes(log.data[o + 4096 + 256: o + 4096 + struct.unpack_from("<I", h, 96)[0]]))
                  for o, h in log.entries[:m]]
        apply_log(want, prefix)
        _compare_final(gpu, want)
        if kind == "chain":  # without the chain check the file replays whole
            gpu2 = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 16, window_events_max=16 * bm)
            try:
                from tigerbeetle_amd._lib import AOF_NO_CHAIN

                st2 = gpu2.aof_replay(data, AOF_NO_CHAIN)
                assert st2["error"] is None and st2["entries"] == len(log.entries)
            finally:
                gpu2.close()
    finally:
        gpu.close()
        want.close()


@pytest.mark.gpu
def test_aof_replay_skips_control_plane_and_queries():
    """A register prepare (vsr-reserved) and a lookup prepare change nothing and are skipped."""
    from tigerbeetle_amd import StateMachine

    bm = 16
    ref = OracleStateMachine(batch_max=bm)
    gpu = StateMachine(batch_max=bm, accounts_max=1 << 10, transfers_max=1 << 12)
    try:
        log = AofLog()
        ch = Chaos(5, pending=0.0, postvoid=0.0, limits=0.0)
        log.append(2, b"", 10)  # register
        acc = ch.accounts_batch(bm)
        log.append(int(Operation.create_accounts), acc.tobytes(), 100)
        log.append(int(Operation.lookup_accounts), bytes(16), 200)
        xf = ch.transfers_batch(bm)
        log.append(int(Operation.create_transfers), xf.tobytes(), 300)
        st = gpu.aof_replay(bytes(log.data))
        assert st["error"] is None and st["skipped"] == 2 and st["prepares"] == 2, st
        ref.commit(0, 0, 100, Operation.create_accounts, acc.tobytes())
        ref.commit(0, 0, 300, Operation.create_transfers, xf.tobytes())
        _compare_final(gpu, ref)
        assert prepare_header(1, b"", 1, 1, 0)[114] == 6
    finally:
        gpu.close()
        ref.close()
