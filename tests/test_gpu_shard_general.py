"""Hash-sharded engine, general class (csrc/shard_gx.inc): balance limits and balancing
(the interleaved debit / credit checks of state_machine.zig:1509-1547), two-phase with timeouts
(:1608-1741), in-window duplicate ids, and the pulses (:1874-1929, :2018-2173) on shards. Windows
the order-free path can take still take it; the others go batch by batch through the gathered read
set and the scratch engine. Against the CPU restatement batch by batch under the harness protocol:
every reply, pulse_next_timestamp after every window, and the union of the shards' stores and
TransferPending statuses, each record on the shard its id hashes to."""
import os
import socket

import numpy as np
import pytest

from chaos import Chaos, run_protocol
from oracle_sm import OracleStateMachine, lib as oracle_lib
from test_gpu_shard import LocalShards, _compare_sharded, same_pulse_log
from test_gpu_window import oracle_batches
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import NS_PER_S, Operation


def _statuses(sh):
    rows = []
    for s in sh.shards:
        t = s.sm.dump_transfers()
        rows.append((t["timestamp"], s.sm.dump_transfer_status()))
    ts = np.concatenate([r[0] for r in rows])
    st = np.concatenate([r[1] for r in rows])
    return st[np.argsort(ts, kind="stable")]


def oracle_logged(ref, op, batches, tick_ns, log):
    """The restatement batch by batch under the harness protocol, logging (T, pulse()) before every
    batch (state_machine.zig:589-596 at prepare_timestamp = T, before that batch's pulse)."""
    out = []
    for k, ev in enumerate(batches):
        tick = tick_ns if k == 0 else 0
        T = ref.prepare_timestamp + tick + 1 + len(ev)
        log.append((T, bool(oracle_lib().tbo_pulse_needed(ref.h, T))))
        out.append(run_protocol(ref, op, ev, tick))
    return out


def _check(sh, ref):
    _compare_sharded(sh, ref)
    assert _statuses(sh).tobytes() == ref.dump_transfer_status().tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("G,seed,win,bm,general", [(2, 0, 4, 16, "window"), (3, 1, 3, 32, "window"),
                                                   (8, 2, 4, 16, "window"), (4, 3, 2, 64, "window"),
                                                   (2, 0, 4, 16, "batch"), (8, 2, 4, 16, "batch")])
def test_shard_general_chaos(G, seed, win, bm, general):
    """Chaos streams (limits, balancing, two-phase with 1-9 s timeouts, posts/voids, chains with
    rollback, duplicate ids in and across windows, invalid fields) with clock ticks, interleaved with
    plain uniform windows (the order-free path); windows outside it through the general path a whole
    window at a time (one read set, pulses inside modelled by the scratch engine) or batch by batch."""
    sh = LocalShards(G, bm, 4096, 1 << 16, win * bm, general=general)
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(7000 + seed, n_accounts=30)
    fast = general = 0
    ref_log = []
    try:
        for w in range(26):
            if w == 0 or w % 5 == 4:
                op = Operation.create_accounts  # fresh unique valid accounts: the order-free class
                batches = [workload.accounts(10**6 + w * 10**4 + k * bm, ch.rng.randint(1, bm), seed=w)
                           for k in range(win)]
            elif w == 1:
                op = Operation.create_accounts
                batches = [ch.accounts_batch(ch.rng.randint(1, bm)) for _ in range(win)]
            else:
                op = Operation.create_transfers
                batches = [ch.transfers_batch(ch.rng.choice([1, 3, bm // 2, bm])) for _ in range(win)]
            tick = 0 if op == Operation.create_accounts else ch.rng.choice([0, 0, NS_PER_S, 2 * NS_PER_S])
            g, took_fast = sh.commit_any(op, batches, tick)
            r = oracle_logged(ref, op, batches, tick, ref_log)
            assert g == r, f"window {w} (fast={took_fast})"
            # pulse() before every batch, the first one of the stream included (replica.zig:9459-9467)
            assert same_pulse_log(sh.pulse_log, ref_log), f"window {w}"
            assert sh.shards[0].pulse_next() == ref.pulse_next_timestamp(), f"window {w}"
            fast += int(took_fast)
            general += int(not took_fast)
        _check(sh, ref)
        assert fast > 0 and general > 0, (fast, general)
    finally:
        sh.close()
        ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("G", [2, 3, 8])
def test_shard_pulse_lockstep(G):
    """pulse() on the shards equals the restatement's before every batch, from the very first one
    (pulse_next_timestamp starts at timestamp_min on every engine, :2063): order-free account and
    transfer windows, then two-phase batches with timeouts and ticks (pulses that expire, pulses that
    expire nothing, and reset by post/void), then order-free windows again."""
    bm = 16
    sh = LocalShards(G, bm, 2048, 1 << 14, 4 * bm, general="batch")  # every pulse() observable
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(7300 + G, n_accounts=20, pending=0.5, postvoid=0.3, limits=0.0, balancing=0.0, linked=0.1,
               invalid=0.0)
    ref_log = []
    try:
        assert sh.shards[0].pulse(1) and oracle_lib().tbo_pulse_needed(ref.h, 1)
        plan = ([(Operation.create_accounts, [ch.accounts_batch(bm) for _ in range(2)], 0)] +
                [(Operation.create_transfers, [workload.transfers_uniform(k * bm, bm, seed=5, n_accounts=20,
                                                                          id_offset=100_000) for k in range(3)], 0)] +
                [(Operation.create_transfers, [ch.transfers_batch(ch.rng.choice([1, bm // 2, bm]))],
                  ch.rng.choice([0, NS_PER_S, 3 * NS_PER_S])) for _ in range(30)] +
                [(Operation.create_transfers, [workload.transfers_uniform(k * bm, bm, seed=6, n_accounts=20,
                                                                          id_offset=200_000) for k in range(3)], 70 * NS_PER_S)])
        for w, (op, batches, tick) in enumerate(plan):
            g, _ = sh.commit_any(op, batches, tick)
            assert g == oracle_logged(ref, op, batches, tick, ref_log), f"window {w}"
            assert same_pulse_log(sh.pulse_log, ref_log), f"window {w}"
            assert sh.shards[0].pulse_next() == ref.pulse_next_timestamp(), f"window {w}"
        assert sum(p for _, p in ref_log) >= 3, ref_log
        _check(sh, ref)
    finally:
        sh.close()
        ref.close()


@pytest.mark.gpu
def test_shard_general_expiry_cap():
    """More transfers due at once than a pulse may expire (batch_max): each shard offers its
    cap + 1 smallest, the scratch engine selects the global cap smallest, the rest follow in later
    pulses."""
    G, bm = 3, 8
    sh = LocalShards(G, bm, 1024, 1 << 14, bm)
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(7100, n_accounts=10, pending=0.9, postvoid=0.05, limits=0.0, balancing=0.0, linked=0.05, invalid=0.0)
    try:
        for b in range(40):
            if b < 2:
                ev, op = ch.accounts_batch(bm), Operation.create_accounts
            else:
                ev, op = ch.transfers_batch(bm), Operation.create_transfers
            tick = 5 * NS_PER_S if b % 8 == 7 else 0
            g, _ = sh.commit_any(op, [ev], tick)
            assert g == [run_protocol(ref, op, ev, tick)], f"batch {b}"
            assert sh.shards[0].pulse_next() == ref.pulse_next_timestamp()
        _check(sh, ref)
        assert (ref.dump_transfer_status() == 4).sum() > bm  # expired, over several capped pulses
    finally:
        sh.close()
        ref.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dist_stream(seed, bm):
    ch = Chaos(seed, n_accounts=20)
    out = []
    for b in range(30):
        if b < 2:
            out.append((Operation.create_accounts, ch.accounts_batch(bm), 0))
        else:
            out.append((Operation.create_transfers, ch.transfers_batch(ch.rng.choice([1, bm // 2, bm])),
                        ch.rng.choice([0, NS_PER_S])))
    return out


def _rank_main(rank, world, port, seed, bm, out_dir):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tigerbeetle_amd.sharding import ShardedStateMachine, exchange_gloo

    sh = ShardedStateMachine(world, rank, exchange_gloo, batch_max=bm, accounts_max=1024, transfers_max=1 << 14,
                             window_events_max=bm)
    ts, replies, pulses = 0, [], []
    for op, ev, tick in _dist_stream(seed, bm):
        ts += tick + 1 + len(ev)
        pulses.append(sh.pulse(ts))  # pulse() before every batch, the first one included
        d_ev = torch.from_numpy(np.frombuffer(ev.tobytes(), np.uint8).copy()).cuda()
        torch.cuda.synchronize()
        replies.append(sh.commit_general(op, d_ev.data_ptr(), len(ev), ts).hex())
    np.save(os.path.join(out_dir, f"acc{rank}.npy"), sh.sm.dump_accounts())
    np.save(os.path.join(out_dir, f"xfer{rank}.npy"), sh.sm.dump_transfers())
    np.save(os.path.join(out_dir, f"st{rank}.npy"), sh.sm.dump_transfer_status())
    import json

    with open(os.path.join(out_dir, f"rep{rank}.json"), "w") as f:
        json.dump({"replies": replies, "pulses": pulses}, f)
    sh.close()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_shard_general_two_rank_gloo(tmp_path):
    """Two processes (one shard each, sharing cuda:0), every exchange a torch.distributed
    all-reduce: each rank returns every batch's reply, equal to the restatement's."""
    import json

    import torch.multiprocessing as mp

    world, seed, bm = 2, 7200, 16
    mp.spawn(_rank_main, args=(world, _free_port(), seed, bm, str(tmp_path)), nprocs=world, join=True)
    ref = OracleStateMachine(batch_max=bm)
    try:
        log = []
        expect = [oracle_logged(ref, op, [ev], tick, log)[0].hex() for op, ev, tick in _dist_stream(seed, bm)]
        for r in range(world):
            with open(tmp_path / f"rep{r}.json") as f:
                got = json.load(f)
            assert got["replies"] == expect
            assert got["pulses"] == [p for _, p in log]
        assert log[0][1]  # the first pulse() is true
        acc = np.concatenate([np.load(tmp_path / f"acc{r}.npy") for r in range(world)])
        xfer = np.concatenate([np.load(tmp_path / f"xfer{r}.npy") for r in range(world)])
        st = np.concatenate([np.load(tmp_path / f"st{r}.npy") for r in range(world)])
        o = np.argsort(xfer["timestamp"], kind="stable")
        assert acc[np.argsort(acc["timestamp"], kind="stable")].tobytes() == ref.dump_accounts().tobytes()
        assert xfer[o].tobytes() == ref.dump_transfers().tobytes()
        assert st[o].tobytes() == ref.dump_transfer_status().tobytes()
    finally:
        ref.close()


def _general_stream(sh, ref, op, batches, ticks, win=1):
    """`win` batches per window (each with its own tick) through LocalShards.commit_any, the
    restatement batch by batch."""
    for w0 in range(0, len(batches), win):
        bs, tk = batches[w0:w0 + win], ticks[w0:w0 + win]
        g, _ = sh.commit_any(op, bs, ticks=tk)
        assert g == [run_protocol(ref, op, ev, t) for ev, t in zip(bs, tk)], f"window at batch {w0}"
        assert sh.shards[0].pulse_next() == ref.pulse_next_timestamp()


@pytest.mark.gpu
@pytest.mark.parametrize("G,win", [(2, 1), (4, 1), (8, 1), (2, 6), (8, 6)])
def test_shard_cfg3_shape(G, win):
    """cfg3's shape (Zipf(1.2) debits over accounts with debits_must_not_exceed_credits, funded from
    treasury accounts) on G shards: every transfer batch reads balances across shards; windows of
    `win` batches (one read set per window)."""
    bm, n_acc, top, treasury = 512, 3000, 100, 50
    sh = LocalShards(G, bm, 4096, 1 << 15, win * bm)
    ref = OracleStateMachine(batch_max=bm)
    try:
        acc = workload.accounts_cfg3(0, n_acc + treasury, 45, n_acc, top)
        _general_stream(sh, ref, Operation.create_accounts, [acc[i:i + bm] for i in range(0, len(acc), bm)],
                        [0] * ((len(acc) + bm - 1) // bm))
        fund = workload.funding_cfg3(0, n_acc, 45, n_acc, treasury, 20_000, 10**15)
        _general_stream(sh, ref, Operation.create_transfers, [fund[i:i + bm] for i in range(0, len(fund), bm)],
                        [0] * ((len(fund) + bm - 1) // bm))
        xf = workload.transfers_zipf(0, 6 * bm, 45, n_acc, workload.zipf_cdf(n_acc))
        _general_stream(sh, ref, Operation.create_transfers, [xf[i:i + bm] for i in range(0, len(xf), bm)], [0] * 6,
                        win)
        _check(sh, ref)
    finally:
        sh.close()
        ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("G,win", [(2, 1), (4, 1), (8, 1), (2, 8), (8, 8)])
def test_shard_cfg4_shape(G, win):
    """cfg4's shape (30 % pending with 1-60 s timeouts, posts / voids of earlier pending transfers,
    chains with injected failures), +1 s per batch so a pulse with expiries precedes most batches;
    windows of `win` batches (the pulses inside modelled by the scratch engine)."""
    bm, n_acc = 512, 2000
    sh = LocalShards(G, bm, 4096, 1 << 15, win * bm)
    ref = OracleStateMachine(batch_max=bm)
    try:
        acc = workload.accounts(0, n_acc, seed=46)
        _general_stream(sh, ref, Operation.create_accounts, [acc[i:i + bm] for i in range(0, n_acc, bm)],
                        [0] * ((n_acc + bm - 1) // bm))
        xf = workload.transfers_cfg4(0, 40 * bm, 46, n_acc, bm)
        _general_stream(sh, ref, Operation.create_transfers, [xf[i:i + bm] for i in range(0, len(xf), bm)],
                        [NS_PER_S] * 40, win)
        _check(sh, ref)
        assert (ref.dump_transfer_status() == 4).sum() > 0  # expiries ran on the shards
    finally:
        sh.close()
        ref.close()


def _fallbacks(sh):
    return {k: sum(s.gw_fallbacks[k] for s in sh.shards) for k in ("due_overflow", "rejected")}


@pytest.mark.gpu
def test_shard_general_window_due_overflow_falls_back():
    """A shard with more entries due in a window's span than due_cap (here 3): the window path is
    abandoned after phase 1's counts (nothing written) and the window goes batch by batch, each pulse
    selecting among every shard's cap + 1 smallest. Replies, pulse_next_timestamp after every window,
    and the union of the stores and statuses equal the restatement's."""
    G, bm, win = 3, 16, 4
    sh = LocalShards(G, bm, 2048, 1 << 14, win * bm, general="window")
    for s in sh.shards:
        s.due_cap = 3
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(7400, n_accounts=12, pending=0.8, postvoid=0.1, limits=0.0, balancing=0.0, linked=0.05, invalid=0.0)
    ref_log = []
    try:
        for w in range(14):
            op = Operation.create_accounts if w < 1 else Operation.create_transfers
            batches = [ch.accounts_batch(bm) if w < 1 else ch.transfers_batch(bm) for _ in range(win)]
            tick = 0 if w < 2 else 3 * NS_PER_S
            g, _ = sh.commit_any(op, batches, tick)
            assert g == oracle_logged(ref, op, batches, tick, ref_log), f"window {w}"
            assert sh.shards[0].pulse_next() == ref.pulse_next_timestamp(), f"window {w}"
        _check(sh, ref)
        assert _fallbacks(sh)["due_overflow"] > 0
        assert (ref.dump_transfer_status() == 4).sum() > 0
    finally:
        sh.close()
        ref.close()


@pytest.mark.gpu
def test_shard_general_window_rejected_by_scratch_falls_back():
    """Windows that read balances (limit flags on most accounts) with pulses due inside them (a tick
    before every batch, 1-9 s timeouts): the scratch engine rejects them after modelling nothing
    (TBG_E_WINDOW, the apply kernels check its verdict on the device), no shard applies anything, and
    the window goes batch by batch. Stores, statuses and pulse_next_timestamp after every window equal
    the restatement's."""
    G, bm, win = 2, 16, 4
    sh = LocalShards(G, bm, 2048, 1 << 14, win * bm, general="window")
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(7500, n_accounts=16, pending=0.5, postvoid=0.2, limits=0.7, balancing=0.1, linked=0.1)
    try:
        for w in range(16):
            op = Operation.create_accounts if w < 1 else Operation.create_transfers
            batches = [ch.accounts_batch(bm) if w < 1 else ch.transfers_batch(bm) for _ in range(win)]
            ticks = [0] * win if w < 1 else [NS_PER_S] * win
            g, _ = sh.commit_any(op, batches, ticks=ticks)
            assert g == [run_protocol(ref, op, ev, t) for ev, t in zip(batches, ticks)], f"window {w}"
            assert sh.shards[0].pulse_next() == ref.pulse_next_timestamp(), f"window {w}"
        _check(sh, ref)
        assert _fallbacks(sh)["rejected"] > 0
    finally:
        sh.close()
        ref.close()


@pytest.mark.gpu
def test_shard_general_window_large_read_set():
    """A window of 4 x 4096 events (more than one workgroup's worth of new records: the apply's
    device-wide scan) whose read set spans most of 20000 accounts, two-phase and limits mixed in,
    at G = 2 and 8 against the restatement."""
    bm, win = 4096, 4
    for G in (2, 8):
        sh = LocalShards(G, bm, 32768, 1 << 17, win * bm, general="window")
        ref = OracleStateMachine(batch_max=bm)
        try:
            acc = workload.accounts(0, 20000, seed=48)
            for k in range(0, 20000, bm):
                ev = acc[k:k + bm]
                g, _ = sh.commit_any(Operation.create_accounts, [ev], 0)
                assert g == [run_protocol(ref, Operation.create_accounts, ev, 0)]
            xf = workload.transfers_cfg4(0, 3 * win * bm, 48, 20000, bm)
            for w in range(3):
                batches = [xf[(w * win + k) * bm:(w * win + k + 1) * bm] for k in range(win)]
                ticks = [NS_PER_S] * win
                g, took_fast = sh.commit_any(Operation.create_transfers, batches, ticks=ticks)
                assert not took_fast
                assert g == [run_protocol(ref, Operation.create_transfers, ev, t) for ev, t in zip(batches, ticks)], w
                assert sh.shards[0].pulse_next() == ref.pulse_next_timestamp()
            assert max(s._gw_n[0] for s in sh.shards) > 8192
            _check(sh, ref)
            assert _fallbacks(sh) == {"due_overflow": 0, "rejected": 0}
        finally:
            sh.close()
            ref.close()
