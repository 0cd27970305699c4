"""The rest of the StateMachine surface on a hash-sharded engine, against the CPU restatement:

- open (state_machine.zig:527-541): every shard is handed the forest's whole object set (accounts,
  transfers, TransferPending statuses, account_balances rows) and keeps what it owns; the stream then
  continues on the shards exactly as on the restatement;
- lookup_accounts / lookup_transfers (:1309-1344) and get_account_transfers / get_account_balances
  (:786-996, 1346-1419): gathered from the owners (csrc/shard_read.inc), byte-identical replies;
- historical_balance rows (:1806-1841) on shards: history accounts leave the order-free class, the
  general path writes the rows beside the owned records;
- the write-back stream per shard (lsm/groove.zig:905-1000): after every window the union of the
  shards' logs covers every changed record, each equal to the restatement's;
at G = 2, 3, 8 shards on one GPU, and two processes with real gloo all-reduces."""
import json
import os
import socket

import numpy as np
import pytest

from chaos import Chaos, run_protocol
from oracle_sm import OracleStateMachine
from test_gpu_queries import _filter
from test_gpu_shard import LocalShards
from test_gpu_shard_general import _check, oracle_logged
from tigerbeetle_amd.types import NS_PER_S, Operation

READS = (Operation.lookup_accounts, Operation.lookup_transfers)
QUERIES = (Operation.get_account_transfers, Operation.get_account_balances)


def _ids(rng, pool, k, extra):
    ids = [rng.choice(pool) for _ in range(k)] + [rng.randint(1, extra) for _ in range(k // 4)]
    rng.shuffle(ids)
    out = np.zeros(2 * len(ids), np.uint64)
    out[0::2] = ids
    return out.tobytes()


def _reads(sh, ref, rng, bm, k=12):
    acc = [int(x) for x in ref.dump_accounts()["id_lo"]]
    xf = [int(x) for x in ref.dump_transfers()["id_lo"]]
    ts = [int(t) for t in ref.dump_transfers()["timestamp"]]
    nonempty = 0
    for _ in range(k):
        for op, pool in ((Operation.lookup_accounts, acc), (Operation.lookup_transfers, xf)):
            if not pool:
                continue
            q = _ids(rng, pool, rng.randint(1, bm // 2), 5000)
            assert sh.read(op, q) == ref.commit(0, 1, ref.prepare_timestamp, op, q), op.name
        q = _filter(rng, 40, ts, bm)
        for op in QUERIES:
            g, r = sh.read(op, q), ref.commit(0, 1, ref.prepare_timestamp, op, q)
            assert g == r, f"{op.name}: {len(g)} vs {len(r)} bytes"
            nonempty += int(len(r) > 0)
    return nonempty


def _stream(ch, bm, n):
    for w in range(n):
        if w < 2 or w % 6 == 5:
            yield Operation.create_accounts, [ch.accounts_batch(ch.rng.randint(1, bm))], 0
        else:
            yield (Operation.create_transfers, [ch.transfers_batch(ch.rng.choice([1, bm // 2, bm]))],
                   ch.rng.choice([0, 0, NS_PER_S]))


@pytest.mark.gpu
@pytest.mark.parametrize("G,seed", [(2, 0), (3, 1), (8, 2)])
def test_shard_open_reads_history(G, seed):
    """A restatement-built state (history accounts, limits, two-phase with timeouts) opened on G
    shards, then the stream continues on both; lookups and queries (random filters, both directions,
    limits around batch_max, invalid ones) gathered from the owners after every few batches."""
    import random

    bm = 32
    rng = random.Random(8000 + seed)
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(8000 + seed, n_accounts=40, id_space=2000, history=0.3)
    for op, batches, tick in _stream(ch, bm, 14):
        oracle_logged(ref, op, batches, tick, [])
    sh = LocalShards(G, bm, 2048, 1 << 14, bm)
    try:
        x = ref.dump_transfers()
        st = ref.dump_transfer_status()
        hist = np.frombuffer(ref.dump_account_balances().tobytes(), np.uint8)
        for s in sh.shards:
            s.open(ref.dump_accounts(), x, st, hist)
        sh.prepare_timestamp = ref.prepare_timestamp
        _check(sh, ref)
        assert len(hist) > 0
        nonempty = _reads(sh, ref, rng, bm)
        # (no pulse-log comparison here: an opened state machine starts at pulse_next =
        # timestamp_min, :2063, the restatement that never restarted does not; the pulses that
        # follow expire the same transfers)
        for w, (op, batches, tick) in enumerate(_stream(ch, bm, 24)):
            g, _ = sh.commit_any(op, batches, tick)
            assert g == oracle_logged(ref, op, batches, tick, []), f"batch {w}"
            if w % 6 == 3:
                nonempty += _reads(sh, ref, rng, bm, 4)
        _check(sh, ref)
        nonempty += _reads(sh, ref, rng, bm)
        assert nonempty > 5
    finally:
        sh.close()
        ref.close()


def _by_id(arr):
    return {(int(r["id_lo"]), int(r["id_hi"])): r.tobytes() for r in arr}


@pytest.mark.gpu
@pytest.mark.parametrize("G,seed", [(2, 0), (3, 1), (8, 2)])
def test_shard_change_log(G, seed):
    """Per shard write-back streams: order-free windows and general-path batches (limits,
    two-phase, expiries by pulses) — after each window, every logged record equals the
    restatement's, every changed account / inserted transfer / changed TransferPending row is in
    exactly the log of the shard that owns it."""
    from tigerbeetle_amd import workload
    from tigerbeetle_amd.sharding import shard_of

    bm = 32
    sh = LocalShards(G, bm, 2048, 1 << 14, 4 * bm, change_log=True)
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(8100 + seed, n_accounts=30, id_space=3000)
    rows_seen = 0
    try:
        for w in range(22):
            acc0, x0 = ref.dump_accounts(), ref.dump_transfers()
            st0 = dict(zip(x0["timestamp"].tolist(), ref.dump_transfer_status().tolist()))
            if w < 2:
                op, batches, tick = Operation.create_accounts, [ch.accounts_batch(bm)], 0
            elif w % 5 == 4:  # an order-free window (the fast path)
                op, tick = Operation.create_transfers, 0
                batches = [workload.transfers_uniform(k * bm, bm, seed=w, n_accounts=30, id_offset=10**6 + w * 1000)
                           for k in range(3)]
            else:
                op, batches, tick = (Operation.create_transfers, [ch.transfers_batch(ch.rng.choice([1, bm // 2, bm]))],
                                     ch.rng.choice([0, NS_PER_S, 2 * NS_PER_S]))
            sh.logs.clear()
            g, _ = sh.commit_any(op, batches, tick)
            assert g == [run_protocol(ref, op, ev, tick if k == 0 else 0) for k, ev in enumerate(batches)]
            acc1, x1 = ref.dump_accounts(), ref.dump_transfers()
            st1 = dict(zip(x1["timestamp"].tolist(), ref.dump_transfer_status().tolist()))
            after, before = _by_id(acc1), _by_id(acc0)
            x1_by_id = _by_id(x1)
            changed_acc = {k for k, v in after.items() if before.get(k) != v}
            new_x = {(int(r["id_lo"]), int(r["id_hi"])) for r in x1[len(x0):]}
            changed_rows = {ts for ts, v in st1.items() if v != 0 and st0.get(ts) != v}
            # the union of every commit call's log (pulses and batches), each record from its owner;
            # a later call's record supersedes an earlier one's
            got_acc, got_x, got_rows = {}, {}, {}
            for r, la, lx, rows in sh.logs:
                for a in la:
                    k = (int(a["id_lo"]), int(a["id_hi"]))
                    assert shard_of(k[0], k[1], G) == r
                    got_acc[k] = a.tobytes()
                for t in lx:
                    k = (int(t["id_lo"]), int(t["id_hi"]))
                    assert shard_of(k[0], k[1], G) == r
                    got_x[k] = t.tobytes()
                for row in rows:
                    got_rows[int(row["timestamp"])] = int(row["status"])
            for k, v in got_acc.items():
                assert after[k] == v, f"window {w}: logged account {k}"
            for k, v in got_x.items():
                assert x1_by_id[k] == v, f"window {w}: logged transfer {k}"
            for ts, v in got_rows.items():
                assert st1[ts] == v, f"window {w}: row {ts}"
            assert changed_acc <= set(got_acc), f"window {w}: {sorted(changed_acc - set(got_acc))[:4]}"
            assert new_x == set(got_x), f"window {w}"
            assert changed_rows <= set(got_rows), f"window {w}: {sorted(changed_rows - set(got_rows))[:4]}"
            rows_seen += len(got_rows)
        _check(sh, ref)
        assert rows_seen > 0
    finally:
        sh.close()
        ref.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dist_plan(seed, bm):
    ch = Chaos(seed, n_accounts=30, id_space=2000, history=0.3)
    return list(_stream(ch, bm, 16)), list(_stream(ch, bm, 16))


def _rank_main(rank, world, port, seed, bm, out_dir):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tigerbeetle_amd.sharding import ShardedStateMachine, exchange_gloo

    _, second = _dist_plan(seed, bm)
    blob = np.load(os.path.join(out_dir, "forest.npz"))
    sh = ShardedStateMachine(world, rank, exchange_gloo, batch_max=bm, accounts_max=1024, transfers_max=1 << 14,
                             window_events_max=bm)
    sh.open(blob["acc"], blob["xfer"], blob["st"], blob["hist"])
    ts = int(blob["ts"])
    replies, reads = [], []
    for op, batches, tick in second:
        for k, ev in enumerate(batches):
            ts += (tick if k == 0 else 0) + 1 + len(ev)
            d_ev = torch.from_numpy(np.frombuffer(ev.tobytes(), np.uint8).copy()).cuda()
            torch.cuda.synchronize()
            replies.append(sh.commit_general(op, d_ev.data_ptr(), len(ev), ts).hex())
    for q in blob["reads"]:
        op = int(q[0])
        reads.append(sh.read(Operation(op), bytes(q[1:1 + int(q[-1])].astype(np.uint8))).hex())
    with open(os.path.join(out_dir, f"rep{rank}.json"), "w") as f:
        json.dump({"replies": replies, "reads": reads}, f)
    sh.close()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_shard_surface_two_rank_gloo(tmp_path):
    """Two processes (one shard each, sharing cuda:0): open from the restatement's objects, continue
    the stream through the general path, then lookups and queries through gloo all-reduces."""
    import random

    import torch.multiprocessing as mp

    world, seed, bm = 2, 8200, 16
    first, second = _dist_plan(seed, bm)
    ref = OracleStateMachine(batch_max=bm)
    try:
        for op, batches, tick in first:
            for k, ev in enumerate(batches):
                run_protocol(ref, op, ev, tick if k == 0 else 0)
        # the reads after the second part, as (op, request bytes padded to 1024, length) rows
        rng = random.Random(seed)
        expect_rep = []
        for op, batches, tick in second:
            for k, ev in enumerate(batches):
                expect_rep.append(run_protocol(ref, op, ev, tick if k == 0 else 0).hex())
        reads, expect_reads = [], []
        acc_ids = [int(v) for v in ref.dump_accounts()["id_lo"]]
        x_ids = [int(v) for v in ref.dump_transfers()["id_lo"]]
        ts_all = [int(t) for t in ref.dump_transfers()["timestamp"]]
        for _ in range(10):
            for op, data in ((Operation.lookup_accounts, _ids(rng, acc_ids, 6, 500)),
                             (Operation.lookup_transfers, _ids(rng, x_ids, 6, 5000)),
                             (Operation.get_account_transfers, _filter(rng, 30, ts_all, bm)),
                             (Operation.get_account_balances, _filter(rng, 30, ts_all, bm))):
                row = np.zeros(1 + 1024 + 1, np.uint64)
                row[0] = int(op)
                row[1:1 + len(data)] = np.frombuffer(data, np.uint8)
                row[-1] = len(data)
                reads.append(row)
                expect_reads.append(ref.commit(0, 1, ref.prepare_timestamp, op, data).hex())
        # the forest as it was after the first part
        ref2 = OracleStateMachine(batch_max=bm)
        for op, batches, tick in first:
            for k, ev in enumerate(batches):
                run_protocol(ref2, op, ev, tick if k == 0 else 0)
        ts = ref2.prepare_timestamp
        np.savez(tmp_path / "forest.npz", acc=ref2.dump_accounts(), xfer=ref2.dump_transfers(),
                 st=ref2.dump_transfer_status(), hist=np.frombuffer(ref2.dump_account_balances().tobytes(), np.uint8),
                 ts=np.uint64(ts), reads=np.array(reads))
        ref2.close()
        mp.spawn(_rank_main, args=(world, _free_port(), seed, bm, str(tmp_path)), nprocs=world, join=True)
        for r in range(world):
            with open(tmp_path / f"rep{r}.json") as f:
                got = json.load(f)
            assert got["replies"] == expect_rep
            assert got["reads"] == expect_reads
    finally:
        ref.close()
