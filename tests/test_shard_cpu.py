"""CPU tests of the hash-sharded path (no GPU): the ownership hash matches the library's, and the
routed decomposition of csrc/route.h (home route -> all-to-all -> owners' replies -> all-to-all ->
home decide -> all-to-all of commit bytes -> owned effects, tests/shard_model.py) reproduces the CPU
restatement, with real gloo all-to-alls at world size 2 and 3."""
import os
import socket

import numpy as np
import pytest

from tigerbeetle_amd.sharding import shard_of

BM = 64
WINDOW_BATCHES = 3


def test_shard_of_matches_library():
    from tigerbeetle_amd import _lib

    L = _lib.lib()
    rng = np.random.default_rng(0)
    lo = rng.integers(0, 2**63, 2000, dtype=np.uint64) * np.uint64(2) + np.uint64(1)
    hi = np.where(rng.integers(0, 4, 2000) == 0, rng.integers(0, 2**63, 2000, dtype=np.uint64), 0).astype(np.uint64)
    for G in (1, 2, 3, 7, 8):
        got = shard_of(lo, hi, G)
        want = [L.tbg_shard_of(int(a), int(b), G) for a, b in zip(lo, hi)]
        assert got.tolist() == want
        assert set(got.tolist()) == set(range(G))  # every shard owns something


def test_shard_of_balances_sequential_ids():
    ids = np.arange(1, 800_001, dtype=np.uint64)
    counts = np.bincount(shard_of(ids, np.zeros_like(ids), 8), minlength=8)
    assert counts.min() > 0.98 * len(ids) / 8


def _stream(seed, n_acc, n_batches):
    """Mixed create_accounts / create_transfers batches inside the sharded class."""
    from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE

    rng = np.random.default_rng(seed)
    out = []
    a = np.zeros(n_acc, ACCOUNT_DTYPE)
    a["id_lo"] = rng.permutation(np.arange(1, n_acc + 1, dtype=np.uint64))
    a["ledger"] = 1 + a["id_lo"] % 2
    a["code"] = 1
    a["flags"] = np.where(rng.integers(0, 10, n_acc) == 0, 1, 0)
    a["reserved"] = np.where(rng.integers(0, 40, n_acc) == 0, 1, 0)
    out += [("a", a[i:i + BM]) for i in range(0, n_acc, BM)]
    again = a[: BM].copy()
    again["user_data_64"] = rng.integers(0, 2, BM)
    out.append(("a", again))
    next_id = win_start = 1
    used = set()
    for k_batch in range(n_batches):
        if k_batch % WINDOW_BATCHES == 0:
            win_start = next_id  # retries only of ids from earlier windows: no in-window duplicates
            used = set()         # (nor one earlier id retried twice in a window)
        n = int(rng.integers(1, BM + 1))
        t = np.zeros(n, TRANSFER_DTYPE)
        t["id_lo"] = np.arange(next_id, next_id + n, dtype=np.uint64)
        if win_start > 200:
            k = min(n // 6, 10)
            pool = np.array(sorted(set(range(1, win_start - 1)) - used), dtype=np.uint64)
            t["id_lo"][:k] = rng.choice(pool, k, replace=False)
            used.update(int(x) for x in t["id_lo"][:k])
        next_id += n
        dr = rng.integers(1, n_acc + 5, n)
        cr = rng.integers(1, n_acc + 5, n)
        t["debit_account_id_lo"] = dr
        t["credit_account_id_lo"] = cr
        t["amount_lo"] = rng.integers(0, 500, n)
        t["ledger"] = np.where(rng.integers(0, 20, n) == 0, 2 - dr % 2, 1 + dr % 2)
        t["code"] = rng.integers(0, 4, n)
        t["user_data_32"] = rng.integers(0, 2, n)
        t["flags"] = np.where(rng.integers(0, 7, n) == 0, 1, 0)
        t["timestamp"] = np.where(rng.integers(0, 80, n) == 0, 3, 0)
        out.append(("t", t))
    return out


def _alltoall(blocks, world):
    """Uneven all-to-all of byte blocks (blocks[d] goes to rank d): gloo all_to_all_single."""
    import torch
    import torch.distributed as dist

    send_sizes = [len(b) for b in blocks]
    recv_sizes = torch.zeros(world, dtype=torch.int64)
    dist.all_to_all_single(recv_sizes, torch.tensor(send_sizes, dtype=torch.int64))
    recv_sizes = recv_sizes.tolist()
    send = torch.from_numpy(np.frombuffer(b"".join(blocks), np.uint8).copy())
    recv = torch.empty(sum(recv_sizes), dtype=torch.uint8)
    dist.all_to_all_single(recv, send, recv_sizes, send_sizes)
    r = recv.numpy().tobytes()
    out, o = [], 0
    for n in recv_sizes:
        out.append(r[o: o + n])
        o += n
    return out


def _rank(rank, world, port, seed, n_acc, n_batches, out_dir):
    import torch.distributed as dist

    from shard_model import ShardModel
    from tigerbeetle_amd.sharding import route_bounds

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = ShardModel(world, rank)
    T, mine = 0, {}
    for wi, (op, batches) in enumerate(_windows(seed, n_acc, n_batches)):
        ts = []
        for ev in batches:
            T += 1 + len(ev)
            ts.append(T)
        bounds = route_bounds(len(batches), world)
        if wi % 3 == 2:  # uneven homes: one shard home for the whole window
            bounds = [0] * (world - 1 - wi % world) + [len(batches)] * (2 + wi % world)
            bounds = bounds[: world + 1]
            bounds[0] = 0
            bounds[-1] = len(batches)
        recv_a = _alltoall(m.route(op, batches, ts, bounds), world)
        recv_b = _alltoall(m.own(recv_a), world)
        replies, c = m.decide(recv_b)
        recv_c = _alltoall(c, world)
        assert m.apply(recv_c) == 0
        for k, b in enumerate(range(bounds[rank], bounds[rank + 1])):
            mine[(wi, b)] = np.frombuffer(replies[k], np.uint32).reshape(-1, 2)
    np.save(os.path.join(out_dir, f"acc{rank}.npy"), np.array(list(m.accounts.values())))
    np.save(os.path.join(out_dir, f"xfer{rank}.npy"), np.array(list(m.transfers.values())))
    keys = sorted(mine)
    np.save(os.path.join(out_dir, f"keys{rank}.npy"), np.array(keys, np.int64).reshape(-1, 2))
    np.save(os.path.join(out_dir, f"rep{rank}.npy"), np.concatenate(
        [np.concatenate([[[len(mine[k]), 0]], mine[k]]).astype(np.uint32) for k in keys]
        or [np.zeros((0, 2), np.uint32)]))
    dist.destroy_process_group()


def _windows(seed, n_acc, n_batches, per=None):
    """The stream grouped into windows of up to `per` consecutive batches of one operation."""
    per = per or WINDOW_BATCHES
    out = []
    for op, ev in _stream(seed, n_acc, n_batches):
        if out and out[-1][0] == op and len(out[-1][1]) < per:
            out[-1][1].append(ev)
        else:
            out.append((op, [ev]))
    return out


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_protocol_matches_oracle(world, tmp_path):
    import torch.multiprocessing as mp

    from chaos import run_protocol
    from oracle_sm import OracleStateMachine
    from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE, Operation

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    seed, n_acc, n_batches = 11, 150, 40
    mp.spawn(_rank, args=(world, port, seed, n_acc, n_batches, str(tmp_path)), nprocs=world, join=True)
    ref = OracleStateMachine(batch_max=BM)
    try:
        expect = {}
        for wi, (op, batches) in enumerate(_windows(seed, n_acc, n_batches)):
            for b, ev in enumerate(batches):
                r = run_protocol(ref, Operation.create_accounts if op == "a" else Operation.create_transfers, ev)
                expect[(wi, b)] = np.frombuffer(r, np.uint32).reshape(-1, 2)
        assert any(len(v) for v in expect.values())
        got = {}
        for r in range(world):
            keys = [tuple(k) for k in np.load(tmp_path / f"keys{r}.npy").tolist()]
            rep = np.load(tmp_path / f"rep{r}.npy")
            pos = 0
            for k in keys:
                n = int(rep[pos, 0])
                assert k not in got, "two homes for one batch"
                got[k] = rep[pos + 1: pos + 1 + n]
                pos += 1 + n
        assert sorted(got) == sorted(expect)
        for k in expect:
            assert np.array_equal(got[k], expect[k]), k
        acc = np.concatenate([np.load(tmp_path / f"acc{r}.npy").astype(ACCOUNT_DTYPE) for r in range(world)])
        xfer = np.concatenate([np.load(tmp_path / f"xfer{r}.npy").astype(TRANSFER_DTYPE) for r in range(world)])
        acc = acc[np.argsort(acc["timestamp"], kind="stable")]
        xfer = xfer[np.argsort(xfer["timestamp"], kind="stable")]
        assert acc.tobytes() == ref.dump_accounts().tobytes()
        assert xfer.tobytes() == ref.dump_transfers().tobytes()
    finally:
        ref.close()
