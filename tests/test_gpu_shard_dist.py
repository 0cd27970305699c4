"""Hash-sharded engine across processes: two ranks (one engine each, sharing cuda:0), the exchanges real
torch.distributed collectives (gloo through pinned host memory here; RCCL on a multi-GPU node): the
replicated protocol's all-reduce, or the routed protocol's all-to-alls with each rank holding only its
home batches.
The ranks' replies (each for its home batches) and the union of their stores must equal the CPU
restatement's."""
import os
import socket

import numpy as np
import pytest

BM, WIN = 1024, 4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stream(seed, n_acc, n_windows):
    """Accounts in one window, then transfer windows with invalid fields, chains and cross-window
    retries (no in-window duplicates: the sharded class)."""
    from test_gpu_shard import _mixed_accounts, _mixed_transfers

    rng = np.random.default_rng(seed)
    ids = np.arange(1, n_acc + 1, dtype=np.uint64)
    acc = _mixed_accounts(rng, ids)
    wins = [("a", [acc[i:i + BM] for i in range(0, n_acc, BM)])]
    next_id = 1
    for _ in range(n_windows):
        # retries of ids from earlier windows, each at most once per window
        old = rng.permutation(np.arange(1, next_id, dtype=np.uint64))[: WIN * 40]
        batches = []
        for b in range(WIN):
            n = int(rng.integers(1, BM + 1))
            t = _mixed_transfers(rng, np.arange(next_id, next_id + n, dtype=np.uint64), n_acc)
            mine = old[b * 40: (b + 1) * 40][: n // 8]
            t["id_lo"][: len(mine)] = mine
            next_id += n
            batches.append(t)
        wins.append(("t", batches))
    return wins


def _pack(replies):
    """Per-window replies as one byte string with length prefixes (comparable across processes)."""
    return b"".join(b"".join(len(x).to_bytes(4, "little") + x for x in w) + b"|" for w in replies)


def _rank_main(rank, world, port, seed, n_acc, n_windows, out_dir, protocol="replicated"):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from test_gpu_shard import LocalShards  # noqa: F401  (same harness timestamps)

    from tigerbeetle_amd.sharding import ShardedStateMachine, alltoall_gloo, exchange_gloo, route_bounds
    from tigerbeetle_amd.state_machine import to_host
    from tigerbeetle_amd.types import Operation

    sh = ShardedStateMachine(world, rank, exchange_gloo, batch_max=BM, accounts_max=n_acc,
                             transfers_max=1 << 16, window_events_max=WIN * BM)
    sh.alltoall = alltoall_gloo
    prepare_ts, replies = 0, []
    for kind, batches in _stream(seed, n_acc, n_windows):
        op = Operation.create_accounts if kind == "a" else Operation.create_transfers
        ns, ts = [], []
        for ev in batches:
            prepare_ts += 1 + len(ev)
            ns.append(len(ev))
            ts.append(prepare_ts)
        if protocol == "routed":  # partitioned ingestion: this rank holds only its home batches
            bounds = route_bounds(len(ns), world)
            part = batches[bounds[rank]: bounds[rank + 1]]
        else:
            part = batches
        data = (np.concatenate([np.frombuffer(ev.tobytes(), np.uint8) for ev in part]) if part else
                np.zeros(128, np.uint8))
        d_ev = torch.from_numpy(data.copy()).cuda()
        d_res = torch.zeros(max(sum(ns), 1) * 8, dtype=torch.uint8, device="cuda")
        d_base = torch.zeros(len(ns) + 1, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        if protocol == "routed":
            if sh.pulse(ts[0]):
                sh.commit_pulse(ts[0])
            first, count = sh.commit_window_routed(op, d_ev.data_ptr(), ns, ts, d_res.data_ptr(), d_base.data_ptr(),
                                                   bounds)
        else:
            first, count = sh.commit_window(op, d_ev.data_ptr(), ns, ts, d_res.data_ptr(), d_base.data_ptr())
        sh.sync()
        res, base = to_host(d_res).tobytes(), to_host(d_base)
        replies.append([first] + [res[base[k] * 8: base[k + 1] * 8] for k in range(count)])
    np.save(os.path.join(out_dir, f"acc{rank}.npy"), sh.sm.dump_accounts())
    np.save(os.path.join(out_dir, f"xfer{rank}.npy"), sh.sm.dump_transfers())
    import json

    with open(os.path.join(out_dir, f"rep{rank}.json"), "w") as f:
        json.dump([[w[0]] + [x.hex() for x in w[1:]] for w in replies], f)
    sh.close()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("protocol", ["replicated", "routed"])
def test_two_rank_gloo_matches_oracle(tmp_path, protocol):
    import torch.multiprocessing as mp

    from oracle_sm import OracleStateMachine
    from test_gpu_window import oracle_batches
    from tigerbeetle_amd.types import Operation

    world, seed, n_acc, n_windows = 2, 5, 600, 6
    mp.spawn(_rank_main, args=(world, _free_port(), seed, n_acc, n_windows, str(tmp_path), protocol), nprocs=world,
             join=True)
    ref = OracleStateMachine(batch_max=BM)
    try:
        expect = []
        for kind, batches in _stream(seed, n_acc, n_windows):
            op = Operation.create_accounts if kind == "a" else Operation.create_transfers
            expect.append(oracle_batches(ref, op, batches))
        assert any(len(b) for w in expect[1:] for b in w)  # the stream really fails events
        import json

        got = [[None] * len(w) for w in expect]
        for r in range(world):
            with open(tmp_path / f"rep{r}.json") as f:
                for wi, (first, *reps) in enumerate(json.load(f)):
                    for k, x in enumerate(reps):
                        assert got[wi][first + k] is None, "two homes for one batch"
                        got[wi][first + k] = bytes.fromhex(x)
        assert _pack(got) == _pack(expect)
        acc = np.concatenate([np.load(tmp_path / f"acc{r}.npy") for r in range(world)])
        xfer = np.concatenate([np.load(tmp_path / f"xfer{r}.npy") for r in range(world)])
        acc = acc[np.argsort(acc["timestamp"], kind="stable")]
        xfer = xfer[np.argsort(xfer["timestamp"], kind="stable")]
        assert acc.tobytes() == ref.dump_accounts().tobytes()
        assert xfer.tobytes() == ref.dump_transfers().tobytes()
    finally:
        ref.close()
