"""Host-fed windows (tbg_commit_window_host): prepare bodies in pinned host memory, staged through
two device slots on a copy stream while the previous window computes, replies copied back; several
windows in flight at once. Same replies and stores as the CPU restatement committing the batches
one by one (harness protocol)."""
import numpy as np
import pytest

from chaos import Chaos
from oracle_sm import OracleStateMachine
from test_gpu_parity import _compare_final
from test_gpu_window import oracle_batches
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import NS_PER_S, Operation


def _submit(gpu, op, batches, tick_ns):
    """Pinned host buffers for one window; returns (ticket, buffers, batch count)."""
    import torch

    gpu.prepare_timestamp += tick_ns
    ns, ts = [], []
    for ev in batches:
        gpu.prepare_timestamp += 1 + len(ev)
        ns.append(len(ev))
        ts.append(gpu.prepare_timestamp)
    data = np.concatenate([np.frombuffer(ev.tobytes(), np.uint8) for ev in batches])
    h_ev = torch.empty(max(len(data), 128), dtype=torch.uint8, pin_memory=True)
    h_ev[: len(data)] = torch.from_numpy(data.copy())
    # 0xFF until the window's D2H lands (a reply read too early cannot look right)
    h_res = torch.full((max(sum(ns), 1) * 8,), 0xFF, dtype=torch.uint8, pin_memory=True)
    h_base = torch.full((len(ns) + 1,), -1, dtype=torch.int32, pin_memory=True)
    t = gpu.commit_window_host(op, h_ev.data_ptr(), ns, ts, h_res.data_ptr(), h_base.data_ptr(), True, ts[0])
    return t, (h_ev, h_res, h_base), len(ns)


def _replies(bufs, nb):
    _, h_res, h_base = bufs
    res = h_res.numpy().tobytes()
    base = h_base.numpy()
    return [res[base[b] * 8: base[b + 1] * 8] for b in range(nb)]


@pytest.mark.gpu
@pytest.mark.parametrize("seed,win,bm,depth", [(0, 4, 32, 3), (1, 8, 16, 4), (2, 2, 128, 2)])
def test_host_fed_chaos_pipelined(seed, win, bm, depth):
    from tigerbeetle_amd import StateMachine

    gpu = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 16, window_events_max=win * bm)
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(6100 + seed, n_accounts=50, id_space=1500)
    try:
        pending = []
        for w in range(16):
            if w < 2:
                op = Operation.create_accounts
                batches = [ch.accounts_batch(ch.rng.randint(1, bm)) for _ in range(win)]
            else:
                op = Operation.create_transfers
                batches = [ch.transfers_batch(ch.rng.choice([1, 3, bm // 2, bm])) for _ in range(win)]
            t, bufs, nb = _submit(gpu, op, batches, NS_PER_S)
            pending.append((t, bufs, nb, oracle_batches(ref, op, batches, NS_PER_S)))
            if len(pending) >= depth:  # keep `depth` windows in flight
                t0, b0, n0, r0 = pending.pop(0)
                while not gpu.window_done(t0):
                    pass
                assert _replies(b0, n0) == r0
        gpu.sync()
        for t0, b0, n0, r0 in pending:
            assert gpu.window_done(t0)
            assert _replies(b0, n0) == r0
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_host_fed_uniform_128_batch_windows():
    from tigerbeetle_amd import StateMachine

    bm, n_acc, win, n_win = 8190, 100_000, 32, 4
    gpu = StateMachine(batch_max=bm, accounts_max=n_acc, transfers_max=n_win * win * bm, window_events_max=win * bm)
    ref = OracleStateMachine(batch_max=bm)
    try:
        acc = workload.accounts(0, n_acc, seed=61)
        ab = [acc[i:i + bm] for i in range(0, n_acc, bm)]
        t, bufs, nb = _submit(gpu, Operation.create_accounts, ab, 0)
        gpu.sync()
        assert _replies(bufs, nb) == oracle_batches(ref, Operation.create_accounts, ab)
        xf = workload.transfers_uniform(0, n_win * win * bm, 61, n_acc)
        subs = []
        for w in range(n_win):
            batches = [xf[(w * win + b) * bm:(w * win + b + 1) * bm] for b in range(win)]
            subs.append((_submit(gpu, Operation.create_transfers, batches, 0), batches))
        gpu.sync()
        for (t, bufs, nb), batches in subs:
            assert _replies(bufs, nb) == oracle_batches(ref, Operation.create_transfers, batches)
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_host_fed_done_is_per_ticket():
    """tbg_host_window_done(t) may report 1 only once window t's replies have landed, also after two
    later windows were submitted on its slot: a large window (a ~128 MB H2D) followed at
    once by two tiny ones; whenever done(t) says 1, the reply buffers (pre-filled with 0xFF) must hold
    the final bytes, and done is monotone in the ticket order."""
    from tigerbeetle_amd import StateMachine

    bm, n_acc, win = 8190, 100_000, 128
    gpu = StateMachine(batch_max=bm, accounts_max=n_acc, transfers_max=2 * win * bm, window_events_max=win * bm)
    ref = OracleStateMachine(batch_max=bm)
    try:
        acc = workload.accounts(0, n_acc, seed=62)
        ab = [acc[i:i + bm] for i in range(0, n_acc, bm)]
        t, bufs, nb = _submit(gpu, Operation.create_accounts, ab, 0)
        gpu.sync()
        assert _replies(bufs, nb) == oracle_batches(ref, Operation.create_accounts, ab)
        xf = workload.transfers_uniform(0, win * bm + 2, 62, n_acc)
        big = [xf[b * bm:(b + 1) * bm] for b in range(win)]
        small = [[xf[win * bm:win * bm + 1]], [xf[win * bm + 1:win * bm + 2]]]
        subs = [_submit(gpu, Operation.create_transfers, big, 0)]
        for s in small:
            subs.append(_submit(gpu, Operation.create_transfers, s, 0))
        expect = [oracle_batches(ref, Operation.create_transfers, w) for w in [big] + small]
        for _ in range(200000):
            done = [gpu.window_done(s[0]) for s in subs]
            for k in range(3):
                if done[k]:
                    assert _replies(subs[k][1], subs[k][2]) == expect[k], f"ticket {k}: done before its replies"
            assert all(done[k] or not done[k + 1] for k in range(2)), done
            if all(done):
                break
        gpu.sync()
        assert all(gpu.window_done(s[0]) for s in subs)
        for k in range(3):
            assert _replies(subs[k][1], subs[k][2]) == expect[k]
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_read_device_any_size_and_alignment():
    """tbg_read_device: a kernel copy through the engine's pinned block, after the stream's work; any
    byte count (beyond one pinned block too) and any alignment of the device source."""
    import torch

    from tigerbeetle_amd import StateMachine

    sm = StateMachine(batch_max=64, accounts_max=1024, transfers_max=1024)
    try:
        g = torch.Generator().manual_seed(5)
        src = torch.randint(0, 256, (3 * 64 * 128 + 77,), dtype=torch.uint8, generator=g)
        d = src.cuda()
        torch.cuda.synchronize()
        for off, n in [(0, 0), (0, 1), (3, 17), (16, 4096), (5, 64 * 128 + 3), (1, 3 * 64 * 128 + 70)]:
            got = sm.read_device(d[off: off + n])
            assert np.array_equal(got, src[off: off + n].numpy()), (off, n)
        w = torch.arange(1000, dtype=torch.int32).cuda()
        torch.cuda.synchronize()
        assert np.array_equal(sm.read_device(w), np.arange(1000, dtype=np.int32))
    finally:
        sm.close()
