"""Super-batched commit windows (tbg_commit_window) must reproduce batch-by-batch results exactly:
per-batch replies and final stores vs the CPU restatement committing the same batches one at a time
under the harness protocol."""
import numpy as np
import pytest

from chaos import Chaos, run_protocol
from oracle_sm import OracleStateMachine
from test_gpu_parity import _compare_final
from tigerbeetle_amd import workload
from tigerbeetle_amd.state_machine import to_host
from tigerbeetle_amd.types import NS_PER_S, RESULT_DTYPE, Operation


def commit_window(sm, op, batches, tick_ns=0):
    """Harness timestamps for each batch of the window; one tbg_commit_window call; per-batch replies."""
    import torch

    sm.prepare_timestamp += tick_ns
    ns, ts = [], []
    for ev in batches:
        sm.prepare_timestamp += 1 + len(ev)
        ns.append(len(ev))
        ts.append(sm.prepare_timestamp)
    data = np.concatenate([np.frombuffer(ev.tobytes(), np.uint8) for ev in batches])
    d_ev = torch.from_numpy(data.copy()).cuda() if len(data) else torch.zeros(128, dtype=torch.uint8).cuda()
    d_res = torch.zeros(max(sum(ns), 1) * 8, dtype=torch.uint8).cuda()
    d_base = torch.zeros(len(ns) + 1, dtype=torch.int32).cuda()
    torch.cuda.synchronize()
    sm.commit_window(op, d_ev.data_ptr(), ns, ts, d_res.data_ptr(), d_base.data_ptr(), True, ts[0])
    sm.sync()
    res = to_host(d_res).tobytes()
    base = to_host(d_base)
    return [res[base[b] * 8: base[b + 1] * 8] for b in range(len(ns))]


def oracle_batches(ref, op, batches, tick_ns=0):
    out = []
    for k, ev in enumerate(batches):
        out.append(run_protocol(ref, op, ev, tick_ns if k == 0 else 0))
    return out


@pytest.mark.gpu
def test_window_uniform_stream():
    from tigerbeetle_amd import StateMachine

    n_acc, n_xfer, bm, win = 10_000, 300_000, 8190, 8
    gpu = StateMachine(batch_max=bm, accounts_max=n_acc, transfers_max=n_xfer, window_events_max=win * bm)
    ref = OracleStateMachine(batch_max=bm)
    try:
        acc = [workload.accounts(f, min(bm, n_acc - f), seed=5) for f in range(0, n_acc, bm)]
        assert commit_window(gpu, Operation.create_accounts, acc) == oracle_batches(ref, Operation.create_accounts, acc)
        xf = [workload.transfers_uniform(f, min(bm, n_xfer - f), seed=5, n_accounts=n_acc) for f in range(0, n_xfer, bm)]
        for w0 in range(0, len(xf), win):
            g = commit_window(gpu, Operation.create_transfers, xf[w0:w0 + win])
            r = oracle_batches(ref, Operation.create_transfers, xf[w0:w0 + win])
            assert g == r
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,win,bm", [(0, 4, 16), (1, 8, 16), (2, 3, 64), (3, 16, 32), (4, 2, 512), (5, 6, 128)])
def test_window_chaos(seed, win, bm):
    """Chaos streams in windows; a 1 s tick before every window keeps pulses at window starts."""
    from tigerbeetle_amd import StateMachine

    gpu = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 17, window_events_max=win * bm)
    ref = OracleStateMachine(batch_max=bm)
    ch = Chaos(1000 + seed, n_accounts=60, id_space=2000)
    try:
        for w in range(12):
            if w < 2:
                op = Operation.create_accounts
                batches = [ch.accounts_batch(ch.rng.randint(1, bm)) for _ in range(win)]
            else:
                op = Operation.create_transfers
                batches = [ch.transfers_batch(ch.rng.choice([1, 3, bm // 2, bm])) for _ in range(win)]
            g = commit_window(gpu, op, batches, NS_PER_S)
            r = oracle_batches(ref, op, batches, NS_PER_S)
            for b in range(win):
                assert g[b] == r[b], (w, b, np.frombuffer(g[b], RESULT_DTYPE), np.frombuffer(r[b], RESULT_DTYPE))
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_window_rejects_due_pulse():
    """A window spanning a due expiry is flagged (tbg_sync -> TBG_E_STATE), never silently wrong."""
    from tigerbeetle_amd import StateMachine
    from tigerbeetle_amd.types import set_u128

    gpu = StateMachine(batch_max=8, accounts_max=64, transfers_max=256, window_events_max=64)
    try:
        acc = [workload.accounts(0, 4, seed=1)]
        commit_window(gpu, Operation.create_accounts, acc)
        t = workload.transfers_uniform(0, 1, seed=1, n_accounts=4)
        t["flags"] = 2
        t["timeout"] = 1
        commit_window(gpu, Operation.create_transfers, [t])
        # next window: T_b1 = expires_at - 1 (no pulse due at its start), T_b2 = expires_at + 2
        b1 = workload.transfers_uniform(10, 2, seed=1, n_accounts=4)
        b2 = workload.transfers_uniform(20, 2, seed=1, n_accounts=4)
        with pytest.raises(RuntimeError):
            commit_window(gpu, Operation.create_transfers, [b1, b2], tick_ns=NS_PER_S - 4)
    finally:
        gpu.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,win,bm", [(11, 1, 64), (12, 4, 128), (13, 2, 1024)])
def test_components_match_sequential_walker(seed, win, bm):
    """Component-parallel walkers (cpw.h) vs the single sequential walker on chaos streams with
    limits stripped from the accounts (so that windows qualify): identical replies and stores."""
    from tigerbeetle_amd import StateMachine

    out = []
    for components in (True, False):
        gpu = StateMachine(batch_max=bm, accounts_max=1 << 12, transfers_max=1 << 17, window_events_max=win * bm,
                           components=components)
        ch = Chaos(2000 + seed, n_accounts=60, id_space=2000)
        replies = []
        try:
            for w in range(14):
                if w < 2:
                    op = Operation.create_accounts
                    batches = [ch.accounts_batch(ch.rng.randint(1, bm)) for _ in range(win)]
                    for b in batches:
                        b["flags"] &= ~np.uint16(6)  # no balance limits
                else:
                    op = Operation.create_transfers
                    batches = [ch.transfers_batch(ch.rng.choice([1, 3, bm // 2, bm])) for _ in range(win)]
                    for b in batches:
                        b["flags"] &= ~np.uint16(0x30)  # no balancing
                replies.append(commit_window(gpu, op, batches, NS_PER_S))
            st = gpu.stats()
            out.append((replies, gpu.dump_accounts().tobytes(), gpu.dump_transfers().tobytes(), st))
        finally:
            gpu.close()
    assert out[0][0] == out[1][0]
    assert out[0][1] == out[1][1] and out[0][2] == out[1][2]
    assert out[0][3]["component_events"] > 0 and out[1][3]["component_events"] == 0
