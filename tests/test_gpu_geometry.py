"""Parity at the bench's own geometry (bench.py): 1M accounts and 128-batch windows of 8190-event
batches (~1M events per window), the windows bench.py commits; the GPU engine vs the CPU
restatement batch by batch under the harness protocol. Replies per batch, then the stores: byte for
byte and through the whole-state digest (tbg_digest vs tigerbeetle_amd.digest over the oracle's
dumps).

- cfg2: uniform transfers, device-generated exactly as bench.py generates them, window by window
  and queued without syncs (fused-only windows, the bench's timed path);
- cfg4 mixed at window scale: two-phase, posts/voids, chains with injected failures in 1M-event
  windows (no tick inside a window: the component walkers and the pulse_next replay at scale);
- cfg4 as bench.py runs it: +1 s per batch, 128-batch windows with ~127 pulses inside each;
- cfg3: Zipf(1.2) with limits, pre-funded, bench.py's 32-batch windows (the account-parallel
  resolver at 262K-event windows);
- cfg5: G = 8 hash shards on one GPU at 128-batch windows, 12.5M accounts' shape scaled to 1M.
"""
import numpy as np
import pytest

from oracle_sm import OracleStateMachine
from test_gpu_parity import _compare_final
from test_gpu_window import commit_window, oracle_batches
from tigerbeetle_amd import workload
from tigerbeetle_amd.digest import digest
from tigerbeetle_amd.state_machine import to_host
from tigerbeetle_amd.types import Operation

BM = 8190
N_ACC = 1_000_000


def _batches(arr, first=0, count=None):
    count = len(arr) if count is None else count
    return [arr[i:i + BM] for i in range(first, first + count, BM)]


def _check_digest(gpu, ref):
    rx = ref.dump_transfers()
    want = digest(ref.dump_accounts(), rx, ref.dump_transfer_status(), ref.pulse_next_timestamp())
    assert gpu.digest() == want


def _accounts(gpu, ref, seed, order=0, perm_seed=0):
    acc = _batches(workload.permute_ids(workload.accounts(0, N_ACC, seed), order, perm_seed))
    for w0 in range(0, len(acc), 128):
        assert commit_window(gpu, Operation.create_accounts, acc[w0:w0 + 128]) == \
            oracle_batches(ref, Operation.create_accounts, acc[w0:w0 + 128])


@pytest.mark.gpu
@pytest.mark.parametrize("id_order", ["sequential", "random", "reversed", "time"])
def test_geometry_cfg2_uniform(id_order):
    """bench.py's cfg2 path: device-generated stream, tbg_commit_window over 128 batches; with
    `bench.py --id-order` random / reversed (the reference benchmark's IdPermutation, cli.zig:263-265)
    every account and transfer id is permuted, so the windows take the hashed id path (no sorted
    prefix, key-map claims); time = the recommended time-based 128-bit ids (strictly increasing, high
    word nonzero): fused pass and sorted prefix in u128 order."""
    import torch

    from tigerbeetle_amd import StateMachine, _lib

    L = _lib.lib()
    n_win, seed = 3, 44
    order = workload.ID_ORDERS[id_order]
    perm_seed = workload.benchmark_permutation_seed(seed)
    n_x = n_win * 128 * BM
    gpu = StateMachine(batch_max=BM, accounts_max=N_ACC, transfers_max=n_x, window_events_max=128 * BM)
    ref = OracleStateMachine(batch_max=BM)
    try:
        _accounts(gpu, ref, seed, order, perm_seed)
        d_x = torch.empty(n_x * 128, dtype=torch.uint8, device="cuda")
        d_res = torch.zeros(128 * BM * 8, dtype=torch.uint8, device="cuda")
        d_base = torch.zeros(129, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        _lib.check(L.tbg_gen_transfers_uniform(d_x.data_ptr(), 0, n_x, seed, N_ACC, 0, gpu.stream), "gen")
        _lib.check(L.tbg_gen_permute_ids(d_x.data_ptr(), n_x, 1, order, perm_seed, gpu.stream), "permute")
        host = workload.permute_ids(workload.transfers_uniform(0, n_x, seed, N_ACC), order, perm_seed)
        for w in range(n_win):
            ns, ts = [], []
            for _ in range(128):
                gpu.prepare_timestamp += 1 + BM
                ns.append(BM)
                ts.append(gpu.prepare_timestamp)
            gpu.commit_window(Operation.create_transfers, d_x.data_ptr() + w * 128 * BM * 128, ns, ts,
                              d_res.data_ptr(), d_base.data_ptr(), True, ts[0])
            gpu.sync()
            base = to_host(d_base)
            res = to_host(d_res).tobytes()
            r = oracle_batches(ref, Operation.create_transfers, _batches(host, w * 128 * BM, 128 * BM))
            assert [res[base[b] * 8: base[b + 1] * 8] for b in range(128)] == r
        st = gpu.stats()
        assert st["transfers"] == n_x
        rising = id_order in ("sequential", "time")
        assert (st["sorted_transfers"] == n_x) == rising
        # every window is order-free and committed by the fused pass (fused.h): rising ids by their
        # order, the others in claim mode (one key-map claim per id: in-window duplicates)
        assert st["fused_windows"] == n_win
        if id_order == "time":  # lookups through the u128 sorted prefix: every id, one absent
            q = np.zeros(BM, [("lo", "<u8"), ("hi", "<u8")])
            pick = np.linspace(0, n_x - 1, BM - 1).astype(np.int64)
            q["lo"][:-1], q["hi"][:-1] = host["id_lo"][pick], host["id_hi"][pick]
            q["lo"][-1], q["hi"][-1] = host["id_lo"][5] + 1, host["id_hi"][5]
            assert gpu.commit(0, 1, 0, Operation.lookup_transfers, q.tobytes()) == \
                ref.commit(0, 1, 0, Operation.lookup_transfers, q.tobytes())
        _check_digest(gpu, ref)
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("id_order", ["sequential", "time"])
def test_geometry_cfg2_change_log(id_order):
    """The drop-in configuration (TBG_FLAG_CHANGE_LOG, write-back to the forest) at the
    bench's geometry: windows committed by the fused pass with the change log on; after each window
    the logged transfers are the window's records and the logged accounts exactly the accounts it
    changed, each equal to the restatement's record."""
    import torch

    from test_gpu_changes import _by_id
    from tigerbeetle_amd import StateMachine, _lib

    L = _lib.lib()
    n_win, seed = 2, 46
    order = workload.ID_ORDERS[id_order]
    perm_seed = workload.benchmark_permutation_seed(seed)
    n_x = n_win * 128 * BM
    gpu = StateMachine(batch_max=BM, accounts_max=N_ACC, transfers_max=n_x, window_events_max=128 * BM,
                       change_log=True)
    ref = OracleStateMachine(batch_max=BM)
    try:
        _accounts(gpu, ref, seed, order, perm_seed)
        d_x = torch.empty(n_x * 128, dtype=torch.uint8, device="cuda")
        d_res = torch.zeros(128 * BM * 8, dtype=torch.uint8, device="cuda")
        d_base = torch.zeros(129, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        _lib.check(L.tbg_gen_transfers_uniform(d_x.data_ptr(), 0, n_x, seed, N_ACC, 0, gpu.stream), "gen")
        _lib.check(L.tbg_gen_permute_ids(d_x.data_ptr(), n_x, 1, order, perm_seed, gpu.stream), "permute")
        host = workload.permute_ids(workload.transfers_uniform(0, n_x, seed, N_ACC), order, perm_seed)
        for w in range(n_win):
            acc0, nx0 = ref.dump_accounts(), len(ref.dump_transfers())
            ns, ts = [], []
            for _ in range(128):
                gpu.prepare_timestamp += 1 + BM
                ns.append(BM)
                ts.append(gpu.prepare_timestamp)
            gpu.commit_window(Operation.create_transfers, d_x.data_ptr() + w * 128 * BM * 128, ns, ts,
                              d_res.data_ptr(), d_base.data_ptr(), True, ts[0])
            gpu.sync()
            base = to_host(d_base)
            res = to_host(d_res).tobytes()
            r = oracle_batches(ref, Operation.create_transfers, _batches(host, w * 128 * BM, 128 * BM))
            assert [res[base[b] * 8: base[b + 1] * 8] for b in range(128)] == r
            acc1, x1 = ref.dump_accounts(), ref.dump_transfers()
            la, lx, rows = gpu.window_changes()
            assert lx.tobytes() == x1[nx0:].tobytes()
            after, before, logged = _by_id(acc1), _by_id(acc0), _by_id(la)
            changed = {k for k, v in after.items() if before.get(k) != v}
            assert set(logged) == changed and len(logged) == len(la)
            assert all(after[k] == v for k, v in logged.items())
            assert len(rows) == 0
        assert gpu.stats()["fused_windows"] == n_win
        _check_digest(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_geometry_cfg2_queued_fused_only_windows():
    """bench.py's timed cfg2 path exactly: 128-batch windows queued back to back with no sync in
    between (each launched fused-only: pulse + k_ct_fused + k_fu_final), each with its own reply
    buffers, then one tbg_sync; every window's replies, the stores and the digest vs the restatement."""
    import torch

    from tigerbeetle_amd import StateMachine, _lib

    L = _lib.lib()
    n_win, seed = 3, 45
    n_x = n_win * 128 * BM
    gpu = StateMachine(batch_max=BM, accounts_max=N_ACC, transfers_max=n_x, window_events_max=128 * BM)
    ref = OracleStateMachine(batch_max=BM)
    try:
        _accounts(gpu, ref, seed)
        d_x = torch.empty(n_x * 128, dtype=torch.uint8, device="cuda")
        outs = [(torch.zeros(128 * BM * 8, dtype=torch.uint8, device="cuda"),
                 torch.zeros(129, dtype=torch.int32, device="cuda")) for _ in range(n_win)]
        torch.cuda.synchronize()
        _lib.check(L.tbg_gen_transfers_uniform(d_x.data_ptr(), 0, n_x, seed, N_ACC, 0, gpu.stream), "gen")
        gpu.sync()
        host = workload.transfers_uniform(0, n_x, seed, N_ACC)
        for w in range(n_win):
            ns, ts = [], []
            for _ in range(128):
                gpu.prepare_timestamp += 1 + BM
                ns.append(BM)
                ts.append(gpu.prepare_timestamp)
            d_res, d_base = outs[w]
            gpu.commit_window(Operation.create_transfers, d_x.data_ptr() + w * 128 * BM * 128, ns, ts,
                              d_res.data_ptr(), d_base.data_ptr(), True, ts[0])
        gpu.sync()
        for w in range(n_win):
            d_res, d_base = outs[w]
            base, res = to_host(d_base), to_host(d_res).tobytes()
            r = oracle_batches(ref, Operation.create_transfers, _batches(host, w * 128 * BM, 128 * BM))
            assert [res[base[b] * 8: base[b + 1] * 8] for b in range(128)] == r
        st = gpu.stats()
        assert st["transfers"] == n_x and st["fused_windows"] == n_win
        _check_digest(gpu, ref)
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_geometry_cfg4_mixed_windows():
    """cfg4's event mix (30 % pending with timeouts, posts/voids of earlier pending transfers, 10 %
    of events in chains with injected failures) in 128-batch windows on 1M accounts."""
    from tigerbeetle_amd import StateMachine

    n_win, seed = 2, 46
    n_x = n_win * 128 * BM
    gpu = StateMachine(batch_max=BM, accounts_max=N_ACC, transfers_max=n_x, window_events_max=128 * BM)
    ref = OracleStateMachine(batch_max=BM)
    try:
        _accounts(gpu, ref, seed)
        host = workload.transfers_cfg4(0, n_x, seed, N_ACC, BM)
        for w in range(n_win):
            xb = _batches(host, w * 128 * BM, 128 * BM)
            g = commit_window(gpu, Operation.create_transfers, xb)
            r = oracle_batches(ref, Operation.create_transfers, xb)
            bad = [b for b in range(128) if g[b] != r[b]]
            assert not bad, f"window {w}: batches {bad[:8]} differ"
            assert gpu.pulse_next_timestamp() == ref.pulse_next_timestamp()
        st = gpu.stats()
        assert st["component_events"] + st["walker_events"] > 0  # the order-dependent part ran
        _check_digest(gpu, ref)
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_geometry_cfg4_bench_windows_with_pulses():
    """bench.py's cfg4 exactly: +1 s per batch in 128-batch windows on 1M accounts, so ~127 pulses
    with expiries fall due inside every window (csrc/xwin.h); replies, pulse_next_timestamp after
    every window, the stores and the digest vs the restatement run batch by batch."""
    from test_gpu_xwin import commit_ticked, oracle_ticked
    from tigerbeetle_amd import StateMachine
    from tigerbeetle_amd.types import NS_PER_S

    n_win, seed = 3, 46
    n_x = n_win * 128 * BM
    gpu = StateMachine(batch_max=BM, accounts_max=N_ACC, transfers_max=n_x, window_events_max=128 * BM)
    ref = OracleStateMachine(batch_max=BM)
    try:
        _accounts(gpu, ref, seed)
        host = workload.transfers_cfg4(0, n_x, seed, N_ACC, BM)
        inner = 0
        for w in range(n_win):
            xb = _batches(host, w * 128 * BM, 128 * BM)
            g, rej = commit_ticked(gpu, Operation.create_transfers, xb, [NS_PER_S] * 128)
            r, n_inner = oracle_ticked(ref, Operation.create_transfers, xb, [NS_PER_S] * 128)
            assert not rej, f"window {w} rejected"
            bad = [b for b in range(128) if g[b] != r[b]]
            assert not bad, f"window {w}: batches {bad[:8]} differ"
            assert gpu.pulse_next_timestamp() == ref.pulse_next_timestamp()
            inner += n_inner
        assert inner > n_win * 100
        _check_digest(gpu, ref)
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_geometry_cfg3_zipf_limits():
    """bench.py's cfg3: Zipf(1.2) with debits_must_not_exceed_credits limits, funded from treasury
    accounts, 32-batch windows."""
    from tigerbeetle_amd import StateMachine

    seed, top, treasury, fund, fund_id = 45, 1000, 1000, 1_000_000, 10**15
    n_win, win = 4, 32
    n_x = n_win * win * BM
    gpu = StateMachine(batch_max=BM, accounts_max=N_ACC + treasury, transfers_max=n_x + N_ACC,
                       window_events_max=128 * BM)
    ref = OracleStateMachine(batch_max=BM)
    try:
        acc = _batches(workload.accounts_cfg3(0, N_ACC + treasury, seed, N_ACC, top))
        for w0 in range(0, len(acc), 128):
            assert commit_window(gpu, Operation.create_accounts, acc[w0:w0 + 128]) == \
                oracle_batches(ref, Operation.create_accounts, acc[w0:w0 + 128])
        fb = _batches(workload.funding_cfg3(0, N_ACC, seed, N_ACC, treasury, fund, fund_id))
        for w0 in range(0, len(fb), 128):
            assert commit_window(gpu, Operation.create_transfers, fb[w0:w0 + 128]) == \
                oracle_batches(ref, Operation.create_transfers, fb[w0:w0 + 128])
        host = workload.transfers_zipf(0, n_x, seed, N_ACC, workload.zipf_cdf(N_ACC))
        fails = 0
        for w in range(n_win):
            xb = _batches(host, w * win * BM, win * BM)
            g = commit_window(gpu, Operation.create_transfers, xb)
            r = oracle_batches(ref, Operation.create_transfers, xb)
            assert g == r, f"window {w}"
            fails += sum(len(x) // 8 for x in r)
        assert fails > 0  # exceeds_credits happens
        assert gpu.stats()["resolver_events"] > 0
        assert gpu.stats()["chunked_windows"] == n_win  # the single-workgroup resolver (chunks.h)
        _check_digest(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_geometry_cfg5_g8_128_batch_windows():
    """cfg5's protocol at G = 8 (hash shards on one GPU, exchanges summed in-process) with
    128-batch windows: ~7/8 of the transfers cross-shard."""
    from test_gpu_shard import LocalShards, _compare_sharded

    G, seed, n_win = 8, 47, 2
    n_x = n_win * 128 * BM
    sh = LocalShards(G, BM, N_ACC // G + 65536, n_x // G + 128 * BM, 128 * BM)
    ref = OracleStateMachine(batch_max=BM)
    try:
        acc = _batches(workload.accounts(0, N_ACC, seed))
        for w0 in range(0, len(acc), 128):
            assert sh.commit_window(Operation.create_accounts, acc[w0:w0 + 128]) == \
                oracle_batches(ref, Operation.create_accounts, acc[w0:w0 + 128])
        host = workload.transfers_uniform(0, n_x, seed, N_ACC)
        for w in range(n_win):
            xb = _batches(host, w * 128 * BM, 128 * BM)
            assert sh.commit_window(Operation.create_transfers, xb) == \
                oracle_batches(ref, Operation.create_transfers, xb)
        _compare_sharded(sh, ref)
    finally:
        sh.close()
        ref.close()
