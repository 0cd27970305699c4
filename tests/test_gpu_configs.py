"""BASELINE configs at reduced size, GPU (windowed device path) vs CPU restatement (batch by batch,
harness protocol): identical per-batch replies and final stores. Also: the device stream
generators are bit-identical to their numpy twins."""
import numpy as np
import pytest

from oracle_sm import OracleStateMachine
from test_gpu_parity import _compare_final
from test_gpu_window import commit_window, oracle_batches
from tigerbeetle_amd import workload
from tigerbeetle_amd.state_machine import to_host
from tigerbeetle_amd.types import ACCOUNT_DTYPE, NS_PER_S, TRANSFER_DTYPE, Operation

BM = 8190


def _device_gen(fn, count, dtype, *args):
    import torch

    from tigerbeetle_amd import _lib

    d = torch.empty(count * 128, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    _lib.check(fn(d.data_ptr(), *args, None), "gen")
    torch.cuda.synchronize()
    return np.frombuffer(to_host(d).tobytes(), dtype)


@pytest.mark.gpu
def test_device_generators_match_numpy():
    import torch

    from tigerbeetle_amd import _lib

    L = _lib.lib()
    first, count = 123_457, 20_000
    g = _device_gen(L.tbg_gen_accounts, count, ACCOUNT_DTYPE, first, count, 42, 2, 1, 0)
    assert g.tobytes() == workload.accounts(first, count, 42).tobytes()
    g = _device_gen(L.tbg_gen_transfers_uniform, count, TRANSFER_DTYPE, first, count, 42, 10_000, 7)
    assert g.tobytes() == workload.transfers_uniform(first, count, 42, 10_000, 7).tobytes()
    d = torch.empty(count * 128, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    _lib.check(L.tbg_gen_transfers_uniform(d.data_ptr(), first, count, 42, 10_000, 7, None), "gen")
    _lib.check(L.tbg_gen_mark_pending(d.data_ptr(), first, count, 100, 3600, None), "pending")
    torch.cuda.synchronize()
    want = workload.mark_pending(workload.transfers_uniform(first, count, 42, 10_000, 7), first, 100, 3600)
    assert to_host(d).tobytes() == want.tobytes()
    assert (want["flags"] == 2).sum() == count // 100
    g = _device_gen(L.tbg_gen_accounts_cfg3, count, ACCOUNT_DTYPE, first, count, 43, 130_000, 1000)
    assert g.tobytes() == workload.accounts_cfg3(first, count, 43, 130_000, 1000).tobytes()
    g = _device_gen(L.tbg_gen_funding_cfg3, count, TRANSFER_DTYPE, first, count, 43, 200_000, 100, 10**6, 5)
    assert g.tobytes() == workload.funding_cfg3(first, count, 43, 200_000, 100, 10**6, 5).tobytes()
    cdf = workload.zipf_cdf(50_000)
    d_cdf = torch.from_numpy(cdf.view(np.int64).copy()).cuda()
    g = _device_gen(L.tbg_gen_transfers_zipf, count, TRANSFER_DTYPE, first, count, 43, 50_000, d_cdf.data_ptr(), 9)
    assert g.tobytes() == workload.transfers_zipf(first, count, 43, 50_000, cdf, 9).tobytes()
    g = _device_gen(L.tbg_gen_transfers_cfg4, count, TRANSFER_DTYPE, first, count, 44, 30_000, BM, 3)
    assert g.tobytes() == workload.transfers_cfg4(first, count, 44, 30_000, BM, 3).tobytes()


def _batches(arr):
    return [arr[i:i + BM] for i in range(0, len(arr), BM)]


@pytest.mark.gpu
def test_cfg3_zipf_limits_parity():
    """cfg3 shape: Zipf(1.2) accounts, limited ranks incl. the top, pre-funded, windows of 8 batches."""
    from tigerbeetle_amd import StateMachine

    n, treasury, top, n_xfer, win, seed = 20_000, 100, 200, 160_000, 8, 43
    gpu = StateMachine(batch_max=BM, accounts_max=n + treasury, transfers_max=n + n_xfer,
                       window_events_max=win * BM)
    ref = OracleStateMachine(batch_max=BM)
    try:
        acc = _batches(workload.accounts_cfg3(0, n + treasury, seed, n, top))
        assert commit_window(gpu, Operation.create_accounts, acc) == oracle_batches(ref, Operation.create_accounts, acc)
        fund = _batches(workload.funding_cfg3(0, n, seed, n, treasury, 30_000, 10**12))
        assert commit_window(gpu, Operation.create_transfers, fund) == oracle_batches(
            ref, Operation.create_transfers, fund)
        cdf = workload.zipf_cdf(n)
        xf = _batches(workload.transfers_zipf(0, n_xfer, seed, n, cdf))
        fails = 0
        for w0 in range(0, len(xf), win):
            g = commit_window(gpu, Operation.create_transfers, xf[w0:w0 + win])
            r = oracle_batches(ref, Operation.create_transfers, xf[w0:w0 + win])
            assert g == r
            fails += sum(len(x) for x in r) // 8
        assert fails > 0  # the limits bind: exceeds_credits occurs
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_cfg4_two_phase_chains_parity():
    """cfg4 shape: two-phase with timeouts + chains, +1 s per batch (pulse before every batch)."""
    from tigerbeetle_amd import StateMachine

    n, n_xfer, seed = 20_000, 120_000, 44
    gpu = StateMachine(batch_max=BM, accounts_max=n, transfers_max=n_xfer, window_events_max=BM)
    ref = OracleStateMachine(batch_max=BM)
    try:
        for b in _batches(workload.accounts(0, n, seed)):
            assert commit_window(gpu, Operation.create_accounts, [b]) == oracle_batches(
                ref, Operation.create_accounts, [b])
        xf = _batches(workload.transfers_cfg4(0, n_xfer, seed, n, BM))
        codes = set()
        for b in xf:
            g = commit_window(gpu, Operation.create_transfers, [b], NS_PER_S)
            r = oracle_batches(ref, Operation.create_transfers, [b], NS_PER_S)
            assert g == r
            codes |= set(np.frombuffer(r[0], "<u4")[1::2].tolist())
        # rollbacks, expiry and two-phase outcomes all occur
        assert {1, 12, 15, 35}.issubset(codes), codes
        _compare_final(gpu, ref)
        st = gpu.stats()
        assert st["component_events"] > 0 and st["walker_events"] == 0, st
    finally:
        gpu.close()
        ref.close()
