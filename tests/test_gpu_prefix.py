"""Sorted transfer prefix and claim-free windows (Globals::x_sorted, bmap_direct).

Windows whose transfer ids are strictly increasing and above every stored id append their records
to a prefix found by binary search instead of hashing them, and skip the window key-map claims.
Every later lookup path must still see those records: `exists` on retries, post/void of pending
transfers in the prefix, lookup_transfers, and a non-monotone window (which freezes the prefix and
must fall back to claims even when k_ct_prep speculated claim-free). All vs the CPU restatement."""
import numpy as np
import pytest

from chaos import run_protocol
from oracle_sm import OracleStateMachine
from test_gpu_parity import _compare_final
from test_gpu_window import commit_window, oracle_batches
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import Operation

BM = 512


def _both(gpu, ref, op, batches):
    g = commit_window(gpu, op, batches)
    r = oracle_batches(ref, op, batches)
    assert g == r
    return r


def _lookup(gpu, ref, ids):
    q = np.zeros((len(ids), 2), np.uint64)
    q[:, 0] = ids
    g = run_protocol(gpu, Operation.lookup_transfers, q)
    r = run_protocol(ref, Operation.lookup_transfers, q)
    assert g == r
    return g


@pytest.mark.gpu
def test_prefix_monotone_then_retries_and_two_phase():
    from tigerbeetle_amd import StateMachine

    n_acc = 2048
    gpu = StateMachine(batch_max=BM, accounts_max=n_acc, transfers_max=1 << 16, window_events_max=4 * BM)
    ref = OracleStateMachine(batch_max=BM)
    rng = np.random.default_rng(7)
    try:
        acc = [workload.accounts(f, BM, seed=3) for f in range(0, n_acc, BM)]
        _both(gpu, ref, Operation.create_accounts, acc[:4])
        # three monotone windows: the prefix grows (ids 1..6144), the third one with pending transfers
        nid = 0
        for w in range(3):
            batches = []
            for _ in range(4):
                t = workload.transfers_uniform(nid, BM, seed=3, n_accounts=n_acc)
                if w == 2:
                    t["flags"] = np.where(np.arange(BM) % 3 == 0, 2, 0).astype(np.uint16)  # pending
                batches.append(t)
                nid += BM
            _both(gpu, ref, Operation.create_transfers, batches)
        st = gpu.stats()
        assert st["transfers"] == nid
        # lookups of prefix records (found by binary search), and of absent ids
        _lookup(gpu, ref, np.array([1, 2, 777, 4096, nid, nid + 5, 0], np.uint64))
        # a window of new increasing ids preceded by retries of old ids: not monotone, so claims
        # (k_claim_fix under speculation) and exists / exists_with_different_* via the prefix
        old = ref.dump_transfers()
        retry = old[rng.choice(len(old), 100, replace=False)].copy()
        retry["timestamp"] = 0
        retry["amount_lo"][::2] += 1
        fresh = workload.transfers_uniform(nid, BM - 100, seed=4, n_accounts=n_acc)
        nid += BM - 100
        r = _both(gpu, ref, Operation.create_transfers, [np.concatenate([retry, fresh])])
        codes = set(np.frombuffer(r[0], "<u4")[1::2].tolist())
        assert 46 in codes and len(codes) >= 2, codes  # exists, exists_with_different_amount
        # post / void the prefix's pending transfers (pending_id found by binary search)
        pend = old[(old["flags"] & 2) != 0][:300]
        pv = np.zeros(len(pend), old.dtype)
        pv["id_lo"] = np.arange(nid + 1, nid + 1 + len(pend), dtype=np.uint64)
        nid += len(pend)
        pv["pending_id_lo"] = pend["id_lo"]
        pv["flags"] = np.where(np.arange(len(pend)) % 2 == 0, 4, 8).astype(np.uint16)  # post / void
        _both(gpu, ref, Operation.create_transfers, [pv])
        _lookup(gpu, ref, np.concatenate([pend["id_lo"][:5], pv["id_lo"][:5]]))
        # monotone again: the prefix stays frozen (records hashed), results unchanged
        t = workload.transfers_uniform(nid, BM, seed=5, n_accounts=n_acc)
        t["id_lo"] = np.arange(nid + 1, nid + 1 + BM, dtype=np.uint64)
        _both(gpu, ref, Operation.create_transfers, [t])
        _lookup(gpu, ref, np.array([3, nid + 1, nid + BM], np.uint64))
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_speculation_duplicates_in_window():
    """A claim-free window followed by one with an in-window duplicate id and a post/void of an
    in-window pending transfer: the speculated claim-free prep must be corrected by k_claim_fix."""
    from tigerbeetle_amd import StateMachine

    n_acc = 64
    gpu = StateMachine(batch_max=64, accounts_max=n_acc, transfers_max=1 << 12, window_events_max=128)
    ref = OracleStateMachine(batch_max=64)
    try:
        _both(gpu, ref, Operation.create_accounts, [workload.accounts(0, n_acc, seed=1)])
        t = workload.transfers_uniform(0, 64, seed=1, n_accounts=n_acc)
        _both(gpu, ref, Operation.create_transfers, [t])  # claim-free, extends the prefix
        t = workload.transfers_uniform(64, 64, seed=2, n_accounts=n_acc)
        t["id_lo"][10] = t["id_lo"][3]  # duplicate in the window
        t["flags"][20] = 2  # pending ...
        t["flags"][30] = 4  # ... posted in the same window
        t["pending_id_lo"][30] = t["id_lo"][20]
        t["debit_account_id_lo"][30] = t["credit_account_id_lo"][30] = 0
        t["ledger"][30] = t["code"][30] = t["amount_lo"][30] = 0
        r = _both(gpu, ref, Operation.create_transfers, [t])
        assert r[0], "expected failures (exists*)"
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()
