"""Chunked resolver (csrc/chunks.h) eligibility and its hand-offs, vs the CPU restatement.

A window whose hot accounts (after k_bind_decide) fit the chunked resolver (<= 4094, window amounts
below 2^62) is decided by one workgroup; a window with more hot accounts goes to the grid-wide
relaxation -- or, right after a chunked window (the host then skips the relaxation launches), to the
sequential walker. Windows of each kind are interleaved here, with amounts below and above 2^24 (the
int32 and int64 wave walks) and a window whose amounts sum above 2^62; every reply and the final
stores must equal the restatement's, and the chunked count must be exactly the eligible windows."""
import numpy as np
import pytest

from oracle_sm import OracleStateMachine
from test_gpu_parity import _compare_final
from test_gpu_window import commit_window, oracle_batches
from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE, Operation

N_ACC, TREASURY, BM, WIN = 8000, 4, 1024, 8


def _accounts():
    a = np.zeros(N_ACC + TREASURY, ACCOUNT_DTYPE)
    a["id_lo"] = np.arange(1, N_ACC + TREASURY + 1, dtype=np.uint64)
    a["ledger"], a["code"] = 5, 1
    a["flags"][:N_ACC] = 2  # debits_must_not_exceed_credits; the treasury accounts are unlimited
    return a


def _transfers(first_id, n, rng, kind):
    t = np.zeros(n, TRANSFER_DTYPE)
    t["id_lo"] = np.arange(first_id, first_id + n, dtype=np.uint64)
    if kind == "funding":
        t["debit_account_id_lo"] = N_ACC + 1 + rng.integers(0, TREASURY, n)
        t["credit_account_id_lo"] = rng.integers(1, N_ACC + 1, n)
        t["amount_lo"] = 10
    else:
        hot = kind in ("few", "few_big", "huge_sum")
        span = 40 if hot else N_ACC
        dr = rng.integers(0, span, n)
        cr = rng.integers(0, span, n)
        cr = np.where(cr == dr, (cr + 1) % span, cr)
        t["debit_account_id_lo"] = dr + 1
        t["credit_account_id_lo"] = cr + 1
        lo, hi = {"few": (1, 200), "few_big": (1 << 24, 1 << 26), "many": (50, 200),
                  "huge_sum": (1 << 56, 1 << 57)}[kind]
        t["amount_lo"] = rng.integers(lo, hi, n, dtype=np.uint64)
    t["ledger"], t["code"] = 5, 1
    return t


@pytest.mark.gpu
def test_chunked_resolver_eligibility_and_handoffs():
    from tigerbeetle_amd import StateMachine

    rng = np.random.default_rng(11)
    kinds = ["few", "many", "many", "few", "few_big", "many", "huge_sum", "few", "many", "few_big"]
    n_x = (len(kinds) + 2) * WIN * BM
    gpu = StateMachine(batch_max=BM, accounts_max=N_ACC + TREASURY, transfers_max=n_x, window_events_max=WIN * BM)
    ref = OracleStateMachine(batch_max=BM)
    try:
        acc = _accounts()
        batches = [acc[i:i + BM] for i in range(0, len(acc), BM)]
        assert commit_window(gpu, Operation.create_accounts, batches) == oracle_batches(
            ref, Operation.create_accounts, batches)
        next_id = 1
        # a little funding everywhere: the many-account windows' debits bind nearly everywhere
        f = _transfers(next_id, WIN * BM, rng, "funding")
        next_id += len(f)
        batches = [f[i:i + BM] for i in range(0, len(f), BM)]
        assert commit_window(gpu, Operation.create_transfers, batches) == oracle_batches(
            ref, Operation.create_transfers, batches)
        codes = set()
        for w, kind in enumerate(kinds):
            x = _transfers(next_id, WIN * BM, rng, kind)
            next_id += len(x)
            batches = [x[i:i + BM] for i in range(0, len(x), BM)]
            g = commit_window(gpu, Operation.create_transfers, batches)
            r = oracle_batches(ref, Operation.create_transfers, batches)
            assert g == r, f"window {w} ({kind})"
            for b in r:
                codes.update(np.frombuffer(b, np.uint32)[1::2].tolist())
        _compare_final(gpu, ref)
        st = gpu.stats()
        assert st["chunked_windows"] == sum(k in ("few", "few_big") for k in kinds)
        assert st["walker_events"] > 0  # a many-account window right after a chunked one
        assert st["resolver_events"] > 0
        assert 54 in codes  # exceeds_credits
    finally:
        gpu.close()
        ref.close()
