"""Non-binding limits (k_bind_*, engine.hip): an account with debits_must_not_exceed_credits whose
balances at the window start plus every debit of the window still pass cannot fail a check in that
window, whatever the order: it needs no ordering, so events on it are decided in parallel. Windows
where no limited account can bind run without the walkers and the resolver; windows where a few
bind keep exactly those accounts hot. Replies and stores vs the CPU restatement."""
import numpy as np
import pytest

from oracle_sm import OracleStateMachine
from test_gpu_parity import _compare_final
from test_gpu_window import commit_window, oracle_batches
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE, Operation

N_ACC, TREASURY = 2000, 10


def _accounts(limited_credit_cap):
    a = workload.accounts(0, N_ACC + TREASURY, seed=3)
    a["flags"] = np.where(np.arange(N_ACC + TREASURY) < N_ACC, 2, 0).astype(np.uint16)  # debits<=credits
    return a


def _funding(amounts):
    t = np.zeros(N_ACC, TRANSFER_DTYPE)
    t["id_lo"] = np.arange(1, N_ACC + 1, dtype=np.uint64) + np.uint64(10**12)
    t["debit_account_id_lo"] = np.uint64(N_ACC + 1) + np.arange(N_ACC, dtype=np.uint64) % np.uint64(TREASURY)
    t["credit_account_id_lo"] = np.arange(1, N_ACC + 1, dtype=np.uint64)
    t["amount_lo"] = amounts
    t["ledger"], t["code"] = 2, 1
    return t


def _run(fund, bm=512, win=8, n_x=40 * 512):
    from tigerbeetle_amd import StateMachine

    gpu = StateMachine(batch_max=bm, accounts_max=N_ACC + TREASURY, transfers_max=n_x + N_ACC,
                       window_events_max=win * bm)
    ref = OracleStateMachine(batch_max=bm)
    try:
        acc = _accounts(None)
        batches = [acc[i:i + bm] for i in range(0, len(acc), bm)]
        assert commit_window(gpu, Operation.create_accounts, batches) == oracle_batches(ref, Operation.create_accounts,
                                                                                        batches)
        f = _funding(fund)
        batches = [f[i:i + bm] for i in range(0, len(f), bm)]
        assert commit_window(gpu, Operation.create_transfers, batches) == oracle_batches(ref, Operation.create_transfers,
                                                                                         batches)
        before = gpu.stats()
        xf = workload.transfers_uniform(0, n_x, seed=4, n_accounts=N_ACC)
        fails = 0
        for w0 in range(0, n_x, win * bm):
            batches = [xf[i:i + bm] for i in range(w0, min(w0 + win * bm, n_x), bm)]
            g = commit_window(gpu, Operation.create_transfers, batches)
            r = oracle_batches(ref, Operation.create_transfers, batches)
            assert g == r
            fails += sum(len(x) // 8 for x in r)
        _compare_final(gpu, ref)
        after = gpu.stats()
        ordered = sum(after[k] - before[k] for k in ("walker_events", "resolver_events", "component_events"))
        return fails, ordered
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_limits_that_cannot_bind_need_no_ordering():
    """Every limited account funded far above what the stream can debit: no event is ordered."""
    fails, ordered = _run(np.full(N_ACC, 10**12, np.uint64))
    assert fails == 0 and ordered == 0


@pytest.mark.gpu
def test_a_few_binding_accounts_stay_ordered():
    """Most accounts well funded, one in fifty nearly empty: those bind (exceeds_credits happens)
    and only the events around them are ordered."""
    fund = np.full(N_ACC, 10**12, np.uint64)
    fund[::50] = 5
    fails, ordered = _run(fund)
    assert fails > 0 and 0 < ordered < 40 * 512
