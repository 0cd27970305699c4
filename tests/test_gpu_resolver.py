"""Account-parallel resolvers (csrc/relax.h windowed relaxation, the default, and csrc/resolver.h
wait-based walkers) vs the CPU restatement and vs the sequential walker.

Streams of limit-checked transfers that hover at the limit (small funding, hot accounts, both
limit directions, pending and posted) in multi-batch windows: identical per-batch replies and final
stores, and the resolver (not the walker) decided the W events."""
import numpy as np
import pytest

from oracle_sm import OracleStateMachine
from test_gpu_parity import _compare_final
from test_gpu_window import commit_window, oracle_batches
from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE, Operation

DC, CD = 2, 4  # debits_must_not_exceed_credits, credits_must_not_exceed_debits


def _accounts(n, rng):
    a = np.zeros(n, ACCOUNT_DTYPE)
    a["id_lo"] = np.arange(1, n + 1, dtype=np.uint64)
    a["ledger"] = 7
    a["code"] = 3
    kind = rng.integers(0, 10, n)
    a["flags"] = np.where(kind < 5, DC, np.where(kind < 7, CD, 0)).astype(np.uint16)
    a["flags"][:4] = DC  # the hottest ranks are limited
    return a


def _transfers(first_id, count, n, rng, pending_pct, zipf_s, amount_max, funding=False):
    t = np.zeros(count, TRANSFER_DTYPE)
    t["id_lo"] = np.arange(first_id, first_id + count, dtype=np.uint64)
    if funding:
        # from unlimited-by-construction sources: credits to every account, debits from CD accounts
        dr = rng.integers(0, n, count)
        cr = rng.integers(0, n, count)
    else:
        w = 1.0 / np.arange(1, n + 1) ** zipf_s
        p = w / w.sum()
        dr = rng.choice(n, count, p=p)
        cr = rng.choice(n, count, p=p)
    cr = np.where(cr == dr, (cr + 1) % n, cr)
    t["debit_account_id_lo"] = dr + 1
    t["credit_account_id_lo"] = cr + 1
    t["amount_lo"] = rng.integers(1, amount_max, count, dtype=np.uint64)
    t["ledger"] = 7
    t["code"] = 1
    t["flags"] = np.where(rng.integers(0, 100, count) < pending_pct, 2, 0).astype(np.uint16)
    return t


def _run(resolver, seed, n_acc, win, bm, n_windows, pending_pct, zipf_s, amount_max):
    from tigerbeetle_amd import StateMachine

    rng = np.random.default_rng(seed)
    gpu = StateMachine(batch_max=bm, accounts_max=n_acc, transfers_max=(n_windows + 2) * win * bm,
                       window_events_max=win * bm, resolver=resolver)
    ref = OracleStateMachine(batch_max=bm)
    replies = []
    try:
        acc = _accounts(n_acc, rng)
        batches = [acc[i:i + bm] for i in range(0, n_acc, bm)]
        for w0 in range(0, len(batches), win):
            assert commit_window(gpu, Operation.create_accounts, batches[w0:w0 + win]) == oracle_batches(
                ref, Operation.create_accounts, batches[w0:w0 + win])
        next_id = 1
        for w in range(n_windows):
            batches = []
            for _ in range(win):
                n = int(rng.integers(1, bm + 1))
                batches.append(_transfers(next_id, n, n_acc, rng, pending_pct, zipf_s, amount_max))
                next_id += n
            g = commit_window(gpu, Operation.create_transfers, batches)
            r = oracle_batches(ref, Operation.create_transfers, batches)
            assert g == r, f"window {w}"
            replies.append(g)
        _compare_final(gpu, ref)
        return replies, gpu.stats()
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n_acc,win,bm,pending_pct,zipf_s,amount_max", [
    (1, 50, 4, 512, 0, 1.2, 100),       # tiny, very hot: most debits hover at zero
    (2, 200, 8, 1024, 30, 1.2, 1000),   # pending debits/credits mixed in
    (3, 2000, 16, 8190, 10, 1.1, 5000), # many accounts, long hot lists (multi-step walks)
    (4, 20, 2, 8190, 50, 0.5, 50),      # few accounts, everything hot, near-uniform
    (5, 100, 4, 2048, 20, 1.2, 1 << 61), # window amount sums above 2^62: 128-bit walker steps
    (6, 100, 4, 2048, 20, 1.2, 1 << 36), # amounts >= 2^24: chunked resolver's int64 wave walks
])
def test_resolver_matches_oracle_and_walker(seed, n_acc, win, bm, pending_pct, zipf_s, amount_max, monkeypatch):
    rep_r, st_r = _run("relax", seed, n_acc, win, bm, 6, pending_pct, zipf_s, amount_max)
    assert st_r["resolver_events"] > 0 and st_r["chunked_windows"] == 0
    # the chunked single-workgroup resolver (default) where the window fits it (amounts < 2^62)
    rep_k, st_k = _run(True, seed, n_acc, win, bm, 6, pending_pct, zipf_s, amount_max)
    assert st_k["resolver_events"] > 0
    assert (st_k["chunked_windows"] > 0) == (amount_max < 1 << 60)
    assert rep_r == rep_k
    rep_x, st_x = _run("wait", seed, n_acc, win, bm, 6, pending_pct, zipf_s, amount_max)
    assert st_x["resolver_events"] > 0
    assert rep_r == rep_x
    # relaxation windows much smaller than the commit window: many chunk advances
    monkeypatch.setenv("TBG_RELAX_CHUNK", "200")
    rep_c, st_c = _run("relax", seed, n_acc, win, bm, 6, pending_pct, zipf_s, amount_max)
    assert st_c["resolver_events"] > 0
    assert rep_r == rep_c
    rep_w, st_w = _run(False, seed, n_acc, win, bm, 6, pending_pct, zipf_s, amount_max)
    assert st_w["resolver_events"] == 0
    assert rep_r == rep_w
    # the stream really exercises the limit codes
    codes = set()
    for win_rep in rep_r:
        for b in win_rep:
            codes.update(np.frombuffer(b, np.uint32)[1::2].tolist())
    assert codes & {54, 55}, codes
