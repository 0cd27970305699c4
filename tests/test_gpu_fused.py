"""The fused pass (tigerbeetle_amd/csrc/fused.h): an order-free create_transfers window committed in
one launch must give exactly what the general path and the CPU restatement give (per-batch replies,
every stored record and status, lookups afterwards). Covered: windows with static failures and
retries of stored ids (exists codes), monotonic windows whose records are hashed instead of
extending the sorted prefix (k_fu_post indexing), and windows that leave the class partway (every
block's speculative balance adds undone, then the general path), each kind followed by more simple
windows so the back-off re-arms the speculation."""
import numpy as np
import pytest

from oracle_sm import OracleStateMachine
from test_gpu_parity import _compare_final
from test_gpu_window import commit_window, oracle_batches
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import Operation

BM = 1024  # events per batch
WIN = 8    # batches per window


def _engines(n_acc, n_xfer, fused=True):
    from tigerbeetle_amd import StateMachine

    gpu = StateMachine(batch_max=BM, accounts_max=n_acc + 8, transfers_max=n_xfer, window_events_max=WIN * BM,
                       fused=fused)
    ref = OracleStateMachine(batch_max=BM)
    return gpu, ref


def _accounts(gpu, ref, n_acc, flags=None):
    acc = workload.accounts(0, n_acc, seed=11)
    if flags:
        for slot, fl in flags.items():
            acc["flags"][slot] = fl
    batches = [acc[f:f + BM] for f in range(0, n_acc, BM)]
    assert commit_window(gpu, Operation.create_accounts, batches) == oracle_batches(ref, Operation.create_accounts,
                                                                                   batches)


def _window(first, n_acc, seed=11, id_offset=0):
    t = workload.transfers_uniform(first, WIN * BM, seed=seed, n_accounts=n_acc, id_offset=id_offset)
    return [t[k * BM:(k + 1) * BM].copy() for k in range(WIN)]


def _check(gpu, ref, batches):
    g = commit_window(gpu, Operation.create_transfers, batches)
    r = oracle_batches(ref, Operation.create_transfers, batches)
    for b, (x, y) in enumerate(zip(g, r)):
        assert x == y, (b, np.frombuffer(x, "<u4")[:16], np.frombuffer(y, "<u4")[:16])


def _inject_static_failures(batches, rng, n_acc):
    """Failures every decision of which is static (validation, lookups, ledgers): the window stays
    in the fused class and its ranks shift."""
    for ev in batches:
        k = rng.choice(BM, size=24, replace=False)
        ev["ledger"][k[0:4]] = 3                     # transfer_must_have_the_same_ledger_as_accounts
        ev["debit_account_id_lo"][k[4:8]] = n_acc + 100   # debit_account_not_found
        ev["credit_account_id_lo"][k[8:10]] = n_acc + 101  # credit_account_not_found
        ev["amount_lo"][k[10:13]] = 0                 # amount_must_not_be_zero
        ev["timestamp"][k[13:15]] = 7                 # timestamp_must_be_zero
        ev["flags"][k[15:17]] = 1 << 9                # reserved_flag (padding bit)
        ev["code"][k[17:19]] = 0                      # code_must_not_be_zero
        ev["credit_account_id_lo"][k[19:21]] = ev["debit_account_id_lo"][k[19:21]]  # accounts_must_be_different
        ev["timeout"][k[21:24]] = 5                   # timeout_reserved_for_pending_transfer


@pytest.mark.gpu
def test_fused_matches_oracle_with_static_failures_and_retries():
    n_acc = 3000
    gpu, ref = _engines(n_acc, 1 << 19)
    rng = np.random.default_rng(5)
    try:
        _accounts(gpu, ref, n_acc)
        first = 0
        for w in range(6):
            batches = _window(first, n_acc)
            first += WIN * BM
            if w % 2 == 1:
                _inject_static_failures(batches, rng, n_acc)
            _check(gpu, ref, batches)
        assert gpu.stats()["fused_windows"] == 6
        assert gpu.stats()["sorted_transfers"] == gpu.stats()["transfers"]
        # retries: the stored ids again (exists / exists_with_different_*), still increasing, then new
        # ids: first id below x_id_max, so the window's records are hashed (not the sorted prefix)
        old = _window(WIN * BM, n_acc)  # window 1's ids (with some fields changed below)
        flat = np.concatenate(old)
        flat["amount_lo"][::7] += 1
        flat["user_data_64"][::11] ^= 1
        retry = np.concatenate([flat[:3 * BM], workload.transfers_uniform(first, 5 * BM, seed=12, n_accounts=n_acc)])
        first += 5 * BM
        batches = [retry[k * BM:(k + 1) * BM].copy() for k in range(WIN)]
        _check(gpu, ref, batches)
        st = gpu.stats()
        assert st["fused_windows"] == 7
        assert st["sorted_transfers"] < st["transfers"]  # the prefix froze: records hashed by k_fu_post
        # later monotonic windows stay fused and hashed; a retry of hashed ids finds them
        for w in range(2):
            batches = _window(first, n_acc, seed=13)
            first += WIN * BM
            _check(gpu, ref, batches)
        hashed = np.concatenate([retry[3 * BM:], np.concatenate(batches)])[:WIN * BM]
        _check(gpu, ref, [hashed[k * BM:(k + 1) * BM].copy() for k in range(WIN)])
        assert gpu.stats()["fused_windows"] == 10
        ids = np.concatenate([retry["id_lo"][:50], hashed["id_lo"][-50:], np.array([first + 10**6], np.uint64)])
        q = np.zeros(len(ids), [("lo", "<u8"), ("hi", "<u8")])
        q["lo"] = ids
        assert gpu.commit(0, 99, 0, Operation.lookup_transfers, q.tobytes()) == \
            ref.commit(0, 99, 0, Operation.lookup_transfers, q.tobytes())
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


OUT_OF_CLASS = ["void", "linked", "limit", "history", "order", "huge", "balancing", "post"]


@pytest.mark.gpu
@pytest.mark.parametrize("kind", OUT_OF_CLASS)
@pytest.mark.parametrize("where", ["first", "last"])
def test_fused_speculation_undone(kind, where):
    """One event outside the class (first or last block of the window): the blocks that applied
    their balance adds are undone, the general path commits the window, replies and stores equal the
    restatement's; simple windows after it go back to the fused pass."""
    n_acc = 2000
    # two accounts the uniform stream never touches: n_acc + 1 debits_must_not_exceed_credits,
    # n_acc + 2 flags.history
    gpu, ref = _engines(n_acc, 1 << 19)
    try:
        _accounts(gpu, ref, n_acc + 2, flags={n_acc: 2, n_acc + 1: 8})
        first = 0
        for w in range(2):
            _check(gpu, ref, _window(first, n_acc))
            first += WIN * BM
        batches = _window(first, n_acc)
        first += WIN * BM
        b, j = (0, 3) if where == "first" else (WIN - 1, BM - 5)
        ev = batches[b]
        if kind == "void":
            ev["flags"][j] = 8
            ev["pending_id_lo"][j] = 17
            ev["amount_lo"][j] = 0
        elif kind == "linked":
            ev["flags"][j] = 1
        elif kind == "limit":
            ev["debit_account_id_lo"][j] = n_acc + 1
            ev["credit_account_id_lo"][j] = 9
        elif kind == "history":
            ev["debit_account_id_lo"][j] = 9
            ev["credit_account_id_lo"][j] = n_acc + 2
        elif kind == "order":  # an id below its predecessor's: not claim-free
            ev["id_lo"][j] = ev["id_lo"][j - 2]
        elif kind == "huge":
            ev["amount_lo"][j] = 1 << 50
        elif kind == "balancing":
            ev["flags"][j] = 16
        elif kind == "post":
            ev["flags"][j] = 4
            ev["pending_id_lo"][j] = 17
            ev["amount_lo"][j] = 0
        _check(gpu, ref, batches)
        assert gpu.stats()["fused_windows"] == 2
        for w in range(6):  # back-off: two general-path windows, then fused again
            _check(gpu, ref, _window(first, n_acc))
            first += WIN * BM
        assert gpu.stats()["fused_windows"] >= 5
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_fused_equals_general_path_digest():
    """The same uniform stream through the fused pass and through the general path (fused off):
    identical digests and dumps."""
    n_acc = 4000
    a, ref = _engines(n_acc, 1 << 19, fused=True)
    b, _ = _engines(n_acc, 1 << 19, fused=False)
    rng = np.random.default_rng(9)
    try:
        _accounts(a, ref, n_acc)
        acc = workload.accounts(0, n_acc, seed=11)
        commit_window(b, Operation.create_accounts, [acc[f:f + BM] for f in range(0, n_acc, BM)])
        first = 0
        for w in range(5):
            batches = _window(first, n_acc, seed=21)
            first += WIN * BM
            if w == 2:
                _inject_static_failures(batches, rng, n_acc)
            ga = commit_window(a, Operation.create_transfers, batches)
            gb = commit_window(b, Operation.create_transfers, batches)
            assert ga == gb
        assert a.stats()["fused_windows"] == 5 and b.stats()["fused_windows"] == 0
        assert a.digest() == b.digest()
        assert a.dump_accounts().tobytes() == b.dump_accounts().tobytes()
        assert a.dump_transfers().tobytes() == b.dump_transfers().tobytes()
    finally:
        a.close()
        b.close()
        ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("bad_windows", [(2,), (0, 3), (5,), ()])
def test_fused_only_windows_replayed_at_sync(bad_windows):
    """Windows queued without a sync in between (the device-resident path, launched fused-only while
    the stream is order-free): a window that leaves the class stops every later one on the device,
    and tbg_sync replays it and all later windows through the general path. An accounts window in
    the middle is replayed too. Every window's replies and the final stores equal the restatement's."""
    import torch

    from tigerbeetle_amd.state_machine import to_host

    n_acc = 2000
    gpu, ref = _engines(n_acc + 64, 1 << 19)
    try:
        _accounts(gpu, ref, n_acc + 2, flags={n_acc: 2, n_acc + 1: 8})
        first, keep, outs, expect = 0, [], [], []
        for wi in range(8):
            if wi == 4:  # create_accounts between transfer windows
                acc = workload.accounts(n_acc + 2, 40, seed=11)
                op, batches = Operation.create_accounts, [acc]
            else:
                op, batches = Operation.create_transfers, _window(first, n_acc)
                first += WIN * BM
                if wi in bad_windows:
                    ev = batches[WIN // 2]
                    ev["flags"][100] = 2  # pending
                    ev["timeout"][100] = 0
                    ev["debit_account_id_lo"][200] = n_acc + 1  # the limited account
            ns, ts = [], []
            for ev in batches:
                gpu.prepare_timestamp += 1 + len(ev)
                ns.append(len(ev))
                ts.append(gpu.prepare_timestamp)
            data = np.concatenate([np.frombuffer(ev.tobytes(), np.uint8) for ev in batches])
            d_ev = torch.from_numpy(data.copy()).cuda()
            d_res = torch.zeros(max(sum(ns), 1) * 8, dtype=torch.uint8).cuda()
            d_base = torch.zeros(len(ns) + 1, dtype=torch.int32).cuda()
            torch.cuda.synchronize()
            gpu.commit_window(op, d_ev.data_ptr(), ns, ts, d_res.data_ptr(), d_base.data_ptr(), True, ts[0])
            keep.append((d_ev, d_res, d_base, len(ns)))
            expect.append(oracle_batches(ref, op, batches))
        gpu.sync()
        for (d_ev, d_res, d_base, nb), r in zip(keep, expect):
            res, base = to_host(d_res).tobytes(), to_host(d_base)
            assert [res[base[b] * 8: base[b + 1] * 8] for b in range(nb)] == r
        st = gpu.stats()
        assert st["fused_windows"] >= (1 if bad_windows else 7)
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_fused_only_pulse_skip_until_pending_timeouts():
    """Fused-only windows skip their pulse launch while pulse_next is "never" (host.inc
    launch_window). Queued without syncs: simple windows, then one that creates pending transfers
    with a 1 s timeout (it leaves the class: replayed at sync), then, 2 s later, windows whose harness
    pulse expires them. Every window's replies, pulse_next and the stores equal the restatement's."""
    import torch

    from tigerbeetle_amd.state_machine import to_host
    from tigerbeetle_amd.types import NS_PER_S
    from test_gpu_window import oracle_batches as ob

    n_acc = 2000
    gpu, ref = _engines(n_acc, 1 << 19)
    try:
        _accounts(gpu, ref, n_acc)
        first = 0

        def submit(batches, tick):
            nonlocal first
            gpu.prepare_timestamp += tick
            ns, ts = [], []
            for ev in batches:
                gpu.prepare_timestamp += 1 + len(ev)
                ns.append(len(ev))
                ts.append(gpu.prepare_timestamp)
            data = np.concatenate([np.frombuffer(ev.tobytes(), np.uint8) for ev in batches])
            d_ev = torch.from_numpy(data.copy()).cuda()
            d_res = torch.zeros(sum(ns) * 8, dtype=torch.uint8).cuda()
            d_base = torch.zeros(len(ns) + 1, dtype=torch.int32).cuda()
            torch.cuda.synchronize()
            gpu.commit_window(Operation.create_transfers, d_ev.data_ptr(), ns, ts, d_res.data_ptr(),
                              d_base.data_ptr(), True, ts[0])
            return (d_ev, d_res, d_base, len(ns)), ob(ref, Operation.create_transfers, batches, tick)

        def check(outs):
            for (d_ev, d_res, d_base, nb), r in outs:
                res, base = to_host(d_res).tobytes(), to_host(d_base)
                assert [res[base[b] * 8: base[b + 1] * 8] for b in range(nb)] == r

        outs = []
        for w in range(2):  # before the first settle: pulses launched
            outs.append(submit(_window(first, n_acc), 0))
            first += WIN * BM
        gpu.sync()  # settle: pulse_next is never from here
        check(outs)
        outs = [submit(_window(first, n_acc), 0)]
        first += WIN * BM
        pend = _window(first, n_acc)
        first += WIN * BM
        for ev in pend[2:5]:
            ev["flags"][::50] = 2   # pending
            ev["timeout"][::50] = 1  # expires 1 s after its timestamp
        outs.append(submit(pend, 0))
        for tick in (2 * NS_PER_S, 0, NS_PER_S):  # pulses due from here
            outs.append(submit(_window(first, n_acc), tick))
            first += WIN * BM
        gpu.sync()
        check(outs)
        assert gpu.pulse_next_timestamp() == ref.pulse_next_timestamp()
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


def _queue(gpu, batches, tick=0, op=Operation.create_transfers):
    """One device-resident window (tbg_commit_window, harness pulse), no sync."""
    import torch

    gpu.prepare_timestamp += tick
    ns, ts = [], []
    for ev in batches:
        gpu.prepare_timestamp += 1 + len(ev)
        ns.append(len(ev))
        ts.append(gpu.prepare_timestamp)
    data = np.concatenate([np.frombuffer(ev.tobytes(), np.uint8) for ev in batches])
    d_ev = torch.from_numpy(data.copy()).cuda()
    d_res = torch.zeros(max(sum(ns), 1) * 8, dtype=torch.uint8).cuda()
    d_base = torch.zeros(len(ns) + 1, dtype=torch.int32).cuda()
    torch.cuda.synchronize()
    gpu.commit_window(op, d_ev.data_ptr(), ns, ts, d_res.data_ptr(), d_base.data_ptr(), True, ts[0])
    return d_ev, d_res, d_base, len(ns)


def _replies(handle):
    from tigerbeetle_amd.state_machine import to_host

    _, d_res, d_base, nb = handle
    res, base = to_host(d_res).tobytes(), to_host(d_base)
    return [res[base[b] * 8: base[b + 1] * 8] for b in range(nb)]


@pytest.mark.gpu
def test_fused_backoff_from_device_commit_then_fused_only_windows():
    """A tbg_commit_device batch outside the class (its fused attempt backs the speculation off, and
    no settle follows) and then device-resident windows queued without syncs: the first of them
    finds the back-off in k_ct_fused and must hand itself to settle()'s replay instead of being
    dropped (the window was silently never committed)."""
    import torch

    from tigerbeetle_amd.state_machine import to_host

    n_acc = 2000
    gpu, ref = _engines(n_acc, 1 << 19)
    try:
        _accounts(gpu, ref, n_acc)
        first = 0
        _check(gpu, ref, _window(first, n_acc))
        first += WIN * BM
        gpu.sync()
        # one batch through tbg_commit_device, outside the class (a pending transfer)
        ev = workload.transfers_uniform(first, BM, seed=17, n_accounts=n_acc)
        first += BM
        ev["flags"][10] = 2
        gpu.prepare_timestamp += 1 + BM
        T = gpu.prepare_timestamp
        d_ev = torch.from_numpy(np.frombuffer(ev.tobytes(), np.uint8).copy()).cuda()
        d_res = torch.zeros(BM * 8, dtype=torch.uint8).cuda()
        d_cnt = torch.zeros(1, dtype=torch.int32).cuda()
        torch.cuda.synchronize()
        gpu.commit_device(Operation.create_transfers, T, d_ev.data_ptr(), BM, d_res.data_ptr(), d_cnt.data_ptr(),
                          True, T)
        want0 = oracle_batches(ref, Operation.create_transfers, [ev])[0]
        outs, expect = [], []
        for w in range(4):
            batches = _window(first, n_acc, seed=18)
            first += WIN * BM
            outs.append(_queue(gpu, batches))
            expect.append(oracle_batches(ref, Operation.create_transfers, batches))
        gpu.sync()
        c = int(to_host(d_cnt)[0])
        assert to_host(d_res).tobytes()[:c * 8] == want0
        for h, r in zip(outs, expect):
            assert _replies(h) == r
        assert gpu.stats()["transfers"] == len(ref.dump_transfers())
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_sync_pending_commit_then_fused_only_windows_pulse():
    """After a settle found pulse_next "never", a synchronous tbg_commit (prefetch + commit) creates
    pending transfers with a 1 s timeout; fused-only windows queued 2 s later must launch their pulse
    and expire them (the general path left pn_never set, so the expiries were skipped)."""
    from chaos import run_protocol

    from tigerbeetle_amd.types import NS_PER_S

    n_acc = 2000
    gpu, ref = _engines(n_acc, 1 << 19)
    try:
        _accounts(gpu, ref, n_acc)
        first = 0
        for w in range(2):
            _check(gpu, ref, _window(first, n_acc))
            first += WIN * BM
        gpu.sync()  # pulse_next is never here
        ev = workload.transfers_uniform(first, 64, seed=19, n_accounts=n_acc)
        first += 64
        ev["flags"][::4] = 2
        ev["timeout"][::4] = 1
        assert run_protocol(gpu, Operation.create_transfers, ev) == run_protocol(ref, Operation.create_transfers, ev)
        outs, expect = [], []
        for w, tick in enumerate((2 * NS_PER_S, 0)):
            batches = _window(first, n_acc, seed=20)
            first += WIN * BM
            outs.append(_queue(gpu, batches, tick))
            expect.append(oracle_batches(ref, Operation.create_transfers, batches, tick))
        gpu.sync()
        for h, r in zip(outs, expect):
            assert _replies(h) == r
        assert gpu.pulse_next_timestamp() == ref.pulse_next_timestamp()
        st = gpu.dump_transfer_status()
        assert (st == 4).sum() == 16  # every pending transfer expired
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_fused_overflow_bound_retightened_at_checkpoints():
    """Globals::ovf_bound sums every committed amount (it must bound every dp+dpo / cp+cpo without
    reading them). Amounts just below the fused class's 2^43 cap add ~2^56 per 8192-event window, so
    without re-tightening the bound would pass 2^63 after ~128 windows and the fused pass would stop.
    The engine re-tightens it at a fixed point of the commit stream (every OVF_RESCAN_EVERY-th window,
    restore.h k_ovf_rescan, gated on the device), never at a state read: 132 queued windows stay on the
    fused pass, state reads run no rescan, and replies and stores match the restatement."""
    n_acc = 2000
    gpu, ref = _engines(n_acc, 1 << 21)
    try:
        _accounts(gpu, ref, n_acc)
        first, outs = 0, []
        big = (1 << 43) - 1

        def win():
            nonlocal first
            b = _window(first, n_acc, seed=23)
            first += WIN * BM
            for ev in b:
                ev["amount_lo"] = big - (ev["amount_lo"] % 4096)
            return b

        st_start = gpu.stats()
        for w in range(132):
            b = win()
            outs.append((_queue(gpu, b), oracle_batches(ref, Operation.create_transfers, b)))
        gpu.sync()
        st0 = gpu.stats()
        assert st0["ovf_rescans"] >= 1  # the checkpoint inside the queue re-tightened the bound
        assert st0["fused_windows"] - st_start["fused_windows"] == 132  # it never reached 2^63
        for h, r in outs:
            assert _replies(h) == r
        for _ in range(4):  # state reads are not checkpoints
            assert gpu.stats()["ovf_rescans"] == st0["ovf_rescans"]
        outs = []
        for w in range(6):
            b = win()
            h = _queue(gpu, b)
            gpu.sync()
            outs.append((h, oracle_batches(ref, Operation.create_transfers, b)))
        for h, r in outs:
            assert _replies(h) == r
        assert gpu.stats()["fused_windows"] == st0["fused_windows"] + 6
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["random", "reversed"])
def test_fused_claim_mode_ids_that_do_not_rise(order):
    """Ids that do not rise (the reference benchmark's random and reversed IdPermutation): the fused
    pass runs in claim mode (each id that reaches the exists check claims its entry in the transfer
    table, pointing at its in-place record), records hashed. A window with an in-window duplicate id
    leaves the class (the second claimant) and goes to the general path (every claim removed first);
    retries of stored ids are exists codes; a rising window after them commits with claims and switches
    back to the rising-id test."""
    n_acc = 2000
    gpu, ref = _engines(n_acc, 1 << 20)
    code = workload.ID_ORDERS[order]
    try:
        _accounts(gpu, ref, n_acc)
        first = 0

        def win(seed=31):
            nonlocal first
            b = _window(first, n_acc, seed=seed)
            first += WIN * BM
            flat = workload.permute_ids(np.concatenate(b), code, 99)
            # (the account ids stay: only the transfer ids are permuted)
            flat["debit_account_id_lo"], flat["debit_account_id_hi"] = np.concatenate(b)["debit_account_id_lo"], 0
            flat["credit_account_id_lo"], flat["credit_account_id_hi"] = np.concatenate(b)["credit_account_id_lo"], 0
            return [flat[k * BM:(k + 1) * BM].copy() for k in range(WIN)]

        for w in range(3):
            _check(gpu, ref, win())
        assert gpu.stats()["fused_windows"] == 3
        dup = win()
        dup[5]["id_lo"][7], dup[5]["id_hi"][7] = dup[1]["id_lo"][3], dup[1]["id_hi"][3]  # in-window duplicate
        _check(gpu, ref, dup)
        assert gpu.stats()["fused_windows"] == 3
        retry = win()
        old = dup[2][:100].copy()
        old["amount_lo"][::3] += 1  # exists_with_different_amount for some
        retry[4][:100] = old
        for w in range(4):  # back-off, then fused again (retries included)
            _check(gpu, ref, retry if w == 0 else win())
        # rising sequential ids (below the stored random ones: hashed, no prefix extension)
        _check(gpu, ref, _window(first + 10**7, n_acc, seed=33))
        _check(gpu, ref, _window(first + 2 * 10**7, n_acc, seed=34))
        st = gpu.stats()
        assert st["fused_windows"] >= 5
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_fused_claim_mode_moves_aborts_and_lookups():
    """Claim mode with records that move (static failures early in each window: the claims of the
    records after them are re-pointed to their ranks), an id whose first event fails before the exists
    check and whose second commits (not a duplicate, as in the reference: the failed event stored
    nothing), a window that leaves the class after its claims were made (every claim removed, the
    general path commits it), retries of moved records (exists codes through the re-pointed claims) and
    a lookup of every id: equal to the restatement throughout."""
    n_acc = 2000
    gpu, ref = _engines(n_acc, 1 << 20)
    rng = np.random.default_rng(17)
    code = workload.ID_ORDERS["random"]
    try:
        _accounts(gpu, ref, n_acc)
        first = 0
        committed = []

        def win(seed=41):
            nonlocal first
            b = _window(first, n_acc, seed=seed)
            first += WIN * BM
            flat = np.concatenate(b)
            ids = workload.permute_ids(flat.copy(), code, 7)
            flat["id_lo"], flat["id_hi"] = ids["id_lo"], ids["id_hi"]
            return [flat[k * BM:(k + 1) * BM].copy() for k in range(WIN)]

        for w in range(4):
            b = win()
            _inject_static_failures(b, rng, n_acc)
            if w == 2:
                # event 5 of batch 3 fails (debit account not found); a later event reuses its id
                b[3]["debit_account_id_lo"][5] = n_acc + 500
                b[6]["id_lo"][9], b[6]["id_hi"][9] = b[3]["id_lo"][5], b[3]["id_hi"][5]
            _check(gpu, ref, b)
            committed.append(np.concatenate(b))
        assert gpu.stats()["fused_windows"] == 4
        # leaves the class in its last batch (a linked event): claims made, then removed
        b = win()
        b[7]["flags"][100] = 1  # linked (a chain of two)
        _check(gpu, ref, b)
        committed.append(np.concatenate(b))
        assert gpu.stats()["fused_windows"] == 4
        for w in range(3):  # back-off, then claim mode again with retries of moved records
            b = win()
            if w == 2:
                old = committed[1][BM:BM + 300].copy()
                old["amount_lo"][::5] += 1
                b[2][:300] = old
            _check(gpu, ref, b)
            committed.append(np.concatenate(b))
        assert gpu.stats()["fused_windows"] >= 5
        allx = np.concatenate(committed)
        for f in range(0, len(allx), BM):  # (a lookup batch holds batch_max ids)
            q = np.zeros(min(BM, len(allx) - f), [("lo", "<u8"), ("hi", "<u8")])
            q["lo"], q["hi"] = allx["id_lo"][f:f + len(q)], allx["id_hi"][f:f + len(q)]
            assert gpu.commit(0, 99, 0, Operation.lookup_transfers, q.tobytes()) == \
                ref.commit(0, 99, 0, Operation.lookup_transfers, q.tobytes()), f
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_sync_prefetch_commit_runs_the_fused_pass():
    """The synchronous StateMachine calls (pulse() check, prefetch, commit per batch: a replica that
    does not pipeline): order-free batches, pending ones with timeouts included, commit through the
    fused pass (the prefetch only stages the request); batches outside the class (a limit account,
    chains, posts/voids of earlier pending transfers) all through the stream are replayed through the
    general path inside the same commit, and the speculation's back-off (capped at 8 batches) leaves
    most clean batches on the fused pass. Replies and stores equal the restatement's."""
    from chaos import run_protocol

    n_acc = 2000
    gpu, ref = _engines(n_acc + 2, 1 << 19)
    try:
        _accounts(gpu, ref, n_acc + 2, flags={n_acc: 2})
        first = 0
        clean = 0
        for b in range(48):
            ev = workload.transfers_uniform(first, BM, seed=41, n_accounts=n_acc)
            first += BM
            if b % 8 == 1:
                ev["flags"][::37] = 2  # pending, in the class
                ev["timeout"][::37] = 1
            elif b % 8 == 4:
                ev["debit_account_id_lo"][5] = n_acc + 1  # the account with a limit flag
            elif b % 8 == 5:
                ev["flags"][10:14] = 1  # a chain
            elif b % 8 == 7:
                ev["flags"][20] = 4  # post of an earlier pending transfer
                ev["pending_id_lo"][20] = ev["id_lo"][0] - 6 * BM
                ev["amount_lo"][20] = 0
            clean += int(b % 8 not in (4, 5, 7))
            tick = 2 * 10**9 if b % 8 == 3 else 0
            assert run_protocol(gpu, Operation.create_transfers, ev, tick) == \
                run_protocol(ref, Operation.create_transfers, ev, tick), b
        assert gpu.stats()["fused_windows"] >= clean // 2, (gpu.stats()["fused_windows"], clean)
        assert gpu.pulse_next_timestamp() == ref.pulse_next_timestamp()
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["sequential", "random"])
def test_fused_pending_creates_in_class(order):
    """About 1 % pending creates (half of them with 1-3 s timeouts) in order-free windows stay on the
    fused pass: debits/credits_pending, the TransferPending rows, pulse_next_timestamp lowered to the
    earliest expiry, live expiry entries. Later windows (a 4 s tick: the harness pulse expires them;
    posts and voids of some on the general path) and the final stores equal the restatement's."""
    n_acc = 2000
    gpu, ref = _engines(n_acc, 1 << 20)
    code = workload.ID_ORDERS[order]
    rng = np.random.default_rng(9)
    try:
        _accounts(gpu, ref, n_acc)
        first, pend_ids = 0, []
        st0 = gpu.stats()
        for w in range(5):
            b = _window(first, n_acc)
            first += WIN * BM
            if code:  # transfer ids that do not rise (claim mode); the accounts stay
                for ev in b:
                    ev["id_lo"], ev["id_hi"] = workload.encode_ids(ev["id_lo"], code, 3)
            for ev in b:
                k = rng.choice(BM, size=10, replace=False)
                ev["flags"][k] = 2
                ev["timeout"][k[:5]] = rng.integers(1, 4, size=5)
                pend_ids += list(zip(ev["id_lo"][k], ev["id_hi"][k]))
            _check(gpu, ref, b)
            assert gpu.pulse_next_timestamp() == ref.pulse_next_timestamp()
        assert gpu.stats()["fused_windows"] - st0["fused_windows"] == 5
        # posts / voids of some of them (general path), then a tick: the harness pulse expires the rest
        pv = _window(first, n_acc)
        first += WIN * BM
        for j, ev in enumerate(pv[:2]):
            for q in range(8):
                lo, hi = pend_ids[j * 8 + q]
                ev["flags"][q] = 4 if q % 2 == 0 else 8
                ev["pending_id_lo"][q], ev["pending_id_hi"][q] = lo, hi
                ev["amount_lo"][q] = 0
        _check(gpu, ref, pv)
        gpu.prepare_timestamp += 4 * 10**9
        ref.prepare_timestamp += 4 * 10**9
        for w in range(2):
            b = _window(first, n_acc)
            first += WIN * BM
            _check(gpu, ref, b)
        assert gpu.pulse_next_timestamp() == ref.pulse_next_timestamp()
        assert (ref.dump_transfer_status() == 4).sum() > 0
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()


@pytest.mark.gpu
def test_fused_claim_mode_aborts_leave_the_table_bounded():
    """Claim mode (random ids) with every window leaving the class after its claims were made (a chain
    in its last batch, a post of a stored pending transfer in another): the claims are reverted to the
    empty entries they took, so after every window the transfer table holds exactly one entry per
    hashed record (no removed entries accumulate: ADVICE r5, a table with no empty entry left would
    make every probe loop), and replies and stores equal the restatement's."""
    from tigerbeetle_amd import _lib
    import ctypes

    n_acc = 2000
    gpu, ref = _engines(n_acc, 1 << 17)
    code = workload.ID_ORDERS["random"]
    L = _lib.lib()

    def used():
        a, x = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.check(L.tbg_debug_table_used(gpu.h, ctypes.byref(a), ctypes.byref(x)), "table_used")
        return a.value, x.value

    try:
        _accounts(gpu, ref, n_acc)
        first = 0
        for w in range(10):
            b = _window(first, n_acc, seed=61 + w)
            first += WIN * BM
            flat = np.concatenate(b)
            ids = workload.permute_ids(flat.copy(), code, 5)
            flat["id_lo"], flat["id_hi"] = ids["id_lo"], ids["id_hi"]
            b = [flat[k * BM:(k + 1) * BM].copy() for k in range(WIN)]
            if w % 3 != 2:  # (every third window stays in the class: the speculation re-arms)
                b[WIN - 1]["flags"][BM - 10] = 1  # linked: a chain of two, in the last block
            _check(gpu, ref, b)
            st = gpu.stats()
            acc_used, x_used = used()
            assert acc_used == st["accounts"], (w, acc_used, st)
            assert x_used == st["transfers"] - st["sorted_transfers"], (w, x_used, st)
        assert gpu.stats()["fused_windows"] >= 2
        _compare_final(gpu, ref)
    finally:
        gpu.close()
        ref.close()
