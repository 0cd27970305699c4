"""Hash-sharded engines (csrc/shard.h) vs the CPU restatement.

G engines share one GPU in one process; the exchange is an in-process element-wise sum of their
exchange words (what the RCCL all-reduce computes across GPUs). Every shard's per-batch replies must
equal the oracle's, and the union of the shards' stores (merged by timestamp) must equal the oracle's
stores byte for byte. Windows outside the sharded class must be rejected whole, on every shard."""
import numpy as np
import pytest

from oracle_sm import OracleStateMachine
from test_gpu_window import oracle_batches
from tigerbeetle_amd import workload
from tigerbeetle_amd.state_machine import to_host
from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE, Operation

BM = 8190


def same_pulse_log(got, want):
    """pulse() logs equal, where the sharded one observed it (None: modelled inside a general window)."""
    return len(got) == len(want) and all(t == u and (p is None or p == q) for (t, p), (u, q) in zip(got, want))


class LocalShards:
    """G shards of one engine on cuda:0, driven like one StateMachine (harness timestamps)."""

    def __init__(self, G, batch_max, accounts_max, transfers_max, window_events_max, change_log=False,
                 general="window"):
        from tigerbeetle_amd.sharding import ShardedStateMachine

        self.shards = [ShardedStateMachine(G, r, None, batch_max=batch_max, accounts_max=accounts_max,
                                           transfers_max=transfers_max, window_events_max=window_events_max,
                                           change_log=change_log)
                       for r in range(G)]
        self.prepare_timestamp = 0
        # (T, pulse()) before every batch, the harness order (:2719-2739); None where a general window
        # models the pulse inside it (not observable from outside)
        self.pulse_log = []
        # windows outside the order-free class: "window" = one read set per window (commit_general_window),
        # "batch" = batch by batch (commit_general_batch, every pulse() observable)
        self.general = general
        # with change_log: every commit call's write-back stream per shard, drained after each call
        # (a replica hands each one to its forest): lists of (shard, accounts, transfers, rows)
        self.logs = [] if change_log else None

    def _drain(self):
        if self.logs is not None:
            for r, s in enumerate(self.shards):
                self.logs.append((r,) + tuple(s.window_changes()))

    def close(self):
        for s in self.shards:
            s.close()

    def summed(self, tensors):
        """The exchange, in-process: every tensor becomes the sum of all of them."""
        import torch

        for s in self.shards:  # engine streams are non-blocking: wait for each explicitly
            s.stream.synchronize()
        total = tensors[0].clone()
        for t in tensors[1:]:
            total += t
        for t in tensors:
            t.copy_(total)
        torch.cuda.synchronize()

    def pulse_before(self, T):
        """The harness pulse before a batch at T (state_machine.zig:2719-2739): pulse() on the
        shards, and when it is true commit(.pulse) at T through the general path."""
        from tigerbeetle_amd.sharding import pulse_general

        due = self.shards[0].pulse(T)
        assert all(s.pulse(T) == due for s in self.shards)
        if due:
            pulse_general(self.shards, self.summed, T)
            self._drain()
        return due

    def commit_any(self, op, batches, tick_ns=0, ticks=None):
        """A window through the order-free path when no pulse can be due in it (after the harness
        pulse before its first batch), else (or when the window is outside the order-free class)
        through the general path (csrc/shard_gx.inc): the whole window at once, or batch by batch.
        `ticks`: a clock tick before each batch (general path only; tick_ns is then ignored).
        Returns (per-batch replies, took the fast path)."""
        import torch

        from tigerbeetle_amd._lib import UnsupportedWindow
        from tigerbeetle_amd.sharding import commit_general_batch

        ts0 = self.prepare_timestamp
        if ticks is None:
            ticks = [tick_ns] + [0] * max(len(batches) - 1, 0)
        tick_ns = ticks[0] if ticks else 0
        t_last = ts0 + sum(ticks) + sum(1 + len(ev) for ev in batches)
        log0 = len(self.pulse_log)
        if batches:
            T0 = ts0 + tick_ns + 1 + len(batches[0])
            self.pulse_log.append((T0, self.pulse_before(T0)))
        if t_last < self.shards[0].pulse_next() and not any(ticks[1:]):
            try:
                return self.commit_window(op, batches, tick_ns, _pulsed=True), True
            except UnsupportedWindow:
                for s in self.shards:  # every shard reports the rejected window once
                    try:
                        s.sync()
                    except UnsupportedWindow:
                        pass
                self.prepare_timestamp = ts0
        del self.pulse_log[log0 + 1:]
        if self.general == "window" and batches:
            from tigerbeetle_amd.sharding import commit_general_window

            ns, ts = [], []
            self.prepare_timestamp = ts0
            for ev, tk in zip(batches, ticks):
                self.prepare_timestamp += tk + 1 + len(ev)
                ns.append(len(ev))
                ts.append(self.prepare_timestamp)
            self.pulse_log.extend((t, None) for t in ts[1:])
            data = np.concatenate([np.frombuffer(ev.tobytes(), np.uint8) for ev in batches])
            d_ev = torch.from_numpy(data.copy()).cuda() if len(data) else torch.zeros(128, dtype=torch.uint8).cuda()
            torch.cuda.synchronize()
            out = commit_general_window(self.shards, self.summed, op, d_ev.data_ptr(), ns, ts, auto_pulse=False)
            self._drain()
            return out, False
        out = []
        self.prepare_timestamp = ts0
        for k, ev in enumerate(batches):
            self.prepare_timestamp += ticks[k] + 1 + len(ev)
            if k > 0:  # batch 0's pulse ran above
                self.pulse_log.append((self.prepare_timestamp, self.pulse_before(self.prepare_timestamp)))
            data = np.frombuffer(ev.tobytes(), np.uint8)
            d_ev = torch.from_numpy(data.copy()).cuda() if len(data) else torch.zeros(128, dtype=torch.uint8).cuda()
            torch.cuda.synchronize()
            out.append(commit_general_batch(self.shards, self.summed, op, d_ev.data_ptr(), len(ev),
                                            self.prepare_timestamp, auto_pulse=False))
            self._drain()
        return out, False

    def commit_window(self, op, batches, tick_ns=0, _pulsed=False):
        """The harness pulse before the first batch when due, then the three steps of csrc/shard.h
        with the exchange summed in-process; returns the per-batch replies assembled from every
        shard's home batches."""
        import torch

        self.prepare_timestamp += tick_ns
        ns, ts = [], []
        for ev in batches:
            self.prepare_timestamp += 1 + len(ev)
            ns.append(len(ev))
            ts.append(self.prepare_timestamp)
        if not _pulsed and ts:
            self.pulse_log.append((ts[0], self.pulse_before(ts[0])))
        # no pulse is due at any later batch of the window (the device checks it too)
        self.pulse_log.extend((t, self.shards[0].pulse(t)) for t in ts[1:])
        data = np.concatenate([np.frombuffer(ev.tobytes(), np.uint8) for ev in batches])
        d_ev = torch.from_numpy(data.copy()).cuda() if len(data) else torch.zeros(128, dtype=torch.uint8).cuda()
        torch.cuda.synchronize()

        summed = self.summed
        summed([s.prepare_window(op, d_ev.data_ptr(), ns, ts) for s in self.shards])
        outs = []
        for s in self.shards:
            first, count = s.home_range(len(ns))
            d_res = torch.zeros(max(sum(ns), 1) * 8, dtype=torch.uint8).cuda()
            d_base = torch.zeros(count + 1, dtype=torch.int32).cuda()
            torch.cuda.synchronize()
            s.commit_prepared(first, count, d_res.data_ptr(), d_base.data_ptr())
            outs.append((first, count, d_res, d_base))
        for s in self.shards:
            s.sync()
        self._drain()
        replies = [None] * len(ns)
        for first, count, d_res, d_base in outs:
            res = to_host(d_res).tobytes()
            base = to_host(d_base)
            for k in range(count):
                replies[first + k] = res[base[k] * 8: base[k + 1] * 8]
        assert all(r is not None for r in replies)
        return replies

    def read(self, op, data):
        """A lookup or query, gathered from the owners (csrc/shard_read.inc)."""
        from tigerbeetle_amd.sharding import read_general

        return read_general(self.shards, self.summed, op, data)

    def dump_accounts(self):
        a = np.concatenate([s.sm.dump_accounts() for s in self.shards])
        return a[np.argsort(a["timestamp"], kind="stable")]

    def dump_transfers(self):
        t = np.concatenate([s.sm.dump_transfers() for s in self.shards])
        return t[np.argsort(t["timestamp"], kind="stable")]


def _diff_rows(g, r):
    """Mismatch report: differing rows and fields (for an assertion message)."""
    if len(g) != len(r):
        return f"lengths {len(g)} vs {len(r)}"
    rows = np.nonzero((g.view(np.uint8).reshape(-1, 128) != r.view(np.uint8).reshape(-1, 128)).any(1))[0]
    out = [f"{len(rows)} rows differ, first {rows[:8].tolist()}"]
    for j in rows[:3]:
        fields = [f for f in g.dtype.names if g[j][f] != r[j][f]]
        out.append(f"row {j}: " + ", ".join(f"{f} {g[j][f]} vs {r[j][f]}" for f in fields))
    return "; ".join(out)


def _compare_sharded(sh, ref):
    ga, ra = sh.dump_accounts(), ref.dump_accounts()
    if ga.tobytes() != ra.tobytes():
        per = [(s.stats()["accounts"], int((s.sm.dump_accounts()["id_lo"] == 0).sum())) for s in sh.shards]
        raise AssertionError(f"accounts: {_diff_rows(ga, ra)}; per shard (count, zero ids) {per}")
    gt, rt = sh.dump_transfers(), ref.dump_transfers()
    assert gt.tobytes() == rt.tobytes(), f"transfers: {_diff_rows(gt, rt)}"
    # every shard owns exactly the records whose id hashes to it
    from tigerbeetle_amd.sharding import shard_of

    G = len(sh.shards)
    for r, s in enumerate(sh.shards):
        a = s.sm.dump_accounts()
        assert (shard_of(a["id_lo"], a["id_hi"], G) == r).all()
        t = s.sm.dump_transfers()
        assert (shard_of(t["id_lo"], t["id_hi"], G) == r).all()


def _batches(arr, bm=BM):
    return [arr[i:i + bm] for i in range(0, len(arr), bm)]


@pytest.mark.gpu
@pytest.mark.parametrize("G", [1, 2, 3, 8])
def test_shard_uniform_stream(G):
    """cfg5 shape at reduced size: uniform transfers, ~(G-1)/G of them cross-shard."""
    n_acc, n_xfer, win = 30_000, 250_000, 8
    sh = LocalShards(G, BM, n_acc // G + 4096, n_xfer // G + 16384, win * BM)
    ref = OracleStateMachine(batch_max=BM)
    try:
        acc = _batches(workload.accounts(0, n_acc, seed=9))
        for w0 in range(0, len(acc), win):
            assert sh.commit_window(Operation.create_accounts, acc[w0:w0 + win]) == oracle_batches(
                ref, Operation.create_accounts, acc[w0:w0 + win])
        xf = _batches(workload.transfers_uniform(0, n_xfer, seed=9, n_accounts=n_acc))
        for w0 in range(0, len(xf), win):
            g = sh.commit_window(Operation.create_transfers, xf[w0:w0 + win])
            assert g == oracle_batches(ref, Operation.create_transfers, xf[w0:w0 + win])
        _compare_sharded(sh, ref)
    finally:
        sh.close()
        ref.close()


def _mixed_accounts(rng, ids, retry=None):
    """Accounts with invalid fields, linked chains (some failing) and, if `retry`, re-creations of
    existing ids with one field changed (exists* codes). No limit flags (a limit is a balance read)."""
    n = len(ids)
    a = np.zeros(n, ACCOUNT_DTYPE)
    a["id_lo"] = ids
    a["ledger"] = 1 + (ids % 2)
    a["code"] = 1 + rng.integers(0, 3, n)
    a["user_data_64"] = rng.integers(0, 3, n)
    k = rng.integers(0, 100, n)
    a["reserved"] = np.where(k == 0, 1, 0)
    a["flags"] = np.where(k == 1, 6, 0)          # flags_are_mutually_exclusive
    a["ledger"] = np.where(k == 2, 0, a["ledger"])
    a["timestamp"] = np.where(k == 3, 5, 0)
    a["flags"] |= np.where(rng.integers(0, 100, n) < 15, 1, 0).astype(np.uint16)  # linked
    if retry is not None:
        a["user_data_64"] = np.where(retry, a["user_data_64"] + (k % 2), a["user_data_64"])
    return a


def _mixed_transfers(rng, ids, n_acc):
    n = len(ids)
    t = np.zeros(n, TRANSFER_DTYPE)
    t["id_lo"] = ids
    dr = rng.integers(1, n_acc + 20, n)
    cr = rng.integers(1, n_acc + 20, n)
    t["debit_account_id_lo"] = dr
    t["credit_account_id_lo"] = cr
    t["amount_lo"] = rng.integers(0, 1000, n)     # some zero: amount_must_not_be_zero
    t["ledger"] = 1 + (dr % 2)
    t["ledger"] = np.where(rng.integers(0, 100, n) < 5, 3 - t["ledger"], t["ledger"])
    t["code"] = rng.integers(0, 4, n)             # some zero
    t["user_data_32"] = rng.integers(0, 3, n)
    k = rng.integers(0, 200, n)
    t["timestamp"] = np.where(k == 0, 9, 0)
    t["flags"] = np.where(k == 1, 1 << 7, 0).astype(np.uint16)  # reserved flag
    t["id_lo"] = np.where(k == 2, 0, t["id_lo"])
    t["flags"] |= np.where(rng.integers(0, 100, n) < 15, 1, 0).astype(np.uint16)  # linked
    return t


@pytest.mark.gpu
@pytest.mark.parametrize("G,seed", [(2, 1), (3, 2), (4, 3)])
def test_shard_mixed_results(G, seed):
    """Every validation code, account-not-found, ledger mismatches, linked chains with rollback and
    chain-open, exists* on cross-window retries, all decided from the exchanged owner facts."""
    rng = np.random.default_rng(seed)
    bm, win, n_acc = 512, 4, 400
    sh = LocalShards(G, bm, 4096, 1 << 16, win * bm)
    ref = OracleStateMachine(batch_max=bm)
    codes = set()
    try:
        ids = np.arange(1, n_acc + 1, dtype=np.uint64)
        rng.shuffle(ids)
        acc = _batches(_mixed_accounts(rng, ids), bm)
        assert sh.commit_window(Operation.create_accounts, acc) == oracle_batches(ref, Operation.create_accounts, acc)
        # re-create some ids (exists, exists_with_different_user_data_64), plus new ones
        again = np.concatenate([ids[:150], np.arange(n_acc + 1, n_acc + 60, dtype=np.uint64)])
        acc = _batches(_mixed_accounts(rng, again, retry=np.arange(len(again)) < 150), bm)
        r = oracle_batches(ref, Operation.create_accounts, acc)
        assert sh.commit_window(Operation.create_accounts, acc) == r
        codes |= {int(x) for b in r for x in np.frombuffer(b, "<u4")[1::2]}
        next_id, committed = 1, []
        for w in range(8):
            batches = []
            used = set()
            for _ in range(win):
                n = int(rng.integers(1, bm + 1))
                new = np.arange(next_id, next_id + n, dtype=np.uint64)
                next_id += n
                t = _mixed_transfers(rng, new, n_acc)
                if committed:
                    # retries of earlier windows' ids, each at most once per window
                    k = min(n // 8, len(committed))
                    pick = rng.choice(len(committed), k, replace=False)
                    for j, p in enumerate(pick):
                        rec = committed[p].copy()
                        if int(rec["id_lo"]) in used:
                            continue
                        used.add(int(rec["id_lo"]))
                        rec["timestamp"] = 0
                        rec["flags"] &= np.uint16(0xFFFE)
                        if j % 3 == 1:
                            rec["user_data_32"] += 1
                        elif j % 3 == 2:
                            rec["amount_lo"] += 1
                        t[j] = rec
                batches.append(t)
            g = sh.commit_window(Operation.create_transfers, batches)
            r = oracle_batches(ref, Operation.create_transfers, batches)
            assert g == r, f"window {w}"
            codes |= {int(x) for b in r for x in np.frombuffer(b, "<u4")[1::2]}
            committed = list(ref.dump_transfers())
        _compare_sharded(sh, ref)
        assert {1, 2, 3, 21, 22, 23, 24, 39, 43, 46}.issubset(codes), sorted(codes)
    finally:
        sh.close()
        ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["pending", "duplicate", "limit", "post", "balancing", "history"])
def test_shard_rejects_windows_outside_class(kind):
    """Windows outside the sharded class fail with TBG_E_UNSUPPORTED and change nothing anywhere."""
    from tigerbeetle_amd._lib import UnsupportedWindow

    G, n_acc = 2, 64
    sh = LocalShards(G, 64, 1024, 4096, 256)
    try:
        a = workload.accounts(0, n_acc + 1, seed=3)
        a["flags"][5] = 2  # account 6: debits_must_not_exceed_credits
        a["flags"][n_acc] = 8  # account 65 (outside the uniform stream): flags.history
        sh.commit_window(Operation.create_accounts, [a[:n_acc], a[n_acc:]])  # batch_max 64
        t = workload.transfers_uniform(0, 40, seed=3, n_accounts=n_acc)
        t["debit_account_id_lo"] = np.where(t["debit_account_id_lo"] == 6, 7, t["debit_account_id_lo"])
        t["credit_account_id_lo"] = np.where(t["credit_account_id_lo"] == 7, 8, t["credit_account_id_lo"])
        t["credit_account_id_lo"] = np.where(t["credit_account_id_lo"] == t["debit_account_id_lo"], 9,
                                             t["credit_account_id_lo"])
        t["debit_account_id_lo"] = np.where(t["credit_account_id_lo"] == t["debit_account_id_lo"], 10,
                                            t["debit_account_id_lo"])
        assert sh.commit_window(Operation.create_transfers, [t[:20]]) == [b""]
        before = (sh.dump_accounts().tobytes(), sh.dump_transfers().tobytes())
        bad = t[20:].copy()
        if kind == "pending":
            bad["flags"][3] = 2
        elif kind == "duplicate":
            bad["id_lo"][7] = bad["id_lo"][2]
        elif kind == "limit":
            bad["debit_account_id_lo"][4] = 6
            bad["credit_account_id_lo"][4] = 12
        elif kind == "history":  # a historical_balance row (state_machine.zig:1806-1841)
            bad["debit_account_id_lo"][4] = n_acc + 1
            bad["credit_account_id_lo"][4] = 12
        elif kind == "post":
            bad["flags"][5] = 4
            bad["pending_id_lo"][5] = 1
            bad["debit_account_id_lo"][5] = bad["credit_account_id_lo"][5] = 0
            bad["ledger"][5] = bad["code"][5] = bad["amount_lo"][5] = 0
        else:
            bad["flags"][6] = 16
        with pytest.raises(UnsupportedWindow):
            sh.commit_window(Operation.create_transfers, [bad])
        assert (sh.dump_accounts().tobytes(), sh.dump_transfers().tobytes()) == before
    finally:
        sh.close()
