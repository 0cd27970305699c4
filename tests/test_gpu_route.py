"""Routed sharded windows (csrc/route.h: partitioned ingestion, three all-to-alls) vs the CPU restatement.

G engines share one GPU in one process. Each shard receives only the events of its home batches; the
all-to-alls are in-process block copies (what RCCL's grouped send / receive computes across GPUs).
Every home's per-batch replies must equal the oracle's, and the union of the shards' stores (merged by
timestamp) must equal the oracle's byte for byte. Windows outside the class are rejected on every
shard with nothing applied."""
import numpy as np
import pytest

from oracle_sm import OracleStateMachine
from test_gpu_shard import BM, LocalShards, _batches, _compare_sharded, _mixed_accounts, _mixed_transfers
from test_gpu_window import oracle_batches
from tigerbeetle_amd import workload
from tigerbeetle_amd.state_machine import to_host
from tigerbeetle_amd.types import Operation


class RoutedShards(LocalShards):
    """LocalShards whose order-free windows take the routed path: shard r gets its home batches only."""

    def commit_window(self, op, batches, tick_ns=0, _pulsed=False, bounds=None):
        import torch

        from tigerbeetle_amd.sharding import commit_routed_inprocess, route_bounds

        G = len(self.shards)
        self.prepare_timestamp += tick_ns
        ns, ts = [], []
        for ev in batches:
            self.prepare_timestamp += 1 + len(ev)
            ns.append(len(ev))
            ts.append(self.prepare_timestamp)
        if not _pulsed and ts:
            self.pulse_log.append((ts[0], self.pulse_before(ts[0])))
        self.pulse_log.extend((t, self.shards[0].pulse(t)) for t in ts[1:])
        bounds = bounds or route_bounds(len(ns), G)
        homes, res, bases, keep = [], [], [], []
        for r in range(G):
            part = batches[bounds[r]:bounds[r + 1]]
            data = (np.concatenate([np.frombuffer(ev.tobytes(), np.uint8) for ev in part]) if part else
                    np.zeros(0, np.uint8))
            d_ev = torch.from_numpy(data.copy()).cuda() if len(data) else torch.zeros(128, dtype=torch.uint8).cuda()
            d_res = torch.zeros(max(len(data) // 128, 1) * 8, dtype=torch.uint8).cuda()
            d_base = torch.zeros(bounds[r + 1] - bounds[r] + 1, dtype=torch.int32).cuda()
            keep.append(d_ev)
            homes.append(d_ev.data_ptr())
            res.append(d_res)
            bases.append(d_base)
        torch.cuda.synchronize()
        out = commit_routed_inprocess(self.shards, op, homes, ns, ts, [t.data_ptr() for t in res],
                                      [t.data_ptr() for t in bases], bounds)
        for s in self.shards:
            s.sync()
        self._drain()
        replies = [None] * len(ns)
        for r, (first, count) in enumerate(out):
            rb = to_host(res[r]).tobytes()
            base = to_host(bases[r])
            for k in range(count):
                replies[first + k] = rb[base[k] * 8: base[k + 1] * 8]
        assert all(x is not None for x in replies)
        return replies


@pytest.mark.gpu
@pytest.mark.parametrize("G", [2, 3, 8])
def test_route_uniform_stream(G):
    """cfg5 shape at reduced size: uniform transfers, ~(G-1)/G of each event's owners remote."""
    n_acc, n_xfer, win = 30_000, 250_000, 8
    sh = RoutedShards(G, BM, n_acc // G + 4096, n_xfer // G + 16384, win * BM)
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
        st = [s.stats() for s in sh.shards]
        # rising ids above every stored one: every shard's records extend its sorted prefix
        assert all(x["sorted_transfers"] == x["transfers"] for x in st)
    finally:
        sh.close()
        ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("G,seed", [(2, 1), (3, 2), (4, 3), (8, 4)])
def test_route_mixed_results(G, seed):
    """Validation codes, account-not-found, ledger mismatches, linked chains with rollback and
    chain-open, exists* on cross-window retries (ids that do not rise: the owners claim), uneven and
    empty home ranges, all decided by the homes from the owners' replies."""
    rng = np.random.default_rng(seed)
    bm, win, n_acc = 512, 5, 400
    sh = RoutedShards(G, bm, 4096, 1 << 16, win * bm)
    ref = OracleStateMachine(batch_max=bm)
    codes = set()
    try:
        ids = np.arange(1, n_acc + 1, dtype=np.uint64)
        rng.shuffle(ids)
        acc = _batches(_mixed_accounts(rng, ids), bm)
        assert sh.commit_window(Operation.create_accounts, acc) == oracle_batches(ref, Operation.create_accounts, acc)
        again = np.concatenate([ids[:150], np.arange(n_acc + 1, n_acc + 60, dtype=np.uint64)])
        acc = _batches(_mixed_accounts(rng, again, retry=np.arange(len(again)) < 150), bm)
        r = oracle_batches(ref, Operation.create_accounts, acc)
        assert sh.commit_window(Operation.create_accounts, acc) == r
        codes |= {int(x) for b in r for x in np.frombuffer(b, "<u4")[1::2]}
        next_id, committed = 1, []
        for w in range(8):
            batches, used = [], set()
            for _ in range(win):
                n = int(rng.integers(0 if w == 3 else 1, bm + 1))  # (window 3: empty batches too)
                new = np.arange(next_id, next_id + n, dtype=np.uint64)
                next_id += n
                t = _mixed_transfers(rng, new, n_acc)
                if committed:
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
            # uneven home ranges: some shards home for nothing this window
            bounds = None if w % 2 == 0 else sorted([0, win] + list(rng.integers(0, win + 1, G - 1)))
            g = sh.commit_window(Operation.create_transfers, batches, bounds=bounds)
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
@pytest.mark.parametrize("kind", ["pending", "duplicate", "limit", "post", "balancing", "history", "huge"])
def test_route_rejects_windows_outside_class(kind):
    """Windows outside the class fail with TBG_E_UNSUPPORTED on every shard and change nothing; the
    shards keep committing afterwards."""
    from tigerbeetle_amd._lib import UnsupportedWindow

    G, n_acc = 3, 64
    sh = RoutedShards(G, 64, 1024, 4096, 256)
    try:
        a = workload.accounts(0, n_acc + 1, seed=3)
        a["flags"][5] = 2  # account 6: debits_must_not_exceed_credits
        a["flags"][n_acc] = 8  # account 65 (outside the uniform stream): flags.history
        sh.commit_window(Operation.create_accounts, [a[:n_acc], a[n_acc:]])
        t = workload.transfers_uniform(0, 60, seed=3, n_accounts=n_acc)
        t["debit_account_id_lo"] = np.where(t["debit_account_id_lo"] == 6, 7, t["debit_account_id_lo"])
        t["credit_account_id_lo"] = np.where(t["credit_account_id_lo"] == 7, 8, t["credit_account_id_lo"])
        t["credit_account_id_lo"] = np.where(t["credit_account_id_lo"] == t["debit_account_id_lo"], 9,
                                             t["credit_account_id_lo"])
        t["debit_account_id_lo"] = np.where(t["credit_account_id_lo"] == t["debit_account_id_lo"], 10,
                                            t["debit_account_id_lo"])
        assert sh.commit_window(Operation.create_transfers, [t[:20]]) == [b""]
        before = (sh.dump_accounts().tobytes(), sh.dump_transfers().tobytes())
        bad = t[20:40].copy()
        if kind == "pending":
            bad["flags"][3] = 2
        elif kind == "duplicate":  # the two claimants in different batches (different homes)
            bad["id_lo"][17] = bad["id_lo"][2]
        elif kind == "limit":
            bad["debit_account_id_lo"][4] = 6
            bad["credit_account_id_lo"][4] = 12
        elif kind == "history":
            bad["debit_account_id_lo"][4] = n_acc + 1
            bad["credit_account_id_lo"][4] = 12
        elif kind == "post":
            bad["flags"][5] = 4
            bad["pending_id_lo"][5] = 1
            bad["debit_account_id_lo"][5] = bad["credit_account_id_lo"][5] = 0
            bad["ledger"][5] = bad["code"][5] = bad["amount_lo"][5] = 0
        elif kind == "huge":
            bad["amount_hi"][9] = 1
        else:
            bad["flags"][6] = 16
        with pytest.raises(UnsupportedWindow):
            sh.commit_window(Operation.create_transfers, [bad[:7], bad[7:14], bad[14:]])
            for s in sh.shards:
                s.sync()
        for s in sh.shards:  # every shard reports the rejected window once
            try:
                s.sync()
            except UnsupportedWindow:
                pass
        assert (sh.dump_accounts().tobytes(), sh.dump_transfers().tobytes()) == before
        assert sh.commit_window(Operation.create_transfers, [t[40:50], t[50:]]) == [b"", b""]
    finally:
        sh.close()


def _defined(phase, blk, L, src, dst, n_id, n_side):
    """The bytes of a message block that the protocol defines (padding and unused capacity excluded):
    `src` is the block's HOME shard (its layout), `dst` the owner."""
    if phase == 0:
        s0 = 256 + L.c1[src] * 128
        return blk[:48] + blk[256: 256 + n_id * 128] + blk[s0: s0 + n_side * 32]
    if phase == 1:
        return blk[:4] + blk[64: 64 + n_id] + blk[L.b_side(src): L.b_side(src) + n_side * 8]
    return (blk[:4] + blk[64: 64 + 4 * L.nch(src)] + blk[L.c_hdr(src): L.c_hdr(src) + n_id] +
            blk[L.c_side(src): L.c_side(src) + n_side])


@pytest.mark.gpu
@pytest.mark.parametrize("G", [2, 3])
def test_route_blocks_match_cpu_model(G):
    """The engine's message blocks of every exchange are byte-equal (in every defined byte) to the CPU
    model's (tests/shard_model.py), window after window of a mixed stream; stores equal the oracle's."""
    import struct

    import torch

    from shard_model import ShardModel
    from test_shard_cpu import BM as MBM
    from test_shard_cpu import _windows
    from tigerbeetle_amd.sharding import route_bounds, route_exchange_inprocess

    sh = RoutedShards(G, MBM, 1024, 1 << 14, 3 * MBM)
    models = [ShardModel(G, r) for r in range(G)]
    ref = OracleStateMachine(batch_max=MBM)
    T = 0
    try:
        for wi, (op, batches) in enumerate(_windows(5, 150, 30)):
            ts = []
            for ev in batches:
                T += 1 + len(ev)
                ts.append(T)
            oracle_batches(ref, Operation.create_accounts if op == "a" else Operation.create_transfers, batches)
            bounds = route_bounds(len(batches), G) if wi % 2 else [0] + [len(batches)] * G
            keep, res, bases = [], [], []
            for r, s in enumerate(sh.shards):
                part = batches[bounds[r]:bounds[r + 1]]
                data = np.concatenate([np.frombuffer(e.tobytes(), np.uint8) for e in part]) if part else np.zeros(128, np.uint8)
                d_ev = torch.from_numpy(data.copy()).cuda()
                keep.append(d_ev)
                res.append(torch.zeros(4096, dtype=torch.uint8).cuda())
                bases.append(torch.zeros(8, dtype=torch.int32).cuda())
            torch.cuda.synchronize()
            operation = Operation.create_accounts if op == "a" else Operation.create_transfers
            sh.pulse_before(ts[0])  # (the harness pulse: afterwards none is due inside the window)
            for r, s in enumerate(sh.shards):
                s.route_prepare(operation, keep[r].data_ptr(), [len(b) for b in batches], ts, bounds)
            sent = [m.route(op, batches, ts, bounds) for m in models]
            L = models[0].L
            counts = [[struct.unpack_from("<II", sent[s][d], 0) for d in range(G)] for s in range(G)]
            for phase in range(3):
                for s in sh.shards:
                    s.stream.synchronize()
                for src in range(G):
                    send, ss, _, _ = sh.shards[src].route_views(phase)
                    dev = to_host(send).tobytes()
                    off = 0
                    for dst in range(G):
                        blk = dev[off: off + ss[dst]]
                        off += ss[dst]
                        n_id, n_side = counts[src][dst] if phase != 1 else counts[dst][src]
                        want = _defined(phase, sent[src][dst], L, src if phase != 1 else dst, dst if phase != 1 else src,
                                        n_id, n_side)
                        got = _defined(phase, blk, L, src if phase != 1 else dst, dst if phase != 1 else src,
                                       n_id, n_side)
                        assert got == want, f"window {wi} phase {phase} block {src}->{dst}"
                route_exchange_inprocess(sh.shards, phase)
                recv = [[sent[s][d] for s in range(G)] for d in range(G)]
                if phase == 0:
                    for s in sh.shards:
                        s.route_step("own")
                    sent = [m.own(recv[r]) for r, m in enumerate(models)]
                elif phase == 1:
                    for s in sh.shards:
                        s.route_step("decide")
                    sent = [m.decide(recv[r])[1] for r, m in enumerate(models)]
                else:
                    for r, s in enumerate(sh.shards):
                        s.route_apply(res[r].data_ptr(), bases[r].data_ptr())
                    assert all(m.apply(recv[r]) == 0 for r, m in enumerate(models))
            for s in sh.shards:
                s.sync()
        _compare_sharded(sh, ref)
    finally:
        sh.close()
        ref.close()
