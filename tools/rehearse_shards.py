"""Per-shard GPU time of the hash-sharded commit at G shards, rehearsed on ONE GPU.

G ShardedStateMachine engines live on cuda:0 in this process. Each window runs shard by shard, with
HIP events on each engine's stream around each step: --protocol routed (default; csrc/route.h) routes
each shard's home slice, then own / decide / apply between in-process all-to-alls; --protocol
replicated (csrc/shard.h) prepares the whole window on every shard, sums the facts in-process (what the
RCCL all-reduce computes) and commits. A shard's GPU time per window is what one GPU of a G-GPU node
spends on the window apart from the collective, so

    estimated G-GPU rate = global events / sum over windows of max over shards (prepare + commit)

is an upper bound for the real node (the all-reduce of 2 B per event is added on top).
Not a bench line: evidence for DESIGN.md §7. Usage (on the GPU box):

    python tools/rehearse_shards.py --shards 8 --accounts 2000000 --transfers 40000000 --window 64
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

BATCH = 8190


def general(a):
    """--stream cfg3|cfg4: the general class (csrc/shard_gw.inc, a whole window per read set) at G
    shards on this GPU against ONE unsharded engine on the same stream. Per window and shard, wall
    time of its steps (gather 1: collect + write, gather 2: collect + write, commit: the scratch
    engine's window + this shard's apply), each synchronized on its own (the in-process sums of the
    exchanges between them are not counted); the unsharded engine's wall time per window
    (commit_window + sync) beside it."""
    import time

    import torch

    from tigerbeetle_amd import StateMachine, _lib, workload
    from tigerbeetle_amd.sharding import ShardedStateMachine, commit_general_window, pulse_general
    from tigerbeetle_amd.state_machine import to_host
    from tigerbeetle_amd.types import NS_PER_S, Operation

    L = _lib.lib()
    G, win, n_acc, n_x = a.shards, a.window, a.accounts, a.transfers
    tick = NS_PER_S if a.stream == "cfg4" else 0
    treasury = 1000 if a.stream == "cfg3" else 0
    shards = [ShardedStateMachine(G, r, None, batch_max=BATCH, accounts_max=int((n_acc + treasury) / G * 1.2) + 65536,
                                  transfers_max=int((n_x + n_acc) / G * 1.2) + win * BATCH, window_events_max=win * BATCH)
              for r in range(G)]
    one = StateMachine(batch_max=BATCH, accounts_max=n_acc + treasury, transfers_max=n_x + n_acc + win * BATCH,
                       window_events_max=win * BATCH)
    d_acc = torch.empty((n_acc + treasury) * 128, dtype=torch.uint8, device="cuda")
    d_fund = torch.empty(max(n_acc, 1) * 128, dtype=torch.uint8, device="cuda")
    d_x = torch.empty(n_x * 128, dtype=torch.uint8, device="cuda")
    st = one.stream
    if a.stream == "cfg3":
        d_cdf = torch.from_numpy(workload.zipf_cdf(n_acc).view(np.int64).copy()).cuda()
        torch.cuda.synchronize()
        _lib.check(L.tbg_gen_accounts_cfg3(d_acc.data_ptr(), 0, n_acc + treasury, a.seed, n_acc, 1000, st), "gen")
        _lib.check(L.tbg_gen_funding_cfg3(d_fund.data_ptr(), 0, n_acc, a.seed, n_acc, treasury, 1_000_000, 10**15,
                                          st), "gen")
        _lib.check(L.tbg_gen_transfers_zipf(d_x.data_ptr(), 0, n_x, a.seed, n_acc, d_cdf.data_ptr(), 0, st), "gen")
    else:
        _lib.check(L.tbg_gen_accounts(d_acc.data_ptr(), 0, n_acc, a.seed, 2, 1, 0, st), "gen")
        _lib.check(L.tbg_gen_transfers_cfg4(d_x.data_ptr(), 0, n_x, a.seed, n_acc, BATCH, 0, st), "gen")
    torch.cuda.synchronize()
    d_res = torch.empty(win * BATCH * 8, dtype=torch.uint8, device="cuda")
    d_base = torch.zeros(256, dtype=torch.int32, device="cuda")

    def summed(tensors):
        torch.cuda.synchronize()
        total = tensors[0].clone()
        for t in tensors[1:]:
            total += t
        for t in tensors:
            t.copy_(total)
        torch.cuda.synchronize()

    ts_sh, ts_one = [0], [0]
    rows = []

    def windows(op, d_ev, n_total, tk, timed):
        nb = (n_total + BATCH - 1) // BATCH
        for b0 in range(0, nb, win):
            ns, ts = [], []
            for b in range(b0, min(b0 + win, nb)):
                n = min(BATCH, n_total - b * BATCH)
                ts_sh[0] += tk + 1 + n
                ns.append(n)
                ts.append(ts_sh[0])
            ptr = d_ev.data_ptr() + b0 * BATCH * 128
            # one unsharded engine
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            one.commit_window(op, ptr, ns, ts, d_res.data_ptr(), d_base.data_ptr(), True, ts[0])
            one.sync()
            t_one = time.perf_counter() - t0
            want = to_host(d_base)
            # the shards: batch 0's harness pulse (per-batch general path), then the window through
            # sharding.commit_general_window with each shard's steps timed (csrc/shard_gw.inc)
            if shards[0].pulse(ts[0]):
                pulse_general(shards, summed, ts[0])
            for s_ in shards:
                s_.gw_times = {}
            reps = commit_general_window(shards, summed, op, ptr, ns, ts, auto_pulse=False)
            per = [[s_.gw_times.get(0, 0.0) + s_.gw_times.get(1, 0.0), s_.gw_times.get(2, 0.0) + s_.gw_times.get(3, 0.0),
                    s_.gw_times.get(4, 0.0)] for s_ in shards]
            for s_ in shards:
                s_.gw_times = None
            fails = sum(len(x) // 8 for x in reps)
            assert fails == int(want[len(ns)]), (fails, int(want[len(ns)]))
            E = sum(ns)
            if timed:
                rows.append((E, t_one, per))

    windows(Operation.create_accounts, d_acc, n_acc + treasury, 0, False)
    if a.stream == "cfg3":
        windows(Operation.create_transfers, d_fund, n_acc, 0, False)
    windows(Operation.create_transfers, d_x, n_x, tick, True)
    timed = rows[a.warmup:]
    ev = sum(r[0] for r in timed)
    one_s = sum(r[1] for r in timed)
    crit = sum(max(sum(p) for p in r[2]) for r in timed)
    steps = np.array([[p for p in r[2]] for r in timed])  # windows x shards x 3
    out = {"stream": a.stream, "shards": G, "window_batches": win, "timed_windows": len(timed), "events_timed": ev,
           "unsharded_ms_per_window": round(one_s / len(timed) * 1000, 3),
           "unsharded_rate": round(ev / one_s, 1),
           "shard_ms_per_window": {"gather1_mean": round(float(steps[:, :, 0].mean()) * 1000, 3),
                                   "gather2_mean": round(float(steps[:, :, 1].mean()) * 1000, 3),
                                   "decide_apply_mean": round(float(steps[:, :, 2].mean()) * 1000, 3),
                                   "max_shard_mean": round(crit / len(timed) * 1000, 3)},
           "estimated_rate_excl_collective": round(ev / crit, 1),
           "note": "wall clock per step (host launches and syncs included); exchanges summed in-process, not counted",
           "shard_ms_per_window_split": {"gather1": round(float(steps[:, :, 0].mean()) * 1000, 3),
                                         "gather2": round(float(steps[:, :, 1].mean()) * 1000, 3),
                                         "scratch_commit_and_apply": round(float(steps[:, :, 2].mean()) * 1000, 3)}}
    out["scratch_objects_last_window"] = {"accounts": int(shards[0]._gw_n[0]), "transfers": int(shards[0]._gw_n[1])}
    print(json.dumps(out), flush=True)
    for s_ in shards:
        s_.close()
    one.close()


SLEEP_CYCLES = 400_000  # ~0.2 ms of GPU clock ahead of each timed step


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--shards", type=int, default=8)
    p.add_argument("--accounts", type=int, default=2_000_000, help="total over all shards")
    p.add_argument("--transfers", type=int, default=40_000_000, help="total over all shards")
    p.add_argument("--window", type=int, default=64, help="batches per (global) window")
    p.add_argument("--warmup", type=int, default=2, help="untimed windows")
    p.add_argument("--seed", type=int, default=47)
    p.add_argument("--protocol", default="routed", choices=["routed", "replicated"],
                   help="cfg5: routed = partitioned ingestion (csrc/route.h); replicated = every shard holds "
                        "the window, one all-reduce of facts (csrc/shard.h)")
    p.add_argument("--stream", default="cfg5", choices=["cfg5", "cfg3", "cfg4"],
                   help="cfg5: the order-free fast path; cfg3 / cfg4: the general class a window at a time")
    a = p.parse_args()
    if a.stream != "cfg5":
        return general(a)

    import torch

    from tigerbeetle_amd import _lib
    from tigerbeetle_amd.sharding import ShardedStateMachine
    from tigerbeetle_amd.types import Operation

    L = _lib.lib()
    G, win = a.shards, a.window
    n_acc, n_x = a.accounts, a.transfers
    shards = [ShardedStateMachine(G, r, None, batch_max=BATCH, accounts_max=int(n_acc / G * 1.05) + 65536,
                                  transfers_max=int(n_x / G * 1.05) + win * BATCH, window_events_max=win * BATCH)
              for r in range(G)]
    d_acc = torch.empty(n_acc * 128, dtype=torch.uint8, device="cuda")
    d_x = torch.empty(n_x * 128, dtype=torch.uint8, device="cuda")
    s0 = shards[0].sm.stream
    _lib.check(L.tbg_gen_accounts(d_acc.data_ptr(), 0, n_acc, a.seed, 2, 1, 0, s0), "gen")
    _lib.check(L.tbg_gen_transfers_uniform(d_x.data_ptr(), 0, n_x, a.seed, n_acc, 0, s0), "gen")
    torch.cuda.synchronize()
    d_res = torch.empty(win * BATCH * 8, dtype=torch.uint8, device="cuda")
    d_base = torch.zeros(G * 256, dtype=torch.int32, device="cuda")
    prepare_ts = 0
    times = []  # per window: per shard (prep ms, commit ms)

    def timed_step(fn):
        """Runs fn() on each shard's stream between two events; returns fn's results and the events."""
        outs, evs = [], []
        for r, s in enumerate(shards):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s.stream):
                # keep the GPU busy while the host submits, so e0..e1 is device time, not launch latency
                torch.cuda._sleep(SLEEP_CYCLES)
                e0.record()
                outs.append(fn(r, s))
                e1.record()
            s.stream.synchronize()
            evs.append((e0, e1))
        return outs, evs

    def summed(tensors):
        total = tensors[0].clone()
        for t in tensors[1:]:
            total += t
        for t in tensors:
            t.copy_(total)
        torch.cuda.synchronize()

    routed = a.protocol == "routed"
    xbytes = []  # routed: per window, the bytes each shard sends to the others (max over shards)

    def window_routed(op, d_ev, b0, b1, n_total, timed):
        """Partitioned ingestion (csrc/route.h): shard r reads only its home batches (a contiguous
        slice of the stream); the three all-to-alls are in-process block copies (not timed)."""
        nonlocal prepare_ts
        from tigerbeetle_amd.sharding import route_bounds, route_exchange_inprocess

        ns, ts = [], []
        for b in range(b0, b1):
            n = min(BATCH, n_total - b * BATCH)
            prepare_ts += 1 + n
            ns.append(n)
            ts.append(prepare_ts)
        if shards[0].pulse(ts[0]):  # the harness pulse before the window (the first one only here)
            from tigerbeetle_amd.sharding import pulse_general

            pulse_general(shards, summed, ts[0])
        bounds = route_bounds(len(ns), G)
        homes = [d_ev.data_ptr() + (b0 + bounds[r]) * BATCH * 128 for r in range(G)]
        _, ev1 = timed_step(lambda r, s: s.route_prepare(op, homes[r], ns, ts, bounds))
        sent = 0
        for phase in range(3):
            views = [s.route_views(phase) for s in shards]
            sent += max(sum(v[1]) - v[1][r] for r, v in enumerate(views))
            route_exchange_inprocess(shards, phase)
            if phase == 0:
                _, ev2 = timed_step(lambda r, s: s.route_step("own"))
            elif phase == 1:
                _, ev3 = timed_step(lambda r, s: s.route_step("decide"))
        _, ev4 = timed_step(lambda r, s: s.route_apply(d_res.data_ptr() + r * (d_res.numel() // G // 16 * 16),
                                                       d_base.data_ptr() + r * 256 * 4))
        for s in shards:
            s.sync()
        if timed:
            times.append([tuple(e[0].elapsed_time(e[1]) for e in evs) for evs in zip(ev1, ev2, ev3, ev4)])
            xbytes.append(sent)
        return sum(ns)

    def window(op, d_ev, b0, b1, n_total, timed):
        nonlocal prepare_ts
        if routed:
            return window_routed(op, d_ev, b0, b1, n_total, timed)
        ns, ts = [], []
        for b in range(b0, b1):
            n = min(BATCH, n_total - b * BATCH)
            prepare_ts += 1 + n
            ns.append(n)
            ts.append(prepare_ts)
        ptr = d_ev.data_ptr() + b0 * BATCH * 128
        if shards[0].pulse(ts[0]):  # the harness pulse before the window (the first one only here)
            from tigerbeetle_amd.sharding import pulse_general

            pulse_general(shards, summed, ts[0])
        words, ev1 = timed_step(lambda r, s: s.prepare_window(op, ptr, ns, ts))
        summed(words)
        _, ev2 = timed_step(lambda r, s: s.commit_prepared(*s.home_range(len(ns)), d_res.data_ptr(),
                                                           d_base.data_ptr() + r * 256 * 4))
        for s in shards:
            s.sync()
        if timed:
            times.append([(a[0].elapsed_time(a[1]), b_[0].elapsed_time(b_[1])) for a, b_ in zip(ev1, ev2)])
        return sum(ns)

    nb_acc = (n_acc + BATCH - 1) // BATCH
    for b0 in range(0, nb_acc, win):
        window(Operation.create_accounts, d_acc, b0, min(b0 + win, nb_acc), n_acc, False)
    nb = (n_x + BATCH - 1) // BATCH
    events = 0
    for k, b0 in enumerate(range(0, nb, win)):
        n = window(Operation.create_transfers, d_x, b0, min(b0 + win, nb), n_x, k >= a.warmup)
        if k >= a.warmup:
            events += n
    t = np.array(times)  # windows x shards x steps, ms
    per_shard = t.sum(axis=2)
    crit = per_shard.max(axis=1).sum() / 1000.0
    if routed:
        names = ["route", "own", "decide", "apply"]
        out = {
            "protocol": "routed", "shards": G, "window_batches": win, "timed_windows": len(times),
            "events_timed": events,
            "shard_ms_per_window": dict({n + "_mean": round(float(t[:, :, k].mean()), 4) for k, n in enumerate(names)},
                                        max_shard_mean=round(float(per_shard.max(axis=1).mean()), 4)),
            "estimated_rate_excl_collective": round(events / crit, 1),
            "alltoall_bytes_per_window_per_gpu_max": int(np.mean(xbytes)),
            "stats_shard0": shards[0].stats(),
        }
        print(json.dumps(out), flush=True)
        for s in shards:
            s.close()
        return
    out = {
        "shards": G, "window_batches": win, "timed_windows": len(times), "events_timed": events,
        "shard_ms_per_window": {"scan_mean": round(float(t[:, :, 0].mean()), 4),
                                "decide_apply_mean": round(float(t[:, :, 1].mean()), 4),
                                "max_shard_mean": round(float(per_shard.max(axis=1).mean()), 4)},
        "estimated_rate_excl_collective": round(events / crit, 1),
        "exchange_bytes_per_window": int(L.tbg_shard_exchange_bytes(int(Operation.create_transfers), win * BATCH, G)),
        "stats_shard0": shards[0].stats(),
    }
    print(json.dumps(out), flush=True)
    for s in shards:
        s.close()


if __name__ == "__main__":
    main()
