"""Per-shard GPU time of the hash-sharded commit at G shards, rehearsed on ONE GPU.

G ShardedStateMachine engines live on cuda:0 in this process. Each window runs shard by shard
(prepare -> in-process byte-wise sum of the facts, i.e. what the RCCL all-reduce computes -> decide
(home batches) -> sum of the commit bits -> commit), with HIP events on each engine's stream around
each step. A shard's GPU time per window is what one GPU of a G-GPU node spends on the window apart
from the collectives, so

    estimated G-GPU rate = global events / sum over windows of max over shards (prep + decide + commit)

is an upper bound for the real node (the all-reduces of 9 B + 1 bit per event are added on top).
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


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--shards", type=int, default=8)
    p.add_argument("--accounts", type=int, default=2_000_000, help="total over all shards")
    p.add_argument("--transfers", type=int, default=40_000_000, help="total over all shards")
    p.add_argument("--window", type=int, default=64, help="batches per (global) window")
    p.add_argument("--warmup", type=int, default=2, help="untimed windows")
    p.add_argument("--seed", type=int, default=47)
    a = p.parse_args()

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

    def window(op, d_ev, b0, b1, n_total, timed):
        nonlocal prepare_ts
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
        bits, ev2 = timed_step(lambda r, s: s.decide_window(*s.home_range(len(ns)), d_res.data_ptr(),
                                                            d_base.data_ptr() + r * 256 * 4))
        summed(bits)
        _, ev3 = timed_step(lambda r, s: s.commit_decided())
        for s in shards:
            s.sync()
        if timed:
            times.append([(a[0].elapsed_time(a[1]), b_[0].elapsed_time(b_[1]), c[0].elapsed_time(c[1]))
                          for a, b_, c in zip(ev1, ev2, ev3)])
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
    t = np.array(times)  # windows x shards x (prep, decide, commit), ms
    per_shard = t.sum(axis=2)
    crit = per_shard.max(axis=1).sum() / 1000.0
    out = {
        "shards": G, "window_batches": win, "timed_windows": len(times), "events_timed": events,
        "shard_ms_per_window": {"prep_mean": round(float(t[:, :, 0].mean()), 4),
                                "decide_mean": round(float(t[:, :, 1].mean()), 4),
                                "commit_mean": round(float(t[:, :, 2].mean()), 4),
                                "max_shard_mean": round(float(per_shard.max(axis=1).mean()), 4)},
        "estimated_rate_excl_collective": round(events / crit, 1),
        "exchange_bytes_per_window": (16 + 2 * win * BATCH + 8 * G * 4096) + 16 + win * BATCH // 8,
        "stats_shard0": shards[0].stats(),
    }
    print(json.dumps(out), flush=True)
    for s in shards:
        s.close()


if __name__ == "__main__":
    main()
