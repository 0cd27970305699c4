"""Host-fed routed windows through the native group (include/tbg.h tbg_group_commit_window), G shards on
ONE GPU with the copy exchange: each shard copies only its home batches host -> device (1/G of the
window's bytes), the three all-to-alls are device copies. Reports, per window, the H2D bytes per shard
and the wall time of the whole group call (host launches, the copy exchange's syncs and the replies'
read-back included). Not a bench line: evidence for DESIGN.md §7 (partitioned ingestion).

    python tools/group_hostfed.py --shards 8 --accounts 1000000 --transfers 20000000 --window 128
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

BATCH = 8190


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--shards", type=int, default=8)
    p.add_argument("--accounts", type=int, default=1_000_000)
    p.add_argument("--transfers", type=int, default=20_000_000)
    p.add_argument("--window", type=int, default=128)
    p.add_argument("--warmup", type=int, default=2)
    a = p.parse_args()

    from tigerbeetle_amd import workload
    from tigerbeetle_amd.group import GroupStateMachine
    from tigerbeetle_amd.types import Operation

    G, win = a.shards, a.window
    g = GroupStateMachine(G, batch_max=BATCH, accounts_max=int(a.accounts / G * 1.1) + 65536,
                          transfers_max=int(a.transfers / G * 1.1) + win * BATCH, window_events_max=win * BATCH)
    acc = workload.accounts(0, a.accounts, seed=47)
    for w0 in range(0, a.accounts, win * BATCH):
        part = acc[w0: w0 + win * BATCH]
        g.commit_window(Operation.create_accounts, [part[i:i + BATCH] for i in range(0, len(part), BATCH)])
    rows = []
    for k, w0 in enumerate(range(0, a.transfers, win * BATCH)):
        n = min(win * BATCH, a.transfers - w0)
        x = workload.transfers_uniform(w0, n, seed=47, n_accounts=a.accounts)
        batches = [x[i:i + BATCH] for i in range(0, n, BATCH)]
        t0 = time.perf_counter()
        reps = g.commit_window(Operation.create_transfers, batches)
        dt = time.perf_counter() - t0
        assert all(r == b"" for r in reps)
        if k >= a.warmup:
            rows.append((n, dt, len(batches)))
    ev = sum(r[0] for r in rows)
    wall = sum(r[1] for r in rows)
    nb = rows[0][2]
    per_shard_batches = [nb * (r + 1) // G - nb * r // G for r in range(G)]
    out = {"shards": G, "window_batches": win, "timed_windows": len(rows), "events_timed": ev,
           "ms_per_window": round(wall / len(rows) * 1000, 3), "rate_events_per_s": round(ev / wall, 1),
           "h2d_bytes_per_window_total": nb * BATCH * 128,
           "h2d_bytes_per_window_per_shard": [b * BATCH * 128 for b in per_shard_batches],
           "exchange": "copy (every shard on this GPU; host-synchronized device copies)",
           "stats_shard0": g.shards[0].stats()}
    print(json.dumps(out), flush=True)
    g.close()


if __name__ == "__main__":
    main()
