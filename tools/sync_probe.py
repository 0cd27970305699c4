"""Where the synchronous StateMachine path's time goes (bench.py sync_commit): per call wall times of
pulse(), prefetch() and commit() over k batches of the cfg2 stream from a pinned message pool, the
same through the raw C ABI (no Python wrapper), and the bare H2D of one 1 MiB request. Evidence for
DESIGN.md, not a bench line. Usage (GPU box): python tools/sync_probe.py [--batches 64]"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

BATCH = 8190


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batches", type=int, default=64)
    p.add_argument("--accounts", type=int, default=100_000)
    p.add_argument("--no-copy-probe", action="store_true", help="end after the raw ABI loop (device timelines)")
    a = p.parse_args()
    import torch

    from tigerbeetle_amd import StateMachine, _lib, workload
    from tigerbeetle_amd.state_machine import HostBuffer
    from tigerbeetle_amd.types import Operation

    L = _lib.lib()
    k = a.batches
    sm = StateMachine(batch_max=BATCH, accounts_max=a.accounts, transfers_max=4 * k * BATCH + 1024)
    acc = workload.accounts(0, a.accounts, seed=3)
    for f in range(0, a.accounts, BATCH):
        body = acc[f:f + BATCH].tobytes()
        sm.prepare_timestamp += len(body) // 128
        sm.commit(0, 1, sm.prepare_timestamp, Operation.create_accounts, body)
    pool = HostBuffer(3 * k * BATCH * 128)
    evs = workload.transfers_uniform(0, 3 * k * BATCH, 7, a.accounts)
    pool.array[:] = evs.view(np.uint8).reshape(-1)
    bodies = [pool.array[b * BATCH * 128:(b + 1) * BATCH * 128] for b in range(3 * k)]
    out = {}

    def wrapper_loop(bs):
        tp = tf = tc = 0.0
        t0 = time.perf_counter()
        for b in bs:
            sm.prepare_timestamp += 1 + BATCH
            T = sm.prepare_timestamp
            x0 = time.perf_counter()
            if sm.pulse():
                sm.commit(0, 1, T, Operation.pulse, b"")
            x1 = time.perf_counter()
            sm.prefetch_timestamp = T
            sm.prefetch(2, Operation.create_transfers, b)
            x2 = time.perf_counter()
            sm.commit(0, 2, T, Operation.create_transfers, b)
            x3 = time.perf_counter()
            tp, tf, tc = tp + x1 - x0, tf + x2 - x1, tc + x3 - x2
        n = len(bs)
        return {"us_per_batch": round((time.perf_counter() - t0) / n * 1e6, 1), "pulse_us": round(tp / n * 1e6, 1),
                "prefetch_us": round(tf / n * 1e6, 1), "commit_us": round(tc / n * 1e6, 1)}

    wrapper_loop(bodies[:8])  # warm-up
    out["wrapper"] = wrapper_loop(bodies[8:8 + k])

    # the raw C ABI (what a Zig replica calls): no numpy views, no wrapper
    h = sm.h
    res = np.zeros(BATCH * 8, np.uint8)
    n_out = ctypes.c_uint64()
    need = ctypes.c_int()
    tp = tf = tc = 0.0
    t0 = time.perf_counter()
    for b in bodies[8 + k:8 + 2 * k]:
        sm.prepare_timestamp += 1 + BATCH
        T = sm.prepare_timestamp
        ptr = b.ctypes.data
        x0 = time.perf_counter()
        L.tbg_pulse_needed(h, T, ctypes.byref(need))
        if need.value:
            L.tbg_commit(h, 1, T, int(Operation.pulse), None, 0, res.ctypes.data, res.size, ctypes.byref(n_out))
        x1 = time.perf_counter()
        L.tbg_prefetch(h, 2, int(Operation.create_transfers), ptr, BATCH * 128, T)
        x2 = time.perf_counter()
        rc = L.tbg_commit(h, 2, T, int(Operation.create_transfers), ptr, BATCH * 128, res.ctypes.data, res.size,
                          ctypes.byref(n_out))
        x3 = time.perf_counter()
        assert rc == 0
        tp, tf, tc = tp + x1 - x0, tf + x2 - x1, tc + x3 - x2
    out["raw_abi"] = {"us_per_batch": round((time.perf_counter() - t0) / k * 1e6, 1),
                      "pulse_us": round(tp / k * 1e6, 1), "prefetch_us": round(tf / k * 1e6, 1),
                      "commit_us": round(tc / k * 1e6, 1)}
    if a.no_copy_probe:
        print(json.dumps(out), flush=True)
        return
    # the bare copy: one 1 MiB H2D from pinned memory, synchronized
    dst = torch.empty(BATCH * 128, dtype=torch.uint8, device="cuda")
    src = torch.from_numpy(bodies[0])
    ts = []
    for _ in range(32):
        torch.cuda.synchronize()
        x0 = time.perf_counter()
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - x0)
    out["h2d_1MiB_us"] = round(float(np.median(ts)) * 1e6, 1)
    ts = []
    for _ in range(32):
        x0 = time.perf_counter()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - x0)
    out["empty_sync_us"] = round(float(np.median(ts)) * 1e6, 1)
    out["fused_windows"] = sm.stats()["fused_windows"]
    print(json.dumps(out), flush=True)
    bodies = None
    pool.close()
    sm.close()


if __name__ == "__main__":
    main()
