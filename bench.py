"""Benchmark: committed create_transfers per second on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], "cfg2"): 1M accounts, then 100M uniform-random create_transfers
(no flags) in 8190-event batches, generated directly in HBM (synthetic; shape of
src/tigerbeetle/benchmark_load.zig:206-327). A "step" is one create_transfers batch of the stream,
committed through the engine's device-resident C ABI in windows of --window consecutive batches
(tbg_commit_window: pulse decision + pulse, then the batches with their own timestamps and replies,
state_machine.zig:2719-2739). The first W batches are warmup; the next K are timed between barrier +
stream syncs, max over ranks.

Multi-GPU (torchrun, one rank per GPU): every rank owns an independent account shard and its own
stream of the same shape (weak scaling, no data-path collective yet; cross-shard exchange is the
next step).

Extra JSON fields: `roofline` for the dominant kernel (HIP events on the engine stream over the
timed region) and `cpu_baseline` (the single-threaded C restatement, oracle/, on a bounded sample
of the same stream, rank 0 only).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BATCH = 8190
PHASES = ["prep", "link", "classify", "wcount", "wlist", "walk", "final", "pulse"]
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s HBM3E spec

# Algorithmic bytes per event of each kernel on the cfg2 path (DESIGN.md §5 derives them).
KERNEL_BYTES_PER_EVENT = {
    # event read 128, two account-table entries 2x32, transfer-id probe 32, window key-map entry 32,
    # per-event scratch written 72 (code, cls, batch, 4 slots/entries, amt, ...)
    "prep": 128 + 2 * 32 + 32 + 32 + 72,
    # event read 128, record append 128, id-table entry 32, two balance pairs read+write 2x64 (atomics),
    # scratch read 40, key-map entry reset 32
    "final": 128 + 128 + 32 + 2 * 64 + 40 + 32,
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None, help="timed batches (default: rest of the 100M stream)")
    p.add_argument("--warmup", type=int, default=256, help="warmup batches (rounded to whole windows)")
    p.add_argument("--window", type=int, default=32, help="batches per commit window (super-batching)")
    p.add_argument("--accounts", type=int, default=1_000_000)
    p.add_argument("--transfers", type=int, default=100_000_000)
    p.add_argument("--seed", type=int, default=44)
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget (commit time)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-phase-timing", action="store_true")
    p.add_argument("--verify", action="store_true", help="check all results ok and the balance invariants")
    return p.parse_args()


def cpu_baseline(args, n_accounts, seed):
    """Single-threaded C restatement (oracle/liboracle.so) on a time-bounded prefix of the same
    stream; only commit calls are timed."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_sm import lib as olib

    from tigerbeetle_amd import workload
    from tigerbeetle_amd.types import RESULT_DTYPE

    L = olib()
    h = L.tbo_create(BATCH)
    out = np.zeros(BATCH, RESULT_DTYPE)
    ts = 0
    for first in range(0, n_accounts, BATCH):
        ev = workload.accounts(first, min(BATCH, n_accounts - first), seed)
        ts += 1 + len(ev)
        L.tbo_create_accounts(h, ts, ev.ctypes.data, len(ev), out.ctypes.data)
    if L.tbo_pulse_needed(h, ts):
        L.tbo_pulse(h, ts)
    spent, events, first = 0.0, 0, 0
    chunk = 32 * BATCH
    while spent < args.cpu_seconds and first < args.transfers:
        evs = workload.transfers_uniform(first, chunk, seed, n_accounts)
        for b in range(0, chunk, BATCH):
            ev = evs[b:b + BATCH]
            ts += 1 + len(ev)
            t0 = time.perf_counter()
            if L.tbo_pulse_needed(h, ts):
                L.tbo_pulse(h, ts)
            c = L.tbo_create_transfers(h, ts, ev.ctypes.data, len(ev), out.ctypes.data)
            spent += time.perf_counter() - t0
            assert c == 0
            events += len(ev)
        first += chunk
    L.tbo_destroy(h)
    return {
        "value": events / spent,
        "unit": "transfers/s",
        "cores": 1,
        "kind": "port",
        "sample": f"first {events} transfers of the same cfg2 stream after {n_accounts} accounts, "
                  f"{spent:.1f} s of commit time on 1 host core (oracle/tb_oracle.c, -O2)",
    }


def main():
    args = parse()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        torch.cuda.set_device(0)
    device = torch.cuda.current_device()

    from tigerbeetle_amd import StateMachine, _lib
    from tigerbeetle_amd.types import Operation

    L = _lib.lib()
    n_acc = args.accounts
    total_batches = (args.transfers + BATCH - 1) // BATCH
    steps = args.steps if args.steps is not None else total_batches - args.warmup
    n_batches = min(total_batches, args.warmup + steps)
    n_xfer = min(args.transfers, n_batches * BATCH)
    seed = args.seed + 1000 * rank  # independent stream per shard

    win = max(1, min(args.window, 64))
    sm = StateMachine(device=device, batch_max=BATCH, accounts_max=n_acc, transfers_max=n_xfer,
                      window_events_max=win * BATCH)
    stream = sm.stream
    ext = torch.cuda.ExternalStream(stream)

    # Inputs resident in HBM before timing.
    d_acc = torch.empty(n_acc * 128, dtype=torch.uint8, device="cuda")
    d_xfer = torch.empty(n_xfer * 128, dtype=torch.uint8, device="cuda")
    d_res = torch.empty(max(n_xfer, n_acc) * 8, dtype=torch.uint8, device="cuda")
    n_windows_max = (max(n_batches, (n_acc + BATCH - 1) // BATCH) + win - 1) // win + 1
    d_base = torch.zeros(n_windows_max * 65, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    _lib.check(L.tbg_gen_accounts(d_acc.data_ptr(), 0, n_acc, seed, 2, 1, 0, stream), "gen accounts")
    _lib.check(L.tbg_gen_transfers_uniform(d_xfer.data_ptr(), 0, n_xfer, seed, n_acc, 0, stream), "gen transfers")

    prepare_ts = 0
    windows = []  # (op, first_event, [n_b]) for verification

    def commit_range(op, d_events, first_batch, last_batch, n_total, widx):
        """Commits batches [first_batch, last_batch) as one window; harness timestamps (:2719-2739)."""
        nonlocal prepare_ts
        ns, ts = [], []
        for b in range(first_batch, last_batch):
            n = min(BATCH, n_total - b * BATCH)
            prepare_ts += 1 + n
            ns.append(n)
            ts.append(prepare_ts)
        first_ev = first_batch * BATCH
        sm.commit_window(op, d_events.data_ptr() + first_ev * 128, ns, ts, d_res.data_ptr() + first_ev * 8,
                         d_base.data_ptr() + widx * 65 * 4, True, ts[0])
        windows.append((op, widx, len(ns)))

    acc_batches = (n_acc + BATCH - 1) // BATCH
    widx = 0
    for b0 in range(0, acc_batches, win):
        commit_range(Operation.create_accounts, d_acc, b0, min(b0 + win, acc_batches), n_acc, widx)
        widx += 1
    _lib.check(L.tbg_sync(sm.h), "sync (accounts)")
    acc_fail = sum(int(d_base[w * 65 + nb].item()) for _, w, nb in windows)
    windows.clear()
    d_base.zero_()

    warm = min(((args.warmup + win - 1) // win) * win, max(0, n_batches - win))
    widx = 0
    for b0 in range(0, warm, win):
        commit_range(Operation.create_transfers, d_xfer, b0, min(b0 + win, warm), n_xfer, widx)
        widx += 1
    _lib.check(L.tbg_sync(sm.h), "sync (warmup)")
    if dist:
        dist.barrier()
    NPH = len(PHASES)
    L.tbg_timing_collect(sm.h, (ctypes.c_double * NPH)(), (ctypes.c_uint64 * NPH)(), NPH)  # reset
    L.tbg_timing_enable(sm.h, 0 if args.no_phase_timing else 1)

    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    start.record(ext)
    for b0 in range(warm, n_batches, win):
        commit_range(Operation.create_transfers, d_xfer, b0, min(b0 + win, n_batches), n_xfer, widx)
        widx += 1
    end.record(ext)
    _lib.check(L.tbg_sync(sm.h), "sync (timed)")
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    gpu_ms = start.elapsed_time(end)
    if dist:
        dist.barrier()
    L.tbg_timing_enable(sm.h, 0)
    ms = (ctypes.c_double * NPH)()
    launches = (ctypes.c_uint64 * NPH)()
    L.tbg_timing_collect(sm.h, ms, launches, NPH)
    args.warmup = warm

    timed_batches = n_batches - args.warmup
    timed_events = n_xfer - args.warmup * BATCH
    elapsed = max(wall, gpu_ms / 1000.0)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        ev_t = torch.tensor([timed_events], dtype=torch.float64, device="cuda")
        dist.all_reduce(ev_t, op=dist.ReduceOp.SUM)
        all_events = float(ev_t.item())
    else:
        all_events = float(timed_events)

    bases = d_base.view(-1, 65).cpu().numpy()
    fails = int(sum(bases[w, nb] for _, w, nb in windows))
    stats = sm.stats()
    if args.verify:
        assert acc_fail == 0 and fails == 0, (acc_fail, fails)
        assert stats["transfers"] == n_xfer

    if rank == 0:
        per_phase = {PHASES[p]: (ms[p] / launches[p] * 1000.0 if launches[p] else None) for p in range(NPH)}
        dom = max(("prep", "final"), key=lambda k: per_phase[k] or 0.0)
        roof = None
        if per_phase[dom]:
            us = per_phase[dom]
            ev_per_launch = timed_events / max(launches[PHASES.index(dom)], 1)
            bytes_launch = int(KERNEL_BYTES_PER_EVENT[dom] * ev_per_launch)
            achieved = bytes_launch / (us * 1e-6) / 1e9
            kname = {"prep": "k_ct_prep", "final": "k_final<true>"}[dom]
            roof = {"bound": "hbm", "kernel": kname, "events_per_launch": int(ev_per_launch), "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                    "avg_launch_us": round(us, 2), "alg_bytes_per_launch": bytes_launch,
                    "phase_avg_us": {k: (round(v, 2) if v else None) for k, v in per_phase.items()},
                    "path_alg_GBs": round(640 * all_events / elapsed / 1e9 / max(world, 1), 1)}
        line = {
            "metric": "committed transfers/sec (create_transfers)",
            "value": round(all_events / elapsed, 1),
            "unit": "transfers/s",
            "n_gpus": world,
            "steps": timed_batches,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1000.0 / timed_batches, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u128",
            "data": "synthetic (device-generated, seed %d)" % args.seed,
            "config": {"workload": "cfg2: %d accounts, %d uniform create_transfers (no flags), %d/batch"
                                   % (n_acc, n_xfer, BATCH),
                       "batch": BATCH, "window_batches": win, "accounts_per_gpu": n_acc, "transfers_per_gpu": n_xfer,
                       "parallelism": "independent account shards" if world > 1 else "single GPU"},
            "results": {"failed_events": fails, "walker_events": stats["walker_events"],
                        "gpu_ms_timed": round(gpu_ms, 3), "wall_ms_timed": round(wall * 1000, 3)},
            "roofline": roof,
        }
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args, n_acc, seed)
        print(json.dumps(line), flush=True)
    sm.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
