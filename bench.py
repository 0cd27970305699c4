"""Benchmark: committed create_transfers per second on MI355X (BASELINE.json metric).

Default workload (BASELINE.json configs[1], "cfg2"): 1M accounts, then 100M uniform-random
create_transfers (no flags) in 8190-event batches, generated directly in HBM (synthetic; shape of
src/tigerbeetle/benchmark_load.zig:206-327). `--config` selects the other BASELINE configs:
  cfg1  10k accounts, 1M uniform transfers (the reference CPU benchmark shape)
  cfg3  Zipf(1.2) hot accounts, debits_must_not_exceed_credits on >= 50 % (incl. the top 1000),
        pre-funded from treasury accounts (funding untimed), 10M transfers
  cfg4  two-phase (30 % pending, post/void, expiry) + linked chains with injected failures,
        synthetic clock +1 s per batch (a pulse is due before every batch), 10M transfers, in
        128-batch windows whose inner pulses the engine models (csrc/xwin.h)
  cfg5  hash-sharded over the N GPUs (default when N > 1): 12.5M accounts and 125M uniform transfers
        per GPU (100M / 1B at N = 8), ~(N-1)/N of the transfers cross-shard; one stream for the whole
        job, resident in every GPU's HBM; per window one RCCL all-reduce of the per-event owner facts
        (2 B), after which every shard decides every event (tigerbeetle_amd/sharding.py, csrc/shard.h)

A "step" is one create_transfers batch of the stream, committed through the engine's
device-resident C ABI in windows of --window consecutive batches (tbg_commit_window: pulse
decision + pulse, then the batches with their own timestamps and replies, the harness order of
state_machine.zig:2719-2739). The whole configured stream is always committed (so the engine's
state reaches the config's full size): the first W batches (rounded up to whole windows) are
warmup, and every later batch is timed between barrier + stream syncs, max over ranks; --steps K is
a minimum, and `steps` reports the timed count. `value` counts every committed event (failed ones too:
they are committed with a result code); `results.ok_events_per_s` counts the successful ones.

Multi-GPU (torchrun, one rank per GPU): cfg5 shards one global stream over the ranks (accounts and
transfer ids hash-partitioned, cross-shard facts exchanged by RCCL all-reduce; weak scaling: the
stream grows with N). cfg1-cfg4 at N > 1 run N independent databases (one per rank, own stream, no
data-path collective) and are labelled "replicas", not a scaling run. See DESIGN.md §7.

Extra JSON fields: `roofline` for the dominant kernel (HIP events on the engine stream over the
timed region) and `cpu_baseline` (the single-threaded C restatement, oracle/, on a bounded prefix
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
WINDOW_BATCHES_MAX = 128  # csrc/window.h MAXB: batches per commit window
PHASES = ["prep", "resolve", "classify", "wcount", "wlist", "walk", "final", "pulse", "cpw", "fused"]
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s HBM3E spec
NS_PER_S = 1_000_000_000

# Algorithmic bytes per window event of each phase: SURVEY §8(d)'s 640 B/event path (event read 128,
# dr/cr account records 2 x 128, balance pairs written 2 x 32, transfer append 128, id keys 4 x 16)
# split over the phases that move them; none of the engine's own scratch columns count.
PHASE_ALG_BYTES = {
    # event read 128, id keys: two account-id probes and the transfer-id probe 3 x 16, transfer
    # record appended 128
    "prep": 128 + 3 * 16 + 128,
    # the dr/cr account records 2 x 128 and their balance pairs written 2 x 32, the transfer-id insert 16
    "final": 2 * 128 + 2 * 32 + 16,
    # the chunked resolver (balance-limit windows): per event side its amount 16 and its check bit
    "resolve": 2 * (16 + 1),
    # the fused pass (csrc/fused.h) moves the whole path in one launch: all of SURVEY 8(d)'s 640 B
    "fused": 640,
}
# the kernels each timed phase launches (the first is the one named in `roofline.kernel`)
PHASE_KERNELS = {
    "prep": ["k_ct_prep", "k_prep_reduce", "k_claim_fix", "k_bind_sum", "k_bind_decide", "k_bind_finish"],
    "final": ["k_final<true>"],
    "resolve": ["k_rc_run", "k_res_keys", "k_rc_build", "k_rc_sum", "k_res_apply", "k_res_final"],
    "cpw": ["k_cc_walk<true>", "k_cc_init", "k_cc_link", "k_cc_keys", "onesweep sort", "k_cc_segs"],
    "classify": ["k_classify<true>"], "wlist": ["k_wlist"], "walk": ["k_walk<true>", "k_wfold"],
    "pulse": ["k_pulse", "k_xwin_rb", "k_xwin_minlive", "k_xwin_replay", "k_xwin_expire"],
    "fused": ["k_ct_fused<false>"],  # k_fu_final (replies, ~12 us per 1M) runs outside the timed phase
}
# the walkers (cpw, walk) run the reference loop for the events they decide: event 128, balance
# pairs 2 x 32, record 128 per walked event
WALKED_EVENT_BYTES = 128 + 2 * 32 + 128

CONFIGS = {
    "cfg1": dict(accounts=10_000, transfers=1_000_000, window=32, seed=42, tick=0),
    "cfg2": dict(accounts=1_000_000, transfers=100_000_000, window=128, seed=44, tick=0),
    "cfg3": dict(accounts=1_000_000, transfers=10_000_000, window=32, seed=45, tick=0),
    "cfg4": dict(accounts=1_000_000, transfers=10_000_000, window=128, seed=46, tick=NS_PER_S),
    # per GPU (weak scaling): 100M accounts / 1B transfers at 8 GPUs
    "cfg5": dict(accounts=12_500_000, transfers=125_000_000, window=128, seed=47, tick=0),
}
PENDING_TIMEOUT = 3600  # --pending-every: pending creates that stay pending for the whole run
CFG3_TREASURY, CFG3_TOP, CFG3_FUND, CFG3_FUND_ID = 1000, 1000, 1_000_000, 10**15


def warm_phases(sm, nph):
    """Per-phase average launch time (us) over the warmup windows, timed with every phase recording
    events, and the roofline kernel's phase (prep or final, whichever is longer)."""
    from tigerbeetle_amd import _lib
    L = _lib.lib()
    ms = (ctypes.c_double * nph)()
    launches = (ctypes.c_uint64 * nph)()
    L.tbg_timing_collect(sm.h, ms, launches, nph)
    per_phase = {PHASES[p]: (ms[p] / launches[p] * 1000.0 if launches[p] else None) for p in range(nph)}
    dom = max(PHASES, key=lambda k: per_phase[k] or 0.0)
    return per_phase, dom


def pmc_tag(args):
    """The name of this bench line's PMC summary: the config, then the options that change the
    kernels' traffic (the id order, the change log, the pending share), e.g. cfg2_random."""
    tag = args.config
    if args.id_order != "sequential":
        tag += "_" + args.id_order
    if args.change_log:
        tag += "_changelog"
    if args.pending_every:
        tag += "_pending%d" % args.pending_every
    return tag


def pmc_traffic(config, kernel, events_per_launch):
    """Per-launch HBM traffic of `kernel` from the committed rocprofv3 PMC summary of this exact line
    (profiles/r<N>/pmc_<pmc_tag>.json, made by `tools/gpu.sh prof <pmc_tag> <bench args>`: separate
    FETCH_SIZE and WRITE_SIZE passes over the same bench command, summarized by tools/pmc_summary.py),
    scaled to this run's events per launch. None when this line has no summary of its own (a
    variant's traffic is never borrowed from another line's). Returns (raw FETCH+WRITE bytes, bytes
    with FETCH doubled per the gfx950 streaming-read correction, source) or None."""
    for rnd in ("r6", "r5", "r4", "r3", "r2", "r1"):  # the latest round's summary of this config
        path = os.path.join(ROOT, "profiles", rnd, "pmc_%s.json" % config)
        if os.path.exists(path):
            break
    else:
        return None
    with open(path) as f:
        ks = json.load(f)["kernels"]
    k = ks.get(kernel) or ks.get(kernel.split("<")[0])  # (earlier rounds' summaries: untemplated names)
    if not k:
        return None
    # per-event grids scale with this run's events per launch; a fixed grid (k_rc_run: one workgroup)
    # reports the profiled launch as is
    scale = events_per_launch / max(k["grid"], 1) if k["grid"] * 2 >= events_per_launch else 1.0
    return (round(k["traffic_bytes"] * scale), round(k["traffic_fetch_x2_bytes"] * scale),
            os.path.relpath(path, ROOT))


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--config", default=None, choices=sorted(CONFIGS),
                   help="default: cfg2 on one GPU, cfg5 (sharded) on several")
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                   help="process group; gloo lets ranks share one GPU (rehearsal), exchange via host")
    p.add_argument("--steps", type=int, default=None,
                   help="minimum timed batches: the whole configured stream is always committed, the first "
                        "--warmup batches untimed and every later batch timed (so the timed count is >= steps)")
    p.add_argument("--warmup", type=int, default=None, help="warmup batches (rounded to whole windows)")
    p.add_argument("--window", type=int, default=None, help="batches per commit window (super-batching)")
    p.add_argument("--accounts", type=int, default=None)
    p.add_argument("--transfers", type=int, default=None)
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget (commit time)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-phase-timing", action="store_true")
    p.add_argument("--resolver", default="chunks", choices=["chunks", "relax", "wait", "off"],
                   help="balance-limit windows: chunked single-workgroup resolver where the window fits it "
                        "(default), grid-wide windowed relaxation, wait-based walkers, walker only")
    p.add_argument("--verify", action="store_true", help="setup all ok; cfg1/cfg2: every transfer ok")
    p.add_argument("--host-fed-transfers", type=int, default=None,
                   help="cfg1/cfg2: after the timed run, commit this many further transfers of the same stream "
                        "from pinned host memory (tbg_commit_window_host, H2D overlapped with compute) and report "
                        "it as `host_fed` (never `value`); default 32 windows (the pipeline fill, one unoverlapped H2D, is 1/32 of it), 0 = off")
    p.add_argument("--id-order", default="sequential", choices=["sequential", "random", "reversed", "time"],
                   help="account and transfer ids as the reference benchmark's --id-order (cli.zig:97, 263-265; "
                        "testing/id.zig IdPermutation; random = pseudo-UUIDs from Xoshiro256, the reference's own ids "
                        "for the permutation seed DefaultPrng(seed) draws first); time = the time-based 128-bit ids "
                        "the reference's docs recommend (docs/develop/data-modeling.md:186-203: 48-bit ms above 80 "
                        "random bits, strictly increasing)")
    p.add_argument("--sync-commit-batches", type=int, default=None,
                   help="cfg1/cfg2: after the timed run, commit this many further batches one at a time through the "
                        "synchronous tbg_prefetch + tbg_commit from host memory (a replica that does not pipeline) and "
                        "report it as `sync_commit` (never `value`); default 64, 0 = off")
    p.add_argument("--pending-every", type=int, default=0,
                   help="cfg1/cfg2 mixed stream: every N-th transfer is a pending create (flags.pending, timeout "
                        "%d s; N=100 is ~1%% pending), 0 = none (the headline stream)" % PENDING_TIMEOUT)
    p.add_argument("--change-log", action="store_true",
                   help="engine keeps the write-back change log (TBG_FLAG_CHANGE_LOG): its device cost")
    a = p.parse_args()
    if a.config is None:
        a.config = "cfg5" if int(os.environ.get("WORLD_SIZE", "1")) > 1 else "cfg2"
    c = CONFIGS[a.config]
    a.window_set = a.window is not None
    for k in ("accounts", "transfers", "window", "seed"):
        if getattr(a, k) is None:
            setattr(a, k, c[k])
    if a.warmup is None:
        a.warmup = 256 if a.config == "cfg2" else 32
    if a.host_fed_transfers is None:
        a.host_fed_transfers = 32 * min(a.window if a.config == "cfg2" else 32, WINDOW_BATCHES_MAX) * BATCH if a.config in ("cfg1", "cfg2") else 0
    if a.sync_commit_batches is None:
        a.sync_commit_batches = 64 if a.config in ("cfg1", "cfg2") else 0
    a.tick = c["tick"]
    if a.pending_every and a.config not in ("cfg1", "cfg2"):
        p.error("--pending-every applies to the uniform streams (cfg1, cfg2)")
    from tigerbeetle_amd import workload

    a.id_order_code = workload.ID_ORDERS[a.id_order]
    a.perm_seed = workload.benchmark_permutation_seed(a.seed)
    return a


class HostStream:
    """Numpy twin of the device stream (tigerbeetle_amd/workload.py), for the CPU baseline."""

    def __init__(self, args, seed):
        from tigerbeetle_amd import workload

        self.w, self.a, self.seed = workload, args, seed
        self.cdf = workload.zipf_cdf(args.accounts) if args.config == "cfg3" else None

    def n_accounts_total(self):
        return self.a.accounts + (CFG3_TREASURY if self.a.config == "cfg3" else 0)

    def _ids(self, recs):
        return self.w.permute_ids(recs, self.a.id_order_code, self.a.perm_seed)

    def accounts(self, first, count):
        if self.a.config == "cfg3":
            return self._ids(self.w.accounts_cfg3(first, count, self.seed, self.a.accounts, CFG3_TOP))
        return self._ids(self.w.accounts(first, count, self.seed))

    def funding(self, first, count):
        return self._ids(self.w.funding_cfg3(first, count, self.seed, self.a.accounts, CFG3_TREASURY, CFG3_FUND,
                                             CFG3_FUND_ID))

    def transfers(self, first, count):
        a = self.a
        if a.config == "cfg3":
            return self._ids(self.w.transfers_zipf(first, count, self.seed, a.accounts, self.cdf))
        if a.config == "cfg4":
            return self._ids(self.w.transfers_cfg4(first, count, self.seed, a.accounts, BATCH))
        return self._ids(self.w.mark_pending(self.w.transfers_uniform(first, count, self.seed, a.accounts), first,
                                             a.pending_every, PENDING_TIMEOUT))


def host_cpu():
    """The host's CPU model and core counts (the baseline names its cores)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = None
    return {"cpu_model": model, "nproc": os.cpu_count(), "usable_cpus": usable}


def host_fed(args, sm, torch, first, n_acc, seed, win):
    """The replica-shaped input path: `n` further transfers of the same stream staged in pinned host
    memory, committed with tbg_commit_window_host (each window's H2D on a copy stream overlapping the
    previous window's kernels, replies copied back to pinned host memory). Timed from the first
    submission to the last reply."""
    from tigerbeetle_amd import _lib
    from tigerbeetle_amd.types import Operation

    L = _lib.lib()
    n = (args.host_fed_transfers // BATCH) * BATCH
    d_tmp = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    _lib.check(L.tbg_gen_transfers_uniform(d_tmp.data_ptr(), first, n, seed, n_acc, 0, sm.stream), "gen")
    _lib.check(L.tbg_gen_mark_pending(d_tmp.data_ptr(), first, n, args.pending_every, PENDING_TIMEOUT, sm.stream),
               "pending")
    _lib.check(L.tbg_gen_permute_ids(d_tmp.data_ptr(), n, 1, args.id_order_code, args.perm_seed, sm.stream), "ids")
    sm.sync()
    h_ev = torch.empty(n * 128, dtype=torch.uint8, pin_memory=True)
    h_ev.copy_(d_tmp)
    del d_tmp
    h_res = torch.zeros(n * 8, dtype=torch.uint8, pin_memory=True)
    n_win = n // (win * BATCH) + (1 if n % (win * BATCH) else 0)
    h_base = torch.zeros(n_win * (WINDOW_BATCHES_MAX + 1), dtype=torch.int32, pin_memory=True)
    torch.cuda.synchronize()
    ts = sm.prepare_timestamp
    nb_total = n // BATCH
    t0 = time.perf_counter()
    for wi, b0 in enumerate(range(0, nb_total, win)):
        nb = min(win, nb_total - b0)
        ns, tss = [], []
        for _ in range(nb):
            ts += 1 + BATCH
            ns.append(BATCH)
            tss.append(ts)
        sm.commit_window_host(Operation.create_transfers, h_ev.data_ptr() + b0 * BATCH * 128, ns, tss,
                              h_res.data_ptr() + b0 * BATCH * 8, h_base.data_ptr() + wi * (WINDOW_BATCHES_MAX + 1) * 4,
                              True, tss[0])
    sm.sync()
    wall = time.perf_counter() - t0
    sm.prepare_timestamp = ts
    bases = h_base.numpy().reshape(-1, WINDOW_BATCHES_MAX + 1)
    fails = 0
    for wi, b0 in enumerate(range(0, nb_total, win)):
        fails += int(bases[wi, min(win, nb_total - b0)])
    return {"value": round(n / wall, 1), "unit": "transfers/s", "transfers": n, "windows": n_win,
            "window_batches": win, "failed_events": fails, "wall_ms": round(wall * 1000, 3),
            "h2d_GBs": round(n * 128 / wall / 1e9, 2),
            "path": "pinned host prepare bodies -> tbg_commit_window_host (two device slots, copy stream "
                    "overlapping the previous window's kernels) -> replies D2H to pinned host memory"}


def sync_commit(args, sm, first, n_acc, seed):
    """The replica that does not pipeline: `k` further batches of the same stream, each through the
    synchronous StateMachine calls of the reference protocol (state_machine.zig:2719-2739: pulse()
    check, prefetch, commit), request bytes in a pinned message pool, replies copied back per batch
    (include/tbg.h tbg_prefetch / tbg_commit). Timed from the first call to the last reply."""
    from tigerbeetle_amd import workload
    from tigerbeetle_amd.types import Operation

    from tigerbeetle_amd.state_machine import HostBuffer

    k = args.sync_commit_batches
    evs = workload.transfers_uniform(first, k * BATCH, seed, n_acc)
    evs = workload.permute_ids(workload.mark_pending(evs, first, args.pending_every, PENDING_TIMEOUT),
                               args.id_order_code, args.perm_seed)
    # the replica's message pool: every prepare body lands in a buffer allocated once, pinned
    # (tbg_host_alloc), so the request reaches the device by one DMA
    pool = HostBuffer(k * BATCH * 128)
    raw = evs.view(np.uint8).reshape(-1)
    pool.array[:raw.size] = raw
    bodies = [pool.array[b * BATCH * 128:(b + 1) * BATCH * 128] for b in range(k)]
    fails = 0
    t0 = time.perf_counter()
    for b, body in enumerate(bodies):
        sm.prepare_timestamp += 1 + BATCH
        T = sm.prepare_timestamp
        if sm.pulse():
            sm.commit(0, 2 * b, T, Operation.pulse, b"")
        sm.prefetch_timestamp = T
        sm.prefetch(2 * b + 1, Operation.create_transfers, body)
        fails += len(sm.commit(0, 2 * b + 1, T, Operation.create_transfers, body)) // 8
    wall = time.perf_counter() - t0
    bodies = None
    pool.close()
    return {"value": round(k * BATCH / wall, 1), "unit": "transfers/s", "batches": k, "transfers": k * BATCH,
            "failed_events": fails, "us_per_batch": round(wall / k * 1e6, 1),
            "path": "per batch: pulse() check (host mirror of pulse_next), tbg_prefetch (one DMA of the 1 MiB "
                    "request from the pinned message pool), tbg_commit (device commit; Globals and reply read "
                    "back behind one sync) - the reference StateMachine call sequence"}


def cpu_baseline(args, seed):
    """Single-threaded C restatement (oracle/liboracle.so) on a time-bounded prefix of the same
    stream, same harness protocol (pulse when due, then the batch); only the commit calls are
    timed. Setup (accounts, cfg3 funding) is untimed, as on the GPU. The process is
    pinned to one host core for the measurement (restored after)."""
    host = host_cpu()  # (before pinning: the usable CPUs of the process)
    try:
        saved = os.sched_getaffinity(0)
        pinned = min(saved)
        os.sched_setaffinity(0, {pinned})
    except (AttributeError, OSError):
        saved, pinned = None, None
    try:
        line = _cpu_baseline(args, seed)
    finally:
        if saved is not None:
            os.sched_setaffinity(0, saved)
    line.update(host)
    line["pinned_cpu"] = pinned
    return line


def _cpu_baseline(args, seed):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_sm import lib as olib

    from tigerbeetle_amd.types import RESULT_DTYPE

    st = HostStream(args, seed)
    L = olib()
    h = L.tbo_create(BATCH)
    out = np.zeros(BATCH, RESULT_DTYPE)
    ts = 0

    def commit(create, ev, tick):
        nonlocal ts
        ts += tick + 1 + len(ev)
        t0 = time.perf_counter()
        if L.tbo_pulse_needed(h, ts):
            L.tbo_pulse(h, ts)
        create(h, ts, ev.ctypes.data, len(ev), out.ctypes.data)
        return time.perf_counter() - t0

    n_acc = st.n_accounts_total()
    for first in range(0, n_acc, BATCH):
        commit(L.tbo_create_accounts, st.accounts(first, min(BATCH, n_acc - first)), 0)
    if args.config == "cfg3":
        for first in range(0, args.accounts, BATCH):
            commit(L.tbo_create_transfers, st.funding(first, min(BATCH, args.accounts - first)), 0)
    spent, events, first = 0.0, 0, 0
    chunk = 32 * BATCH
    while spent < args.cpu_seconds and first < args.transfers:
        evs = st.transfers(first, min(chunk, args.transfers - first))
        for b in range(0, len(evs), BATCH):
            ev = evs[b:b + BATCH]
            spent += commit(L.tbo_create_transfers, ev, args.tick)
            events += len(ev)
        first += chunk
    L.tbo_destroy(h)
    line = {
        "value": events / spent,
        "unit": "transfers/s",
        "cores": 1,
        "kind": "port",
        "sample": f"first {events} transfers of the same {args.config} stream (same accounts and setup), "
                  f"{spent:.1f} s of commit time on 1 pinned host core (oracle/tb_oracle.c, -O2 -march=x86-64-v2)",
    }
    return line


# Algorithmic bytes per HOME event of the routed kernels (csrc/route.h) on one of G shards (DESIGN.md
# §5, §7): with uniform hashing each shard receives about as many messages as it has home events.
ROUTE_PHASES = {"prep": "route", "resolve": "own", "classify": "decide", "final": "apply"}
ROUTE_KERNELS = {"prep": ["k_rt_route1<true>", "k_rt_scan", "k_rt_route2<true>"], "resolve": ["k_rt_own<true>"],
                 "classify": ["k_rt_decide<true>"], "final": ["k_rt_apply<true>"]}


def route_kernel_bytes(phase, prefix):
    """Algorithmic bytes per home event of the routed kernels."""
    if phase == "prep":
        # the event read (128, twice: count and scatter passes), the stamped record written to its id
        # owner's block (128) and two 32 B side messages
        return 2 * 128 + 128 + 2 * 32
    if phase == "resolve":
        # id owner: the record read (128) and a 1 B reply (fresh rising ids probe nothing); account
        # owners: per side the 32 B message, one 32 B table entry, a 4 B slot and an 8 B reply
        return 128 + 1 + 2 * (32 + 32 + 4 + 8)
    if phase == "classify":
        # per home event: code, owners, positions, ledger (28 B of scratch), three replies (1 + 2 x 8),
        # three commit bytes, the code written back
        return 28 + 17 + 3 + 4
    # apply: per side its commit byte, slot 4, message 32, balance word read + write 2 x 16; per record
    # its commit byte, read 128 + write 128, id-table entry 32 unless the window extends the sorted prefix
    return 2 * (1 + 4 + 32 + 32) + 1 + 256 + (0 if prefix else 32) + 8


def run_sharded(args, torch, dist, world, rank, device):
    """cfg5 on N > 1 GPUs: one global stream, hash-sharded over the ranks with partitioned ingestion
    (tigerbeetle_amd/sharding.py, csrc/route.h): each rank generates and holds only its home batches of
    every window (1/N of the stream) and the three per-window all-to-alls carry the rest over RCCL."""
    from tigerbeetle_amd import _lib
    from tigerbeetle_amd.sharding import (ShardedStateMachine, alltoall_gloo, alltoall_nccl, exchange_gloo,
                                          exchange_nccl, route_bounds)
    from tigerbeetle_amd.state_machine import to_host
    from tigerbeetle_amd.types import Operation

    L = _lib.lib()
    G, me = world, rank
    n_acc = args.accounts * G
    n_xfer = args.transfers * G
    total_batches = (n_xfer + BATCH - 1) // BATCH
    # a routed window holds up to 128 batches per home: G x 128 by default (one home slice = 1M events)
    win = max(1, min(args.window if args.window_set else WINDOW_BATCHES_MAX * G, WINDOW_BATCHES_MAX * G))
    # The whole configured stream is committed (the state always reaches its full size); --warmup
    # batches are untimed and every later batch is timed (>= --steps of them).
    warm = min(((args.warmup + win - 1) // win) * win, max(0, total_batches - win))
    n_batches = total_batches
    acc_cap = int(n_acc / G * 1.02) + 65536
    x_cap = int(n_xfer / G * 1.02) + win * BATCH
    gloo = args.backend == "gloo"
    # (the all-reduce serves the general path: the harness pulses; the all-to-alls the routed windows)
    sm = ShardedStateMachine(G, me, exchange_gloo if gloo else exchange_nccl, device=device, batch_max=BATCH,
                             accounts_max=acc_cap, transfers_max=x_cap, window_events_max=WINDOW_BATCHES_MAX * BATCH)
    sm.alltoall = alltoall_gloo if gloo else alltoall_nccl
    stream = sm.sm.stream

    def home_slices(n_total):
        """This rank's home batches of every window: (window's first batch, batches, home bounds, event
        offset of the rank's slice in its home buffer, events)."""
        nb = (n_total + BATCH - 1) // BATCH
        out, off = [], 0
        for b0 in range(0, nb, win):
            b1 = min(b0 + win, nb)
            bounds = route_bounds(b1 - b0, G)
            e0 = min((b0 + bounds[me]) * BATCH, n_total)
            e1 = min((b0 + bounds[me + 1]) * BATCH, n_total)
            out.append((b0, b1, bounds, off, e0, e1 - e0))
            off += e1 - e0
        return out, off

    # This rank's home slices of the job's stream, resident in HBM before timing (1/N of it).
    acc_sl, n_acc_home = home_slices(n_acc)
    x_sl, n_x_home = home_slices(n_xfer)
    d_acc = torch.empty(max(n_acc_home, 1) * 128, dtype=torch.uint8, device="cuda")
    d_xfer = torch.empty(max(n_x_home, 1) * 128, dtype=torch.uint8, device="cuda")
    d_res = torch.empty(WINDOW_BATCHES_MAX * BATCH * 8, dtype=torch.uint8, device="cuda")
    n_windows_max = max(len(acc_sl), len(x_sl)) + 1
    d_base = torch.zeros(n_windows_max * (WINDOW_BATCHES_MAX + 1), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    for (_, _, _, off, e0, n) in acc_sl:
        if n:
            _lib.check(L.tbg_gen_accounts(d_acc.data_ptr() + off * 128, e0, n, args.seed, 2, 1, 0, stream), "gen")
            _lib.check(L.tbg_gen_permute_ids(d_acc.data_ptr() + off * 128, n, 0, args.id_order_code, args.perm_seed,
                                             stream), "ids")
    for (_, _, _, off, e0, n) in x_sl:
        if n:
            _lib.check(L.tbg_gen_transfers_uniform(d_xfer.data_ptr() + off * 128, e0, n, args.seed, n_acc, 0,
                                                   stream), "gen")
            _lib.check(L.tbg_gen_permute_ids(d_xfer.data_ptr() + off * 128, n, 1, args.id_order_code, args.perm_seed,
                                             stream), "ids")
    sm.stream.synchronize()

    prepare_ts = 0

    def commit_slice(op, d_home, sl, n_total, widx):
        nonlocal prepare_ts
        b0, b1, bounds, off, _, _ = sl
        ns, ts = [], []
        for b in range(b0, b1):
            n = min(BATCH, n_total - b * BATCH)
            prepare_ts += 1 + n
            ns.append(n)
            ts.append(prepare_ts)
        if sm.pulse(ts[0]):  # the harness pulse before the window (general path; then never due again)
            sm.commit_pulse(ts[0])
        _, count = sm.commit_window_routed(op, d_home.data_ptr() + off * 128, ns, ts, d_res.data_ptr(),
                                           d_base.data_ptr() + widx * (WINDOW_BATCHES_MAX + 1) * 4, bounds)
        return widx, count  # this rank's home batches: d_base[widx, count] = their failures

    def failures(wins):
        bases = to_host(d_base).reshape(-1, WINDOW_BATCHES_MAX + 1)
        return int(sum(bases[wi, nb] for wi, nb in wins))

    wins = [commit_slice(Operation.create_accounts, d_acc, sl, n_acc, i) for i, sl in enumerate(acc_sl)]
    sm.sync()
    acc_fail = failures(wins)
    d_base.zero_()

    NPH = len(PHASES)
    n_warm_w = warm // win
    L.tbg_timing_collect(sm.h, (ctypes.c_double * NPH)(), (ctypes.c_uint64 * NPH)(), NPH)  # reset
    L.tbg_timing_enable(sm.h, 0 if args.no_phase_timing else -1)  # warmup: every phase
    warm_windows = [commit_slice(Operation.create_transfers, d_xfer, x_sl[w], n_xfer, w) for w in range(n_warm_w)]
    sm.sync()
    per_phase, _ = warm_phases(sm, NPH)
    dom = max(ROUTE_PHASES, key=lambda k: per_phase[k] or 0.0)
    # timed region: only the roofline kernel's phase records events (two per window)
    L.tbg_timing_enable(sm.h, 0 if args.no_phase_timing else (1 << PHASES.index(dom)))
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    timed_windows = [commit_slice(Operation.create_transfers, d_xfer, x_sl[w], n_xfer, w)
                     for w in range(n_warm_w, len(x_sl))]
    sm.sync()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if dist:
        dist.barrier()
    L.tbg_timing_enable(sm.h, 0)
    ms = (ctypes.c_double * NPH)()
    launches = (ctypes.c_uint64 * NPH)()
    L.tbg_timing_collect(sm.h, ms, launches, NPH)

    timed_batches = n_batches - warm
    timed_events = n_xfer - warm * BATCH  # global: the ranks' home slices partition the stream
    timed_home = sum(x_sl[w][5] for w in range(n_warm_w, len(x_sl)))
    timed_fails = failures(timed_windows)
    fails = failures(warm_windows) + timed_fails
    elapsed = wall
    dev = "cpu" if args.backend == "gloo" else "cuda"
    if dist:
        # each rank replied for its home batches: failures are summed, the time is the max
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        f = torch.tensor([acc_fail, fails, timed_fails], dtype=torch.float64, device=dev)
        dist.all_reduce(f, op=dist.ReduceOp.SUM)
        acc_fail, fails, timed_fails = (int(x) for x in f.tolist())
    st = sm.stats()
    if args.verify:
        assert acc_fail == 0 and fails == 0, (acc_fail, fails)
    if rank == 0:
        roof = None
        di = PHASES.index(dom)
        if launches[di]:
            us = ms[di] / launches[di] * 1000.0
            ev_per_launch = timed_home / launches[di]
            prefix = st["sorted_transfers"] == st["transfers"]
            bytes_launch = int(route_kernel_bytes(dom, prefix) * ev_per_launch)
            achieved = bytes_launch / (us * 1e-6) / 1e9
            kname = ROUTE_KERNELS[dom][0]
            roof = {"bound": "hbm", "kernel": kname, "phase": ROUTE_PHASES[dom], "phase_kernels": ROUTE_KERNELS[dom],
                    "events_per_launch": int(ev_per_launch), "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                    "traffic_source": None, "avg_launch_us": round(us, 2), "alg_bytes_per_launch": bytes_launch,
                    "alg_bytes_basis": "per home event (bench.py route_kernel_bytes)",
                    "phase_avg_us_warmup": {ROUTE_PHASES[k]: (round(per_phase[k], 2) if per_phase[k] else None)
                                            for k in ROUTE_PHASES},
                    # per window and GPU, to the other GPUs: records + sides (A), replies (B), commit bytes (C)
                    "alltoall_bytes_per_event": round((G - 1) / G * (128 + 2 * 32 + 1 + 2 * 8 + 3), 1)}
        line = {
            "metric": "committed transfers/sec (create_transfers)",
            "value": round(timed_events / elapsed, 1),
            "unit": "transfers/s",
            "n_gpus": world,
            "steps": timed_batches,
            "steps_requested": args.steps,
            "warmup": warm,
            "ms_per_step": round(elapsed * 1000.0 / timed_batches, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u128",
            "data": "synthetic (device-generated, seed %d; each GPU generates and holds its home batches)" % args.seed,
            "config": {"workload": "cfg5: %d accounts hash-sharded over %d GPUs, %d uniform create_transfers "
                                   "(%.1f %% cross-shard), %d/batch" % (n_acc, G, n_xfer, 100.0 * (G - 1) / G, BATCH),
                       "batch": BATCH, "window_batches": win, "accounts_per_gpu": args.accounts,
                       "id_order": args.id_order, "pending_every": args.pending_every,
                       "transfers_per_gpu": args.transfers,
                       "parallelism": "hash-sharded accounts+ids, partitioned ingestion (home batch ranges), "
                                      "three RCCL all-to-alls per window (route / replies / commit)"},
            "results": {"failed_events_timed": int(timed_fails),
                        "ok_events_per_s": round((timed_events - timed_fails) / elapsed, 1),
                        "shard0_accounts": st["accounts"], "shard0_transfers": st["transfers"],
                        "backend": args.backend, "wall_ms_timed": round(wall * 1000, 3)},
            "roofline": roof,
        }
        print(json.dumps(line), flush=True)
    sm.close()
    if dist:
        dist.destroy_process_group()


def launch_ranks(args):
    """`--gpus N` (N > 1) without a launcher: start one rank per GPU the way the driver does (torchrun
    on 127.0.0.1) as a child process, before anything touches the GPU, and return its exit code."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if world_env is not None and int(world_env) != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%s (one rank per GPU)" % (args.gpus, world_env))
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "gloo":  # rehearsal: ranks may share a GPU
            torch.cuda.set_device(local_rank % torch.cuda.device_count())
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        torch.cuda.set_device(0)
    device = torch.cuda.current_device()
    if args.config == "cfg5" and world > 1:
        return run_sharded(args, torch, dist, world, rank, device)
    # (cfg5 on one GPU: one shard is the unsharded engine, its fused pass)

    from tigerbeetle_amd import StateMachine, _lib, workload
    from tigerbeetle_amd.state_machine import to_host
    from tigerbeetle_amd.types import Operation

    L = _lib.lib()
    cfg = args.config
    n_acc = args.accounts
    n_acc_total = n_acc + (CFG3_TREASURY if cfg == "cfg3" else 0)
    n_setup = n_acc if cfg == "cfg3" else 0
    total_batches = (args.transfers + BATCH - 1) // BATCH
    win = max(1, min(args.window, WINDOW_BATCHES_MAX))
    # The whole configured stream is committed (the state always reaches its full size); --warmup
    # batches are untimed and every later batch is timed (>= --steps of them).
    warm = min(((args.warmup + win - 1) // win) * win, max(0, total_batches - win))
    n_batches = total_batches
    n_xfer = args.transfers
    seed = args.seed + 1000 * rank  # independent stream per shard

    sm = StateMachine(device=device, batch_max=BATCH, accounts_max=n_acc_total,
                      transfers_max=n_xfer + n_setup + args.host_fed_transfers + args.sync_commit_batches * BATCH,
                      window_events_max=win * BATCH,
                      resolver={"chunks": True, "relax": "relax", "wait": "wait", "off": False}[args.resolver],
                      change_log=args.change_log)
    stream = sm.stream
    ext = torch.cuda.ExternalStream(stream)

    # Inputs resident in HBM before timing.
    d_acc = torch.empty(n_acc_total * 128, dtype=torch.uint8, device="cuda")
    d_xfer = torch.empty(n_xfer * 128, dtype=torch.uint8, device="cuda")
    d_setup = torch.empty(max(n_setup, 1) * 128, dtype=torch.uint8, device="cuda")
    d_res = torch.empty(max(n_xfer, n_acc_total, n_setup) * 8, dtype=torch.uint8, device="cuda")
    n_windows_max = (max(n_batches, (n_acc_total + BATCH - 1) // BATCH) + win - 1) // win + 1
    d_base = torch.zeros(n_windows_max * (WINDOW_BATCHES_MAX + 1), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    if cfg == "cfg3":
        d_cdf = torch.from_numpy(workload.zipf_cdf(n_acc).view(np.int64).copy()).cuda()
        torch.cuda.synchronize()
        _lib.check(L.tbg_gen_accounts_cfg3(d_acc.data_ptr(), 0, n_acc_total, seed, n_acc, CFG3_TOP, stream), "gen")
        _lib.check(L.tbg_gen_funding_cfg3(d_setup.data_ptr(), 0, n_setup, seed, n_acc, CFG3_TREASURY, CFG3_FUND,
                                          CFG3_FUND_ID, stream), "gen")
        _lib.check(L.tbg_gen_transfers_zipf(d_xfer.data_ptr(), 0, n_xfer, seed, n_acc, d_cdf.data_ptr(), 0, stream),
                   "gen")
    else:
        _lib.check(L.tbg_gen_accounts(d_acc.data_ptr(), 0, n_acc_total, seed, 2, 1, 0, stream), "gen accounts")
        if cfg == "cfg4":
            _lib.check(L.tbg_gen_transfers_cfg4(d_xfer.data_ptr(), 0, n_xfer, seed, n_acc, BATCH, 0, stream), "gen")
        else:
            _lib.check(L.tbg_gen_transfers_uniform(d_xfer.data_ptr(), 0, n_xfer, seed, n_acc, 0, stream), "gen")
            _lib.check(L.tbg_gen_mark_pending(d_xfer.data_ptr(), 0, n_xfer, args.pending_every, PENDING_TIMEOUT,
                                              stream), "pending")
    # --id-order: one bijection over every generated id (accounts, funding, transfers)
    for d, n, kind in ((d_acc, n_acc_total, 0), (d_setup, n_setup, 1), (d_xfer, n_xfer, 1)):
        _lib.check(L.tbg_gen_permute_ids(d.data_ptr(), n, kind, args.id_order_code, args.perm_seed, stream), "ids")

    prepare_ts = 0

    def commit_range(op, d_events, first_batch, last_batch, n_total, widx, tick):
        """Commits batches [first_batch, last_batch) as one window; harness timestamps (:2719-2739)."""
        nonlocal prepare_ts
        ns, ts = [], []
        for b in range(first_batch, last_batch):
            n = min(BATCH, n_total - b * BATCH)
            prepare_ts += tick + 1 + n
            ns.append(n)
            ts.append(prepare_ts)
        first_ev = first_batch * BATCH
        sm.commit_window(op, d_events.data_ptr() + first_ev * 128, ns, ts, d_res.data_ptr() + first_ev * 8,
                         d_base.data_ptr() + widx * (WINDOW_BATCHES_MAX + 1) * 4, True, ts[0])
        return widx, len(ns)

    def failures(wins):
        bases = to_host(d_base).reshape(-1, WINDOW_BATCHES_MAX + 1)
        return int(sum(bases[wi, nb] for wi, nb in wins))

    def commit_all(op, d_events, n_total):
        nb = (n_total + BATCH - 1) // BATCH
        wins = [commit_range(op, d_events, b0, min(b0 + win, nb), n_total, i, 0)
                for i, b0 in enumerate(range(0, nb, win))]
        _lib.check(L.tbg_sync(sm.h), "sync (setup)")
        f = failures(wins)
        d_base.zero_()
        return f

    acc_fail = commit_all(Operation.create_accounts, d_acc, n_acc_total)
    setup_fail = commit_all(Operation.create_transfers, d_setup, n_setup) if n_setup else 0

    widx = 0
    warm_windows = []
    NPH = len(PHASES)
    L.tbg_timing_collect(sm.h, (ctypes.c_double * NPH)(), (ctypes.c_uint64 * NPH)(), NPH)  # reset
    L.tbg_timing_enable(sm.h, 0 if args.no_phase_timing else -1)  # warmup: every phase
    for b0 in range(0, warm, win):
        warm_windows.append(commit_range(Operation.create_transfers, d_xfer, b0, min(b0 + win, warm), n_xfer, widx,
                                         args.tick))
        widx += 1
    _lib.check(L.tbg_sync(sm.h), "sync (warmup)")
    per_phase, dom = warm_phases(sm, NPH)
    stats_before = sm.stats()
    walker_before = stats_before["walker_events"]
    if dist:
        dist.barrier()
    # timed region: only the roofline kernel's phase records events (two per window)
    L.tbg_timing_enable(sm.h, 0 if args.no_phase_timing else (1 << PHASES.index(dom)))

    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    start.record(ext)
    timed_windows = []
    for b0 in range(warm, n_batches, win):
        timed_windows.append(commit_range(Operation.create_transfers, d_xfer, b0, min(b0 + win, n_batches), n_xfer,
                                          widx, args.tick))
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

    timed_batches = n_batches - warm
    timed_events = n_xfer - warm * BATCH
    elapsed = max(wall, gpu_ms / 1000.0)
    timed_fails = failures(timed_windows)
    fails = failures(warm_windows) + timed_fails
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        ev_t = torch.tensor([timed_events, timed_fails], dtype=torch.float64, device="cuda")
        dist.all_reduce(ev_t, op=dist.ReduceOp.SUM)
        all_events, all_fails = float(ev_t[0].item()), float(ev_t[1].item())
    else:
        all_events, all_fails = float(timed_events), float(timed_fails)

    stats = sm.stats()
    dbg = (ctypes.c_uint64 * 8)()
    L.tbg_debug_counters(sm.h, dbg, 8)
    if os.environ.get("TBG_DEBUG"):
        print("resolver counters", list(dbg), file=sys.stderr)
    if args.verify:
        assert acc_fail == 0 and setup_fail == 0, (acc_fail, setup_fail)
        if cfg in ("cfg1", "cfg2"):
            assert fails == 0, fails
            assert stats["transfers"] == n_xfer

    if rank == 0:
        roof = None
        di = PHASES.index(dom)
        if launches[di]:
            us = ms[di] / launches[di] * 1000.0
            ev_per_launch = timed_events / launches[di]
            prefix = stats["sorted_transfers"] == stats["transfers"]  # every window extended the prefix
            if dom in ("cpw", "walk"):
                key = "component_events" if dom == "cpw" else "walker_events"
                walked = stats[key] - stats_before[key]
                per_event = WALKED_EVENT_BYTES * walked / max(timed_events, 1)
            else:
                per_event = PHASE_ALG_BYTES.get(dom)
            kname = PHASE_KERNELS[dom][0]
            roof = {"bound": "hbm", "kernel": kname, "phase": dom, "phase_kernels": PHASE_KERNELS[dom],
                    "events_per_launch": int(ev_per_launch), "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": None, "traffic": None, "avg_launch_us": round(us, 2), "alg_bytes_per_event": per_event,
                    "alg_bytes_basis": "SURVEY 8(d) 640 B/event path split over the phases (bench.py PHASE_ALG_BYTES); "
                                       "no scratch columns", "sorted_prefix": prefix,
                    "phase_avg_us_warmup": {k: (round(v, 2) if v else None) for k, v in per_phase.items()},
                    "path_alg_GBs": round(640 * all_events / elapsed / 1e9 / max(world, 1), 1),
                    "path_frac": round(640 * all_events / elapsed / 1e9 / max(world, 1) / HBM_PEAK_GBS, 4)}
            if per_event:
                bytes_launch = int(per_event * ev_per_launch)
                achieved = bytes_launch / (us * 1e-6) / 1e9
                tr = pmc_traffic(pmc_tag(args), kname, ev_per_launch)
                roof.update({"achieved": round(achieved, 1), "frac": round(achieved / HBM_PEAK_GBS, 4),
                             "alg_bytes_per_launch": bytes_launch, "traffic": tr[0] if tr else None,
                             "traffic_fetch_x2": tr[1] if tr else None, "traffic_source": tr[2] if tr else None})
        desc = {
            "cfg1": "cfg1: %d accounts, %d uniform create_transfers, %d/batch",
            "cfg2": "cfg2: %d accounts, %d uniform create_transfers (no flags), %d/batch" if not args.pending_every
            else "cfg2 mixed: %%d accounts, %%d uniform create_transfers, every %d-th pending (timeout %d s), %%d/batch"
            % (args.pending_every, PENDING_TIMEOUT),
            "cfg3": "cfg3: %d accounts (Zipf 1.2, debits<=credits limits, pre-funded), %d transfers, %d/batch",
            "cfg4": "cfg4: %d accounts, %d two-phase/linked transfers, +1 s per batch, %d/batch",
            "cfg5": "cfg5 on one GPU (one shard = the unsharded engine): %d accounts, %d uniform create_transfers, "
                    "%d/batch",
        }[cfg] % (n_acc, n_xfer, BATCH)
        line = {
            "metric": "committed transfers/sec (create_transfers)",
            "value": round(all_events / elapsed, 1),
            "unit": "transfers/s",
            "n_gpus": world,
            "steps": timed_batches,
            "steps_requested": args.steps,
            "warmup": warm,
            "ms_per_step": round(elapsed * 1000.0 / timed_batches, 4),
            "higher_is_better": True,
            "scaling": "weak" if world == 1 else "replicas",
            "vs_baseline": None,
            "dtype": "u128",
            "data": "synthetic (device-generated, seed %d)" % args.seed,
            "config": {"workload": desc, "batch": BATCH, "window_batches": win, "accounts_per_gpu": n_acc,
                       "id_order": args.id_order, "pending_every": args.pending_every,
                       "transfers_per_gpu": n_xfer, "resolver": args.resolver, "change_log": bool(args.change_log),
                       "parallelism": "independent databases, one per rank (not sharded)" if world > 1 else "single GPU"},
            "results": {"failed_events_timed": int(all_fails),
                        "ok_events_per_s": round((all_events - all_fails) / elapsed, 1),
                        "walker_events_timed": stats["walker_events"] - walker_before,
                        "gpu_ms_timed": round(gpu_ms, 3), "wall_ms_timed": round(wall * 1000, 3)},
            "roofline": roof,
        }
        if os.environ.get("TBG_BENCH_DBG"):  # the engine's instrumentation counters (tbg_debug_counters)
            dbg = (ctypes.c_uint64 * 8)()
            L.tbg_debug_counters(sm.h, dbg, 8)
            line["results"]["debug_counters"] = list(dbg)
        if args.host_fed_transfers and cfg in ("cfg1", "cfg2") and world == 1:
            sm.prepare_timestamp = prepare_ts
            line["host_fed"] = host_fed(args, sm, torch, n_xfer, n_acc, seed, win)
            prepare_ts = sm.prepare_timestamp
        if args.sync_commit_batches and cfg in ("cfg1", "cfg2") and world == 1:
            sm.prepare_timestamp = prepare_ts
            line["sync_commit"] = sync_commit(args, sm, n_xfer + args.host_fed_transfers // BATCH * BATCH, n_acc,
                                              seed)
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args, seed)
        print(json.dumps(line), flush=True)
    sm.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
