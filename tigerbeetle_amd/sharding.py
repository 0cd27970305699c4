"""Hash-sharded commit over the GPUs of one node: one engine per GPU, one process per GPU.

Account a lives on shard `shard_of(a.id)`, transfer t on shard `shard_of(t.id)` (csrc/shard.h).
Every shard receives the same prepared window (the replica hands each GPU the same prepare body,
state_machine.zig:1107-1146) and is the home of a contiguous range of its batches (`home_range`).
A window commits in three steps through the C ABI (include/tbg.h):

  tbg_shard_prepare_window   one pass over the window: the owners validate and resolve what they own
                             (accounts, ids) and write the owner facts (2 B per transfer: the id
                             owner's code, the account sides' states; one writer per bit)
  exchange                   byte-wise sum of the facts across the shards, on the engine's stream
                             (RCCL uint8 all-reduce over xGMI: torch "nccl")
  tbg_shard_commit_window    every shard decides every event from the facts (the same outcome
                             everywhere: no second exchange), writes its home batches' replies and
                             applies the owned effects of the committed events

The `exchange` callable is the only collective on the data path; with one shard there is none.
Per shard, the work is the window's ids plus 1/G of the rest: it falls as G grows.

pulse() (state_machine.zig:589-596) starts true on every shard (pulse_next_timestamp =
timestamp_min, :2063), as on one engine. A pulse needs every shard's due expiry entries, so it runs
through the general path (`pulse_general`): the due entries and their accounts are gathered, every
shard expires the same ones, in the reference's (expires_at, timestamp) order and cap. A window goes
through the five steps above only when no pulse is due at any of its batches (checked on the device:
tbg_sync reports TBG_E_STATE otherwise).
"""
import ctypes

import numpy as np

from . import _lib
from .state_machine import StateMachine
from .types import Operation

WINDOW_BATCHES_MAX = 128  # csrc/window.h MAXB

_M1, _M2 = np.uint64(0xFF51AFD7ED558CCD), np.uint64(0xC4CEB9FE1A85EC53)


def _mix64(x):
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint64(33))
        x = x * _M1
        x = x ^ (x >> np.uint64(33))
        x = x * _M2
        return x ^ (x >> np.uint64(33))


def shard_of(id_lo, id_hi, shard_count):
    """Numpy twin of shard_of() in csrc/shard.h (high half of the table hash, scaled to G)."""
    lo = np.asarray(id_lo, np.uint64)
    hi = np.asarray(id_hi, np.uint64)
    with np.errstate(over="ignore"):
        h = _mix64(lo ^ _mix64(hi + np.uint64(0x9E3779B97F4A7C15)))
        return (((h >> np.uint64(32)) * np.uint64(shard_count)) >> np.uint64(32)).astype(np.uint32)


def exchange_nccl(t):
    """In-place sum across the process group on the current (engine) stream: RCCL on ROCm."""
    import torch.distributed as dist

    dist.all_reduce(t)


def exchange_gloo(t):
    """Same reduction through host memory (gloo): for ranks that share one GPU in tests. Copies go
    through pinned memory on the current (engine) stream and are waited for explicitly."""
    import torch
    import torch.distributed as dist

    c = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    c.copy_(t, non_blocking=True)
    torch.cuda.current_stream().synchronize()
    dist.all_reduce(c)
    t.copy_(c, non_blocking=True)
    torch.cuda.current_stream().synchronize()


def alltoall_nccl(send, send_sizes, recv, recv_sizes):
    """Uneven all-to-all of byte blocks across the process group on the current (engine) stream:
    grouped ncclSend / ncclRecv under RCCL (torch "nccl" on ROCm)."""
    import torch.distributed as dist

    dist.all_to_all_single(recv, send, list(recv_sizes), list(send_sizes))


def alltoall_gloo(send, send_sizes, recv, recv_sizes):
    """The same through host memory (gloo): for ranks that share one GPU in tests."""
    import torch
    import torch.distributed as dist

    s = torch.empty(send.shape, dtype=send.dtype, pin_memory=True)
    s.copy_(send, non_blocking=True)
    torch.cuda.current_stream().synchronize()
    r = torch.empty(recv.shape, dtype=recv.dtype)
    dist.all_to_all_single(r, s, list(recv_sizes), list(send_sizes))
    recv.copy_(r, non_blocking=True)
    torch.cuda.current_stream().synchronize()


def route_bounds(n_batches, shard_count):
    """Home batch bounds of a routed window: shard r is home for [bounds[r], bounds[r + 1])."""
    return [n_batches * r // shard_count for r in range(shard_count + 1)]


class _timed:
    """(rehearsal) wall time of a general-window step on this shard, synced, when gw_times is set:
    slots 0-1 phase 1 (collect, write), 2-3 phase 2, 4 commit (scratch engine + apply)."""

    def __init__(self, shard, slot):
        self.shard, self.slot = shard, slot

    def __enter__(self):
        import time

        if getattr(self.shard, "gw_times", None) is not None:
            import torch

            torch.cuda.synchronize(self.shard.device)
            self.t0 = time.perf_counter()

    def __exit__(self, *exc):
        import time

        t = getattr(self.shard, "gw_times", None)
        if t is not None and not exc[0]:
            self.shard.stream.synchronize()
            t[self.slot] = t.get(self.slot, 0.0) + time.perf_counter() - self.t0
        return False


def home_range(n_batches, shard_count, shard_index):
    """Home batches [first, first + count) of `shard_index`: contiguous, as even as possible."""
    lo = n_batches * shard_index // shard_count
    hi = n_batches * (shard_index + 1) // shard_count
    return lo, hi - lo


class ShardedStateMachine:
    """One shard of a hash-sharded engine. `exchange(t)` must sum the uint8 tensor `t` in place
    across all shards (None for a single shard)."""

    def __init__(self, shard_count, shard_index, exchange=None, device=0, batch_max=8190, accounts_max=1 << 16,
                 transfers_max=1 << 20, window_events_max=0, change_log=False):
        import torch

        self.sm = StateMachine(device=device, batch_max=batch_max, accounts_max=accounts_max,
                               transfers_max=transfers_max, window_events_max=window_events_max,
                               shard_count=shard_count, shard_index=shard_index, change_log=change_log)
        self.shard_count, self.shard_index = shard_count, shard_index
        self.batch_max, self.device = batch_max, device
        self.scratch = None
        self.exchange = exchange
        events_max = window_events_max or batch_max
        dev = torch.device("cuda", device)
        L = _lib.lib()
        xb = max(L.tbg_shard_exchange_bytes(int(op), events_max, shard_count)
                 for op in (Operation.create_accounts, Operation.create_transfers))
        self.xch = torch.zeros(int(xb), dtype=torch.uint8, device=dev)
        self.stream = torch.cuda.ExternalStream(self.sm.stream, device=dev)
        self._n_events = 0
        self._pulse_next = None  # cached pulse_next_timestamp (order-free windows never change it)
        # general windows: due entries each shard can offer (more sends the window batch by batch)
        self.due_cap = max(4 * batch_max, min(events_max, 1 << 16))
        self.gw_events = 0
        self.wscratch = None
        self.gw_times = None  # (rehearsal: tools/rehearse_shards.py) per-step wall times of general windows
        self.gw_fallbacks = {"due_overflow": 0, "rejected": 0}  # general windows sent batch by batch
        self.gw_acc_base = None  # accounts the general windows' scratch engine holds (None: starts over)
        self.rt = None           # routed windows: the six exchange buffers (attached at the first one)
        self.alltoall = None     # routed windows: this process's all-to-all (alltoall_nccl / alltoall_gloo)
        torch.cuda.synchronize(device)

    @property
    def h(self):
        return self.sm.h

    def close(self):
        if self.scratch is not None:
            self.scratch.close()
        if self.wscratch is not None:
            self.wscratch.close()
        self.sm.close()

    def home_range(self, n_batches):
        return home_range(n_batches, self.shard_count, self.shard_index)

    # --------------------------------------------------------------------------------------------
    # Routed windows (csrc/route.h): partitioned ingestion. This shard holds only its home batches'
    # events; three all-to-alls carry the messages to the owners, their replies to the homes and the
    # commit bytes back to the owners.
    # --------------------------------------------------------------------------------------------
    def _route_init(self):
        import torch

        if getattr(self, "rt", None) is not None:
            return
        L = _lib.lib()
        b = (ctypes.c_uint64 * 6)()
        _lib.check(L.tbg_route_buffer_bytes(self.sm.h, b), "route_buffer_bytes")
        dev = torch.device("cuda", self.device)
        self.rt = [torch.empty(max(int(x), 16), dtype=torch.uint8, device=dev) for x in b]
        torch.cuda.synchronize(self.device)
        ptrs = (ctypes.c_void_p * 6)(*[t.data_ptr() for t in self.rt])
        _lib.check(L.tbg_route_attach(self.sm.h, ptrs), "route_attach")

    def route_prepare(self, operation, d_home_events, batch_events, batch_timestamps, bounds=None):
        """Step 1 of a routed window: this shard's home events (batches [bounds[me], bounds[me + 1]),
        contiguous at d_home_events) routed into message blocks. Returns (home_first, home_count)."""
        self._route_init()
        self.invalidate_scratch()
        nb = len(batch_events)
        bounds = bounds or route_bounds(nb, self.shard_count)
        ev = (ctypes.c_uint32 * nb)(*batch_events)
        ts = (ctypes.c_uint64 * nb)(*batch_timestamps)
        hb = (ctypes.c_uint32 * (self.shard_count + 1))(*bounds)
        _lib.check(_lib.lib().tbg_route_prepare(self.sm.h, int(operation), d_home_events, nb, ev, ts, hb),
                   "route_prepare")
        r = self.shard_index
        return bounds[r], bounds[r + 1] - bounds[r]

    def route_views(self, phase):
        """The exchange of phase 0 / 1 / 2 (A / B / C): (send, send_sizes, recv, recv_sizes), uint8
        views of the attached buffers: the splits of an uneven all-to-all."""
        G = self.shard_count
        sp, rp = ctypes.c_void_p(), ctypes.c_void_p()
        ss, rs = (ctypes.c_uint64 * G)(), (ctypes.c_uint64 * G)()
        _lib.check(_lib.lib().tbg_route_buffers(self.sm.h, phase, ctypes.byref(sp), ss, ctypes.byref(rp), rs),
                   "route_buffers")
        send_t = self.rt[2 * phase]
        recv_t = self.rt[2 * phase + 1]
        assert sp.value == send_t.data_ptr() and rp.value == recv_t.data_ptr()
        ss, rs = [int(x) for x in ss], [int(x) for x in rs]
        return send_t[: sum(ss)], ss, recv_t[: sum(rs)], rs

    def route_step(self, step):
        """Steps 2-4 between the exchanges: "own", "decide"."""
        fn = {"own": _lib.lib().tbg_route_own, "decide": _lib.lib().tbg_route_decide}[step]
        _lib.check(fn(self.sm.h), "route_" + step)

    def route_apply(self, d_results, d_batch_base):
        _lib.check(_lib.lib().tbg_route_apply(self.sm.h, d_results, d_batch_base), "route_apply")

    def commit_window_routed(self, operation, d_home_events, batch_events, batch_timestamps, d_results,
                             d_batch_base, bounds=None):
        """A routed window with this process's all-to-all (`alltoall(send, send_sizes, recv, recv_sizes)`),
        asynchronous on the engine stream. Replies of the home batches land in d_results / d_batch_base;
        returns (home_first, home_count). The harness pulse before the first batch must have run (no
        pulse may fall due inside the window: the window is rejected otherwise)."""
        import torch

        first, count = self.route_prepare(operation, d_home_events, batch_events, batch_timestamps, bounds)
        for phase, step in ((0, "own"), (1, "decide"), (2, None)):
            if self.alltoall is not None:
                with torch.cuda.stream(self.stream):
                    self.alltoall(*self.route_views(phase))
            else:  # (one shard: its only block is its own)
                send, ss, recv, rs = self.route_views(phase)
                with torch.cuda.stream(self.stream):
                    recv.copy_(send)
            if step:
                self.route_step(step)
        self.route_apply(d_results, d_batch_base)
        return first, count

    def prepare_window(self, operation, d_events, batch_events, batch_timestamps):
        """Step 1; returns the facts tensor to be summed across the shards."""
        self.invalidate_scratch()
        nb = len(batch_events)
        ev = (ctypes.c_uint32 * nb)(*batch_events)
        ts = (ctypes.c_uint64 * nb)(*batch_timestamps)
        _lib.check(_lib.lib().tbg_shard_prepare_window(self.sm.h, int(operation), d_events, nb, ev, ts,
                                                       self.xch.data_ptr()), "shard_prepare_window")
        self._n_events = sum(batch_events)
        n = _lib.lib().tbg_shard_exchange_bytes(int(operation), self._n_events, self.shard_count)
        return self.xch[:n]

    def commit_prepared(self, home_first, home_count, d_results, d_batch_base):
        """Step 3 (after the facts were summed): decide, reply for the home batches, apply."""
        _lib.check(_lib.lib().tbg_shard_commit_window(self.sm.h, self.xch.data_ptr(), home_first, home_count,
                                                      d_results, d_batch_base), "shard_commit_window")

    def commit_window(self, operation, d_events, batch_events, batch_timestamps, d_results, d_batch_base):
        """Asynchronous on the engine stream (after the harness pulse before the first batch, when
        one is due: the general path, synchronous). Replies of this shard's home batches
        (home_range) land in d_results / d_batch_base (d_batch_base[0..home_count]); returns
        (home_first, home_count). No pulse may fall due at a later batch of the window."""
        import torch

        if batch_timestamps and self.pulse(batch_timestamps[0]):
            self.commit_pulse(batch_timestamps[0])  # the harness pulse before the first batch
        first, count = self.home_range(len(batch_events))
        words = self.prepare_window(operation, d_events, batch_events, batch_timestamps)
        if self.exchange is not None:
            with torch.cuda.stream(self.stream):
                self.exchange(words)
        self.commit_prepared(first, count, d_results, d_batch_base)
        return first, count

    def sync(self):
        self.sm.sync()

    def stats(self):
        return self.sm.stats()

    # --------------------------------------------------------------------------------------------
    # General class (csrc/shard_gx.inc): one batch at a time, decided on every shard from the
    # gathered read set by a scratch unsharded engine.
    # --------------------------------------------------------------------------------------------
    # --------------------------------------------------------------------------------------------
    # The rest of the StateMachine surface on a shard (csrc/shard_read.inc, tbg_open, the write-back
    # stream): every shard gets the same call; reads gather from the owners through the exchange.
    # --------------------------------------------------------------------------------------------
    def open(self, accounts, transfers, pending_status, account_balances=None):
        """StateMachine.open (state_machine.zig:527-541): the same whole set of forest objects on every
        shard; each keeps what it owns."""
        self.sm.open(accounts, transfers, pending_status, account_balances)
        self._pulse_next = None
        self.invalidate_scratch()

    def read_request(self, operation, data):
        """Step 1 of a lookup or query: this shard's part of the read buffer (to be summed)."""
        import torch

        L = _lib.lib()
        op = int(operation)
        dev = torch.device("cuda", self.device)
        with torch.cuda.stream(self.stream):  # the zero fill before the engine kernels that write into it
            return self._read_request(L, op, dev, data)

    def _read_request(self, L, op, dev, data):
        import torch

        if op in (int(Operation.lookup_accounts), int(Operation.lookup_transfers)):
            buf = torch.zeros(max(int(L.tbg_shard_lookup_bytes(len(data) // 16)), 1), dtype=torch.uint8, device=dev)
            raw = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
            _lib.check(L.tbg_shard_lookup(self.sm.h, op, raw.ctypes.data, len(data), buf.data_ptr()), "shard_lookup")
        else:
            buf = torch.zeros(int(L.tbg_shard_query_bytes(self.shard_count, self.batch_max)), dtype=torch.uint8,
                              device=dev)
            raw = np.frombuffer(data, np.uint8)
            _lib.check(L.tbg_shard_query(self.sm.h, op, raw.ctypes.data, len(data), buf.data_ptr()), "shard_query")
        self.stream.synchronize()
        return buf

    def read_reply(self, operation, data, buf):
        """Step 2 (after the buffers were summed): the reply bytes."""
        L = _lib.lib()
        op = int(operation)
        out = self.sm._out
        n = ctypes.c_uint64()
        if op in (int(Operation.lookup_accounts), int(Operation.lookup_transfers)):
            _lib.check(L.tbg_shard_lookup_reply(self.sm.h, buf.data_ptr(), len(data), out.ctypes.data, len(out),
                                                ctypes.byref(n)), "shard_lookup_reply")
        else:
            raw = np.frombuffer(data, np.uint8)
            _lib.check(L.tbg_shard_query_merge(self.sm.h, op, raw.ctypes.data, buf.data_ptr(), out.ctypes.data,
                                               len(out), ctypes.byref(n)), "shard_query_merge")
        return out[: n.value].tobytes()

    def read(self, operation, data):
        """lookup_* / get_account_* with this process's exchange: the reply bytes."""
        buf = self.read_request(operation, data)
        self._sum([buf])
        return self.read_reply(operation, data, buf)

    def window_changes(self):
        """The write-back stream of this shard's last commit (its own objects)."""
        return self.sm.window_changes()

    def pulse_next(self):
        """pulse_next_timestamp, the same on every shard. Cached: an order-free window holds no
        pending transfer and no timeout, so only the general path and pulses change it."""
        if self._pulse_next is None:
            self._pulse_next = self.sm.stats()["pulse_next_timestamp"]
        return self._pulse_next

    def pulse(self, prepare_timestamp):
        """StateMachine.pulse() (state_machine.zig:589-596): pulse_next_timestamp <= prepare_timestamp."""
        return self.pulse_next() <= prepare_timestamp

    def _sum(self, tensors):
        """This process's exchange over `tensors`, ordered on the engine stream: the tensors were
        written by engine kernels still in flight (no sync after the gathers), and exchange_nccl /
        exchange_gloo run on the current stream."""
        import torch

        if self.exchange is None:
            return
        with torch.cuda.stream(self.stream):
            for t in tensors:
                self.exchange(t)

    def commit_pulse(self, timestamp):
        """commit(.pulse) at `timestamp` with this process's exchange (the replica logs one when
        pulse() is true, vsr/replica.zig:9459-9487; the harness runs one before a batch at the
        batch's timestamp, :2719-2739)."""
        pulse_general([self], self._sum, timestamp)

    # --------------------------------------------------------------------------------------------
    # General class, a whole window at a time (csrc/shard_gw.inc): each shard lists what it owns of
    # the window's read set (compact: each object once), the lists are concatenated across the shards
    # by two rounds of (count exchange, record exchange), every shard's scratch engine commits the
    # window (the pulses inside it modelled, xwin.h), and each shard applies its own part by position.
    # --------------------------------------------------------------------------------------------
    def _gw_init(self, n_events):
        import torch

        if getattr(self, "gw_events", 0) >= max(n_events, 1):
            return
        dev = torch.device("cuda", self.device)
        need_e = max(n_events, 1)
        self.gw_cnt = torch.zeros(16 * self.shard_count, dtype=torch.uint8, device=dev)
        self.gw_res = torch.zeros(need_e * 8, dtype=torch.uint8, device=dev)
        self.gw_base = torch.zeros(WINDOW_BATCHES_MAX + 1, dtype=torch.int32, device=dev)
        self.gw_events = need_e
        torch.cuda.synchronize(self.device)

    def _gw_scratch(self, acc_need, x_need, n_events):
        """The scratch engine (kept across windows) and the exchange buffers, grown when a window needs
        more: its account store is bound to gw_acc during a commit, gathered transfers go through gw_x."""
        import torch

        sc = self.wscratch
        if sc is not None and self.gw_acc_cap >= acc_need and self.gw_x_cap >= x_need and self.gw_sc_events >= n_events:
            return
        # (accounts doubling: a stream whose read set grows window by window re-creates the scratch
        # engine, and restarts it with a full reload, a logarithmic number of times)
        acc_cap = max(2 * acc_need + 1024, 2 * getattr(self, "gw_acc_cap", 0) if sc is not None else 0)
        x_cap = max(int(x_need * 1.25) + 1024, getattr(self, "gw_x_cap", 0))  # (its table is reset per window)
        ev_cap = max(n_events, getattr(self, "gw_sc_events", 0))
        if sc is not None:
            sc.close()
        self.gw_acc_base = 0  # (a new scratch holds nothing: only sized when the window starts over)
        self.wscratch = StateMachine(device=self.device, batch_max=self.batch_max, accounts_max=acc_cap,
                                     transfers_max=x_cap, window_events_max=ev_cap)
        dev = torch.device("cuda", self.device)
        self.gw_acc = torch.empty(acc_cap * 128, dtype=torch.uint8, device=dev)
        self.gw_x = torch.empty(x_cap * 128, dtype=torch.uint8, device=dev)
        self.gw_xst = torch.empty(x_cap, dtype=torch.uint8, device=dev)
        self.gw_acc_cap, self.gw_x_cap, self.gw_sc_events = acc_cap, x_cap, ev_cap
        torch.cuda.synchronize(self.device)

    def invalidate_scratch(self):
        """Something other than a general window changed this shard's state: the scratch engine starts
        over at the next general window (every shard makes the same calls, so every one does)."""
        self.gw_acc_base = None

    def gw_collect(self, operation, d_events, n_events, t_last, phase, restart=False):
        """Phase 1 or 2 of a general window: this shard's list of what it owns of the read set (phase 1
        without the accounts the scratch engine holds from the previous general windows, unless it
        starts over); returns the count buffer to be summed across the shards (asynchronous)."""
        self._gw_init(n_events)
        if phase == 1:
            restart = restart or self.gw_acc_base is None or self.wscratch is None
            if restart:
                self.gw_acc_base = 0
        xg, nx = (self.gw_x.data_ptr(), self._gw_n[1]) if phase == 2 else (None, 0)
        with _timed(self, 0 if phase == 1 else 2):
            _lib.check(_lib.lib().tbg_gw_collect(self.sm.h, int(operation), d_events, n_events, t_last, phase,
                                                 self.due_cap, xg, nx, self.gw_cnt.data_ptr(), int(restart)),
                       "gw_collect")
        return self.gw_cnt

    def gw_plan(self, operation, n_events):
        """After phase 1's counts were summed: "ok", "restart" (the scratch engine would outgrow its
        capacity with the accounts it holds: collect again from scratch) or "overflow" (a shard had more
        entries due than the window path holds: the window goes batch by batch). Sizes the scratch engine
        for the window's read set (phase 2 adds at most two accounts per gathered transfer)."""
        from .state_machine import to_host

        with _timed(self, 1):
            c = self.sm.read_device(self.gw_cnt).view(np.uint32).reshape(self.shard_count, 4)
        if (c[:, 3] > self.due_cap).any():
            self.gw_fallbacks["due_overflow"] += 1
            self.invalidate_scratch()
            return "overflow"
        a1, x1 = int(c[:, 0].sum()), int(c[:, 1].sum())
        xfer = int(operation) == int(Operation.create_transfers)
        acc_need = self.gw_acc_base + a1 + 2 * x1 + (0 if xfer else n_events)
        x_need = x1 + (n_events if xfer else 0)
        if self.gw_acc_base and (acc_need > self.gw_acc_cap or x_need > self.gw_x_cap or n_events > self.gw_sc_events):
            self.invalidate_scratch()
            return "restart"
        self._gw_scratch(acc_need, x_need, n_events)
        return "ok"

    def gw_write(self, phase):
        """After the phase's counts were summed: this shard's records at its offset of the exchange
        regions; returns the regions to be summed across the shards."""
        L = _lib.lib()
        na, nx, ovf = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_int()
        b = self.gw_acc_base  # (the gathered accounts go after the ones the scratch holds)
        with _timed(self, 1 if phase == 1 else 3):
            _lib.check(L.tbg_gw_write(self.sm.h, phase, self.gw_cnt.data_ptr(), self.gw_acc.data_ptr() + b * 128,
                                      self.gw_acc_cap - b, self.gw_x.data_ptr(), self.gw_xst.data_ptr(), self.gw_x_cap,
                                      ctypes.byref(na), ctypes.byref(nx), ctypes.byref(ovf)), "gw_write")
        assert not ovf.value  # (gw_plan checked the due counts)
        if phase == 1:
            self._gw_n = [na.value, nx.value]
            return [self.gw_acc[b * 128: (b + na.value) * 128], self.gw_x[: nx.value * 128], self.gw_xst[: nx.value]]
        a1 = b + self._gw_n[0]
        return [self.gw_acc[a1 * 128: (a1 + na.value) * 128]]

    def gw_commit(self, operation, d_events, batch_events, batch_timestamps, auto_pulse):
        """After both phases were summed: the window on the scratch engine, then this shard's part.
        Returns the per-batch replies, or None when the scratch engine rejected the window (nothing
        applied: a pulse inside it reaching the expiry cap, or one falling due in a window that reads
        balances); the caller then commits it batch by batch."""
        from .state_machine import to_host

        L = _lib.lib()
        nb = len(batch_events)
        ev = (ctypes.c_uint32 * nb)(*batch_events)
        ts = (ctypes.c_uint64 * nb)(*batch_timestamps)
        rej, held = ctypes.c_int(), ctypes.c_uint64()
        with _timed(self, 4):
            _lib.check(L.tbg_gw_commit(self.sm.h, self.wscratch.h, int(operation), d_events, nb, ev, ts,
                                       self.gw_acc.data_ptr(), self.gw_acc_base, self.gw_x.data_ptr(),
                                       self.gw_xst.data_ptr(), self.gw_res.data_ptr(), self.gw_base.data_ptr(),
                                       int(bool(auto_pulse)), batch_timestamps[0]), "gw_commit")
            _lib.check(L.tbg_gw_result(self.sm.h, self.wscratch.h, ctypes.byref(rej), ctypes.byref(held)),
                       "gw_result")
        self._pulse_next = None
        if rej.value:
            self.gw_fallbacks["rejected"] += 1
            self.invalidate_scratch()  # (its first pulse may have run in the scratch: it starts over)
            return None
        self.gw_acc_base = held.value
        base = self.sm.read_device(self.gw_base)
        res = self.sm.read_device(self.gw_res[: int(base[nb]) * 8]).tobytes()
        return [res[base[b] * 8: base[b + 1] * 8] for b in range(nb)]

    def commit_general_window(self, operation, d_events, batch_events, batch_timestamps, auto_pulse=True):
        """A window of the general class with this process's exchange; every shard returns the
        window's whole per-batch reply. Falls back to batch by batch when the window path cannot
        hold it."""
        return commit_general_window([self], self._sum, operation, d_events, batch_events, batch_timestamps,
                                     auto_pulse)

    def _gx_init(self):
        import torch

        if getattr(self, "scratch", None) is not None:
            return
        bm, G = self.batch_max, self.shard_count
        C = bm + 1
        dev = torch.device("cuda", self.device)
        self.gx = torch.zeros(_gx_layout(bm, G, C)["bytes"], dtype=torch.uint8, device=dev)
        self.scratch = StateMachine(device=self.device, batch_max=bm, accounts_max=4 * bm + 2 * G * C + 64,
                                    transfers_max=3 * bm + G * C + G + 64, window_events_max=bm)
        self.gx_res = torch.zeros(max(bm, 1) * 8, dtype=torch.uint8, device=dev)
        self.gx_base = torch.zeros(2, dtype=torch.int32, device=dev)
        torch.cuda.synchronize(self.device)  # (the fills ran on the current stream; the engine's next)

    def gather(self, operation, d_events, n, timestamp, phase):
        """Gather phase 1 or 2 of one batch; returns the region to be summed across the shards."""
        import torch

        self._gx_init()
        lay = _gx_layout(n, self.shard_count, self.batch_max + 1)
        _lib.check(_lib.lib().tbg_shard_gather(self.sm.h, int(operation), d_events, n, timestamp, phase,
                                               self.gx.data_ptr()), "shard_gather")
        torch.cuda.synchronize(self.device)
        return self.gx[: lay["p2"]] if phase == 1 else self.gx[lay["p2"]: lay["bytes"]]

    def commit_general(self, operation, d_events, n, timestamp):
        """One batch (its harness pulse included) through the general path with this process's
        exchange; every shard returns the batch's whole reply."""
        return commit_general_batch([self], self._sum, operation, d_events, n, timestamp)

    def decide_apply(self, operation, d_events, n, timestamp, auto_pulse=True):
        """After both gathers were summed: the batch (and its pulse when due, unless the caller
        already ran it: auto_pulse False) on the scratch engine, then the owned post-batch objects
        applied here. Returns the batch's reply bytes."""
        import torch

        from .state_machine import to_host

        G, C = self.shard_count, self.batch_max + 1
        lay = _gx_layout(n, G, C)
        g = self.gx

        def recs(off, count):
            return g[off: off + count * 128].view(count, 128)

        self.invalidate_scratch()
        pulse = int(operation) == int(Operation.pulse)
        xfer = int(operation) == int(Operation.create_transfers)
        accs = [recs(lay["ra"], 2 * n), recs(lay["rq"], 2 * G * C)]
        if xfer:
            accs.append(recs(lay["rp"], 2 * n))
        acc = _unique_by_timestamp(torch.cat(accs))[0]
        xs = [recs(lay["rx"], 2 * n), recs(lay["rd"], G * C), recs(lay["rn"], G)]
        st = [g[lay["rs"]: lay["rs"] + 2 * n], torch.ones(G * C + G, dtype=torch.uint8, device=g.device)]
        x, xst = _unique_by_timestamp(torch.cat(xs), torch.cat(st))
        pn = self.pulse_next()
        sc = self.scratch
        torch.cuda.synchronize(self.device)  # the dedupe ran on torch's stream; the open reads it on the scratch's
        sc.reset()
        L = _lib.lib()
        _lib.check(L.tbg_open_device(sc.h, acc.data_ptr(), acc.shape[0], x.data_ptr(), xst.data_ptr(), x.shape[0], pn),
                   "open_device")
        sc.prepare_timestamp = timestamp
        if pulse:  # commit(.pulse): the expiry runs whatever pulse_next says (:1874-1929)
            reply = sc.commit(0, 0, timestamp, Operation.pulse, b"")
        else:
            sc.commit_window(operation, d_events, [n], [timestamp], self.gx_res.data_ptr(), self.gx_base.data_ptr(),
                             auto_pulse, timestamp)
            sc.sync()
            base = self.sm.read_device(self.gx_base)
            reply = self.sm.read_device(self.gx_res[: int(base[1]) * 8]).tobytes()
        pa, na, px, ps, nx, pn2 = (ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_void_p(), ctypes.c_void_p(),
                                   ctypes.c_uint64(), ctypes.c_uint64())
        _lib.check(L.tbg_device_state(sc.h, ctypes.byref(pa), ctypes.byref(na), ctypes.byref(px), ctypes.byref(ps),
                                      ctypes.byref(nx), ctypes.byref(pn2)), "device_state")
        ph, phs = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check(L.tbg_device_history(sc.h, ctypes.byref(ph), ctypes.byref(phs)), "device_history")
        _lib.check(L.tbg_shard_apply(self.sm.h, pa, na.value, px, ps, nx.value, ph, phs, pn2.value), "shard_apply")
        self.sm.sync()
        self._pulse_next = pn2.value
        return reply


def _gx_layout(E, G, C):
    """Byte offsets of the gather buffer (mirror of gx_view, csrc/shard_gx.inc)."""
    def al(x):
        return (x + 255) & ~255

    o = 256
    lay = {}
    lay["ra"], o = o, al(o + 2 * E * 128)
    lay["rx"], o = o, al(o + 2 * E * 128)
    lay["rs"], o = o, al(o + 2 * E)
    lay["rd"], o = o, al(o + G * C * 128)
    lay["rn"], o = o, al(o + G * 128)
    lay["p2"] = o
    lay["rp"], o = o, al(o + 2 * E * 128)
    lay["rq"], o = o, al(o + 2 * G * C * 128)
    lay["bytes"] = o
    return lay


def _unique_by_timestamp(recs, status=None):
    """Gathered 128-byte records (timestamp at byte 120; 0 = empty slot) -> distinct ones in
    timestamp order (= creation order, what tbg_open_device expects), with their status bytes."""
    import torch

    ts = recs.view(torch.int64)[:, 15]
    keep = ts != 0
    recs, ts = recs[keep], ts[keep]
    if status is not None:
        status = status[keep]
    order = torch.argsort(ts, stable=True)
    recs, ts = recs[order], ts[order]
    if status is not None:
        status = status[order]
    first = torch.ones_like(ts, dtype=torch.bool)
    if ts.numel() > 1:
        first[1:] = ts[1:] != ts[:-1]
    recs = recs[first].contiguous()
    if status is not None:
        status = status[first].contiguous()
    return recs, status


def pulse_general(shards, summed, timestamp):
    """commit(.pulse) at `timestamp` on `shards` (all shards in-process, or this process's one):
    every shard offers its batch_max + 1 smallest due (expires_at, timestamp) entries and its
    smallest live entry not yet due (gather 1), their accounts (gather 2); every shard then expires
    the same global batch_max smallest on its scratch engine (:1010-1105, :1874-1929, :2018-2173) and
    keeps what it owns."""
    op = Operation.create_transfers  # the gather's layout for zero events: only the due rows
    summed([s.gather(op, 0, 0, timestamp, 1) for s in shards])
    summed([s.gather(op, 0, 0, timestamp, 2) for s in shards])
    for s in shards:
        s.decide_apply(Operation.pulse, 0, 0, timestamp)


def read_general(shards, summed, operation, data):
    """A lookup or query on `shards` (all shards in-process, or this process's one): each writes what
    it owns, the buffers are summed, every shard builds the same reply."""
    bufs = [s.read_request(operation, data) for s in shards]
    summed(bufs)
    replies = [s.read_reply(operation, data, b) for s, b in zip(shards, bufs)]
    assert all(r == replies[0] for r in replies)
    return replies[0]


def commit_general_window(shards, summed, operation, d_events, batch_events, batch_timestamps, auto_pulse=True):
    """A window of the general class on `shards` (all shards in-process, or this process's one): the
    window's read set gathered in two rounds (csrc/shard_gw.inc), decided by each shard's scratch engine
    with the pulses inside the window modelled, each shard applying its own part. With auto_pulse the
    harness pulse before batch 0 runs with it when due; without, the caller ran it. Returns the
    per-batch replies (the same on every shard; in-process they are checked equal); falls back to
    commit_general_batch per batch when a shard has more due entries than the window path gathers or
    the scratch engine rejects the window (nothing applied then)."""
    E = sum(batch_events)
    t_last = batch_timestamps[-1]
    plan = "ok" if E > 0 else "empty"
    for attempt in range(2):
        if plan != "ok":
            break
        summed([s.gw_collect(operation, d_events, E, t_last, 1, restart=attempt > 0) for s in shards])
        plans = [s.gw_plan(operation, E) for s in shards]
        assert all(p == plans[0] for p in plans)
        plan = plans[0]
        if plan == "restart":  # the held accounts and the window's read set exceed the scratch
            plan = "ok"
            continue
        break
    if plan == "ok":
        parts = [s.gw_write(1) for s in shards]
        for k in range(3):
            summed([p[k] for p in parts])
        if shards[0]._gw_n[1]:  # (phase 2: the accounts of the gathered transfers)
            summed([s.gw_collect(operation, d_events, E, t_last, 2) for s in shards])
            summed([s.gw_write(2)[0] for s in shards])
        out = [s.gw_commit(operation, d_events, batch_events, batch_timestamps, auto_pulse) for s in shards]
        assert all((o is None) == (out[0] is None) for o in out)
        if out[0] is not None:
            assert all(o == out[0] for o in out), "shards decided the window differently"
            return out[0]
    replies, off = [], 0
    for k, (n, T) in enumerate(zip(batch_events, batch_timestamps)):
        if k > 0 and shards[0].pulse(T):
            pulse_general(shards, summed, T)
        replies.append(commit_general_batch(shards, summed, operation, d_events + off * 128, n, T,
                                            auto_pulse=auto_pulse and k == 0))
        off += n
    return replies


def commit_general_batch(shards, summed, operation, d_events, n, timestamp, auto_pulse=True):
    """One batch through the general path on `shards` (all shards in-process, or this process's
    one); `summed(list of tensors)` sums them across all shards in place. With auto_pulse the
    harness pulse before the batch runs with it when due; without, the caller ran it
    (pulse_general: a capped pulse leaves pulse() true, and only one pulse precedes a batch).
    Returns the reply."""
    summed([s.gather(operation, d_events, n, timestamp, 1) for s in shards])
    summed([s.gather(operation, d_events, n, timestamp, 2) for s in shards])
    replies = [s.decide_apply(operation, d_events, n, timestamp, auto_pulse) for s in shards]
    assert all(r == replies[0] for r in replies), "shards decided the batch differently"
    return replies[0]


def route_exchange_inprocess(shards, phase):
    """The all-to-all of a routed window's phase among shards of this process (one GPU): block
    [src -> dst] of src's send buffer into dst's receive buffer at src's offset."""
    import torch

    views = [s.route_views(phase) for s in shards]
    for s in shards:  # (engine streams are non-blocking: wait for each explicitly)
        s.stream.synchronize()
    G = len(shards)
    for src in range(G):
        send, ss = views[src][0], views[src][1]
        soff = 0
        for dst in range(G):
            recv, rs = views[dst][2], views[dst][3]
            assert rs[src] == ss[dst], (phase, src, dst, rs[src], ss[dst])
            roff = sum(rs[:src])
            recv[roff: roff + ss[dst]].copy_(send[soff: soff + ss[dst]])
            soff += ss[dst]
    torch.cuda.synchronize()


def commit_routed_inprocess(shards, operation, home_events, batch_events, batch_timestamps, results, bases,
                            bounds=None):
    """A routed window over the shards of this process: home_events[r] = the device pointer of shard r's
    home events; results[r] / bases[r] its reply buffers. Returns each shard's (home_first, home_count)."""
    G = len(shards)
    bounds = bounds or route_bounds(len(batch_events), G)
    homes = [s.route_prepare(operation, home_events[r], batch_events, batch_timestamps, bounds)
             for r, s in enumerate(shards)]
    for phase, step in ((0, "own"), (1, "decide"), (2, None)):
        route_exchange_inprocess(shards, phase)
        if step:
            for s in shards:
                s.route_step(step)
    for r, s in enumerate(shards):
        s.route_apply(results[r], bases[r])
    return homes
