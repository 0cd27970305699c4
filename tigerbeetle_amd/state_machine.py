"""StateMachine boundary over the MI355X engine (libtbgpu.so).

Mirrors the reference interface (src/state_machine.zig): `input_valid` (:543-572), `prepare`
(:575-587), `pulse` (:589-596), `prefetch` (:598-648), `commit` (:1107-1146) and the public
timestamp fields (:433-435), with the test-harness hook `setup_balances` (:2545-2561). Every call
goes through the C ABI in include/tbg.h; there is no CPU fallback.
"""
import ctypes

import numpy as np

from . import _lib
from .types import ACCOUNT_DTYPE, BATCH_MAX, TRANSFER_DTYPE, Operation

PENDING_ROW_DTYPE = np.dtype([("timestamp", "<u8"), ("status", "u1"), ("padding", "u1", (7,))])  # 16 B

MESSAGE_BODY_SIZE_MAX = 1048576 - 256


def to_host(t):
    """Device tensor -> numpy copy through pinned memory, ordered on the current stream."""
    import torch

    c = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    c.copy_(t, non_blocking=True)
    torch.cuda.current_stream().synchronize()
    return c.numpy().copy()


def _np_dtype(dt):
    import torch

    return {torch.uint8: np.uint8, torch.int32: np.int32, torch.int64: np.int64, torch.uint32: np.uint32,
            torch.float32: np.float32}[dt]


class HostBuffer:
    """Pinned host memory from tbg_host_alloc, as a uint8 array: a replica's message buffer (allocated
    once, vsr/message_pool.zig). A request in it reaches the device by one DMA (include/tbg.h
    tbg_host_register)."""

    def __init__(self, nbytes):
        p = ctypes.c_void_p()
        _lib.check(_lib.lib().tbg_host_alloc(nbytes, ctypes.byref(p)), "host_alloc")
        self.ptr = p.value
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(self.ptr))

    def close(self):
        p, self.ptr = getattr(self, "ptr", None), None
        if p and _lib is not None and _lib.lib is not None:
            self.array = None
            _lib.lib().tbg_host_free(p)

    def __del__(self):
        self.close()


class StateMachine:
    def __init__(self, device=0, batch_max=BATCH_MAX, accounts_max=1 << 16, transfers_max=1 << 20,
                 window_events_max=0, resolver=True, components=True, shard_count=0, shard_index=0,
                 change_log=False, fused=True):
        L = _lib.lib()
        # resolver: True = chunked single-workgroup resolver (chunks.h) where the window fits it, else
        # windowed relaxation (relax.h); "relax" = relaxation only; "wait" = wait-based walkers
        # (resolver.h); False = sequential walker only
        flags = ((0 if resolver else _lib.FLAG_NO_RESOLVER) | (0 if components else _lib.FLAG_NO_COMPONENTS) |
                 (_lib.FLAG_RES_WAIT if resolver == "wait" else 0) |
                 (_lib.FLAG_NO_CHUNKS if resolver == "relax" else 0) | (_lib.FLAG_CHANGE_LOG if change_log else 0) |
                 (0 if fused else _lib.FLAG_NO_FUSED))
        # fused: order-free transfer windows may commit in one pass (csrc/fused.h); False = general path
        cfg = _lib.Config(device, batch_max, accounts_max, transfers_max, window_events_max, flags, shard_count,
                          shard_index)
        h = ctypes.c_void_p()
        _lib.check(L.tbg_create(ctypes.byref(cfg), ctypes.byref(h)), "tbg_create")
        self.h = h
        self.batch_max = batch_max
        self.prepare_timestamp = 0
        self.prefetch_timestamp = 0
        self.commit_timestamp = 0
        self._out = np.zeros(MESSAGE_BODY_SIZE_MAX, np.uint8)

    def close(self):
        h, self.h = getattr(self, "h", None), None
        if h and _lib is not None and _lib.lib is not None:  # module globals may be gone at exit
            _lib.lib().tbg_destroy(h)

    def __del__(self):
        self.close()

    @property
    def stream(self):
        return _lib.lib().tbg_stream(self.h)

    def input_valid(self, operation, data):
        return bool(_lib.lib().tbg_input_valid(self.h, int(operation), len(data)))

    def prepare(self, operation, data):
        assert self.input_valid(operation, data)
        if operation in (Operation.create_accounts, Operation.create_transfers):
            self.prepare_timestamp += len(data) // 128

    def pulse(self):
        needed = ctypes.c_int()
        _lib.check(_lib.lib().tbg_pulse_needed(self.h, self.prepare_timestamp, ctypes.byref(needed)), "pulse")
        return bool(needed.value)

    def prefetch(self, op, operation, data):
        self._pf_data = data
        self._pf = np.frombuffer(data, np.uint8) if len(data) else np.zeros(0, np.uint8)
        ptr = self._pf.ctypes.data if len(data) else None
        _lib.check(_lib.lib().tbg_prefetch(self.h, op, int(operation), ptr, len(data), self.prefetch_timestamp),
                   "prefetch")

    def commit(self, client, op, timestamp, operation, data):
        # the prefetched request (the same buffer, so tbg_commit finds its prefetch)
        pf = getattr(self, "_pf", None)
        same = pf is not None and (data is self._pf_data or
                                   np.array_equal(pf, np.frombuffer(data, np.uint8) if len(data) else pf[:0]))
        buf = pf if same else (
            np.frombuffer(data, np.uint8) if len(data) else np.zeros(0, np.uint8))
        ptr = buf.ctypes.data if len(data) else None
        n = ctypes.c_uint64()
        _lib.check(_lib.lib().tbg_commit(self.h, op, timestamp, int(operation), ptr, len(data),
                                         self._out.ctypes.data, len(self._out), ctypes.byref(n)), "commit")
        self._pf = None
        if operation in (Operation.create_accounts, Operation.create_transfers):
            self.commit_timestamp = timestamp
        return self._out[: n.value].tobytes()

    # ---- test hooks / introspection -----------------------------------------------------------
    def setup_balances(self, ident, dp, dpo, cp, cpo):
        args = [ctypes.byref(_lib.u128(v)) for v in (ident, dp, dpo, cp, cpo)]
        _lib.check(_lib.lib().tbg_setup_balances(self.h, *args), "setup_balances")

    def stats(self):
        s = _lib.Stats()
        _lib.check(_lib.lib().tbg_get_stats(self.h, ctypes.byref(s)), "stats")
        return {f: getattr(s, f) for f, _ in _lib.Stats._fields_}

    def window_changes(self):
        """Write-back stream of the last committed create_* window (include/tbg.h tbg_window_changes):
        (changed/new account records, inserted transfer records, TransferPending rows as a structured
        array of (timestamp, status))."""
        L = _lib.lib()
        na, nt, npd = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        rc = L.tbg_window_changes(self.h, None, 0, ctypes.byref(na), None, 0, ctypes.byref(nt), None, 0,
                                  ctypes.byref(npd))
        if rc not in (0, -2):
            _lib.check(rc, "window_changes")
        acc = np.zeros(na.value, ACCOUNT_DTYPE)
        xfer = np.zeros(nt.value, TRANSFER_DTYPE)
        rows = np.zeros(npd.value, PENDING_ROW_DTYPE)
        _lib.check(L.tbg_window_changes(self.h, acc.ctypes.data, len(acc), ctypes.byref(na), xfer.ctypes.data,
                                        len(xfer), ctypes.byref(nt), rows.ctypes.data, len(rows),
                                        ctypes.byref(npd)), "window_changes")
        return acc, xfer, rows

    def pulse_next_timestamp(self):
        return self.stats()["pulse_next_timestamp"]

    def dump_accounts(self):
        n0 = self.stats()["accounts"]
        out = np.zeros(max(n0, 1), ACCOUNT_DTYPE)
        n = ctypes.c_uint64()
        _lib.check(_lib.lib().tbg_dump_accounts(self.h, out.ctypes.data, n0, ctypes.byref(n)), "dump")
        return out[: n.value]

    def dump_transfers(self):
        n0 = self.stats()["transfers"]
        out = np.zeros(max(n0, 1), TRANSFER_DTYPE)
        n = ctypes.c_uint64()
        _lib.check(_lib.lib().tbg_dump_transfers(self.h, out.ctypes.data, n0, ctypes.byref(n)), "dump")
        return out[: n.value]

    def dump_transfer_status(self):
        n0 = self.stats()["transfers"]
        out = np.zeros(max(n0, 1), np.uint8)
        n = ctypes.c_uint64()
        _lib.check(_lib.lib().tbg_dump_transfer_status(self.h, out.ctypes.data, n0, ctypes.byref(n)), "dump")
        return out[: n.value]

    # ---- device-resident streaming ------------------------------------------------------------
    def commit_device(self, operation, timestamp, d_events, n, d_results, d_count, auto_pulse, prepare_timestamp):
        _lib.check(_lib.lib().tbg_commit_device(self.h, int(operation), timestamp, d_events, n, d_results, d_count,
                                                int(auto_pulse), prepare_timestamp), "commit_device")

    def commit_window(self, operation, d_events, batch_events, batch_timestamps, d_results, d_batch_base,
                      auto_pulse, prepare_timestamp):
        """Super-batched commit of consecutive batches (tbg_commit_window); asynchronous."""
        nb = len(batch_events)
        ev = (ctypes.c_uint32 * nb)(*batch_events)
        ts = (ctypes.c_uint64 * nb)(*batch_timestamps)
        _lib.check(_lib.lib().tbg_commit_window(self.h, int(operation), d_events, nb, ev, ts, d_results,
                                                d_batch_base, int(auto_pulse), prepare_timestamp),
                   "commit_window")

    def commit_window_host(self, operation, h_events, batch_events, batch_timestamps, h_results, h_batch_base,
                           auto_pulse, prepare_timestamp):
        """Host-fed window (tbg_commit_window_host): pinned host pointers; asynchronous; returns a
        ticket for window_done()."""
        nb = len(batch_events)
        ev = (ctypes.c_uint32 * nb)(*batch_events)
        ts = (ctypes.c_uint64 * nb)(*batch_timestamps)
        t = ctypes.c_uint64()
        _lib.check(_lib.lib().tbg_commit_window_host(self.h, int(operation), h_events, nb, ev, ts, h_results,
                                                     h_batch_base, int(auto_pulse), prepare_timestamp,
                                                     ctypes.byref(t)), "commit_window_host")
        return t.value

    def window_done(self, ticket):
        done = ctypes.c_int()
        _lib.check(_lib.lib().tbg_host_window_done(self.h, ticket, ctypes.byref(done)), "host_window_done")
        return bool(done.value)

    def sync(self):
        _lib.check(_lib.lib().tbg_sync(self.h), "sync")

    def read_device(self, t):
        """A device tensor (contiguous) as a numpy array, after the work queued on the engine stream:
        a kernel copy through the engine's pinned block (tbg_read_device), no copy-engine handoff."""
        out = np.empty(t.numel() * t.element_size(), dtype=np.uint8)
        _lib.check(_lib.lib().tbg_read_device(self.h, out.ctypes.data, t.data_ptr(), out.nbytes), "read_device")
        return out.view(_np_dtype(t.dtype)).reshape(tuple(t.shape))

    # ---- the rest of the reference surface the replica drives ------------------------------
    def open(self, accounts, transfers, pending_status, account_balances=None):
        """StateMachine.open (state_machine.zig:527-541): an empty engine takes the forest's objects
        (records in timestamp order, one TransferPending status per transfer, and the
        account_balances groove's 256 B rows in timestamp order)."""
        acc = np.ascontiguousarray(accounts)
        xf = np.ascontiguousarray(transfers)
        st = np.ascontiguousarray(pending_status, dtype=np.uint8)
        hb = np.ascontiguousarray(account_balances if account_balances is not None else np.zeros(0, np.uint8),
                                  dtype=np.uint8)
        _lib.check(_lib.lib().tbg_open(self.h, acc.ctypes.data if len(acc) else None, len(acc),
                                       xf.ctypes.data if len(xf) else None, len(xf),
                                       st.ctypes.data if len(st) else None,
                                       hb.ctypes.data if len(hb) else None, len(hb) // 256), "open")

    def reset(self):
        """StateMachine.reset (state_machine.zig:486-501)."""
        _lib.check(_lib.lib().tbg_reset(self.h), "reset")
        self.prepare_timestamp = self.prefetch_timestamp = self.commit_timestamp = 0

    def prefetch_done(self):
        done = ctypes.c_int()
        _lib.check(_lib.lib().tbg_prefetch_poll(self.h, ctypes.byref(done)), "prefetch_poll")
        return bool(done.value)

    def compact(self, op):
        _lib.check(_lib.lib().tbg_compact(self.h, op), "compact")

    def checkpoint(self):
        _lib.check(_lib.lib().tbg_checkpoint(self.h), "checkpoint")

    def digest(self):
        """tbg_digest: [accounts, transfers, statuses, pulse_next_timestamp] (tigerbeetle_amd.digest)."""
        out = (ctypes.c_uint64 * 4)()
        _lib.check(_lib.lib().tbg_digest(self.h, out), "digest")
        return list(out)

    def windows_committed(self):
        """(applied, submitted) create_* windows since creation (tbg_windows_committed)."""
        a, s = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.check(_lib.lib().tbg_windows_committed(self.h, ctypes.byref(a), ctypes.byref(s)), "windows_committed")
        return a.value, s.value

    def aof_replay(self, data, flags=0):
        """tbg_aof_replay: applies an AOF file's prepares (bytes / uint8 array, e.g. np.memmap) in
        order, every checksum verified on the GPU. Returns the stats as a dict; `error` names the
        AOF.Iterator error at `error_entry` (the entries before it are applied) or is None."""
        buf = np.ascontiguousarray(np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray)) else data)
        st = _lib.AofStats()
        rc = _lib.lib().tbg_aof_replay(self.h, buf.ctypes.data if buf.size else None, buf.size, flags,
                                       ctypes.byref(st))
        if rc not in (0, -1) or (rc == -1 and st.error == 0):
            _lib.check(rc, "aof_replay")
        out = {k: getattr(st, k) for k, _ in _lib.AofStats._fields_ if k != "reserved"}
        out["error"] = _lib.AOF_ERRORS[st.error]
        return out
