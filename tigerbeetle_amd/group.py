"""StateMachine interface over a hash-sharded group of engines driven natively (include/tbg.h
tbg_group_*, csrc/group.inc): G shards in one process, one host thread, the group's own exchanges
(device copies, or RCCL over xGMI with one communicator per GPU). The same calls and reply bytes as
StateMachine (src/state_machine.zig:589-648, 1107-1146); the dispatch (routed order-free windows, the
general path, pulses, lookups) is the library's, not Python's."""
import ctypes

import numpy as np

from . import _lib
from .state_machine import MESSAGE_BODY_SIZE_MAX, StateMachine
from .types import BATCH_MAX, Operation


class _ShardView(StateMachine):
    """One shard's engine inside a group (owned by the group: never destroyed here)."""

    def __init__(self, h, batch_max):
        self.h = h
        self.batch_max = batch_max
        self._out = np.zeros(16, np.uint8)

    def close(self):
        self.h = None


class GroupStateMachine:
    def __init__(self, shard_count, devices=None, exchange="copy", batch_max=BATCH_MAX, accounts_max=1 << 16,
                 transfers_max=1 << 20, window_events_max=0, change_log=False):
        L = _lib.lib()
        devs = list(devices) if devices is not None else [0] * shard_count
        self._devs = (ctypes.c_int32 * shard_count)(*devs)
        cfg = _lib.GroupConfig(shard_count, _lib.EXCHANGE_RCCL if exchange == "rccl" else _lib.EXCHANGE_COPY,
                               self._devs, batch_max, window_events_max, accounts_max, transfers_max,
                               _lib.FLAG_CHANGE_LOG if change_log else 0, 0)
        h = ctypes.c_void_p()
        _lib.check(L.tbg_group_create(ctypes.byref(cfg), ctypes.byref(h)), "tbg_group_create")
        self.h = h
        self.G = shard_count
        self.batch_max = batch_max
        self.prepare_timestamp = self.prefetch_timestamp = self.commit_timestamp = 0
        self._out = np.zeros(MESSAGE_BODY_SIZE_MAX, np.uint8)
        self.shards = []
        for r in range(shard_count):
            e = ctypes.c_void_p()
            _lib.check(L.tbg_group_engine(self.h, r, ctypes.byref(e)), "group_engine")
            self.shards.append(_ShardView(e, batch_max))

    def close(self):
        h, self.h = getattr(self, "h", None), None
        if h and _lib is not None and _lib.lib is not None:
            _lib.lib().tbg_group_destroy(h)

    def __del__(self):
        self.close()

    def input_valid(self, operation, data):
        return bool(_lib.lib().tbg_input_valid(None, int(operation), len(data)))

    def prepare(self, operation, data):
        assert self.input_valid(operation, data)
        if operation in (Operation.create_accounts, Operation.create_transfers):
            self.prepare_timestamp += len(data) // 128

    def pulse(self):
        needed = ctypes.c_int()
        _lib.check(_lib.lib().tbg_group_pulse_needed(self.h, self.prepare_timestamp, ctypes.byref(needed)), "pulse")
        return bool(needed.value)

    def prefetch(self, op, operation, data):
        self._pf = np.frombuffer(data, np.uint8) if len(data) else np.zeros(0, np.uint8)
        _lib.check(_lib.lib().tbg_group_prefetch(self.h, op, int(operation), self._pf.ctypes.data if len(data) else None,
                                                 len(data), self.prefetch_timestamp), "prefetch")

    def commit(self, client, op, timestamp, operation, data):
        buf = np.frombuffer(data, np.uint8) if len(data) else np.zeros(0, np.uint8)
        n = ctypes.c_uint64()
        _lib.check(_lib.lib().tbg_group_commit(self.h, op, timestamp, int(operation), buf.ctypes.data if len(data) else None,
                                               len(data), self._out.ctypes.data, len(self._out), ctypes.byref(n)),
                   "group_commit")
        if operation in (Operation.create_accounts, Operation.create_transfers):
            self.commit_timestamp = timestamp
        return self._out[: n.value].tobytes()

    def commit_window(self, operation, batches, tick_ns=0):
        """Host batches under the harness protocol (a pulse check before each): per-batch replies."""
        ns, ts = [], []
        self.prepare_timestamp += tick_ns
        for ev in batches:
            self.prepare_timestamp += 1 + len(ev)
            ns.append(len(ev))
            ts.append(self.prepare_timestamp)
        data = np.concatenate([np.frombuffer(ev.tobytes(), np.uint8) for ev in batches]) if batches else \
            np.zeros(0, np.uint8)
        res = np.zeros(max(len(data) // 128, 1) * 8, np.uint8)
        base = np.zeros(len(ns) + 1, np.uint32)
        nb = len(ns)
        _lib.check(_lib.lib().tbg_group_commit_window(self.h, int(operation), data.ctypes.data if len(data) else None, nb,
                                                      (ctypes.c_uint32 * nb)(*ns), (ctypes.c_uint64 * nb)(*ts),
                                                      res.ctypes.data, base.ctypes.data), "group_commit_window")
        rb = res.tobytes()
        return [rb[base[b] * 8: base[b + 1] * 8] for b in range(nb)]

    def stats(self):
        return self.shards[0].stats()

    def pulse_next_timestamp(self):
        return self.shards[0].stats()["pulse_next_timestamp"]

    def dump_accounts(self):
        a = np.concatenate([s.dump_accounts() for s in self.shards])
        return a[np.argsort(a["timestamp"], kind="stable")]

    def dump_transfers(self):
        t = np.concatenate([s.dump_transfers() for s in self.shards])
        return t[np.argsort(t["timestamp"], kind="stable")]

    def dump_transfer_status(self):
        parts = [(s.dump_transfers()["timestamp"], s.dump_transfer_status()) for s in self.shards]
        ts = np.concatenate([p[0] for p in parts])
        st = np.concatenate([p[1] for p in parts])
        return st[np.argsort(ts, kind="stable")]
