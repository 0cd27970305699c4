"""Hash-sharded commit over the GPUs of one node: one engine per GPU, one process per GPU.

Account a lives on shard `shard_of(a.id)`, transfer t on shard `shard_of(t.id)` (csrc/shard.h).
Every shard receives the same prepared window (the replica hands each GPU the same prepare body,
state_machine.zig:1107-1146) and is the home of a contiguous range of its batches (`home_range`).
A window commits in five steps through the C ABI (include/tbg.h):

  tbg_shard_prepare_window   owned roles only: validate, resolve the owned accounts / ids, write the
                             owner facts (9 B per transfer: debit / credit ledger, exists code +
                             limit bits; one writer per bit)
  exchange                   byte-wise sum of the facts across the shards, on the engine's stream
                             (RCCL uint8 all-reduce over xGMI: torch "nccl")
  tbg_shard_decide_window    home batches only: decide, write their replies and one commit bit per
                             event
  exchange                   byte-wise sum of the commit bits (E/8 B) across the shards
  tbg_shard_commit_window    owned effects of the committed events

The `exchange` callable is the only collective on the data path; with one shard there is none.
Per shard, the work is the window's ids plus 1/G of the rest: it falls as G grows.
"""
import ctypes

import numpy as np

from . import _lib
from .state_machine import StateMachine

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


def home_range(n_batches, shard_count, shard_index):
    """Home batches [first, first + count) of `shard_index`: contiguous, as even as possible."""
    lo = n_batches * shard_index // shard_count
    hi = n_batches * (shard_index + 1) // shard_count
    return lo, hi - lo


class ShardedStateMachine:
    """One shard of a hash-sharded engine. `exchange(t)` must sum the uint8 tensor `t` in place
    across all shards (None for a single shard)."""

    def __init__(self, shard_count, shard_index, exchange=None, device=0, batch_max=8190, accounts_max=1 << 16,
                 transfers_max=1 << 20, window_events_max=0):
        import torch

        self.sm = StateMachine(device=device, batch_max=batch_max, accounts_max=accounts_max,
                               transfers_max=transfers_max, window_events_max=window_events_max,
                               shard_count=shard_count, shard_index=shard_index)
        self.shard_count, self.shard_index = shard_count, shard_index
        self.exchange = exchange
        events_max = window_events_max or batch_max
        dev = torch.device("cuda", device)
        self.xch = torch.zeros(16 + 9 * events_max, dtype=torch.uint8, device=dev)
        self.bits = torch.zeros(int(_lib.lib().tbg_shard_commit_bits_bytes(events_max)), dtype=torch.uint8, device=dev)
        self.stream = torch.cuda.ExternalStream(self.sm.stream, device=dev)
        self._n_events = 0
        torch.cuda.synchronize(device)

    @property
    def h(self):
        return self.sm.h

    def close(self):
        self.sm.close()

    def home_range(self, n_batches):
        return home_range(n_batches, self.shard_count, self.shard_index)

    def prepare_window(self, operation, d_events, batch_events, batch_timestamps):
        """Step 1; returns the facts tensor to be summed across the shards."""
        nb = len(batch_events)
        ev = (ctypes.c_uint32 * nb)(*batch_events)
        ts = (ctypes.c_uint64 * nb)(*batch_timestamps)
        _lib.check(_lib.lib().tbg_shard_prepare_window(self.sm.h, int(operation), d_events, nb, ev, ts,
                                                       self.xch.data_ptr()), "shard_prepare_window")
        self._n_events = sum(batch_events)
        n = _lib.lib().tbg_shard_exchange_bytes(int(operation), self._n_events)
        return self.xch[:n]

    def decide_window(self, home_first, home_count, d_results, d_batch_base):
        """Step 3 (after the facts were summed); returns the commit-bit tensor to be summed."""
        _lib.check(_lib.lib().tbg_shard_decide_window(self.sm.h, self.xch.data_ptr(), home_first, home_count,
                                                      d_results, d_batch_base, self.bits.data_ptr()),
                   "shard_decide_window")
        return self.bits[:_lib.lib().tbg_shard_commit_bits_bytes(self._n_events)]

    def commit_decided(self):
        """Step 5 (after the commit bits were summed)."""
        _lib.check(_lib.lib().tbg_shard_commit_window(self.sm.h, self.xch.data_ptr(), self.bits.data_ptr()),
                   "shard_commit_window")

    def commit_window(self, operation, d_events, batch_events, batch_timestamps, d_results, d_batch_base):
        """Asynchronous on the engine stream. Replies of this shard's home batches (home_range) land
        in d_results / d_batch_base (d_batch_base[0..home_count]); returns (home_first, home_count)."""
        import torch

        first, count = self.home_range(len(batch_events))
        words = self.prepare_window(operation, d_events, batch_events, batch_timestamps)
        if self.exchange is not None:
            with torch.cuda.stream(self.stream):
                self.exchange(words)
        bits = self.decide_window(first, count, d_results, d_batch_base)
        if self.exchange is not None:
            with torch.cuda.stream(self.stream):
                self.exchange(bits)
        self.commit_decided()
        return first, count

    def sync(self):
        self.sm.sync()

    def stats(self):
        return self.sm.stats()
