"""StateMachine boundary over the CPU restatement (oracle/liboracle.so). TEST INFRASTRUCTURE.

Same surface as tigerbeetle_amd.StateMachine (the product), so the KAT harness (tests/kat.py)
drives both identically. Follows state_machine.zig:543-648 (input_valid/prepare/pulse/prefetch)
and :1107-1146 (commit).
"""
import ctypes
import os
import subprocess

import numpy as np

from tigerbeetle_amd.types import ACCOUNT_DTYPE, BALANCE_DTYPE, BATCH_MAX, RESULT_DTYPE, TRANSFER_DTYPE, Operation

ORACLE_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")
_lib = None


class U128(ctypes.Structure):
    _fields_ = [("lo", ctypes.c_uint64), ("hi", ctypes.c_uint64)]


def u128(v):
    return U128(v & 0xFFFFFFFFFFFFFFFF, v >> 64)


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(ORACLE_DIR, "liboracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = ctypes.CDLL(path)
        vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
        L.tbo_create.restype = vp
        L.tbo_create.argtypes = [u32]
        L.tbo_destroy.argtypes = [vp]
        L.tbo_pulse_needed.argtypes = [vp, u64]
        L.tbo_pulse_next_timestamp.argtypes = [vp]
        L.tbo_pulse_next_timestamp.restype = u64
        L.tbo_pulse.argtypes = [vp, u64]
        L.tbo_pulse.restype = u32
        for f in (L.tbo_create_accounts, L.tbo_create_transfers):
            f.argtypes = [vp, u64, vp, u32, vp]
            f.restype = u32
        for f in (L.tbo_lookup_accounts, L.tbo_lookup_transfers):
            f.argtypes = [vp, vp, u32, vp]
            f.restype = u32
        L.tbo_setup_balances.argtypes = [vp, U128, U128, U128, U128, U128]
        L.tbo_account_count.argtypes = [vp]
        L.tbo_account_count.restype = u64
        L.tbo_transfer_count.argtypes = [vp]
        L.tbo_transfer_count.restype = u64
        L.tbo_dump_accounts.argtypes = [vp, vp, u64]
        L.tbo_dump_accounts.restype = u64
        L.tbo_dump_transfers.argtypes = [vp, vp, u64]
        L.tbo_dump_transfers.restype = u64
        L.tbo_pending_status.argtypes = [vp, u64]
        L.tbo_pending_status.restype = u32
        L.tbo_input_valid.argtypes = [u32, u64, u32]
        for f in (L.tbo_get_account_transfers, L.tbo_get_account_balances):
            f.argtypes = [vp, vp, vp]
            f.restype = u32
        L.tbo_dump_account_balances.argtypes = [vp, vp, u64]
        L.tbo_dump_account_balances.restype = u64
        L.tbo_dump_transfer_status.argtypes = [vp, vp, u64]
        L.tbo_dump_transfer_status.restype = u64
        _lib = L
    return _lib


class OracleStateMachine:
    def __init__(self, batch_max=BATCH_MAX):
        self.batch_max = batch_max
        self.h = lib().tbo_create(batch_max)
        self.prepare_timestamp = 0
        self.prefetch_timestamp = 0
        self.commit_timestamp = 0

    def close(self):
        if self.h:
            lib().tbo_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def input_valid(self, operation, data):
        return bool(lib().tbo_input_valid(int(operation), len(data), self.batch_max))

    def prepare(self, operation, data):
        assert self.input_valid(operation, data)
        if operation in (Operation.create_accounts, Operation.create_transfers):
            self.prepare_timestamp += len(data) // 128

    def pulse(self):
        return bool(lib().tbo_pulse_needed(self.h, self.prepare_timestamp))

    def prefetch(self, op, operation, data):
        assert self.input_valid(operation, data)

    def commit(self, client, op, timestamp, operation, data):
        L = lib()
        buf = np.frombuffer(data, np.uint8).copy() if data else np.zeros(16, np.uint8)
        if operation == Operation.pulse:
            L.tbo_pulse(self.h, timestamp)
            return b""
        if operation in (Operation.create_accounts, Operation.create_transfers):
            n = len(data) // 128
            out = np.zeros(max(n, 1), RESULT_DTYPE)
            fn = L.tbo_create_accounts if operation == Operation.create_accounts else L.tbo_create_transfers
            c = fn(self.h, timestamp, buf.ctypes.data, n, out.ctypes.data)
            self.commit_timestamp = timestamp
            return out[:c].tobytes()
        if operation in (Operation.lookup_accounts, Operation.lookup_transfers):
            n = len(data) // 16
            dt = ACCOUNT_DTYPE if operation == Operation.lookup_accounts else TRANSFER_DTYPE
            out = np.zeros(max(n, 1), dt)
            fn = L.tbo_lookup_accounts if operation == Operation.lookup_accounts else L.tbo_lookup_transfers
            c = fn(self.h, buf.ctypes.data, n, out.ctypes.data)
            return out[:c].tobytes()
        if operation in (Operation.get_account_transfers, Operation.get_account_balances):
            # input_valid (state_machine.zig:548-552) admits exactly one 64 B AccountFilter
            out = np.zeros(self.batch_max, TRANSFER_DTYPE if operation == Operation.get_account_transfers
                           else BALANCE_DTYPE)
            fn = (L.tbo_get_account_transfers if operation == Operation.get_account_transfers
                  else L.tbo_get_account_balances)
            c = fn(self.h, buf.ctypes.data, out.ctypes.data)
            return out[:c].tobytes()
        raise NotImplementedError(operation)

    # test hooks
    def setup_balances(self, ident, dp, dpo, cp, cpo):
        rc = lib().tbo_setup_balances(self.h, u128(ident), u128(dp), u128(dpo), u128(cp), u128(cpo))
        assert rc == 0

    def pulse_next_timestamp(self):
        return lib().tbo_pulse_next_timestamp(self.h)

    def dump_accounts(self):
        L = lib()
        n = L.tbo_account_count(self.h)
        out = np.zeros(max(n, 1), ACCOUNT_DTYPE)
        L.tbo_dump_accounts(self.h, out.ctypes.data, n)
        return out[:n]

    def dump_transfers(self):
        L = lib()
        n = L.tbo_transfer_count(self.h)
        out = np.zeros(max(n, 1), TRANSFER_DTYPE)
        L.tbo_dump_transfers(self.h, out.ctypes.data, n)
        return out[:n]

    def dump_transfer_status(self):
        L = lib()
        n = L.tbo_transfer_count(self.h)
        out = np.zeros(max(n, 1), np.uint8)
        L.tbo_dump_transfer_status(self.h, out.ctypes.data, n)
        return out[:n]

    def dump_account_balances(self):
        """The account_balances groove's rows, timestamp order (256 B each)."""
        L = lib()
        n = L.tbo_dump_account_balances(self.h, None, 0)
        out = np.zeros(max(n, 1) * 256, np.uint8)
        L.tbo_dump_account_balances(self.h, out.ctypes.data, n)
        return out[: n * 256]
