"""Loader for the in-tree HIP library (libtbgpu.so). The product path has no fallback: if the
library is missing or cannot load, every entry point raises."""
import ctypes
import os

from .types import ACCOUNT_DTYPE  # noqa: F401  (keeps the dtypes importable alongside the lib)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libtbgpu.so")

# Every symbol declared in include/tbg.h.
EXPORTS = [
    "tbg_create", "tbg_destroy", "tbg_input_valid", "tbg_pulse_needed", "tbg_prefetch", "tbg_commit",
    "tbg_commit_device", "tbg_commit_window", "tbg_sync", "tbg_read_device", "tbg_stream", "tbg_setup_balances", "tbg_get_stats",
    "tbg_dump_accounts", "tbg_dump_transfers", "tbg_dump_transfer_status", "tbg_device_stores",
    "tbg_gen_accounts", "tbg_gen_transfers_uniform", "tbg_gen_permute_ids", "tbg_gen_mark_pending", "tbg_version", "tbg_debug_last_batch",
    "tbg_timing_enable", "tbg_timing_collect", "tbg_gen_accounts_cfg3", "tbg_gen_funding_cfg3",
    "tbg_gen_transfers_zipf", "tbg_gen_transfers_cfg4", "tbg_debug_counters", "tbg_shard_of",
    "tbg_shard_prepare_window", "tbg_shard_commit_window", "tbg_shard_exchange_bytes",
    "tbg_window_changes", "tbg_windows_committed",
    "tbg_open", "tbg_reset", "tbg_prefetch_poll", "tbg_compact", "tbg_checkpoint", "tbg_digest",
    "tbg_commit_window_host", "tbg_host_window_done", "tbg_host_alloc", "tbg_host_free", "tbg_host_register",
    "tbg_host_unregister", "tbg_checksum",
    "tbg_demux_init", "tbg_demux_decode", "tbg_aof_replay", "tbg_shard_gather_bytes", "tbg_shard_gather",
    "tbg_gw_collect", "tbg_gw_write", "tbg_gw_commit", "tbg_gw_result",
    "tbg_shard_apply", "tbg_open_device", "tbg_device_state", "tbg_device_history", "tbg_shard_lookup_bytes",
    "tbg_shard_lookup", "tbg_shard_lookup_reply", "tbg_shard_query_bytes", "tbg_shard_query", "tbg_shard_query_merge",
    "tbg_debug_table_used", "tbg_route_prepare", "tbg_route_buffers", "tbg_route_buffer_bytes", "tbg_route_attach", "tbg_route_own", "tbg_route_decide",
    "tbg_route_apply", "tbg_group_create", "tbg_group_destroy", "tbg_group_pulse_needed", "tbg_group_prefetch",
    "tbg_group_commit", "tbg_group_commit_window", "tbg_group_engine",
]


class U128(ctypes.Structure):
    _fields_ = [("lo", ctypes.c_uint64), ("hi", ctypes.c_uint64)]


def u128(v):
    return U128(v & 0xFFFFFFFFFFFFFFFF, (v >> 64) & 0xFFFFFFFFFFFFFFFF)


class Config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("batch_max", ctypes.c_uint32),
                ("accounts_max", ctypes.c_uint64), ("transfers_max", ctypes.c_uint64),
                ("window_events_max", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("shard_count", ctypes.c_uint32), ("shard_index", ctypes.c_uint32)]


FLAG_NO_RESOLVER = 1
FLAG_NO_COMPONENTS = 2
FLAG_RES_WAIT = 4
FLAG_CHANGE_LOG = 8
FLAG_NO_XWIN = 16
FLAG_NO_CHUNKS = 32
FLAG_NO_FUSED = 64


class GroupConfig(ctypes.Structure):
    _fields_ = [("shard_count", ctypes.c_uint32), ("exchange", ctypes.c_uint32),
                ("devices", ctypes.POINTER(ctypes.c_int32)), ("batch_max", ctypes.c_uint32),
                ("window_events_max", ctypes.c_uint32), ("accounts_max", ctypes.c_uint64),
                ("transfers_max", ctypes.c_uint64), ("flags", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


EXCHANGE_COPY = 0
EXCHANGE_RCCL = 1


class Stats(ctypes.Structure):
    _fields_ = [("accounts", ctypes.c_uint64), ("transfers", ctypes.c_uint64),
                ("expiry_entries", ctypes.c_uint64), ("pulse_next_timestamp", ctypes.c_uint64),
                ("events_total", ctypes.c_uint64), ("walker_events", ctypes.c_uint64),
                ("resolver_events", ctypes.c_uint64), ("component_events", ctypes.c_uint64),
                ("sorted_transfers", ctypes.c_uint64), ("chunked_windows", ctypes.c_uint64),
                ("fused_windows", ctypes.c_uint64), ("ovf_rescans", ctypes.c_uint64)]


class Demuxer(ctypes.Structure):
    _fields_ = [("results", ctypes.c_void_p), ("count", ctypes.c_uint32), ("operation", ctypes.c_uint32)]


class AofStats(ctypes.Structure):
    _fields_ = [("entries", ctypes.c_uint64), ("prepares", ctypes.c_uint64), ("pulses", ctypes.c_uint64),
                ("skipped", ctypes.c_uint64), ("windows", ctypes.c_uint64), ("events", ctypes.c_uint64),
                ("failed_events", ctypes.c_uint64), ("error_entry", ctypes.c_int64), ("error", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


AOF_ERRORS = {0: None, 1: "AOFShortRead", 2: "AOFMagicNumberMismatch", 3: "AOFChecksumMismatch",
              4: "AOFBodyChecksumMismatch", 5: "AOFChecksumChainMismatch", 6: "InvalidPrepareBody"}
AOF_NO_CHAIN = 1
WINDOW_LOG = 2

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: torch ships its own libamdhip64 (same soname). Loading torch first
    # makes libtbgpu bind to that copy; loading libtbgpu first and torch later would put two runtimes
    # in the process and torch would see no GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(LIB_PATH)
    vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32
    P = ctypes.POINTER
    sig = {
        "tbg_create": ([P(Config), P(vp)], i32),
        "tbg_destroy": ([vp], i32),
        "tbg_input_valid": ([vp, u32, u64], i32),
        "tbg_pulse_needed": ([vp, u64, P(ctypes.c_int)], i32),
        "tbg_prefetch": ([vp, u64, u32, vp, u64, u64], i32),
        "tbg_commit": ([vp, u64, u64, u32, vp, u64, vp, u64, P(u64)], i32),
        "tbg_commit_device": ([vp, u32, u64, vp, u32, vp, vp, ctypes.c_int, u64], i32),
        "tbg_commit_window": ([vp, u32, vp, u32, vp, vp, vp, vp, ctypes.c_int, u64], i32),
        "tbg_sync": ([vp], i32),
        "tbg_read_device": ([vp, vp, vp, u64], i32),
        "tbg_stream": ([vp], vp),
        "tbg_setup_balances": ([vp, P(U128), P(U128), P(U128), P(U128), P(U128)], i32),
        "tbg_get_stats": ([vp, P(Stats)], i32),
        "tbg_dump_accounts": ([vp, vp, u64, P(u64)], i32),
        "tbg_dump_transfers": ([vp, vp, u64, P(u64)], i32),
        "tbg_dump_transfer_status": ([vp, vp, u64, P(u64)], i32),
        "tbg_device_stores": ([vp, P(vp), P(vp)], i32),
        "tbg_gen_accounts": ([vp, u64, u64, u64, u32, ctypes.c_uint16, ctypes.c_uint16, vp], i32),
        "tbg_gen_transfers_uniform": ([vp, u64, u64, u64, u64, u64, vp], i32),
        "tbg_gen_permute_ids": ([vp, u64, u32, u32, u64, vp], i32),
        "tbg_gen_mark_pending": ([vp, u64, u64, u64, u32, vp], i32),
        "tbg_version": ([], ctypes.c_char_p),
        "tbg_debug_last_batch": ([vp, vp, vp, u32], i32),
        "tbg_timing_enable": ([vp, ctypes.c_int], i32),
        "tbg_timing_collect": ([vp, vp, vp, u32], i32),
        "tbg_gen_accounts_cfg3": ([vp, u64, u64, u64, u64, u64, vp], i32),
        "tbg_gen_funding_cfg3": ([vp, u64, u64, u64, u64, u64, u64, u64, vp], i32),
        "tbg_gen_transfers_zipf": ([vp, u64, u64, u64, u64, vp, u64, vp], i32),
        "tbg_gen_transfers_cfg4": ([vp, u64, u64, u64, u64, u64, u64, vp], i32),
        "tbg_debug_counters": ([vp, vp, u32], i32),
        "tbg_debug_table_used": ([vp, P(u64), P(u64)], i32),
        "tbg_shard_of": ([u64, u64, u32], u32),
        "tbg_shard_prepare_window": ([vp, u32, vp, u32, vp, vp, vp], i32),
        "tbg_shard_commit_window": ([vp, vp, u32, u32, vp, vp], i32),
        "tbg_window_changes": ([vp, vp, u64, P(u64), vp, u64, P(u64), vp, u64, P(u64)], i32),
        "tbg_shard_exchange_bytes": ([u32, u32, u32], u64),
        "tbg_windows_committed": ([vp, P(u64), P(u64)], i32),
        "tbg_open": ([vp, vp, u64, vp, u64, vp, vp, u64], i32),
        "tbg_reset": ([vp], i32),
        "tbg_prefetch_poll": ([vp, P(ctypes.c_int)], i32),
        "tbg_compact": ([vp, u64], i32),
        "tbg_checkpoint": ([vp], i32),
        "tbg_digest": ([vp, P(u64)], i32),
        "tbg_commit_window_host": ([vp, u32, vp, u32, vp, vp, vp, vp, ctypes.c_int, u64, P(u64)], i32),
        "tbg_host_window_done": ([vp, u64, P(ctypes.c_int)], i32),
        "tbg_host_alloc": ([ctypes.c_size_t, P(vp)], i32),
        "tbg_host_free": ([vp], i32),
        "tbg_host_register": ([vp, ctypes.c_size_t], i32),
        "tbg_host_unregister": ([vp], i32),
        "tbg_checksum": ([vp, vp, vp, u32, vp, vp], i32),
        "tbg_demux_init": ([P(Demuxer), u32, vp, u32], i32),
        "tbg_demux_decode": ([P(Demuxer), u32, u32, P(vp), P(u32)], i32),
        "tbg_aof_replay": ([vp, vp, u64, u32, P(AofStats)], i32),
        "tbg_shard_gather_bytes": ([u32, u32, u32, P(u64)], u64),
        "tbg_shard_gather": ([vp, u32, vp, u32, u64, u32, vp], i32),
        "tbg_gw_collect": ([vp, u32, vp, u32, u64, u32, u32, vp, u32, vp, ctypes.c_int], i32),
        "tbg_gw_write": ([vp, u32, vp, vp, u64, vp, vp, u64, P(u32), P(u32), P(ctypes.c_int)], i32),
        "tbg_gw_commit": ([vp, vp, u32, vp, u32, vp, vp, vp, u64, vp, vp, vp, vp, ctypes.c_int, u64], i32),
        "tbg_gw_result": ([vp, vp, P(ctypes.c_int), P(u64)], i32),
        "tbg_shard_apply": ([vp, vp, u64, vp, vp, u64, vp, vp, u64], i32),
        "tbg_device_history": ([vp, P(vp), P(vp)], i32),
        "tbg_shard_lookup_bytes": ([u32], u64),
        "tbg_shard_lookup": ([vp, u32, vp, u64, vp], i32),
        "tbg_shard_lookup_reply": ([vp, vp, u64, vp, u64, P(u64)], i32),
        "tbg_shard_query_bytes": ([u32, u32], u64),
        "tbg_shard_query": ([vp, u32, vp, u64, vp], i32),
        "tbg_shard_query_merge": ([vp, u32, vp, vp, vp, u64, P(u64)], i32),
        "tbg_open_device": ([vp, vp, u64, vp, vp, u64, u64], i32),
        "tbg_device_state": ([vp, P(vp), P(u64), P(vp), P(vp), P(u64), P(u64)], i32),
        "tbg_route_prepare": ([vp, u32, vp, u32, vp, vp, vp], i32),
        "tbg_route_buffers": ([vp, u32, P(vp), vp, P(vp), vp], i32),
        "tbg_route_buffer_bytes": ([vp, vp], i32),
        "tbg_route_attach": ([vp, vp], i32),
        "tbg_route_own": ([vp], i32),
        "tbg_route_decide": ([vp], i32),
        "tbg_route_apply": ([vp, vp, vp], i32),
        "tbg_group_create": ([P(GroupConfig), P(vp)], i32),
        "tbg_group_destroy": ([vp], i32),
        "tbg_group_pulse_needed": ([vp, u64, P(ctypes.c_int)], i32),
        "tbg_group_prefetch": ([vp, u64, u32, vp, u64, u64], i32),
        "tbg_group_commit": ([vp, u64, u64, u32, vp, u64, vp, u64, P(u64)], i32),
        "tbg_group_commit_window": ([vp, u32, vp, u32, vp, vp, vp, vp], i32),
        "tbg_group_engine": ([vp, u32, P(vp)], i32),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


E_UNSUPPORTED = -5
E_WINDOW = -6


class UnsupportedWindow(RuntimeError):
    """A sharded engine rejected a window outside its class (nothing was applied)."""


class RejectedWindow(RuntimeError):
    """A commit window spanned a due pulse: it and every window queued after it were skipped whole
    (tbg_commit_window); resubmit them in smaller windows."""


def check(rc, what):
    if rc == E_UNSUPPORTED:
        raise UnsupportedWindow(f"{what}: window outside the sharded class (status {rc})")
    if rc == E_WINDOW:
        raise RejectedWindow(f"{what}: a window spanned a due pulse and was skipped whole (status {rc})")
    if rc != 0:
        raise RuntimeError(f"{what} failed with status {rc}")
