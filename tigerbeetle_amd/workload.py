"""Deterministic synthetic streams (numpy twin of csrc/workload.hip, bit-identical).

Shapes follow src/tigerbeetle/benchmark_load.zig:206-327 (see workload.hip's header). Used by the
CPU-side tests to rebuild any slice of a stream, and by the GPU tests to check the device generator.
"""
import numpy as np

from .types import ACCOUNT_DTYPE, TRANSFER_DTYPE

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def rnd(seed, idx, lane):
    with np.errstate(over="ignore"):
        z = (np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15)
             + np.asarray(idx, np.uint64) * np.uint64(0xD1B54A32D192ED03)
             + np.uint64(lane) * np.uint64(0xAEF17502108EF2D9))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def amount(r0, r1):
    x = r0 | np.uint64(1)
    # leading zeros of a nonzero u64
    g = np.zeros(x.shape, np.uint64)
    for b in (32, 16, 8, 4, 2, 1):
        m = (x >> np.uint64(64 - b)) == 0
        g = np.where(m, g + np.uint64(b), g)
        x = np.where(m, x << np.uint64(b), x)
    frac = r1 & np.uint64(0xFFFF)
    with np.errstate(over="ignore"):
        return np.uint64(1) + ((((g << np.uint64(16)) | frac) * np.uint64(6931)) >> np.uint64(16))


def accounts(first, count, seed, ledger=2, code=1, flags=0):
    idx = np.arange(first, first + count, dtype=np.uint64)
    a = np.zeros(count, ACCOUNT_DTYPE)
    a["id_lo"] = idx + np.uint64(1)
    a["user_data_128_lo"] = rnd(seed, idx, 0)
    a["user_data_128_hi"] = rnd(seed, idx, 1)
    a["user_data_64"] = rnd(seed, idx, 2)
    a["user_data_32"] = (rnd(seed, idx, 3) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    a["ledger"] = ledger
    a["code"] = code
    a["flags"] = flags
    return a


def transfers_uniform(first, count, seed, n_accounts, id_offset=0):
    idx = np.arange(first, first + count, dtype=np.uint64)
    n = np.uint64(n_accounts)
    dr = rnd(seed, idx, 10) % n
    cr = rnd(seed, idx, 11) % n
    cr = np.where(cr == dr, (cr + np.uint64(1)) % n, cr)
    t = np.zeros(count, TRANSFER_DTYPE)
    t["id_lo"] = np.uint64(id_offset) + idx + np.uint64(1)
    t["debit_account_id_lo"] = dr + np.uint64(1)
    t["credit_account_id_lo"] = cr + np.uint64(1)
    t["amount_lo"] = amount(rnd(seed, idx, 12), rnd(seed, idx, 13))
    t["user_data_128_lo"] = rnd(seed, idx, 14)
    t["user_data_128_hi"] = rnd(seed, idx, 15)
    t["user_data_64"] = rnd(seed, idx, 16)
    t["user_data_32"] = (rnd(seed, idx, 17) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    t["ledger"] = 2
    c = (rnd(seed, idx, 18) & np.uint64(0xFFFF)) + np.uint64(1)
    t["code"] = np.minimum(c, np.uint64(0xFFFF)).astype(np.uint16)
    return t
