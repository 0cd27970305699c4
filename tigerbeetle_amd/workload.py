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


# ------------------------------------------------------------------------------------------------
# cfg3: Zipf hot accounts with debits_must_not_exceed_credits limits (see csrc/workload.hip).
# ------------------------------------------------------------------------------------------------
def zipf_cdf(n, s=1.2):
    """u64 thresholds: draw k = first index with cdf[k] > u for a uniform u64 u."""
    w = np.arange(1, n + 1, dtype=np.float64) ** (-s)
    c = np.cumsum(w)
    c /= c[-1]
    thr = (c * 2.0 ** 63).astype(np.uint64) << np.uint64(1)
    thr[-1] = np.uint64(0xFFFFFFFFFFFFFFFF)
    return thr


def zipf_draw(cdf, u):
    k = np.searchsorted(cdf, u, side="right")
    return np.minimum(k, len(cdf) - 1).astype(np.uint64)


def cfg3_limited(seed, r, limited_top):
    r = np.asarray(r, np.uint64)
    return (r < np.uint64(limited_top)) | ((rnd(seed, r, 7) & np.uint64(1)) == 1)


def accounts_cfg3(first, count, seed, n_accounts, limited_top):
    a = accounts(first, count, seed, ledger=2, code=1, flags=0)
    idx = np.arange(first, first + count, dtype=np.uint64)
    lim = cfg3_limited(seed, idx, limited_top) & (idx < np.uint64(n_accounts))
    a["flags"] = np.where(lim, 2, 0).astype(np.uint16)
    return a


def _common(t, seed, idx):
    t["user_data_128_lo"] = rnd(seed, idx, 14)
    t["user_data_128_hi"] = rnd(seed, idx, 15)
    t["user_data_64"] = rnd(seed, idx, 16)
    t["user_data_32"] = (rnd(seed, idx, 17) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    t["ledger"] = 2
    c = (rnd(seed, idx, 18) & np.uint64(0xFFFF)) + np.uint64(1)
    t["code"] = np.minimum(c, np.uint64(0xFFFF)).astype(np.uint16)


def funding_cfg3(first, count, seed, n_accounts, treasury, amount, id_offset):
    idx = np.arange(first, first + count, dtype=np.uint64)
    t = np.zeros(count, TRANSFER_DTYPE)
    t["id_lo"] = np.uint64(id_offset) + idx + np.uint64(1)
    t["debit_account_id_lo"] = np.uint64(n_accounts) + idx % np.uint64(treasury) + np.uint64(1)
    t["credit_account_id_lo"] = idx + np.uint64(1)
    t["amount_lo"] = np.uint64(amount)
    _common(t, seed, idx)
    return t


def transfers_zipf(first, count, seed, n_accounts, cdf, id_offset=0):
    idx = np.arange(first, first + count, dtype=np.uint64)
    n = np.uint64(n_accounts)
    dr = zipf_draw(cdf, rnd(seed, idx, 20))
    cr = zipf_draw(cdf, rnd(seed, idx, 21))
    cr = np.where(cr == dr, zipf_draw(cdf, rnd(seed, idx, 22)), cr)
    cr = np.where(cr == dr, (cr + np.uint64(1)) % n, cr)
    t = np.zeros(count, TRANSFER_DTYPE)
    t["id_lo"] = np.uint64(id_offset) + idx + np.uint64(1)
    t["debit_account_id_lo"] = dr + np.uint64(1)
    t["credit_account_id_lo"] = cr + np.uint64(1)
    t["amount_lo"] = amount(rnd(seed, idx, 12), rnd(seed, idx, 13))
    _common(t, seed, idx)
    return t


# ------------------------------------------------------------------------------------------------
# cfg4: two-phase + linked chains (see csrc/workload.hip).
# ------------------------------------------------------------------------------------------------
def cfg4_kind(seed, k):
    r = rnd(seed, k, 30) % np.uint64(100)
    return np.where(r < 30, 1, np.where(r < 50, 2, np.where(r < 60, 3, 0))).astype(np.int64)


def transfers_cfg4(first, count, seed, n_accounts, batch, id_offset=0):
    idx = np.arange(first, first + count, dtype=np.uint64)
    n = np.uint64(n_accounts)
    t = np.zeros(count, TRANSFER_DTYPE)
    t["id_lo"] = np.uint64(id_offset) + idx + np.uint64(1)
    _common(t, seed, idx)
    kind = cfg4_kind(seed, idx)
    back = np.uint64(1) + rnd(seed, idx, 31) % np.uint64(4 * batch)
    pv = (kind == 2) | (kind == 3)
    ok = pv & (back <= idx)
    j = np.where(ok, idx.astype(np.int64) - back.astype(np.int64), -1)
    target = np.full(count, -1, np.int64)
    for _ in range(64):
        live = ok & (target < 0) & (j >= 0)
        if not live.any():
            break
        kj = cfg4_kind(seed, np.maximum(j, 0).astype(np.uint64))
        hit = live & (kj == 1)
        target = np.where(hit, j, target)
        j = np.where(live & ~hit, j - 1, j)
    kind = np.where(pv & (target < 0), 0, kind)
    pv = (kind == 2) | (kind == 3)
    dr = rnd(seed, idx, 10) % n
    cr = rnd(seed, idx, 11) % n
    cr = np.where(cr == dr, (cr + np.uint64(1)) % n, cr)
    tgt = np.maximum(target, 0).astype(np.uint64)
    pa = amount(rnd(seed, tgt, 12), rnd(seed, tgt, 13))
    own = amount(rnd(seed, idx, 12), rnd(seed, idx, 13))
    r32 = rnd(seed, idx, 32)
    post_amt = r32 % (pa + np.uint64(1))
    void_amt = np.where((r32 & np.uint64(1)) == 1, pa, np.uint64(0))
    t["debit_account_id_lo"] = np.where(pv, 0, dr + np.uint64(1))
    t["credit_account_id_lo"] = np.where(pv, 0, cr + np.uint64(1))
    t["pending_id_lo"] = np.where(pv, np.uint64(id_offset) + tgt + np.uint64(1), 0)
    t["ledger"] = np.where(pv, 0, 2)
    t["code"] = np.where(pv, 0, t["code"])
    t["amount_lo"] = np.where(kind == 2, post_amt, np.where(kind == 3, void_amt, own))
    flags = np.where(kind == 1, 2, np.where(kind == 2, 4, np.where(kind == 3, 8, 0))).astype(np.uint16)
    t["timeout"] = np.where(kind == 1, (np.uint64(1) + rnd(seed, idx, 33) % np.uint64(60)), 0).astype(np.uint32)
    # chains
    slot = idx // np.uint64(8)
    pos = idx % np.uint64(8)
    chain = (rnd(seed, slot, 40) % np.uint64(100)) < np.uint64(16)
    L = np.uint64(2) + rnd(seed, slot, 41) % np.uint64(7)
    member = chain & (pos < L)
    flags = np.where(member & (pos + np.uint64(1) < L), flags | 1, flags).astype(np.uint16)
    inject = member & ((rnd(seed, slot, 42) % np.uint64(4)) == 0) & (pos == rnd(seed, slot, 43) % L)
    inj_pv = inject & pv
    inj_cr = inject & ~pv
    t["pending_id_lo"] = np.where(inj_pv, np.uint64(0xFFFFFFFFFFFFFFFF), t["pending_id_lo"])
    t["pending_id_hi"] = np.where(inj_pv, np.uint64(0xFFFFFFFFFFFFFFFF), 0)
    t["credit_account_id_lo"] = np.where(inj_cr, t["debit_account_id_lo"], t["credit_account_id_lo"])
    t["flags"] = flags
    return t


# ------------------------------------------------------------------------------------------------
# Id orders of `tigerbeetle benchmark --id-order` (csrc/workload.hip k_permute_ids): the reference's
# IdPermutation.encode (testing/id.zig:8-48) with Zig std's DefaultPrng (Xoshiro256++, SplitMix64
# seeding).
# ------------------------------------------------------------------------------------------------
ID_ORDERS = {"sequential": 0, "random": 1, "reversed": 2, "time": 3}
TIME_BASE_MS = 1700000000000
TIME_PER_MS_LOG2 = 18
_M64 = (1 << 64) - 1


def _splitmix_seed(z):
    """The four Xoshiro256 state words of DefaultPrng.init(z) (uint64 arrays)."""
    out = []
    with np.errstate(over="ignore"):
        for _ in range(4):
            z = z + np.uint64(0x9E3779B97F4A7C15)
            x = z
            x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            out.append(x ^ (x >> np.uint64(31)))
    return out


def _rotl(x, k):
    return (x << np.uint64(k)) | (x >> np.uint64(64 - k))


def _xoshiro_next(s):
    with np.errstate(over="ignore"):
        r = _rotl(s[0] + s[3], 23) + s[0]
        t = s[1] << np.uint64(17)
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = _rotl(s[3], 45)
    return r


def benchmark_permutation_seed(seed):
    """The random IdPermutation's seed the reference benchmark draws: DefaultPrng.init(seed), first
    random.int(u64) (benchmark_load.zig:120-125)."""
    s = _splitmix_seed(np.array([seed], np.uint64))
    return int(_xoshiro_next(s)[0])


def encode_ids(data, order, seed=0):
    """IdPermutation.encode(data) for uint64 `data` (> 0): (lo, hi) uint64 arrays."""
    data = np.asarray(data, np.uint64)
    if order == 0:
        return data.copy(), np.zeros_like(data)
    if order == 2:
        return ~data, np.full_like(data, np.uint64(_M64))
    if order == 3:  # time-based ids (workload.hip wl_encode_id)
        with np.errstate(over="ignore"):
            d1 = data - np.uint64(1)
            ms = np.uint64(TIME_BASE_MS) + (d1 >> np.uint64(TIME_PER_MS_LOG2))
            k = d1 & np.uint64((1 << TIME_PER_MS_LOG2) - 1)
            r_lo = rnd(seed, ms, 7)
            r_hi = rnd(seed, ms, 8) & np.uint64(0x7FFF)
            lo = r_lo + k
            hi = (ms << np.uint64(16)) | (r_hi + (lo < r_lo).astype(np.uint64))
        return lo, hi
    with np.errstate(over="ignore"):
        s = _splitmix_seed(data + np.uint64(seed))
    r0 = _xoshiro_next(s)
    r1 = _xoshiro_next(s)
    lo = (data << np.uint64(32)) | (r0 & np.uint64(0xFFFFFFFF))
    hi = (data >> np.uint64(32)) | (r1 & np.uint64(0xFFFFFFFF00000000))
    return lo, hi


def permute_ids(recs, order, seed=0):
    """Numpy twin of tbg_gen_permute_ids: records generated with sequential ids, rewritten in place
    (accounts: id; transfers: id, debit and credit account ids, pending_id; 0 and ids >= 2^64
    stay)."""
    if order == 0:
        return recs
    fields = ["id"] + (["debit_account_id", "credit_account_id", "pending_id"]
                       if "debit_account_id_lo" in recs.dtype.names else [])
    for f in fields:
        lo, hi = recs[f + "_lo"], recs[f + "_hi"]
        m = (hi == 0) & (lo != 0)
        elo, ehi = encode_ids(lo, order, seed)
        recs[f + "_lo"] = np.where(m, elo, lo)
        recs[f + "_hi"] = np.where(m, ehi, hi)
    return recs


def mark_pending(recs, first, every, timeout):
    """Numpy twin of tbg_gen_mark_pending: transfer (first + k) with (first + k) % every == every - 1
    becomes a pending create with `timeout` seconds."""
    if every:
        k = np.arange(first, first + len(recs), dtype=np.uint64)
        m = k % np.uint64(every) == np.uint64(every - 1)
        recs["timeout"][m] = timeout
        recs["flags"][m] |= np.uint16(1 << 1)
    return recs
