// workload.hip — deterministic synthetic request streams, generated on the device.
//
// Shapes follow the reference benchmark (src/tigerbeetle/benchmark_load.zig:206-327): accounts with
// sequential ids 1..N (IdPermutation.identity, testing/id.zig:30), ledger 2, code 1; transfers with
// id = index + 1, uniform debit/credit account (credit bumped by one on a collision, :287-291),
// ledger 2, code = rand_u16 +| 1, amount exponential-like with mean ~10^4 (:312). The reference's
// Xoshiro stream is not reproducible here (parity unpinned at the generator); this one is a
// counter-based splitmix hash, mirrored bit-for-bit by tigerbeetle_amd/workload.py so CPU-side
// tests can rebuild any slice of a stream without the device.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tb_types.h"

__host__ __device__ inline uint64_t wl_rnd(uint64_t seed, uint64_t idx, uint64_t lane) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + idx * 0xD1B54A32D192ED03ull + lane * 0xAEF17502108EF2D9ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Exponential-like amount with mean ~10^4 using integers only: (G + U) * ln2 * 10^4 where G is
// geometric(1/2) from the leading zeros of one draw and U a 16-bit uniform fraction.
__host__ __device__ inline uint64_t wl_amount(uint64_t r0, uint64_t r1) {
  uint64_t x = r0 | 1ull;
  uint64_t g = 0;
  while (!(x >> 63)) {
    x <<= 1;
    g++;
  }
  const uint64_t frac = r1 & 0xFFFFull;
  return 1 + (((g << 16) | frac) * 6931ull >> 16);
}

__global__ void k_gen_accounts(tb_account_t* out, uint64_t first, uint64_t count, uint64_t seed, uint32_t ledger,
                               uint16_t code, uint16_t flags) {
  const uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (k >= count) return;
  const uint64_t idx = first + k;
  tb_account_t a;
  a.id.lo = idx + 1;
  a.id.hi = 0;
  a.debits_pending = {0, 0};
  a.debits_posted = {0, 0};
  a.credits_pending = {0, 0};
  a.credits_posted = {0, 0};
  a.user_data_128.lo = wl_rnd(seed, idx, 0);
  a.user_data_128.hi = wl_rnd(seed, idx, 1);
  a.user_data_64 = wl_rnd(seed, idx, 2);
  a.user_data_32 = (uint32_t)wl_rnd(seed, idx, 3);
  a.reserved = 0;
  a.ledger = ledger;
  a.code = code;
  a.flags = flags;
  a.timestamp = 0;
  out[k] = a;
}

__global__ void k_gen_transfers_uniform(tb_transfer_t* out, uint64_t first, uint64_t count, uint64_t seed,
                                        uint64_t n_accounts, uint64_t id_offset) {
  const uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (k >= count) return;
  const uint64_t idx = first + k;
  const uint64_t dr = wl_rnd(seed, idx, 10) % n_accounts;
  uint64_t cr = wl_rnd(seed, idx, 11) % n_accounts;
  if (cr == dr) cr = (cr + 1) % n_accounts;
  tb_transfer_t t;
  t.id.lo = id_offset + idx + 1;
  t.id.hi = 0;
  t.debit_account_id.lo = dr + 1;
  t.debit_account_id.hi = 0;
  t.credit_account_id.lo = cr + 1;
  t.credit_account_id.hi = 0;
  t.amount.lo = wl_amount(wl_rnd(seed, idx, 12), wl_rnd(seed, idx, 13));
  t.amount.hi = 0;
  t.pending_id = {0, 0};
  t.user_data_128.lo = wl_rnd(seed, idx, 14);
  t.user_data_128.hi = wl_rnd(seed, idx, 15);
  t.user_data_64 = wl_rnd(seed, idx, 16);
  t.user_data_32 = (uint32_t)wl_rnd(seed, idx, 17);
  t.timeout = 0;
  t.ledger = 2;
  const uint32_t c = (uint32_t)(wl_rnd(seed, idx, 18) & 0xFFFF) + 1;
  t.code = (uint16_t)(c > 0xFFFF ? 0xFFFF : c);
  t.flags = 0;
  t.timestamp = 0;
  out[k] = t;
}

extern "C" int tbg_gen_accounts(void* d_out, uint64_t first, uint64_t count, uint64_t seed, uint32_t ledger,
                                uint16_t code, uint16_t flags, void* stream) {
  if (!count) return 0;
  k_gen_accounts<<<(unsigned)((count + 255) / 256), 256, 0, (hipStream_t)stream>>>((tb_account_t*)d_out, first, count,
                                                                                  seed, ledger, code, flags);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int tbg_gen_transfers_uniform(void* d_out, uint64_t first, uint64_t count, uint64_t seed,
                                         uint64_t n_accounts, uint64_t id_offset, void* stream) {
  if (!count) return 0;
  k_gen_transfers_uniform<<<(unsigned)((count + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      (tb_transfer_t*)d_out, first, count, seed, n_accounts, id_offset);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// ------------------------------------------------------------------------------------------------
// cfg3: Zipf(s) hot accounts with debits_must_not_exceed_credits limits.
//   accounts: rank r (id r+1) is limited iff r < limited_top or bit 0 of rnd(seed, r, 7) is set;
//             treasury accounts (ids n_accounts+1 .. n_accounts+treasury) are unlimited.
//   funding:  transfer k (k < n_accounts) credits account k from treasury account k % treasury.
//   stream:   debit and credit ranks drawn from the Zipf table (u64 CDF thresholds, shared by the
//             device and numpy generators); an equal credit is redrawn once, then bumped by one.
// ------------------------------------------------------------------------------------------------
__host__ __device__ inline bool cfg3_limited(uint64_t seed, uint64_t r, uint64_t limited_top) {
  return r < limited_top || (wl_rnd(seed, r, 7) & 1);
}

__device__ inline uint64_t zipf_draw(const uint64_t* cdf, uint64_t n, uint64_t u) {
  // first k with cdf[k] > u
  uint64_t lo = 0, hi = n - 1;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (cdf[mid] > u)
      hi = mid;
    else
      lo = mid + 1;
  }
  return lo;
}

__global__ void k_gen_accounts_cfg3(tb_account_t* out, uint64_t first, uint64_t count, uint64_t seed,
                                    uint64_t n_accounts, uint64_t limited_top) {
  const uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (k >= count) return;
  const uint64_t idx = first + k;
  tb_account_t a;
  a.id.lo = idx + 1;
  a.id.hi = 0;
  a.debits_pending = {0, 0};
  a.debits_posted = {0, 0};
  a.credits_pending = {0, 0};
  a.credits_posted = {0, 0};
  a.user_data_128.lo = wl_rnd(seed, idx, 0);
  a.user_data_128.hi = wl_rnd(seed, idx, 1);
  a.user_data_64 = wl_rnd(seed, idx, 2);
  a.user_data_32 = (uint32_t)wl_rnd(seed, idx, 3);
  a.reserved = 0;
  a.ledger = 2;
  a.code = 1;
  a.flags = (idx < n_accounts && cfg3_limited(seed, idx, limited_top)) ? TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS : 0;
  a.timestamp = 0;
  out[k] = a;
}

__device__ inline void wl_fill_common(tb_transfer_t& t, uint64_t seed, uint64_t idx) {
  t.pending_id = {0, 0};
  t.user_data_128.lo = wl_rnd(seed, idx, 14);
  t.user_data_128.hi = wl_rnd(seed, idx, 15);
  t.user_data_64 = wl_rnd(seed, idx, 16);
  t.user_data_32 = (uint32_t)wl_rnd(seed, idx, 17);
  t.timeout = 0;
  t.ledger = 2;
  const uint32_t c = (uint32_t)(wl_rnd(seed, idx, 18) & 0xFFFF) + 1;
  t.code = (uint16_t)(c > 0xFFFF ? 0xFFFF : c);
  t.flags = 0;
  t.timestamp = 0;
}

__global__ void k_gen_funding_cfg3(tb_transfer_t* out, uint64_t first, uint64_t count, uint64_t seed,
                                   uint64_t n_accounts, uint64_t treasury, uint64_t amount, uint64_t id_offset) {
  const uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (k >= count) return;
  const uint64_t idx = first + k;
  tb_transfer_t t;
  t.id.lo = id_offset + idx + 1;
  t.id.hi = 0;
  t.debit_account_id.lo = n_accounts + (idx % treasury) + 1;
  t.debit_account_id.hi = 0;
  t.credit_account_id.lo = idx + 1;
  t.credit_account_id.hi = 0;
  t.amount.lo = amount;
  t.amount.hi = 0;
  wl_fill_common(t, seed, idx);
  out[k] = t;
}

__global__ void k_gen_transfers_zipf(tb_transfer_t* out, uint64_t first, uint64_t count, uint64_t seed,
                                     uint64_t n_accounts, const uint64_t* cdf, uint64_t id_offset) {
  const uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (k >= count) return;
  const uint64_t idx = first + k;
  const uint64_t dr = zipf_draw(cdf, n_accounts, wl_rnd(seed, idx, 20));
  uint64_t cr = zipf_draw(cdf, n_accounts, wl_rnd(seed, idx, 21));
  if (cr == dr) cr = zipf_draw(cdf, n_accounts, wl_rnd(seed, idx, 22));
  if (cr == dr) cr = (cr + 1) % n_accounts;
  tb_transfer_t t;
  t.id.lo = id_offset + idx + 1;
  t.id.hi = 0;
  t.debit_account_id.lo = dr + 1;
  t.debit_account_id.hi = 0;
  t.credit_account_id.lo = cr + 1;
  t.credit_account_id.hi = 0;
  t.amount.lo = wl_amount(wl_rnd(seed, idx, 12), wl_rnd(seed, idx, 13));
  t.amount.hi = 0;
  wl_fill_common(t, seed, idx);
  out[k] = t;
}

// ------------------------------------------------------------------------------------------------
// cfg4: two-phase + linked chains.
//   kind(k) by rnd(k, 30) % 100: < 30 pending (timeout 1..60 s), < 50 post, < 60 void, else posted.
//   post/void target: walk back from k - (1 + rnd(k, 31) % (4 * batch)) to the nearest pending-kind
//     event (at most 64 steps; none found -> plain transfer). post amount U[0, p.amount] (0 = full),
//     void amount 0 or p.amount.
//   chains: slot s = k / 8 hosts a chain when rnd(s, 40) % 100 < 16, of length L = 2 + rnd(s, 41) % 7,
//     linked on its first L-1 events; a quarter of the chains get one injected failure (member
//     rnd(s, 43) % L: debit == credit for creates, pending_id = u128 max for post/void).
// ------------------------------------------------------------------------------------------------
__host__ __device__ inline uint32_t cfg4_kind(uint64_t seed, uint64_t k) {
  const uint32_t r = (uint32_t)(wl_rnd(seed, k, 30) % 100);
  return r < 30 ? 1u : r < 50 ? 2u : r < 60 ? 3u : 0u;  // 1 pending, 2 post, 3 void, 0 posted
}

__host__ __device__ inline uint64_t cfg4_amount(uint64_t seed, uint64_t k) {
  return wl_amount(wl_rnd(seed, k, 12), wl_rnd(seed, k, 13));
}

__global__ void k_gen_transfers_cfg4(tb_transfer_t* out, uint64_t first, uint64_t count, uint64_t seed,
                                     uint64_t n_accounts, uint64_t batch, uint64_t id_offset) {
  const uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (k >= count) return;
  const uint64_t idx = first + k;
  tb_transfer_t t;
  t.id.lo = id_offset + idx + 1;
  t.id.hi = 0;
  wl_fill_common(t, seed, idx);
  uint32_t kind = cfg4_kind(seed, idx);
  int64_t target = -1;
  if (kind == 2 || kind == 3) {
    const uint64_t back = 1 + wl_rnd(seed, idx, 31) % (4 * batch);
    if (back <= idx) {
      int64_t j = (int64_t)(idx - back);
      for (int step = 0; step < 64 && j >= 0; step++, j--) {
        if (cfg4_kind(seed, (uint64_t)j) == 1) {
          target = j;
          break;
        }
      }
    }
    if (target < 0) kind = 0;
  }
  const uint64_t dr = wl_rnd(seed, idx, 10) % n_accounts;
  uint64_t cr = wl_rnd(seed, idx, 11) % n_accounts;
  if (cr == dr) cr = (cr + 1) % n_accounts;
  if (kind == 2 || kind == 3) {
    const uint64_t pa = cfg4_amount(seed, (uint64_t)target);
    t.debit_account_id = {0, 0};
    t.credit_account_id = {0, 0};
    t.pending_id.lo = id_offset + (uint64_t)target + 1;
    t.pending_id.hi = 0;
    t.ledger = 0;
    t.code = 0;
    if (kind == 2) {
      t.flags = TB_TRANSFER_POST_PENDING;
      t.amount.lo = wl_rnd(seed, idx, 32) % (pa + 1);
    } else {
      t.flags = TB_TRANSFER_VOID_PENDING;
      t.amount.lo = (wl_rnd(seed, idx, 32) & 1) ? pa : 0;
    }
    t.amount.hi = 0;
  } else {
    t.debit_account_id.lo = dr + 1;
    t.debit_account_id.hi = 0;
    t.credit_account_id.lo = cr + 1;
    t.credit_account_id.hi = 0;
    t.amount.lo = cfg4_amount(seed, idx);
    t.amount.hi = 0;
    if (kind == 1) {
      t.flags = TB_TRANSFER_PENDING;
      t.timeout = 1 + (uint32_t)(wl_rnd(seed, idx, 33) % 60);
    }
  }
  // chains
  const uint64_t slot = idx / 8, pos = idx % 8;
  if (wl_rnd(seed, slot, 40) % 100 < 16) {
    const uint64_t L = 2 + wl_rnd(seed, slot, 41) % 7;
    if (pos < L) {
      if (pos + 1 < L) t.flags |= TB_TRANSFER_LINKED;
      if (wl_rnd(seed, slot, 42) % 4 == 0 && pos == wl_rnd(seed, slot, 43) % L) {
        if (t.flags & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) {
          t.pending_id.lo = ~0ull;
          t.pending_id.hi = ~0ull;
        } else {
          t.credit_account_id = t.debit_account_id;
        }
      }
    }
  }
  out[k] = t;
}

#define WL_GRID(count) (unsigned)(((count) + 255) / 256), 256

extern "C" int tbg_gen_accounts_cfg3(void* d_out, uint64_t first, uint64_t count, uint64_t seed, uint64_t n_accounts,
                                     uint64_t limited_top, void* stream) {
  if (!count) return 0;
  k_gen_accounts_cfg3<<<WL_GRID(count), 0, (hipStream_t)stream>>>((tb_account_t*)d_out, first, count, seed,
                                                                  n_accounts, limited_top);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int tbg_gen_funding_cfg3(void* d_out, uint64_t first, uint64_t count, uint64_t seed, uint64_t n_accounts,
                                    uint64_t treasury, uint64_t amount, uint64_t id_offset, void* stream) {
  if (!count) return 0;
  k_gen_funding_cfg3<<<WL_GRID(count), 0, (hipStream_t)stream>>>((tb_transfer_t*)d_out, first, count, seed,
                                                                 n_accounts, treasury, amount, id_offset);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int tbg_gen_transfers_zipf(void* d_out, uint64_t first, uint64_t count, uint64_t seed, uint64_t n_accounts,
                                      const void* d_cdf, uint64_t id_offset, void* stream) {
  if (!count) return 0;
  k_gen_transfers_zipf<<<WL_GRID(count), 0, (hipStream_t)stream>>>((tb_transfer_t*)d_out, first, count, seed,
                                                                   n_accounts, (const uint64_t*)d_cdf, id_offset);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int tbg_gen_transfers_cfg4(void* d_out, uint64_t first, uint64_t count, uint64_t seed, uint64_t n_accounts,
                                      uint64_t batch, uint64_t id_offset, void* stream) {
  if (!count) return 0;
  k_gen_transfers_cfg4<<<WL_GRID(count), 0, (hipStream_t)stream>>>((tb_transfer_t*)d_out, first, count, seed,
                                                                   n_accounts, batch, id_offset);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// ------------------------------------------------------------------------------------------------
// Id orders of the reference benchmark (`tigerbeetle benchmark --id-order`, cli.zig:97, 263-265;
// benchmark_load.zig:122-126, 222, 292-300): every account id and transfer id is
// IdPermutation.encode(index + 1) (testing/id.zig:8-48):
//   sequential  identity:  data
//   reversed    inversion: maxInt(u128) - data
//   random      pseudo-UUID: data << 32 | (Xoshiro256(seed +% data).int(u128) & ~(maxInt(u64) << 32))
// plus one order the reference benchmark does not have but its docs recommend for every application
// (docs/develop/data-modeling.md:186-203, the clients' id()):
//   time        48-bit millisecond timestamp above 80 random bits, the random part incremented for
//               the ids of the same millisecond: strictly increasing 128-bit ids whose high word is
//               never zero. The stream's clock advances one millisecond every 2^18 ids (about the
//               rate of the fused pass); each millisecond draws a fresh random part (below 2^79, so
//               the increments never carry into the timestamp).
// Zig std's DefaultPrng is Xoshiro256++ seeded through SplitMix64, and Random.int(u128) reads two
// next() words little-endian, so the ids are the reference's own for the same permutation seed
// (benchmark_load.zig:120-125 draws it as the first u64 of DefaultPrng.init(seed)).
// k_permute_ids rewrites, in place, the ids of records generated with sequential ids (data = the
// stored low word): an account's id; a transfer's id, debit and credit account ids and pending_id
// (one bijection for all, so a stream keeps its outcomes under any order).
// ------------------------------------------------------------------------------------------------
__host__ __device__ inline uint64_t wl_rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

#define WL_TIME_BASE_MS 1700000000000ull  // (2023-11-14, 48 bits)
#define WL_TIME_PER_MS_LOG2 18

__host__ __device__ inline tb_uint128_t wl_encode_id(uint64_t data, uint32_t order, uint64_t seed) {
  tb_uint128_t id;
  if (order == 1) {
    uint64_t s[4], z = seed + data;  // DefaultPrng.init(seed +% data): SplitMix64 seeding
    for (int k = 0; k < 4; k++) {
      z += 0x9e3779b97f4a7c15ull;
      uint64_t x = z;
      x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
      x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
      s[k] = x ^ (x >> 31);
    }
    uint64_t r[2];
    for (int k = 0; k < 2; k++) {  // xoshiro256++ next()
      r[k] = wl_rotl(s[0] + s[3], 23) + s[0];
      const uint64_t t = s[1] << 17;
      s[2] ^= s[0];
      s[3] ^= s[1];
      s[1] ^= s[2];
      s[0] ^= s[3];
      s[2] ^= t;
      s[3] = wl_rotl(s[3], 45);
    }
    id.lo = (data << 32) | (r[0] & 0xFFFFFFFFull);
    id.hi = (data >> 32) | (r[1] & 0xFFFFFFFF00000000ull);
  } else if (order == 2) {
    id.lo = ~data;
    id.hi = ~0ull;
  } else if (order == 3) {
    const uint64_t ms = WL_TIME_BASE_MS + ((data - 1) >> WL_TIME_PER_MS_LOG2);
    const uint64_t k = (data - 1) & ((1ull << WL_TIME_PER_MS_LOG2) - 1);
    const uint64_t r_lo = wl_rnd(seed, ms, 7), r_hi = wl_rnd(seed, ms, 8) & 0x7FFFull;
    id.lo = r_lo + k;
    id.hi = (ms << 16) | (r_hi + (id.lo < r_lo ? 1ull : 0ull));
  } else {
    id.lo = data;
    id.hi = 0;
  }
  return id;
}

__global__ void k_permute_ids(uint8_t* recs, uint64_t count, uint32_t transfers, uint32_t order, uint64_t seed) {
  const uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (k >= count) return;
  tb_uint128_t* r = reinterpret_cast<tb_uint128_t*>(recs + k * 128);
  // id (0); transfers: debit_account_id (1), credit_account_id (2), pending_id (4)
  const int fields[4] = {0, 1, 2, 4};
  const int n = transfers ? 4 : 1;
  for (int j = 0; j < n; j++) {
    tb_uint128_t& v = r[fields[j]];
    if (v.hi == 0 && v.lo != 0) v = wl_encode_id(v.lo, order, seed);  // 0 and ids >= 2^64 stay
  }
}

extern "C" int tbg_gen_permute_ids(void* d_records, uint64_t count, uint32_t transfers, uint32_t order, uint64_t seed,
                                   void* stream) {
  if (order > 3) return -1;
  if (!count || order == 0) return 0;
  k_permute_ids<<<(unsigned)((count + 255) / 256), 256, 0, (hipStream_t)stream>>>((uint8_t*)d_records, count,
                                                                                transfers, order, seed);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Mixed streams: every `every`-th generated transfer (global index first + k with (first + k) % every ==
// every - 1) becomes a pending create (flags.pending, timeout `timeout` seconds); the rest are untouched.
__global__ void k_mark_pending(uint8_t* recs, uint64_t first, uint64_t count, uint64_t every, uint32_t timeout) {
  const uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (k >= count || (first + k) % every != every - 1) return;
  uint8_t* r = recs + k * 128;
  *reinterpret_cast<uint32_t*>(r + 108) = timeout;
  *reinterpret_cast<uint16_t*>(r + 118) |= (uint16_t)(1u << 1);
}

extern "C" int tbg_gen_mark_pending(void* d_records, uint64_t first, uint64_t count, uint64_t every, uint32_t timeout,
                                    void* stream) {
  if (!count || !every) return 0;
  k_mark_pending<<<(unsigned)((count + 255) / 256), 256, 0, (hipStream_t)stream>>>((uint8_t*)d_records, first, count,
                                                                                 every, timeout);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
