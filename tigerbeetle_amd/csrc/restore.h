// restore.h — engine state from the LSM forest's objects (StateMachine.open after a restart or a
// state sync, state_machine.zig:527-541, 486-501) and the whole-state digest.
//
// open: the grooves hold every Account and Transfer object and every TransferPending row; the
// engine is rebuilt from them in timestamp order (= its dense store order): the records are copied
// into the stores, the id tables are rebuilt, the TransferPending status lands per transfer slot,
// and the live expires_at list is every pending transfer with a scan-visible timeout
// (state_machine.zig:229-238, lsm/composite_key.zig:47-49). pulse_next_timestamp starts at
// timestamp_min as in a freshly initialised StateMachine (:2063): the first pulse scans.
#pragma once
#include "window.h"

// Upper bound of every balance sum (dp + dpo, cp + cpo) of the loaded accounts: max of the high
// words (with a saturation flag) and max of the low words among sums below 2^64 (ovf_bound only has
// to be >= every sum; a looser bound only sends more windows down the exact overflow path).
struct LoadBound {
  unsigned long long hi_max;  // max high word of any sum; ~0 = a sum wrapped 128 bits
  unsigned long long lo_max;  // max of the sums that fit 64 bits
};

__global__ void __launch_bounds__(256) k_load_accounts(Dev d, uint64_t first, uint64_t n, LoadBound* lb) {
  for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t slot = first + k;
    const tb_account_t a = d.acc[slot];
    acc_insert(d.acc_tab, d.acc_mask, a.id, (uint32_t)slot, a.ledger, a.flags);
    d.hot[slot] = 0;
    if (a.flags & (TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS | TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS))
      atomicAdd(reinterpret_cast<unsigned long long*>(&d.g->limited_accounts), 1ull);
    const u128 dp = U(a.debits_pending), cp = U(a.credits_pending);
    const u128 s1 = dp + U(a.debits_posted), s2 = cp + U(a.credits_posted);
    const bool sat = s1 < dp || s2 < cp;
    const u128 m = s1 > s2 ? s1 : s2;
    const unsigned long long hi = sat ? ~0ull : (unsigned long long)(m >> 64);
    if (hi) atomicMax(&lb->hi_max, hi);
    else atomicMax(&lb->lo_max, (unsigned long long)m);
  }
}

// Exact bounds on the stored ids (Globals::x_id_max) from the rare bulk paths (open, the sharded
// general path's applies): each block of a grid of at most IDMAX_BLOCKS 256-thread blocks stores its
// maximum, and the one-block finishing kernel folds them (a word-wise pair of 64-bit atomics would
// give (max hi, max lo): far above the true maximum with time-based ids, whose low words are random).
#define IDMAX_BLOCKS 4096u
__device__ inline void block_idmax_out(u128 v, u128* out) {
  __shared__ u128 l[4];
  v = wave_max_u128(v);
  if ((threadIdx.x & 63) == 0) l[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = umax128(umax128(l[0], l[1]), umax128(l[2], l[3]));
}
// The maximum of nblk block maxima, in thread 0 of a 256-thread block (every thread calls it).
__device__ inline u128 fold_idmax(const u128* in, uint32_t nblk) {
  __shared__ u128 l[4];
  u128 m = 0;
  for (uint32_t j = threadIdx.x; j < nblk; j += 256) m = umax128(m, in[j]);
  m = wave_max_u128(m);
  if ((threadIdx.x & 63) == 0) l[threadIdx.x >> 6] = m;
  __syncthreads();
  return umax128(umax128(l[0], l[1]), umax128(l[2], l[3]));
}

__global__ void __launch_bounds__(256) k_load_transfers(Dev d, uint64_t first, uint64_t n, u128* idmax) {
  u128 m = 0;
  for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t slot = first + k;
    const tb_transfer_t t = d.xr[slot];
    x_insert(d.x_tab, d.x_mask, t.id, (uint32_t)slot);
    m = umax128(m, U(t.id));
    if (!(t.flags & TB_TRANSFER_PENDING) || t.timeout == 0 || d.xstatus[slot] != TB_PENDING_PENDING) continue;
    const uint64_t expires_at = expires_at_of(t);
    if ((t.timestamp >> 63) || expires_at > TB_TIMESTAMP_MAX) continue;  // never visible to the scan
    ExpEntry e;
    e.expires_at = expires_at;
    e.slot = (uint32_t)slot;
    e.pad = 0;
    const uint64_t q = atomicAdd(reinterpret_cast<unsigned long long*>(&d.g->exp_count), 1ull);
    d.exp[*d.exp_cur][q] = e;
  }
  block_idmax_out(m, idmax);
}

// The account_balances groove's rows (sorted by timestamp): each lands on the slot of the transfer
// with its timestamp (binary search over the timestamp-ordered store).
__global__ void __launch_bounds__(256) k_load_history(Dev d, const tb_account_balances_value_t* rows, uint64_t n,
                                                      uint64_t n_x) {
  for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x) {
    const tb_account_balances_value_t r = rows[k];
    uint64_t a = 0, b = n_x;
    while (a < b) {
      const uint64_t m = (a + b) >> 1;
      if (d.xr[m].timestamp < r.timestamp) a = m + 1; else b = m;
    }
    if (a >= n_x || d.xr[a].timestamp != r.timestamp) continue;  // no such transfer: not a row of ours
    HistRow h;
    h.dr[0] = U(r.dr_debits_pending), h.dr[1] = U(r.dr_debits_posted);
    h.dr[2] = U(r.dr_credits_pending), h.dr[3] = U(r.dr_credits_posted);
    h.cr[0] = U(r.cr_debits_pending), h.cr[1] = U(r.cr_debits_posted);
    h.cr[2] = U(r.cr_credits_pending), h.cr[3] = U(r.cr_credits_posted);
    d.hist[a] = h;
    d.hist_side[a] = (U(r.dr_account_id) != 0 ? 1u : 0u) | (U(r.cr_account_id) != 0 ? 2u : 0u);
  }
}

__global__ void __launch_bounds__(256) k_load_finish(Dev d, const LoadBound* lb, uint64_t n_acc, uint64_t n_x,
                                                     const u128* idmax, uint32_t nblk) {
  const u128 m = fold_idmax(idmax, nblk);
  if (threadIdx.x != 0) return;
  Globals* g = d.g;
  if (m > g->x_id_max) g->x_id_max = m;
  g->acc_count = n_acc;
  g->x_count = n_x;
  g->x_sorted = 0;  // every loaded transfer is hashed
  g->mono_prev = 0;
  g->pulse_next = TB_TIMESTAMP_MIN;
  if (lb->hi_max == ~0ull)
    g->ovf_bound = MAX128;
  else if (lb->hi_max)
    g->ovf_bound = ((u128)lb->hi_max << 64) | (u128)~0ull;
  else
    g->ovf_bound = lb->lo_max;
}

// ------------------------------------------------------------------------------------------------
// Re-tightening the overflow bound. Globals::ovf_bound only grows while windows commit (each adds its
// amount sum: it must stay >= every dp+dpo and cp+cpo without reading them), so after enough volume
// it is far above any real balance sum and the overflow-free fast paths (fused pass: below 2^63;
// 64-bit no-return adds: below 2^64) would stay off for good. The host launches this pair at a fixed
// point of the commit stream (every OVF_RESCAN_EVERY-th window, host.inc ovf_checkpoint), so replicas
// fed the same windows take the same paths; on the device both kernels return at once unless the bound
// is past OVF_RESCAN_AT, and then one grid pass sets it to the accounts' largest sum again (the
// LoadBound rule of open: exact while every sum fits 64 bits).
// ------------------------------------------------------------------------------------------------
#define OVF_RESCAN_AT ((u128)1 << 62)
#define OVF_RESCAN_EVERY 64u

__device__ inline bool ovf_rescan_due(const Globals* g) { return !g->window_error && g->ovf_bound >= OVF_RESCAN_AT; }

__global__ void __launch_bounds__(256) k_ovf_rescan(Dev d, LoadBound* lb) {
  __shared__ unsigned long long lh[256 / 64], ll[256 / 64];
  if (!ovf_rescan_due(d.g)) return;  // (uniform: every thread reads the same words)
  const uint64_t n = d.g->acc_count;
  unsigned long long hi = 0, lo = 0;
  for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x) {
    const tb_account_t& a = d.acc[k];
    const u128 dp = U(a.debits_pending), cp = U(a.credits_pending);
    const u128 s1 = dp + U(a.debits_posted), s2 = cp + U(a.credits_posted);
    const u128 m = s1 > s2 ? s1 : s2;
    const unsigned long long h = (s1 < dp || s2 < cp) ? ~0ull : (unsigned long long)(m >> 64);
    if (h) hi = h > hi ? h : hi;
    else lo = (unsigned long long)m > lo ? (unsigned long long)m : lo;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long y = __shfl_xor(hi, o, 64), z = __shfl_xor(lo, o, 64);
    hi = y > hi ? y : hi;
    lo = z > lo ? z : lo;
  }
  if ((threadIdx.x & 63) == 0) {
    lh[threadIdx.x >> 6] = hi;
    ll[threadIdx.x >> 6] = lo;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < 256 / 64; q++) {
      hi = lh[q] > hi ? lh[q] : hi;
      lo = ll[q] > lo ? ll[q] : lo;
    }
    if (hi) atomicMax(&lb->hi_max, hi);
    if (lo) atomicMax(&lb->lo_max, lo);
  }
}

__global__ void k_ovf_finish(Dev d, LoadBound* lb) {
  Globals* g = d.g;
  if (!ovf_rescan_due(g)) return;
  g->ovf_bound = lb->hi_max == ~0ull ? MAX128 : lb->hi_max ? (((u128)lb->hi_max << 64) | (u128)~0ull) : (u128)lb->lo_max;
  g->ovf_rescans++;
  lb->hi_max = lb->lo_max = 0;  // (zero for the next checkpoint's pass)
}

// ------------------------------------------------------------------------------------------------
// Digest: a position-sensitive 64-bit sum over the dense stores (every 8-byte word of every record,
// each record mixed with its slot), the pending statuses and pulse_next_timestamp. Replicas holding
// the same state have the same digest; tests recompute it from the CPU restatement's dumps
// (tigerbeetle_amd/digest.py).
// ------------------------------------------------------------------------------------------------
__device__ inline unsigned long long digest_record(const uint64_t* w, uint64_t slot) {
  unsigned long long h = 0x243f6a8885a308d3ull ^ slot;
#pragma unroll
  for (int k = 0; k < 16; k++) h = mix64(h ^ w[k] ^ ((unsigned long long)k << 56));
  return mix64(h + slot * 0x9e3779b97f4a7c15ull);
}

__global__ void __launch_bounds__(256) k_digest(const uint8_t* records, uint64_t n, const uint8_t* status,
                                                unsigned long long* out) {
  unsigned long long sr = 0, ss = 0;
  for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x) {
    sr += digest_record(reinterpret_cast<const uint64_t*>(records + k * 128), k);
    if (status) ss += mix64((k << 8) | status[k]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sr += __shfl_xor(sr, o, 64);
    ss += __shfl_xor(ss, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&out[0], sr);
    if (status) atomicAdd(&out[1], ss);
  }
}
