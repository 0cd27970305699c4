// query.h — get_account_transfers / get_account_balances (state_machine.zig:786-996, 1346-1419)
// from the device stores, and the history rows they read (historical_balance, :1806-1841).
//
// The reference answers both from the transfers groove's debit_account_id / credit_account_id
// indexes: a union of the two prefix scans over [timestamp_min, timestamp_max], ascending or
// descending, into a buffer of min(limit, batch_max) results; get_account_balances then looks each
// transfer's timestamp up in the account_balances groove. Here the dense transfer store is itself
// in timestamp order, so a query is a filtered, ordered stream compaction over a slot range found
// by binary search: chunks of slots in scan order, per-block match counts, then ordered emission of
// the matching slots until the limit is reached (the host stops launching chunks there). History
// rows live beside the transfer records, one 128 B row per slot (the dr and cr accounts' balances
// after the transfer, each present if that account has flags.history).
#pragma once
#include "window.h"

// One query: the filter plus the slot range it scans.
struct QFilter {
  uint64_t id_lo, id_hi;
  uint64_t lo, hi;  // slots [lo, hi) have timestamps in the filter's range
  uint32_t debits, credits, reversed;
  uint32_t pad;
};

// Slot range of [tmin, tmax] (binary searches over the timestamp-ordered store) and, for
// get_account_balances, whether the account exists with flags.history. out: lo, hi, account flags
// + (found << 16).
__global__ void k_q_bounds(Dev d, uint64_t tmin, uint64_t tmax, tb_uint128_t account, uint64_t* out) {
  const uint64_t n = d.g->x_count;
  uint64_t a = 0, b = n;
  while (a < b) {  // first slot with timestamp >= tmin
    const uint64_t m = (a + b) >> 1;
    if (d.xr[m].timestamp < tmin) a = m + 1; else b = m;
  }
  const uint64_t lo = a;
  b = n;
  while (a < b) {  // first slot with timestamp > tmax
    const uint64_t m = (a + b) >> 1;
    if (d.xr[m].timestamp <= tmax) a = m + 1; else b = m;
  }
  out[0] = lo;
  out[1] = a;
  AccEntry e;
  const uint32_t slot = acc_find(d.acc_tab, d.acc_mask, account, &e);
  out[2] = slot == NONE32 ? 0 : ((1ull << 16) | d.acc[slot].flags);
}

// Scan position pos of the chunk [.., p1) (positions count from the first slot in scan order).
__device__ inline bool q_match(const Dev& d, const QFilter& q, uint64_t pos, uint64_t p1, uint64_t* slot_out) {
  if (pos >= p1 || pos >= q.hi - q.lo) return false;
  const uint64_t slot = q.reversed ? q.hi - 1 - pos : q.lo + pos;
  const tb_transfer_t* t = &d.xr[slot];
  *slot_out = slot;
  const bool dr = q.debits && t->debit_account_id.lo == q.id_lo && t->debit_account_id.hi == q.id_hi;
  const bool cr = q.credits && t->credit_account_id.lo == q.id_lo && t->credit_account_id.hi == q.id_hi;
  return dr || cr;
}

// Per block of SEG scan positions [p0 + SEG*block, ...): the number of matches.
__global__ void __launch_bounds__(SEG) k_q_count(Dev d, Scratch s, QFilter q, uint64_t p0, uint64_t p1) {
  __shared__ uint32_t lds[SEG / 64];
  uint64_t slot;
  const uint32_t m = q_match(d, q, p0 + (uint64_t)blockIdx.x * SEG + threadIdx.x, p1, &slot) ? 1u : 0u;
  const uint32_t n = block_sum<SEG / 64>(m, lds);
  if (threadIdx.x == 0) s.cnt_w[blockIdx.x] = n;
}

// Ordered emission: match k of this chunk goes to result position found + k while that is below
// `limit`; the chunk's total match count is added to *total.
__global__ void __launch_bounds__(SEG) k_q_emit(Dev d, Scratch s, QFilter q, uint64_t p0, uint64_t p1,
                                                uint32_t found, uint32_t limit, uint32_t* total) {
  __shared__ uint32_t lds[SEG / 64];
  if (s.cnt_w[blockIdx.x] == 0) return;  // uniform per block
  const uint32_t prefix = seg_prefix<SEG>(s.cnt_w, blockIdx.x, lds);
  uint64_t slot = 0;
  const uint32_t m = q_match(d, q, p0 + (uint64_t)blockIdx.x * SEG + threadIdx.x, p1, &slot) ? 1u : 0u;
  uint32_t tot;
  const uint32_t pos = found + prefix + block_excl<SEG / 64>(m, lds, &tot);
  if (m && pos < limit) s.wlist[pos] = (uint32_t)slot;
  if (threadIdx.x == 0) atomicAdd(total, tot);
}

__global__ void __launch_bounds__(256) k_q_gather_transfers(Dev d, Scratch s, uint32_t n, tb_transfer_t* out) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) out[k] = d.xr[s.wlist[k]];
}

// AccountBalance rows (execute_get_account_balances, :1383-1414): the queried account's side of
// each transfer's history row, in scan order. One workgroup. A transfer without that row (the
// expired post/void quirk record, :1689-1696) is skipped: the reference's scan lookup would reach
// `unreachable` there (lsm/scan_lookup.zig).
__global__ void __launch_bounds__(1024) k_q_gather_balances(Dev d, Scratch s, uint32_t n, tb_uint128_t account,
                                                            tb_account_balance_t* out, uint32_t* out_count) {
  __shared__ uint32_t lds[1024 / 64];
  uint32_t carry = 0;
  for (uint32_t base = 0; base < n; base += 1024) {
    const uint32_t k = base + threadIdx.x;
    uint32_t side = 0, ok = 0, slot = 0;
    if (k < n) {
      slot = s.wlist[k];
      const tb_transfer_t* t = &d.xr[slot];
      side = (t->debit_account_id.lo == account.lo && t->debit_account_id.hi == account.hi) ? 0u : 1u;
      ok = (d.hist_side[slot] >> side) & 1u;
    }
    uint32_t tot;
    const uint32_t pos = carry + block_excl<1024 / 64>(ok, lds, &tot);
    if (ok) {
      const u128* b = side ? d.hist[slot].cr : d.hist[slot].dr;
      tb_account_balance_t r;
      memset(&r, 0, sizeof r);
      r.debits_pending = W(b[0]);
      r.debits_posted = W(b[1]);
      r.credits_pending = W(b[2]);
      r.credits_posted = W(b[3]);
      r.timestamp = d.xr[slot].timestamp;
      out[pos] = r;
    }
    carry += tot;
  }
  if (threadIdx.x == 0) *out_count = carry;
}
