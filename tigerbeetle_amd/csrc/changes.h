// changes.h — the write-back stream of a committed window (TBG_FLAG_CHANGE_LOG).
//
// The reference's commit leaves its effects in the grooves (groove.insert / groove.update,
// lsm/groove.zig:905-1000): inserted transfers and accounts, updated account balances, inserted and
// updated TransferPending rows (state_machine.zig:259-269). A replica that keeps its LSM forest on
// the host needs exactly those records after each commit. Here:
//   - inserted records are the store slice [base, count) of the window (commit = timestamp order);
//   - every account whose balances a committed event changed is marked with the window number
//     (k_chg_mark; plain stores, every writer stores the same value), then listed in slot order
//     (k_chg_count, k_chg_scan, k_chg_list). The fused pass (fused.h) marks its accounts in `fmark`
//     while it applies, before it knows whether it commits the window: those marks count only when
//     it did (Globals::sp_done with fu_epoch = the window), and the general path's own marks in
//     `mark` otherwise;
//   - earlier pending transfers that a committed post/void resolved are listed by k_chg_mark.
// k_pulse_tail marks the accounts and lists the transfers of every expiry the same way. A commit
// call's log covers its pulse (if any) and its window. tbg_window_changes gathers and copies them.
#pragma once
#include "window.h"

struct ChgLog {
  uint32_t* mark;      // per account slot: window number of the last change
  uint32_t* fmark;     // per account slot: window number of the last fused-pass change (speculative)
  uint32_t* list;      // changed account slots, ascending
  uint32_t* pend;      // transfer slots of earlier pending transfers resolved in the window
  uint32_t* seg;       // per account segment: count, then exclusive offset
  uint32_t* cnt;       // [0] changed accounts, [1] resolved pending transfers
  tb_account_t* gather;          // staging for the changed account records
  tb_transfer_pending_t* rows;   // staging for TransferPending rows
};

template <bool XFER>
__global__ void __launch_bounds__(256) k_chg_mark(Scratch s, const Globals* g, uint32_t E, uint32_t epoch, ChgLog c) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  // (a window the fused pass committed left no scratch columns: its marks are in fmark)
  if (i >= E || WIN_REJECTED(g) || SP_DONE(g) || s.code[i] != TB_CT_OK) return;
  if (!XFER) return;  // new accounts are the store slice
  const uint32_t dr = s.dr_slot[i], cr = s.cr_slot[i];
  // a post/void of a pending transfer created in this window may carry no slots: its creator,
  // committed in the same window, marked the same accounts
  if (dr != NONE32) c.mark[dr] = epoch;
  if (cr != NONE32) c.mark[cr] = epoch;
  if ((s.cls[i] & C_POSTVOID) && s.p_tslot[i] != NONE32) c.pend[atomicAdd(&c.cnt[1], 1u)] = s.p_tslot[i];
}

// Whether account `slot` changed in log `epoch` (the general path's marks, or the fused pass's when it
// committed that window).
__device__ inline bool chg_marked(const Globals* g, const ChgLog& c, uint64_t slot, uint32_t epoch) {
  if (slot >= g->acc_count) return false;
  if (c.mark[slot] == epoch) return true;
  return g->sp_done && g->fu_epoch == epoch && c.fmark[slot] == epoch;
}

__global__ void __launch_bounds__(SEG) k_chg_count(Dev d, uint32_t epoch, ChgLog c) {
  __shared__ uint32_t lds[SEG / 64];
  const uint64_t slot = (uint64_t)blockIdx.x * SEG + threadIdx.x;
  const uint32_t m = chg_marked(d.g, c, slot, epoch) ? 1u : 0u;
  const uint32_t tot = block_sum<SEG / 64>(m, lds);
  if (threadIdx.x == 0) c.seg[blockIdx.x] = tot;
}

// One block: exclusive offsets of the segment counts (in place) and the total.
__global__ void __launch_bounds__(1024) k_chg_scan(uint32_t nseg, ChgLog c) {
  __shared__ uint32_t lds[1024 / 64];
  uint32_t carry = 0;
  for (uint32_t base = 0; base < nseg; base += 1024) {
    const uint32_t j = base + threadIdx.x;
    const uint32_t v = j < nseg ? c.seg[j] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl<1024 / 64>(v, lds, &tot);
    if (j < nseg) c.seg[j] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) c.cnt[0] = carry;
}

__global__ void __launch_bounds__(SEG) k_chg_list(Dev d, uint32_t epoch, ChgLog c) {
  __shared__ uint32_t lds[SEG / 64];
  const uint64_t slot = (uint64_t)blockIdx.x * SEG + threadIdx.x;
  const bool m = chg_marked(d.g, c, slot, epoch);
  uint32_t tot;
  const uint32_t r = c.seg[blockIdx.x] + block_excl<SEG / 64>(m ? 1u : 0u, lds, &tot);
  if (m) c.list[r] = (uint32_t)slot;
}

// Zeroes a log's counters at the start of a commit call, except while a fused-only window waits for
// its replay (window_error bit 3): its pulse already listed its expiries here, and the replay keeps
// that log (host.inc settle()).
__global__ void k_chg_begin(const Globals* g, ChgLog c) {
  if (g->window_error & 8u) return;
  c.cnt[0] = 0;
  c.cnt[1] = 0;
  c.cnt[2] = 0;
  c.cnt[3] = 0;
}

// Gathers the changed account records and the resolved pending transfers' rows.
__global__ void __launch_bounds__(256) k_chg_gather(Dev d, ChgLog c, uint32_t n_acc, uint32_t n_pend) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n_acc) c.gather[k] = d.acc[c.list[k]];
  if (k < n_pend) {
    const uint32_t slot = c.pend[k];
    tb_transfer_pending_t r;
    r.timestamp = d.xr[slot].timestamp;
    r.status = d.xstatus[slot];
    for (int q = 0; q < 7; q++) r.padding[q] = 0;
    c.rows[k] = r;
  }
}
