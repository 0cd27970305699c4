// xwin.h — commit windows with pulses inside (super-batching across expiries).
//
// The harness runs a pulse check before every batch (state_machine.zig:2719-2739). A window that
// spans a second or more (the cfg4 shape: +1 s per batch, timeouts of 1-60 s) has pulses due inside
// it. They are modelled exactly, not split off, when three conditions hold (k_xwin_decide rejects
// the window otherwise, before anything of it beyond its first pulse is applied):
//   - no account of the window is read by a decision (no hot account: limits, balancing), no event
//     writes a history row, and the window is overflow-free, so the expiries' balance effects
//     commute with everything else;
//   - no pulse inside the window hits the batch_max cap (counted conservatively per due batch), and
//     the window's first pulse finished its scan (scan_lookup buffer not full);
// Then an entry (a pending transfer with a scan-visible timeout) due at batch b (the first batch
// with T_b >= expires_at) expires at b's pulse unless a committed post/void removed it first. Its
// only readers inside the window are post/voids of it: k_ct_prep and the walkers see it as expired
// from batch b on (pending_transfer_expired). Its effects (status expired, dp / cp released,
// :1874-1929) are applied after the window (k_xwin_expire), in any order: they commute.
// pulse_next_timestamp follows the reference batch by batch (k_xwin_replay): before batch b >= 1 a
// pulse runs iff pulse_next <= T_b, and its finish sets the smallest expires_at live after it (a
// per-batch minimum kept in a segment tree over the window's batches, k_xwin_minlive); then the
// batch's creations that ran ok lower it and an effective post/void reset sets timestamp_min.
#pragma once
#include "window.h"

// Per due batch: an upper bound of the entries its pulse expires (live list entries due in the
// window, pending creations of the window that may be due in it).
__global__ void __launch_bounds__(256) k_xwin_count(Dev d, Scratch s, WinDesc w) {
  __shared__ uint32_t cnt[MAXB];
  if (WIN_REJECTED(d.g)) return;
  for (uint32_t j = threadIdx.x; j < MAXB; j += blockDim.x) cnt[j] = 0;
  __syncthreads();
  const uint64_t T_last = w.T[w.nb - 1];
  const ExpEntry* list = d.exp[*d.exp_cur];
  const uint64_t n = d.g->exp_count;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += stride) {
    const ExpEntry e = list[j];
    if (e.expires_at <= T_last && d.xstatus[e.slot] == TB_PENDING_PENDING) atomicAdd(&cnt[xw_due(w, e.expires_at)], 1u);
  }
  for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < w.E; k += stride) {
    const uint32_t cls = s.cls[k];
    if (!(cls & C_PNOP) || (cls & C_POSTVOID)) continue;
    const uint64_t x = s.pnv[k];
    if (x <= T_last && xw_visible(win_ts(w, s.batch[k], (uint32_t)k), x)) atomicAdd(&cnt[xw_due(w, x)], 1u);
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < MAXB; j += blockDim.x)
    if (cnt[j]) atomicAdd(&s.xw_cnt[j], cnt[j]);
}

// Rejects the window (nothing of it applied beyond its first pulse; tbg_sync: TBG_E_WINDOW) when a
// pulse inside it could hit the cap, or a balance is read, or it is not overflow-free; resets the
// per-window state k_ct_prep / k_prep_reduce left.
__global__ void k_xwin_decide(Dev d, Scratch s, WinDesc w, uint32_t cap) {
  Globals* g = d.g;
  if (WIN_REJECTED(g)) return;
  // (history rows hold the balances after each event: an expiry inside the window would move them)
  bool bad = g->hot_count != 0 || g->batch_huge || ovf128(g->ovf_bound, g->batch_amount_sum) || (g->win_flags & 16u);
  // (a pulse that fills its buffer, cap entries or more, ends buffer_finished: not modelled)
  for (uint32_t b = 1; b < w.nb; b++) bad = bad || s.xw_cnt[b] >= cap;
  for (uint32_t b = 0; b < MAXB; b++) s.xw_cnt[b] = 0;  // (zero again for the next window's count)
  if (!bad) return;
  atomicOr(&g->window_error, 1u);
  g->hot_count = 0;
  g->hot_live = 0;
  g->batch_amount_sum = 0;
  g->batch_huge = 0;
  g->res_inelig = 0;
}

// Removal batch of each pending transfer the window created (committed post/voids of it).
__global__ void __launch_bounds__(256) k_xwin_rb(Dev d, Scratch s, WinDesc w) {
  if (WIN_REJECTED(d.g)) return;
  // k_xwin_minlive's minima start at "none" (xw_tree, xw_minx, xw_miny: one allocation)
  if (blockIdx.x == 0)
    for (uint32_t j = threadIdx.x; j < 4 * MAXB; j += blockDim.x) s.xw_tree[j] = ~0ull;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < w.E; k += gridDim.x * blockDim.x) {
    const uint32_t cls = s.cls[k];
    if ((cls & C_POSTVOID) && (cls & C_PNOP) && s.code[k] == TB_CT_OK && s.p_tslot[k] == NONE32)
      s.pn_rb[s.pn_src[k]] = s.batch[k];
  }
}

__device__ inline void xw_tree_min(unsigned long long* tree, uint32_t lo, uint32_t hi, unsigned long long v) {
  // batches [lo, hi] take v (iterative segment tree, leaves at MAXB + b)
  uint32_t l = lo + MAXB, r = hi + MAXB + 1;
  while (l < r) {
    if (l & 1) atomicMin(&tree[l++], v);
    if (r & 1) atomicMin(&tree[--r], v);
    l >>= 1;
    r >>= 1;
  }
}

// The smallest expires_at live after each batch's pulse, and per batch the smallest creation
// expiry and reset candidate among the events that ran ok (the replay's fast path).
__global__ void __launch_bounds__(256) k_xwin_minlive(Dev d, Scratch s, WinDesc w) {
  __shared__ unsigned long long tree[2 * MAXB];
  __shared__ unsigned long long minx[MAXB], miny[MAXB];
  if (WIN_REJECTED(d.g)) return;
  for (uint32_t j = threadIdx.x; j < 2 * MAXB; j += blockDim.x) tree[j] = ~0ull;
  for (uint32_t j = threadIdx.x; j < MAXB; j += blockDim.x) minx[j] = miny[j] = ~0ull;
  __syncthreads();
  const uint32_t nb = w.nb;
  const uint64_t base = d.g->base;
  const ExpEntry* list = d.exp[*d.exp_cur];
  const uint64_t n = d.g->exp_count;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  // entries from before the window that nothing removed in it (the ones it removed: below)
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += stride) {
    const ExpEntry e = list[j];
    if (e.slot >= base || d.xstatus[e.slot] != TB_PENDING_PENDING) continue;
    const uint32_t due = xw_due(w, e.expires_at);
    if (due > 1) xw_tree_min(tree, 1, due - 1, e.expires_at);
  }
  for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < w.E; k += stride) {
    const uint32_t cls = s.cls[k];
    if (!(cls & C_PNOP)) continue;
    const uint32_t b = s.batch[k];
    const uint64_t v = s.pnv[k];
    const bool committed = s.code[k] == TB_CT_OK;
    const bool ranok = committed || (cls & C_RANOK);
    if (cls & C_POSTVOID) {
      if (ranok) atomicMin(&miny[b], v);
      const uint32_t ps = s.p_tslot[k];
      if (!committed || ps == NONE32) continue;  // in-window pending transfers: their creations
      // a pending transfer from before the window, live until this post/void removed it
      if (!xw_visible(d.xr[ps].timestamp, v)) continue;
      const uint32_t hi = min(b, xw_due(w, v) - 1);
      if (hi >= 1) xw_tree_min(tree, 1, hi, v);
    } else {
      if (ranok) atomicMin(&minx[b], v);
      if (!committed || !xw_visible(win_ts(w, b, (uint32_t)k), v)) continue;
      const uint32_t rb = s.pn_rb[k];
      const uint32_t hi = min(rb == 0xFFFFu ? nb - 1 : (uint32_t)rb, xw_due(w, v) - 1);
      if (hi >= b + 1) xw_tree_min(tree, b + 1, hi, v);
    }
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < 2 * MAXB; j += blockDim.x)
    if (tree[j] != ~0ull) atomicMin(&s.xw_tree[j], tree[j]);
  for (uint32_t j = threadIdx.x; j < MAXB; j += blockDim.x) {
    if (minx[j] != ~0ull) atomicMin(&s.xw_minx[j], minx[j]);
    if (miny[j] != ~0ull) atomicMin(&s.xw_miny[j], miny[j]);
  }
}

#define XW_THREADS 1024

// The replay's reset candidates, per batch (one block each): a post/void op (value v, a pending
// transfer's expires_at) resets pulse_next where v == min(pn, pm), pm the smallest creation value of
// the batch before it (k_pn's "before"); only v <= pm can ever qualify, and only whether a batch
// resets matters. So each candidate is kept as one word: v, with bit 63 set when v == pm (it resets
// iff pm <= pn; otherwise iff v == pn). Listed per batch from its first event's position in the t2
// area (free after k_final); values stay below 2^63 (TB_TIMESTAMP_MAX).
#define XW_CAND_EQ (1ull << 63)
__global__ void __launch_bounds__(XW_THREADS) k_xwin_pm(Dev d, Scratch s, WinDesc w) {
  __shared__ unsigned long long ldsm[XW_THREADS / 64];
  __shared__ uint32_t lds[XW_THREADS / 64];
  if (WIN_REJECTED(d.g)) return;
  const uint32_t b = blockIdx.x;
  if (s.xw_miny[b] == ~0ull) {  // (k_xwin_minlive: no post/void op in the batch ran ok)
    if (threadIdx.x == 0) s.xw_ccnt[b] = 0;
    return;
  }
  unsigned long long* cv = reinterpret_cast<unsigned long long*>(s.t2);
  unsigned long long carry = ~0ull;
  uint32_t nc = 0;
  for (uint32_t c0 = w.off[b]; c0 < w.off[b + 1]; c0 += XW_THREADS) {
    const uint32_t k = c0 + threadIdx.x;
    uint64_t v = 0;
    const uint32_t op = k < w.off[b + 1] ? pn_op(s, k, &v) : 0u;
    unsigned long long tot;
    const unsigned long long pm = umin64(carry, block_excl_min_u64<XW_THREADS / 64>(op == 1 ? v : ~0ull, ldsm, &tot));
    const bool cand = op == 2 && v <= pm && v <= TB_TIMESTAMP_MAX;
    uint32_t tc;
    const uint32_t r = block_excl<XW_THREADS / 64>(cand ? 1u : 0u, lds, &tc);
    if (cand) cv[w.off[b] + nc + r] = v | (v == pm ? XW_CAND_EQ : 0ull);
    nc += tc;
    carry = umin64(carry, tot);
  }
  if (threadIdx.x == 0) s.xw_ccnt[b] = nc;
}

#define XW_LDS_CAND 4096  // candidates the replay holds in LDS (the rest are read from the t2 area)

// pulse_next_timestamp through the window, batch by batch (one workgroup): a batch resets it if any
// of its candidates qualifies (k_xwin_pm), else its creations lower it to minx. The candidates go to
// LDS first, so the batch loop has no dependent global load.
__global__ void __launch_bounds__(XW_THREADS) k_xwin_replay(Dev d, Scratch s, WinDesc w) {
  __shared__ unsigned long long tree[2 * MAXB], minx[MAXB], miny[MAXB];
  __shared__ uint32_t coff[MAXB + 1];
  __shared__ unsigned long long cl[XW_LDS_CAND];
  if (WIN_REJECTED(d.g)) return;
  for (uint32_t j = threadIdx.x; j < 2 * MAXB; j += XW_THREADS) tree[j] = s.xw_tree[j];
  for (uint32_t j = threadIdx.x; j < MAXB; j += XW_THREADS) {
    minx[j] = s.xw_minx[j];
    miny[j] = s.xw_miny[j];
  }
  for (uint32_t b = threadIdx.x; b < w.nb; b += XW_THREADS) coff[b + 1] = (uint32_t)s.xw_ccnt[b];
  __syncthreads();
  if (threadIdx.x == 0) {  // (<= 128 batches, in LDS)
    coff[0] = 0;
    for (uint32_t b = 0; b < w.nb; b++) coff[b + 1] += coff[b];
  }
  __syncthreads();
  const unsigned long long* cv = reinterpret_cast<const unsigned long long*>(s.t2);
  // (flattened: candidate x of the window belongs to the batch b with coff[b] <= x < coff[b + 1])
  const uint32_t held = min(coff[w.nb], (uint32_t)XW_LDS_CAND);
  for (uint32_t x = threadIdx.x; x < held; x += XW_THREADS) {
    uint32_t lo = 0, hi = w.nb;  // the last b with coff[b] <= x
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (coff[mid] <= x) lo = mid; else hi = mid;
    }
    cl[x] = cv[w.off[lo] + (x - coff[lo])];
  }
  __syncthreads();
  // Per batch, in parallel: the value a pulse before it would set (the smallest entry live after it,
  // from the segment tree), and whether the batch resets pulse_next when it starts from that value.
  // The batch-by-batch loop below then only reads LDS words (it re-evaluates the candidates only for a
  // batch that starts without a pulse).
  __shared__ unsigned long long pv[MAXB];
  __shared__ uint32_t rp[MAXB];
  for (uint32_t b = threadIdx.x; b < w.nb; b += XW_THREADS) {
    unsigned long long m = ~0ull;
    for (uint32_t node = MAXB + b; node >= 1; node >>= 1) m = umin64(m, tree[node]);
    pv[b] = m == ~0ull ? TB_TIMESTAMP_MAX : m;
    rp[b] = 0;
  }
  __syncthreads();
  for (uint32_t x = threadIdx.x; x < coff[w.nb]; x += XW_THREADS) {
    uint32_t lo = 0, hi = w.nb;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (coff[mid] <= x) lo = mid; else hi = mid;
    }
    const unsigned long long c = x < XW_LDS_CAND ? cl[x] : cv[w.off[lo] + (x - coff[lo])];
    const unsigned long long v = c & ~XW_CAND_EQ, p0 = pv[lo];
    if ((c & XW_CAND_EQ) ? v <= p0 : v == p0) rp[lo] = 1;
  }
  __syncthreads();
  uint64_t pn = d.g->pulse_next;  // after the window's first pulse
  for (uint32_t b = 0; b < w.nb; b++) {
    bool reset = false;
    if (b >= 1 && pn <= w.T[b]) {
      pn = pv[b];  // the pulse before batch b: its finish takes the smallest entry live after it
      reset = miny[b] <= pn && rp[b];
    } else if (miny[b] <= pn) {  // (else no reset can take effect: it needs expires_at == pulse_next <= pn)
      const uint32_t n = coff[b + 1] - coff[b];
      for (uint32_t c0 = 0; c0 < n && !reset; c0 += XW_THREADS) {
        const uint32_t j = c0 + threadIdx.x, x = coff[b] + j;
        bool q = false;
        if (j < n) {
          const unsigned long long c = x < XW_LDS_CAND ? cl[x] : cv[w.off[b] + j];
          const unsigned long long v = c & ~XW_CAND_EQ;
          q = (c & XW_CAND_EQ) ? v <= pn : v == pn;
        }
        reset = __syncthreads_or(q ? 1 : 0) != 0;
      }
    }
    pn = reset ? TB_TIMESTAMP_MIN : umin64(pn, minx[b]);  // (:1706-1707; the next batch's pulse check is true)
  }
  if (threadIdx.x == 0) d.g->pulse_next = pn;
}

// The pulses inside the window, applied: every live entry due in it that is still pending expires
// (execute_expire_pending_transfers, :1874-1929; the effects commute, see above). Entries stay in the
// list and are dropped by the next scan.
__global__ void __launch_bounds__(256) k_xwin_expire(Dev d, WinDesc w, ChgLog chg, uint32_t chg_epoch) {
  if (WIN_REJECTED(d.g)) return;
  const uint64_t T_last = w.T[w.nb - 1];
  const ExpEntry* list = d.exp[*d.exp_cur];
  const uint64_t n = d.g->exp_count;
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    const ExpEntry e = list[j];
    if (e.expires_at > T_last || d.xstatus[e.slot] != TB_PENDING_PENDING) continue;
    const tb_transfer_t x = d.xr[e.slot];
    AccEntry de, ce;
    const uint32_t drs = acc_find(d.acc_tab, d.acc_mask, x.debit_account_id, &de);
    const uint32_t crs = acc_find(d.acc_tab, d.acc_mask, x.credit_account_id, &ce);
    const u128 amt = U(x.amount);
    atomic_sub_u128(&d.acc[drs].debits_pending, amt);
    atomic_sub_u128(&d.acc[crs].credits_pending, amt);
    d.xstatus[e.slot] = TB_PENDING_EXPIRED;
    if (chg.mark) {
      chg.mark[drs] = chg_epoch;
      chg.mark[crs] = chg_epoch;
      chg.pend[atomicAdd(&chg.cnt[1], 1u)] = e.slot;
    }
  }
}
