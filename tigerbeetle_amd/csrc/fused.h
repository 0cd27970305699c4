// fused.h — one pass over an order-free create_transfers window (the cfg1 / cfg2 shape: plain
// single-phase transfers with strictly increasing ids between unlimited accounts).
//
// The general path (k_ct_prep -> k_prep_reduce -> k_classify -> k_wlist -> k_walk -> k_final) writes
// ~72 B of scratch columns per event and reads ~40 B of them back, in seven launches. For a window in
// which every outcome is order-free that traffic buys nothing: k_ct_fused decides each event
// (state_machine.zig:1462-1507 validation, lookups, ledgers, create_transfer_exists :1587-1606; the
// balance tail :1509-1547 cannot fail, below), applies its balance effects (:1549-1575) and stores its
// record in place (slot base + i, final when no earlier event of the window failed); k_fu_final then
// writes the replies and moves the records after the window's first failure down to their ranks
// (nothing to move in a window without failures). No block waits for another: a decoupled look-back
// for the ranks measured 50 us per 1M-event window of blocks idling behind slower predecessors.
//
// Simple = every event of the window is either decided statically (validation, lookups, ledgers,
// exists) or is a create (single-phase, or pending with or without a timeout; no linked / post / void /
// balancing flag) whose accounts carry no limit and no history flag, the ids are strictly increasing over the window in u128 order
// (64-bit sequences and the reference's time-based 128-bit ids alike, docs/develop/data-modeling.md:
// 186-203; so no id repeats: the window is claim-free), and every amount reaching the account checks is below
// 2^43 with the overflow bound below 2^63 (so no balance field leaves its low 64-bit word: the
// overflow checks of :1532-1545 cannot fail, and the balance adds are exact no-return 64-bit adds).
// Then every outcome is a function of the pre-window state and the event alone. A
// pending create (round 5) adds to debits_pending / credits_pending instead of the posted fields
// (:1555-1566), inserts its TransferPending row as pending, lowers pulse_next_timestamp to its expiry
// when it has a timeout (:1576-1581: the last block folds the window's minimum) and gets a live entry
// in the expires_at list (k_fu_final, once the window commits). None of it is read by another event
// of an order-free window: no post/void is in the class, and the window's own timeouts fall due after
// it (a window reaches the fused pass only if it spans less than a second).
//
// Speculation. Each block applies its balance adds as soon as its own events are simple; whether the
// whole window is simple is known after the launch (Globals::fu_abort = this window's epoch when a
// block was not). If it is not, k_fu_final subtracts the adds of every block that applied (its ok
// events, from the per-wave bitmap the applying blocks wrote; the accounts probed again), and
// the general path runs the window as if this pass had not (its record and status stores are all
// rewritten or beyond the store's end). Globals::sp_done tells the general path's kernels to return
// at once when the fused pass committed the window. A window that is not simple backs the speculation
// off exponentially (Globals::sp_skip windows, k_final counts them down).
#pragma once

#define FU_T 256
#define FU_AMOUNT_MAX (1ull << 43)  // per-event amount bound: 2^20 events x 2^43 <= 2^63
#define FU_BACKOFF_MAX 8u           // transfer windows the speculation waits at most after a miss
#ifndef FU_FINAL_GRID
#define FU_FINAL_GRID 1024u         // k_fu_final's blocks at most (each finishes every FU_FINAL_GRID-th group)
#endif

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long y = __shfl_xor(v, o, 64);
    v = y > v ? y : v;
  }
  return v;
}

// One event's decision on the fused path. `simple` is cleared when the event puts the window outside
// the class; then the other outputs are meaningless. `ok` events insert and apply `amount` to the
// debit account's debits_posted and the credit account's credits_posted (:1569-1575).
struct FuEv {
  uint32_t code, dr, cr;
  unsigned long long amount;  // C_REACH events: the amount (every one counts toward the overflow bound)
  u128 id_key;                // C_REACH events: the id (x_id_max bound)
  uint64_t expires_at;        // a pending create with a timeout: its expiry (0 = none)
  uint32_t cpos;              // claim mode: the table position of the event's claim (NONE32: none)
  bool simple, reach, pending;
};

// Claim mode (windows whose ids are not known to rise: Globals::mono_prev = 0): an event that reaches
// the exists check claims its id in the transfer table itself (x_probe_claim: its entry points at its
// in-place record, slot base + i), so one probe sequence finds a stored transfer, finds an in-window
// duplicate (another event's claim: outside the class) and indexes the new record. k_fu_final re-points
// the claims of records that move down to their ranks (by the claim's position, fs.cpos: never by a
// search, which could meet another record's re-pointed entry), and removes every claim of a window
// that leaves the class (reverted to the empty entries they took: the table is restored exactly). (Round 4 claimed in the window key map and inserted into the table after the
// window: two random probe sequences per event.)

// prev_id: the id of event i - 1 (i > 0). ts: the event's timestamp (the record as inserted). base:
// the window's first record slot. claim: claim mode (ev: the window's events, E of them), else the
// ids must rise.
__device__ __forceinline__ void fu_decide(const Dev& d, uint32_t i, u128 prev_id, const tb_transfer_t& t, uint64_t ts,
                                          u128 x_id_max, uint64_t P, uint64_t base, FuEv* o, bool claim = false,
                                          const tb_transfer_t* ev = nullptr, uint32_t E = 0) {
  const uint16_t f = t.flags;
  o->dr = o->cr = NONE32;
  o->amount = 0;
  o->id_key = 0;
  o->expires_at = 0;
  o->cpos = NONE32;
  o->reach = false;
  o->pending = (f & TB_TRANSFER_PENDING) != 0;
  // no chain, no post/void; claim-free (ids strictly increasing over the window, k_ct_prep's test)
  // unless in claim mode
  bool simple = !(f & TB_TRANSFER_LINKED) && !(f & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING));
  if (i > 0 && !claim) simple = simple && U(t.id) > prev_id;
  uint32_t code;
  if (t.timestamp != 0) {
    code = TB_CT_TIMESTAMP_MUST_BE_ZERO;  // :1251
  } else {
    code = ct_head(t);
    if (code == CONT) {
      if (f & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING | TB_TRANSFER_BALANCING_DEBIT |
               TB_TRANSFER_BALANCING_CREDIT)) {
        simple = false;
      } else {
        code = ct_validate(t);
        if (code == CONT) {
          // three independent probes in flight together (k_ct_prep)
          const uint64_t hd = hash_id(t.debit_account_id.lo, t.debit_account_id.hi) & d.acc_mask;
          const uint64_t hc = hash_id(t.credit_account_id.lo, t.credit_account_id.hi) & d.acc_mask;
          const bool mx = x_may_exist(t.id, x_id_max);
          const uint64_t hx = hash_id(t.id.lo, t.id.hi);
          const AccEntry ed = d.acc_tab[hd], ec = d.acc_tab[hc];
          // (claim mode claims without reading the entry first: x_probe_claim's compare-and-swap
          // returns what the entry holds, so the claim is one memory-side atomic on the 2 GB table
          // instead of a line read plus the atomic)
          const XEntry ex = (mx && !claim) ? d.x_tab[hx & d.x_mask] : X_EMPTY;
          AccEntry de, ce;
          o->dr = acc_probe_from(d.acc_tab, d.acc_mask, hd, ed, t.debit_account_id, &de);
          o->cr = acc_probe_from(d.acc_tab, d.acc_mask, hc, ec, t.credit_account_id, &ce);
          if (o->dr == NONE32)
            code = TB_CT_DEBIT_ACCOUNT_NOT_FOUND;
          else if (o->cr == NONE32)
            code = TB_CT_CREDIT_ACCOUNT_NOT_FOUND;
          else
            code = ct_ledgers(t, de.ledger, ce.ledger);
          if (code == CONT) {
            o->reach = true;
            o->amount = t.amount.lo;
            o->id_key = U(t.id);
            // a limit or history flag reads (or records) balances in order: not order-free
            if (((de.flags | ce.flags) & TB_ACCOUNT_HISTORY) || (de.flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) ||
                (ce.flags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS) || t.amount.hi != 0 || t.amount.lo >= FU_AMOUNT_MAX)
              simple = false;
            // the balance tail (:1509-1547) after exists: its overflow checks cannot fail here (the
            // amounts and the bound, above), the timeout's can (a single-phase create has timeout 0);
            // computed first, so that an event failing it claims nothing
            const uint64_t tns = (uint64_t)t.timeout * TB_NS_PER_S;
            const bool tovf = t.timeout != 0 && ovf64(ts, tns);
            uint32_t xs = NONE32;
            if (claim) {
              // the sorted prefix first (a transfer found there is not in the table), then the claim
              if (mx) xs = x_prefix_find(d.xr, P, t.id);
              bool dup = false;
              if (xs == NONE32) {
                // (an event that will not insert must read the entry: it only looks for its id)
                const XEntry e0 = tovf ? d.x_tab[hx & d.x_mask] : X_EMPTY;
                xs = x_probe_claim(d.x_tab, d.xr, ev, d.x_mask, hx, e0, t.id, base, i, E, !tovf, &dup, &o->cpos);
              }
              if (dup) simple = false;  // in-window duplicate
            } else {
              xs = mx ? x_probe_from(d.x_tab, d.xr, d.x_mask, hx, ex, t.id) : NONE32;
              if (xs == NONE32 && mx) xs = x_prefix_find(d.xr, P, t.id);
            }
            // :1506-1507
            code = xs != NONE32 ? ct_exists(t, d.xr[xs]) : (tovf ? (uint32_t)TB_CT_OVERFLOWS_TIMEOUT : (uint32_t)TB_CT_OK);
            if (code == TB_CT_OK && t.timeout != 0) o->expires_at = ts + tns;
          }
        }
      }
    }
  }
  o->code = code;
  o->simple = simple;
}

// A per-window count kept as [63:32] epoch | [31:0] count and never reset: the block's atomicMax moves a
// stale tag to this epoch with count 0 (a no-op once it is there), then its atomicAdd returns the
// count before it. Two atomics per block, where a compare-and-swap loop measured quadratic in the
// blocks contending for it (16 ms per 1M-event window with a count in every block).
__device__ __forceinline__ uint32_t epoch_count_add(unsigned long long* word, uint32_t epoch, uint32_t n) {
  (void)atomicMax(word, (unsigned long long)epoch << 32);
  return (uint32_t)atomicAdd(word, (unsigned long long)n);
}

// Scratch of the fused pass (per 256-event block; per 64-event wave).
struct FuScratch {
  uint32_t* cnt;            // per block: failed events
  unsigned long long* pay;  // per block: its reaching amounts' sum
  u128* idmax;              // per block: its largest reaching id
  uint8_t* applied;         // per block: its balance adds were applied (k_fu_final undoes them)
  unsigned long long* ok;   // per wave: ok-event bitmap
  unsigned long long* pend; // per wave: ok pending creates
  unsigned long long* pto;  // per wave: ok pending creates with a timeout the expiry scan can see
  unsigned long long* pnmin;  // per block: smallest expiry of its ok creates with a timeout (~0: none)
  uint32_t* pbase;          // per block: its first live expiry entry within its slot (fu_slot_base)
  uint32_t* cpos;           // per event, claim mode: its claim's table position (NONE32: none)
  unsigned long long* slots;  // FU_SLOTS failure counts, then FU_SLOTS expiry-entry counts (epoch_count_add)
};

// Window-wide counts spread over FU_SLOTS words (block k adds to slot k % FU_SLOTS): same-address
// atomics serialize at the L2 (~30 ns each with a return; one per block of a 1M-event window cost
// 240 us), one slot per 64 blocks does not. Readers sum the slots with one wave.
#define FU_SLOTS 64
// Lane j < FU_SLOTS of the calling wave: slot j's count for this epoch (0 when stale).
__device__ __forceinline__ uint32_t fu_slot_count(const unsigned long long* slots, uint32_t epoch) {
  const uint32_t j = threadIdx.x & 63;
  const unsigned long long v = slots[j];
  return (uint32_t)(v >> 32) == epoch ? (uint32_t)v : 0u;
}

// The balance fields a create adds to: posted, or pending for a pending transfer (:1555-1566).
__device__ __forceinline__ unsigned long long* fu_dr_field(const Dev& d, const FuEv& fe) {
  return reinterpret_cast<unsigned long long*>(fe.pending ? &d.acc[fe.dr].debits_pending : &d.acc[fe.dr].debits_posted);
}
__device__ __forceinline__ unsigned long long* fu_cr_field(const Dev& d, const FuEv& fe) {
  return reinterpret_cast<unsigned long long*>(fe.pending ? &d.acc[fe.cr].credits_pending : &d.acc[fe.cr].credits_posted);
}

__device__ __forceinline__ void fu_store_records(Dev d, const uint4* src, bool ok, unsigned long long okm,
                                                 uint64_t first_slot, uint4* ws) {
  // the wave's ok records as one contiguous run from first_slot, through LDS in two halves of 64 B
  // (each store instruction writes whole 64 B sectors)
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nins = (uint32_t)__popcll(okm);
  const uint32_t pos = ok ? (uint32_t)__popcll(okm & ((1ull << lane) - 1ull)) : 0u;
  uint4* dst = reinterpret_cast<uint4*>(d.xr + first_slot);
#pragma unroll
  for (int half = 0; half < 2; half++) {
    wave_sync();
    if (ok) {
#pragma unroll
      for (int q = 0; q < 4; q++) ws[pos * 4 + q] = src[half * 4 + q];
    }
    wave_sync();
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t idx = c * 64 + lane, r = idx >> 2, q = idx & 3;
      if (r < nins) st_stream(dst + r * 8 + half * 4 + q, ws[idx]);
    }
  }
}

// Decide, apply, store in place. Writes nothing but scratch, the in-place records and statuses (slots
// at or beyond the store's end) and, when its events are simple, the balance adds.
// HOST (the synchronous path): `ev` is the request in pinned host memory, copied through to ev_copy
// (below). (Issuing all eight of a lane's 16 B loads before the first use measured slower: 43 against
// 38 us per 8190-event batch.)
template <bool HOST>
__global__ void __launch_bounds__(FU_T) k_ct_fused(Dev d, Scratch s, FuScratch fs, const tb_transfer_t* __restrict__ ev,
                                                   WinDesc w, uint32_t epoch, uint32_t fo_only, uint32_t* fmark,
                                                   uint32_t pn_skip, uint4* __restrict__ ev_copy) {
  __shared__ uint4 stage[FU_T * 4];  // half of each inserted record per round (16 KiB)
  __shared__ uint32_t lds[FU_T / 64];
  __shared__ unsigned long long ldsu[FU_T / 64];
  __shared__ u128 ldsm[FU_T / 64];
  __shared__ uint32_t ldsn[FU_T / 64];
  __shared__ unsigned long long ldsp[FU_T / 64];
  __shared__ uint32_t ldsx[FU_T / 64];
  Globals* g = d.g;
  const bool rejected = WIN_REJECTED(g);
  const uint32_t k = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // Another block may flag the window at any time, so waves of this block can read fu_abort
  // differently: each wave reads it once (wave-uniform), and the block applies its adds only if NO
  // wave saw it set (folded into the block vote below), so every wave and fs.applied[k] agree on
  // whether this block applies (k_fu_final undoes exactly those).
  const bool skip = !rejected && g->sp_skip != 0;
  const bool aborted = rejected || skip || __builtin_amdgcn_readfirstlane(__hip_atomic_load(&g->fu_abort, __ATOMIC_RELAXED,
                                                                                __HIP_MEMORY_SCOPE_AGENT) == epoch
                                                                  ? 1
                                                                  : 0) != 0;
  // ev_copy (the synchronous path): `ev` is the request in pinned host memory, read once over the link
  // by this pass, which stores it to ev_copy in HBM as it goes (every later kernel and a replay read
  // that), whatever the window's fate, instead of a separate copy launch ahead of it. A wave that does
  // not decide copies its 64 records here.
  if (HOST && aborted) {
    const uint32_t i0 = k * FU_T + wave * 64;
    const uint32_t n16 = i0 < w.E ? min(64u, w.E - i0) * 8u : 0u;
    const uint4* src = reinterpret_cast<const uint4*>(ev + i0);
    for (uint32_t q = lane; q < n16; q += 64) ev_copy[(size_t)i0 * 8 + q] = src[q];
  }
  if (rejected) return;
  if (skip) {  // backed off: the general path decides this window
    if (k == 0 && threadIdx.x == 0) {
      g->sp_done = 0;
      // a fused-only window has no general path behind it (a non-fused-only window outside the class
      // left the back-off on): hand it to settle()'s replay like a window found outside the class
      if (fo_only) {
        g->fu_fail_epoch = epoch;
        atomicOr(&g->window_error, 8u);
      }
    }
    return;
  }
  const uint32_t i = k * FU_T + threadIdx.x;
  const uint32_t E = w.E;
  const uint64_t base = g->x_count, P = g->x_sorted;
  const u128 x_id_max = g->x_id_max;
  const u128 ovf = g->ovf_bound;
  // window-level condition: the balance fields stay below 2^64 (ovf + 2^20 x 2^43 < 2^64)
  // pn_skip: the host launched no pulse before this window (pulse_next was "never" at its last read);
  // an earlier fused window may have lowered it since (a pending create with a timeout): if a pulse
  // could be due before or inside this window, it leaves the class (replayed with its pulse)
  const bool glob_ok = (uint64_t)(ovf >> 64) == 0 && (uint64_t)ovf < (1ull << 63) && !g->batch_huge &&
                       !(pn_skip && g->pulse_next <= w.T[w.nb - 1]);
  // claim mode: the previous transfer window's ids did not rise (e.g. random ids): in-window
  // duplicates are found by claims instead of by the rising-id test
  const bool claim = g->mono_prev == 0;
  if (k == 0 && threadIdx.x == 0) {
    // what k_fu_final reads while its last block updates the store counts
    g->fu_epoch = epoch;
    g->fu_base = base;
    g->fu_exp_base = g->exp_count;  // (unchanged until k_fu_final's last block)
    g->fu_claim = claim ? 1u : 0u;  // (k_fu_final re-points or removes this window's claims)
    // the window may extend the sorted prefix (first id above every stored id; its ids must rise
    // too: Globals::fu_nonmono, k_fu_final)
    g->fu_prefix = (P == base && U(ev[0].id) > x_id_max) ? 1u : 0u;
  }

  tb_transfer_t t;
  FuEv fe;
  fe.simple = true;
  fe.reach = false;
  fe.code = TB_CT_OK;
  fe.amount = fe.id_key = 0;
  fe.dr = fe.cr = NONE32;
  u128 prev = 0;
  if (!aborted) {
    // the wave's 64 records through LDS in two 64 B halves (16 B per lane per load, row-swizzled so
    // the per-lane row reads are conflict-free), nontemporal: the stream passes by while the account
    // table and records stay in the Infinity Cache (per-lane strided loads measured slower)
    uint4* ws = stage + wave * 256;
    const uint32_t i0 = i - lane;
    const uint32_t nrec = i0 < E ? min(64u, E - i0) : 0u;
    const uint4* src = reinterpret_cast<const uint4*>(ev + i0);
    uint4* tw = reinterpret_cast<uint4*>(&t);
#pragma unroll
    for (int half = 0; half < 2; half++) {
      wave_sync();
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const uint32_t idx = c * 64 + lane, r = idx >> 2, q = idx & 3;
        if (r < nrec) {
          const uint4 v = ld_stream(src + r * 8 + half * 4 + q);
          ws[r * 4 + (q ^ ((r >> 2) & 3))] = v;
          if (HOST) ev_copy[(size_t)(i0 + r) * 8 + half * 4 + q] = v;
        }
      }
      wave_sync();
#pragma unroll
      for (int q = 0; q < 4; q++) tw[half * 4 + q] = ws[lane * 4 + (q ^ ((lane >> 2) & 3))];
    }
    // the previous event's id: the neighbour lane's (lane 0: the previous wave's last event; a wave
    // wholly past the window's end reads nothing, ev ends at E)
    prev = ((u128)__shfl_up(t.id.hi, 1, 64) << 64) | __shfl_up(t.id.lo, 1, 64);
    if (lane == 0 && i > 0 && i < E) prev = U(ev[i - 1].id);
  }
  bool nonmono = false;  // (claim mode: whether the ids rise after all, for the next window)
  fe.pending = false;
  fe.expires_at = 0;
  if (i < E && !aborted) {
    const uint64_t ts = win_ts(w, win_batch(w, i), i);  // :1253 (the record as inserted)
    fu_decide(d, i, prev, t, ts, x_id_max, P, base, &fe, claim, ev, E);
    nonmono = i > 0 && !(U(t.id) > prev);
    t.timestamp = ts;
  }
  // claim mode: every event's claim position (NONE32 where it made none: a wave that skipped its
  // decisions too), for k_fu_final
  if (claim && i < E) fs.cpos[i] = aborted ? NONE32 : fe.cpos;
  const bool blk_simple = __syncthreads_and(fe.simple && !aborted) && glob_ok;
  if (threadIdx.x == 0) {
    fs.applied[k] = blk_simple ? 1 : 0;
    // (a later block that reads this skips its work; k_fu_final reads it after the launch)
    if (!blk_simple) __hip_atomic_store(&g->fu_abort, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (!blk_simple) return;
  const bool ok = i < E && fe.code == TB_CT_OK;
  if (ok) {
    // no-return 64-bit adds: every field stays below 2^64 this window (glob_ok, FU_AMOUNT_MAX)
    (void)atomicAdd(fu_dr_field(d, fe), fe.amount);
    (void)atomicAdd(fu_cr_field(d, fe), fe.amount);
    if (fmark) {
      // write-back stream (changes.h): the accounts this window changed, tagged with its number;
      // counted only if the pass commits the window (k_chg_count)
      fmark[fe.dr] = epoch;
      fmark[fe.cr] = epoch;
    }
  }
  const bool bad = i < E && !ok;
  if (bad) s.code[i] = fe.code;
  const unsigned long long okm = __ballot(ok);
  // a pending create's live expiry entry needs a timestamp the expiry scan can see (composite key)
  const bool pto = ok && fe.expires_at != 0 && !(t.timestamp >> 63) && fe.expires_at <= TB_TIMESTAMP_MAX;
  const unsigned long long pendm = __ballot(ok && fe.pending), ptom = __ballot(pto);
  if (lane == 0 && i < E) {
    fs.ok[i >> 6] = okm;
    fs.pend[i >> 6] = pendm;
    fs.pto[i >> 6] = ptom;
  }
  if (ok) d.xstatus[base + i] = fe.pending ? (uint8_t)TB_PENDING_PENDING : (uint8_t)0;
  if (okm) {  // in place: slot base + i
    const uint32_t first = (uint32_t)__builtin_ctzll(okm);
    fu_store_records(d, reinterpret_cast<const uint4*>(&t), ok, okm, base + (i - lane) + first, stage + wave * 256);
  }
  // this block's failures, reaching amounts' sum and largest reaching id (k_fu_final folds them)
  const uint32_t wbad = (uint32_t)__popcll(__ballot(bad));
  const unsigned long long wsum = wave_sum_u64(fe.reach ? fe.amount : 0ull);
  const u128 wmax = wave_max_u128(fe.reach ? fe.id_key : (u128)0);
  const bool wnm = __ballot(nonmono) != 0;
  // pulse_next (:1576-1581): every ok create with a timeout, visible to the scan or not
  unsigned long long pmin = ok && fe.expires_at ? fe.expires_at : ~0ull;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long y = __shfl_xor(pmin, o, 64);
    pmin = y < pmin ? y : pmin;
  }
  if (lane == 0) {
    lds[wave] = wbad;
    ldsu[wave] = wsum;
    ldsm[wave] = wmax;
    ldsn[wave] = wnm ? 1u : 0u;
    ldsp[wave] = pmin;
    ldsx[wave] = (uint32_t)__popcll(ptom);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t nbad = 0, nm = 0, nexp = 0;
    unsigned long long bsum = 0, bpmin = ~0ull;
    u128 bmax = 0;
#pragma unroll
    for (uint32_t q = 0; q < FU_T / 64; q++) {
      nbad += lds[q];
      bsum += ldsu[q];
      bmax = umax128(bmax, ldsm[q]);
      nm |= ldsn[q];
      bpmin = ldsp[q] < bpmin ? ldsp[q] : bpmin;
      nexp += ldsx[q];
    }
    fs.cnt[k] = nbad;
    if (nexp) {
      // this block's live expiry entries: one reservation per block (k_fu_final writes them; per-wave
      // appends there serialized ~16K same-address atomics per 1M-event window of 1 % pending creates)
      fs.pbase[k] = epoch_count_add(fs.slots + FU_SLOTS + k % FU_SLOTS, epoch, nexp);
    }
    fs.pnmin[k] = bpmin;
    // (claim mode) this block's ids do not rise: the window is hashed, and the next one claims too
    if (nm) __hip_atomic_store(&g->fu_nonmono, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    fs.pay[k] = bsum;
    fs.idmax[k] = bmax;
    // the window's failure count, tagged with its epoch (no reset between windows)
    if (nbad) (void)epoch_count_add(fs.slots + k % FU_SLOTS, epoch, nbad);
  }
}

// After k_ct_fused (same grid). A window outside the class: the balance adds of every block that
// applied them are subtracted (the same decisions from the same inputs) and the general path runs.
// A committed window: replies, batch bases, the records after the first failure moved to their ranks,
// the ids indexed when the records do not extend the sorted prefix, and (last block) the window's
// totals into Globals.
// fo_only: the general path was not launched for this window (host.inc launch_window); a window
// outside the class then stops every later window (window_error bit 3) until the host replays them.
// k: the 256-event group (k_ct_fused's block) of nblk this call finishes.
__device__ __forceinline__ void fu_final_body(const Dev& d, const Scratch& s, const FuScratch& fs,
                                              const tb_transfer_t* __restrict__ ev, const WinDesc& w, uint32_t epoch,
                                              const FinalOut& o, uint32_t fo_only, uint32_t k, uint32_t nblk) {
  __shared__ uint4 stage[FU_T * 4];
  __shared__ uint32_t lds[FU_T / 64];
  __shared__ unsigned long long red[FU_T / 64];
  __shared__ u128 redm[FU_T / 64];
  __shared__ unsigned long long redp[FU_T / 64];
  Globals* g = d.g;
  // (bit 0 only: this kernel itself may set bit 3, and every block must still undo its adds)
  if ((g->window_error & 1u) || g->fu_epoch != epoch) return;  // (k_ct_fused backed off or skipped)
  const uint32_t i = k * FU_T + threadIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t E = w.E;
  if (g->fu_abort == epoch) {
    if (k == 0 && threadIdx.x == 0) {
      g->sp_done = 0;
      const uint32_t fails = g->sp_fails + 1;
      g->sp_fails = fails;
      // back-off capped at FU_BACKOFF_MAX windows: a stream that leaves the class now and then keeps
      // the fused pass for every clean stretch longer than that
      g->sp_skip = fails >= 3 ? FU_BACKOFF_MAX : (1u << fails);
      if (fo_only) {
        g->fu_fail_epoch = epoch;
        atomicOr(&g->window_error, 8u);
      }
    }
    if (i >= E) return;
    // claim mode: every claim of the window reverted to the empty entry it took (blocks that applied or
    // not). The window's claims are the only writes the table had since the previous window, and
    // nothing here probes the table (the undo below reads the ok bitmap), so reverting all of them
    // restores the table exactly: no tombstones accumulate over aborted windows.
    if (g->fu_claim) {
      const uint32_t p = fs.cpos[i];
      if (p != NONE32) d.x_tab[p] = X_EMPTY;
    }
    if (!fs.applied[k]) return;
    // the adds this block applied: its ok events (k_ct_fused's per-wave bitmap, written by every
    // applying block), each to its two accounts' posted or pending fields
    if (!((fs.ok[i >> 6] >> lane) & 1ull)) return;
    const tb_transfer_t& t = ev[i];
    AccEntry ae;
    FuEv fe;
    fe.pending = (t.flags & TB_TRANSFER_PENDING) != 0;
    fe.dr = acc_find(d.acc_tab, d.acc_mask, t.debit_account_id, &ae);
    fe.cr = acc_find(d.acc_tab, d.acc_mask, t.credit_account_id, &ae);
    if (fe.dr == NONE32 || fe.cr == NONE32) return;  // (never: an ok event found both)
    (void)atomicAdd(fu_dr_field(d, fe), 0ull - t.amount.lo);
    (void)atomicAdd(fu_cr_field(d, fe), 0ull - t.amount.lo);
    return;
  }
  const uint64_t base = g->fu_base;
  const bool mono = g->fu_nonmono != epoch;
  const bool prefix_win = g->fu_prefix != 0 && mono;
  __shared__ uint32_t tb_lds;
  if (threadIdx.x < 64) {  // the window's failures: the slots summed by the first wave
    const uint32_t t = wave_sum(fu_slot_count(fs.slots, epoch));
    if (threadIdx.x == 0) tb_lds = t;
  }
  __syncthreads();
  const uint32_t total_bad = tb_lds;
  if (!total_bad && prefix_win && k != nblk - 1 && fs.pnmin[k] == ~0ull) {
    // nothing moves, nothing to index, no expiry entry: only a block where a batch starts has a reply
    // base to write
    const uint32_t lo = k * FU_T, hi = min(E, lo + FU_T), b = win_batch(w, lo);
    if (w.off[b] != lo && !(b + 1 < w.nb && w.off[b + 1] < hi)) return;
  }
  // the failures of the earlier blocks (only a window with failures pays for the sum)
  uint32_t ex_bad = 0;
  if (total_bad) {
    uint32_t v = 0;
    for (uint32_t j = threadIdx.x; j < k; j += FU_T) v += fs.cnt[j];
    ex_bad = block_sum<FU_T / 64>(v, lds);
  }
  const bool ok = i < E && ((fs.ok[i >> 6] >> lane) & 1ull);
  const bool pend = i < E && ((fs.pend[i >> 6] >> lane) & 1ull);
  const bool pto = i < E && ((fs.pto[i >> 6] >> lane) & 1ull);
  const bool bad = i < E && !ok;
  uint32_t tot;
  const uint32_t rbad = ex_bad + (total_bad ? block_excl<FU_T / 64>(bad ? 1u : 0u, lds, &tot) : 0u);
  const uint32_t rins = i - rbad;
  if (i < E) {
    const uint32_t b = win_batch(w, i);
    if (i == w.off[b]) {
      // event i opens batch b and every empty batch just before it
      for (int32_t bb = (int32_t)b; bb >= 0 && w.off[bb] == i; bb--) o.batch_base[bb] = rbad;
    }
    if (bad) {
      tb_create_result_t r;
      r.index = i - w.off[b];
      r.result = s.code[i];
      o.results[rbad] = r;
    }
  }
  if (__ballot(ok && rbad != 0)) {
    // an earlier event failed: this wave's records move down to their ranks (from the input; the
    // branch is wave-uniform, so the run's store loop has every lane)
    // (the record as 16 B words, not a struct whose address is taken: that put it in scratch memory)
    uint4 rec[8];
    const uint4* src = reinterpret_cast<const uint4*>(ev) + (size_t)i * 8;
#pragma unroll
    for (int q = 0; q < 8; q++) rec[q] = ok ? src[q] : make_uint4(0, 0, 0, 0);
    if (ok) {
      rw_stamp(rec, win_ts(w, win_batch(w, i), i));
      d.xstatus[base + rins] = pend ? (uint8_t)TB_PENDING_PENDING : (uint8_t)0;
    }
    const unsigned long long okm = __ballot(ok);
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)rins, (int)__builtin_ctzll(okm));
    fu_store_records(d, rec, ok, okm, base + r0, stage + wave * 256);
  }
  if (g->fu_claim) {
    // claim mode: the ok events' claims index their records already (in a window that extends the
    // sorted prefix too: a record found by both finds the same slot); a record that moved down to its
    // rank is re-pointed
    if (ok && rins != i) {
      const uint32_t p = fs.cpos[i];  // (an ok event of a committed claim window made its claim)
      d.x_tab[p] = (d.x_tab[p] & 0xFFFFFFFF00000000ull) | (uint32_t)(base + rins);
    }
  } else if (ok && !prefix_win) {
    x_insert(d.x_tab, d.x_mask, ev[i].id, (uint32_t)(base + rins));
  }
  if (__syncthreads_or(pto)) {
    // live expires_at entries of the window's pending creates with a timeout, in event order, at this
    // block's reservation (k_ct_fused): after the entries of the slots before its own
    __shared__ uint32_t xbase_lds;
    if (threadIdx.x < 64) {
      const uint32_t c = fu_slot_count(fs.slots + FU_SLOTS, epoch);
      const uint32_t before = wave_sum(threadIdx.x < k % FU_SLOTS ? c : 0u);
      if (threadIdx.x == 0) xbase_lds = before;
    }
    __syncthreads();
    uint32_t nx;
    const uint32_t rx = block_excl<FU_T / 64>(pto ? 1u : 0u, lds, &nx);
    if (pto) {
      ExpEntry x;
      x.expires_at = win_ts(w, win_batch(w, i), i) + (uint64_t)ev[i].timeout * TB_NS_PER_S;
      x.slot = (uint32_t)(base + rins);
      x.pad = 0;
      d.exp[*d.exp_cur][g->fu_exp_base + xbase_lds + fs.pbase[k] + rx] = x;
    }
  }
  if (k == nblk - 1) {
    // the window's totals: the per-block sums folded, the store counts and the window state
    unsigned long long sum = 0, pn = ~0ull;
    u128 mx = 0;
    for (uint32_t j = threadIdx.x; j < nblk; j += FU_T) {
      sum += fs.pay[j];
      mx = umax128(mx, fs.idmax[j]);
      pn = fs.pnmin[j] < pn ? fs.pnmin[j] : pn;
    }
    sum = wave_sum_u64(sum);
    mx = wave_max_u128(mx);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long y = __shfl_xor(pn, o, 64);
      pn = y < pn ? y : pn;
    }
    if (lane == 0) {
      red[wave] = sum;
      redm[wave] = mx;
      redp[wave] = pn;
    }
    __shared__ uint32_t xtot_lds;
    if (threadIdx.x < 64) {  // the window's live expiry entries over all slots
      const uint32_t t = wave_sum(fu_slot_count(fs.slots + FU_SLOTS, epoch));
      if (threadIdx.x == 0) xtot_lds = t;
    }
    __syncthreads();
    const uint32_t xtot = xtot_lds;
    if (threadIdx.x == 0) {
      for (uint32_t q = 1; q < FU_T / 64; q++) {
        sum += red[q];
        mx = umax128(mx, redm[q]);
        pn = redp[q] < pn ? redp[q] : pn;
      }
      if (pn < g->pulse_next) g->pulse_next = pn;  // :1576-1581
      g->exp_count = g->fu_exp_base + xtot;
      const uint32_t total_ins = E - total_bad;
      for (int32_t bb = (int32_t)w.nb; bb >= 0 && w.off[bb] == E; bb--) o.batch_base[bb] = total_bad;
      if (o.out_count) *o.out_count = total_bad;
      g->result_count = total_bad;
      g->base = base;
      if (prefix_win) g->x_sorted = base + total_ins;
      g->x_count = base + total_ins;
      g->win_flags = 1u | (prefix_win ? 2u : 0u);
      g->mono_prev = mono ? 1u : 0u;  // (a window outside claim mode only commits with rising ids)
      g->ovf_bound += (u128)sum;  // below 2^64 (glob_ok, FU_AMOUNT_MAX)
      if (mx > g->x_id_max) g->x_id_max = mx;
      g->windows_applied++;
      g->events_total += E;
      g->w_count = 0;
      g->cpw_want = 0;
      g->rc_last = 0;
      g->sp_done = 1;
      g->sp_fails = 0;
      g->fu_windows++;
    }
  }
}

// The synchronous path's reply (HOST, a fused-only batch): the block that finishes last copies the
// Globals and the reply block (count and results) to pinned host memory through its device mapping,
// as k_reply_out does in its own launch on the other paths (host.inc reply_out).
struct ReplyOut {
  uint4* host;       // h_pinned's device mapping
  uint32_t g16;      // Globals words
  uint32_t reply16;  // the reply block's first word (H_REPLY_OFF / 16), the same on both sides
  uint32_t n_max;
  unsigned long long* flag;  // written with seq after every word (the host polls it)
  unsigned long long seq;
};
template <bool HOST>
__global__ void __launch_bounds__(FU_T) k_fu_final(Dev d, Scratch s, FuScratch fs, const tb_transfer_t* __restrict__ ev,
                                                   WinDesc w, uint32_t epoch, FinalOut o, uint32_t fo_only, ReplyOut ro) {
  // a block finishes every gridDim-th group (a clean window's groups mostly exit at once: fewer,
  // longer-lived blocks than k_ct_fused's grid)
  const uint32_t nblk = (w.E + FU_T - 1) / FU_T;
  for (uint32_t k = blockIdx.x; k < nblk; k += gridDim.x) {
    __syncthreads();  // (the body's LDS words are reused by the next group)
    fu_final_body(d, s, fs, ev, w, epoch, o, fo_only, k, nblk);
  }
  if (HOST) {
    __shared__ uint32_t last;
    if (last_block_done(&d.g->fu_done, &last)) {
      const uint4* dev = reinterpret_cast<const uint4*>(d.g);
      const uint32_t c = min(*reinterpret_cast<const volatile uint32_t*>(dev + ro.reply16), ro.n_max);
      const uint32_t words = ro.g16 + 1u + (c * 8u + 15u) / 16u;
      for (uint32_t k = threadIdx.x; k < words; k += FU_T) {
        const uint32_t j = k < ro.g16 ? k : ro.reply16 + (k - ro.g16);
        ro.host[j] = dev[j];
      }
      __threadfence_system();
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_store(ro.flag, ro.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}
