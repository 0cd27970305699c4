// engine.hip — MI355X batch-apply engine for the StateMachine commit path (libtbgpu.so).
//
// A commit window (window.h: 1..128 consecutive prepared batches, up to the configured event cap)
// runs as six launches on the engine's stream:
//
//   k_*_prep     grid   stateless validation (state_machine.zig:1424-1439, 1465-1489, 1614-1624),
//                       account resolution through 32 B account-table entries (id, slot, ledger,
//                       flags), pre-window transfer id / pending_id resolution, static post/void
//                       evaluation (:1626-1696); every id / pending_id enters a window-local key map;
//                       accounts read by balance-dependent decisions (limits, balancing) become hot.
//   k_classify   grid   order-dependence ("U": duplicate ids, in-window pending targets, contended
//                       pending transfers, balance reads, any overflow risk) and the walker set
//                       W = U + events touching a hot account, closed over linked chains
//                       (one thread per chain head); all other events get their final outcome here,
//                       including whole static chains (first failure + linked_event_failed fill).
//   k_wlist      grid   ordered W list (segment prefix + block scan).
//   k_walk       1 WG   the sequential walker over W only (walker.h).
//   k_final      grid   ordered per-batch replies, insert ranks, inserts (records appended in
//                       timestamp order, id tables, pending status, expires_at list) and the
//                       commutative balance deltas of every non-W event as exact 128-bit atomics.
//
// Outside W every event is order-free by construction, so the window runs fully
// parallel apart from the walker, which carries only the events whose outcome depends on order.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cstddef>
#include <new>
#include <vector>
#include <mutex>
#include <utility>

#include <rocprim/device/device_radix_sort.hpp>

// Onesweep radix sort at every size (merge_sort_limit 0): rocprim's default picks its merge-sort
// path up to 2^20 items, ~11 launches (~140 us) for a 1M-event window's keys.
using SortCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>;

#include "../../include/tbg.h"
#include "dev_common.h"
#include "sm_logic.h"
#include "walker.h"
#include "resolver.h"
#include "relax.h"
#include "chunks.h"
#include "window.h"
#include "changes.h"
#include "restore.h"
#include "query.h"

// k_final's streams, nontemporal: the window's event records (read for the last time) and the
// inserted transfer records pass by, while the account table and records stay cached across windows
// (A/B on one box, cfg2: +1.5-2 % transfers/s, prep 155 -> 148 us per 1M events; k_ct_prep's own
// event loads are 8 strided 16 B loads per lane and get slower nontemporal, 155 -> 189 us).
#ifndef TBG_NT_LOAD
#define TBG_NT_LOAD 1
#endif
#ifndef TBG_NT_STORE
#define TBG_NT_STORE 1
#endif
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_stream(const uint4* p) {
#if TBG_NT_LOAD
  const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
#else
  return *p;
#endif
}
__device__ __forceinline__ void st_stream(uint4* p, uint4 v) {
#if TBG_NT_STORE
  const u32x4_t x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<u32x4_t*>(p));
#else
  *p = v;
#endif
}

// Probe continuation after a first entry was already loaded (lets the first probes of several
// independent lookups be in flight together).
__device__ inline uint32_t acc_probe_from(const AccEntry* __restrict__ tab, uint64_t mask, uint64_t h, AccEntry e,
                                          tb_uint128_t id, AccEntry* out) {
  for (;;) {
    if (e.slot == NONE32) return NONE32;
    if (e.id_lo == id.lo && e.id_hi == id.hi) {
      *out = e;
      return e.slot;
    }
    h = (h + 1) & mask;
    e = tab[h];
  }
}

// A balance-reading decision makes the read account hot for this window: every event touching it
// is then decided in order (resolver.h or the walker). The first marker gets the account a dense
// rank (k_ct_prep: one counter atomic per block, after its marks).
// blk: this block's claimed slots (LDS, MARK_LDS entries): at most one lane per block and account
// goes on to the global exchange (Zipf-hot accounts would serialize every marking lane on one word).
#define MARK_LDS 512
__device__ inline bool mark_first(Dev d, uint32_t slot, uint32_t epoch, uint32_t* blk) {
  // a plain read first: a hot account is marked by many events (a stale read only costs the atomic)
  if (d.hot[slot] == epoch) return false;
  uint32_t h = (slot * 2654435761u) & (MARK_LDS - 1);
  for (int probe = 0; probe < 8; probe++, h = (h + 1) & (MARK_LDS - 1)) {
    const uint32_t k = atomicCAS(&blk[h], NONE32, slot);
    if (k == NONE32) break;  // this lane marks it for the block
    if (k == slot) return false;   // another lane of the block does
  }
  return atomicExch(&d.hot[slot], epoch) != epoch;
}
__device__ inline void hot_rank_set(Dev d, Scratch s, uint32_t slot, uint32_t rank) {
  d.hot_rank[slot] = rank;
  s.bind_slot[rank] = slot;
  s.bind_adv[rank] = 0;
}

// ------------------------------------------------------------------------------------------------
// Non-binding limits. A limit check reads an account's balances (debits_must_not_exceed_credits:
// dp + dpo + amount > cpo, tigerbeetle.zig:31-39); within a window only the window's own debits can
// raise dp + dpo (posts and voids of pending transfers and expiries lower it, credits raise cpo).
// So if the account's balances at the window start plus EVERY debit amount of the window that
// reaches its check still pass (dp + dpo + sum <= cpo), every one of those checks passes whatever
// the order and the other outcomes: the account needs no ordering. The same for credits of a
// credits_must_not_exceed_debits account. Balancing transfers read the balances for their amount:
// their accounts stay hot. k_bind_sum folds the sums per hot rank (LDS hash per block, one global
// add per distinct rank per block: Zipf-hot accounts would serialize on one address otherwise),
// k_bind_decide un-marks the non-binding accounts, k_classify then drops their read bits.
// ------------------------------------------------------------------------------------------------
#define BIND_LDS 4096
#define BIND_T 1024  // threads (events) per k_bind_sum block
#define BIND_FORCE (1ull << 63)
#define BIND_AMOUNT_MAX (1ull << 40)  // larger amounts keep their account hot (the sums stay < 2^63)

__device__ inline void bind_add(Dev d, Scratch s, uint32_t* tk, unsigned long long* tv, uint32_t slot, u128 amount,
                                bool force) {
  const uint32_t r = d.hot_rank[slot];
  if (force || amount >= BIND_AMOUNT_MAX) {
    atomicOr(&s.bind_adv[r], BIND_FORCE);
    return;
  }
  const unsigned long long v = (unsigned long long)amount;
  uint32_t h = (r * 2654435761u) & (BIND_LDS - 1);
  for (int probe = 0; probe < 8; probe++, h = (h + 1) & (BIND_LDS - 1)) {
    uint32_t k = tk[h];
    if (k == NONE32) k = atomicCAS(&tk[h], NONE32, r), k = (k == NONE32) ? r : k;
    if (k == r) {
      atomicAdd(&tv[h], v);
      return;
    }
  }
  atomicAdd(&s.bind_adv[r], v);  // LDS table crowded: straight to memory
}

__global__ void __launch_bounds__(BIND_T) k_bind_sum(Dev d, Scratch s, uint32_t E, uint32_t epoch) {
  __shared__ uint32_t tk[BIND_LDS];
  __shared__ unsigned long long tv[BIND_LDS];
  if (WIN_REJECTED(d.g) || SP_DONE(d.g) || !d.g->hot_count) return;
  for (uint32_t j = threadIdx.x; j < BIND_LDS; j += blockDim.x) {
    tk[j] = NONE32;
    tv[j] = 0;
  }
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < E) {
    const uint32_t cls = s.cls[i];
    const bool bal = cls & C_BAL;
    if (cls & C_READS_DR) bind_add(d, s, tk, tv, s.dr_slot[i], s.amt[i], bal);
    if (cls & C_READS_CR) bind_add(d, s, tk, tv, s.cr_slot[i], s.amt[i], bal);
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < BIND_LDS; j += blockDim.x)
    if (tk[j] != NONE32) atomicAdd(&s.bind_adv[tk[j]], tv[j]);
}

// Per hot rank: un-mark the account when its checks cannot fail this window.
__global__ void __launch_bounds__(256) k_bind_decide(Dev d, Scratch s) {
  Globals* g = d.g;
  if (WIN_REJECTED(g) || SP_DONE(g)) return;
  const uint32_t n = g->hot_count;
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  bool cold = false;
  if (r < n) {
    const unsigned long long adv = s.bind_adv[r];
    if (!(adv & BIND_FORCE)) {
      const uint32_t slot = s.bind_slot[r];
      const tb_account_t& a = d.acc[slot];
      const u128 sum_d = U(a.debits_pending) + U(a.debits_posted), sum_c = U(a.credits_pending) + U(a.credits_posted);
      if (a.flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) {
        const u128 x = sum_d + (u128)adv;
        cold = sum_d >= U(a.debits_pending) && x >= sum_d && x <= U(a.credits_posted);
      } else if (a.flags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS) {
        const u128 x = sum_c + (u128)adv;
        cold = sum_c >= U(a.credits_pending) && x >= sum_c && x <= U(a.debits_posted);
      }
      if (cold) d.hot[slot] = 0;
    }
  }
  const unsigned long long m = __ballot(cold);
  const int lane = threadIdx.x & 63;
  if (m && lane == __builtin_ctzll(m)) atomicAdd(&g->cold_count, (uint32_t)__popcll(m));
  // the accounts that stay hot get compact ranks 0..hot_live-1 (the resolver's keys, chunks.h)
  const unsigned long long live = __ballot(r < n && !cold);
  if (live) {
    const int leader = __builtin_ctzll(live);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&g->hot_live, (uint32_t)__popcll(live));
    base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);  // (leader is wave-uniform)
    if (r < n && !cold) d.hot_rank[s.bind_slot[r]] = base + (uint32_t)__popcll(live & ((1ull << lane) - 1));
  }
}

// Every hot account non-binding: the window reads no balance after all (cpw / order-free paths).
__global__ void k_bind_finish(Globals* g) {
  if (WIN_REJECTED(g) || SP_DONE(g)) return;
  if (g->hot_count && g->cold_count == g->hot_count) g->hot_count = 0;
  g->cold_count = 0;
}

// ------------------------------------------------------------------------------------------------
// create_transfers: prep
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_ct_prep(Dev d, Scratch s, const tb_transfer_t* __restrict__ ev, WinDesc w,
                                                 uint32_t epoch) {
  __shared__ u128 red[256];
  __shared__ uint4 stage[256 * 4];  // half of each event's record (16 KiB): the in-place record store
  // bit 0 huge amount, bit 1 ids not strictly increasing, bit 6 a post/void (either: not claim-free),
  // bit 2 first id above every stored id, bit 3 pulse_next op
  __shared__ uint32_t aux;
  __shared__ u128 id_max[256 / 64];  // per wave: largest id this block may insert (Globals::x_id_max)
  __shared__ uint32_t marked[MARK_LDS];  // mark_first: accounts this block marks
  __shared__ uint32_t nfirst, fbase;      // accounts this block marked first, their first rank
  if (WIN_REJECTED(d.g) || SP_DONE(d.g)) return;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  for (uint32_t j = threadIdx.x; j < MARK_LDS; j += blockDim.x) marked[j] = NONE32;
  if (threadIdx.x == 0) {
    aux = 0;
    nfirst = 0;
  }
  __syncthreads();
  uint32_t first_slot[2] = {NONE32, NONE32};  // accounts this event marked first (debit, credit side)
  u128 amount_upper = 0;
  tb_transfer_t t;  // the event, stamped (also the record a plain create stores in place)
  bool prec = false;
  u128 my_id = 0;  // the id, if the event reaches the exists check (an upper bound of what it may store)
  if (i < w.E) {
    const u128 x_id_max = d.g->x_id_max;
    const uint64_t P = d.g->x_sorted;
    // speculation: claim-free like the previous window (k_claim_fix claims if it was not)
    const bool spec = d.g->mono_prev != 0;
    t = ev[i];
    const uint8_t* evb = reinterpret_cast<const uint8_t*>(ev);
    const uint32_t b = win_batch(w, i);
    {
      // claim-free: ids strictly increasing (u128 order) over the window (bit 1) and no post/void
      // (bit 6); the records extend the sorted prefix with rising fresh ids, post/voids or not
      if (t.flags & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) atomicOr(&aux, 64u);
      if (i > 0 && !(U(t.id) > U(ev[i - 1].id))) atomicOr(&aux, 2u);
      if (i == 0 && U(t.id) > x_id_max) atomicOr(&aux, 4u);
    }
    uint32_t cls = 0, code;
    uint32_t dr_slot = NONE32, cr_slot = NONE32, id_tslot = NONE32, p_tslot = NONE32, id_ent = NONE32,
             pid_ent = NONE32;
    u128 amt = 0, pamt = 0;
    uint64_t pnv = 0;
    const uint16_t f = t.flags;
    if (f & TB_TRANSFER_LINKED) cls |= C_LINKED;
    if (t.timestamp != 0) {
      cls |= C_TSNZ | C_STATIC;
      code = TB_CT_TIMESTAMP_MUST_BE_ZERO;
    } else {
      t.timestamp = win_ts(w, b, i);  // :1253
      code = ct_head(t);
      if (code != CONT) {
        cls |= C_STATIC;
      } else if (f & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) {
        cls |= C_POSTVOID | ((f & TB_TRANSFER_POST_PENDING) ? C_POST : 0);
        code = pv_validate(t);
        if (code != CONT) {
          cls |= C_STATIC;
        } else {
          cls |= C_REACH;
          const uint64_t hx = hash_id(t.id.lo, t.id.hi);
          const uint64_t hp = hash_id(t.pending_id.lo, t.pending_id.hi);
          const bool mx = x_may_exist(t.id, x_id_max), mp = x_may_exist(t.pending_id, x_id_max);
          const XEntry ex = mx ? d.x_tab[hx & d.x_mask] : X_EMPTY;
          const XEntry ep = mp ? d.x_tab[hp & d.x_mask] : X_EMPTY;
          if (!spec) {  // a post/void window is never claim-free: under speculation k_claim_fix claims
            id_ent = bmap_claim(s.bmap, s.bmask, evb, t.id, i, 0, epoch);
            pid_ent = bmap_claim(s.bmap, s.bmask, evb, t.pending_id, i, 1, epoch);
          }
          id_tslot = x_probe_from(d.x_tab, d.xr, d.x_mask, hx, ex, t.id);
          p_tslot = x_probe_from(d.x_tab, d.xr, d.x_mask, hp, ep, t.pending_id);
          if (id_tslot == NONE32 && mx) id_tslot = x_prefix_find(d.xr, P, t.id);
          if (p_tslot == NONE32 && mp) p_tslot = x_prefix_find(d.xr, P, t.pending_id);
          if (p_tslot == NONE32) {
            code = TB_CT_PENDING_TRANSFER_NOT_FOUND;  // unless created in-window (then U)
          } else {
            cls |= C_PV_PREBATCH;
            const tb_transfer_t p = d.xr[p_tslot];
            if ((p.flags & TB_TRANSFER_PENDING) && p.timeout > 0) {
              // if it runs ok, it removes p's expires_at entry and may reset pulse_next (:1698-1708):
              // only if expires_at == pulse_next then, which is <= its value now (after this
              // window's pulse; it only falls inside a window until a reset)
              pnv = expires_at_of(p);
              cls |= C_PNOP;
              if (pnv <= d.g->pulse_next) atomicOr(&aux, 16u);
            }
            code = pv_against(t, p, &amt);
            if (p.flags & TB_TRANSFER_PENDING) {
              AccEntry de, ce;
              dr_slot = acc_find(d.acc_tab, d.acc_mask, p.debit_account_id, &de);
              cr_slot = acc_find(d.acc_tab, d.acc_mask, p.credit_account_id, &ce);
              if ((dr_slot != NONE32 && (de.flags & TB_ACCOUNT_HISTORY)) ||
                  (cr_slot != NONE32 && (ce.flags & TB_ACCOUNT_HISTORY)))
                cls |= C_HIST;
            }
            if (code == CONT && id_tslot != NONE32) code = pv_exists(t, d.xr[id_tslot], p);
            if (code == CONT) {
              uint8_t pst = d.xstatus[p_tslot];
              // a pulse of the window expired p at or before this batch (xwin.h)
              if (pst == TB_PENDING_PENDING && xw_expired_before(w, p, b)) pst = TB_PENDING_EXPIRED;
              code = pv_status(pst);
            }
            if (code == CONT) {
              cls |= C_INSERT;
              pamt = U(p.amount);
              if (p.timeout > 0 && expires_at_of(p) <= t.timestamp)
                code = TB_CT_PENDING_TRANSFER_EXPIRED;  // inserted anyway (:1689-1696)
              else
                code = TB_CT_OK;
            }
          }
        }
      } else {
        code = ct_validate(t);
        if (code != CONT) {
          cls |= C_STATIC;
        } else {
          // Three independent probes in flight together.
          const uint64_t hd = hash_id(t.debit_account_id.lo, t.debit_account_id.hi) & d.acc_mask;
          const uint64_t hc = hash_id(t.credit_account_id.lo, t.credit_account_id.hi) & d.acc_mask;
          const uint64_t hx = hash_id(t.id.lo, t.id.hi);
          const AccEntry ed = d.acc_tab[hd], ec = d.acc_tab[hc];
          const XEntry ex = x_may_exist(t.id, x_id_max) ? d.x_tab[hx & d.x_mask] : X_EMPTY;
          AccEntry de, ce;
          dr_slot = acc_probe_from(d.acc_tab, d.acc_mask, hd, ed, t.debit_account_id, &de);
          cr_slot = acc_probe_from(d.acc_tab, d.acc_mask, hc, ec, t.credit_account_id, &ce);
          if (dr_slot == NONE32)
            code = TB_CT_DEBIT_ACCOUNT_NOT_FOUND;
          else if (cr_slot == NONE32)
            code = TB_CT_CREDIT_ACCOUNT_NOT_FOUND;
          else
            code = ct_ledgers(t, de.ledger, ce.ledger);
          if (code != CONT) {
            cls |= C_STATIC;
          } else {
            cls |= C_REACH;
            if ((de.flags | ce.flags) & TB_ACCOUNT_HISTORY) cls |= C_HIST;
            id_ent = spec ? bmap_direct(s.bmap, s.bmask, i, epoch) : bmap_claim(s.bmap, s.bmask, evb, t.id, i, 0, epoch);
            const bool bal = f & (TB_TRANSFER_BALANCING_DEBIT | TB_TRANSFER_BALANCING_CREDIT);
            amount_upper = U(t.amount);
            if (bal && amount_upper == 0) amount_upper = (u128)0xFFFFFFFFFFFFFFFFull;
            id_tslot = x_probe_from(d.x_tab, d.xr, d.x_mask, hx, ex, t.id);
            if (id_tslot == NONE32 && x_may_exist(t.id, x_id_max)) id_tslot = x_prefix_find(d.xr, P, t.id);
            if (id_tslot != NONE32) {
              code = ct_exists(t, d.xr[id_tslot]);
            } else {
              if (f & TB_TRANSFER_PENDING) cls |= C_PENDING;
              // A balance-reading decision makes the read account hot for this window (every event
              // touching it then runs on the walker, in order).
              if ((de.flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) || (f & TB_TRANSFER_BALANCING_DEBIT))
                cls |= C_READS_DR;
              if ((ce.flags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS) || (f & TB_TRANSFER_BALANCING_CREDIT))
                cls |= C_READS_CR;
              if (f & (TB_TRANSFER_BALANCING_DEBIT | TB_TRANSFER_BALANCING_CREDIT)) cls |= C_BAL;
              amt = U(t.amount);
              // Overflow checks cannot fail in an overflow-free window (checked in k_classify).
              if (ovf64(t.timestamp, (uint64_t)t.timeout * TB_NS_PER_S)) {
                code = TB_CT_OVERFLOWS_TIMEOUT;
              } else {
                code = TB_CT_OK;
                cls |= C_INSERT;
                if (!(f & TB_TRANSFER_PENDING)) {
                  // the stamped record goes to its own position (stored below): final if every
                  // earlier event of the window inserts (k_final then neither re-reads the event
                  // nor stores it)
                  cls |= C_PREP_REC;
                }
                if ((f & TB_TRANSFER_PENDING) && t.timeout > 0) {
                  // if it runs ok, pulse_next = min(pulse_next, expires_at) (:1576-1581)
                  pnv = t.timestamp + (uint64_t)t.timeout * TB_NS_PER_S;
                  cls |= C_PNOP;
                  if (w.xwin) s.pn_rb[i] = 0xFFFFu;  // not removed (k_xwin_rb)
                }
              }
            }
          }
        }
      }
    }
    if ((uint64_t)(amount_upper >> 64) != 0) atomicOr(&aux, 1u);
    if (cls & C_PNOP) {
      s.pnv[i] = pnv;
      atomicOr(&aux, 8u);
    }
    if (cls & C_HIST) atomicOr(&aux, 32u);
    if (cls & C_REACH) my_id = U(t.id);
    if ((i & (SEG - 1)) == 0) {  // the segment counts k_classify accumulates
      s.cnt_w[i / SEG] = 0;
      s.cnt_bad[i / SEG] = 0;
      s.cnt_ins[i / SEG] = 0;
    }
    prec = (cls & C_PREP_REC) != 0;
    // Hot marks: the first marker of an account this window gives it the next dense rank.
    if ((cls & C_READS_DR) && mark_first(d, dr_slot, epoch, marked)) first_slot[0] = dr_slot;
    if ((cls & C_READS_CR) && mark_first(d, cr_slot, epoch, marked)) first_slot[1] = cr_slot;
    s.code[i] = code;
    s.cls[i] = cls;
    s.batch[i] = (uint16_t)b;
    s.dr_slot[i] = dr_slot;
    s.cr_slot[i] = cr_slot;
    s.id_tslot[i] = id_tslot;
    s.p_tslot[i] = p_tslot;
    s.id_ent[i] = id_ent;
    s.pid_ent[i] = pid_ent;
    s.wrow[2 * i] = make_uint4(code, id_tslot, id_ent, pid_ent);
    s.wrow[2 * i + 1] = make_uint4(dr_slot, cr_slot, p_tslot, b);
    s.amt[i] = amt;
    if (cls & C_POSTVOID) s.pamt[i] = pamt;  // read only for post/void events (k_final)
    s.ins[i] = 0;
  }
  // The wave's records at slots base + i0 .. base + i0 + 63, through LDS in two halves (64 B of
  // each record per round), so each store instruction writes whole 64 B sectors instead of 16 B
  // pieces of 64 records. Lanes without a record write garbage rows: such a slot is either beyond
  // the window's insert count or rewritten by k_final (the event ranked there is not in place).
  if (__ballot(prec) != 0) {
    const uint32_t lane = threadIdx.x & 63, i0 = i - lane;
    const uint32_t nrec = i0 < w.E ? min(64u, w.E - i0) : 0u;
    uint4* ws = stage + (threadIdx.x >> 6) * 256;
    const uint4* src = reinterpret_cast<const uint4*>(&t);
    uint4* dst = reinterpret_cast<uint4*>(d.xr + (d.g->x_count + i0));
#pragma unroll
    for (int half = 0; half < 2; half++) {
      wave_sync();
#pragma unroll
      for (int q = 0; q < 4; q++) ws[lane * 4 + q] = src[half * 4 + q];
      wave_sync();
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t idx = k * 64 + lane, r = idx >> 2, q = idx & 3;
        if (r < nrec) st_stream(dst + r * 8 + half * 4 + q, ws[idx]);
      }
    }
  }
  // Window amount bound: block reduction into this block's partial (k_prep_reduce sums them; a
  // same-address atomic per block serializes thousands of blocks on one memory-side word).
  {
    // dense ranks for the accounts this block marked first: one counter atomic per block
    const bool f0 = first_slot[0] != NONE32, f1 = first_slot[1] != NONE32;
    uint32_t k0 = 0, k1 = 0;
    if (f0) k0 = atomicAdd(&nfirst, 1u);
    if (f1) k1 = atomicAdd(&nfirst, 1u);
    if (__syncthreads_or(f0 || f1)) {
      if (threadIdx.x == 0) fbase = atomicAdd(&d.g->hot_count, nfirst);
      __syncthreads();
      if (f0) hot_rank_set(d, s, first_slot[0], fbase + k0);
      if (f1) hot_rank_set(d, s, first_slot[1], fbase + k1);
    }
  }
  {
    const u128 wm = wave_max_u128(my_id);
    if ((threadIdx.x & 63) == 0) id_max[threadIdx.x >> 6] = wm;
  }
  red[threadIdx.x] = ((uint64_t)(amount_upper >> 64) != 0) ? 0 : amount_upper;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    s.blk_amt[blockIdx.x] = red[0];
    s.blk_aux[blockIdx.x] = aux;
    // an upper bound of every id this window may store (the failures' ids included; k_prep_reduce
    // folds the blocks' exact maxima)
    u128 m = id_max[0];
    for (int q = 1; q < 256 / 64; q++) m = umax128(m, id_max[q]);
    s.blk_idmax[blockIdx.x] = m;
  }
}

// One block: folds the prep blocks' partials into Globals (window amount sum, huge flag) before
// k_classify reads them. Sums of < 2^64 amounts over <= 2^20 events cannot wrap 128 bits.
__device__ inline u128 block_sum_u128(u128 v, u128* lds) {
  lds[threadIdx.x] = v;
  __syncthreads();
  for (uint32_t off = blockDim.x / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off) lds[threadIdx.x] += lds[threadIdx.x + off];
    __syncthreads();
  }
  return lds[0];
}

__global__ void __launch_bounds__(1024) k_prep_reduce(Dev d, Scratch s, uint32_t nblk) {
  __shared__ u128 red[1024];
  __shared__ u128 idm[1024 / 64];
  __shared__ uint32_t aux;
  if (WIN_REJECTED(d.g) || SP_DONE(d.g)) return;
  if (threadIdx.x == 0) aux = 0;
  __syncthreads();
  u128 v = 0, m = 0;
  uint32_t a = 0;
  for (uint32_t j = threadIdx.x; j < nblk; j += 1024) {
    v += s.blk_amt[j];
    a |= s.blk_aux[j];
    m = umax128(m, s.blk_idmax[j]);
  }
  if (a) atomicOr(&aux, a);
  m = wave_max_u128(m);
  if ((threadIdx.x & 63) == 0) idm[threadIdx.x >> 6] = m;
  const u128 tot = block_sum_u128(v, red);  // (its barriers order the idm stores)
  if (threadIdx.x == 0) {
    Globals* g = d.g;
    g->batch_amount_sum += tot;
    if (aux & 1u) g->batch_huge = 1;
    const bool claim_free = !(aux & (2u | 64u));
    const bool prefix = !(aux & 2u) && (aux & 4u) && g->x_sorted == g->x_count;
    // bit 2: pulse_next ops; bit 3: a post/void that may reset pulse_next (k_final replays the
    // window's ops in order only then; else pulse_next = min(itself, the creations that ran ok))
    // bit 4: history rows: the sequential walker (exact balances after each event) decides W
    g->win_flags = (claim_free ? 1u : 0u) | (prefix ? 2u : 0u) | ((aux & 8u) ? 4u : 0u) | ((aux & 16u) ? 8u : 0u) |
                   ((aux & 32u) ? 16u : 0u);
    // every balance field stays below 2^64 this window (k_walk computes the same for k_final; the
    // component walkers, which run before k_walk, read it from here)
    const u128 sum = g->ovf_bound + g->batch_amount_sum;
    g->small_win = !g->batch_huge && sum >= g->ovf_bound && (uint64_t)(sum >> 64) == 0;
    u128 wm = idm[0];
    for (int q = 1; q < 1024 / 64; q++) wm = umax128(wm, idm[q]);
    if (wm > g->x_id_max) g->x_id_max = wm;
  }
}

// After k_prep_reduce: a window k_ct_prep treated as claim-free (speculation, Globals::mono_prev)
// that is not gets its key-map claims here, before anything reads the map.
__global__ void __launch_bounds__(256) k_claim_fix(Dev d, Scratch s, const tb_transfer_t* __restrict__ ev, uint32_t E,
                                                   uint32_t epoch) {
  if (WIN_REJECTED(d.g) || SP_DONE(d.g) || !d.g->mono_prev || (d.g->win_flags & 1u)) return;
  // grid-stride over a capped grid: the common case (speculation right) is a launch whose blocks
  // exit at once, so it pays for few blocks
  const uint8_t* evb = reinterpret_cast<const uint8_t*>(ev);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < E; i += gridDim.x * blockDim.x) {
    const uint32_t cls = s.cls[i];
    if (!(cls & C_REACH)) continue;
    const uint32_t ie = bmap_claim(s.bmap, s.bmask, evb, ev[i].id, i, 0, epoch);
    s.id_ent[i] = ie;
    s.wrow[2 * i].z = ie;
    if (cls & C_POSTVOID) {
      const uint32_t pe = bmap_claim(s.bmap, s.bmask, evb, ev[i].pending_id, i, 1, epoch);
      s.pid_ent[i] = pe;
      s.wrow[2 * i].w = pe;
    }
  }
}


// ------------------------------------------------------------------------------------------------
// create_transfers: link
// ------------------------------------------------------------------------------------------------
__device__ inline bool window_ovf_mode(const Globals* g) {
  if (g->batch_huge) return true;
  return ovf128(g->ovf_bound, g->batch_amount_sum);
}

// ------------------------------------------------------------------------------------------------
// create_accounts: prep
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_ca_prep(Dev d, Scratch s, const tb_account_t* __restrict__ ev, WinDesc w,
                                                 uint32_t epoch) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= w.E || WIN_REJECTED(d.g)) return;
  const tb_account_t a = ev[i];
  const uint32_t b = win_batch(w, i);
  if ((i & (SEG - 1)) == 0) {  // the segment counts k_classify accumulates
    s.cnt_w[i / SEG] = 0;
    s.cnt_bad[i / SEG] = 0;
    s.cnt_ins[i / SEG] = 0;
  }
  uint32_t cls = 0, code, id_ent = NONE32, slot = NONE32;
  if (a.flags & TB_ACCOUNT_LINKED) cls |= C_LINKED;
  if (a.timestamp != 0) {
    cls |= C_TSNZ | C_STATIC;
    code = TB_CA_TIMESTAMP_MUST_BE_ZERO;
  } else {
    code = ca_validate(a);
    if (code != CONT) {
      cls |= C_STATIC;
    } else {
      cls |= C_REACH;
      id_ent = bmap_claim(s.bmap, s.bmask, reinterpret_cast<const uint8_t*>(ev), a.id, i, 0, epoch);
      AccEntry e;
      slot = acc_find(d.acc_tab, d.acc_mask, a.id, &e);
      if (slot != NONE32) {
        code = ca_exists(a, d.acc[slot]);
      } else {
        code = TB_CA_OK;
        cls |= C_INSERT;
      }
    }
  }
  s.code[i] = code;
  s.cls[i] = cls;
  s.batch[i] = (uint16_t)b;
  s.id_ent[i] = id_ent;
  s.pid_ent[i] = NONE32;
  s.id_tslot[i] = slot;
  s.dr_slot[i] = NONE32;
  s.cr_slot[i] = NONE32;
  s.ins[i] = 0;
}

// ------------------------------------------------------------------------------------------------
// classify: W closure over chains + final outcome of every non-W event.
// ------------------------------------------------------------------------------------------------
// U: the event's outcome depends on order or state.
template <bool XFER>
__device__ inline bool is_u(const Scratch& s, uint32_t j, uint32_t cls, uint32_t epoch, bool ovf_mode,
                            bool claim_free) {
  if (!(cls & C_REACH)) return false;
  if (!XFER) return bmap_idc(s.bmap, s.id_ent[j], epoch) > 1;  // duplicate account id in the window
  if (ovf_mode || (cls & (C_READS_DR | C_READS_CR | C_HIST))) return true;
  if (claim_free) return false;  // no id repeats and no post/void in the window (k_prep_reduce)
  const uint32_t e = s.id_ent[j];
  // duplicate transfer id, or a post/void in the window targets this id
  if (bmap_idc(s.bmap, e, epoch) > 1 || bmap_pidc(s.bmap, e, epoch) > 0) return true;
  if (cls & C_POSTVOID) {
    // pending transfer created in the window, or several post/voids of one pending transfer
    const uint32_t pe = s.pid_ent[j];
    if (bmap_idc(s.bmap, pe, epoch) > 0 || bmap_pidc(s.bmap, pe, epoch) > 1) return true;
  }
  return false;
}

// W: runs on the walker (U, or touches an account some U event reads).
template <bool XFER>
__device__ inline bool is_w(const Dev& d, const Scratch& s, uint32_t j, uint32_t* cls, uint32_t epoch, bool ovf_mode,
                            bool claim_free, bool any_hot) {
  // a read of a non-binding account (k_bind_decide un-marked it) passes whatever the order
  if (XFER && (*cls & (C_READS_DR | C_READS_CR)) && !(*cls & C_BAL)) {
    if ((*cls & C_READS_DR) && d.hot[s.dr_slot[j]] != epoch) *cls &= ~C_READS_DR;
    if ((*cls & C_READS_CR) && d.hot[s.cr_slot[j]] != epoch) *cls &= ~C_READS_CR;
  }
  if (is_u<XFER>(s, j, *cls, epoch, ovf_mode, claim_free)) {
    *cls |= C_U;
    return true;
  }
  if (!XFER || !(*cls & C_REACH) || !any_hot) return false;
  const uint32_t dr = s.dr_slot[j], cr = s.cr_slot[j];
  return (dr != NONE32 && d.hot[dr] == epoch) || (cr != NONE32 && d.hot[cr] == epoch);
}

// A W event outside the resolver's class (resolver.h) sends the whole window to the walker.
__device__ inline bool res_bad(const Scratch& s, uint32_t j, uint32_t cls, uint32_t epoch) {
  if (cls & (C_LINKED | C_POSTVOID | C_BAL | C_HIST)) return true;
  if (!(cls & C_REACH)) return false;
  const uint32_t e = s.id_ent[j];
  return bmap_idc(s.bmap, e, epoch) > 1 || bmap_pidc(s.bmap, e, epoch) > 0;
}

// The walker's id fact for a W transfer event: claim-free windows give every id a private entry.
template <bool XFER>
__device__ inline uint32_t id_alone_bit(const Scratch& s, uint32_t j, uint32_t cls, uint32_t epoch, bool claim_free) {
  if (!XFER || !(cls & C_REACH)) return 0u;
  return (claim_free || bmap_idc(s.bmap, s.id_ent[j], epoch) == 1) ? C_IDALONE : 0u;
}

// Segment counts (W events; failures and inserts of the others), kept by the thread that decides
// each event: its block's segment in `packed` (11-bit fields: W | bad << 11 | inserted << 22, at most
// SEG each), another segment's (a chain running past the segment end) by global atomics. The
// counters were zeroed by the window's prep kernel.
struct SegTally {
  uint32_t seg, packed;
  __device__ void add(const Scratch& s, uint32_t j, uint32_t cls, uint32_t code) {
    const bool w = cls & C_W;
    const uint32_t v = w ? 1u : (((code != TB_CT_OK) ? 1u << 11 : 0u) | ((cls & C_INSERTED) ? 1u << 22 : 0u));
    const uint32_t sg = j / SEG;
    if (sg == seg) {
      packed += v;
      return;
    }
    if (v & 0x7FFu) atomicAdd(&s.cnt_w[sg], 1u);
    if (v & (1u << 11)) atomicAdd(&s.cnt_bad[sg], 1u);
    if (v & (1u << 22)) atomicAdd(&s.cnt_ins[sg], 1u);
  }
};

template <bool XFER>
__device__ inline bool classify_event(const Dev& d, const Scratch& s, const WinDesc& w, uint32_t i, uint32_t epoch,
                                      bool ovf_mode, bool claim_free, bool any_hot, SegTally& t) {
  const uint32_t b = s.batch[i];
  const uint32_t first = w.off[b], last = w.off[b + 1] - 1;
  uint32_t cls = s.cls[i];
  const bool linked = cls & C_LINKED;
  if (i != first && (s.cls[i - 1] & C_LINKED)) return false;  // chain member: its head decides
  if (!linked) {
    // singleton (:1255-1259, :1289-1290)
    if (is_w<XFER>(d, s, i, &cls, epoch, ovf_mode, claim_free, any_hot)) {
      s.cls[i] = cls | C_W | id_alone_bit<XFER>(s, i, cls, epoch, claim_free);
      t.add(s, i, C_W, 0);
      return res_bad(s, i, cls, epoch);
    }
    const uint32_t code = s.code[i];
    const uint32_t fin = cls | (code == TB_CT_OK ? C_COMMIT : 0) | ((cls & C_INSERT) ? C_INSERTED : 0);
    s.cls[i] = fin;
    t.add(s, i, fin, code);
    return false;
  }
  // chain head: members i..end, end = first unlinked event or the batch's last event (:1240-1300)
  uint32_t end = i;
  bool any_w = false;
  uint32_t f = NONE32;
  for (uint32_t j = i;; j++) {
    uint32_t cj = s.cls[j];
    if (is_w<XFER>(d, s, j, &cj, epoch, ovf_mode, claim_free, any_hot)) any_w = true;
    const bool lj = cj & C_LINKED;
    const uint32_t code = (lj && j == last) ? (uint32_t)TB_CT_LINKED_EVENT_CHAIN_OPEN : s.code[j];
    if (code != TB_CT_OK && f == NONE32) f = j;
    end = j;
    if (!lj || j == last) break;
  }
  for (uint32_t j = i; j <= end; j++) {
    const uint32_t cj = s.cls[j];
    if (any_w) {
      s.cls[j] = cj | C_W | id_alone_bit<XFER>(s, j, cj, epoch, claim_free);
      t.add(s, j, C_W, 0);
      continue;
    }
    uint32_t code = s.code[j];
    if ((cj & C_LINKED) && j == last)
      code = TB_CT_LINKED_EVENT_CHAIN_OPEN;
    else if (f != NONE32 && f != j)
      code = TB_CT_LINKED_EVENT_FAILED;
    const bool commit = f == NONE32;
    s.code[j] = code;
    // members before the first failure ran ok before the rollback (their pulse_next ops stand)
    const uint32_t ranok = (f != NONE32 && j < f) ? C_RANOK : 0u;
    const uint32_t fin = cj | ranok | (commit ? C_COMMIT : 0) | ((commit && (cj & C_INSERT)) ? C_INSERTED : 0);
    s.cls[j] = fin;
    t.add(s, j, fin, code);
  }
  return any_w;  // a chain in W: walker
}

template <bool XFER>
__global__ void __launch_bounds__(256) k_classify(Dev d, Scratch s, WinDesc w, uint32_t epoch) {
  __shared__ uint32_t lds[4];
  if (WIN_REJECTED(d.g) || SP_DONE(d.g)) return;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  SegTally t{blockIdx.x * 256u / SEG, 0u};
  const bool ovf_mode = XFER && window_ovf_mode(d.g);
  bool bad = false;
  // transfer windows: claim-free (k_prep_reduce) skips the key-map reads, no hot account skips the
  // hot-mark reads
  const bool claim_free = XFER && (d.g->win_flags & 1u) != 0;
  const bool any_hot = !XFER || d.g->hot_count != 0;
  if (i < w.E) bad = classify_event<XFER>(d, s, w, i, epoch, ovf_mode, claim_free, any_hot, t);
  if (XFER && i == 0) {
    // the resolver's 128-bit signed arithmetic needs every balance sum below 2^126
    const u128 sum = d.g->ovf_bound + d.g->batch_amount_sum;
    if (ovf_mode || (sum >> 126) != 0) bad = true;
  }
  // a sticky flag: read before the atomic (same-address atomics from every wave serialize)
  if (XFER && __any(bad) && (threadIdx.x & 63) == 0 && !__hip_atomic_load(&d.g->res_inelig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    atomicOr(&d.g->res_inelig, 1u);
  // this block's share of its segment's counts (four blocks per segment)
  const uint32_t c = block_sum<4>(t.packed, lds);
  if (threadIdx.x == 0) {
    if (c & 0x7FFu) atomicAdd(&s.cnt_w[t.seg], c & 0x7FFu);
    if ((c >> 11) & 0x7FFu) atomicAdd(&s.cnt_bad[t.seg], (c >> 11) & 0x7FFu);
    if (c >> 22) atomicAdd(&s.cnt_ins[t.seg], c >> 22);
  }
}

#include "cpw.h"
#include "cps.h"

// ------------------------------------------------------------------------------------------------
// The ordered W list (one event per thread, one 1024-event segment per block; k_classify counted).
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(SEG) k_wlist(const Globals* g, Scratch s, uint32_t E) {
  __shared__ uint32_t lds[SEG / 64];
  if (SP_DONE(g) || s.cnt_w[blockIdx.x] == 0) return;  // uniform per block
  const uint32_t prefix = seg_prefix<SEG>(s.cnt_w, blockIdx.x, lds);
  const uint32_t i = blockIdx.x * SEG + threadIdx.x;
  const uint32_t w = (i < E && (s.cls[i] & C_W)) ? 1u : 0u;
  uint32_t tot;
  const uint32_t pos = prefix + block_excl<SEG / 64>(w, lds, &tot);
  if (w) s.wlist[pos] = i;
}

// ------------------------------------------------------------------------------------------------
// The walker (one workgroup; thread 0 walks, then the block folds W outcomes into the counts).
// ------------------------------------------------------------------------------------------------
#define WALK_THREADS 1024
#define MAX_SEGS 1024

template <bool XFER>
__global__ void __launch_bounds__(WALK_THREADS) k_walk(Dev d, Scratch s, const uint8_t* ev, WinDesc w,
                                                        uint32_t nseg, uint32_t epoch) {
  __shared__ uint32_t lds[WALK_THREADS / 64];
  __shared__ uint32_t sbad[MAX_SEGS], sins[MAX_SEGS];
  if (WIN_REJECTED(d.g) || SP_DONE(d.g)) return;
  if (threadIdx.x == 0) {
    Globals* g = d.g;
    g->base = XFER ? g->x_count : g->acc_count;
    // Every balance field <= ovf_bound; if ovf_bound + Σ window amounts < 2^64, no field leaves its
    // low word during the window, so k_final's commutative adds are exact as 64-bit adds.
    const u128 sum = g->ovf_bound + g->batch_amount_sum;
    g->small_win = XFER && !g->batch_huge && sum >= g->ovf_bound && (uint64_t)(sum >> 64) == 0;
  }
  uint32_t v = 0;
  for (uint32_t j = threadIdx.x; j < nseg; j += WALK_THREADS) v += s.cnt_w[j];
  const uint32_t w_count = block_sum<WALK_THREADS / 64>(v, lds);
  if (threadIdx.x == 0) {
    // the host launches the component walkers only while recent windows had W events they could
    // take (no hot account): balance-limit windows (resolver) skip their launches and sort
    d.g->cpw_want = (d.g->cpw_want & 2u) | (w_count != 0 && cpw_active(d.g) ? 1u : 0u);
  }
  if (w_count == 0) {
    if (threadIdx.x == 0) {
      d.g->events_total += w.E;
      d.g->w_count = 0;
    }
    return;
  }
  if (threadIdx.x == 0) d.g->w_count = w_count;
  if (XFER && d.g->res_done) {
    // resolver.h decided every W event and folded them into the segment counts
    if (threadIdx.x == 0) {
      d.g->res_events_total += w_count;
      d.g->events_total += w.E;
    }
    return;
  }
  if (d.g->cpw_done) {  // cpw.h walked W; k_wfold folds the outcomes with the whole grid
    if (threadIdx.x == 0) {
      d.g->cpw_events_total += w_count;
      d.g->events_total += w.E;
    }
    return;
  }
  if (threadIdx.x == 0) {
    Walker wk;
    wk.d = d;
    wk.s = s;
    wk.ev = ev;
    wk.w = &w;
    wk.epoch = epoch;
    wk.atomic_bal = false;
    wk.template run<XFER>(s.wlist, w_count);
    d.g->w_events_total += w_count;
    d.g->events_total += w.E;
  }
  for (uint32_t j = threadIdx.x; j < nseg; j += WALK_THREADS) {
    sbad[j] = 0;
    sins[j] = 0;
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < w_count; k += WALK_THREADS) {
    const uint32_t i = s.wlist[k];
    const uint32_t seg = i / SEG;
    if (s.code[i] != TB_CT_OK) atomicAdd(&sbad[seg], 1u);
    if (s.ins[i]) atomicAdd(&sins[seg], 1u);
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < nseg; j += WALK_THREADS) {
    if (sbad[j]) s.cnt_bad[j] += sbad[j];
    if (sins[j]) s.cnt_ins[j] += sins[j];
  }
}

// The W outcomes of a component-walked window into the segment counts (k_walk folds the sequential
// walker's own): per block an LDS histogram over the segments, then one global add per non-zero bin.
__global__ void __launch_bounds__(1024) k_wfold(Dev d, Scratch s, uint32_t nseg) {
  __shared__ uint32_t sbad[MAX_SEGS], sins[MAX_SEGS];
  if (WIN_REJECTED(d.g) || !d.g->cpw_done) return;
  const uint32_t w_count = d.g->w_count;
  for (uint32_t j = threadIdx.x; j < nseg; j += blockDim.x) sbad[j] = sins[j] = 0;
  __syncthreads();
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < w_count; k += gridDim.x * blockDim.x) {
    const uint32_t i = s.wlist[k];
    const uint32_t seg = i / SEG;
    if (s.code[i] != TB_CT_OK) atomicAdd(&sbad[seg], 1u);
    if (s.ins[i]) atomicAdd(&sins[seg], 1u);
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < nseg; j += blockDim.x) {
    if (sbad[j]) atomicAdd(&s.cnt_bad[j], sbad[j]);
    if (sins[j]) atomicAdd(&s.cnt_ins[j], sins[j]);
  }
}

// ------------------------------------------------------------------------------------------------
// pulse_next_timestamp, exact (state_machine.zig:1576-1581, 1704-1708, 2112-2145). The reference
// keeps it outside every groove, so a chain rollback undoes none of its edits:
//   - every create_transfer that runs ok with a timeout lowers it to its expires_at (:1576-1581);
//   - every post/void that runs ok on a pending transfer with a timeout resets it to timestamp_min
//     when it equals that transfer's expires_at (:1704-1708).
// Once reset, it stays timestamp_min until the next batch's pulse check (the harness pulses before
// every batch, :2719-2739), where the pulse expires nothing (the window check guarantees it) and
// its finish sets the first live expires_at or timestamp_max (:2126-2135). k_pn replays exactly
// that over the window's ops in event order; events that ran ok are the committed ones plus the
// rolled-back chain members marked C_RANOK.
// ------------------------------------------------------------------------------------------------
// The event's op: 0 none, 1 creation (value x), 2 reset candidate (value y).
__device__ inline uint32_t pn_op(const Scratch& s, uint32_t i, uint64_t* v) {
  const uint32_t cls = s.cls[i];
  if (!(cls & C_PNOP)) return 0;
  if (s.code[i] != TB_CT_OK && !(cls & C_RANOK)) return 0;
  *v = s.pnv[i];
  return (cls & C_POSTVOID) ? 2u : 1u;
}

__device__ inline unsigned long long umin64(unsigned long long a, unsigned long long b) { return a < b ? a : b; }

// Block-wide minimum of a u64 (one LDS word per wave), result valid in every thread.
template <int NWAVES>
__device__ inline unsigned long long block_min_u64(unsigned long long v, unsigned long long* lds) {
  return ~block_max_u64<NWAVES>(~v, lds);
}

// A u64 through one DPP move per 32-bit half; lanes without a source lane get ~0 (the min identity).
template <int CTRL, int ROWS>
__device__ inline unsigned long long dpp_mov_u64(unsigned long long x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)(uint32_t)x, CTRL, ROWS, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)(uint32_t)(x >> 32), CTRL, ROWS, 0xf, false);
  return ((unsigned long long)hi << 32) | lo;
}
template <int CTRL, int ROWS>
__device__ inline unsigned long long dpp_min_u64(unsigned long long x) {
  return umin64(x, dpp_mov_u64<CTRL, ROWS>(x));
}

// Exclusive prefix minimum over the block's threads (identity ~0); *total = the block minimum.
template <int NWAVES>
__device__ inline unsigned long long block_excl_min_u64(unsigned long long v, unsigned long long* lds,
                                                        unsigned long long* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // inclusive wave scan with DPP (row shifts, row broadcasts; lanes without a source keep the
  // identity), then the exclusive value by a wave shift right by one
  unsigned long long inc = v;
  inc = dpp_min_u64<0x111, 0xf>(inc);  // row_shr:1
  inc = dpp_min_u64<0x112, 0xf>(inc);  // row_shr:2
  inc = dpp_min_u64<0x114, 0xf>(inc);  // row_shr:4
  inc = dpp_min_u64<0x118, 0xf>(inc);  // row_shr:8
  inc = dpp_min_u64<0x142, 0xa>(inc);  // row_bcast:15
  inc = dpp_min_u64<0x143, 0xc>(inc);  // row_bcast:31
  const unsigned long long ex = dpp_mov_u64<0x138, 0xf>(inc);  // wave_shr:1 (lane 0: ~0)
  if (lane == 63) lds[wave] = inc;
  __syncthreads();
  unsigned long long wp = ~0ull, tot = ~0ull;
#pragma unroll
  for (int k = 0; k < NWAVES; k++) {
    const unsigned long long x = lds[k];
    if (k < wave) wp = umin64(wp, x);
    tot = umin64(tot, x);
  }
  __syncthreads();
  *total = tot;
  return umin64(wp, ex);
}

// Per segment (one k_final block): the minimum creation value and the number of reset candidates
// that can take effect before any in-window pulse, over the events that ran ok. Until the first
// reset pulse_next only falls from pn0 (its value after the window's pulse), so a reset needs
// expires_at <= pn0.
__device__ inline void pn_seg_summary(const Scratch& s, uint32_t i, uint32_t E, uint64_t pn0, uint32_t* lds,
                                      unsigned long long* ldsm) {
  unsigned long long x = ~0ull;
  uint32_t r = 0;
  if (i < E) {
    uint64_t v = 0;
    const uint32_t op = pn_op(s, i, &v);
    if (op == 1) x = v;
    if (op == 2 && v <= pn0) r = 1;
  }
  const unsigned long long m = block_min_u64<SEG / 64>(x, ldsm);
  const uint32_t n = block_sum<SEG / 64>(r, lds);
  if (threadIdx.x == 0) {
    s.pn_min[blockIdx.x] = m;
    s.pn_res[blockIdx.x] = n;
  }
}

#define PN_THREADS 1024

// The pulse at the start of batch b >= 1 after a reset: nothing is due (window check), so its
// finish sets the minimum expires_at among the entries live at that point, else timestamp_max.
// Live then = (A) entries pending now and created before batch b (pre-window slots, or records
// stamped <= T_{b-1}), plus (B) pending transfers that a committed post/void of batch >= b removed,
// created before batch b. Rare (a reset inside a multi-batch window): one workgroup, plain loops.
__device__ uint64_t pn_minlive(const Dev& d, const Scratch& s, const WinDesc& w, uint32_t b,
                               unsigned long long* ldsm) {
  const uint64_t base = d.g->base;
  const uint64_t t_prev = w.T[b - 1];
  unsigned long long m = ~0ull;
  const ExpEntry* list = d.exp[*d.exp_cur];
  const uint64_t cnt = d.g->exp_count;
  for (uint64_t j = threadIdx.x; j < cnt; j += PN_THREADS) {
    const ExpEntry e = list[j];
    if (d.xstatus[e.slot] != TB_PENDING_PENDING) continue;
    if (e.slot >= base && d.xr[e.slot].timestamp > t_prev) continue;  // created in batch >= b
    m = umin64(m, e.expires_at);
  }
  for (uint32_t k = w.off[b] + threadIdx.x; k < w.E; k += PN_THREADS) {
    const uint32_t cls = s.cls[k];
    if (!(cls & C_POSTVOID) || !(cls & C_PNOP) || s.code[k] != TB_CT_OK) continue;
    uint64_t pts;
    const uint32_t ps = s.p_tslot[k];
    if (ps != NONE32) {
      pts = d.xr[ps].timestamp;  // created before the window
    } else {
      const uint32_t pc = s.pn_src[k];
      if (s.batch[pc] >= b) continue;
      pts = win_ts(w, s.batch[pc], pc);
    }
    const uint64_t y = s.pnv[k];
    if ((pts >> 63) || y > TB_TIMESTAMP_MAX) continue;  // never visible to the scan (composite key)
    m = umin64(m, y);
  }
  m = block_min_u64<PN_THREADS / 64>(m, ldsm);
  return m == ~0ull ? TB_TIMESTAMP_MAX : m;
}

// The replay, by the last k_final block of a window with pulse_next ops (PN_THREADS threads).
__device__ void pn_replay(const Dev& d, const Scratch& s, const WinDesc& w, unsigned long long* ldsm,
                          uint32_t* sh) {
  uint32_t& first_eff = sh[0];
  uint32_t& next_seg = sh[1];
  const uint32_t E = w.E, nseg = (E + SEG - 1) / SEG;
  const uint64_t pn0 = d.g->pulse_next;  // after the pulse before the window
  uint64_t pn = pn0;
  // after an in-window pulse pulse_next may exceed pn0: the segment summaries (resets <= pn0) no
  // longer bound the candidates, so every later event is replayed one by one
  bool all_events = false;
  uint32_t i = 0;
  while (i < E) {
    if (i % SEG == 0 && !all_events) {
      // fold whole segments without a reset candidate; stop at the next one that has some
      const uint32_t s0 = i / SEG;
      if (threadIdx.x == 0) next_seg = NONE32;
      __syncthreads();
      for (uint32_t j = s0 + threadIdx.x; j < nseg; j += PN_THREADS)
        if (s.pn_res[j]) atomicMin(&next_seg, j);
      __syncthreads();
      const uint32_t stop = next_seg == NONE32 ? nseg : next_seg;
      unsigned long long m = ~0ull;
      for (uint32_t j = s0 + threadIdx.x; j < stop; j += PN_THREADS) m = umin64(m, s.pn_min[j]);
      pn = umin64(pn, block_min_u64<PN_THREADS / 64>(m, ldsm));
      if (stop == nseg) break;
      i = stop * SEG;
    }
    // event by event, within one segment and one batch
    const uint32_t b = s.batch[i];
    const uint32_t end = min(min((i / SEG + 1) * SEG, E), w.off[b + 1]);
    const uint32_t k = i + threadIdx.x;
    uint64_t v = 0;
    const uint32_t op = k < end ? pn_op(s, k, &v) : 0u;
    unsigned long long tot;
    const unsigned long long before = umin64(pn, block_excl_min_u64<PN_THREADS / 64>(op == 1 ? v : ~0ull, ldsm, &tot));
    if (threadIdx.x == 0) first_eff = NONE32;
    __syncthreads();
    if (op == 2 && before == v) atomicMin(&first_eff, k);
    __syncthreads();
    if (first_eff != NONE32 && w.log) {
      // a log's window: no pulse until the log's next pulse prepare, so timestamp_min stands
      pn = TB_TIMESTAMP_MIN;
      break;
    }
    if (first_eff != NONE32) {
      // reset to timestamp_min (:1706-1707); the next batch's pulse finds nothing due
      i = w.off[b + 1];
      pn = b + 1 < w.nb ? pn_minlive(d, s, w, b + 1, ldsm) : TB_TIMESTAMP_MIN;
      all_events = all_events || pn > pn0;
    } else {
      pn = umin64(pn, tot);
      i = end;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) d.g->pulse_next = pn;
}

#include "xwin.h"

// ------------------------------------------------------------------------------------------------
// final: ordered replies + insert ranks + effects (one event per thread, one segment per block)
// ------------------------------------------------------------------------------------------------
struct FinalOut {
  tb_create_result_t* results;  // window replies, concatenated per batch
  uint32_t* batch_base;         // [nb + 1]: batch b's replies are results[base[b] .. base[b+1])
  uint32_t* out_count;          // optional: total failures (single-batch callers)
};

// A 128-bit atomic add split in two phases so that several can be in flight before any carry is
// resolved: issue() adds the low word (returning the old value); finish() adds the high word plus
// the carry out of the low word. Concurrent adds compose to the exact 128-bit sum.
struct Add128 {
  unsigned long long* hi = nullptr;  // null: nothing issued
  unsigned long long lo_add, hi_add, old;
  bool small;
  // small: the window keeps every balance field below 2^64 (Globals::small_win), so the delta is
  // exact as a no-return 64-bit add on the low word (negative deltas wrap mod 2^64 to the right value)
  __device__ void issue(tb_uint128_t* p, u128 v, bool small_win) {
    unsigned long long* w = reinterpret_cast<unsigned long long*>(p);
    small = small_win;
    hi = w + 1;
    lo_add = (unsigned long long)v;
    hi_add = (unsigned long long)(v >> 64);
    if (small) {
      (void)atomicAdd(w, lo_add);
      return;
    }
    old = atomicAdd(w, lo_add);
  }
  __device__ void finish() const {
    if (!hi || small) return;
    const unsigned long long carry = (old + lo_add) < old ? 1ull : 0ull;
    if (hi_add + carry) atomicAdd(hi, hi_add + carry);
  }
};

// tb_transfer_t as eight 16 B words, indexed statically so the record stays in registers: q0 id,
// q1 debit_account_id, q2 credit_account_id, q3 amount, q4 pending_id, q5 user_data_128,
// q6 {user_data_64, user_data_32, timeout}, q7 {ledger, code | flags << 16, timestamp}.
static_assert(offsetof(tb_transfer_t, user_data_64) == 96 && offsetof(tb_transfer_t, timeout) == 108 &&
                  offsetof(tb_transfer_t, ledger) == 112 && offsetof(tb_transfer_t, code) == 116 &&
                  offsetof(tb_transfer_t, flags) == 118 && offsetof(tb_transfer_t, timestamp) == 120,
              "tb_transfer_t word layout");
static_assert(offsetof(tb_account_t, ledger) == 112 && offsetof(tb_account_t, flags) == 118 &&
                  offsetof(tb_account_t, timestamp) == 120,
              "tb_account_t word layout");
__device__ inline uint64_t rw_u64(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
__device__ inline tb_uint128_t rw_u128(const uint4& q) {
  tb_uint128_t v;
  v.lo = rw_u64(q.x, q.y);
  v.hi = rw_u64(q.z, q.w);
  return v;
}
__device__ inline void rw_stamp(uint4* r, uint64_t ts) {
  r[7].z = (uint32_t)ts;
  r[7].w = (uint32_t)(ts >> 32);
}
// pv_record (sm_logic.h) over the words: the posting/voiding record built from event r and pending p.
__device__ inline void rw_post_void(uint4* r, const tb_transfer_t* pending, u128 amount) {
  const uint4* p = reinterpret_cast<const uint4*>(pending);
  r[1] = p[1];
  r[2] = p[2];
  r[3] = make_uint4((uint32_t)amount, (uint32_t)((uint64_t)amount >> 32), (uint32_t)(amount >> 64),
                    (uint32_t)(amount >> 96));
  const uint4 p5 = p[5], p6 = p[6], p7 = p[7];
  if ((r[5].x | r[5].y | r[5].z | r[5].w) == 0) r[5] = p5;
  if ((r[6].x | r[6].y) == 0) {
    r[6].x = p6.x;
    r[6].y = p6.y;
  }
  if (r[6].z == 0) r[6].z = p6.z;
  r[6].w = 0;
  r[7].x = p7.x;
  r[7].y = (p7.y & 0xFFFFu) | (r[7].y & 0xFFFF0000u);
}


// Final write-out, one event per thread. The 128 B event records pass through LDS (8 KiB per wave):
// each wave loads its 64 input records with contiguous 16 B-per-lane loads, and stores its inserted
// records -- which own the contiguous slot range [base + first rins, +count) -- the same way, instead
// of 8 strided 16 B accesses per lane touching 64 lines each.
template <bool XFER>
__global__ void __launch_bounds__(SEG) k_final(Dev d, Scratch s, const uint8_t* ev_bytes, WinDesc w, FinalOut o) {
  __shared__ uint32_t lds[SEG / 64];
  __shared__ unsigned long long ldsm[SEG / 64];
  __shared__ uint4 stage[SEG * 8];  // one 128 B record per event: 128 KiB
  if (WIN_REJECTED(d.g) || SP_DONE(d.g)) return;
  const bool prefix_win = XFER && (d.g->win_flags & 2u) != 0;  // k_prep_reduce
  const uint32_t E = w.E;
  const uint32_t i = blockIdx.x * SEG + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t i0 = i - lane;  // the wave's first event
  uint4* ws = stage + (threadIdx.x >> 6) * 512;
  uint32_t cls = 0, code = TB_CT_OK;
  bool ins = false, wdefer = false;
  uint8_t wi = 0;  // W events: 1 sequential walker, 2 component walker (Walker::commit_record)
  if (i < E) {
    cls = s.cls[i];
    code = s.code[i];
    wi = (cls & C_W) ? s.ins[i] : 0;
    ins = (cls & C_W) ? wi != 0 : (cls & C_INSERTED) != 0;
    // a component walker's commit: its balance effects are applied here (Walker::commit_record)
    wdefer = XFER && wi == 2 && code == TB_CT_OK;
  }
  const uint32_t bad = code != TB_CT_OK;
  // The earlier segments' failure and insert counts, and this event's ranks inside the segment, in
  // one pass with one barrier: per wave the segment-count partials (each < 2^21, packed in 64 bits)
  // and the in-segment scan of bad << 16 | inserted (each <= SEG).
  uint32_t rbad, rins;
  {
    const uint32_t wave = threadIdx.x >> 6;
    uint32_t vb = 0, vi = 0;
    for (uint32_t j = threadIdx.x; j < blockIdx.x; j += SEG) {
      vb += s.cnt_bad[j];
      vi += s.cnt_ins[j];
    }
    const unsigned long long segp = ((unsigned long long)wave_sum(vb) << 32) | wave_sum(vi);
    const uint32_t mine = (bad << 16) | (ins ? 1u : 0u);
    const uint32_t inc = wave_incl_scan(mine);
    if (lane == 63) lds[wave] = inc;
    if (lane == 0) ldsm[wave] = segp;
    __syncthreads();
    uint32_t wp = 0;
    unsigned long long sp = 0;
#pragma unroll
    for (uint32_t k = 0; k < SEG / 64; k++) {
      if (k < wave) wp += lds[k];
      sp += ldsm[k];
    }
    __syncthreads();  // lds / ldsm are reused below
    const uint32_t ex = wp + inc - mine;
    rbad = (uint32_t)(sp >> 32) + (ex >> 16);
    rins = (uint32_t)sp + (ex & 0xFFFFu);
  }
  const uint64_t xbase = d.g->base;
  // k_ct_prep already stored the stamped input record of each plain create it expected to insert
  // at its own position (base + i). That record is final when the event inserts at rank i (no
  // earlier event of the window failed) and is neither W (walker record) nor a post/void (posting
  // record) nor pending (status and expiry below need its fields). A wave whose lanes are all such
  // events (or insert nothing) neither loads its input rows nor stores records.
  const bool direct = XFER && ins && rins == i && !(cls & (C_W | C_POSTVOID | C_PENDING)) && (cls & C_PREP_REC);
  const bool wave_rec = __ballot(ins && !direct) != 0;
  // a wave that stores records stores all of its inserted ones (one contiguous run)
  const bool in_place = direct && !wave_rec;
  if (wave_rec) {
    const uint4* src = reinterpret_cast<const uint4*>(ev_bytes) + (size_t)i0 * 8;
    const uint32_t nrec = i0 < E ? min(64u, E - i0) : 0u;
#pragma unroll
    for (uint32_t q = 0; q < 8; q++) {
      const uint32_t k = q * 64 + lane;
      if ((k >> 3) < nrec) ws[k] = ld_stream(src + k);
    }
  }
  wave_sync();
  // this event's output record (the input record, stamped; W events carry theirs in s.t2)
  uint4 rec[8];
  // its live expires_at entry, if any (appended per wave below: one counter atomic per wave)
  bool xapp = false;
  ExpEntry xent;
  // a component walker's create: its input row, stamped (the walker stored no record)
  const bool wcreate = XFER && wi == 2 && !(cls & C_POSTVOID);
  if (XFER && (cls & C_W) && !wcreate) {
    const uint4* t2 = reinterpret_cast<const uint4*>(&s.t2[i]);
#pragma unroll
    for (int q = 0; q < 8; q++) rec[q] = t2[q];
  } else if (wave_rec) {
#pragma unroll
    for (int q = 0; q < 8; q++) rec[q] = ws[lane * 8 + q];
  } else {
#pragma unroll
    for (int q = 0; q < 8; q++) rec[q] = make_uint4(0, 0, 0, 0);
  }
  if (i < E) {
    const uint32_t b = s.batch[i];
    if (i == w.off[b]) {
      // event i opens batch b and every empty batch just before it
      for (int32_t bb = (int32_t)b; bb >= 0 && w.off[bb] == i; bb--) o.batch_base[bb] = rbad;
    }
    if (bad) {
      tb_create_result_t r;
      r.index = i - w.off[b];
      r.result = code;
      o.results[rbad] = r;
    }
    const bool wev = cls & C_W;
    if (XFER) {
      // Balance deltas of non-W commits: low-word atomics issued first, carries resolved after the
      // record and table writes below.
      // named slots, not an indexed array (which the compiler keeps in scratch): debit and credit
      // side, and a post's posted pair
      Add128 a_dr, a_cr, a_dr2, a_cr2;
      const bool small = d.g->small_win != 0;
      if ((!wev && (cls & C_COMMIT)) || wdefer) {
        tb_account_t* dra = &d.acc[s.dr_slot[i]];
        tb_account_t* cra = &d.acc[s.cr_slot[i]];
        const u128 a = s.amt[i];
        if (cls & (C_RES_DR | C_RES_CR)) {
          // decided by the resolver, which applied the hot side(s); only a plain single-phase or
          // pending create reaches here
          const bool pend = cls & C_PENDING;
          if (!(cls & C_RES_DR)) a_dr.issue(pend ? &dra->debits_pending : &dra->debits_posted, a, small);
          if (!(cls & C_RES_CR)) a_cr.issue(pend ? &cra->credits_pending : &cra->credits_posted, a, small);
        } else if (cls & C_POSTVOID) {
          const u128 pa = s.pamt[i];
          a_dr.issue(&dra->debits_pending, (u128)0 - pa, small);
          a_cr.issue(&cra->credits_pending, (u128)0 - pa, small);
          if (cls & C_POST) {
            a_dr2.issue(&dra->debits_posted, a, small);
            a_cr2.issue(&cra->credits_posted, a, small);
          }
          if (!wev) d.xstatus[s.p_tslot[i]] = (cls & C_POST) ? TB_PENDING_POSTED : TB_PENDING_VOIDED;
        } else if (cls & C_PENDING) {
          a_dr.issue(&dra->debits_pending, a, small);
          a_cr.issue(&cra->credits_pending, a, small);
        } else {
          a_dr.issue(&dra->debits_posted, a, small);
          a_cr.issue(&cra->credits_posted, a, small);
        }
      }
      if (ins && in_place) {
        // the record is in place (k_ct_prep): index it unless the window extends the sorted prefix
        const uint64_t slot = xbase + rins;
        if (!prefix_win) {
          const tb_uint128_t id = reinterpret_cast<const tb_transfer_t*>(ev_bytes)[i].id;
          x_insert(d.x_tab, d.x_mask, id, (uint32_t)slot);
        }
        d.xstatus[slot] = 0;
      } else if (ins) {
        const uint64_t slot = xbase + rins;
        if (!wev || wcreate) rw_stamp(rec, win_ts(w, b, i));
        if (!wev && (cls & C_POSTVOID)) rw_post_void(rec, &d.xr[s.p_tslot[i]], s.amt[i]);
        if (wev && wi == 1 && s.hside[i]) {  // historical_balance row (the walker computed it)
          d.hist[slot] = s.hrow[i];
          d.hist_side[slot] = s.hside[i];
        }
        // records of a prefix-extending window are found by binary search (x_prefix_find)
        if (!prefix_win) x_insert(d.x_tab, d.x_mask, rw_u128(rec[0]), (uint32_t)slot);
        uint8_t st = 0;
        if ((rec[7].y >> 16) & TB_TRANSFER_PENDING) {
          st = wev ? s.bstatus[i] : (uint8_t)TB_PENDING_PENDING;
          const uint32_t timeout = rec[6].w;
          if (timeout > 0) {
            const uint64_t ts = rw_u64(rec[7].z, rec[7].w);
            const uint64_t expires_at = ts + (uint64_t)timeout * TB_NS_PER_S;  // expires_at_of
            // (pulse_next is k_pn's: it also counts creations that a failing chain rolled back)
            const bool visible = !(ts >> 63) && expires_at <= TB_TIMESTAMP_MAX;
            if (st == TB_PENDING_PENDING && visible) {
              xapp = true;
              xent.expires_at = expires_at;
              xent.slot = (uint32_t)slot;
              xent.pad = 0;
            }
          }
        }
        d.xstatus[slot] = st;
      }
      a_dr.finish();
      a_cr.finish();
      a_dr2.finish();
      a_cr2.finish();
    } else if (ins) {
      const uint64_t slot = xbase + rins;
      rw_stamp(rec, win_ts(w, b, i));
      const uint32_t aflags = rec[7].y >> 16;
      d.hot[slot] = 0;
      acc_insert(d.acc_tab, d.acc_mask, rw_u128(rec[0]), (uint32_t)slot, rec[7].x, aflags);
      if (aflags & (TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS | TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS))
        atomicAdd(reinterpret_cast<unsigned long long*>(&d.g->limited_accounts), 1ull);
    }
  }
  if (XFER) {
    // the block's entries from ONE counter atomic: one per wave on the same word serialized at the
    // memory side (a cfg4 window appends from almost every wave)
    __shared__ uint32_t xw[SEG / 64];
    __shared__ unsigned long long xq;
    const unsigned long long m = __ballot(xapp);
    const uint32_t wave = threadIdx.x >> 6;
    if (lane == 0) xw[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (uint32_t k = 0; k < SEG / 64; k++) {
      const uint32_t v = xw[k];
      before += k < wave ? v : 0u;
      tot += v;
    }
    if (threadIdx.x == 0 && tot)
      xq = atomicAdd(reinterpret_cast<unsigned long long*>(&d.g->exp_count), (unsigned long long)tot);
    __syncthreads();
    if (xapp) d.exp[*d.exp_cur][xq + before + (unsigned long long)__popcll(m & ((1ull << lane) - 1))] = xent;
  }
  // Compact this wave's inserted records in LDS, then store them as one contiguous run (a wave
  // with only in-place records stores nothing).
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)rins, 0);
  const uint32_t nins = wave_rec ? (uint32_t)__popcll(__ballot(ins)) : 0u;
  wave_sync();
  if (ins && wave_rec) {
#pragma unroll
    for (int q = 0; q < 8; q++) ws[(rins - r0) * 8 + q] = rec[q];
  }
  wave_sync();
  uint4* dst = reinterpret_cast<uint4*>(XFER ? (void*)d.xr : (void*)d.acc) + (size_t)(xbase + r0) * 8;
  for (uint32_t k = lane; k < nins * 8; k += 64) st_stream(dst + k, ws[k]);

  if (i == E - 1) {
    // the window's last event: totals and window-level state
    const uint32_t total_bad = rbad + bad, total_ins = rins + (ins ? 1u : 0u);
    for (int32_t bb = (int32_t)w.nb; bb >= 0 && w.off[bb] == E; bb--) o.batch_base[bb] = total_bad;
    if (o.out_count) *o.out_count = total_bad;
    Globals* gw = d.g;
    gw->result_count = total_bad;
    if (XFER) {
      if (prefix_win) gw->x_sorted = xbase + total_ins;
      gw->mono_prev = gw->win_flags & 1u;
      gw->x_count = xbase + total_ins;
      const u128 sum = gw->ovf_bound + gw->batch_amount_sum;
      gw->ovf_bound = (gw->batch_huge || sum < gw->ovf_bound) ? MAX128 : sum;
      gw->batch_amount_sum = 0;
      gw->batch_huge = 0;
      if (gw->sp_skip) gw->sp_skip--;  // the fused pass's back-off (fused.h)
    } else {
      gw->acc_count = xbase + total_ins;
    }
    gw->windows_applied++;
    gw->hot_count = 0;
    gw->hot_live = 0;
    gw->rc_last = gw->res_chunked;
    gw->res_chunked = 0;
    gw->res_inelig = 0;
    gw->res_error = 0;
    gw->res_done = 0;
    gw->heavy_count = 0;
    gw->light_count = 0;
    gw->cpw_done = 0;
  }
  // (windows with pulses inside replay pulse_next in k_xwin_replay)
  const uint32_t wf = (XFER && !w.xwin) ? d.g->win_flags : 0u;
  if (wf & 8u) {
    // a post/void may reset pulse_next: this segment's summary, then the last block to finish
    // replays the window's ops in event order into pulse_next
    __shared__ uint32_t pn_sh[3];
    pn_seg_summary(s, i, E, d.g->pulse_next, lds, ldsm);
    if (last_block_done(&d.g->final_done, &pn_sh[2])) pn_replay(d, s, w, ldsm, pn_sh);
  } else if (wf & 4u) {
    // no reset possible: pulse_next = min(pulse_next, every creation that ran ok) (:1576-1581)
    uint64_t v = 0;
    const unsigned long long m = block_min_u64<SEG / 64>((i < E && pn_op(s, i, &v) == 1) ? v : ~0ull, ldsm);
    if (threadIdx.x == 0 && m != ~0ull) atomicMin(reinterpret_cast<unsigned long long*>(&d.g->pulse_next), m);
  }
}

#include "fused.h"
#include "shard.h"
#include "route.h"

// ------------------------------------------------------------------------------------------------
// Pulse: ExpirePendingTransfers scan + execute_expire_pending_transfers (state_machine.zig:
// 1010-1105, 1874-1929, 2112-2166). The live list holds scan-visible pending-with-timeout entries;
// an entry is live while its transfer's status is `pending`.
// ------------------------------------------------------------------------------------------------
// The window a pulse decision precedes: a window of several batches is valid only if no pulse can
// fall due inside it (the harness runs a pulse check before every batch, state_machine.zig:
// 2719-2739). Live expires_at entries are >= pulse_next (an invariant of the reference value too:
// finish sets it to the first live entry past the scan, creations only lower it, and a post/void
// reset only lowers it); entries the window creates expire >= its first timestamp + 1 s.
struct WinChk {
  uint32_t nb;
  uint32_t xwin;  // the window models the pulses inside it (xwin.h)
  uint64_t T_last, first_ts;
};
__device__ inline bool window_spans_pulse(const WinChk& c, uint64_t pulse_next) {
  if (c.xwin) return false;
  return c.nb > 1 && (c.T_last >= pulse_next || c.T_last >= c.first_ts + TB_NS_PER_S);
}

// The pulse before a window, in one launch: pulse() (:589-596), the expires_at scan (:1010-1043,
// value_next :2147-2166) over the live list by the whole grid (due entries to `cand`, the others to
// the alternate list), then, in the last block to finish: selection of the `cap` smallest
// (expires_at, slot) keys when more are due (12-pass LDS radix select, 8-bit digits over the 96-bit
// key; slot order = timestamp order), the finish (:2112-2145) into pulse_next, the window check
// against that new value, execute_expire_pending_transfers (:1874-1929) and the list swap.
// When no pulse is due every block returns at once, block 0 having checked the window against the
// current pulse_next. A window that spans a due pulse is rejected whole (window_error bit 0): it and
// every window after it change nothing until tbg_sync reports it; the scan only read the live list,
// so a rejected pulse leaves everything as it was. cand_count, alt_count and next_min are zero on
// entry (the tail leaves them so).
#define PULSE_BLOCKS 64  // few blocks: each pays an agent-scope fence before the last one runs the tail
__global__ void __launch_bounds__(1024) k_pulse(Dev d, Scratch s, uint64_t T, uint64_t prepare_timestamp,
                                               uint32_t cap, ChgLog chg, uint32_t chg_epoch, WinChk chk) {
  __shared__ uint32_t hist[256];
  __shared__ uint64_t prefix_hi;
  __shared__ uint32_t prefix_lo;
  __shared__ uint32_t want;
  __shared__ uint32_t flag;
  Globals* g = d.g;
  if (WIN_REJECTED(g)) return;
  const uint64_t pn = g->pulse_next;
  if (!(pn <= prepare_timestamp)) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && window_spans_pulse(chk, pn)) atomicOr(&g->window_error, 1u);
    return;
  }
  const uint32_t cur = *d.exp_cur;
  const ExpEntry* list = d.exp[cur];
  ExpEntry* alt = d.exp[cur ^ 1];
  const uint64_t count = g->exp_count;
  // (appends aggregated per block and pass, the minimum per wave: same-address atomics serialize)
  __shared__ uint32_t wd[1024 / 64], wl[1024 / 64];
  __shared__ uint32_t bd, bl;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned long long lt = (1ull << lane) - 1;
  unsigned long long nmin = ~0ull;
  for (uint64_t j0 = blockIdx.x * (uint64_t)blockDim.x; j0 < count; j0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t j = j0 + threadIdx.x;  // (block-uniform trip count: the barriers below)
    ExpEntry e{};
    bool live = false;
    if (j < count) {
      e = list[j];
      live = d.xstatus[e.slot] == TB_PENDING_PENDING;  // else removed from the index
    }
    const bool due = live && e.expires_at <= T;
    const bool later = live && !due;
    const unsigned long long md = __ballot(due), ml = __ballot(later);
    if (lane == 0) {
      wd[wave] = (uint32_t)__popcll(md);
      wl[wave] = (uint32_t)__popcll(ml);
    }
    __syncthreads();
    uint32_t pd = 0, pl = 0, td = 0, tl = 0;
#pragma unroll
    for (uint32_t k = 0; k < 1024 / 64; k++) {
      const uint32_t vd = wd[k], vl = wl[k];
      pd += k < wave ? vd : 0u;
      pl += k < wave ? vl : 0u;
      td += vd;
      tl += vl;
    }
    if (threadIdx.x == 0) {
      bd = td ? atomicAdd(&g->cand_count, td) : 0u;
      bl = tl ? atomicAdd(&g->alt_count, tl) : 0u;
    }
    __syncthreads();
    if (due) s.cand[bd + pd + (uint32_t)__popcll(md & lt)] = e;
    if (later) {
      alt[bl + pl + (uint32_t)__popcll(ml & lt)] = e;
      nmin = umin64(nmin, e.expires_at);
    }
    __syncthreads();  // (wd, wl, bd, bl: the next pass)
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) nmin = umin64(nmin, (unsigned long long)__shfl_xor(nmin, o, 64));
  if (lane == 0 && nmin != ~0ull) atomicMin(reinterpret_cast<unsigned long long*>(&g->next_min), nmin);
  if (!last_block_done(&g->pulse_done, &flag)) return;
  // ---- the last block: selection, finish, window check, apply ----
  const uint32_t m = __hip_atomic_load(&g->cand_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the buffer-full check precedes each next() (lsm/scan_lookup.zig:151-156): with exactly `cap`
  // entries due the scan ends buffer_finished too, and pulse_next is the last one's expires_at
  const bool select_all = m < cap;
  if (threadIdx.x == 0) {
    prefix_hi = 0;
    prefix_lo = 0;
    want = cap;  // 1-based rank of the last selected key
  }
  __syncthreads();
  for (int pass = 0; !select_all && pass < 12; pass++) {
    const int shift = 88 - 8 * pass;  // bit position of this digit in the 96-bit key
    for (int b = threadIdx.x; b < 256; b += blockDim.x) hist[b] = 0;
    __syncthreads();
    const int fixed_bits = 8 * pass;
    for (uint32_t j = threadIdx.x; j < m; j += blockDim.x) {
      const ExpEntry e = s.cand[j];
      bool match = true;
      if (fixed_bits > 0 && fixed_bits <= 64) {
        const uint64_t mask = fixed_bits == 64 ? ~0ull : ~((~0ull) >> fixed_bits);
        match = (e.expires_at & mask) == (prefix_hi & mask);
      } else if (fixed_bits > 64) {
        const uint32_t mask = ~((~0u) >> (fixed_bits - 64));
        match = e.expires_at == prefix_hi && (e.slot & mask) == (prefix_lo & mask);
      }
      if (!match) continue;
      const uint32_t digit =
          shift >= 32 ? (uint32_t)(e.expires_at >> (shift - 32)) & 0xFF : (e.slot >> shift) & 0xFF;
      atomicAdd(&hist[digit], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t acc = 0, digit = 0;
      for (; digit < 256; digit++) {
        if (acc + hist[digit] >= want) break;
        acc += hist[digit];
      }
      want -= acc;
      if (shift >= 32)
        prefix_hi |= (uint64_t)digit << (shift - 32);
      else
        prefix_lo |= digit << shift;
    }
    __syncthreads();
  }
  // finish: scan_finished -> the first live entry beyond T, else timestamp_max; buffer_finished ->
  // the last included expires_at (another pulse follows)
  const uint32_t n_alt = __hip_atomic_load(&g->alt_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t pn_after = select_all ? (n_alt > 0 ? g->next_min : TB_TIMESTAMP_MAX) : prefix_hi;
  const uint64_t thr_e = prefix_hi;
  const uint32_t thr_s = prefix_lo;
  // (a window modelling its pulses needs this one to have finished its scan)
  if (window_spans_pulse(chk, pn_after) || (chk.xwin && !select_all)) {
    __syncthreads();
    if (threadIdx.x == 0) {
      atomicOr(&g->window_error, 1u);
      g->cand_count = 0;
      g->alt_count = 0;
      g->next_min = ~0ull;
    }
    return;
  }
  for (uint32_t j = threadIdx.x; j < m; j += blockDim.x) {
    const ExpEntry e = s.cand[j];
    const bool take = select_all || e.expires_at < thr_e || (e.expires_at == thr_e && e.slot <= thr_s);
    if (!take) {
      const uint32_t k = atomicAdd(&g->alt_count, 1u);
      alt[k] = e;
      continue;
    }
    const tb_transfer_t x = d.xr[e.slot];
    AccEntry de, ce;
    const uint32_t drs = acc_find(d.acc_tab, d.acc_mask, x.debit_account_id, &de);
    const uint32_t crs = acc_find(d.acc_tab, d.acc_mask, x.credit_account_id, &ce);
    const u128 amt = U(x.amount);
    atomic_sub_u128(&d.acc[drs].debits_pending, amt);
    atomic_sub_u128(&d.acc[crs].credits_pending, amt);
    d.xstatus[e.slot] = TB_PENDING_EXPIRED;
    if (chg.mark) {  // change log (changes.h): both accounts and the expired TransferPending row
      chg.mark[drs] = chg_epoch;
      chg.mark[crs] = chg_epoch;
      chg.pend[atomicAdd(&chg.cnt[1], 1u)] = e.slot;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    *d.exp_cur = cur ^ 1u;
    g->exp_count = g->alt_count;
    g->pulse_next = pn_after;
    g->expired_count = select_all ? m : cap;
    g->cand_count = 0;
    g->alt_count = 0;
    g->next_min = ~0ull;
  }
}

// ------------------------------------------------------------------------------------------------
// lookup_accounts / lookup_transfers (state_machine.zig:1309-1344): found records, input order.
// ------------------------------------------------------------------------------------------------
#define LOOKUP_THREADS 1024
#define LOOKUP_ITEMS 8
template <bool ACC>
__global__ void __launch_bounds__(LOOKUP_THREADS) k_lookup(Dev d, const tb_uint128_t* ids, uint32_t n, uint8_t* out,
                                                           uint32_t* out_count) {
  __shared__ uint32_t lds[LOOKUP_THREADS / 64];
  uint32_t slot[LOOKUP_ITEMS];
  uint32_t found = 0;
  const uint32_t base = threadIdx.x * LOOKUP_ITEMS;
  for (int k = 0; k < LOOKUP_ITEMS; k++) {
    const uint32_t i = base + k;
    slot[k] = NONE32;
    if (i < n) {
      if (ACC) {
        AccEntry e;
        slot[k] = acc_find(d.acc_tab, d.acc_mask, ids[i], &e);
      } else {
        slot[k] = x_find(d.x_tab, d.xr, d.x_mask, ids[i]);
        if (slot[k] == NONE32) slot[k] = x_prefix_find(d.xr, d.g->x_sorted, ids[i]);
      }
    }
    found += slot[k] != NONE32;
  }
  uint32_t total;
  uint32_t pos = block_excl<LOOKUP_THREADS / 64>(found, lds, &total);
  for (int k = 0; k < LOOKUP_ITEMS; k++) {
    if (slot[k] == NONE32) continue;
    const uint4* src =
        ACC ? reinterpret_cast<const uint4*>(&d.acc[slot[k]]) : reinterpret_cast<const uint4*>(&d.xr[slot[k]]);
    uint4* dst = reinterpret_cast<uint4*>(out + (size_t)pos++ * 128);
#pragma unroll
    for (int q = 0; q < 8; q++) dst[q] = src[q];
  }
  if (threadIdx.x == 0) *out_count = total;
}

// Engine state initialization and flag clearing happen in kernels (see tbg_create).
__global__ void k_init_globals(Globals* g, Globals v) { *g = v; }
__global__ void k_clear_bits(uint32_t* p, uint32_t bits) { atomicAnd(p, ~bits); }

// The synchronous path's host <-> device bytes as kernels on the engine stream (host.inc
// stage_request, reply_out), reading and writing pinned host memory through its device mapping: a
// copy-engine transfer waits ~10 us for the compute queue on each side of it (measured,
// DESIGN.md §5), more than the transfer of a whole 1 MiB request.
__global__ void __launch_bounds__(256) k_copy_in(uint4* __restrict__ dst, const uint4* __restrict__ src, uint32_t n16) {
  for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < n16; k += gridDim.x * 256) dst[k] = src[k];
}
// Any bytes (tbg_read_device): 16-byte words when both sides are aligned, then the tail.
__global__ void __launch_bounds__(256) k_copy_bytes(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint32_t n) {
  const uint32_t n16 = ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) ? n / 16 : 0u;
  for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < n16; k += gridDim.x * 256)
    reinterpret_cast<uint4*>(dst)[k] = reinterpret_cast<const uint4*>(src)[k];
  for (uint32_t k = n16 * 16 + blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) dst[k] = src[k];
}
// The Globals ([0, g16) words) and, with the reply, the reply block at H_REPLY_OFF (its count and the
// first min(count, n_max) results): the same layout on both sides. flag (one block only): written
// with `seq` after every word, for the host to poll (reply_flag_out).
__device__ inline void reply_flag_out(unsigned long long* flag, unsigned long long seq) {
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void __launch_bounds__(256) k_reply_out(const uint4* __restrict__ dev, uint4* __restrict__ host, uint32_t g16,
                                                   uint32_t reply16, uint32_t n_max, uint32_t with_reply,
                                                   unsigned long long* flag, unsigned long long seq) {
  const uint32_t c = with_reply ? min(*reinterpret_cast<const uint32_t*>(dev + reply16), n_max) : 0u;
  const uint32_t r16 = with_reply ? 1u + (c * 8u + 15u) / 16u : 0u;
  for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < g16 + r16; k += gridDim.x * 256) {
    const uint32_t j = k < g16 ? k : reply16 + (k - g16);
    host[j] = dev[j];
  }
  if (flag) reply_flag_out(flag, seq);
}

// Entries in use of the two hash tables (tbg_debug_table_used): out[0] accounts, out[1] transfers.
__global__ void __launch_bounds__(256) k_table_used(Dev d, unsigned long long* out) {
  unsigned long long na = 0, nx = 0;
  for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k <= d.x_mask || k <= d.acc_mask;
       k += (uint64_t)gridDim.x * 256) {
    if (k <= d.acc_mask && d.acc_tab[k].slot != NONE32) na++;
    if (k <= d.x_mask && d.x_tab[k] != X_EMPTY) nx++;
  }
  na = wave_sum_u64(na);
  nx = wave_sum_u64(nx);
  if ((threadIdx.x & 63) == 0) {
    if (na) atomicAdd(out, na);
    if (nx) atomicAdd(out + 1, nx);
  }
}

// Harness `setup` (state_machine.zig:2545-2561).
__global__ void k_setup(Dev d, tb_uint128_t id, tb_uint128_t dp, tb_uint128_t dpo, tb_uint128_t cp, tb_uint128_t cpo,
                        int* found) {
  AccEntry e;
  const uint32_t slot = acc_find(d.acc_tab, d.acc_mask, id, &e);
  *found = slot != NONE32;
  if (slot == NONE32) return;
  tb_account_t* a = &d.acc[slot];
  a->debits_pending = dp;
  a->debits_posted = dpo;
  a->credits_pending = cp;
  a->credits_posted = cpo;
  const u128 s1 = U(dp) + U(dpo), s2 = U(cp) + U(cpo);
  const bool sat = s1 < U(dp) || s2 < U(cp);
  u128 m = s1 > s2 ? s1 : s2;
  if (sat) m = MAX128;
  if (m > d.g->ovf_bound) d.g->ovf_bound = m;
}

#include "shard_gw.h"
#include "host.inc"
#include "aof.inc"
#include "shard_gx.inc"
#include "shard_gw.inc"
#include "shard_read.inc"
#include "route.inc"
#include "group.inc"
