// shard.h — hash-sharded commit across G GPUs of one node (one engine per GPU), with home slices.
//
// Ownership: an account belongs to shard_of(account id), a transfer to shard_of(transfer id). Every
// shard holds the whole prepared window in HBM (the replica hands each GPU the same prepare body).
// Each shard is also the HOME of a contiguous range of the window's batches: it writes their replies.
// Per window, three launches and one exchange:
//
//   k_sh_scan     one pass over the window, one event per thread: the ids (64 B) give the owners; the
//                 id owner validates the event (state_machine.zig:1424-1439, 1465-1489), claims the id
//                 when the window's ids are not known to rise, and compares it with a stored transfer
//                 (`exists`, :1506-1507); the debit / credit owners resolve their account (state
//                 against the event's ledger, limit flags) and keep its slot. Each owner writes its part
//                 of the event's 2 B of facts; each block ORs its verdicts into the trailer itself.
//   (caller)      exchange 1: byte-wise sum all-reduce of the facts (RCCL over xGMI). Every bit has
//                 exactly one writer, so the sum is the union.
//   k_sh_decide   every event on every shard, from the facts alone: account lookups (:1496-1497),
//                 ledgers (:1503-1504), exists, linked chains (:1240-1300). The same outcome on every
//                 shard, so no second exchange (round 4 decided on the homes and all-reduced commit bits).
//   k_sh_apply    the home batches' replies; the account owners add the amounts, the id owner appends
//                 the record.
//
// The sharded class is the order-free one: no balance read (no limit flag on a touched
// account, no balancing), no history row (no flags.history on a touched account), no two-phase, no
// in-window duplicate id, overflow-free window. Then every event's outcome is a function of the owners'
// facts alone, and the effects commute. A window outside the class is detected before anything is
// applied (by an owner: exchange 1's trailer; by every shard's decide: a committed event reading a
// balance), so every shard reaches the same verdict and the window fails with TBG_E_UNSUPPORTED at
// tbg_sync: no shard applies any of it.
#pragma once
#include "changes.h"
#include "sm_logic.h"
#include "walker.h"
#include "window.h"

// Exchange bytes of a window of E events over G shards (summed byte-wise over the shards: every bit
// has exactly one writer, so the byte sum is the union with no carries; one uint8 all-reduce):
//   [0, 16)         trailer: word `par` (the window's parity, 0 / 1) this shard's verdict bytes (k_sh_scan;
//                   ZW_* below); the other word zeroed for the next window by this one's scan; words 2-3 zero
//   [16, M)         fixed-size counters, zeroed for the next window by k_sh_apply (each word has one writer
//                   shard, so the byte sum keeps it whole):
//                     G u64: shard g's room in its store (x_max - x_count or acc_max - acc_count)
//                     G x SH_OWN_SLOTS u32: shard g's owned ids reaching the exists check, by scan block
//                       k in slot k % SH_OWN_SLOTS (no-return adds: no same-address serialization)
//                     G x SH_MIS_SLOTS u64 ledger-mismatch slots, shard g's at [g * SH_MIS_SLOTS, ...):
//                       valid << 63 | side << 52 | event << 32 | the account's ledger
//                   M = 16 + 8 G + 4 G SH_OWN_SLOTS + 8 G SH_MIS_SLOTS
//   [M, M+E)        the id owner's byte: 1 + the code, static / linked bits (ZW_*)
//   create_transfers:
//   [M+E, M+2E)     the account sides' states (SH_ACC_*): bits 0-1 the debit account, 2-3 the credit
//                   account, each by its owner against the event's ledger; bits 4 / 5 the limit or
//                   history flag of the debit / credit account
// A side's ledger is needed only when both accounts mismatch the event's ledger (then whether they
// match each other decides between accounts_must_have_the_same_ledger and
// transfer_must_have_the_same_ledger_as_accounts, :1503-1504), so the 8 B of ledgers per event of the
// first protocol are 2 bits of state per side plus rare mismatch slots: 2 B per event instead of 9.
enum : uint32_t { SH_ACC_OK = 1, SH_ACC_MISSING = 2, SH_ACC_MISMATCH = 3 };
#define SH_MIS_SLOTS 4096u  // per shard; more mismatches in one window: outside the class (trailer 0)

#define SH_OWN_SLOTS 64u
struct XchView {
  uint32_t* trailer;
  unsigned long long* room;  // G
  uint32_t* own;             // G x SH_OWN_SLOTS
  unsigned long long* mis;   // G x SH_MIS_SLOTS (transfers only use them)
  uint8_t* zw;
  uint8_t* acc;              // transfers only
  uint32_t G;
  uint32_t par;              // the window's trailer word
};
// the fixed-size counters after the trailer: rooms, owned-id slots, mismatch slots (k_sh_apply zeroes them)
__host__ __device__ inline uint64_t xch_counters_words(uint32_t G) {  // (in u32 words)
  return 2ull * G + (uint64_t)G * SH_OWN_SLOTS + 2ull * G * SH_MIS_SLOTS;
}
__host__ __device__ inline uint64_t xch_facts_off(uint32_t G) { return 16 + 4 * xch_counters_words(G); }
__host__ __device__ inline uint64_t xch_bytes(bool xfer, uint32_t E, uint32_t G) {
  return xch_facts_off(G) + (xfer ? 2ull : 1ull) * E;
}
__host__ __device__ inline XchView xch_view(void* base, uint32_t E, bool xfer, uint32_t G, uint32_t par) {
  uint8_t* p = reinterpret_cast<uint8_t*>(base);
  XchView v;
  v.trailer = reinterpret_cast<uint32_t*>(p);
  v.room = reinterpret_cast<unsigned long long*>(p + 16);
  v.own = reinterpret_cast<uint32_t*>(p + 16 + 8ull * G);
  v.mis = reinterpret_cast<unsigned long long*>(p + 16 + 8ull * G + 4ull * G * SH_OWN_SLOTS);
  v.zw = p + xch_facts_off(G);
  v.acc = xfer ? v.zw + E : nullptr;
  v.G = G;
  v.par = par;
  return v;
}
// A side's ledger from the mismatch slots (both sides mismatched; never expected to be missing).
__device__ inline uint32_t xch_mis_ledger(const XchView& x, uint32_t e, uint32_t side) {
  const unsigned long long want = (1ull << 63) | ((unsigned long long)side << 52) | ((unsigned long long)e << 32);
  for (uint32_t k = 0; k < x.G * SH_MIS_SLOTS; k++) {
    const unsigned long long v = x.mis[k];
    if ((v & 0xFFFFFFFF00000000ull) == want) return (uint32_t)v;
  }
  return 0;
}

// Guard on every computed index of the sharded path: a violation is recorded (first one wins:
// check id << 48 | shard-local value, in Globals::dbg[7]), the window is failed as a device error
// (window_error bit 2, reported by tbg_sync) and the access is skipped. Never expected to fire.
__device__ inline bool sh_guard(Globals* g, bool ok, uint32_t check, uint64_t value) {
  if (ok) return true;
  atomicCAS(reinterpret_cast<unsigned long long*>(&g->dbg[7]), 0ull,
            ((unsigned long long)check << 48) | (value & 0xFFFFFFFFFFFFull));
  atomicOr(&g->window_error, 4u);
  return false;
}

// Owner of an id among G shards: the high half of the table hash (the tables index with the low
// bits, so a shard's own keys still spread over its whole table).
__host__ __device__ inline uint32_t shard_of(uint64_t lo, uint64_t hi, uint32_t G) {
  return (uint32_t)(((hash_id(lo, hi) >> 32) * (uint64_t)G) >> 32);
}

// Window key-map claim for the sharded path: returns the entry and whether the key was already
// claimed in this window (an in-window duplicate id).
__device__ inline uint32_t sh_claim(Globals* g, BEntry* bm, uint32_t mask, const uint8_t* ev, tb_uint128_t key,
                                    uint32_t idx, uint32_t E, uint32_t epoch, bool* dup) {
  const unsigned long long inc = 1ull << 21;
  uint32_t h = (uint32_t)hash_id(key.lo, key.hi) & mask;
  for (;;) {
    unsigned long long old = __hip_atomic_load(&bm[h].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
      if (bk_epoch(old) != epoch) {
        const unsigned long long fresh = ((unsigned long long)epoch << 32) | idx | inc;
        const unsigned long long prev = atomicCAS(&bm[h].key, old, fresh);
        if (prev == old) {
          *dup = false;
          return h;
        }
        old = prev;
        continue;
      }
      if (!sh_guard(g, bk_owner(old) < E && !bk_is_pid(old), 1, old)) {
        *dup = true;
        return h;
      }
      const tb_uint128_t k = bkey(ev, bk_owner(old), bk_is_pid(old));
      if (k.lo != key.lo || k.hi != key.hi) break;  // another key: probe on
      *dup = true;
      return h;
    }
    h = (h + 1) & mask;
  }
}

// End-of-window device state (thread 0 of k_sh_apply's last block). Nothing written here is read
// by k_sh_apply's other blocks, which may still be running: their store base is Globals::base
// (captured by k_sh_icount).
__device__ inline void sh_window_reset(Globals* g, bool xfer, uint64_t count, bool apply) {
  if (apply) {
    if (xfer) {
      g->x_count = count;
      const u128 sum = g->ovf_bound + g->batch_amount_sum;
      g->ovf_bound = (g->batch_huge || sum < g->ovf_bound) ? MAX128 : sum;
    } else {
      g->acc_count = count;
    }
  }
  g->batch_amount_sum = 0;
  g->batch_huge = 0;
}

// Scan-block partials (k_sh_scan's LDS word, then Globals::sh_flags): bit 0 huge amount, bit 1 in-window duplicate id (outside the
// class), bit 2 ids not strictly increasing (or >= 2^64), bit 3 the window's first id is above every
// stored id, bit 4 an event outside the class (SHX_UNSUP), owned ids reaching the exists check << 5.
enum : uint32_t { SHX_HUGE = 1, SHX_DUP = 2, SHX_NONMONO = 4, SHX_FRESH = 8, SHX_OWN_SHIFT = 5 };

// Validation a create_transfers event gets on every shard that looks at it whole (its owners and its
// home): timestamp (:1253-1259), head and field checks (:1465-1489, 1614-1624). Returns the static
// code or CONT; *reach: the event goes on to the account checks; *unsup: it is valid so far but
// outside the sharded class (pending, balancing, post/void).
__device__ inline uint32_t sh_static_ct(tb_transfer_t& t, const WinDesc& w, uint32_t b, uint32_t i, uint32_t* cls,
                                        bool* reach, bool* unsup) {
  *reach = false;
  *unsup = false;
  const uint16_t f = t.flags;
  if (f & TB_TRANSFER_LINKED) *cls |= C_LINKED;
  if (t.timestamp != 0) {
    *cls |= C_TSNZ;
    return TB_CT_TIMESTAMP_MUST_BE_ZERO;
  }
  t.timestamp = win_ts(w, b, i);
  uint32_t code = ct_head(t);
  if (code != CONT) return code;
  if (f & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) {
    code = pv_validate(t);
    if (code == CONT) *unsup = true;  // two-phase resolution: outside the sharded class
    return code;
  }
  code = ct_validate(t);
  if (code == CONT) {
    if (f & (TB_TRANSFER_PENDING | TB_TRANSFER_BALANCING_DEBIT | TB_TRANSFER_BALANCING_CREDIT)) *unsup = true;
    *reach = true;
  }
  return code;
}

__device__ inline uint32_t sh_static_ca(const tb_account_t& a, uint32_t* cls, bool* reach) {
  *reach = false;
  if (a.flags & TB_ACCOUNT_LINKED) *cls |= C_LINKED;
  if (a.timestamp != 0) {
    *cls |= C_TSNZ;
    return TB_CA_TIMESTAMP_MUST_BE_ZERO;
  }
  const uint32_t code = ca_validate(a);
  *reach = code == CONT;
  return code;
}

// A sharded window runs no pulse: the caller ran the harness pulse before its first batch when one
// was due (through the general path), so no pulse may be due at any of its batches
// (pulse_next > T_last), and a window of several batches spans less than a second. The class holds
// no pending transfer, so the window itself cannot lower pulse_next. Kept as a guard (window_error
// bit 3, tbg_sync returns TBG_E_STATE).
__device__ inline void check_window(const WinDesc& w, Globals* g) {
  const uint64_t last = w.T[w.nb - 1];
  const uint64_t first_ts = win_ts(w, 0, w.off[0]);
  if (last >= g->pulse_next || (w.nb > 1 && last >= first_ts + TB_NS_PER_S)) atomicOr(&g->window_error, 8u);
}


// Owned roles of an event (Scratch::bstatus, k_sh_scan): this shard owns its debit account / credit
// account / id.
enum : uint8_t { ROLE_DR = 1, ROLE_CR = 2, ROLE_ID = 4 };

// Exchange 1, per event: the id owner's byte (XchView::zw): bits 0-5 1 + the code, bit 6 the code is
// static (validation, final before the account checks), bit 7 the event is linked (every shard's
// k_sh_decide follows the chains); the account byte (XchView::acc): bits 0-1 / 2-3 the debit / credit
// side's state (SH_ACC_*), bit 4 / 5 the debit / credit account has a limit or flags.history (each by
// its owner). The trailer's first word: one verdict byte per kind, 0 or 1 on each shard (the byte sum
// over the shards is nonzero iff one shard's is): [0] an in-window duplicate id, ids that did not rise
// in a window that made no claims, or the ledger-mismatch slots overflowed; [1] capacity; [2] the
// overflow bound; [3] an event outside the class (pending, balancing, post/void).
enum : uint32_t { ZW_CODE = 0x3F, ZW_STATIC = 0x40, ZW_LINKED = 0x80, ACC_DR_LIMIT = 0x10, ACC_CR_LIMIT = 0x20 };
static_assert(TB_CT_EXCEEDS_DEBITS + 1 <= (int)ZW_CODE && TB_CA_EXISTS + 1 <= (int)ZW_CODE, "codes fit 6 bits");
enum : uint32_t { SHX_UNSUP = 16 };
#define SH_SCAN_T 256  // k_sh_scan's block: small blocks keep more of its latency-bound waves resident
// Resident waves per SIMD requested for k_sh_scan / the unstaged k_sh_apply (0: the compiler's choice);
// A/B builds override them (tools/variants.sh -D...).
#ifndef SH_SCAN_WPE
#define SH_SCAN_WPE 0
#endif
#ifndef SH_APPLY_WPE
#define SH_APPLY_WPE 8
#endif
#ifndef SH_PACK
#define SH_PACK 1  // k_sh_scan packs an owned-side event's slots and amount for k_sh_apply (G = 8: -6 %)
#endif
#ifndef SH_DEC_T
#define SH_DEC_T 256  // k_sh_decide's block (a divisor of SEG; 1024 measured 1 % slower at G = 8)
#endif

__device__ inline bool sh_verdict(const XchView& x) { return x.trailer[x.par] != 0; }

// ------------------------------------------------------------------------------------------------
// k_sh_scan (before exchange 1): one pass over the window, one event per thread, every shard. Each
// event's ids give its owners (64 B read); the owners do their part in the same pass: the id owner
// validates the event (state_machine.zig:1424-1439, 1465-1489), claims its id when the window's ids
// are not known to rise (in-window duplicates through the window key map) and compares it with a
// stored transfer (`exists`, :1506-1507); the debit / credit owners resolve their account (state
// against the event's ledger, limit and history flags) and keep its slot for k_sh_apply. Each block
// ORs its rare verdicts into the trailer, adds its owned-id count to a slot of the exchange (every
// shard checks every shard's room after the exchange) and writes its partials (Scratch::blk_aux,
// blk_amt), which k_sh_decide's first block folds after the exchange: no fold launch, no grid-wide
// wait, no same-address atomic per block. (A last-block-done fold inside the scan measured ~2x
// slower: its agent-scope fence per block writes the XCD's L2 back; a one-block fold launch cost
// ~8 us + a launch gap per window; per-block returning atomics on Globals words ~50 us per 1M events.)
// ------------------------------------------------------------------------------------------------
template <bool XFER>
__global__ void __launch_bounds__(SH_SCAN_T) __attribute__((amdgpu_waves_per_eu(SH_SCAN_WPE))) k_sh_scan(Dev d, Scratch s, const uint8_t* __restrict__ ev_bytes,
                                                       WinDesc w, uint32_t epoch, XchView xch, uint32_t G, uint32_t me) {
  __shared__ u128 red[SH_SCAN_T / 64];
  __shared__ u128 redm[SH_SCAN_T / 64];
  __shared__ uint32_t aux;
  const uint32_t i = blockIdx.x * SH_SCAN_T + threadIdx.x;
  const uint32_t E = w.E;
  Globals* g = d.g;
  if (threadIdx.x == 0) {
    aux = 0;
    if ((i & (SEG - 1)) == 0) {  // this segment's counters (k_sh_decide adds to them)
      s.cnt_bad[i / SEG] = 0;
      s.cnt_ins[i / SEG] = 0;
    }
  }
  if (i == 0) {
    check_window(w, g);
    g->sh_unsup = 0;              // (k_sh_decide: a committed event reading a balance)
    xch.trailer[xch.par ^ 1] = 0;  // the next window's verdict word (its last reader was k_sh_apply)
    xch.room[me] = XFER ? d.x_max - g->x_count : d.acc_max - g->acc_count;
    // the overflow bound (a verdict, so every shard agrees): the window's owned amounts are each below
    // 2^64 (larger ones: SHX_HUGE) and at most E of them, so ovf_bound + E x 2^64 bounds the sum
    if (XFER && g->ovf_bound > MAX128 - ((u128)E << 64)) atomicOr(&xch.trailer[xch.par], 1u << 16);
  }
  // (the mismatch slots are zero: the previous window's k_sh_apply cleared them)
  __syncthreads();
  // the previous fast-path window's ids did not all rise: claims find in-window duplicates
  const bool claim = !XFER || g->mono_prev == 0;
  uint32_t roles = 0, zw = 0, accb = 0;
  uint32_t dslot = NONE32, cslot = NONE32;  // this shard's account slots (NONE32: not owned or missing)
  u128 amount = 0, idm = 0;
  bool owned_id = false;
  uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0, q2 = q0, q3 = q0;
  if (i < E) {
    // per-lane 16 B loads of the record head, all issued together (staging the wave's heads through
    // LDS, four lanes per record, measured slower: 51 against 40 us per 1M-event window at G = 8; so did
    // the previous id from the neighbour lane, whose shuffle splits the loads into two round trips, and
    // the amount loaded only by its owners)
    const uint4* q = reinterpret_cast<const uint4*>(ev_bytes + (size_t)i * 128);
    q0 = q[0];
    if (XFER) {
      q1 = q[1];
      q2 = q[2];
      q3 = q[3];
    }
    const tb_uint128_t id = rw_u128(q0);
    if (shard_of(id.lo, id.hi, G) == me) roles |= ROLE_ID;
    if (XFER) {
      const tb_uint128_t dra = rw_u128(q1), cra = rw_u128(q2);
      if (shard_of(dra.lo, dra.hi, G) == me) roles |= ROLE_DR;
      if (shard_of(cra.lo, cra.hi, G) == me) roles |= ROLE_CR;
      // the window's ids strictly increasing (every shard reads every id: the same verdict everywhere)
      if (i > 0 && !(U(id) > U(reinterpret_cast<const tb_transfer_t*>(ev_bytes)[i - 1].id)))
        atomicOr(&aux, (uint32_t)SHX_NONMONO);
      if (i == 0 && U(id) > g->x_id_max) atomicOr(&aux, (uint32_t)SHX_FRESH);
    }
    if (roles & ROLE_ID) {
      uint32_t cls = 0;
      bool reach, unsup = false, dup = false;
      uint32_t code;
      if (XFER) {
        tb_transfer_t t = reinterpret_cast<const tb_transfer_t*>(ev_bytes)[i];
        code = sh_static_ct(t, w, win_batch(w, i), i, &cls, &reach, &unsup);
        if (reach) {
          if (claim)
            (void)sh_claim(g, s.bmap, s.bmask, ev_bytes, t.id, i, E, epoch, &dup);
          uint32_t xs = NONE32;
          if (x_may_exist(t.id, g->x_id_max)) {
            xs = x_find(d.x_tab, d.xr, d.x_mask, t.id);
            if (xs == NONE32) xs = x_prefix_find(d.xr, g->x_sorted, t.id);
          }
          code = xs == NONE32 ? (uint32_t)TB_CT_OK : ct_exists(t, d.xr[xs]);
          idm = U(t.id);  // (an owned id that may be inserted: k_sh_decide folds the bound on x_id_max)
        }
      } else {
        const tb_account_t a = reinterpret_cast<const tb_account_t*>(ev_bytes)[i];
        code = sh_static_ca(a, &cls, &reach);
        if (reach) {
          (void)sh_claim(g, s.bmap, s.bmask, ev_bytes, a.id, i, E, epoch, &dup);
          AccEntry ae;
          const uint32_t slot = acc_find(d.acc_tab, d.acc_mask, a.id, &ae);
          code = slot == NONE32 ? (uint32_t)TB_CA_OK : ca_exists(a, d.acc[slot]);
        }
      }
      owned_id = reach;
      if (dup) atomicOr(&aux, (uint32_t)SHX_DUP);
      if (unsup) atomicOr(&aux, (uint32_t)SHX_UNSUP);
      zw = (1u + code) | (reach ? 0u : (uint32_t)ZW_STATIC) | ((cls & C_LINKED) ? (uint32_t)ZW_LINKED : 0u);
    }
    if (XFER && (roles & (ROLE_DR | ROLE_CR))) {
      // every amount an account owner sees counts toward the overflow bound, valid event or not
      amount = U(rw_u128(q3));
      const uint32_t ledger = q[7].x;  // each side's state is against the event's ledger
#pragma unroll
      for (uint32_t side = 0; side < 2; side++) {
        if (!(roles & (side ? ROLE_CR : ROLE_DR))) continue;
        AccEntry e;
        const uint32_t slot = acc_find(d.acc_tab, d.acc_mask, rw_u128(side ? q2 : q1), &e);
        (side ? cslot : dslot) = slot;
        uint32_t st = SH_ACC_MISSING;
        if (slot != NONE32) {
          st = e.ledger == ledger ? SH_ACC_OK : SH_ACC_MISMATCH;
          // a limit (a balance read) or flags.history (a historical_balance row of balances after the
          // event, :1806-1841): outside the order-free class if the event commits
          const uint16_t lim = side ? TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS : TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS;
          if (e.flags & (lim | TB_ACCOUNT_HISTORY)) accb |= side ? ACC_CR_LIMIT : ACC_DR_LIMIT;
          if (st == SH_ACC_MISMATCH) {
            const uint32_t k2 = atomicAdd(&g->sh_mis, 1u);
            if (k2 < SH_MIS_SLOTS)
              xch.mis[me * SH_MIS_SLOTS + k2] = (1ull << 63) | ((unsigned long long)side << 52) |
                                                ((unsigned long long)i << 32) | e.ledger;  // (k_sh_decide resets sh_mis)
            else
              atomicOr(&aux, (uint32_t)SHX_DUP);  // (verdict 0: outside the class)
          }
        }
        accb |= st << (2 * side);
      }
    }
    // every byte of this shard's copy: its owned facts, zero elsewhere (the sum is the union)
    xch.zw[i] = (uint8_t)zw;
    if (XFER) {
      xch.acc[i] = (uint8_t)accb;
#if SH_PACK
      // an event with an owned side: its two slots and its amount in one 16 B entry (Scratch::amt),
      // so k_sh_apply reads one sector instead of two slot sectors and the event row (an amount of
      // 2^64 or more puts the window outside the class: the low word is the amount)
      if (roles & (ROLE_DR | ROLE_CR))
        reinterpret_cast<uint4*>(s.amt)[i] = make_uint4(dslot, cslot, (uint32_t)(uint64_t)amount,
                                                        (uint32_t)((uint64_t)amount >> 32));
#else
      // the owned sides' slots only (written and read densely for every event measured slower)
      if (roles & ROLE_DR) s.dr_slot[i] = dslot;
      if (roles & ROLE_CR) s.cr_slot[i] = cslot;
#endif
    }
    s.bstatus[i] = (uint8_t)roles;
  }
  if ((uint64_t)(amount >> 64) != 0) atomicOr(&aux, (uint32_t)SHX_HUGE);
  // this block's partials: owned ids reaching the exists check (an insert bound), the amounts below 2^64
  const uint32_t c = (uint32_t)__popcll(__ballot(owned_id));
  const uint64_t a = ((uint64_t)(amount >> 64) != 0) ? 0ull : (uint64_t)amount;
  u128 v = a;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t lo = __shfl_xor((unsigned long long)(uint64_t)v, o, 64);
    const uint64_t hi = __shfl_xor((unsigned long long)(uint64_t)(v >> 64), o, 64);
    v += ((u128)hi << 64) | lo;
  }
  if (XFER) idm = wave_max_u128(idm);
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = v;
    if (XFER) redm[threadIdx.x >> 6] = idm;
    if (c) atomicAdd(&aux, c << SHX_OWN_SHIFT);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    u128 tot = 0;
#pragma unroll
    for (int w2 = 0; w2 < SH_SCAN_T / 64; w2++) tot += red[w2];
    const uint32_t bits = aux & 31u, own = aux >> SHX_OWN_SHIFT;
    s.blk_amt[blockIdx.x] = tot;
    s.blk_aux[blockIdx.x] = bits;
    if (XFER) {
      u128 bm = redm[0];
      for (int w2 = 1; w2 < SH_SCAN_T / 64; w2++) bm = umax128(bm, redm[w2]);
      s.blk_idmax[blockIdx.x] = bm;
    }
    // this block's verdicts (bytes of this shard's trailer word: [0] duplicate / unchecked
    // non-rising ids / mismatch slots full, [2] overflow bound, [3] outside the class; [1] capacity
    // is decided from the owned-id slots after the exchange)
    const bool claim = !XFER || g->mono_prev == 0;  // (k_sh_decide updates it after this launch)
    uint32_t v = ((bits & SHX_DUP) || (XFER && (bits & SHX_NONMONO) && !claim)) ? 1u : 0u;
    if (bits & SHX_HUGE) v |= 1u << 16;
    if (bits & SHX_UNSUP) v |= 1u << 24;
    if (v) atomicOr(&xch.trailer[xch.par], v);
    if (own) (void)atomicAdd(&xch.own[me * SH_OWN_SLOTS + blockIdx.x % SH_OWN_SLOTS], own);
  }
}

// ------------------------------------------------------------------------------------------------
// k_sh_decide (after exchange 1): every shard decides every event from the summed facts (2 B per
// event: the id owner's code, the account sides' states), so no second exchange is needed: account
// lookups (:1496-1497), ledgers (:1503-1504), exists (:1506-1507), then linked chains (:1240-1300,
// never across a batch). Per event its commit flag (Scratch::ins); the codes of the home batches'
// events (replies); per segment the home failures and the committed owned inserts (k_sh_apply's ranks).
// ------------------------------------------------------------------------------------------------
template <bool XFER>
__device__ inline uint32_t sh_code(const XchView& xch, uint32_t j) {
  const uint32_t zw = xch.zw[j];
  const uint32_t z = (zw & ZW_CODE) - 1;
  if (!XFER || (zw & ZW_STATIC)) return z;
  const uint32_t acc = xch.acc[j], dst = acc & 3u, cst = (acc >> 2) & 3u;
  if (dst == SH_ACC_MISSING) return TB_CT_DEBIT_ACCOUNT_NOT_FOUND;  // :1496-1497
  if (cst == SH_ACC_MISSING) return TB_CT_CREDIT_ACCOUNT_NOT_FOUND;
  // :1503-1504 from the states against the event's ledger: one side off it means the accounts
  // differ; both off it, their own ledgers decide
  if (dst == SH_ACC_MISMATCH || cst == SH_ACC_MISMATCH) {
    if (dst != cst) return TB_CT_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER;
    if (xch_mis_ledger(xch, j, 0) != xch_mis_ledger(xch, j, 1)) return TB_CT_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER;
    return TB_CT_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS;
  }
  return z;  // exists* or ok (:1506-1507)
}

template <bool XFER>
__global__ void __launch_bounds__(SH_DEC_T) k_sh_decide(Dev d, Scratch s, const uint8_t* __restrict__ ev_bytes, WinDesc w,
                                                   XchView xch, uint32_t e0, uint32_t e1) {
  __shared__ uint32_t nbad, nins;
  Globals* g = d.g;
  if (blockIdx.x == 0) {
    // k_sh_scan's partials folded (read by k_sh_apply and the next window; nothing else here reads
    // them), whatever the verdict: its blocks' flags and amounts, and every shard's owned inserts
    // against its room (the same capacity verdict on every shard)
    __shared__ uint32_t f_bits, f_cap;
    __shared__ u128 f_red[SH_DEC_T / 64], f_mx[SH_DEC_T / 64];
    if (threadIdx.x == 0) f_bits = f_cap = 0;
    __syncthreads();
    const uint32_t nblk = (w.E + SH_SCAN_T - 1) / SH_SCAN_T;
    uint32_t fb = 0;
    u128 fa = 0, fm = 0;
    for (uint32_t j = threadIdx.x; j < nblk; j += SH_DEC_T) {
      fb |= s.blk_aux[j];
      if (XFER) {
        fa += s.blk_amt[j];
        fm = umax128(fm, s.blk_idmax[j]);
      }
    }
    if (fb) atomicOr(&f_bits, fb);
    // shard g's owned-id slots: wave g, one slot per lane
    for (uint32_t sg = threadIdx.x >> 6; sg < xch.G; sg += SH_DEC_T / 64) {
      const uint32_t tot = wave_sum(xch.own[sg * SH_OWN_SLOTS + (threadIdx.x & 63)]);
      if ((threadIdx.x & 63) == 0 && tot > xch.room[sg]) atomicOr(&f_cap, 1u);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t lo = __shfl_xor((unsigned long long)(uint64_t)fa, o, 64);
      const uint64_t hi = __shfl_xor((unsigned long long)(uint64_t)(fa >> 64), o, 64);
      fa += ((u128)hi << 64) | lo;
    }
    if (XFER) fm = wave_max_u128(fm);
    if ((threadIdx.x & 63) == 0) {
      f_red[threadIdx.x >> 6] = fa;
      f_mx[threadIdx.x >> 6] = fm;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t bits = f_bits;
      g->sh_cap_bad = f_cap;
      if (XFER) {
        u128 amt = 0, mx = 0;
        for (int q = 0; q < SH_DEC_T / 64; q++) {
          amt += f_red[q];
          mx = umax128(mx, f_mx[q]);
        }
        // a bound on the stored ids (the owned ids that reached the exists check, inserted or not:
        // an id above it cannot exist; the window's first id above it extends the sorted prefix)
        if (mx > g->x_id_max) g->x_id_max = mx;
        g->batch_amount_sum += amt;
        if (bits & SHX_HUGE) g->batch_huge = 1;
        // every owned balance field stays below 2^64 this window: k_sh_apply's adds need no carry
        const u128 top = g->ovf_bound + g->batch_amount_sum;
        g->small_win = (!g->batch_huge && top >= g->ovf_bound && (uint64_t)(top >> 64) == 0) ? 1u : 0u;
        const bool prefix = !(bits & SHX_NONMONO) && (bits & SHX_FRESH) && g->x_sorted == g->x_count;
        g->win_flags = prefix ? 2u : 0u;
        g->mono_prev = (bits & SHX_NONMONO) ? 0u : 1u;  // the next window's claim mode (the same on every shard)
        g->sh_mis = 0;
      }
      g->base = XFER ? g->x_count : g->acc_count;  // k_sh_apply's insert base
    }
  }
  if (sh_verdict(xch)) return;  // outside the class: k_sh_apply reports it
  if (threadIdx.x == 0) nbad = nins = 0;
  __syncthreads();
  const uint32_t i = blockIdx.x * SH_DEC_T + threadIdx.x, seg = i / SEG;  // (blocks of one segment share its counters)
  uint32_t lbad = 0, lins = 0;
  if (i < w.E) {
    const uint32_t b = win_batch(w, i);
    const uint32_t first = w.off[b], last = w.off[b + 1] - 1;
    const bool head = i == first || !(xch.zw[i - 1] & ZW_LINKED);
    if (head) {
      // a single event, or the head of a chain i..end: no member's outcome depends on another member's
      // effects in a class window, so the chain fails at its first failing member
      uint32_t end = i, f = NONE32;
      for (uint32_t j = i;; j++) {
        const bool lj = xch.zw[j] & ZW_LINKED;
        uint32_t code = sh_code<XFER>(xch, j);
        if (lj && j == last) code = XFER ? (uint32_t)TB_CT_LINKED_EVENT_CHAIN_OPEN : (uint32_t)TB_CA_LINKED_EVENT_CHAIN_OPEN;
        if (j >= e0 && j < e1) s.code[j] = code;
        // a committed event reading a balance (limit) or writing a history row: outside the class
        if (XFER && code == TB_CT_OK && (xch.acc[j] & (ACC_DR_LIMIT | ACC_CR_LIMIT))) atomicOr(&g->sh_unsup, 1u);
        if (code != TB_CT_OK && f == NONE32) f = j;
        end = j;
        if (!lj || j == last) break;
      }
      for (uint32_t j = i; j <= end; j++) {
        const bool commit = f == NONE32;
        if (!commit && j != f && j >= e0 && j < e1 && !((xch.zw[j] & ZW_LINKED) && j == last))
          s.code[j] = XFER ? (uint32_t)TB_CT_LINKED_EVENT_FAILED : (uint32_t)TB_CA_LINKED_EVENT_FAILED;
        s.ins[j] = commit ? 1 : 0;
        const uint32_t bad = (!commit && j >= e0 && j < e1) ? 1u : 0u;
        const uint32_t ins = (commit && (s.bstatus[j] & ROLE_ID)) ? 1u : 0u;
        if (j / SEG == seg) {
          lbad += bad;
          lins += ins;
        } else {  // (a chain running into the next segment)
          if (bad) atomicAdd(&s.cnt_bad[j / SEG], 1u);
          if (ins) atomicAdd(&s.cnt_ins[j / SEG], 1u);
        }
      }
    }
  }
  const uint32_t wb = wave_sum(lbad), wi = wave_sum(lins);
  if ((threadIdx.x & 63) == 0) {
    if (wb) atomicAdd(&nbad, wb);
    if (wi) atomicAdd(&nins, wi);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (nbad) atomicAdd(&s.cnt_bad[seg], nbad);
    if (nins) atomicAdd(&s.cnt_ins[seg], nins);
  }
}

// ------------------------------------------------------------------------------------------------
// k_sh_apply: the home batches' replies (batch_base relative to hb0, indices batch-relative), then the
// owned effects of the committed events: the account owners add the amounts (no-return 64-bit adds
// when the window keeps every balance field below 2^64, else exact 128-bit atomics), the id owner
// appends the record in event order (sorted prefix when the window's ids rise above every stored id)
// and indexes it. The last block folds the inserted ids' exact maximum and closes the window. A window outside the class (exchange 1's verdict, or a committed event reading a balance)
// changes nothing on any shard: window_error bit 1 (TBG_E_UNSUPPORTED at tbg_sync).
// ------------------------------------------------------------------------------------------------
__device__ inline bool sh_abort(const XchView& x, const Globals* g) {
  return sh_verdict(x) || g->sh_unsup != 0 || g->sh_cap_bad != 0;
}

// STAGE (one shard: every event is owned, the inserts are dense): a wave's inserted records are
// compacted in LDS and stored as one contiguous run (as in k_final); with several shards the inserts
// are sparse and each inserting lane stores its record whole (no 128 KiB of LDS: twice the resident
// blocks).
template <bool XFER, bool STAGE>
__global__ void __launch_bounds__(SEG) __attribute__((amdgpu_waves_per_eu(STAGE ? 4 : SH_APPLY_WPE))) k_sh_apply(Dev d, Scratch s, const uint8_t* ev_bytes, WinDesc w, XchView xch,
                                                  uint32_t hb0, uint32_t hb1, uint32_t e0, uint32_t e1, FinalOut o,
                                                  ChgLog chg, uint32_t chg_epoch) {
  __shared__ uint32_t lds[SEG / 64];
  __shared__ uint4 stage[XFER && STAGE ? SEG * 8 : 1];
  Globals* g = d.g;
  // the counters zeroed for the next window (k_sh_decide was their last reader)
  const uint32_t nw = (uint32_t)xch_counters_words(xch.G);
  uint32_t* cw = reinterpret_cast<uint32_t*>(xch.room);
  for (uint32_t k = blockIdx.x * SEG + threadIdx.x; k < nw; k += gridDim.x * SEG) cw[k] = 0;
  if (sh_abort(xch, g)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      atomicOr(&g->window_error, 2u);
      sh_window_reset(g, XFER, 0, false);
    }
    return;
  }
  const bool prefix_win = XFER && (g->win_flags & 2u) != 0;  // k_sh_scan
  const bool small = XFER && g->small_win != 0;              // k_sh_scan
  const uint64_t xbase = g->base;                            // k_sh_decide
  const uint32_t i = blockIdx.x * SEG + threadIdx.x;
  const bool in = i < w.E;
  const bool commit = in && s.ins[i];
  const uint32_t roles = in ? s.bstatus[i] : 0u;
  // ---- replies of the home batches ----
  const bool home = i >= e0 && i < e1;
  const uint32_t code = home ? s.code[i] : (uint32_t)TB_CT_OK;
  const uint32_t bad = home && code != TB_CT_OK ? 1u : 0u;
  uint32_t tot;
  const uint32_t rbad = seg_prefix<SEG>(s.cnt_bad, blockIdx.x, lds) + block_excl<SEG / 64>(bad, lds, &tot);
  if (home) {
    const uint32_t b = win_batch(w, i);
    if (i == w.off[b]) {
      // event i opens batch b and every empty home batch just before it
      for (int32_t bb = (int32_t)b; bb >= (int32_t)hb0 && w.off[bb] == i; bb--) o.batch_base[bb - hb0] = rbad;
    }
    if (bad && sh_guard(g, rbad < e1 - e0, 2, rbad)) {
      tb_create_result_t r;
      r.index = i - w.off[b];
      r.result = code;
      o.results[rbad] = r;
    }
    if (i == e1 - 1) {
      const uint32_t total_bad = rbad + bad;
      for (int32_t bb = (int32_t)hb1; bb >= (int32_t)hb0 && w.off[bb] == e1; bb--) o.batch_base[bb - hb0] = total_bad;
      if (o.out_count) *o.out_count = total_bad;
      g->result_count = total_bad;
    }
  }
  // ---- owned effects ----
  bool ins = commit && (roles & ROLE_ID);
  const uint32_t pins = seg_prefix<SEG>(s.cnt_ins, blockIdx.x, lds);
  uint32_t tot_ins;
  const uint32_t rins = pins + block_excl<SEG / 64>(ins ? 1u : 0u, lds, &tot_ins);
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)rins, 0);  // the wave's first insert rank
  if (commit) {
    if (XFER) {
#if SH_PACK
      uint4 pk = make_uint4(NONE32, NONE32, 0, 0);
      if (roles & (ROLE_DR | ROLE_CR)) pk = reinterpret_cast<const uint4*>(s.amt)[i];
      uint32_t drs = (roles & ROLE_DR) ? pk.x : NONE32, crs = (roles & ROLE_CR) ? pk.y : NONE32;
#else
      uint32_t drs = (roles & ROLE_DR) ? s.dr_slot[i] : NONE32, crs = (roles & ROLE_CR) ? s.cr_slot[i] : NONE32;
#endif
      if (drs != NONE32 && !sh_guard(g, drs < d.acc_max, 3, drs)) drs = NONE32;
      if (crs != NONE32 && !sh_guard(g, crs < d.acc_max, 4, crs)) crs = NONE32;
      if (ins && !sh_guard(g, xbase + rins < d.x_max, 5, xbase + rins)) ins = false;
      const tb_transfer_t* t = reinterpret_cast<const tb_transfer_t*>(ev_bytes) + i;
      Add128 a_dr, a_cr;
      if (drs != NONE32 || crs != NONE32) {
#if SH_PACK
        const u128 a = ((uint64_t)pk.w << 32) | pk.z;
#else
        const u128 a = U(t->amount);
#endif
        if (drs != NONE32) a_dr.issue(&d.acc[drs].debits_posted, a, small);
        if (crs != NONE32) a_cr.issue(&d.acc[crs].credits_posted, a, small);
        if (chg.mark) {  // write-back stream (changes.h): the owned accounts this window changed
          if (drs != NONE32) chg.mark[drs] = chg_epoch;
          if (crs != NONE32) chg.mark[crs] = chg_epoch;
        }
      }
      if (ins) {
        const uint64_t slot = xbase + rins;
        const uint64_t ts = win_ts(w, win_batch(w, i), i);
        // the record as 16 B words, in two halves (a whole record in registers costs 32 VGPRs)
        const uint4* src = reinterpret_cast<const uint4*>(t);
        uint4* ws = stage + (threadIdx.x >> 6) * 512 + (rins - r0) * 8;
        uint4* dst = reinterpret_cast<uint4*>(d.xr + slot);
        tb_uint128_t id;
#pragma unroll
        for (int half = 0; half < 2; half++) {
          uint4 r[4];
#pragma unroll
          for (int q = 0; q < 4; q++) r[q] = src[half * 4 + q];
          if (half == 0) id = rw_u128(r[0]);
          else {
            r[3].z = (uint32_t)ts;  // the stamped timestamp (word 7)
            r[3].w = (uint32_t)(ts >> 32);
          }
          // ranks of a wave's inserts are consecutive (block_excl); a failed slot guard can only drop
          // a suffix of them, so the staged run below stays gap-free
#pragma unroll
          for (int q = 0; q < 4; q++) {
            if (STAGE)
              ws[half * 4 + q] = r[q];
            else
              st_stream(dst + half * 4 + q, r[q]);
          }
        }
        if (!prefix_win) x_insert(d.x_tab, d.x_mask, id, (uint32_t)slot);
        d.xstatus[slot] = 0;
      }
      a_dr.finish();
      a_cr.finish();
    } else if (ins && sh_guard(g, xbase + rins < d.acc_max, 6, xbase + rins)) {
      // (the record as 16 B words: a struct copy whose address is taken goes to scratch memory)
      const uint64_t slot = xbase + rins;
      const uint4* src = reinterpret_cast<const uint4*>(ev_bytes) + (size_t)i * 8;
      uint4 r[8];
#pragma unroll
      for (int q = 0; q < 8; q++) r[q] = src[q];
      rw_stamp(r, win_ts(w, win_batch(w, i), i));
      uint4* dst = reinterpret_cast<uint4*>(d.acc + slot);
#pragma unroll
      for (int q = 0; q < 8; q++) dst[q] = r[q];
      d.hot[slot] = 0;
      acc_insert(d.acc_tab, d.acc_mask, rw_u128(r[0]), (uint32_t)slot, r[7].x, (uint16_t)(r[7].y >> 16));
    }
  }
  if (XFER && STAGE) {
    const uint32_t nins = (uint32_t)__popcll(__ballot(ins));
    wave_sync();
    if (nins) {
      const uint4* ws = stage + (threadIdx.x >> 6) * 512;
      uint4* dst = reinterpret_cast<uint4*>(d.xr) + (size_t)(xbase + r0) * 8;
      for (uint32_t k = threadIdx.x & 63; k < nins * 8; k += 64) st_stream(dst + k, ws[k]);
    }
  }
  // The last block (by index; the others may still run: they read Globals::base, captured by
  // k_sh_decide, never the counts written here) closes the window from k_sh_decide's per-segment
  // counts (the id bound was folded by k_sh_decide).
  if (blockIdx.x != gridDim.x - 1) return;
  const uint32_t total_ins = pins + tot_ins;
  if (threadIdx.x == 0) {
    const uint64_t total = xbase + total_ins;
    g->events_total += w.E;
    if (prefix_win) g->x_sorted = total;
    sh_window_reset(g, XFER, total, true);
  }
}
