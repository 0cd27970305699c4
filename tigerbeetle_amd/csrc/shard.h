// shard.h — hash-sharded commit across G GPUs of one node (one engine per GPU), with home slices.
//
// Ownership: an account belongs to shard_of(account id), a transfer to shard_of(transfer id). Every
// shard holds the whole prepared window in HBM (the replica hands each GPU the same prepare body).
// Each shard is also the HOME of a contiguous range of the window's batches: it decides those events
// and writes their replies. Per-shard work is the window's ids (64 B per event) plus 1/G of
// everything else, so the work per GPU falls as G grows:
//
//   k_sh_roles    whole window: the ids of each event (64 B); events with a role this shard owns
//                 (debit account, credit account, transfer id) are compacted, in event order, into
//                 per-segment lists, so the owned work below runs on dense waves.
//   k_sh_owned_*  owned events only: the id owner reads the event whole and validates it
//                 (state_machine.zig:1424-1439, 1465-1489); if it reaches the account checks, it
//                 claims the id (in-window duplicates through the window key map) and compares it
//                 with a stored transfer (`exists`, :1506-1507). The debit / credit owners read the
//                 account ids and the amount and resolve their account (ledger, limit flag). Each
//                 owner writes its part of the event's 9 B of facts (exchange 1).
//   (caller)      exchange 1: byte-wise sum all-reduce of the facts (RCCL over xGMI). Every bit has
//                 exactly one writer, so the sum is the union.
//   k_sh_home_*   home slice: validation codes and class checks.
//   k_sh_decide   home slice: account lookups (:1496-1497), ledgers (:1503-1504), exists, then linked
//                 chains (:1240-1300).
//   k_sh_reply    home slice: per-batch replies (failure ranks from k_sh_decide's per-segment
//                 counts); one commit bit per event (exchange 2). Block 0 folds the owned work's
//                 partials into this shard's owner verdicts (k_sh_close does it for a shard home to
//                 no event).
//   (caller)      exchange 2: byte-wise sum all-reduce of the commit bits (E/8 B) and the verdicts.
//   k_sh_icount, k_sh_apply  whole window, owned roles only: the verdict, then the account owners add
//                 the amounts (exact 128-bit atomics) and the id owner appends the record.
//
// The sharded class is the order-free one: no balance read (no limit flag on a touched
// account, no balancing), no history row (no flags.history on a touched account), no two-phase, no
// in-window duplicate id, overflow-free window. Then every
// event's outcome is a function of the owners' facts alone, and the effects commute. A window outside
// the class is detected before anything is applied (by an owner or a home: exchange 2's trailer), so
// every shard reaches the same verdict and the window fails with
// TBG_E_UNSUPPORTED at tbg_sync: no shard applies any of it.
#pragma once
#include "changes.h"
#include "sm_logic.h"
#include "walker.h"
#include "window.h"

// Exchange bytes of a window of E events over G shards (summed byte-wise over the shards: every bit
// has exactly one writer, so the byte sum is the union with no carries; one uint8 all-reduce):
//   [0, 16)         trailer: unused, zero (the owners' verdicts travel in exchange 2's)
//   [16, 16+E)      bits 0-5: 1 + (TB_CT_OK or the exists* code; create_accounts: 1 + the code), by
//                   the id owner; bit 6: the debit account has debits_must_not_exceed_credits or
//                   flags.history (its owner); bit 7: the credit account has
//                   credits_must_not_exceed_debits or flags.history (its owner)
//   create_transfers:
//   [16+E, 16+2E)   the account sides' states (SH_ACC_*): bits 0-1 the debit account, 2-3 the credit
//                   account, each by its owner against the event's ledger
//   [16+2E, ...)    G x SH_MIS_SLOTS u64 ledger-mismatch slots, shard g's at [g * SH_MIS_SLOTS, ...):
//                   valid << 63 | side << 52 | event << 32 | the account's ledger
// A side's ledger is needed only when both accounts mismatch the event's ledger (then whether they
// match each other decides between accounts_must_have_the_same_ledger and
// transfer_must_have_the_same_ledger_as_accounts, :1503-1504), so the 8 B of ledgers per event of the
// first protocol are 2 bits of state per side plus rare mismatch slots: 2 B per event instead of 9.
enum : uint32_t { SH_Z_MASK = 0x3F, SH_DR_LIMIT = 0x40, SH_CR_LIMIT = 0x80 };
enum : uint32_t { SH_ACC_OK = 1, SH_ACC_MISSING = 2, SH_ACC_MISMATCH = 3 };
#define SH_MIS_SLOTS 4096u  // per shard; more mismatches in one window: outside the class (trailer 0)

struct XchView {
  uint32_t* trailer;
  uint8_t* zw;
  uint8_t* acc;              // transfers only
  unsigned long long* mis;   // transfers only: G x SH_MIS_SLOTS
  uint32_t G;
};
__host__ __device__ inline uint64_t xch_mis_off(uint32_t E) { return (16 + 2ull * E + 7) & ~7ull; }
__host__ __device__ inline uint64_t xch_bytes(bool xfer, uint32_t E, uint32_t G) {
  return xfer ? xch_mis_off(E) + 8ull * G * SH_MIS_SLOTS : 16 + (uint64_t)E;
}
__host__ __device__ inline XchView xch_view(void* base, uint32_t E, bool xfer, uint32_t G) {
  uint8_t* p = reinterpret_cast<uint8_t*>(base);
  XchView v;
  v.trailer = reinterpret_cast<uint32_t*>(p);
  v.zw = p + 16;
  v.acc = xfer ? p + 16 + E : nullptr;
  v.mis = xfer ? reinterpret_cast<unsigned long long*>(p + xch_mis_off(E)) : nullptr;
  v.G = G;
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

// Exchange 2 (commit bits): 16 B trailer, 4 x u32 summed over the shards: [0] homes that found an
// event outside the class, [1] shards that saw an in-window duplicate id or overflowed their
// ledger-mismatch slots, [2] shards over capacity, [3] shards whose overflow bound does not clear
// the window's amounts; then one bit per event, in 64-bit words (a word may hold bits of two homes: distinct bits).
__host__ __device__ inline uint64_t xch2_bytes(uint32_t E) { return 16 + 8ull * ((E + 63) / 64); }

// Scan-block partials (Scratch::blk_aux): bit 0 huge amount, bit 1 in-window duplicate id (outside the
// class), bit 2 ids not strictly increasing (or >= 2^64), bit 3 the window's first id is above every
// stored id, owned ids reaching the exists check << 4.
enum : uint32_t { SHX_HUGE = 1, SHX_DUP = 2, SHX_NONMONO = 4, SHX_FRESH = 8, SHX_OWN_SHIFT = 4 };

// After exchange 1 (stream-ordered, one 1024-thread block, red[] one entry per wave: block 0 of
// k_sh_reply, or k_sh_close when this shard is home to no event): folds the scan blocks' partials
// (no same-address atomics across blocks) into this shard's window verdicts, returned to thread 0 as bit 0 (duplicate id or
// mismatch slots overflowed), bit 1 (capacity), bit 2 (overflow bound), and sets
// Globals::win_flags bit 1 (the owned records extend the sorted prefix) and small_win for k_sh_apply.
// The verdicts travel in exchange 2's trailer, so exchange 1 needs no fold before it.
__device__ inline uint32_t sh_close_fold(Dev d, const Scratch& s, uint32_t nblk, uint32_t xfer, u128* red,
                                         uint32_t* bits_s, unsigned long long* own_s) {
  if (threadIdx.x == 0) {
    *bits_s = 0;
    *own_s = 0;
  }
  __syncthreads();
  u128 v = 0;
  uint32_t a = 0;
  unsigned long long own = 0;
  for (uint32_t j = threadIdx.x; j < nblk; j += 1024) {
    const uint32_t x = s.blk_aux[j];
    a |= x & 15u;
    own += x >> SHX_OWN_SHIFT;
    if (xfer) v += s.blk_amt[j];
  }
  if (a) atomicOr(bits_s, a);
  if (own) atomicAdd(own_s, own);
  // the amounts: wave sums of the two 64-bit halves, one LDS word per wave, one barrier
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t lo = __shfl_xor((unsigned long long)(uint64_t)v, o, 64);
    const uint64_t hi = __shfl_xor((unsigned long long)(uint64_t)(v >> 64), o, 64);
    v += ((u128)hi << 64) | lo;
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();  // (also orders the LDS atomics above before thread 0 reads them)
  if (threadIdx.x != 0) return 0;
  u128 tot = 0;
  for (uint32_t w2 = 0; w2 < blockDim.x / 64; w2++) tot += red[w2];
  Globals* g = d.g;
  const uint32_t bits = *bits_s;
  uint32_t verdict = (bits & SHX_DUP) ? 1u : 0u;
  if (xfer) {
    g->batch_amount_sum += tot;
    if (bits & SHX_HUGE) g->batch_huge = 1;
    if (g->x_count + *own_s > d.x_max) verdict |= 2u;
    if (window_ovf_mode(g)) verdict |= 4u;
    // every owned balance field stays below 2^64 this window: k_sh_apply's adds need no carry
    const u128 top = g->ovf_bound + g->batch_amount_sum;
    g->small_win = (!g->batch_huge && top >= g->ovf_bound && (uint64_t)(top >> 64) == 0) ? 1u : 0u;
    const bool prefix = !(bits & SHX_NONMONO) && (bits & SHX_FRESH) && g->x_sorted == g->x_count;
    g->win_flags = prefix ? 2u : 0u;
  } else {
    if (g->acc_count + *own_s > d.acc_max) verdict |= 2u;
  }
  return verdict;
}

// Exchange 2's trailer, written whole by thread 0: the homes' out-of-class flag (k_sh_home /
// k_sh_decide) and this shard's owner verdicts (sh_close_fold), one word each.
__device__ inline void sh_trailer2(uint32_t* trailer2, uint32_t unsup, uint32_t verdict) {
  trailer2[0] = unsup;
  trailer2[1] = verdict & 1u;
  trailer2[2] = (verdict >> 1) & 1u;
  trailer2[3] = (verdict >> 2) & 1u;
}

// A shard home to no event of the window still folds its owner verdicts into exchange 2.
__global__ void __launch_bounds__(1024) k_sh_close(Dev d, Scratch s, uint32_t nblk, uint32_t xfer, uint32_t* trailer2) {
  __shared__ u128 red[1024 / 64];
  __shared__ uint32_t bits_s;
  __shared__ unsigned long long own_s;
  const uint32_t verdict = sh_close_fold(d, s, nblk, xfer, red, &bits_s, &own_s);
  if (threadIdx.x == 0) sh_trailer2(trailer2, 0u, verdict);
}

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

// Owned roles of an event (Scratch::bstatus): it reaches the account checks and this shard owns its
// debit account / credit account / id.
enum : uint8_t { ROLE_DR = 1, ROLE_CR = 2, ROLE_ID = 4 };

// ------------------------------------------------------------------------------------------------
// scan, in two passes so that the long dependent chains (validation, probes, claims) run on dense
// waves: k_sh_roles reads the ids of every event and compacts the events with an owned role, in
// event order, into per-segment lists (Scratch::wlist, segment k at k * SEG, Scratch::cnt_w[k]
// entries: event | candidate roles << 24); k_sh_owned works through those lists.
// ------------------------------------------------------------------------------------------------
__device__ inline uint32_t ol_event(uint32_t x) { return x & 0xFFFFFFu; }
__device__ inline uint32_t ol_roles(uint32_t x) { return x >> 24; }

template <bool XFER>
__global__ void __launch_bounds__(SEG) k_sh_roles(Dev d, Scratch s, const uint8_t* __restrict__ ev_bytes, uint32_t E,
                                                  XchView xch, uint32_t G, uint32_t me) {
  __shared__ uint32_t lds[SEG / 64];
  __shared__ uint32_t aux;
  const uint32_t i = blockIdx.x * SEG + threadIdx.x;
  if (threadIdx.x == 0) aux = 0;
  // exchange 1's trailer (written by later kernels of the window only): zeroed here, not by a memset;
  // so is the homes' out-of-class flag that k_sh_reply turns into exchange 2's trailer
  if (i < 4) xch.trailer[i] = 0;
  if (i == 0) d.g->sh_unsup = 0;
  __syncthreads();
  uint32_t roles = 0;
  if (i < E) {
    const uint4* q = reinterpret_cast<const uint4*>(ev_bytes + (size_t)i * 128);
    const tb_uint128_t id = rw_u128(q[0]);
    if (shard_of(id.lo, id.hi, G) == me) roles |= ROLE_ID;
    if (XFER) {
      const tb_uint128_t dra = rw_u128(q[1]), cra = rw_u128(q[2]);
      if (shard_of(dra.lo, dra.hi, G) == me) roles |= ROLE_DR;
      if (shard_of(cra.lo, cra.hi, G) == me) roles |= ROLE_CR;
      // the owned records extend the sorted prefix if the window's ids are strictly increasing
      bool nm = false;
      if (i > 0) nm = !(U(id) > U(reinterpret_cast<const tb_transfer_t*>(ev_bytes)[i - 1].id));
      if (nm) atomicOr(&aux, (uint32_t)SHX_NONMONO);
      if (i == 0 && U(id) > d.g->x_id_max) atomicOr(&aux, (uint32_t)SHX_FRESH);
      xch.acc[i] = 0;  // k_sh_owned writes the owned facts
    }
    xch.zw[i] = 0;
  }
  if (XFER) {  // the mismatch slots (every shard's, zero but its own writes) and this shard's count
    for (uint32_t k = i; k < G * SH_MIS_SLOTS; k += gridDim.x * SEG) xch.mis[k] = 0;
    if (i == 0) d.g->sh_mis = 0;
  }
  uint32_t tot;
  const uint32_t r = block_excl<SEG / 64>(roles ? 1u : 0u, lds, &tot);
  if (roles) s.wlist[blockIdx.x * SEG + r] = i | (roles << 24);
  if (threadIdx.x == 0) {
    s.cnt_w[blockIdx.x] = tot;
    s.blk_aux[blockIdx.x] = aux;
  }
}

// Owned work of segment blockIdx.x: the owner facts. The id owner reads the event whole, validates
// it and, if it reaches the account checks, claims the id and compares it with a stored transfer.
// The account owners need no validation: they read the account ids and the amount only (facts of an
// event its home rejects statically are never read, and the commit bit gates every effect); every
// amount they see counts toward the overflow bound, valid or not. Rewrites each entry's roles to the
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

// ones that carry effects.
__global__ void __launch_bounds__(SEG) k_sh_owned_ct(Dev d, Scratch s, const tb_transfer_t* __restrict__ ev, WinDesc w,
                                                     uint32_t epoch, XchView xch, uint32_t me) {
  __shared__ u128 red[SEG / 64];
  __shared__ uint32_t aux;
  const uint32_t k = blockIdx.x * SEG + threadIdx.x;
  if (threadIdx.x == 0) aux = 0;
  if (k == 0) check_window(w, d.g);
  // Window ids strictly increasing (k_sh_roles' per-segment bits, one launch per segment here too):
  // no in-window duplicate id can exist, so the id owner skips the key-map claim, a returning CAS per
  // owned id (the sharded path reads the key map for nothing else). Other blocks may be OR-ing
  // their own bits into these words meanwhile; bit SHX_NONMONO is never among them.
  uint32_t nm = 0;
  for (uint32_t j = threadIdx.x; j < gridDim.x; j += SEG)
    nm |= __hip_atomic_load(&s.blk_aux[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & (uint32_t)SHX_NONMONO;
  const bool mono = !__syncthreads_or((int)nm);
  u128 amount_upper = 0;
  const uint32_t n = s.cnt_w[blockIdx.x];
  bool owned_id = false;
  if (threadIdx.x < n) {
    const uint32_t x = s.wlist[k];
    const uint32_t i = ol_event(x), cand = ol_roles(x);
    uint32_t roles = 0, zw = 0;
    if (cand & ROLE_ID) {
      tb_transfer_t t = ev[i];
      uint32_t cls = 0;
      bool reach, unsup;
      (void)sh_static_ct(t, w, win_batch(w, i), i, &cls, &reach, &unsup);
      if (reach) {
        roles |= ROLE_ID;
        owned_id = true;
        bool dup = false;
        if (!mono) (void)sh_claim(d.g, s.bmap, s.bmask, reinterpret_cast<const uint8_t*>(ev), t.id, i, w.E, epoch, &dup);
        if (dup) atomicOr(&aux, (uint32_t)SHX_DUP);
        uint32_t xs = NONE32;
        if (x_may_exist(t.id, d.g->x_id_max)) {
          xs = x_find(d.x_tab, d.xr, d.x_mask, t.id);
          if (xs == NONE32) xs = x_prefix_find(d.xr, d.g->x_sorted, t.id);
        }
        zw |= 1 + (xs == NONE32 ? (uint32_t)TB_CT_OK : ct_exists(t, d.xr[xs]));
      }
    }
    if (cand & (ROLE_DR | ROLE_CR)) {
      const uint4* q = reinterpret_cast<const uint4*>(ev + i);
      const uint4 q1 = q[1], q2 = q[2], q3 = q[3];
      const uint32_t ledger = q[7].x;  // the event's ledger: each side's state is against it
      amount_upper = U(rw_u128(q3));
      uint32_t acc = 0;
      // up to two independent probes, one per owned side
#pragma unroll
      for (uint32_t side = 0; side < 2; side++) {
        if (!(cand & (side ? ROLE_CR : ROLE_DR))) continue;
        roles |= side ? ROLE_CR : ROLE_DR;
        AccEntry e;
        const uint32_t slot = acc_find(d.acc_tab, d.acc_mask, rw_u128(side ? q2 : q1), &e);
        (side ? s.cr_slot : s.dr_slot)[i] = slot;
        uint32_t st = SH_ACC_MISSING;
        if (slot != NONE32) {
          st = e.ledger == ledger ? SH_ACC_OK : SH_ACC_MISMATCH;
          // a limit (a balance read) or flags.history (a historical_balance row of balances after
          // the event, :1806-1841): outside the order-free class if the event commits
          const uint16_t lim = side ? TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS : TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS;
          if (e.flags & (lim | TB_ACCOUNT_HISTORY)) zw |= side ? SH_CR_LIMIT : SH_DR_LIMIT;
          if (st == SH_ACC_MISMATCH) {
            const uint32_t k2 = atomicAdd(&d.g->sh_mis, 1u);
            if (k2 < SH_MIS_SLOTS)
              xch.mis[me * SH_MIS_SLOTS + k2] = (1ull << 63) | ((unsigned long long)side << 52) |
                                                ((unsigned long long)i << 32) | e.ledger;
            else
              atomicOr(&aux, (uint32_t)SHX_DUP);  // (trailer 0: outside the class)
          }
        }
        acc |= st << (2 * side);
      }
      if (acc) xch.acc[i] = (uint8_t)acc;  // (one byte per event: both sides' owners write it only
                                           // when they are the same shard, else their bit pairs)
    }
    if (zw) xch.zw[i] = (uint8_t)zw;
    s.wlist[k] = i | (roles << 24);
  }
  if ((uint64_t)(amount_upper >> 64) != 0) atomicOr(&aux, (uint32_t)SHX_HUGE);
  {  // owned ids reaching the exists check: one LDS add per wave
    const uint32_t c = (uint32_t)__popcll(__ballot(owned_id));
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(&aux, c << SHX_OWN_SHIFT);
  }
  // block sum of the amounts below 2^64: wave sums of the two 64-bit halves, then one LDS word per wave
  const uint64_t a = ((uint64_t)(amount_upper >> 64) != 0) ? 0ull : (uint64_t)amount_upper;
  u128 v = a;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t lo = __shfl_xor((unsigned long long)(uint64_t)v, o, 64);
    const uint64_t hi = __shfl_xor((unsigned long long)(uint64_t)(v >> 64), o, 64);
    v += ((u128)hi << 64) | lo;
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {  // this segment's partials (sh_close_fold folds them)
    u128 tot = 0;
#pragma unroll
    for (int w2 = 0; w2 < SEG / 64; w2++) tot += red[w2];
    s.blk_amt[blockIdx.x] = tot;
    s.blk_aux[blockIdx.x] |= aux;  // k_sh_roles wrote the segment's prefix bits
  }
}

__global__ void __launch_bounds__(SEG) k_sh_owned_ca(Dev d, Scratch s, const tb_account_t* __restrict__ ev, WinDesc w,
                                                     uint32_t epoch, XchView xch) {
  __shared__ uint32_t aux;
  const uint32_t k = blockIdx.x * SEG + threadIdx.x;
  if (threadIdx.x == 0) aux = 0;
  if (k == 0) check_window(w, d.g);
  __syncthreads();
  const uint32_t n = s.cnt_w[blockIdx.x];
  if (threadIdx.x < n) {
    const uint32_t i = ol_event(s.wlist[k]);
    const tb_account_t a = ev[i];
    uint32_t cls = 0, roles = 0;
    bool reach;
    (void)sh_static_ca(a, &cls, &reach);
    if (reach) {
      roles = ROLE_ID;
      atomicAdd(&aux, 1u << SHX_OWN_SHIFT);
      bool dup;
      (void)sh_claim(d.g, s.bmap, s.bmask, reinterpret_cast<const uint8_t*>(ev), a.id, i, w.E, epoch, &dup);
      if (dup) atomicOr(&aux, (uint32_t)SHX_DUP);
      AccEntry e;
      const uint32_t slot = acc_find(d.acc_tab, d.acc_mask, a.id, &e);
      xch.zw[i] = (uint8_t)(1 + (slot == NONE32 ? (uint32_t)TB_CA_OK : ca_exists(a, d.acc[slot])));
    }
    s.wlist[k] = i | (roles << 24);
  }
  __syncthreads();
  if (threadIdx.x == 0) s.blk_aux[blockIdx.x] |= aux;
}

// ------------------------------------------------------------------------------------------------
// home slice [e0, e1): validation codes, decisions, replies, commit bits.
// ------------------------------------------------------------------------------------------------
template <bool XFER>
__global__ void __launch_bounds__(256) k_sh_home(Scratch s, const uint8_t* __restrict__ ev_bytes, WinDesc w,
                                                 uint32_t e0, uint32_t e1, uint32_t* trailer2,
                                                 unsigned long long* bits, uint32_t nwords) {
  // every commit-bit word of the window starts at zero (k_sh_reply writes this home's words; the
  // all-reduce sums every shard's): zeroed here rather than by a memset launch
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < nwords; k += gridDim.x * blockDim.x) bits[k] = 0;
  // so do the home segments' failure counts (k_sh_decide adds to them)
  const uint32_t nseg = (e1 - 1) / SEG - e0 / SEG + 1;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < nseg; k += gridDim.x * blockDim.x) s.cnt_bad[k] = 0;
  const uint32_t i = e0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= e1) return;
  const uint32_t b = win_batch(w, i);
  uint32_t cls = 0, code;
  bool reach, unsup = false;
  if (XFER) {
    tb_transfer_t t = reinterpret_cast<const tb_transfer_t*>(ev_bytes)[i];
    code = sh_static_ct(t, w, b, i, &cls, &reach, &unsup);
  } else {
    code = sh_static_ca(reinterpret_cast<const tb_account_t*>(ev_bytes)[i], &cls, &reach);
  }
  if (unsup) atomicOr(&trailer2[0], 1u);
  if (reach) cls |= C_REACH;
  if (code != CONT) cls |= C_STATIC;
  s.code[i] = code;
  s.cls[i] = cls;
  s.batch[i] = (uint16_t)b;
}

// An event's code from the exchanged owner facts (its static code first).
template <bool XFER>
__device__ inline uint32_t sh_code(const Scratch& s, const uint8_t* ev, const XchView& xch, uint32_t j,
                                   uint32_t* trailer2) {
  const uint32_t code = s.code[j];
  if (code != CONT) return code;
  const uint32_t zw = xch.zw[j];
  const uint32_t z = (zw & SH_Z_MASK) - 1;
  if (!XFER) return z;
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
  if (z != TB_CT_OK) return z;  // exists* (:1506-1507)
  // Reaches the balance checks: overflow cannot fail in a class window; a limit flag on either
  // account is a balance read (:1546-1547), and flags.history a row of balances after the event
  // (:1806-1841): outside the class.
  if (zw & (SH_DR_LIMIT | SH_CR_LIMIT)) atomicOr(&trailer2[0], 1u);
  return TB_CT_OK;
}

template <bool XFER>
__global__ void __launch_bounds__(256) k_sh_decide(Scratch s, const uint8_t* ev, WinDesc w, uint32_t e0, uint32_t e1,
                                                   XchView xch, uint32_t* trailer2) {
  const uint32_t i = e0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= e1) return;
  const uint32_t b = s.batch[i];
  const uint32_t first = w.off[b], last = w.off[b + 1] - 1;
  if (i != first && (s.cls[i - 1] & C_LINKED)) return;  // chain member: its head decides
  const uint32_t cls = s.cls[i];
  const uint32_t k0 = e0 / SEG;  // failures per home segment (s.cnt_bad[seg - k0]: k_sh_reply's ranks)
  if (!(cls & C_LINKED)) {
    const uint32_t code = sh_code<XFER>(s, ev, xch, i, trailer2);
    s.code[i] = code;
    if (code == TB_CT_OK) s.cls[i] = cls | C_COMMIT;
    else atomicAdd(&s.cnt_bad[i / SEG - k0], 1u);
    return;
  }
  // chain head: members i..end (:1240-1300). No member's outcome depends on another member's
  // effects in a class window, so the chain fails at its first failing member.
  uint32_t end = i, f = NONE32;
  for (uint32_t j = i;; j++) {
    const bool lj = s.cls[j] & C_LINKED;
    uint32_t code = sh_code<XFER>(s, ev, xch, j, trailer2);
    if (lj && j == last) code = TB_CT_LINKED_EVENT_CHAIN_OPEN;  // :1247
    s.code[j] = code;
    if (code != TB_CT_OK && f == NONE32) f = j;
    end = j;
    if (!lj || j == last) break;
  }
  for (uint32_t j = i; j <= end; j++) {
    const uint32_t cj = s.cls[j];
    if (f == NONE32) {
      s.cls[j] = cj | C_COMMIT;
    } else if (j != f && !((cj & C_LINKED) && j == last)) {
      s.code[j] = TB_CT_LINKED_EVENT_FAILED;  // back-fill before f, broken chain after f
    }
  }
  if (f != NONE32) {  // every member failed; the chain may span several segments
    for (uint32_t g = i / SEG; g <= end / SEG; g++)
      atomicAdd(&s.cnt_bad[g - k0], std::min(end + 1, (g + 1) * SEG) - std::max(i, g * SEG));
  }
}

// Home slice: replies of batches [hb0, hb1) (batch_base relative to hb0, indices batch-relative) and
// the commit bit of every slice event (one 64-bit word per wave; words are window-aligned).
__global__ void __launch_bounds__(SEG) k_sh_reply(Dev d, Scratch s, WinDesc w, uint32_t hb0, uint32_t hb1, uint32_t e0,
                                                  uint32_t e1, uint32_t k0, FinalOut o, unsigned long long* bits,
                                                  const uint32_t* unsup, uint32_t* trailer2, uint32_t nscan,
                                                  uint32_t xfer) {
  __shared__ uint32_t lds[SEG / 64];
  __shared__ u128 red[SEG / 64];
  __shared__ uint32_t bits_s;
  __shared__ unsigned long long own_s;
  if (blockIdx.x == 0) {  // (block-uniform) exchange 2's trailer, instead of a memset before the homes
    const uint32_t verdict = sh_close_fold(d, s, nscan, xfer, red, &bits_s, &own_s);
    if (threadIdx.x == 0) sh_trailer2(trailer2, *unsup, verdict);
  }
  const uint32_t i = (k0 + blockIdx.x) * SEG + threadIdx.x;
  const bool mine = i >= e0 && i < e1;
  uint32_t cls = 0, code = TB_CT_OK;
  if (mine) {
    cls = s.cls[i];
    code = s.code[i];
  }
  const uint32_t bad = code != TB_CT_OK;
  const uint32_t pbad = seg_prefix<SEG>(s.cnt_bad, blockIdx.x, lds);
  uint32_t tot_bad;
  const uint32_t rbad = pbad + block_excl<SEG / 64>(bad, lds, &tot_bad);
  const unsigned long long m = __ballot(mine && (cls & C_COMMIT));
  if ((threadIdx.x & 63) == 0 && i < e1 && i + 64 > e0) bits[i / 64] = m;
  if (!mine) return;
  const uint32_t b = s.batch[i];
  if (i == w.off[b]) {
    // event i opens batch b and every empty home batch just before it
    for (int32_t bb = (int32_t)b; bb >= (int32_t)hb0 && w.off[bb] == i; bb--) o.batch_base[bb - hb0] = rbad;
  }
  if (bad && sh_guard(d.g, rbad < e1 - e0, 2, rbad)) {
    tb_create_result_t r;
    r.index = i - w.off[b];
    r.result = code;
    o.results[rbad] = r;
  }
  if (i == e1 - 1) {
    const uint32_t total_bad = rbad + bad;
    for (int32_t bb = (int32_t)hb1; bb >= (int32_t)hb0 && w.off[bb] == e1; bb--) o.batch_base[bb - hb0] = total_bad;
    if (o.out_count) *o.out_count = total_bad;
    d.g->result_count = total_bad;
  }
}

// ------------------------------------------------------------------------------------------------
// apply: whole window, owned roles of committed events.
// ------------------------------------------------------------------------------------------------
__device__ inline bool sh_bit(const unsigned long long* bits, uint32_t i) { return (bits[i / 64] >> (i & 63)) & 1ull; }

// Verdict of the window, identical on every shard: exchange 2's trailer (homes: an event outside the
// class; owners: duplicate id, capacity, overflow bound).
__device__ inline bool sh_abort(const uint32_t* trailer2) {
  return (trailer2[0] | trailer2[1] | trailer2[2] | trailer2[3]) != 0;
}

// Per segment: committed owned-id entries (insert counts), over the segment lists.
__global__ void __launch_bounds__(SEG) k_sh_icount(Dev d, Scratch s, uint32_t xfer, const unsigned long long* bits) {
  __shared__ uint32_t lds[SEG / 64];
  if (blockIdx.x == 0 && threadIdx.x == 0) d.g->base = xfer ? d.g->x_count : d.g->acc_count;  // k_sh_apply's base
  uint32_t ins = 0;
  if (threadIdx.x < s.cnt_w[blockIdx.x]) {
    const uint32_t x = s.wlist[blockIdx.x * SEG + threadIdx.x];
    ins = ((ol_roles(x) & ROLE_ID) && sh_bit(bits, ol_event(x))) ? 1u : 0u;
  }
  const uint32_t tot = block_sum<SEG / 64>(ins, lds);
  if (threadIdx.x == 0) s.cnt_ins[blockIdx.x] = tot;
}

template <bool XFER>
__global__ void __launch_bounds__(SEG) k_sh_apply(Dev d, Scratch s, const uint8_t* ev_bytes, WinDesc w,
                                                  const uint32_t* trailer2, const unsigned long long* bits,
                                                  ChgLog chg, uint32_t chg_epoch) {
  __shared__ uint32_t lds[SEG / 64];
  __shared__ u128 ldsm[SEG / 64];
  // inserted transfer records, compacted per wave and stored as one contiguous run (as in k_final)
  __shared__ uint4 stage[XFER ? SEG * 8 : 1];
  Globals* g = d.g;
  const bool last_block = blockIdx.x == gridDim.x - 1;
  if (sh_abort(trailer2)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&g->window_error, 2u);
    if (last_block && threadIdx.x == 0) sh_window_reset(g, XFER, 0, false);
    return;
  }
  const bool prefix_win = XFER && (g->win_flags & 2u) != 0;  // sh_close_fold
  const bool small = XFER && g->small_win != 0;              // sh_close_fold
  const uint64_t xbase = g->base;  // captured by k_sh_icount: the last block rewrites the count
  const uint32_t n = s.cnt_w[blockIdx.x];
  uint32_t i = 0, roles = 0;
  bool commit = false;
  if (threadIdx.x < n) {
    const uint32_t x = s.wlist[blockIdx.x * SEG + threadIdx.x];
    i = ol_event(x);
    roles = ol_roles(x);
    commit = roles && sh_bit(bits, i);
  }
  bool ins = commit && (roles & ROLE_ID);
  const uint32_t pins = seg_prefix<SEG>(s.cnt_ins, blockIdx.x, lds);
  uint32_t tot_ins;
  const uint32_t rins = pins + block_excl<SEG / 64>(ins ? 1u : 0u, lds, &tot_ins);
  if (XFER) {
    const u128 key = ins ? U(reinterpret_cast<const tb_transfer_t*>(ev_bytes)[i].id) : (u128)0;
    const u128 m = wave_max_u128(key);
    if ((threadIdx.x & 63) == 0) ldsm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
      u128 bm = ldsm[0];
      for (int q = 1; q < SEG / 64; q++) bm = umax128(bm, ldsm[q]);
      if (bm > g->x_id_max) atomic_bound_u128(&g->x_id_max, bm);
    }
  }
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)rins, 0);  // the wave's first insert rank (all lanes active here)
  if (commit) {
    if (XFER) {
      uint32_t drs = (roles & ROLE_DR) ? s.dr_slot[i] : NONE32, crs = (roles & ROLE_CR) ? s.cr_slot[i] : NONE32;
      if (drs != NONE32 && !sh_guard(g, drs < d.acc_max, 3, drs)) drs = NONE32;
      if (crs != NONE32 && !sh_guard(g, crs < d.acc_max, 4, crs)) crs = NONE32;
      if (ins && !sh_guard(g, xbase + rins < d.x_max, 5, xbase + rins)) ins = false;
      const u128 a = U(reinterpret_cast<const tb_transfer_t*>(ev_bytes)[i].amount);
      Add128 a_dr, a_cr;
      if (drs != NONE32) a_dr.issue(&d.acc[drs].debits_posted, a, small);
      if (crs != NONE32) a_cr.issue(&d.acc[crs].credits_posted, a, small);
      if (chg.mark) {  // write-back stream (changes.h): the owned accounts this window changed
        if (drs != NONE32) chg.mark[drs] = chg_epoch;
        if (crs != NONE32) chg.mark[crs] = chg_epoch;
      }
      if (ins) {
        const uint64_t slot = xbase + rins;
        tb_transfer_t t2 = reinterpret_cast<const tb_transfer_t*>(ev_bytes)[i];
        t2.timestamp = win_ts(w, win_batch(w, i), i);
        // ranks of a wave's inserts are consecutive (block_excl); a failed slot guard can only drop
        // a suffix of them, so the staged run below stays gap-free
        const uint4* tw = reinterpret_cast<const uint4*>(&t2);
        uint4* ws = stage + (threadIdx.x >> 6) * 512;
#pragma unroll
        for (int q = 0; q < 8; q++) ws[(rins - r0) * 8 + q] = tw[q];
        if (!prefix_win) x_insert(d.x_tab, d.x_mask, t2.id, (uint32_t)slot);
        d.xstatus[slot] = 0;
      }
      a_dr.finish();
      a_cr.finish();
    } else if (ins && sh_guard(g, xbase + rins < d.acc_max, 6, xbase + rins)) {
      const uint64_t slot = xbase + rins;
      tb_account_t a = reinterpret_cast<const tb_account_t*>(ev_bytes)[i];
      a.timestamp = win_ts(w, win_batch(w, i), i);
      d.acc[slot] = a;
      d.hot[slot] = 0;
      acc_insert(d.acc_tab, d.acc_mask, a.id, (uint32_t)slot, a.ledger, a.flags);
    }
  }
  if (XFER) {
    const uint32_t nins = (uint32_t)__popcll(__ballot(ins));
    wave_sync();
    if (nins) {
      const uint4* ws = stage + (threadIdx.x >> 6) * 512;
      uint4* dst = reinterpret_cast<uint4*>(d.xr) + (size_t)(xbase + r0) * 8;
      for (uint32_t k = threadIdx.x & 63; k < nins * 8; k += 64) st_stream(dst + k, ws[k]);
    }
  }
  if (last_block && threadIdx.x == 0) {
    const uint64_t total = xbase + pins + tot_ins;
    g->events_total += w.E;
    if (prefix_win) g->x_sorted = total;
    sh_window_reset(g, XFER, total, true);
  }
}
