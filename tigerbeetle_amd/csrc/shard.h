// shard.h — hash-sharded commit across G GPUs of one node (one engine per GPU).
//
// Ownership: an account belongs to shard_of(account id), a transfer to shard_of(transfer id). Every
// shard holds the whole prepared window in HBM (the replica hands each GPU the same prepare body)
// and walks all of it, but touches state only for what it owns:
//
//   k_sh_prep    grid   stateless validation (identical on every shard, state_machine.zig:1424-1439,
//                       1465-1489); for each event that passes, the debit-account owner resolves the
//                       debit account, the credit-account owner the credit account, the transfer-id
//                       owner the id (pre-window `exists` comparison, :1506-1507, and in-window
//                       duplicates through the window key map). Each writes its part of the event's
//                       9 B of exchange bytes; the other parts stay zero.
//   (caller)            byte-wise sum all-reduce of the exchange bytes across the shards (RCCL over
//                       xGMI). Every bit has exactly one writer, so the sum is the union of the parts.
//   k_sh_decide  grid   every shard now holds the same per-event facts and decides every event the
//                       same way: account lookups (:1496-1497), ledgers (:1503-1504), exists, then
//                       linked chains (:1240-1300); identical replies on all shards.
//   k_sh_count   grid   per-segment failure / owned-insert counts; captures the store base.
//   k_sh_final   grid   replies, and only owned effects: the id owner appends the record and indexes the
//                       id, the debit/credit owners add the amount (exact 128-bit atomics).
//
// The sharded class is the order-free one: no balance read (no limit flag on a touched
// account, no balancing), no two-phase, no in-window duplicate id, overflow-free window. Then every
// event's outcome is a function of the owners' facts alone, and the effects commute. A window outside
// the class is detected before anything is applied, identically on every shard (its flags travel in
// the exchange's trailer or follow from the reduced bytes), and fails with TBG_E_UNSUPPORTED at
// tbg_sync: no shard applies any of it.
#pragma once
#include "sm_logic.h"
#include "walker.h"
#include "window.h"

// Exchange bytes of a window of E events (summed byte-wise over the shards: every bit has exactly
// one writer, so the byte sum is the union with no carries; one uint8 all-reduce):
//   [0, 16)         trailer, 4 x u32: shards that saw an unsupported event, shards over capacity,
//                   shards whose overflow bound does not clear the window's amounts, unused
//   create_transfers:
//   [16, 16+4E)     debit account's ledger (its owner; 0 = not found: a live ledger is never 0, :1436)
//   [16+4E, 16+8E)  credit account's ledger
//   [16+8E, 16+9E)  bits 0-5: 1 + (TB_CT_OK or the exists* code), by the transfer-id owner;
//                   bit 6: the debit account has debits_must_not_exceed_credits (its owner);
//                   bit 7: the credit account has credits_must_not_exceed_debits (its owner)
//   create_accounts:
//   [16, 16+E)      bits 0-5: 1 + the id owner's code
enum : uint32_t { SH_Z_MASK = 0x3F, SH_DR_LIMIT = 0x40, SH_CR_LIMIT = 0x80 };

struct XchView {
  uint32_t* trailer;
  uint32_t *drl, *crl;  // transfers only
  uint8_t* zw;
};
__host__ __device__ inline uint64_t xch_bytes(bool xfer, uint32_t E) { return 16 + (xfer ? 9ull : 1ull) * E; }
__host__ __device__ inline XchView xch_view(void* base, uint32_t E, bool xfer) {
  uint8_t* p = reinterpret_cast<uint8_t*>(base);
  XchView v;
  v.trailer = reinterpret_cast<uint32_t*>(p);
  v.drl = xfer ? reinterpret_cast<uint32_t*>(p + 16) : nullptr;
  v.crl = xfer ? reinterpret_cast<uint32_t*>(p + 16 + 4ull * E) : nullptr;
  v.zw = p + 16 + (xfer ? 8ull * E : 0ull);
  return v;
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

// End-of-window device state (the last event's thread of k_sh_final). Nothing written here is read
// by k_sh_final's other blocks, which may still be running: their store base is Globals::base
// (captured by k_sh_count) and sh_unsup is cleared by the next window's k_sh_close.
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

// After prep (stream-ordered, one block): folds the prep blocks' partials (amount sums, huge /
// unsupported bits, owned-id counts; no same-address atomics across blocks) and closes the window's
// local facts into the trailer words: unsupported, capacity and overflow verdicts. (A separate
// launch, not a last-block pattern: no device fences in the sharded kernels.)
__global__ void __launch_bounds__(1024) k_sh_close(Dev d, Scratch s, uint32_t nblk, uint32_t* trailer, uint32_t xfer) {
  __shared__ u128 red[1024];
  __shared__ uint32_t bits;
  __shared__ unsigned long long own_s;
  if (threadIdx.x == 0) {
    bits = 0;
    own_s = 0;
  }
  __syncthreads();
  u128 v = 0;
  uint32_t a = 0;
  unsigned long long own = 0;
  for (uint32_t j = threadIdx.x; j < nblk; j += 1024) {
    const uint32_t x = s.blk_aux[j];
    a |= x & 3u;
    own += x >> 2;
    if (xfer) v += s.blk_amt[j];
  }
  if (a) atomicOr(&bits, a);
  if (own) atomicAdd(&own_s, own);
  const u128 tot = xfer ? block_sum_u128(v, red) : (u128)0;
  if (threadIdx.x != 0) return;
  Globals* g = d.g;
  g->sh_own = 0;
  g->sh_unsup = 0;  // the previous window's verdict (read by every block of its k_sh_final)
  if (bits & 2u) trailer[0] = 1;
  if (xfer) {
    g->batch_amount_sum += tot;
    if (bits & 1u) g->batch_huge = 1;
    if (g->x_count + own_s > d.x_max) trailer[1] = 1;
    if (window_ovf_mode(g)) trailer[2] = 1;
  } else {
    if (g->acc_count + own_s > d.acc_max) trailer[1] = 1;
  }
}

// ------------------------------------------------------------------------------------------------
// create_transfers: prep
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_sh_prep_ct(Dev d, Scratch s, const tb_transfer_t* __restrict__ ev, WinDesc w,
                                                    uint32_t epoch, XchView xch, uint32_t G, uint32_t me) {
  __shared__ u128 red[256];
  __shared__ uint32_t huge_any, unsup, own;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (threadIdx.x == 0) huge_any = unsup = own = 0;
  if (i == 0) check_window(w, d.g);
  __syncthreads();
  u128 amount_upper = 0;
  if (i < w.E) {
    tb_transfer_t t = ev[i];
    const uint32_t b = win_batch(w, i);
    uint32_t cls = 0, code, dr_slot = NONE32, cr_slot = NONE32, id_ent = NONE32;
    uint32_t drl = 0, crl = 0, zw = 0;
    const uint16_t f = t.flags;
    if (f & TB_TRANSFER_LINKED) cls |= C_LINKED;
    if (t.timestamp != 0) {
      cls |= C_TSNZ;
      code = TB_CT_TIMESTAMP_MUST_BE_ZERO;
    } else {
      t.timestamp = win_ts(w, b, i);
      code = ct_head(t);
      if (code == CONT && (f & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING))) {
        code = pv_validate(t);
        if (code == CONT) atomicOr(&unsup, 1u);  // two-phase resolution: outside the sharded class
      } else if (code == CONT) {
        code = ct_validate(t);
        if (code == CONT) {
          if (f & (TB_TRANSFER_PENDING | TB_TRANSFER_BALANCING_DEBIT | TB_TRANSFER_BALANCING_CREDIT))
            atomicOr(&unsup, 1u);
          cls |= C_REACH;
          amount_upper = U(t.amount);
          // up to three independent probes, one per owned side
          if (shard_of(t.debit_account_id.lo, t.debit_account_id.hi, G) == me) {
            AccEntry e;
            dr_slot = acc_find(d.acc_tab, d.acc_mask, t.debit_account_id, &e);
            if (dr_slot != NONE32) {
              drl = e.ledger;
              if (e.flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) zw |= SH_DR_LIMIT;
            }
          }
          if (shard_of(t.credit_account_id.lo, t.credit_account_id.hi, G) == me) {
            AccEntry e;
            cr_slot = acc_find(d.acc_tab, d.acc_mask, t.credit_account_id, &e);
            if (cr_slot != NONE32) {
              crl = e.ledger;
              if (e.flags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS) zw |= SH_CR_LIMIT;
            }
          }
          if (shard_of(t.id.lo, t.id.hi, G) == me) {
            cls |= C_OWN;
            atomicAdd(&own, 1u);
            bool dup;
            id_ent = sh_claim(d.g, s.bmap, s.bmask, reinterpret_cast<const uint8_t*>(ev), t.id, i, w.E, epoch, &dup);
            if (dup) atomicOr(&unsup, 1u);
            uint32_t xs = NONE32;
            if (x_may_exist(t.id, d.g->x_id_max)) {
              xs = x_find(d.x_tab, d.xr, d.x_mask, t.id);
              if (xs == NONE32) xs = x_prefix_find(d.xr, d.g->x_sorted, t.id);
            }
            zw |= 1 + (xs == NONE32 ? (uint32_t)TB_CT_OK : ct_exists(t, d.xr[xs]));
          }
        }
      }
    }
    if (code != CONT) cls |= C_STATIC;
    s.code[i] = code;
    s.cls[i] = cls;
    s.batch[i] = (uint16_t)b;
    s.dr_slot[i] = dr_slot;
    s.cr_slot[i] = cr_slot;
    s.id_ent[i] = id_ent;
    xch.drl[i] = drl;
    xch.crl[i] = crl;
    xch.zw[i] = (uint8_t)zw;
  }
  if ((uint64_t)(amount_upper >> 64) != 0) atomicOr(&huge_any, 1u);
  red[threadIdx.x] = ((uint64_t)(amount_upper >> 64) != 0) ? 0 : amount_upper;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) {  // this block's partials (k_sh_close folds them)
    s.blk_amt[blockIdx.x] = red[0];
    s.blk_aux[blockIdx.x] = (huge_any ? 1u : 0u) | (unsup ? 2u : 0u) | (own << 2);
  }
}

// ------------------------------------------------------------------------------------------------
// create_accounts: prep
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_sh_prep_ca(Dev d, Scratch s, const tb_account_t* __restrict__ ev, WinDesc w,
                                                    uint32_t epoch, XchView xch, uint32_t G, uint32_t me) {
  __shared__ uint32_t unsup, own;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (threadIdx.x == 0) unsup = own = 0;
  if (i == 0) check_window(w, d.g);
  __syncthreads();
  if (i < w.E) {
    const tb_account_t a = ev[i];
    const uint32_t b = win_batch(w, i);
    uint32_t cls = 0, code, id_ent = NONE32, zw = 0;
    if (a.flags & TB_ACCOUNT_LINKED) cls |= C_LINKED;
    if (a.timestamp != 0) {
      cls |= C_TSNZ;
      code = TB_CA_TIMESTAMP_MUST_BE_ZERO;
    } else {
      code = ca_validate(a);
      if (code == CONT) {
        cls |= C_REACH;
        if (shard_of(a.id.lo, a.id.hi, G) == me) {
          cls |= C_OWN;
          atomicAdd(&own, 1u);
          bool dup;
          id_ent = sh_claim(d.g, s.bmap, s.bmask, reinterpret_cast<const uint8_t*>(ev), a.id, i, w.E, epoch, &dup);
          if (dup) atomicOr(&unsup, 1u);
          AccEntry e;
          const uint32_t slot = acc_find(d.acc_tab, d.acc_mask, a.id, &e);
          zw = 1 + (slot == NONE32 ? (uint32_t)TB_CA_OK : ca_exists(a, d.acc[slot]));
        }
      }
    }
    if (code != CONT) cls |= C_STATIC;
    s.code[i] = code;
    s.cls[i] = cls;
    s.batch[i] = (uint16_t)b;
    s.id_ent[i] = id_ent;
    s.dr_slot[i] = NONE32;
    s.cr_slot[i] = NONE32;
    xch.zw[i] = (uint8_t)zw;
  }
  __syncthreads();
  if (threadIdx.x == 0) s.blk_aux[blockIdx.x] = (unsup ? 2u : 0u) | (own << 2);  // k_sh_close folds them
}

// ------------------------------------------------------------------------------------------------
// decide: every shard, every event, from the reduced exchange words.
// ------------------------------------------------------------------------------------------------
template <bool XFER>
__device__ inline uint32_t sh_code(const Dev& d, const Scratch& s, const uint8_t* ev, const XchView& xch, uint32_t j) {
  const uint32_t code = s.code[j];
  if (code != CONT) return code;
  const uint32_t zw = xch.zw[j];
  const uint32_t z = (zw & SH_Z_MASK) - 1;
  if (!XFER) return z;
  const uint32_t drl = xch.drl[j], crl = xch.crl[j];
  if (drl == 0) return TB_CT_DEBIT_ACCOUNT_NOT_FOUND;  // :1496-1497
  if (crl == 0) return TB_CT_CREDIT_ACCOUNT_NOT_FOUND;
  if (drl != crl) return TB_CT_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER;  // :1503-1504
  if (reinterpret_cast<const tb_transfer_t*>(ev)[j].ledger != drl)
    return TB_CT_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS;
  if (z != TB_CT_OK) return z;  // exists* (:1506-1507)
  // Reaches the balance checks: overflow cannot fail in a class window; a limit flag on either
  // account is a balance read (:1546-1547), outside the class.
  if (zw & (SH_DR_LIMIT | SH_CR_LIMIT)) atomicOr(&d.g->sh_unsup, 1u);
  return TB_CT_OK;
}

template <bool XFER>
__global__ void __launch_bounds__(256) k_sh_decide(Dev d, Scratch s, const uint8_t* ev, WinDesc w, XchView xch) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0 && (xch.trailer[0] | xch.trailer[1] | xch.trailer[2])) atomicOr(&d.g->sh_unsup, 1u);
  if (i >= w.E) return;
  const uint32_t b = s.batch[i];
  const uint32_t first = w.off[b], last = w.off[b + 1] - 1;
  if (i != first && (s.cls[i - 1] & C_LINKED)) return;  // chain member: its head decides
  const uint32_t cls = s.cls[i];
  if (!(cls & C_LINKED)) {
    const uint32_t code = sh_code<XFER>(d, s, ev, xch, i);
    s.code[i] = code;
    if (code == TB_CT_OK) s.cls[i] = cls | C_COMMIT | ((cls & C_OWN) ? C_INSERTED : 0u);
    return;
  }
  // chain head: members i..end (:1240-1300). No member's outcome depends on another member's
  // effects in a class window, so the chain fails at its first failing member.
  uint32_t end = i, f = NONE32;
  for (uint32_t j = i;; j++) {
    const bool lj = s.cls[j] & C_LINKED;
    uint32_t code = sh_code<XFER>(d, s, ev, xch, j);
    if (lj && j == last) code = TB_CT_LINKED_EVENT_CHAIN_OPEN;  // :1247
    s.code[j] = code;
    if (code != TB_CT_OK && f == NONE32) f = j;
    end = j;
    if (!lj || j == last) break;
  }
  for (uint32_t j = i; j <= end; j++) {
    const uint32_t cj = s.cls[j];
    if (f == NONE32) {
      s.cls[j] = cj | C_COMMIT | ((cj & C_OWN) ? C_INSERTED : 0u);
    } else if (j != f && !((cj & C_LINKED) && j == last)) {
      s.code[j] = TB_CT_LINKED_EVENT_FAILED;  // back-fill before f, broken chain after f
    }
  }
}

// Per-segment failure / owned-insert counts (k_wcount with the sharded boundary fences).
__global__ void __launch_bounds__(SEG) k_sh_count(Dev d, Scratch s, uint32_t E, uint32_t xfer) {
  __shared__ uint32_t lds[SEG / 64];
  const uint32_t i = blockIdx.x * SEG + threadIdx.x;
  if (i == 0) d.g->base = xfer ? d.g->x_count : d.g->acc_count;  // k_sh_final's store base
  uint32_t nbad = 0, nins = 0;
  if (i < E) {
    nbad = s.code[i] != TB_CT_OK;
    nins = (s.cls[i] & C_INSERTED) ? 1u : 0u;
  }
  nbad = block_sum<SEG / 64>(nbad, lds);
  nins = block_sum<SEG / 64>(nins, lds);
  if (threadIdx.x == 0) {
    s.cnt_bad[blockIdx.x] = nbad;
    s.cnt_ins[blockIdx.x] = nins;
  }
}

// ------------------------------------------------------------------------------------------------
// final: replies (every shard) and owned effects.
// ------------------------------------------------------------------------------------------------
template <bool XFER>
__global__ void __launch_bounds__(SEG) k_sh_final(Dev d, Scratch s, const uint8_t* ev_bytes, WinDesc w, FinalOut o) {
  __shared__ uint32_t lds[SEG / 64];
  __shared__ unsigned long long ldsm[SEG / 64];
  Globals* g = d.g;
  const bool unsup = __hip_atomic_load(&g->sh_unsup, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  const uint32_t E = w.E;
  const uint32_t i = blockIdx.x * SEG + threadIdx.x;
  uint32_t cls = 0, code = TB_CT_OK;
  if (i < E) {
    cls = s.cls[i];
    code = s.code[i];
  }
  bool ins = (cls & C_INSERTED) != 0;
  const uint32_t bad = code != TB_CT_OK;
  const uint32_t pbad = seg_prefix<SEG>(s.cnt_bad, blockIdx.x, lds);
  const uint32_t pins = seg_prefix<SEG>(s.cnt_ins, blockIdx.x, lds);
  uint32_t tot_bad, tot_ins;
  const uint32_t rbad = pbad + block_excl<SEG / 64>(bad, lds, &tot_bad);
  const uint32_t rins = pins + block_excl<SEG / 64>(ins ? 1u : 0u, lds, &tot_ins);
  if (XFER) {
    const unsigned long long key =
        (!unsup && ins && i < E) ? x_id_key(reinterpret_cast<const tb_transfer_t*>(ev_bytes)[i].id) : 0ull;
    const unsigned long long m = block_max_u64<SEG / 64>(key, ldsm);
    if (threadIdx.x == 0 && m > g->x_id_max) atomicMax(reinterpret_cast<unsigned long long*>(&g->x_id_max), m);
  }
  if (i >= E) return;
  if (unsup) {
    if (i == 0) atomicOr(&g->window_error, 2u);
    if (i == E - 1) sh_window_reset(g, XFER, 0, false);
    return;
  }
  const uint64_t xbase = g->base;  // captured by k_sh_count: the last thread rewrites the count
  const uint32_t b = s.batch[i];
  if (i == w.off[b]) {
    for (int32_t bb = (int32_t)b; bb >= 0 && w.off[bb] == i; bb--) o.batch_base[bb] = rbad;
  }
  if (bad && sh_guard(g, rbad < E, 2, rbad)) {
    tb_create_result_t r;
    r.index = i - w.off[b];
    r.result = code;
    o.results[rbad] = r;
  }
  if (XFER) {
    uint32_t drs = s.dr_slot[i], crs = s.cr_slot[i];
    if (drs != NONE32 && !sh_guard(g, drs < d.acc_max, 3, drs)) drs = NONE32;
    if (crs != NONE32 && !sh_guard(g, crs < d.acc_max, 4, crs)) crs = NONE32;
    if (ins && !sh_guard(g, xbase + rins < d.x_max, 5, xbase + rins)) ins = false;
    if ((cls & C_COMMIT) && ((drs != NONE32) | (crs != NONE32) | ins)) {
      tb_transfer_t t2 = reinterpret_cast<const tb_transfer_t*>(ev_bytes)[i];
      const u128 a = U(t2.amount);
      Add128 a_dr, a_cr;
      if (drs != NONE32) a_dr.issue(&d.acc[drs].debits_posted, a, false);
      if (crs != NONE32) a_cr.issue(&d.acc[crs].credits_posted, a, false);
      if (ins) {
        const uint64_t slot = xbase + rins;
        t2.timestamp = win_ts(w, b, i);
        d.xr[slot] = t2;
        x_insert(d.x_tab, d.x_mask, t2.id, (uint32_t)slot);
        d.xstatus[slot] = 0;
      }
      a_dr.finish();
      a_cr.finish();
    }
  } else if (ins && sh_guard(g, xbase + rins < d.acc_max, 6, xbase + rins)) {
    const uint64_t slot = xbase + rins;
    tb_account_t a = reinterpret_cast<const tb_account_t*>(ev_bytes)[i];
    a.timestamp = win_ts(w, b, i);
    d.acc[slot] = a;
    d.hot[slot] = 0;
    acc_insert(d.acc_tab, d.acc_mask, a.id, (uint32_t)slot, a.ledger, a.flags);
  }
  if (i == E - 1) {
    const uint32_t total_bad = rbad + bad, total_ins = rins + (ins ? 1u : 0u);
    for (int32_t bb = (int32_t)w.nb; bb >= 0 && w.off[bb] == E; bb--) o.batch_base[bb] = total_bad;
    if (o.out_count) *o.out_count = total_bad;
    g->result_count = total_bad;
    g->events_total += E;
    sh_window_reset(g, XFER, xbase + total_ins, true);
  }
}
