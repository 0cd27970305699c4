// engine.hip — MI355X batch-apply engine for the StateMachine commit path (libtbgpu.so).
//
// One create_transfers batch (n <= 8190 events, reference state_machine.zig:1220-1306) runs as
// five launches on the engine's stream:
//
//   k_ct_prep   grid    stateless validation (:1465-1489, 1614-1624), account resolution through
//                       the 32 B account-table entries (id, slot, ledger, flags), pre-batch transfer
//                       id / pending_id resolution, static post/void evaluation (:1626-1696), and
//                       entry of every id / pending_id into a batch-local key map.
//   k_ct_link   grid    order-dependence classification: duplicate ids, in-batch pending targets,
//                       several post/voids of one pending transfer, and balance-reading decisions
//                       (limit flags, balancing) are "U"; accounts read by a U event become hot.
//   k_ct_mark   grid    events touching a hot account join the walker set W.
//   k_scan_walk 1 WG    chain structure (segmented scans), chain closure of W, parallel outcome of
//                       all-static chains (first failure + linked_event_failed back-fill), and the
//                       sequential walker: the reference loop (:1236-1301) over W only, with an
//                       undo log for chain rollback (cache_map.zig:254-301); then the ordered
//                       result compaction (:1289-1290) and insert ranks.
//   k_ct_apply  grid    inserts (records appended in timestamp order, id table, pending status,
//                       expires_at list) and the commutative balance deltas of every non-W event
//                       as exact 128-bit atomics.
//
// Everything outside W is order-free by construction, so the bulk of a batch
// runs fully parallel; W carries only the events whose outcome depends on sequencing.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <new>

#include <algorithm>
#include <vector>

#include "../../include/tbg.h"
#include "dev_common.h"
#include "sm_logic.h"

#define SCAN_THREADS 1024
#define SCAN_ITEMS 8
#define SCAN_CAP (SCAN_THREADS * SCAN_ITEMS)  // 8192 >= batch_max

enum : uint32_t { UNDO_BAL = 1, UNDO_XST, UNDO_BST, UNDO_COMMIT, UNDO_INS };
struct __attribute__((aligned(16))) UndoRec {
  uint32_t kind, a, pad0, pad1;
  u128 old[4];
};

struct Dev {
  AccEntry* acc_tab;
  uint64_t acc_mask;
  tb_account_t* acc;
  uint32_t* hot;  // per account slot: epoch of the last batch that marked it hot
  XEntry* x_tab;
  uint64_t x_mask;
  tb_transfer_t* xr;
  uint8_t* xstatus;
  ExpEntry* exp[2];
  uint32_t* exp_cur;  // device word selecting the live expiry buffer
  Globals* g;
};

struct Scratch {
  uint32_t *code, *cls, *dr_slot, *cr_slot, *id_tslot, *p_tslot, *id_ent, *pid_ent, *ins_rank, *wlist;
  uint8_t *ins, *bstatus;
  u128 *amt, *pamt;
  tb_transfer_t* t2;
  BEntry* bmap;
  uint32_t bmask;
  UndoRec* undo;
  tb_create_result_t* results;
  ExpEntry* cand;
};

// ------------------------------------------------------------------------------------------------
// Batch key map
// ------------------------------------------------------------------------------------------------
__device__ inline tb_uint128_t bkey(const uint8_t* ev, uint32_t owner) {
  const uint32_t idx = owner & 0x7FFFFFFFu;
  const tb_uint128_t* p = reinterpret_cast<const tb_uint128_t*>(ev + (size_t)idx * 128 + ((owner >> 31) ? 64 : 0));
  return *p;
}

__device__ inline uint32_t bmap_claim(BEntry* bm, uint32_t mask, const uint8_t* ev, tb_uint128_t key,
                                      uint32_t owner) {
  uint32_t h = (uint32_t)hash_id(key.lo, key.hi) & mask;
  for (;;) {
    const uint32_t old = atomicCAS(&bm[h].owner, NONE32, owner);
    if (old == NONE32) return h;
    const tb_uint128_t k = bkey(ev, old);
    if (k.lo == key.lo && k.hi == key.hi) return h;
    h = (h + 1) & mask;
  }
}

__device__ inline uint32_t bmap_find(const BEntry* bm, uint32_t mask, const uint8_t* ev, tb_uint128_t key) {
  uint32_t h = (uint32_t)hash_id(key.lo, key.hi) & mask;
  for (;;) {
    const uint32_t o = bm[h].owner;
    if (o == NONE32) return NONE32;
    const tb_uint128_t k = bkey(ev, o);
    if (k.lo == key.lo && k.hi == key.hi) return h;
    h = (h + 1) & mask;
  }
}

__device__ inline void bmap_reset(BEntry* bm, uint32_t e) {
  bm[e].owner = NONE32;
  bm[e].id_count = 0;
  bm[e].pid_count = 0;
  bm[e].committed = -1;
}

__global__ void k_bmap_init(BEntry* bm, uint32_t cap) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cap) bmap_reset(bm, i);
}

// ------------------------------------------------------------------------------------------------
// Block-wide scans over SCAN_CAP items in LDS (1024 threads x 8 consecutive items).
// ------------------------------------------------------------------------------------------------
__device__ uint32_t block_excl_sum(uint32_t* vals, uint32_t* tmp) {
  const int t = threadIdx.x;
  uint32_t local[SCAN_ITEMS];
  uint32_t sum = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; k++) {
    local[k] = vals[t * SCAN_ITEMS + k];
    sum += local[k];
  }
  tmp[t] = sum;
  __syncthreads();
  for (int off = 1; off < SCAN_THREADS; off <<= 1) {
    const uint32_t v = t >= off ? tmp[t - off] : 0;
    __syncthreads();
    tmp[t] += v;
    __syncthreads();
  }
  uint32_t prefix = t > 0 ? tmp[t - 1] : 0;
  const uint32_t total = tmp[SCAN_THREADS - 1];
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; k++) {
    vals[t * SCAN_ITEMS + k] = prefix;
    prefix += local[k];
  }
  __syncthreads();
  return total;
}

__device__ void block_incl_max(uint32_t* vals, uint32_t* tmp) {
  const int t = threadIdx.x;
  uint32_t local[SCAN_ITEMS];
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; k++) {
    m = max(m, vals[t * SCAN_ITEMS + k]);
    local[k] = m;
  }
  tmp[t] = m;
  __syncthreads();
  for (int off = 1; off < SCAN_THREADS; off <<= 1) {
    const uint32_t v = t >= off ? tmp[t - off] : 0;
    __syncthreads();
    tmp[t] = max(tmp[t], v);
    __syncthreads();
  }
  const uint32_t prefix = t > 0 ? tmp[t - 1] : 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; k++) vals[t * SCAN_ITEMS + k] = max(prefix, local[k]);
  __syncthreads();
}

// ------------------------------------------------------------------------------------------------
// create_transfers: k_ct_prep
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_ct_prep(Dev d, Scratch s, const tb_transfer_t* __restrict__ ev, uint32_t n,
                                                 uint64_t T) {
  __shared__ u128 red[256];
  __shared__ uint32_t huge_any;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (threadIdx.x == 0) huge_any = 0;
  u128 amount_upper = 0;
  if (i < n) {
    tb_transfer_t t = ev[i];
    const uint8_t* evb = reinterpret_cast<const uint8_t*>(ev);
    uint32_t cls = 0, code;
    uint32_t dr_slot = NONE32, cr_slot = NONE32, id_tslot = NONE32, p_tslot = NONE32, id_ent = NONE32,
             pid_ent = NONE32;
    u128 amt = 0, pamt = 0;
    const uint16_t f = t.flags;
    if (f & TB_TRANSFER_LINKED) cls |= C_LINKED;
    if (t.timestamp != 0) {
      cls |= C_TSNZ | C_STATIC;
      code = TB_CT_TIMESTAMP_MUST_BE_ZERO;
    } else {
      t.timestamp = T - n + i + 1;  // :1253
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
          id_ent = bmap_claim(s.bmap, s.bmask, evb, t.id, i);
          pid_ent = bmap_claim(s.bmap, s.bmask, evb, t.pending_id, i | 0x80000000u);
          atomicAdd(&s.bmap[id_ent].id_count, 1u);
          atomicAdd(&s.bmap[pid_ent].pid_count, 1u);
          // Resolved for every post/void that reaches the pending lookup: the walker needs it even
          // when the pending transfer itself is created in this batch.
          id_tslot = x_find(d.x_tab, d.x_mask, t.id);
          p_tslot = x_find(d.x_tab, d.x_mask, t.pending_id);
          if (p_tslot == NONE32) {
            code = TB_CT_PENDING_TRANSFER_NOT_FOUND;  // unless created in-batch (then U)
          } else {
            cls |= C_PV_PREBATCH;
            const tb_transfer_t p = d.xr[p_tslot];
            code = pv_against(t, p, &amt);
            if (p.flags & TB_TRANSFER_PENDING) {
              AccEntry de, ce;
              dr_slot = acc_find(d.acc_tab, d.acc_mask, p.debit_account_id, &de);
              cr_slot = acc_find(d.acc_tab, d.acc_mask, p.credit_account_id, &ce);
            }
            if (code == CONT && id_tslot != NONE32) code = pv_exists(t, d.xr[id_tslot], p);
            if (code == CONT) code = pv_status(d.xstatus[p_tslot]);
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
          AccEntry de, ce;
          dr_slot = acc_find(d.acc_tab, d.acc_mask, t.debit_account_id, &de);
          if (dr_slot == NONE32) {
            code = TB_CT_DEBIT_ACCOUNT_NOT_FOUND;
          } else {
            cr_slot = acc_find(d.acc_tab, d.acc_mask, t.credit_account_id, &ce);
            if (cr_slot == NONE32)
              code = TB_CT_CREDIT_ACCOUNT_NOT_FOUND;
            else
              code = ct_ledgers(t, de.ledger, ce.ledger);
          }
          if (code != CONT) {
            cls |= C_STATIC;
          } else {
            cls |= C_REACH;
            id_ent = bmap_claim(s.bmap, s.bmask, evb, t.id, i);
            atomicAdd(&s.bmap[id_ent].id_count, 1u);
            const bool bal = f & (TB_TRANSFER_BALANCING_DEBIT | TB_TRANSFER_BALANCING_CREDIT);
            amount_upper = U(t.amount);
            if (bal && amount_upper == 0) amount_upper = (u128)0xFFFFFFFFFFFFFFFFull;
            id_tslot = x_find(d.x_tab, d.x_mask, t.id);
            if (id_tslot != NONE32) {
              code = ct_exists(t, d.xr[id_tslot]);
            } else {
              if (f & TB_TRANSFER_PENDING) cls |= C_PENDING;
              if ((de.flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) || (f & TB_TRANSFER_BALANCING_DEBIT))
                cls |= C_READS_DR;
              if ((ce.flags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS) || (f & TB_TRANSFER_BALANCING_CREDIT))
                cls |= C_READS_CR;
              amt = U(t.amount);
              // Overflow checks cannot fail in an overflow-free batch (checked in k_ct_link).
              if (ovf64(t.timestamp, (uint64_t)t.timeout * TB_NS_PER_S)) {
                code = TB_CT_OVERFLOWS_TIMEOUT;
              } else {
                code = TB_CT_OK;
                cls |= C_INSERT;
              }
            }
          }
        }
      }
    }
    if ((uint64_t)(amount_upper >> 64) != 0) atomicOr(&huge_any, 1u);
    s.code[i] = code;
    s.cls[i] = cls;
    s.dr_slot[i] = dr_slot;
    s.cr_slot[i] = cr_slot;
    s.id_tslot[i] = id_tslot;
    s.p_tslot[i] = p_tslot;
    s.id_ent[i] = id_ent;
    s.pid_ent[i] = pid_ent;
    s.amt[i] = amt;
    s.pamt[i] = pamt;
    s.ins[i] = 0;
  }
  // Batch amount bound: block reduction, one 128-bit atomic per block.
  red[threadIdx.x] = ((uint64_t)(amount_upper >> 64) != 0) ? 0 : amount_upper;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (red[0]) atomic_add_u128(reinterpret_cast<tb_uint128_t*>(&d.g->batch_amount_sum), red[0]);
    if (huge_any) atomicOr(&d.g->batch_huge, 1u);
  }
}

// ------------------------------------------------------------------------------------------------
// create_transfers: k_ct_link / k_ct_mark
// ------------------------------------------------------------------------------------------------
__device__ inline bool batch_ovf_mode(const Globals* g) {
  if (g->batch_huge) return true;
  return ovf128(g->ovf_bound, g->batch_amount_sum);
}

__global__ void __launch_bounds__(256) k_ct_link(Dev d, Scratch s, uint32_t n, uint32_t epoch) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t cls = s.cls[i];
  if (!(cls & C_REACH)) return;
  const bool ovf_mode = batch_ovf_mode(d.g);
  bool u = ovf_mode || (cls & (C_READS_DR | C_READS_CR));
  const BEntry& e = s.bmap[s.id_ent[i]];
  if (e.id_count > 1 || e.pid_count > 0) u = true;  // duplicate id, or a post/void targets this id
  if (cls & C_POSTVOID) {
    const BEntry& pe = s.bmap[s.pid_ent[i]];
    if (pe.id_count > 0 || pe.pid_count > 1) u = true;  // pending created in-batch, or contended
  }
  if (u) {
    s.cls[i] = cls | C_U | C_W;
    if (!ovf_mode) {
      if (cls & C_READS_DR) d.hot[s.dr_slot[i]] = epoch;
      if (cls & C_READS_CR) d.hot[s.cr_slot[i]] = epoch;
    }
  }
}

__global__ void __launch_bounds__(256) k_ct_mark(Dev d, Scratch s, uint32_t n, uint32_t epoch) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t cls = s.cls[i];
  if (!(cls & C_REACH) || (cls & C_W)) return;
  const uint32_t dr = s.dr_slot[i], cr = s.cr_slot[i];
  if ((dr != NONE32 && d.hot[dr] == epoch) || (cr != NONE32 && d.hot[cr] == epoch)) s.cls[i] = cls | C_W;
}

// ------------------------------------------------------------------------------------------------
// The sequential walker (thread 0 of k_scan_walk): state_machine.zig:1236-1301 over W only.
// ------------------------------------------------------------------------------------------------
struct Walker {
  Dev d;
  Scratch s;
  const uint8_t* ev;
  uint32_t n;
  uint64_t T;
  uint32_t undo_n;
  bool scope;

  __device__ void log_bal(uint32_t slot) {
    if (!scope) return;
    UndoRec& r = s.undo[undo_n++];
    r.kind = UNDO_BAL;
    r.a = slot;
    const Bal b = load_bal(&d.acc[slot]);
    r.old[0] = b.dp;
    r.old[1] = b.dpo;
    r.old[2] = b.cp;
    r.old[3] = b.cpo;
  }
  __device__ void log_small(uint32_t kind, uint32_t a, u128 old) {
    if (!scope) return;
    UndoRec& r = s.undo[undo_n++];
    r.kind = kind;
    r.a = a;
    r.old[0] = old;
  }
  __device__ void rollback() {
    while (undo_n) {
      const UndoRec& r = s.undo[--undo_n];
      switch (r.kind) {
        case UNDO_BAL: {
          Bal b;
          b.dp = r.old[0];
          b.dpo = r.old[1];
          b.cp = r.old[2];
          b.cpo = r.old[3];
          store_bal(&d.acc[r.a], b);
        } break;
        case UNDO_XST: d.xstatus[r.a] = (uint8_t)r.old[0]; break;
        case UNDO_BST: s.bstatus[r.a] = (uint8_t)r.old[0]; break;
        case UNDO_COMMIT: s.bmap[r.a].committed = (int32_t)(uint32_t)r.old[0]; break;
        case UNDO_INS: s.ins[r.a] = 0; break;
      }
    }
  }

  __device__ uint32_t commit_record(uint32_t i, const tb_transfer_t& t2) {
    s.t2[i] = t2;
    log_small(UNDO_INS, i, 0);
    s.ins[i] = 1;
    const uint32_t e = s.id_ent[i];
    log_small(UNDO_COMMIT, e, (uint32_t)s.bmap[e].committed);
    s.bmap[e].committed = (int32_t)i;
    return 0;
  }

  // create_transfer (:1462-1585) from the exists check on; validation results come from k_ct_prep.
  __device__ uint32_t transfer(uint32_t i) {
    const uint32_t cls = s.cls[i];
    if (cls & C_STATIC) return s.code[i];
    tb_transfer_t t = reinterpret_cast<const tb_transfer_t*>(ev)[i];
    t.timestamp = T - n + i + 1;
    if (cls & C_POSTVOID) return post_or_void(i, t);
    if (s.id_tslot[i] != NONE32) return ct_exists(t, d.xr[s.id_tslot[i]]);
    const int32_t c = s.bmap[s.id_ent[i]].committed;
    if (c >= 0) return ct_exists(t, s.t2[c]);
    const uint32_t drs = s.dr_slot[i], crs = s.cr_slot[i];
    tb_account_t* dra = &d.acc[drs];
    tb_account_t* cra = &d.acc[crs];
    Bal dr = load_bal(dra), cr = load_bal(cra);
    u128 amount;
    const uint32_t r = ct_balances(t, dr, dra->flags, cr, cra->flags, &amount);
    if (r != TB_CT_OK) return r;
    t.amount = W(amount);
    commit_record(i, t);
    log_bal(drs);
    log_bal(crs);
    if (t.flags & TB_TRANSFER_PENDING) {
      dr.dp += amount;
      cr.cp += amount;
      s.bstatus[i] = TB_PENDING_PENDING;
    } else {
      dr.dpo += amount;
      cr.cpo += amount;
    }
    store_bal(dra, dr);
    store_bal(cra, cr);
    return TB_CT_OK;
  }

  // post_or_void_pending_transfer (:1608-1741) from the pending lookup on.
  __device__ uint32_t post_or_void(uint32_t i, const tb_transfer_t& t) {
    const uint32_t pslot = s.p_tslot[i];
    int32_t pc = -1;
    uint32_t drs, crs;
    tb_transfer_t p;
    if (pslot != NONE32) {
      p = d.xr[pslot];
      drs = s.dr_slot[i];
      crs = s.cr_slot[i];
    } else {
      pc = s.bmap[s.pid_ent[i]].committed;
      if (pc < 0) return TB_CT_PENDING_TRANSFER_NOT_FOUND;
      p = s.t2[pc];
      drs = s.dr_slot[pc];
      crs = s.cr_slot[pc];
    }
    u128 amount;
    uint32_t r = pv_against(t, p, &amount);
    if (r != CONT) return r;
    if (s.id_tslot[i] != NONE32) return pv_exists(t, d.xr[s.id_tslot[i]], p);
    const int32_t c = s.bmap[s.id_ent[i]].committed;
    if (c >= 0) return pv_exists(t, s.t2[c], p);
    r = pv_status(pc >= 0 ? s.bstatus[pc] : d.xstatus[pslot]);
    if (r != CONT) return r;
    commit_record(i, pv_record(t, p, amount));
    if (p.timeout > 0 && expires_at_of(p) <= t.timestamp) return TB_CT_PENDING_TRANSFER_EXPIRED;
    const uint8_t st = (t.flags & TB_TRANSFER_POST_PENDING) ? TB_PENDING_POSTED : TB_PENDING_VOIDED;
    if (pc >= 0) {
      log_small(UNDO_BST, (uint32_t)pc, s.bstatus[pc]);
      s.bstatus[pc] = st;
    } else {
      log_small(UNDO_XST, pslot, d.xstatus[pslot]);
      d.xstatus[pslot] = st;
    }
    tb_account_t* dra = &d.acc[drs];
    tb_account_t* cra = &d.acc[crs];
    Bal dr = load_bal(dra), cr = load_bal(cra);
    log_bal(drs);
    log_bal(crs);
    const u128 pa = U(p.amount);
    dr.dp -= pa;
    cr.cp -= pa;
    if (t.flags & TB_TRANSFER_POST_PENDING) {
      dr.dpo += amount;
      cr.cpo += amount;
    }
    store_bal(dra, dr);
    store_bal(cra, cr);
    return TB_CT_OK;
  }

  // create_account (:1421-1448) from the exists check on.
  __device__ uint32_t account(uint32_t i) {
    const uint32_t cls = s.cls[i];
    if (cls & C_STATIC) return s.code[i];
    if (s.id_tslot[i] != NONE32) return s.code[i];  // pre-batch exists: static
    const tb_account_t* evs = reinterpret_cast<const tb_account_t*>(ev);
    const uint32_t e = s.id_ent[i];
    const int32_t c = s.bmap[e].committed;
    if (c >= 0) return ca_exists(evs[i], evs[c]);
    log_small(UNDO_INS, i, 0);
    s.ins[i] = 1;
    log_small(UNDO_COMMIT, e, (uint32_t)c);
    s.bmap[e].committed = (int32_t)i;
    return TB_CA_OK;
  }

  template <bool XFER>
  __device__ void run(uint32_t w_count) {
    int32_t chain = -1;
    bool broken = false;
    undo_n = 0;
    scope = false;
    for (uint32_t k = 0; k < w_count; k++) {
      const uint32_t i = s.wlist[k];
      const uint32_t cls = s.cls[i];
      const bool linked = cls & C_LINKED;
      uint32_t r;
      if (linked && chain < 0) {
        chain = (int32_t)i;
        undo_n = 0;
        scope = true;
      }
      if (linked && i == n - 1) {
        r = TB_CT_LINKED_EVENT_CHAIN_OPEN;
      } else if (broken) {
        r = TB_CT_LINKED_EVENT_FAILED;
      } else if (cls & C_TSNZ) {
        r = TB_CT_TIMESTAMP_MUST_BE_ZERO;
      } else {
        r = XFER ? transfer(i) : account(i);
      }
      if (r != TB_CT_OK) {
        if (chain >= 0 && !broken) {
          broken = true;
          rollback();
          for (uint32_t j = (uint32_t)chain; j < i; j++) s.code[j] = TB_CT_LINKED_EVENT_FAILED;
        }
      }
      s.code[i] = r;
      if (chain >= 0 && (!linked || r == TB_CT_LINKED_EVENT_CHAIN_OPEN)) {
        chain = -1;
        broken = false;
        scope = false;
        undo_n = 0;
      }
    }
  }
};

// ------------------------------------------------------------------------------------------------
// k_scan_walk: chain structure, closure, static chain outcomes, walker, result compaction.
// ------------------------------------------------------------------------------------------------
template <bool XFER>
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_walk(Dev d, Scratch s, const uint8_t* ev, uint32_t n, uint64_t T,
                                                           tb_create_result_t* out_results, uint32_t* out_count) {
  __shared__ uint16_t cs[SCAN_CAP];  // chain start of each event
  __shared__ uint32_t A[SCAN_CAP];
  __shared__ uint32_t B[SCAN_CAP];
  __shared__ uint32_t C[SCAN_CAP];
  __shared__ uint32_t tmp[SCAN_THREADS];
  const int t = threadIdx.x;

  // Phase A: chain_start[i] = last j <= i with (j == 0 || !linked[j-1]).
  for (int k = 0; k < SCAN_ITEMS; k++) {
    const uint32_t i = t * SCAN_ITEMS + k;
    uint32_t v = 0;
    if (i < n) v = (i == 0 || !(s.cls[i - 1] & C_LINKED)) ? i : 0;
    A[i] = v;
    B[i] = 0;
    C[i] = NONE32;
  }
  __syncthreads();
  block_incl_max(A, tmp);
  for (int k = 0; k < SCAN_ITEMS; k++) {
    const uint32_t i = t * SCAN_ITEMS + k;
    cs[i] = (uint16_t)A[i];
  }
  __syncthreads();

  // Phase B: chain closure of W.
  for (int k = 0; k < SCAN_ITEMS; k++) {
    const uint32_t i = t * SCAN_ITEMS + k;
    if (i < n && (s.cls[i] & C_W)) atomicOr(&B[cs[i]], 1u);
  }
  __syncthreads();
  // Phase C: first failure of each all-static chain.
  for (int k = 0; k < SCAN_ITEMS; k++) {
    const uint32_t i = t * SCAN_ITEMS + k;
    if (i >= n) continue;
    uint32_t cls = s.cls[i];
    const bool in_chain = (cls & C_LINKED) || (i > 0 && (s.cls[i - 1] & C_LINKED));
    if (in_chain && B[cs[i]] && !(cls & C_W)) {
      cls |= C_W;
      s.cls[i] = cls;
    }
    if (!(cls & C_W) && in_chain) {
      const uint32_t code = ((cls & C_LINKED) && i == n - 1) ? (uint32_t)TB_CT_LINKED_EVENT_CHAIN_OPEN : s.code[i];
      if (code != TB_CT_OK) atomicMin(&C[cs[i]], i);
    }
  }
  __syncthreads();
  for (int k = 0; k < SCAN_ITEMS; k++) {
    const uint32_t i = t * SCAN_ITEMS + k;
    uint32_t w = 0;
    if (i < n) {
      uint32_t cls = s.cls[i];
      if (cls & C_W) {
        w = 1;
      } else {
        const bool in_chain = (cls & C_LINKED) || (i > 0 && (s.cls[i - 1] & C_LINKED));
        uint32_t code = s.code[i];
        bool commit, inserted;
        if (in_chain) {
          const uint32_t f = C[cs[i]];
          if ((cls & C_LINKED) && i == n - 1)
            code = TB_CT_LINKED_EVENT_CHAIN_OPEN;
          else if (f != NONE32 && f != i)
            code = TB_CT_LINKED_EVENT_FAILED;
          commit = (f == NONE32);
          inserted = commit && (cls & C_INSERT);
        } else {
          commit = (code == TB_CT_OK);
          inserted = (cls & C_INSERT) != 0;
        }
        s.code[i] = code;
        s.cls[i] = cls | (commit ? C_COMMIT : 0) | (inserted ? C_INSERTED : 0);
      }
    }
    A[i] = w;
  }
  __syncthreads();

  // Phase D: ordered W list.
  const uint32_t w_count = block_excl_sum(A, tmp);
  for (int k = 0; k < SCAN_ITEMS; k++) {
    const uint32_t i = t * SCAN_ITEMS + k;
    if (i < n && (s.cls[i] & C_W)) s.wlist[A[i]] = i;
  }
  __syncthreads();

  // Phase E: the walker.
  if (t == 0 && w_count) {
    Walker wk;
    wk.d = d;
    wk.s = s;
    wk.ev = ev;
    wk.n = n;
    wk.T = T;
    wk.template run<XFER>(w_count);
  }
  __syncthreads();

  // Phase F: ordered results and insert ranks.
  for (int k = 0; k < SCAN_ITEMS; k++) {
    const uint32_t i = t * SCAN_ITEMS + k;
    uint32_t bad = 0, ins = 0;
    if (i < n) {
      const uint32_t cls = s.cls[i];
      bad = s.code[i] != TB_CT_OK;
      ins = (cls & C_W) ? s.ins[i] : ((cls & C_INSERTED) ? 1u : 0u);
    }
    A[i] = bad;
    B[i] = ins;
  }
  __syncthreads();
  const uint32_t result_count = block_excl_sum(A, tmp);
  const uint32_t insert_count = block_excl_sum(B, tmp);
  for (int k = 0; k < SCAN_ITEMS; k++) {
    const uint32_t i = t * SCAN_ITEMS + k;
    if (i >= n) continue;
    const uint32_t code = s.code[i];
    if (code != TB_CT_OK) {
      tb_create_result_t r;
      r.index = i;
      r.result = code;
      out_results[A[i]] = r;
    }
    s.ins_rank[i] = B[i];
  }
  if (t == 0) {
    d.g->result_count = result_count;
    d.g->insert_count = insert_count;
    d.g->w_count = w_count;
    d.g->base = XFER ? d.g->x_count : d.g->acc_count;
    d.g->w_events_total += w_count;
    d.g->events_total += n;
    if (out_count) *out_count = result_count;
  }
}

// ------------------------------------------------------------------------------------------------
// create_transfers: k_ct_apply
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_ct_apply(Dev d, Scratch s, const tb_transfer_t* __restrict__ ev, uint32_t n,
                                                  uint64_t T) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const Globals* g = d.g;
  if (i < n) {
    const uint32_t cls = s.cls[i];
    const bool w = cls & C_W;
    const bool ins = w ? (s.ins[i] != 0) : ((cls & C_INSERTED) != 0);
    if (ins) {
      const uint64_t slot = g->base + s.ins_rank[i];
      tb_transfer_t t2;
      if (w) {
        t2 = s.t2[i];
      } else {
        t2 = ev[i];
        t2.timestamp = T - n + i + 1;
        if (cls & C_POSTVOID) t2 = pv_record(t2, d.xr[s.p_tslot[i]], s.amt[i]);
      }
      d.xr[slot] = t2;
      x_insert(d.x_tab, d.x_mask, t2.id, (uint32_t)slot);
      uint8_t st = 0;
      if (t2.flags & TB_TRANSFER_PENDING) {
        st = w ? s.bstatus[i] : (uint8_t)TB_PENDING_PENDING;
        if (t2.timeout > 0) {
          const uint64_t expires_at = expires_at_of(t2);
          atomicMin(reinterpret_cast<unsigned long long*>(&d.g->pulse_next), (unsigned long long)expires_at);
          const bool visible = !(t2.timestamp >> 63) && expires_at <= TB_TIMESTAMP_MAX;
          if (st == TB_PENDING_PENDING && visible) {
            const uint64_t k = atomicAdd(reinterpret_cast<unsigned long long*>(&d.g->exp_count), 1ull);
            ExpEntry e;
            e.expires_at = expires_at;
            e.slot = (uint32_t)slot;
            e.pad = 0;
            d.exp[*d.exp_cur][k] = e;
          }
        }
      }
      d.xstatus[slot] = st;
    }
    if (!w && (cls & C_COMMIT)) {
      tb_account_t* dra = &d.acc[s.dr_slot[i]];
      tb_account_t* cra = &d.acc[s.cr_slot[i]];
      const u128 a = s.amt[i];
      if (cls & C_POSTVOID) {
        const u128 pa = s.pamt[i];
        atomic_sub_u128(&dra->debits_pending, pa);
        atomic_sub_u128(&cra->credits_pending, pa);
        if (cls & C_POST) {
          atomic_add_u128(&dra->debits_posted, a);
          atomic_add_u128(&cra->credits_posted, a);
        }
        d.xstatus[s.p_tslot[i]] = (cls & C_POST) ? TB_PENDING_POSTED : TB_PENDING_VOIDED;
      } else if (cls & C_PENDING) {
        atomic_add_u128(&dra->debits_pending, a);
        atomic_add_u128(&cra->credits_pending, a);
      } else {
        atomic_add_u128(&dra->debits_posted, a);
        atomic_add_u128(&cra->credits_posted, a);
      }
    }
    if (s.id_ent[i] != NONE32) bmap_reset(s.bmap, s.id_ent[i]);
    if (s.pid_ent[i] != NONE32) bmap_reset(s.bmap, s.pid_ent[i]);
  }
  if (i == 0) {
    Globals* gw = d.g;
    gw->x_count = gw->base + gw->insert_count;
    const u128 b = gw->ovf_bound + gw->batch_amount_sum;
    gw->ovf_bound = (gw->batch_huge || b < gw->ovf_bound) ? MAX128 : b;
    gw->batch_amount_sum = 0;
    gw->batch_huge = 0;
  }
}

// ------------------------------------------------------------------------------------------------
// create_accounts
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_ca_prep(Dev d, Scratch s, const tb_account_t* __restrict__ ev, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const tb_account_t a = ev[i];
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
      id_ent = bmap_claim(s.bmap, s.bmask, reinterpret_cast<const uint8_t*>(ev), a.id, i);
      atomicAdd(&s.bmap[id_ent].id_count, 1u);
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
  s.id_ent[i] = id_ent;
  s.pid_ent[i] = NONE32;
  s.id_tslot[i] = slot;
  s.ins[i] = 0;
}

__global__ void __launch_bounds__(256) k_ca_link(Scratch s, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t cls = s.cls[i];
  if ((cls & C_REACH) && s.bmap[s.id_ent[i]].id_count > 1) s.cls[i] = cls | C_U | C_W;
}

__global__ void __launch_bounds__(256) k_ca_apply(Dev d, Scratch s, const tb_account_t* __restrict__ ev, uint32_t n,
                                                  uint64_t T) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const Globals* g = d.g;
  if (i < n) {
    const uint32_t cls = s.cls[i];
    const bool ins = (cls & C_W) ? (s.ins[i] != 0) : ((cls & C_INSERTED) != 0);
    if (ins) {
      const uint64_t slot = g->base + s.ins_rank[i];
      tb_account_t a = ev[i];
      a.timestamp = T - n + i + 1;
      d.acc[slot] = a;
      d.hot[slot] = 0;
      acc_insert(d.acc_tab, d.acc_mask, a.id, (uint32_t)slot, a.ledger, a.flags);
    }
    if (s.id_ent[i] != NONE32) bmap_reset(s.bmap, s.id_ent[i]);
  }
  if (i == 0) d.g->acc_count = d.g->base + d.g->insert_count;
}

// ------------------------------------------------------------------------------------------------
// Pulse: ExpirePendingTransfers scan + execute_expire_pending_transfers (state_machine.zig:
// 1010-1105, 1874-1929, 2112-2166). The live list holds scan-visible pending-with-timeout entries;
// an entry is live while its transfer's status is `pending`.
// ------------------------------------------------------------------------------------------------
struct PulseCtl {
  uint32_t active;
  uint32_t select_all;
  uint64_t thr_expires_at;  // selection threshold key (expires_at, slot), inclusive
  uint32_t thr_slot;
  uint32_t pad;
};

__global__ void k_pulse_gate(Dev d, PulseCtl* ctl, uint64_t prepare_timestamp) {
  // pulse() (:589-596)
  ctl->active = d.g->pulse_next <= prepare_timestamp ? 1u : 0u;
  d.g->cand_count = 0;
  d.g->alt_count = 0;
  d.g->next_min = ~0ull;
}

__global__ void __launch_bounds__(256) k_pulse_scan(Dev d, Scratch s, const PulseCtl* ctl, uint64_t T) {
  if (!ctl->active) return;
  const uint32_t cur = *d.exp_cur;
  const ExpEntry* list = d.exp[cur];
  ExpEntry* alt = d.exp[cur ^ 1];
  const uint64_t count = d.g->exp_count;
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < count; j += (uint64_t)gridDim.x * blockDim.x) {
    const ExpEntry e = list[j];
    if (d.xstatus[e.slot] != TB_PENDING_PENDING) continue;  // removed from the index
    if (e.expires_at <= T) {
      const uint32_t k = atomicAdd(&d.g->cand_count, 1u);
      s.cand[k] = e;
    } else {
      const uint32_t k = atomicAdd(&d.g->alt_count, 1u);
      alt[k] = e;
      atomicMin(reinterpret_cast<unsigned long long*>(&d.g->next_min), (unsigned long long)e.expires_at);
    }
  }
}

// Selection of the `cap` smallest (expires_at, slot) keys: 12-pass LDS radix select (8-bit digits
// over the 96-bit key), single workgroup. Only runs when more than `cap` transfers are due.
__global__ void __launch_bounds__(1024) k_pulse_select(Dev d, Scratch s, PulseCtl* ctl, uint32_t cap) {
  __shared__ uint32_t hist[256];
  __shared__ uint64_t prefix_hi;
  __shared__ uint32_t prefix_lo;
  __shared__ uint32_t want;
  if (!ctl->active) return;
  const uint32_t m = d.g->cand_count;
  if (m <= cap) {
    if (threadIdx.x == 0) {
      ctl->select_all = 1;
      // scan_finished: next = first live entry beyond T, else timestamp_max (:2126-2135)
      d.g->pulse_next = d.g->alt_count > 0 ? d.g->next_min : TB_TIMESTAMP_MAX;
      d.g->expired_count = m;
    }
    return;
  }
  if (threadIdx.x == 0) {
    prefix_hi = 0;
    prefix_lo = 0;
    want = cap;  // 1-based rank of the last selected key
  }
  __syncthreads();
  for (int pass = 0; pass < 12; pass++) {
    const int shift = 88 - 8 * pass;  // bit position of this digit in the 96-bit key
    for (int b = threadIdx.x; b < 256; b += blockDim.x) hist[b] = 0;
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < m; j += blockDim.x) {
      const ExpEntry e = s.cand[j];
      // key = expires_at:64 | slot:32 ; match the digits fixed so far
      bool match = true;
      if (pass > 0) {
        const int fixed_bits = 8 * pass;
        // compare the top `fixed_bits` of the key with the prefix
        if (fixed_bits <= 64) {
          const uint64_t mask = fixed_bits == 64 ? ~0ull : ~((~0ull) >> fixed_bits);
          match = (e.expires_at & mask) == (prefix_hi & mask);
        } else {
          const uint32_t lo_bits = fixed_bits - 64;
          const uint32_t mask = ~((~0u) >> lo_bits);
          match = e.expires_at == prefix_hi && (e.slot & mask) == (prefix_lo & mask);
        }
      }
      if (!match) continue;
      uint32_t digit;
      if (shift >= 32)
        digit = (uint32_t)(e.expires_at >> (shift - 32)) & 0xFF;
      else
        digit = (e.slot >> shift) & 0xFF;
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
  if (threadIdx.x == 0) {
    ctl->select_all = 0;
    ctl->thr_expires_at = prefix_hi;
    ctl->thr_slot = prefix_lo;
    d.g->pulse_next = prefix_hi;  // buffer_finished: last included expires_at (:2136-2140)
    d.g->expired_count = cap;
  }
}

__global__ void __launch_bounds__(256) k_pulse_apply(Dev d, Scratch s, const PulseCtl* ctl) {
  if (!ctl->active) return;
  const uint32_t m = d.g->cand_count;
  const uint32_t cur = *d.exp_cur;
  ExpEntry* alt = d.exp[cur ^ 1];
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m; j += gridDim.x * blockDim.x) {
    const ExpEntry e = s.cand[j];
    const bool take = ctl->select_all || e.expires_at < ctl->thr_expires_at ||
                      (e.expires_at == ctl->thr_expires_at && e.slot <= ctl->thr_slot);
    if (!take) {
      const uint32_t k = atomicAdd(&d.g->alt_count, 1u);
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
  }
}

__global__ void k_pulse_finish(Dev d, PulseCtl* ctl) {
  if (!ctl->active) return;
  *d.exp_cur ^= 1u;
  d.g->exp_count = d.g->alt_count;
  ctl->active = 0;
}

// ------------------------------------------------------------------------------------------------
// lookup_accounts / lookup_transfers (state_machine.zig:1309-1344): found records, input order.
// ------------------------------------------------------------------------------------------------
template <bool ACC>
__global__ void __launch_bounds__(SCAN_THREADS) k_lookup(Dev d, const tb_uint128_t* ids, uint32_t n, uint8_t* out,
                                                         uint32_t* out_count) {
  __shared__ uint32_t A[SCAN_CAP];
  __shared__ uint32_t slot_of[SCAN_CAP];
  __shared__ uint32_t tmp[SCAN_THREADS];
  for (uint32_t i = threadIdx.x; i < SCAN_CAP; i += SCAN_THREADS) {
    uint32_t slot = NONE32;
    if (i < n) {
      const tb_uint128_t id = ids[i];
      if (ACC) {
        AccEntry e;
        slot = acc_find(d.acc_tab, d.acc_mask, id, &e);
      } else {
        slot = x_find(d.x_tab, d.x_mask, id);
      }
    }
    slot_of[i] = slot;
    A[i] = slot != NONE32;
  }
  __syncthreads();
  const uint32_t total = block_excl_sum(A, tmp);
  for (uint32_t i = threadIdx.x; i < n; i += SCAN_THREADS) {
    const uint32_t slot = slot_of[i];
    if (slot == NONE32) continue;
    const uint4* src = ACC ? reinterpret_cast<const uint4*>(&d.acc[slot]) : reinterpret_cast<const uint4*>(&d.xr[slot]);
    uint4* dst = reinterpret_cast<uint4*>(out + (size_t)A[i] * 128);
#pragma unroll
    for (int q = 0; q < 8; q++) dst[q] = src[q];
  }
  if (threadIdx.x == 0) *out_count = total;
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

// ================================================================================================
// Host side
// ================================================================================================
struct tbg_engine {
  int device;
  hipStream_t stream;
  uint32_t batch_max;
  uint64_t acc_max, x_max, acc_cap, x_cap;
  Dev d;
  Scratch s;
  PulseCtl* ctl;
  Globals* g;
  void* d_in;      // staged request (batch_max x 128 B)
  uint8_t* d_out;  // lookup replies
  uint32_t* d_count;
  int* d_found;
  void* h_pinned;  // pinned staging for H2D/D2H
  uint64_t acc_upper, x_upper;  // host-side upper bounds of the store counts
  uint32_t epoch;
  // optional per-phase timing (HIP events on the engine stream)
  int timing;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used;
  std::vector<uint32_t> ev_phase;  // phase of each (start, end) pair
  // prefetch bookkeeping
  int pf_valid;
  uint32_t pf_operation;
  const void* pf_input;
  uint64_t pf_len, pf_ts;
};

#define HIPCHK(x)                                                                         \
  do {                                                                                    \
    hipError_t err__ = (x);                                                               \
    if (err__ != hipSuccess) {                                                            \
      fprintf(stderr, "tbg: HIP error %s at %s:%d\n", hipGetErrorString(err__), __FILE__, __LINE__); \
      return TBG_E_DEVICE;                                                                \
    }                                                                                     \
  } while (0)

static uint64_t next_pow2(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

static inline uint32_t grid_for(uint32_t n, uint32_t block = 256) { return (n + block - 1) / block; }

extern "C" const char* tbg_version(void) { return "tbgpu 0.1 gfx950 (create_accounts, create_transfers, pulse, lookups)"; }

extern "C" int tbg_create(const tbg_config* cfg, tbg_engine** out) {
  if (!cfg || !out) return TBG_E_STATE;
  tbg_engine* e = (tbg_engine*)calloc(1, sizeof(tbg_engine));
  new (&e->ev_pool) std::vector<hipEvent_t>();
  new (&e->ev_phase) std::vector<uint32_t>();
  e->device = cfg->device;
  e->batch_max = cfg->batch_max ? cfg->batch_max : TB_BATCH_MAX;
  if (e->batch_max > SCAN_CAP) {
    free(e);
    return TBG_E_STATE;
  }
  e->acc_max = cfg->accounts_max ? cfg->accounts_max : 1024;
  e->x_max = cfg->transfers_max ? cfg->transfers_max : 1024;
  e->acc_cap = next_pow2(2 * e->acc_max);
  e->x_cap = next_pow2(2 * e->x_max);
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));

  Dev& d = e->d;
  d.acc_mask = e->acc_cap - 1;
  d.x_mask = e->x_cap - 1;
  HIPCHK(hipMalloc(&d.acc_tab, e->acc_cap * sizeof(AccEntry)));
  HIPCHK(hipMalloc(&d.acc, e->acc_max * sizeof(tb_account_t)));
  HIPCHK(hipMalloc(&d.hot, e->acc_max * sizeof(uint32_t)));
  HIPCHK(hipMalloc(&d.x_tab, e->x_cap * sizeof(XEntry)));
  HIPCHK(hipMalloc(&d.xr, e->x_max * sizeof(tb_transfer_t)));
  HIPCHK(hipMalloc(&d.xstatus, e->x_max));
  HIPCHK(hipMalloc(&d.exp[0], e->x_max * sizeof(ExpEntry)));
  HIPCHK(hipMalloc(&d.exp[1], e->x_max * sizeof(ExpEntry)));
  HIPCHK(hipMalloc(&d.exp_cur, sizeof(uint32_t)));
  HIPCHK(hipMalloc(&d.g, sizeof(Globals)));
  HIPCHK(hipMemsetAsync(d.acc_tab, 0xFF, e->acc_cap * sizeof(AccEntry), e->stream));
  HIPCHK(hipMemsetAsync(d.x_tab, 0xFF, e->x_cap * sizeof(XEntry), e->stream));
  HIPCHK(hipMemsetAsync(d.hot, 0, e->acc_max * sizeof(uint32_t), e->stream));
  HIPCHK(hipMemsetAsync(d.exp_cur, 0, sizeof(uint32_t), e->stream));
  Globals g0;
  memset(&g0, 0, sizeof g0);
  g0.pulse_next = TB_TIMESTAMP_MIN;  // ExpirePendingTransfers default (:2063)
  g0.next_min = ~0ull;
  HIPCHK(hipMemcpy(d.g, &g0, sizeof g0, hipMemcpyHostToDevice));
  e->g = d.g;

  Scratch& s = e->s;
  const uint32_t N = SCAN_CAP;
  HIPCHK(hipMalloc(&s.code, N * 4));
  HIPCHK(hipMalloc(&s.cls, N * 4));
  HIPCHK(hipMalloc(&s.dr_slot, N * 4));
  HIPCHK(hipMalloc(&s.cr_slot, N * 4));
  HIPCHK(hipMalloc(&s.id_tslot, N * 4));
  HIPCHK(hipMalloc(&s.p_tslot, N * 4));
  HIPCHK(hipMalloc(&s.id_ent, N * 4));
  HIPCHK(hipMalloc(&s.pid_ent, N * 4));
  HIPCHK(hipMalloc(&s.ins_rank, N * 4));
  HIPCHK(hipMalloc(&s.wlist, N * 4));
  HIPCHK(hipMalloc(&s.ins, N));
  HIPCHK(hipMalloc(&s.bstatus, N));
  HIPCHK(hipMalloc(&s.amt, N * sizeof(u128)));
  HIPCHK(hipMalloc(&s.pamt, N * sizeof(u128)));
  HIPCHK(hipMalloc(&s.t2, N * sizeof(tb_transfer_t)));
  const uint32_t bcap = 4 * N;  // 2 keys per event at load <= 1/2
  s.bmask = bcap - 1;
  HIPCHK(hipMalloc(&s.bmap, bcap * sizeof(BEntry)));
  HIPCHK(hipMalloc(&s.undo, 5 * N * sizeof(UndoRec)));
  HIPCHK(hipMalloc(&s.results, N * sizeof(tb_create_result_t)));
  HIPCHK(hipMalloc(&s.cand, e->x_max * sizeof(ExpEntry)));
  k_bmap_init<<<grid_for(bcap), 256, 0, e->stream>>>(s.bmap, bcap);
  HIPCHK(hipGetLastError());

  HIPCHK(hipMalloc(&e->ctl, sizeof(PulseCtl)));
  HIPCHK(hipMemsetAsync(e->ctl, 0, sizeof(PulseCtl), e->stream));
  HIPCHK(hipMalloc(&e->d_in, (size_t)N * 128));
  HIPCHK(hipMalloc(&e->d_out, (size_t)N * 128));
  HIPCHK(hipMalloc(&e->d_count, sizeof(uint32_t)));
  HIPCHK(hipMalloc(&e->d_found, sizeof(int)));
  HIPCHK(hipHostMalloc(&e->h_pinned, (size_t)N * 128 + 4096));
  HIPCHK(hipStreamSynchronize(e->stream));
  *out = e;
  return TBG_OK;
}

extern "C" int tbg_destroy(tbg_engine* e) {
  if (!e) return TBG_OK;
  (void)hipSetDevice(e->device);
  (void)hipStreamSynchronize(e->stream);
  Dev& d = e->d;
  Scratch& s = e->s;
  void* ptrs[] = {d.acc_tab, d.acc, d.hot, d.x_tab, d.xr, d.xstatus, d.exp[0], d.exp[1], d.exp_cur, d.g,
                  s.code, s.cls, s.dr_slot, s.cr_slot, s.id_tslot, s.p_tslot, s.id_ent, s.pid_ent, s.ins_rank,
                  s.wlist, s.ins, s.bstatus, s.amt, s.pamt, s.t2, s.bmap, s.undo, s.results, s.cand, e->ctl,
                  e->d_in, e->d_out, e->d_count, e->d_found};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (e->h_pinned) (void)hipHostFree(e->h_pinned);
  for (hipEvent_t ev : e->ev_pool) (void)hipEventDestroy(ev);
  e->ev_pool.~vector();
  e->ev_phase.~vector();
  (void)hipStreamDestroy(e->stream);
  free(e);
  return TBG_OK;
}

extern "C" int tbg_input_valid(const tbg_engine* e, uint32_t operation, uint64_t len) {
  const uint64_t bm = e ? e->batch_max : TB_BATCH_MAX;
  switch (operation) {
    case TB_OP_PULSE: return len == 0;
    case TB_OP_CREATE_ACCOUNTS:
    case TB_OP_CREATE_TRANSFERS: return len % 128 == 0 && len <= bm * 128;
    case TB_OP_LOOKUP_ACCOUNTS:
    case TB_OP_LOOKUP_TRANSFERS: return len % 16 == 0 && len <= bm * 16;
    case TB_OP_GET_ACCOUNT_TRANSFERS:
    case TB_OP_GET_ACCOUNT_BALANCES: return len == 64;
    default: return 0;
  }
}

extern "C" void* tbg_stream(tbg_engine* e) { return (void*)e->stream; }

extern "C" int tbg_sync(tbg_engine* e) {
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamSynchronize(e->stream));
  return TBG_OK;
}

static int read_globals(tbg_engine* e, Globals* out) {
  HIPCHK(hipMemcpyAsync(e->h_pinned, e->g, sizeof(Globals), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  memcpy(out, e->h_pinned, sizeof(Globals));
  return TBG_OK;
}

extern "C" int tbg_pulse_needed(tbg_engine* e, uint64_t prepare_timestamp, int* needed) {
  Globals g;
  int rc = read_globals(e, &g);
  if (rc) return rc;
  *needed = g.pulse_next <= prepare_timestamp;
  return TBG_OK;
}

enum { PH_PREP, PH_LINK, PH_MARK, PH_SCAN, PH_APPLY, PH_PULSE, PH_COUNT };

static hipEvent_t timing_event(tbg_engine* e) {
  if (e->ev_used == e->ev_pool.size()) {
    hipEvent_t ev;
    if (hipEventCreate(&ev) != hipSuccess) return nullptr;
    e->ev_pool.push_back(ev);
  }
  return e->ev_pool[e->ev_used++];
}
static void phase_begin(tbg_engine* e, uint32_t phase) {
  if (!e->timing) return;
  e->ev_phase.push_back(phase);
  (void)hipEventRecord(timing_event(e), e->stream);
}
static void phase_end(tbg_engine* e) {
  if (!e->timing) return;
  (void)hipEventRecord(timing_event(e), e->stream);
}

static int launch_pulse(tbg_engine* e, uint64_t T, uint64_t prepare_timestamp) {
  hipStream_t st = e->stream;
  phase_begin(e, PH_PULSE);
  k_pulse_gate<<<1, 1, 0, st>>>(e->d, e->ctl, prepare_timestamp);
  k_pulse_scan<<<1024, 256, 0, st>>>(e->d, e->s, e->ctl, T);
  k_pulse_select<<<1, 1024, 0, st>>>(e->d, e->s, e->ctl, e->batch_max);
  k_pulse_apply<<<512, 256, 0, st>>>(e->d, e->s, e->ctl);
  k_pulse_finish<<<1, 1, 0, st>>>(e->d, e->ctl);
  phase_end(e);
  HIPCHK(hipGetLastError());
  return TBG_OK;
}

static int check_capacity(tbg_engine* e, uint32_t operation, uint32_t n) {
  uint64_t* upper = operation == TB_OP_CREATE_ACCOUNTS ? &e->acc_upper : &e->x_upper;
  const uint64_t cap = operation == TB_OP_CREATE_ACCOUNTS ? e->acc_max : e->x_max;
  if (*upper + n <= cap) return TBG_OK;
  Globals g;
  int rc = read_globals(e, &g);
  if (rc) return rc;
  e->acc_upper = g.acc_count;
  e->x_upper = g.x_count;
  if (*upper + n > cap) return TBG_E_CAPACITY;
  return TBG_OK;
}

static int launch_prep(tbg_engine* e, uint32_t operation, const void* d_events, uint32_t n, uint64_t T) {
  hipStream_t st = e->stream;
  phase_begin(e, PH_PREP);
  if (operation == TB_OP_CREATE_TRANSFERS)
    k_ct_prep<<<grid_for(n), 256, 0, st>>>(e->d, e->s, (const tb_transfer_t*)d_events, n, T);
  else
    k_ca_prep<<<grid_for(n), 256, 0, st>>>(e->d, e->s, (const tb_account_t*)d_events, n);
  phase_end(e);
  HIPCHK(hipGetLastError());
  return TBG_OK;
}

static int launch_rest(tbg_engine* e, uint32_t operation, const void* d_events, uint32_t n, uint64_t T,
                       tb_create_result_t* d_results, uint32_t* d_count) {
  hipStream_t st = e->stream;
  const uint32_t epoch = ++e->epoch;
  if (operation == TB_OP_CREATE_TRANSFERS) {
    phase_begin(e, PH_LINK);
    k_ct_link<<<grid_for(n), 256, 0, st>>>(e->d, e->s, n, epoch);
    phase_end(e);
    phase_begin(e, PH_MARK);
    k_ct_mark<<<grid_for(n), 256, 0, st>>>(e->d, e->s, n, epoch);
    phase_end(e);
    phase_begin(e, PH_SCAN);
    k_scan_walk<true><<<1, SCAN_THREADS, 0, st>>>(e->d, e->s, (const uint8_t*)d_events, n, T, d_results, d_count);
    phase_end(e);
    phase_begin(e, PH_APPLY);
    k_ct_apply<<<grid_for(n), 256, 0, st>>>(e->d, e->s, (const tb_transfer_t*)d_events, n, T);
    phase_end(e);
    e->x_upper += n;
  } else {
    k_ca_link<<<grid_for(n), 256, 0, st>>>(e->s, n);
    k_scan_walk<false><<<1, SCAN_THREADS, 0, st>>>(e->d, e->s, (const uint8_t*)d_events, n, T, d_results, d_count);
    k_ca_apply<<<grid_for(n), 256, 0, st>>>(e->d, e->s, (const tb_account_t*)d_events, n, T);
    e->acc_upper += n;
  }
  HIPCHK(hipGetLastError());
  return TBG_OK;
}

extern "C" int tbg_prefetch(tbg_engine* e, uint64_t op, uint32_t operation, const void* input, uint64_t len,
                            uint64_t prefetch_timestamp) {
  (void)op;
  if (!tbg_input_valid(e, operation, len)) return TBG_E_INVALID;
  e->pf_valid = 0;
  if (operation != TB_OP_CREATE_ACCOUNTS && operation != TB_OP_CREATE_TRANSFERS) return TBG_OK;
  const uint32_t n = (uint32_t)(len / 128);
  if (n == 0) return TBG_OK;
  HIPCHK(hipSetDevice(e->device));
  int rc = check_capacity(e, operation, n);
  if (rc) return rc;
  memcpy(e->h_pinned, input, len);
  HIPCHK(hipMemcpyAsync(e->d_in, e->h_pinned, len, hipMemcpyHostToDevice, e->stream));
  rc = launch_prep(e, operation, e->d_in, n, prefetch_timestamp);
  if (rc) return rc;
  e->pf_valid = 1;
  e->pf_operation = operation;
  e->pf_input = input;
  e->pf_len = len;
  e->pf_ts = prefetch_timestamp;
  return TBG_OK;
}

extern "C" int tbg_commit(tbg_engine* e, uint64_t op, uint64_t timestamp, uint32_t operation, const void* input,
                          uint64_t len, void* output, uint64_t output_cap, uint64_t* output_len) {
  (void)op;
  if (!tbg_input_valid(e, operation, len)) return TBG_E_INVALID;
  HIPCHK(hipSetDevice(e->device));
  *output_len = 0;
  if (operation == TB_OP_PULSE) {
    e->pf_valid = 0;
    int rc = launch_pulse(e, timestamp, ~0ull);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(e->stream));
    return TBG_OK;
  }
  if (operation == TB_OP_CREATE_ACCOUNTS || operation == TB_OP_CREATE_TRANSFERS) {
    const uint32_t n = (uint32_t)(len / 128);
    if (n == 0) {
      e->pf_valid = 0;
      return TBG_OK;
    }
    if (output_cap < (uint64_t)n * 8 && output_cap < TB_MESSAGE_BODY_SIZE_MAX) return TBG_E_STATE;
    const bool pf = e->pf_valid && e->pf_operation == operation && e->pf_input == input && e->pf_len == len &&
                    e->pf_ts == timestamp;
    e->pf_valid = 0;
    if (!pf) {
      int rc = check_capacity(e, operation, n);
      if (rc) return rc;
      memcpy(e->h_pinned, input, len);
      HIPCHK(hipMemcpyAsync(e->d_in, e->h_pinned, len, hipMemcpyHostToDevice, e->stream));
      rc = launch_prep(e, operation, e->d_in, n, timestamp);
      if (rc) return rc;
    }
    int rc = launch_rest(e, operation, e->d_in, n, timestamp, e->s.results, e->d_count);
    if (rc) return rc;
    uint32_t* h_count = (uint32_t*)e->h_pinned;
    HIPCHK(hipMemcpyAsync(h_count, e->d_count, 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    const uint32_t c = *h_count;
    if ((uint64_t)c * 8 > output_cap) return TBG_E_STATE;
    if (c) {
      HIPCHK(hipMemcpyAsync((uint8_t*)e->h_pinned + 64, e->s.results, (size_t)c * 8, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(hipStreamSynchronize(e->stream));
      memcpy(output, (uint8_t*)e->h_pinned + 64, (size_t)c * 8);
    }
    *output_len = (uint64_t)c * 8;
    return TBG_OK;
  }
  if (operation == TB_OP_LOOKUP_ACCOUNTS || operation == TB_OP_LOOKUP_TRANSFERS) {
    e->pf_valid = 0;
    const uint32_t n = (uint32_t)(len / 16);
    if (n == 0) return TBG_OK;
    memcpy(e->h_pinned, input, len);
    HIPCHK(hipMemcpyAsync(e->d_in, e->h_pinned, len, hipMemcpyHostToDevice, e->stream));
    if (operation == TB_OP_LOOKUP_ACCOUNTS)
      k_lookup<true><<<1, SCAN_THREADS, 0, e->stream>>>(e->d, (const tb_uint128_t*)e->d_in, n, e->d_out, e->d_count);
    else
      k_lookup<false><<<1, SCAN_THREADS, 0, e->stream>>>(e->d, (const tb_uint128_t*)e->d_in, n, e->d_out, e->d_count);
    HIPCHK(hipGetLastError());
    uint32_t* h_count = (uint32_t*)e->h_pinned;
    HIPCHK(hipMemcpyAsync(h_count, e->d_count, 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    const uint32_t c = *h_count;
    // Records that do not fit the reply are omitted (:1308, :1327).
    const uint64_t fit = std::min<uint64_t>(c, output_cap / 128);
    if (fit) {
      HIPCHK(hipMemcpyAsync(e->h_pinned, e->d_out, fit * 128, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(hipStreamSynchronize(e->stream));
      memcpy(output, e->h_pinned, fit * 128);
    }
    *output_len = fit * 128;
    return TBG_OK;
  }
  return TBG_E_INVALID;  // get_account_transfers / get_account_balances: out of scope
}

extern "C" int tbg_commit_device(tbg_engine* e, uint32_t operation, uint64_t timestamp, const void* d_events,
                                 uint32_t n, void* d_results, uint32_t* d_result_count, int auto_pulse,
                                 uint64_t prepare_timestamp) {
  if (operation != TB_OP_CREATE_ACCOUNTS && operation != TB_OP_CREATE_TRANSFERS) return TBG_E_INVALID;
  if (n > e->batch_max) return TBG_E_INVALID;
  HIPCHK(hipSetDevice(e->device));
  e->pf_valid = 0;
  if (auto_pulse) {
    int rc = launch_pulse(e, timestamp, prepare_timestamp);
    if (rc) return rc;
  }
  if (n == 0) {
    HIPCHK(hipMemsetAsync(d_result_count, 0, 4, e->stream));
    return TBG_OK;
  }
  int rc = check_capacity(e, operation, n);
  if (rc) return rc;
  rc = launch_prep(e, operation, d_events, n, timestamp);
  if (rc) return rc;
  return launch_rest(e, operation, d_events, n, timestamp, (tb_create_result_t*)d_results, d_result_count);
}

extern "C" int tbg_setup_balances(tbg_engine* e, const tb_uint128_t* id, const tb_uint128_t* dp,
                                  const tb_uint128_t* dpo, const tb_uint128_t* cp, const tb_uint128_t* cpo) {
  HIPCHK(hipSetDevice(e->device));
  k_setup<<<1, 1, 0, e->stream>>>(e->d, *id, *dp, *dpo, *cp, *cpo, e->d_found);
  HIPCHK(hipGetLastError());
  int found = 0;
  HIPCHK(hipMemcpyAsync(e->h_pinned, e->d_found, sizeof(int), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  memcpy(&found, e->h_pinned, sizeof(int));
  return found ? TBG_OK : TBG_E_STATE;
}

extern "C" int tbg_get_stats(tbg_engine* e, tbg_stats* out) {
  HIPCHK(hipSetDevice(e->device));
  Globals g;
  int rc = read_globals(e, &g);
  if (rc) return rc;
  out->accounts = g.acc_count;
  out->transfers = g.x_count;
  out->expiry_entries = g.exp_count;
  out->pulse_next_timestamp = g.pulse_next;
  out->events_total = g.events_total;
  out->walker_events = g.w_events_total;
  return TBG_OK;
}

static int dump(tbg_engine* e, const void* src, size_t elem, uint64_t count, void* out, uint64_t cap, uint64_t* n) {
  const uint64_t c = std::min(count, cap);
  if (c) HIPCHK(hipMemcpy(out, src, c * elem, hipMemcpyDeviceToHost));
  *n = c;
  return TBG_OK;
}

extern "C" int tbg_dump_accounts(tbg_engine* e, tb_account_t* out, uint64_t cap, uint64_t* count) {
  HIPCHK(hipSetDevice(e->device));
  Globals g;
  int rc = read_globals(e, &g);
  if (rc) return rc;
  return dump(e, e->d.acc, sizeof(tb_account_t), g.acc_count, out, cap, count);
}

extern "C" int tbg_dump_transfers(tbg_engine* e, tb_transfer_t* out, uint64_t cap, uint64_t* count) {
  HIPCHK(hipSetDevice(e->device));
  Globals g;
  int rc = read_globals(e, &g);
  if (rc) return rc;
  return dump(e, e->d.xr, sizeof(tb_transfer_t), g.x_count, out, cap, count);
}

extern "C" int tbg_dump_transfer_status(tbg_engine* e, uint8_t* out, uint64_t cap, uint64_t* count) {
  HIPCHK(hipSetDevice(e->device));
  Globals g;
  int rc = read_globals(e, &g);
  if (rc) return rc;
  return dump(e, e->d.xstatus, 1, g.x_count, out, cap, count);
}

// Per-phase timing: when enabled, every kernel phase is bracketed by HIP events on the engine
// stream. tbg_timing_collect() synchronizes, sums the elapsed times per phase (ms) and counts the
// launches, then resets.
extern "C" int tbg_timing_enable(tbg_engine* e, int enable) {
  e->timing = enable;
  return TBG_OK;
}

extern "C" int tbg_timing_collect(tbg_engine* e, double* ms, uint64_t* launches, uint32_t n_phases) {
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamSynchronize(e->stream));
  for (uint32_t p = 0; p < n_phases; p++) {
    ms[p] = 0;
    launches[p] = 0;
  }
  for (size_t k = 0; k < e->ev_phase.size(); k++) {
    float t = 0;
    HIPCHK(hipEventElapsedTime(&t, e->ev_pool[2 * k], e->ev_pool[2 * k + 1]));
    const uint32_t p = e->ev_phase[k];
    if (p < n_phases) {
      ms[p] += t;
      launches[p]++;
    }
  }
  e->ev_phase.clear();
  e->ev_used = 0;
  return TBG_OK;
}

// Debug/introspection: per-event class bits and codes of the last batch.
extern "C" int tbg_debug_last_batch(tbg_engine* e, uint32_t* cls, uint32_t* code, uint32_t n) {
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipMemcpy(cls, e->s.cls, (size_t)n * 4, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(code, e->s.code, (size_t)n * 4, hipMemcpyDeviceToHost));
  return TBG_OK;
}

extern "C" int tbg_device_stores(tbg_engine* e, const tb_account_t** accounts, const tb_transfer_t** transfers) {
  *accounts = e->d.acc;
  *transfers = e->d.xr;
  return TBG_OK;
}
