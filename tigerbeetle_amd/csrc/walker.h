// walker.h — the sequential walker: the reference executor loop (state_machine.zig:1236-1301)
// restricted to the window's W events, in window order, with an undo log standing in for
// scope_open/scope_close (lsm/cache_map.zig:254-301). Everything else in the window is order-free
// and already resolved in parallel; W carries exactly the events whose outcome depends on order.
#pragma once
#include "sm_logic.h"
#include "window.h"

// An entry the expires_at scan can return (composite key range, lsm/composite_key.zig:25-57).
__device__ inline bool xw_visible(uint64_t timestamp, uint64_t expires_at) {
  return !(timestamp >> 63) && expires_at <= TB_TIMESTAMP_MAX;
}

// In a window with pulses inside (xwin.h): whether a post/void at batch b finds pending transfer p
// already expired by one of the window's pulses (the first batch with T >= its expires_at).
__device__ inline bool xw_expired_before(const WinDesc& w, const tb_transfer_t& p, uint32_t b) {
  if (!w.xwin || p.timeout == 0) return false;
  const uint64_t exp = expires_at_of(p);
  return xw_visible(p.timestamp, exp) && exp <= w.T[b];
}

// Window key map (see BEntry). `epoch` is the window number.
__device__ inline tb_uint128_t bkey(const uint8_t* ev, uint32_t owner, uint32_t is_pid) {
  return *reinterpret_cast<const tb_uint128_t*>(ev + (size_t)owner * 128 + (is_pid ? 64 : 0));
}

// Claims (or finds) the entry of `key` and bumps its id or pending_id count (saturating at 3).
__device__ inline uint32_t bmap_claim(BEntry* bm, uint32_t mask, const uint8_t* ev, tb_uint128_t key, uint32_t idx,
                                      uint32_t is_pid, uint32_t epoch) {
  const unsigned long long inc = is_pid ? (1ull << 23) : (1ull << 21);
  uint32_t h = (uint32_t)hash_id(key.lo, key.hi) & mask;
  for (;;) {
    unsigned long long old = __hip_atomic_load(&bm[h].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
      if (bk_epoch(old) != epoch) {
        const unsigned long long fresh =
            ((unsigned long long)epoch << 32) | ((unsigned long long)is_pid << 20) | idx | inc;
        const unsigned long long prev = atomicCAS(&bm[h].key, old, fresh);
        if (prev == old) return h;
        old = prev;
        continue;
      }
      const tb_uint128_t k = bkey(ev, bk_owner(old), bk_is_pid(old));
      if (k.lo != key.lo || k.hi != key.hi) break;  // another key: probe on
      if ((is_pid ? bk_pidc(old) : bk_idc(old)) == 3) return h;
      const unsigned long long prev = atomicCAS(&bm[h].key, old, old + inc);
      if (prev == old) return h;
      old = prev;
    }
    h = (h + 1) & mask;
  }
}

// A claim-free window (ids strictly increasing, no post/void: no key can repeat) gives each event a
// private entry past the hashed range instead of a claim: one plain store, no atomic.
__device__ inline uint32_t bmap_direct(BEntry* bm, uint32_t mask, uint32_t idx, uint32_t epoch) {
  const uint32_t e = mask + 1 + idx;
  bm[e].key = ((unsigned long long)epoch << 32) | idx | (1ull << 21);
  return e;
}

__device__ inline uint32_t bmap_idc(const BEntry* bm, uint32_t e, uint32_t epoch) {
  const unsigned long long k = bm[e].key;
  return bk_epoch(k) == epoch ? bk_idc(k) : 0;
}
__device__ inline uint32_t bmap_pidc(const BEntry* bm, uint32_t e, uint32_t epoch) {
  const unsigned long long k = bm[e].key;
  return bk_epoch(k) == epoch ? bk_pidc(k) : 0;
}
__device__ inline int32_t bmap_committed(const BEntry* bm, uint32_t e, uint32_t epoch) {
  const unsigned long long c = bm[e].commit;
  return bk_epoch(c) == epoch ? (int32_t)(uint32_t)c : -1;
}
__device__ inline void bmap_set_committed(BEntry* bm, uint32_t e, uint32_t epoch, int32_t i) {
  bm[e].commit = ((unsigned long long)epoch << 32) | (uint32_t)i;
}

// An event's static inputs (written by k_ct_prep / k_classify before any walker runs, never by a
// walker for a later event).
struct WPre {
  uint32_t i, cls, b, code, id_tslot, id_ent, dr, cr, p_tslot, pid_ent;
};

// Transfers (run_x) load the rest of an event's inputs ahead of its turn as well:
//   WDyn, two turns ahead: the raw key-map commit words of its id and pending id, and its batch's
//         bounds and commit timestamp. A commit made by a turn in between is forwarded (cf, pf).
//   WRec, one turn ahead: its body and, for a post/void, the pending transfer's record, accounts and
//         status (pc: the window event the record was read from; -1: none, or a stored one).
// ok = false: a rollback (or, for WRec, a forwarded pending commit) left the loaded values stale;
// the turn reloads them.
#define FW_NONE (-2)
struct WDyn {
  unsigned long long cw, pw;
  uint32_t off0, off1;
  uint64_t T;
  int32_t cf, pf;
  bool ok;
};
#ifndef WALK_REC_REGS
#define WALK_REC_REGS 1
#endif
struct WRec {
#if WALK_REC_REGS
  tb_transfer_t t;
  uint4 pq[6];  // the pending record's 16 B words 1-3 and 5-7 (all but its id and pending_id, unused)
#else
  uint4 th, ph;  // the body's first and the pending record's second 16 B: their lines, ahead
  const tb_transfer_t* pp;
#endif
  uint32_t drs, crs;
  int32_t pc;
  uint8_t pst;
  bool ok;
};
__device__ __attribute__((always_inline)) inline void prec_load(uint4* pq, const tb_transfer_t* src) {
  const uint4* q = reinterpret_cast<const uint4*>(src);
  pq[0] = q[1];
  pq[1] = q[2];
  pq[2] = q[3];
  pq[3] = q[5];
  pq[4] = q[6];
  pq[5] = q[7];
}
__device__ __attribute__((always_inline)) inline tb_transfer_t prec_view(const uint4* pq) {
  tb_transfer_t p;
  uint4* q = reinterpret_cast<uint4*>(&p);
  q[0] = make_uint4(0, 0, 0, 0);
  q[1] = pq[0];
  q[2] = pq[1];
  q[3] = pq[2];
  q[4] = make_uint4(0, 0, 0, 0);
  q[5] = pq[3];
  q[6] = pq[4];
  q[7] = pq[5];
  return p;
}
// What a turn wrote that inputs already loaded for later turns may hold.
struct WEff {
  uint32_t cent;  // the key-map entry it committed (NONE32: none)
  uint32_t bst;   // the window's pending transfer whose status it set (NONE32: none)
  uint32_t xst;   // the stored pending transfer whose status it set (NONE32: none)
  uint8_t v;      // the status it set
};

// In a window with pulses inside: whether a post/void in a batch committed at T_b finds pending
// transfer p already expired by one of the window's pulses (xw_expired_before, batch time given).
__device__ inline bool xw_expired_at(const WinDesc& w, const tb_transfer_t& p, uint64_t T_b) {
  if (!w.xwin || p.timeout == 0) return false;
  const uint64_t exp = expires_at_of(p);
  return xw_visible(p.timestamp, exp) && exp <= T_b;
}

struct Walker {
  Dev d;
  Scratch s;
  const uint8_t* ev;
  const WinDesc* w;
  uint32_t epoch;
  uint32_t undo_n;
  bool scope;
  // Component-parallel mode (k_cc_walk): other walkers run concurrently on other components and may
  // touch the same accounts, so balance effects are atomic adds (undone by atomic subtracts). Only
  // used in windows where no decision reads a balance (no hot account, no overflow risk), so the
  // racy balance values read below never change an outcome.
  bool atomic_bal;
  // With atomic_bal: the window keeps every balance field below 2^64 (Globals::small_win), so a
  // balance delta is a no-return 64-bit add on the low word (mod 2^64; the true value never leaves
  // the low word) and no walker waits for an atomic's result.
  bool small_bal = false;
  // pulse_next as the window's pulse left it (walkers never change it: k_final and k_xwin_replay run
  // after them) and whether win_flags bit 3 is known to be set: read once per walk instead of on
  // every post/void of a timed pending transfer created in the window.
  uint64_t pn0 = 0;
  bool wf8 = false;

  __device__ __attribute__((always_inline)) void log_bal(uint32_t slot) {
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
  __device__ __attribute__((always_inline)) void log_small(uint32_t kind, uint32_t a, u128 old) {
    if (!scope) return;
    UndoRec& r = s.undo[undo_n++];
    r.kind = kind;
    r.a = a;
    r.old[0] = old;
  }
  __device__ static tb_uint128_t* bal_field(tb_account_t* a, uint32_t f) {
    return f == 0 ? &a->debits_pending : f == 1 ? &a->debits_posted : f == 2 ? &a->credits_pending : &a->credits_posted;
  }
  __device__ __attribute__((always_inline)) void add_bal(uint32_t slot, uint32_t f, u128 v) {
    if (small_bal)
      (void)atomicAdd(reinterpret_cast<unsigned long long*>(bal_field(&d.acc[slot], f)), (unsigned long long)v);
    else
      atomic_add_u128(bal_field(&d.acc[slot], f), v);
    if (!scope) return;
    UndoRec& r = s.undo[undo_n++];
    r.kind = UNDO_ADD;
    r.a = slot;
    r.pad0 = f;
    r.old[0] = v;
  }
  __device__ __attribute__((always_inline)) void rollback() {
    while (undo_n) {
      const UndoRec& r = s.undo[--undo_n];
      switch (r.kind) {
        case UNDO_ADD:
          if (small_bal)
            (void)atomicAdd(reinterpret_cast<unsigned long long*>(bal_field(&d.acc[r.a], r.pad0)),
                            (unsigned long long)((u128)0 - r.old[0]));
          else
            atomic_add_u128(bal_field(&d.acc[r.a], r.pad0), (u128)0 - r.old[0]);
          break;
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
        case UNDO_COMMIT: s.bmap[r.a].commit = (unsigned long long)r.old[0]; break;
        case UNDO_INS: s.ins[r.a] = 0; break;
      }
    }
  }

  // historical_balance (:1806-1841): the row of event i from the accounts' balances after it
  // (sequential mode only: windows with history accounts never run component walkers)
  __device__ __attribute__((always_inline)) void history(uint32_t i, uint32_t drs, const Bal& dr, uint32_t crs, const Bal& cr) {
    const uint16_t fd = d.acc[drs].flags, fc = d.acc[crs].flags;
    if (!((fd | fc) & TB_ACCOUNT_HISTORY)) return;
    HistRow r;
    uint8_t side = 0;
    for (int k = 0; k < 4; k++) r.dr[k] = r.cr[k] = 0;
    if (fd & TB_ACCOUNT_HISTORY) {
      side |= 1;
      r.dr[0] = dr.dp, r.dr[1] = dr.dpo, r.dr[2] = dr.cp, r.dr[3] = dr.cpo;
    }
    if (fc & TB_ACCOUNT_HISTORY) {
      side |= 2;
      r.cr[0] = cr.dp, r.cr[1] = cr.dpo, r.cr[2] = cr.cp, r.cr[3] = cr.cpo;
    }
    s.hrow[i] = r;
    s.hside[i] = side;
  }

  // Inserts event i's record t2 and commits its id (key-map entry e).
  __device__ __attribute__((always_inline)) void commit_record(uint32_t i, uint32_t e, const tb_transfer_t& t2, WEff& f) {
    s.t2[i] = t2;
    s.hside[i] = 0;
    log_small(UNDO_INS, i, 0);
    s.ins[i] = 1;
    // (the entry had no commit this window, or the caller would have found it: undo restores
    // "none", epoch 0, without reading the old word)
    log_small(UNDO_COMMIT, e, 0);
    bmap_set_committed(s.bmap, e, epoch, (int32_t)i);
    f.cent = e;
  }

  __device__ __attribute__((always_inline)) WPre pre(uint32_t i) const {
    WPre e;
    e.i = i;
    e.cls = s.cls[i];
    e.b = s.batch[i];
    e.code = s.code[i];
    e.id_tslot = s.id_tslot[i];
    e.id_ent = s.id_ent[i];
    e.dr = s.dr_slot[i];
    e.cr = s.cr_slot[i];
    e.p_tslot = s.p_tslot[i];
    e.pid_ent = s.pid_ent[i];
    return e;
  }
  // the key-map loads a turn may need (an entry exists only for events that reach the exists check)
  __device__ static __attribute__((always_inline)) bool needs_c(const WPre& e) {
    return (e.cls & (C_REACH | C_STATIC | C_IDALONE)) == C_REACH;
  }
  __device__ static __attribute__((always_inline)) bool needs_pc(const WPre& e) {
    return (e.cls & (C_REACH | C_STATIC | C_POSTVOID)) == (C_REACH | C_POSTVOID) && e.p_tslot == NONE32;
  }
  __device__ __attribute__((always_inline)) WDyn dyn_x(const WPre& e) const {
    WDyn y;
    y.cw = y.pw = 0;
    if (needs_c(e)) y.cw = s.bmap[e.id_ent].commit;
    if (needs_pc(e)) y.pw = s.bmap[e.pid_ent].commit;
    y.off0 = w->off[e.b];
    y.off1 = w->off[e.b + 1];
    y.T = w->T[e.b];
    y.cf = y.pf = FW_NONE;
    y.ok = true;
    return y;
  }
  __device__ __attribute__((always_inline)) int32_t word_commit(unsigned long long c) const {
    return bk_epoch(c) == epoch ? (int32_t)(uint32_t)c : -1;
  }
  __device__ __attribute__((always_inline)) int32_t dyn_c(const WPre& e, const WDyn& y) const {
    if (y.cf != FW_NONE) return y.cf;
    return needs_c(e) ? word_commit(y.cw) : -1;
  }
  __device__ __attribute__((always_inline)) int32_t dyn_pc(const WPre& e, const WDyn& y) const {
    if (y.pf != FW_NONE) return y.pf;
    return needs_pc(e) ? word_commit(y.pw) : -1;
  }
  __device__ __attribute__((always_inline)) WRec rec_x(const WPre& e, const WDyn& y) const {
    WRec r;
    r.ok = true;
    r.pc = -1;
    if (e.cls & C_STATIC) return r;
#if WALK_REC_REGS
    r.t = reinterpret_cast<const tb_transfer_t*>(ev)[e.i];
#else
    r.th = reinterpret_cast<const uint4*>(ev)[(size_t)e.i * 8];
#endif
    if (!(e.cls & C_POSTVOID)) return r;
    const tb_transfer_t* pp = nullptr;
    if (e.p_tslot != NONE32) {
      pp = &d.xr[e.p_tslot];
      r.drs = e.dr;
      r.crs = e.cr;
      r.pst = d.xstatus[e.p_tslot];
    } else {
      r.pc = dyn_pc(e, y);
      if (r.pc >= 0) {
        pp = &s.t2[r.pc];
        r.drs = s.dr_slot[r.pc];
        r.crs = s.cr_slot[r.pc];
        r.pst = s.bstatus[r.pc];
      }
    }
    if (pp) {
#if WALK_REC_REGS
      prec_load(r.pq, pp);
#else
      r.pp = pp;
      r.ph = reinterpret_cast<const uint4*>(pp)[1];
#endif
    }
    return r;
  }
  // A turn's writes into the inputs loaded for the next two turns (before those writes).
  __device__ __attribute__((always_inline)) static void fwd(const WEff& f, int32_t ci, const WPre& e1, WDyn& y1,
                                                            WRec& r1, const WPre& e2, WDyn& y2) {
    if (f.cent != NONE32) {
      if (needs_c(e1) && e1.id_ent == f.cent) y1.cf = ci;
      if (needs_pc(e1) && e1.pid_ent == f.cent) {
        y1.pf = ci;
        r1.ok = false;
      }
      if (needs_c(e2) && e2.id_ent == f.cent) y2.cf = ci;
      if (needs_pc(e2) && e2.pid_ent == f.cent) y2.pf = ci;
    }
    if (f.bst != NONE32 && r1.pc == (int32_t)f.bst) r1.pst = f.v;
    if (f.xst != NONE32 && (e1.cls & C_POSTVOID) && e1.p_tslot == f.xst) r1.pst = f.v;
  }

  // create_transfer (:1462-1585) from the exists check on; validation results come from k_ct_prep.
  __device__ __attribute__((always_inline)) uint32_t transfer(const WPre& e, const WDyn& y, const WRec& rc, WEff& f) {
    const uint32_t i = e.i;
    if (e.cls & C_STATIC) return e.code;
    const int32_t c = dyn_c(e, y);
#if WALK_REC_REGS
    tb_transfer_t t = rc.t;
#else
    tb_transfer_t t;
    {
      const uint4* q = reinterpret_cast<const uint4*>(ev) + (size_t)i * 8;
      uint4* tq = reinterpret_cast<uint4*>(&t);
      tq[0] = rc.th;
#pragma unroll
      for (int k = 1; k < 8; k++) tq[k] = q[k];
    }
#endif
    t.timestamp = y.T - (y.off1 - y.off0) + (i - y.off0) + 1;  // win_ts
    if (e.cls & C_POSTVOID) return post_or_void(e, y, rc, t, c, f);
    if (e.id_tslot != NONE32) return ct_exists(t, d.xr[e.id_tslot]);
    if (c >= 0) return ct_exists(t, s.t2[c]);
    const uint32_t drs = e.dr, crs = e.cr;
    tb_account_t* dra = &d.acc[drs];
    tb_account_t* cra = &d.acc[crs];
    u128 amount;
    if (atomic_bal) {
      // No decision of this window reads a balance (no event has C_READS_*: no limit flag on its
      // accounts, no balancing) and it is overflow-free: the checks see zero balances the same way.
      const Bal z = {0, 0, 0, 0};
      const uint32_t r = ct_balances(t, z, 0, z, 0, &amount);
      if (r != TB_CT_OK) return r;
    }
    Bal dr, cr;
    if (!atomic_bal) {
      dr = load_bal(dra);
      cr = load_bal(cra);
      const uint32_t r = ct_balances(t, dr, dra->flags, cr, cra->flags, &amount);
      if (r != TB_CT_OK) return r;
    }
    t.amount = W(amount);
    commit_record(i, e.id_ent, t, f);
    if (atomic_bal) {
      const bool pend = t.flags & TB_TRANSFER_PENDING;
      add_bal(drs, pend ? 0 : 1, amount);
      add_bal(crs, pend ? 2 : 3, amount);
      if (pend) s.bstatus[i] = TB_PENDING_PENDING;
      return TB_CT_OK;
    }
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
    history(i, drs, dr, crs, cr);  // :1570-1574
    return TB_CT_OK;
  }

  // post_or_void_pending_transfer (:1608-1741) from the pending lookup on. `c`: this event's id
  // committed earlier in the window (or -1); rc.pc: the in-window pending transfer (-1: none, or the
  // pending transfer was stored before the window: p_tslot).
  __device__ __attribute__((always_inline)) uint32_t post_or_void(const WPre& e, const WDyn& y, const WRec& rc,
                                                                  const tb_transfer_t& t, int32_t c, WEff& f) {
    const uint32_t i = e.i;
    const uint32_t pslot = e.p_tslot;
    const int32_t pc = rc.pc;
    if (pslot == NONE32 && pc < 0) return TB_CT_PENDING_TRANSFER_NOT_FOUND;
#if WALK_REC_REGS
    const tb_transfer_t p = prec_view(rc.pq);  // (its id and pending_id read as zero: not used below)
#else
    uint4 pq[6];
    {
      const uint4* q = reinterpret_cast<const uint4*>(rc.pp);
      pq[0] = rc.ph;
      pq[1] = q[2];
      pq[2] = q[3];
      pq[3] = q[5];
      pq[4] = q[6];
      pq[5] = q[7];
    }
    const tb_transfer_t p = prec_view(pq);
#endif
    const uint32_t drs = rc.drs, crs = rc.crs;
    u128 amount;
    uint32_t r = pv_against(t, p, &amount);
    if (r != CONT) return r;
    if (e.id_tslot != NONE32) return pv_exists(t, d.xr[e.id_tslot], p);
    if (c >= 0) return pv_exists(t, s.t2[c], p);
    uint8_t pst = rc.pst;
    if (pst == TB_PENDING_PENDING && xw_expired_at(*w, p, y.T)) pst = TB_PENDING_EXPIRED;
    r = pv_status(pst);
    if (r != CONT) return r;
    commit_record(i, e.id_ent, pv_record(t, p, amount), f);
    if (p.timeout > 0 && expires_at_of(p) <= t.timestamp) return TB_CT_PENDING_TRANSFER_EXPIRED;
    if (pc >= 0 && p.timeout > 0) {
      // p was created in this window (k_ct_prep could not see it): the expires_at removal and the
      // pulse_next reset candidate (:1698-1708) for k_pn
      const uint64_t pnv = expires_at_of(p);
      s.pnv[i] = pnv;
      s.pn_src[i] = (uint32_t)pc;
      s.cls[i] = e.cls | C_PNOP;  // (no turn before this one wrote event i's class)
      // may reset pulse_next (needs expires_at <= pulse_next as it was after the window's pulse,
      // which holds until k_final): k_final then replays the window's ops in order
      if (pnv <= pn0 && !wf8) {
        atomicOr(&d.g->win_flags, 8u);
        wf8 = true;
      }
    }
    const uint8_t st = (t.flags & TB_TRANSFER_POST_PENDING) ? TB_PENDING_POSTED : TB_PENDING_VOIDED;
    f.v = st;
    if (pc >= 0) {
      log_small(UNDO_BST, (uint32_t)pc, rc.pst);
      s.bstatus[pc] = st;
      f.bst = (uint32_t)pc;
    } else {
      log_small(UNDO_XST, pslot, rc.pst);
      d.xstatus[pslot] = st;
      f.xst = pslot;
    }
    const u128 pa = U(p.amount);
    if (atomic_bal) {
      add_bal(drs, 0, (u128)0 - pa);
      add_bal(crs, 2, (u128)0 - pa);
      if (t.flags & TB_TRANSFER_POST_PENDING) {
        add_bal(drs, 1, amount);
        add_bal(crs, 3, amount);
      }
      return TB_CT_OK;
    }
    tb_account_t* dra = &d.acc[drs];
    tb_account_t* cra = &d.acc[crs];
    Bal dr = load_bal(dra), cr = load_bal(cra);
    log_bal(drs);
    log_bal(crs);
    dr.dp -= pa;
    cr.cp -= pa;
    if (t.flags & TB_TRANSFER_POST_PENDING) {
      dr.dpo += amount;
      cr.cpo += amount;
    }
    store_bal(dra, dr);
    store_bal(cra, cr);
    history(i, drs, dr, crs, cr);  // :1732-1736
    return TB_CT_OK;
  }

  // create_account (:1421-1448) from the exists check on.
  __device__ __attribute__((always_inline)) uint32_t account(uint32_t i, uint32_t cls) {
    if (cls & C_STATIC) return s.code[i];
    if (s.id_tslot[i] != NONE32) return s.code[i];  // exists before the window: static
    const tb_account_t* evs = reinterpret_cast<const tb_account_t*>(ev);
    const uint32_t e = s.id_ent[i];
    const int32_t c = bmap_committed(s.bmap, e, epoch);
    if (c >= 0) return ca_exists(evs[i], evs[c]);
    log_small(UNDO_INS, i, 0);
    s.ins[i] = 1;
    log_small(UNDO_COMMIT, e, 0);  // no commit of this id this window (c < 0 above)
    bmap_set_committed(s.bmap, e, epoch, (int32_t)i);
    return TB_CA_OK;
  }

  // The chain bookkeeping of one turn (:1236-1300) around its outcome r; true: it rolled back.
  __device__ __attribute__((always_inline)) bool settle(uint32_t i, uint32_t r, bool linked, int32_t& chain,
                                                        bool& broken) {
    bool rolled = false;
    if (r != TB_CT_OK && chain >= 0 && !broken) {
      broken = true;
      rolled = undo_n != 0;
      rollback();
      for (uint32_t j = (uint32_t)chain; j < i; j++) {
        s.code[j] = TB_CT_LINKED_EVENT_FAILED;
        s.cls[j] |= C_RANOK;  // ran ok before the rollback: its pulse_next op stands (k_pn)
      }
    }
    s.code[i] = r;
    if (chain >= 0 && (!linked || r == TB_CT_LINKED_EVENT_CHAIN_OPEN)) {
      chain = -1;
      broken = false;
      scope = false;
      undo_n = 0;
    }
    return rolled;
  }

  // Transfers: the events list[0..count) (ascending window positions) as a four-stage software
  // pipeline. An event's inputs load over the turns before its own: its list position (four turns
  // ahead), its static inputs (three), its key-map commits and batch bounds (two), its body and its
  // pending transfer's record and status (one). A turn then waits only for loads issued a turn
  // earlier instead of a chain of dependent reads (a component's walk is one such chain per event);
  // what a turn writes is forwarded into the inputs already loaded for the next two (fwd), and a
  // rollback makes them reload.
  __device__ void run_x(const uint32_t* list, uint32_t count) {
    int32_t chain = -1;
    bool broken = false;
    undo_n = 0;
    scope = false;
    pn0 = d.g->pulse_next;
    wf8 = (__hip_atomic_load(&d.g->win_flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 8u) != 0;
    if (!count) return;
    uint32_t i3 = count > 3 ? list[3] : 0u;
    WPre e0 = pre(list[0]), e1, e2;
    if (count > 1) e1 = pre(list[1]);
    if (count > 2) e2 = pre(list[2]);
    WDyn y0 = dyn_x(e0), y1;
    if (count > 1) y1 = dyn_x(e1);
    WRec r0 = rec_x(e0, y0);
    for (uint32_t k = 0; k < count; k++) {
      WPre e3;
      WDyn y2;
      WRec r1;
      uint32_t i4 = 0;
      if (k + 3 < count) {
        e3 = pre(i3);
        if (k + 4 < count) i4 = list[k + 4];
      }
      if (k + 2 < count) y2 = dyn_x(e2);
      if (k + 1 < count) r1 = rec_x(e1, y1);
      if (!y0.ok) {
        y0 = dyn_x(e0);
        r0.ok = false;
      }
      if (!r0.ok) r0 = rec_x(e0, y0);
      const uint32_t i = e0.i, cls = e0.cls;
      const bool linked = cls & C_LINKED;
      WEff f = {NONE32, NONE32, NONE32, 0};
      uint32_t r;
      if (linked && chain < 0) {
        chain = (int32_t)i;
        undo_n = 0;
        scope = true;
      }
      if (linked && i == y0.off1 - 1) {
        r = TB_CT_LINKED_EVENT_CHAIN_OPEN;
      } else if (broken) {
        r = TB_CT_LINKED_EVENT_FAILED;
      } else if (cls & C_TSNZ) {
        r = TB_CT_TIMESTAMP_MUST_BE_ZERO;
      } else {
        r = transfer(e0, y0, r0, f);
      }
      if (settle(i, r, linked, chain, broken)) {
        y1.ok = false;
        r1.ok = false;
        y2.ok = false;
      } else {
        fwd(f, (int32_t)i, e1, y1, r1, e2, y2);
      }
      e0 = e1;
      e1 = e2;
      e2 = e3;
      i3 = i4;
      y0 = y1;
      y1 = y2;
      r0 = r1;
    }
  }

  // Walks the events list[0..count) (ascending window positions).
  template <bool XFER>
  __device__ __attribute__((always_inline)) void run(const uint32_t* list, uint32_t count) {
    if constexpr (XFER) {
      run_x(list, count);
    } else {
      int32_t chain = -1;
      bool broken = false;
      undo_n = 0;
      scope = false;
      for (uint32_t k = 0; k < count; k++) {
        const uint32_t i = list[k];
        const uint32_t cls = s.cls[i];
        const bool linked = cls & C_LINKED;
        const uint32_t b = s.batch[i];
        uint32_t r;
        if (linked && chain < 0) {
          chain = (int32_t)i;
          undo_n = 0;
          scope = true;
        }
        if (linked && i == w->off[b + 1] - 1) {
          r = TB_CT_LINKED_EVENT_CHAIN_OPEN;
        } else if (broken) {
          r = TB_CT_LINKED_EVENT_FAILED;
        } else if (cls & C_TSNZ) {
          r = TB_CT_TIMESTAMP_MUST_BE_ZERO;
        } else {
          r = account(i, cls);
        }
        settle(i, r, linked, chain, broken);
      }
    }
  }
};
