// pwalker.h — the long-component walker (k_cc_walk_long): the reference loop of walker.h over one
// component, run as a four-stage software pipeline.
//
// k_cc_walk runs one walker thread per component. Its time is set by the longest components (a
// component's walk is one chain of dependent reads per event: list position -> static row -> key-map
// commit of the pending id -> the pending record and status), while the many short ones need the
// plain walker's low register count (the whole grid resident). So components of CW_LONG events or
// more are left to this kernel, on a second stream beside k_cc_walk, where an event's inputs load
// over the four turns before its own: list position four turns ahead, static row three, key-map
// commit words and batch bounds two, body and pending record, accounts and status one. A turn waits
// only for loads issued one turn earlier. What a turn writes that the inputs already loaded for the
// next two turns may hold is forwarded into them (PEff: the entry it committed, the status it set),
// and a rollback makes them reload; the forwarded values are what the loads would read after the
// turn's stores, because a component's key-map entries and statuses are written by its own walker
// only. Same outputs as Walker::run<true>.
#pragma once
#include "walker.h"

#ifndef CW_LONG
#define CW_LONG 32  // components of this many events or more: k_cc_walk_long
#endif

struct PPre {
  uint32_t i, cls, b, code, id_tslot, id_ent, dr, cr, p_tslot, pid_ent;
};
// PDyn, two turns ahead: the raw key-map commit words of the event's id and pending id, its batch's
// bounds and commit timestamp; a commit made by a turn in between is forwarded (cf, pf).
// PRec, one turn ahead: its body and, for a post/void, the pending transfer's record (pq: all but
// its id and pending_id), accounts and status (pc: the window event the record was read from; -1:
// none, or a stored one). ok = false: a rollback (or, for PRec, a forwarded pending commit) left the
// loaded values stale; the turn reloads them.
#define FW_NONE (-2)
struct PDyn {
  unsigned long long cw, pw;
  uint32_t off0, off1;
  uint64_t T;
  int32_t cf, pf;
  bool ok;
};
struct PRec {
  tb_transfer_t t;
  uint4 pq[6];
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
struct PEff {
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

struct PWalker : Walker {
  // pulse_next as the window's pulse left it (walkers never change it: k_final and k_xwin_replay run
  // after them) and whether win_flags bit 3 is known to be set: read once per walk
  uint64_t pn0 = 0;
  bool wf8 = false;

  // Inserts event i's record t2 and commits its id (key-map entry e).
  __device__ __attribute__((always_inline)) void commit_x(uint32_t i, uint32_t e, const tb_transfer_t& t2, PEff& f) {
    s.t2[i] = t2;
    s.hside[i] = 0;
    log_small(UNDO_INS, i, 0);
    s.ins[i] = 2;  // the balance effects are k_final's (Walker::commit_record)
    // (the entry had no commit this window, or the caller would have found it: undo restores
    // "none", epoch 0, without reading the old word)
    log_small(UNDO_COMMIT, e, 0);
    bmap_set_committed(s.bmap, e, epoch, (int32_t)i);
    f.cent = e;
  }

  __device__ __attribute__((always_inline)) PPre pre(uint32_t i) const {
    PPre e;
    e.i = i;
    e.cls = s.cls[i];
    const uint4 r0 = s.wrow[2 * i], r1 = s.wrow[2 * i + 1];  // (Scratch::wrow)
    e.code = r0.x;
    e.id_tslot = r0.y;
    e.id_ent = r0.z;
    e.pid_ent = r0.w;
    e.dr = r1.x;
    e.cr = r1.y;
    e.p_tslot = r1.z;
    e.b = r1.w;
    return e;
  }
  // the key-map loads a turn may need (an entry exists only for events that reach the exists check)
  __device__ static __attribute__((always_inline)) bool needs_c(const PPre& e) {
    return (e.cls & (C_REACH | C_STATIC | C_IDALONE)) == C_REACH;
  }
  __device__ static __attribute__((always_inline)) bool needs_pc(const PPre& e) {
    return (e.cls & (C_REACH | C_STATIC | C_POSTVOID)) == (C_REACH | C_POSTVOID) && e.p_tslot == NONE32;
  }
  __device__ __attribute__((always_inline)) PDyn dyn_x(const PPre& e) const {
    PDyn y;
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
  __device__ __attribute__((always_inline)) int32_t dyn_c(const PPre& e, const PDyn& y) const {
    if (y.cf != FW_NONE) return y.cf;
    return needs_c(e) ? word_commit(y.cw) : -1;
  }
  __device__ __attribute__((always_inline)) int32_t dyn_pc(const PPre& e, const PDyn& y) const {
    if (y.pf != FW_NONE) return y.pf;
    return needs_pc(e) ? word_commit(y.pw) : -1;
  }
  __device__ __attribute__((always_inline)) PRec rec_x(const PPre& e, const PDyn& y) const {
    PRec r;
    r.ok = true;
    r.pc = -1;
    if (e.cls & C_STATIC) return r;
    r.t = reinterpret_cast<const tb_transfer_t*>(ev)[e.i];
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
        const uint4 pr = s.wrow[2 * r.pc + 1];
        r.drs = pr.x;
        r.crs = pr.y;
        r.pst = s.bstatus[r.pc];
      }
    }
    if (pp) {
      prec_load(r.pq, pp);
    }
    return r;
  }
  // A turn's writes into the inputs loaded for the next two turns (before those writes).
  __device__ __attribute__((always_inline)) static void fwd(const PEff& f, int32_t ci, const PPre& e1, PDyn& y1,
                                                            PRec& r1, const PPre& e2, PDyn& y2) {
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
  __device__ __attribute__((always_inline)) uint32_t transfer_x(const PPre& e, const PDyn& y, const PRec& rc, PEff& f) {
    const uint32_t i = e.i;
    if (e.cls & C_STATIC) return e.code;
    const int32_t c = dyn_c(e, y);
    tb_transfer_t t = rc.t;
    t.timestamp = y.T - (y.off1 - y.off0) + (i - y.off0) + 1;  // win_ts
    if (e.cls & C_POSTVOID) return post_or_void_x(e, y, rc, t, c, f);
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
    commit_x(i, e.id_ent, t, f);
    if (atomic_bal) {
      // the balance adds are k_final's (s.amt, the account slots: k_ct_prep's)
      if (t.flags & TB_TRANSFER_PENDING) s.bstatus[i] = TB_PENDING_PENDING;
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
  __device__ __attribute__((always_inline)) uint32_t post_or_void_x(const PPre& e, const PDyn& y, const PRec& rc,
                                                                  const tb_transfer_t& t, int32_t c, PEff& f) {
    const uint32_t i = e.i;
    const uint32_t pslot = e.p_tslot;
    const int32_t pc = rc.pc;
    if (pslot == NONE32 && pc < 0) return TB_CT_PENDING_TRANSFER_NOT_FOUND;
    const tb_transfer_t p = prec_view(rc.pq);  // (its id and pending_id read as zero: not used below)
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
    commit_x(i, e.id_ent, pv_record(t, p, amount), f);
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
      // the balance adds are k_final's: the amounts and, for a pending transfer of this window, its
      // accounts (k_ct_prep wrote them for a stored one)
      if (pc >= 0) {
        s.dr_slot[i] = drs;
        s.cr_slot[i] = crs;
      }
      s.pamt[i] = pa;
      s.amt[i] = amount;
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

  // The chain bookkeeping of one turn (:1236-1300) around its outcome r; true: it rolled back.
  __device__ __attribute__((always_inline)) bool settle_x(uint32_t i, uint32_t r, bool linked, int32_t& chain,
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
    PPre e0 = pre(list[0]), e1, e2;
    if (count > 1) e1 = pre(list[1]);
    if (count > 2) e2 = pre(list[2]);
    PDyn y0 = dyn_x(e0), y1;
    if (count > 1) y1 = dyn_x(e1);
    PRec r0 = rec_x(e0, y0);
    for (uint32_t k = 0; k < count; k++) {
      PPre e3;
      PDyn y2;
      PRec r1;
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
      PEff f = {NONE32, NONE32, NONE32, 0};
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
        r = transfer_x(e0, y0, r0, f);
      }
      if (settle_x(i, r, linked, chain, broken)) {
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

};
