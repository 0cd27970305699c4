// walker.h — the sequential walker: the reference executor loop (state_machine.zig:1236-1301)
// restricted to the window's W events, in window order, with an undo log standing in for
// scope_open/scope_close (lsm/cache_map.zig:254-301). Everything else in the window is order-free
// and already resolved in parallel; W carries exactly the events whose outcome depends on order.
#pragma once
#include "sm_logic.h"
#include "window.h"

#ifndef WALK_CREATE_ROW
#define WALK_CREATE_ROW 1  // component walkers: creates decided from k_ct_prep's row (no record load)
#endif

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
// walker for a later event), loaded one event ahead so the walk pays only its dynamic reads.
struct WPre {
  uint32_t i, cls, b, code, id_tslot, id_ent, dr, cr, p_tslot, pid_ent;
  bool id_alone;  // no other event of the window carries this id: no earlier commit of it to look up
  uint4 head;     // transfers: the event's first 16 B (its id), loaded one event ahead: the load brings
                  // the record's line into the cache, so the rest of it is a cache hit when it runs
};

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
  // This walker's recent commits (id key-map entry -> event index), direct-mapped in LDS: a
  // post/void of a pending transfer its component created finds it without the key-map read (a
  // component's keys are committed by its own walker only; cleared on every rollback). nullptr: off.
  uint2* pcache = nullptr;
  // create_transfers component walkers: an event's static inputs from its Scratch::wrow row
  bool rows = false;
#define WCACHE 8
  __device__ __attribute__((always_inline)) int32_t pcache_find(uint32_t ent) const {
    if (!pcache) return -1;
    const uint2 c = pcache[ent & (WCACHE - 1)];
    return c.x == ent ? (int32_t)c.y : -1;
  }

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
    if (pcache)
      for (int k = 0; k < WCACHE; k++) pcache[k] = make_uint2(NONE32, 0);
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

  // Event i's record t2 (pv: a posting record) and its id's commit (key-map entry e). A component
  // walker (atomic_bal) stores no record for a create: k_final stamps the input row, and a later
  // reader here takes the input row too (walk_record); nor a history side (none in its windows).
  __device__ __attribute__((always_inline)) void commit_record(uint32_t i, uint32_t e, const tb_transfer_t& t2, bool pv) {
    if (!atomic_bal || pv) s.t2[i] = t2;
    if (!atomic_bal) s.hside[i] = 0;
    log_small(UNDO_INS, i, 0);
    // 2: component mode, the balance effects are k_final's (an event committed iff ins and code ok)
    s.ins[i] = atomic_bal ? 2 : 1;
    // (the entry had no commit this window, or the caller would have found it: undo restores
    // "none", epoch 0, without reading the old word)
    log_small(UNDO_COMMIT, e, 0);
    bmap_set_committed(s.bmap, e, epoch, (int32_t)i);
    if (pcache) pcache[e & (WCACHE - 1)] = make_uint2(e, i);
  }

  // The record event c committed earlier in the window (the exists checks compare no timestamp).
  __device__ __attribute__((always_inline)) const tb_transfer_t& walk_record(int32_t c) const {
    if (atomic_bal && !(s.cls[c] & C_POSTVOID)) return reinterpret_cast<const tb_transfer_t*>(ev)[c];
    return s.t2[c];
  }

  template <bool XFER>
  __device__ __attribute__((always_inline)) WPre fetch(uint32_t i) {
    WPre e;
    e.i = i;
    e.cls = s.cls[i];
    if (XFER && rows) {
      const uint4 r0 = s.wrow[2 * i], r1 = s.wrow[2 * i + 1];
      e.code = r0.x;
      e.id_tslot = r0.y;
      e.id_ent = r0.z;
      e.pid_ent = r0.w;
      e.dr = r1.x;
      e.cr = r1.y;
      e.p_tslot = r1.z;
      e.b = r1.w;
      // (a component walker loads an event's record only where it reads it: a create's outcome is
      // k_ct_prep's code unless an earlier event of the window committed its id, WALK_CREATE_ROW)
      if (!WALK_CREATE_ROW || !atomic_bal) e.head = reinterpret_cast<const uint4*>(ev)[(size_t)i * 8];
      e.id_alone = (e.cls & C_IDALONE) != 0;
      return e;
    }
    e.b = s.batch[i];
    e.code = s.code[i];
    e.id_tslot = s.id_tslot[i];
    e.id_ent = s.id_ent[i];
    if (XFER) {
      e.dr = s.dr_slot[i];
      e.cr = s.cr_slot[i];
      e.p_tslot = s.p_tslot[i];
      e.pid_ent = s.pid_ent[i];
      e.head = reinterpret_cast<const uint4*>(ev)[(size_t)i * 8];
    }
    e.id_alone = (e.cls & C_IDALONE) != 0;  // k_classify
    return e;
  }

  // create_transfer (:1462-1585) from the exists check on; validation results come from k_ct_prep.
  __device__ __attribute__((always_inline)) uint32_t transfer(const WPre& e) {
    const uint32_t i = e.i;
    if (e.cls & C_STATIC) return e.code;
    // The key-map reads whose entries are known now (this event's id, a post/void's pending id) go
    // out with the event body's load: a component's walk is a chain of dependent reads, and nothing
    // this event does before their original use writes them.
    const bool pv = e.cls & C_POSTVOID;
    const int32_t c = e.id_alone ? -1 : bmap_committed(s.bmap, e.id_ent, epoch);
    int32_t pc = -1;
    if (pv && e.p_tslot == NONE32) {
      pc = pcache_find(e.pid_ent);
      if (pc < 0) pc = bmap_committed(s.bmap, e.pid_ent, epoch);
    }
    if (WALK_CREATE_ROW && atomic_bal && rows && !pv) {
      // create in a component window: k_ct_prep's code is the walker's result (the stored-id exists
      // check, else the zero-balance tail: ok or overflows_timeout; no balancing, no limits here)
      // unless an earlier event of the window committed its id
      if (e.id_tslot != NONE32) return e.code;
      if (c >= 0) {
        tb_transfer_t t = reinterpret_cast<const tb_transfer_t*>(ev)[i];
        t.timestamp = win_ts(*w, e.b, i);
        return ct_exists(t, walk_record(c));
      }
      if (e.code != TB_CT_OK) return e.code;
      tb_transfer_t none;
      commit_record(i, e.id_ent, none, false);  // (a component walker stores no record for a create)
      if (e.cls & C_PENDING) s.bstatus[i] = TB_PENDING_PENDING;
      return TB_CT_OK;
    }
    tb_transfer_t t = reinterpret_cast<const tb_transfer_t*>(ev)[i];
    if (!WALK_CREATE_ROW || !atomic_bal) {
      t.id.lo = ((uint64_t)e.head.y << 32) | e.head.x;
      t.id.hi = ((uint64_t)e.head.w << 32) | e.head.z;
    }
    t.timestamp = win_ts(*w, e.b, i);
    if (pv) return post_or_void(e, t, c, pc);
    if (e.id_tslot != NONE32) return ct_exists(t, d.xr[e.id_tslot]);
    if (c >= 0) return ct_exists(t, walk_record(c));
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
    commit_record(i, e.id_ent, t, false);
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
  // committed earlier in the window (or -1); `pc`: the in-window pending transfer (-1: none, or the
  // pending transfer was stored before the window: p_tslot). The pending record, its accounts and its
  // status are read together.
  __device__ __attribute__((always_inline)) uint32_t post_or_void(const WPre& e, const tb_transfer_t& t, int32_t c,
                                                                  int32_t pc) {
    const uint32_t i = e.i;
    const uint32_t pslot = e.p_tslot;
    uint32_t drs, crs, pb = NONE32;  // pb: the in-window pending transfer's batch (from its row)
    uint8_t pst0;
    const tb_transfer_t* pp;  // one load from the selected record (no merged aggregate)
    if (pslot != NONE32) {
      pp = &d.xr[pslot];
      drs = e.dr;
      crs = e.cr;
      pst0 = d.xstatus[pslot];
    } else {
      if (pc < 0) return TB_CT_PENDING_TRANSFER_NOT_FOUND;
      // (a component walker stored no record for it: its input row, stamped below)
      pp = atomic_bal ? reinterpret_cast<const tb_transfer_t*>(ev) + pc : &s.t2[pc];
      if (rows) {
        const uint4 r1 = s.wrow[2 * pc + 1];
        drs = r1.x;
        crs = r1.y;
        pb = r1.w;
      } else {
        drs = s.dr_slot[pc];
        crs = s.cr_slot[pc];
      }
      pst0 = s.bstatus[pc];
    }
    tb_transfer_t p = *pp;
    if (atomic_bal && pslot == NONE32) p.timestamp = win_ts(*w, pb == NONE32 ? s.batch[pc] : pb, (uint32_t)pc);
    u128 amount;
    uint32_t r = pv_against(t, p, &amount);
    if (r != CONT) return r;
    if (e.id_tslot != NONE32) return pv_exists(t, d.xr[e.id_tslot], p);
    if (c >= 0) return pv_exists(t, walk_record(c), p);
    uint8_t pst = pst0;
    if (pst == TB_PENDING_PENDING && xw_expired_before(*w, p, s.batch[i])) pst = TB_PENDING_EXPIRED;
    r = pv_status(pst);
    if (r != CONT) return r;
    commit_record(i, e.id_ent, pv_record(t, p, amount), true);
    if (p.timeout > 0 && expires_at_of(p) <= t.timestamp) return TB_CT_PENDING_TRANSFER_EXPIRED;
    if (pc >= 0 && p.timeout > 0) {
      // p was created in this window (k_ct_prep could not see it): the expires_at removal and the
      // pulse_next reset candidate (:1698-1708) for k_pn
      s.pnv[i] = expires_at_of(p);
      s.pn_src[i] = (uint32_t)pc;
      s.cls[i] |= C_PNOP;
      // may reset pulse_next (needs expires_at <= pulse_next as it was after the window's pulse,
      // which holds until k_final): k_final then replays the window's ops in order
      if (s.pnv[i] <= d.g->pulse_next && !(__hip_atomic_load(&d.g->win_flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 8u))
        atomicOr(&d.g->win_flags, 8u);
    }
    const uint8_t st = (t.flags & TB_TRANSFER_POST_PENDING) ? TB_PENDING_POSTED : TB_PENDING_VOIDED;
    if (pc >= 0) {
      log_small(UNDO_BST, (uint32_t)pc, pst0);
      s.bstatus[pc] = st;
    } else {
      log_small(UNDO_XST, pslot, pst0);
      d.xstatus[pslot] = st;
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

  // Walks the events list[0..count) (ascending window positions).
  template <bool XFER>
  __device__ __attribute__((always_inline)) void run(const uint32_t* list, uint32_t count) {
    int32_t chain = -1;
    bool broken = false;
    undo_n = 0;
    scope = false;
    // software pipeline: event k + 1's static inputs load while event k runs; list[k + 2] one
    // step earlier still
    WPre nx;
    uint32_t i2 = NONE32;
    if (count) nx = fetch<XFER>(list[0]);
    if (count > 1) i2 = list[1];
    for (uint32_t k = 0; k < count; k++) {
      const WPre cur = nx;
      if (k + 1 < count) {
        nx = fetch<XFER>(i2);
        if (k + 2 < count) i2 = list[k + 2];
      }
      const uint32_t i = cur.i;
      const uint32_t cls = cur.cls;
      const bool linked = cls & C_LINKED;
      const uint32_t b = cur.b;
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
        r = XFER ? transfer(cur) : account(i, cls);
      }
      if (r != TB_CT_OK && chain >= 0 && !broken) {
        broken = true;
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
    }
  }
};
