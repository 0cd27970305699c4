// cps.h — the long components of a component-walked window, decided as a fixed point by one wave
// each (round 6).
//
// cpw.h walks each component of W with one thread: the reference loop (walker.h) in window order, one
// event per step. A step is a chain of dependent reads plus a few hundred instructions issued by one
// lane (~1-1.5 us), so the walk lasts as long as the window's longest component (cfg4: ~320 events,
// ~0.5 ms) long after the other ~140K walkers have finished. Here every component longer than
// `cps_min` events (and at most CPS_NMAX) gets a whole wave, and k_cc_walk skips it.
//
// In a component-walked window an event's outcome reads only (cpw.h):
//   - whether an earlier event of the window with the same id committed it (the exists checks,
//     state_machine.zig:1490-1507 create, :1629-1654 post/void),
//   - for a post/void of a pending transfer created in the window: that creation's commit
//     (:1616-1624), and the pending transfer's status after the earlier post/voids (:1658-1670),
//   - its chain: an event runs iff no earlier member of its chain failed (:1236-1300).
// Earlier event j is VISIBLE to event i iff j ran and committed, and j's chain (if any) completed
// without a failure or i is in that chain (a rolled-back chain's commits are undone when it breaks,
// cache_map.zig:254-301). So every outcome is a function of strictly earlier outcomes:
//   r_i = decide_i(r_j, chain outcomes : j < i),
// a triangular system whose unique solution is the sequential execution. Passes in which every event
// re-decides from the current values reach it in at most (longest dependency path + 1) passes (cfg4:
// 10-22 levels in components of 150-320 events), and a pass that changes nothing proves it. Per pass
// the wave re-decides every event from LDS alone: each id / pending-id key's touchers are sorted once
// per component, and a post/void's checks against its pending transfer (pv_against and the expiry
// bits) are cached per creator. Then the side effects the walker leaves (walker.h: code, C_RANOK,
// ins = 2, posting records, amounts and slots, statuses, the pulse_next ops) are written once, in
// parallel. At most one earlier event can be visible with a given id (a second commit would have
// failed its exists check against the first) and at most one visible post/void of a pending transfer
// can have succeeded (a second finds it posted or voided), so "the earliest visible one" is "the one".
#pragma once
#include "cpw.h"

#define CPS_NMAX 512u   // events per wave-decided component (longer ones stay with k_cc_walk)
#define CPS_SMALL 64u   // the small class: LDS for 64 events per wave, so many waves per CU
#define CPS_N16 0xFFFFu
#define CPS_STORED 0xFFFEu  // cpc: the pending transfer was stored before the window
#define CPS_COM 0x100u      // st: the event committed its record (ok, or the expired-post quirk)
#define CPS_EXPB 1u         // cfl: the pending transfer expired at a pulse before the event's batch
#define CPS_EXPQ 2u         // cfl: expires_at <= the event's timestamp (posting inserted, then expired)
#define CPS_VALL 1u         // vs: committed, ran, and its chain (if any) completed: visible to every later event
#define CPS_VRAN 2u         // vs: committed and ran: visible to the later members of its own chain
#define CPS_VOK 4u          // vs: its result is ok
#define CPS_LDS_PER_EVENT 80u
#ifndef CPS_PROF
#define CPS_PROF 0  // 1: per-phase wall-clock sums of the large class in dbg[0], dbg[5..7] (replaces walk stats)
#endif

// A wave's LDS, per list position k of its component (carved from dynamic LDS for nmax events).
struct CpsShared {
  unsigned long long* tch;  // [2 nmax] touches: key << 32 | list position << 1 | role (1: pending id)
  uint32_t* wi;     // window position
  uint32_t* cls;
  uint32_t* k1;     // id key (window key-map entry; NONE32: not decided dynamically)
  uint32_t* k2;     // post/void: pending-id key
  uint32_t* pslot;  // p_tslot: the pending transfer's slot when stored before the window
  uint32_t* idts;   // id_tslot: a stored transfer with this id
  uint32_t* fpos;   // at a chain's first list position: its first member that failed
  uint32_t* vs;     // per pass: CPS_VALL | CPS_VRAN | CPS_VOK | cs << 16 (cps_vis)
  uint32_t *dr, *cr;  // account slots (k_ct_prep's row): a post/void of an in-window pending transfer takes its creator's
  uint16_t* b;      // batch
  uint16_t* cs;     // first list position of the event's chain (CPS_N16: not chained)
  uint16_t *tp1, *tp2;  // sorted touch positions of k1 / k2
  uint16_t* cpc;    // creator whose checks cag / cfl hold (CPS_STORED, CPS_N16: none yet)
  uint16_t* st;     // result | CPS_COM
  uint8_t* rs;      // static result (0xFF: decided by the passes)
  uint8_t* bal;     // create: ct_balances with the zero balances of a component window
  uint8_t* cag;     // post/void: pv_against's result against cpc (0xFF: CONT)
  uint8_t* cfl;     // post/void: CPS_EXPB | CPS_EXPQ against cpc
  uint8_t* pst0;    // post/void of a stored pending transfer: its status before the window
  uint32_t* cnt;    // touches counted
};

__device__ inline CpsShared cps_carve(unsigned long long* base, uint32_t nmax) {
  CpsShared L;
  L.tch = base;
  uint32_t* p32 = reinterpret_cast<uint32_t*>(base + 2 * nmax);
  L.wi = p32;
  L.cls = p32 + nmax;
  L.k1 = p32 + 2 * nmax;
  L.k2 = p32 + 3 * nmax;
  L.pslot = p32 + 4 * nmax;
  L.idts = p32 + 5 * nmax;
  L.fpos = p32 + 6 * nmax;
  L.vs = p32 + 7 * nmax;
  L.dr = p32 + 8 * nmax;
  L.cr = p32 + 9 * nmax;
  uint16_t* p16 = reinterpret_cast<uint16_t*>(p32 + 10 * nmax);
  L.b = p16;
  L.cs = p16 + nmax;
  L.tp1 = p16 + 2 * nmax;
  L.tp2 = p16 + 3 * nmax;
  L.cpc = p16 + 4 * nmax;
  L.st = p16 + 5 * nmax;
  uint8_t* p8 = reinterpret_cast<uint8_t*>(p16 + 6 * nmax);
  L.rs = p8;
  L.bal = p8 + nmax;
  L.cag = p8 + 2 * nmax;
  L.cfl = p8 + 3 * nmax;
  L.pst0 = p8 + 4 * nmax;
  L.cnt = reinterpret_cast<uint32_t*>(p8 + 5 * nmax + 3 - ((5 * nmax + 3) & 3));  // (5 nmax is a multiple of 4 for nmax % 4 == 0)
  return L;  // 16 + 40 + 12 + 5 <= CPS_LDS_PER_EVENT bytes per event
}

// Event j's visibility word from its result and its chain's first failure.
__device__ inline uint32_t cps_vis(const CpsShared& L, uint32_t j) {
  const uint32_t v = L.st[j], c = L.cs[j];
  const uint32_t fp = c == CPS_N16 ? NONE32 : L.fpos[c];
  uint32_t w = c << 16;
  if ((v & 0xFFu) == TB_CT_OK) w |= CPS_VOK;
  if ((v & CPS_COM) && !(fp < j)) w |= fp == NONE32 ? (CPS_VALL | CPS_VRAN) : CPS_VRAN;
  return w;
}

// The earliest earlier toucher of `key` (sorted touch position tp of an event in chain ck) in `role`
// that is visible to it (and succeeded, `need_ok`): walks the key's run of touches back from tp.
__device__ inline uint32_t cps_find(const CpsShared& L, uint32_t ck, uint32_t key, uint32_t tp, uint32_t role,
                                    bool need_ok) {
  uint32_t found = CPS_N16;
  for (int32_t p = (int32_t)tp - 1; p >= 0; p--) {
    const unsigned long long e = L.tch[p];
    if ((uint32_t)(e >> 32) != key) break;
    if ((e & 1u) != role) continue;
    const uint32_t j = ((uint32_t)e >> 1) & 0x7FFFu;
    const uint32_t v = L.vs[j];
    const bool vis = (v & CPS_VALL) || ((v & CPS_VRAN) && (v >> 16) == ck);
    if (!vis || (need_ok && !(v & CPS_VOK))) continue;
    found = j;
  }
  return found;
}

__device__ inline tb_transfer_t cps_event(const uint8_t* ev, const WinDesc& w, const CpsShared& L, uint32_t k) {
  tb_transfer_t t = reinterpret_cast<const tb_transfer_t*>(ev)[L.wi[k]];
  t.timestamp = win_ts(w, L.b[k], L.wi[k]);
  return t;
}

// Post/void k's pending transfer record as the walker reads it: the stored record, or creator pc's
// input row stamped with its timestamp (walker.h post_or_void, component mode).
__device__ inline tb_transfer_t cps_pending(const Dev& d, const uint8_t* ev, const WinDesc& w, const CpsShared& L,
                                            uint32_t k, uint32_t pc) {
  if (pc == CPS_STORED) return d.xr[L.pslot[k]];
  return cps_event(ev, w, L, pc);
}

// pv_against and the expiry bits of post/void k against creator pc, cached.
__device__ inline void cps_against(const Dev& d, const uint8_t* ev, const WinDesc& w, CpsShared& L, uint32_t k,
                                   uint32_t pc) {
  if (L.cpc[k] == pc) return;
  const tb_transfer_t t = cps_event(ev, w, L, k);
  const tb_transfer_t p = cps_pending(d, ev, w, L, k, pc);
  u128 amount;
  const uint32_t r = pv_against(t, p, &amount);
  uint8_t f = 0;
  if (xw_expired_before(w, p, L.b[k])) f |= CPS_EXPB;
  if (p.timeout > 0 && expires_at_of(p) <= t.timestamp) f |= CPS_EXPQ;
  L.cag[k] = r == CONT ? (uint8_t)0xFF : (uint8_t)r;
  L.cfl[k] = f;
  L.cpc[k] = (uint16_t)pc;
}

// The creator of post/void k visible to it (CPS_STORED: stored before the window; CPS_N16: none).
__device__ inline uint32_t cps_creator(const CpsShared& L, uint32_t k) {
  if (L.pslot[k] != NONE32) return CPS_STORED;
  if (L.k2[k] == NONE32) return CPS_N16;
  return cps_find(L, L.cs[k], L.k2[k], L.tp2[k], 0, false);
}

// The record event c committed (walker.h walk_record): a create's input row, or a post/void's
// posting record (pv_record over its pending transfer; only the exists checks read it, which
// compare no timestamp).
__device__ inline tb_transfer_t cps_record(const Dev& d, const uint8_t* ev, const WinDesc& w, const CpsShared& L,
                                           uint32_t c) {
  const tb_transfer_t t = cps_event(ev, w, L, c);
  if (!(L.cls[c] & C_POSTVOID)) return reinterpret_cast<const tb_transfer_t*>(ev)[L.wi[c]];
  const uint32_t pc = cps_creator(L, c);
  if (pc == CPS_N16) return t;  // (not reached: a committed post/void found its pending transfer)
  const tb_transfer_t p = cps_pending(d, ev, w, L, c, pc);
  u128 amount = 0;
  (void)pv_against(t, p, &amount);
  return pv_record(t, p, amount);
}

// One dynamic event's outcome from the current values (walker.h transfer / post_or_void, from the
// exists check on): result | CPS_COM.
__device__ inline uint32_t cps_eval(const Dev& d, const uint8_t* ev, const WinDesc& w, CpsShared& L, uint32_t k) {
  const uint32_t cls = L.cls[k];
  const bool alone = cls & C_IDALONE;
  if (!(cls & C_POSTVOID)) {
    if (!alone && L.k1[k] != NONE32) {
      const uint32_t c = cps_find(L, L.cs[k], L.k1[k], L.tp1[k], 0, false);
      if (c != CPS_N16) return ct_exists(cps_event(ev, w, L, k), cps_record(d, ev, w, L, c));
    }
    const uint32_t r = L.bal[k];
    return r == TB_CT_OK ? (r | CPS_COM) : r;
  }
  const uint32_t pc = cps_creator(L, k);
  if (pc == CPS_N16) return TB_CT_PENDING_TRANSFER_NOT_FOUND;
  cps_against(d, ev, w, L, k, pc);
  if (L.cag[k] != 0xFF) return L.cag[k];
  if (L.idts[k] != NONE32 || !alone) {
    uint32_t c = CPS_N16;
    if (L.idts[k] == NONE32 && L.k1[k] != NONE32) c = cps_find(L, L.cs[k], L.k1[k], L.tp1[k], 0, false);
    if (L.idts[k] != NONE32 || c != CPS_N16) {
      const tb_transfer_t t = cps_event(ev, w, L, k);
      const tb_transfer_t p = cps_pending(d, ev, w, L, k, pc);
      return pv_exists(t, L.idts[k] != NONE32 ? d.xr[L.idts[k]] : cps_record(d, ev, w, L, c), p);
    }
  }
  uint8_t pst = pc == CPS_STORED ? L.pst0[k] : (uint8_t)TB_PENDING_PENDING;
  const uint32_t sc = L.k2[k] == NONE32 ? CPS_N16 : cps_find(L, L.cs[k], L.k2[k], L.tp2[k], 1, true);
  if (sc != CPS_N16) pst = (L.cls[sc] & C_POST) ? TB_PENDING_POSTED : TB_PENDING_VOIDED;
  if (pst == TB_PENDING_PENDING && (L.cfl[k] & CPS_EXPB)) pst = TB_PENDING_EXPIRED;
  const uint32_t r = pv_status(pst);
  if (r != CONT) return r;
  if (L.cfl[k] & CPS_EXPQ) return TB_CT_PENDING_TRANSFER_EXPIRED | CPS_COM;
  return TB_CT_OK | CPS_COM;
}

// Each chain's first failing member, then every event's visibility word.
template <uint32_t NT>
__device__ inline void cps_fpos(CpsShared& L, uint32_t n) {
  const uint32_t lane = threadIdx.x;
  for (uint32_t k = lane; k < n; k += NT)
    if (L.cs[k] == k) L.fpos[k] = NONE32;
  __syncthreads();
  for (uint32_t k = lane; k < n; k += NT)
    if (L.cs[k] != CPS_N16 && (L.st[k] & 0xFFu) != TB_CT_OK) atomicMin(&L.fpos[L.cs[k]], k);
  __syncthreads();
  for (uint32_t k = lane; k < n; k += NT) L.vs[k] = cps_vis(L, k);
  __syncthreads();
}

// Component rval[start .. start + n), one block of NT threads. Returns the passes it took.
template <uint32_t NT>
__device__ uint32_t cps_component(const Dev& d, const Scratch& s, const uint8_t* ev, const WinDesc& w, CpsShared& L,
                              uint32_t start, uint32_t n) {
  const uint32_t lane = threadIdx.x;
  uint64_t tp0 = CPS_PROF ? wall_clock64() : 0, tp1 = 0, tp2 = 0, tp3 = 0;
  // 1. the events' static inputs (walker.h fetch: the k_ct_prep row) and static results. Each lane
  // issues the loads of up to CPS_U of its events before using any (a component's setup is a few
  // dependent round trips, not one per event).
#define CPS_U 4
  // (grouped segments are in arbitrary order: the window positions first, sorted in LDS)
  uint32_t PW = 1;
  while (PW < n) PW <<= 1;
  for (uint32_t k = lane; k < PW; k += NT) L.wi[k] = k < n ? s.rval[start + k] : 0xFFFFFFFFu;
  __syncthreads();
  for (uint32_t size = 2; size <= PW; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t x = lane; x < PW / 2; x += NT) {
        const uint32_t lo = 2 * stride * (x / stride) + (x % stride), hi = lo + stride;
        const uint32_t A = L.wi[lo], B = L.wi[hi];
        if ((A > B) == ((lo & size) == 0)) {
          L.wi[lo] = B;
          L.wi[hi] = A;
        }
      }
      __syncthreads();
    }
  }
  for (uint32_t k0 = lane; k0 < n; k0 += NT * CPS_U) {
    uint32_t iv[CPS_U], cv[CPS_U];
    uint4 r0v[CPS_U], r1v[CPS_U];
#pragma unroll
    for (int u = 0; u < CPS_U; u++) {
      const uint32_t k = k0 + NT * u;
      iv[u] = k < n ? L.wi[k] : L.wi[0];
    }
#pragma unroll
    for (int u = 0; u < CPS_U; u++) {
      const uint32_t i = iv[u];
      cv[u] = s.cls[i];
      r0v[u] = s.wrow[2 * i];
      r1v[u] = s.wrow[2 * i + 1];
    }
#pragma unroll
    for (int u = 0; u < CPS_U; u++) {
      const uint32_t k = k0 + NT * u;
      if (k >= n) break;
      const uint32_t i = iv[u], cls = cv[u];
      const uint4 r0 = r0v[u], r1 = r1v[u];
      L.cls[k] = cls;
      L.b[k] = (uint16_t)r1.w;
      L.pslot[k] = r1.z;
      L.idts[k] = r0.y;
      L.dr[k] = r1.x;
      L.cr[k] = r1.y;
      L.cpc[k] = CPS_N16;
      const bool open = (cls & C_LINKED) && i == w.off[r1.w + 1] - 1;
      uint32_t rs = 0xFF;
      if (open) rs = TB_CT_LINKED_EVENT_CHAIN_OPEN;
      else if (cls & C_TSNZ) rs = TB_CT_TIMESTAMP_MUST_BE_ZERO;
      else if (cls & C_STATIC) rs = r0.x;
      L.k1[k] = NONE32;
      L.k2[k] = NONE32;
      if (rs == 0xFF && (cls & C_REACH)) {  // (the key-map entries exist for events that reach the exists check)
        L.k1[k] = r0.z;
        if (cls & C_POSTVOID) L.k2[k] = r0.w;
      }
      if (rs == 0xFF && !(cls & C_POSTVOID)) {
        // a create: k_ct_prep's code is its outcome unless an earlier event committed its id (the
        // stored-id exists check is static; else the zero-balance tail: ok or overflows_timeout)
        if (r0.y != NONE32)
          rs = r0.x;
        else
          L.bal[k] = (uint8_t)r0.x;
      }
      L.rs[k] = (uint8_t)rs;
    }
  }
  __syncthreads();
  // 2. chains in list order (walker.h run): k continues k-1's chain iff k-1 is linked and did not
  // close an open chain; a chain's members are consecutive window positions
  for (uint32_t k = lane; k < n; k += NT) {
    uint32_t c = CPS_N16;
    const bool linked = L.cls[k] & C_LINKED;
    bool cont = false;
    if (k > 0) {
      const uint32_t ip = L.wi[k - 1];
      cont = (L.cls[k - 1] & C_LINKED) && !(L.rs[k - 1] == TB_CT_LINKED_EVENT_CHAIN_OPEN && ip == w.off[L.b[k - 1] + 1] - 1);
    }
    if (linked || cont) {
      // the chain's first position: walk back over continuing members (chains are short; a chain
      // never spans a batch)
      uint32_t f = k;
      while (f > 0) {
        const uint32_t q = f - 1;
        const bool qcont = (L.cls[q] & C_LINKED) &&
                           !(L.rs[q] == TB_CT_LINKED_EVENT_CHAIN_OPEN && L.wi[q] == w.off[L.b[q] + 1] - 1);
        if (!qcont) break;
        f = q;
      }
      c = f;
    }
    L.cs[k] = (uint16_t)c;
  }
  // 3. the key touches, sorted by (key, list position): one wave's bitonic sort in LDS
  // (touch order before the sort is immaterial: positions from an LDS counter)
  if (lane == 0) *L.cnt = 0;
  __syncthreads();
  for (uint32_t k = lane; k < n; k += NT) {
    const bool a = L.k1[k] != NONE32, b2 = L.k2[k] != NONE32;
    if (!a && !b2) continue;
    uint32_t o = atomicAdd(L.cnt, (a ? 1u : 0u) + (b2 ? 1u : 0u));
    if (a) L.tch[o++] = ((unsigned long long)L.k1[k] << 32) | (k << 1);
    if (b2) L.tch[o] = ((unsigned long long)L.k2[k] << 32) | (k << 1) | 1u;
  }
  __syncthreads();
  const uint32_t nt = *L.cnt;
  uint32_t P = 2;
  while (P < nt) P <<= 1;
  for (uint32_t q = nt + lane; q < P; q += NT) L.tch[q] = ~0ull;
  __syncthreads();
  for (uint32_t size = 2; size <= P; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t x = lane; x < P / 2; x += NT) {
        const uint32_t lo = 2 * stride * (x / stride) + (x % stride), hi = lo + stride;
        const unsigned long long A = L.tch[lo], B = L.tch[hi];
        const bool up = (lo & size) == 0;
        if ((A > B) == up) {
          L.tch[lo] = B;
          L.tch[hi] = A;
        }
      }
      __syncthreads();
    }
  }
  for (uint32_t q = lane; q < nt; q += NT) {
    const unsigned long long e = L.tch[q];
    const uint32_t k = ((uint32_t)e >> 1) & 0x7FFFu;
    if (e & 1u)
      L.tp2[k] = (uint16_t)q;
    else
      L.tp1[k] = (uint16_t)q;
  }
  __syncthreads();
  // 3b. the checks that read records, once: a create's balance-free checks (or its exists check
  // against a stored transfer with its id); a post/void's checks against the pending transfer its
  // key's first creator in the component would be (cached per creator: a later pass rarely finds
  // another), and a stored pending transfer's status before the window. The record loads of a
  // lane's events go out together.
  for (uint32_t k0 = lane; k0 < n; k0 += NT * 2) {
    tb_transfer_t tv[2], pv2[2];
    uint32_t c0v[2];
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const uint32_t k = k0 + NT * u;
      c0v[u] = CPS_N16;
      if (k >= n || L.rs[k] != 0xFF || !(L.cls[k] & C_POSTVOID)) continue;  // (creates: step 1)
      tv[u] = cps_event(ev, w, L, k);
      if (L.pslot[k] != NONE32) {
        c0v[u] = CPS_STORED;
      } else if (L.k2[k] != NONE32) {
        for (int32_t p = (int32_t)L.tp2[k] - 1; p >= 0; p--) {  // the key's earliest creator before k
          const unsigned long long e = L.tch[p];
          if ((uint32_t)(e >> 32) != L.k2[k]) break;
          if (!(e & 1u)) c0v[u] = ((uint32_t)e >> 1) & 0x7FFFu;
        }
      }
      if (c0v[u] != CPS_N16) pv2[u] = cps_pending(d, ev, w, L, k, c0v[u]);
    }
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const uint32_t k = k0 + NT * u;
      if (k >= n || L.rs[k] != 0xFF || !(L.cls[k] & C_POSTVOID)) continue;
      const tb_transfer_t& t = tv[u];
      const uint32_t c0 = c0v[u];
      if (c0 == CPS_STORED) L.pst0[k] = d.xstatus[L.pslot[k]];
      if (c0 == CPS_N16) continue;
      const tb_transfer_t& p = pv2[u];
      u128 amount;
      const uint32_t r = pv_against(t, p, &amount);
      uint8_t f = 0;
      if (xw_expired_before(w, p, L.b[k])) f |= CPS_EXPB;
      if (p.timeout > 0 && expires_at_of(p) <= t.timestamp) f |= CPS_EXPQ;
      L.cag[k] = r == CONT ? (uint8_t)0xFF : (uint8_t)r;
      L.cfl[k] = f;
      L.cpc[k] = (uint16_t)c0;
    }
  }
  for (uint32_t k = lane; k < n; k += NT)
    L.st[k] = L.rs[k] == 0xFF ? (uint16_t)(TB_CT_OK | CPS_COM) : (uint16_t)L.rs[k];  // (optimistic start)
  __syncthreads();
  cps_fpos<NT>(L, n);
  if (CPS_PROF) tp1 = wall_clock64();
  // 4. passes until nothing changes (bounded: the triangular system settles position k by pass 2k+2)
  uint32_t pass = 0;
  for (; pass < 2 * n + 4; pass++) {
    bool changed = false;
    for (uint32_t k = lane; k < n; k += NT) {
      if (L.rs[k] != 0xFF) continue;
      const uint16_t v = (uint16_t)cps_eval(d, ev, w, L, k);
      if (v != L.st[k]) {
        L.st[k] = v;
        if (L.cs[k] == CPS_N16) L.vs[k] = cps_vis(L, k);  // (chained: after the pass, with its chain)
        changed = true;
      }
    }
    __syncthreads();
    cps_fpos<NT>(L, n);
    if (!__syncthreads_or(changed ? 1 : 0)) break;
  }
  if (pass == 2 * n + 4) {  // (not reached: position k settles by pass 2k + 2) fail the window loudly
    if (lane == 0) atomicOr(&d.g->window_error, 4u);
    return pass;
  }
  if (CPS_PROF) tp2 = wall_clock64();
  // 5. the walker's side effects
  for (uint32_t k = lane; k < n; k += NT) {
    const uint32_t i = L.wi[k];
    const uint32_t v = L.st[k], r = v & 0xFFu, cls = L.cls[k];
    const uint32_t c = L.cs[k];
    const uint32_t fp = c == CPS_N16 ? NONE32 : L.fpos[c];
    const bool ran = !(fp < k);
    uint32_t code, add = 0;
    if (L.rs[k] == TB_CT_LINKED_EVENT_CHAIN_OPEN) {
      code = r;
    } else if (!ran) {
      code = TB_CT_LINKED_EVENT_FAILED;
    } else if (r != TB_CT_OK) {
      code = r;
    } else if (fp != NONE32) {
      code = TB_CT_LINKED_EVENT_FAILED;
      add |= C_RANOK;  // ran ok, then rolled back with its chain: its pulse_next op stands (k_pn)
    } else {
      code = TB_CT_OK;
    }
    const bool kept = (v & CPS_COM) && ran && fp == NONE32;  // its commit survives
    if (kept) s.ins[i] = 2;
    const bool ranok = ran && r == TB_CT_OK && L.rs[k] == 0xFF;
    if (!(cls & C_POSTVOID)) {
      if (ranok && (reinterpret_cast<const tb_transfer_t*>(ev)[i].flags & TB_TRANSFER_PENDING))
        s.bstatus[i] = TB_PENDING_PENDING;
    } else if ((v & CPS_COM) && ran) {
      const uint32_t pc = cps_creator(L, k);
      const tb_transfer_t t = cps_event(ev, w, L, k);
      const tb_transfer_t p = cps_pending(d, ev, w, L, k, pc);
      u128 amount = 0;
      (void)pv_against(t, p, &amount);
      if (kept) s.t2[i] = pv_record(t, p, amount);
      if (r == TB_CT_OK && pc != CPS_STORED && p.timeout > 0) {
        // (walker.h post_or_void: the expires_at removal and pulse_next reset candidate for k_pn)
        const uint64_t x = expires_at_of(p);
        s.pnv[i] = x;
        s.pn_src[i] = L.wi[pc];
        add |= C_PNOP;
        if (x <= d.g->pulse_next && !(__hip_atomic_load(&d.g->win_flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 8u))
          atomicOr(&d.g->win_flags, 8u);
      }
      if (kept && r == TB_CT_OK) {
        if (pc != CPS_STORED) {
          s.dr_slot[i] = L.dr[pc];
          s.cr_slot[i] = L.cr[pc];
        }
        s.pamt[i] = U(p.amount);
        s.amt[i] = amount;
      }
    }
    s.code[i] = code;
    if (add) s.cls[i] = cls | add;
  }
  __syncthreads();
  // the statuses of the pending transfers the kept post/voids posted or voided (after the creations'
  // PENDING above: one writer per pending transfer)
  for (uint32_t k = lane; k < n; k += NT) {
    const uint32_t v = L.st[k], c = L.cs[k];
    if (!(L.cls[k] & C_POSTVOID) || v != (TB_CT_OK | CPS_COM)) continue;
    if (c != CPS_N16 && L.fpos[c] != NONE32) continue;
    const uint8_t stv = (L.cls[k] & C_POST) ? TB_PENDING_POSTED : TB_PENDING_VOIDED;
    const uint32_t pc = cps_creator(L, k);
    if (pc == CPS_STORED)
      d.xstatus[L.pslot[k]] = stv;
    else
      s.bstatus[L.wi[pc]] = stv;
  }
  __syncthreads();
  if (CPS_PROF && lane == 0 && n > CPS_SMALL) {
    tp3 = wall_clock64();
    atomicAdd((unsigned long long*)&d.g->dbg[0], (unsigned long long)(tp1 - tp0));
    atomicAdd((unsigned long long*)&d.g->dbg[5], (unsigned long long)(tp2 - tp1));
    atomicAdd((unsigned long long*)&d.g->dbg[6], (unsigned long long)(tp3 - tp2));
    atomicAdd((unsigned long long*)&d.g->dbg[7], (unsigned long long)n);
  }
  return pass + 1;
}

// The components of more than cps_min (and at most CPS_NMAX) events, listed for k_cc_solve in two
// classes: up to CPS_SMALL events from the bottom of rkey_in / rval_in (start / length), longer ones
// from the top (index E - 1 - x). Those are the component sort's inputs, free once it ran. One
// 64-bit counter add per block.
__global__ void __launch_bounds__(1024) k_cps_list(Dev d, Scratch s, uint32_t E, uint32_t cps_min) {
  __shared__ uint32_t lds[1024 / 64];
  __shared__ unsigned long long base;
  if (!cpw_active(d.g)) return;
  const uint32_t ncc = d.g->cc_count;
  if (blockIdx.x * blockDim.x >= ncc) return;  // (uniform per block)
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t start = 0, len = 0;
  if (j < ncc) {
    start = s.cc_list[j];
    len = s.light[j];  // (grouped: k_cc_place)
  }
  // (every length in (cps_min, CPS_NMAX] in exactly one class: k_cc_walk takes the rest)
  const bool small = len > cps_min && len <= CPS_SMALL, large = len > cps_min && len > CPS_SMALL && len <= CPS_NMAX;
  uint32_t tot;
  // (counts < 2^16 per block: both classes in one scan)
  const uint32_t r = block_excl<1024 / 64>((small ? 1u : 0u) | (large ? 1u << 16 : 0u), lds, &tot);
  if (tot == 0) return;
  if (threadIdx.x == 0)
    base = atomicAdd((unsigned long long*)&d.g->cps_lists,
                     (unsigned long long)(tot & 0xFFFFu) | ((unsigned long long)(tot >> 16) << 32));
  __syncthreads();
  if (small) {
    const uint32_t x = (uint32_t)base + (r & 0xFFFFu);
    s.rkey_in[x] = start;
    s.rval_in[x] = len;
  } else if (large) {
    const uint32_t x = E - 1 - ((uint32_t)(base >> 32) + (r >> 16));
    s.rkey_in[x] = start;
    s.rval_in[x] = len;
  }
}

// One class of the listed components, one block of NT threads each (blocks stride over the list): the
// small class one wave per component, the large class four; dynamic LDS of
// nmax * CPS_LDS_PER_EVENT + 16 bytes.
template <uint32_t NT>
__global__ void __launch_bounds__(NT) k_cc_solve(Dev d, Scratch s, const uint8_t* ev, WinDesc w, uint32_t E,
                                                 uint32_t large) {
  extern __shared__ unsigned long long cps_smem[];
  if (!cpw_active(d.g)) return;
  CpsShared L = cps_carve(cps_smem, large ? CPS_NMAX : CPS_SMALL);
  const unsigned long long lists = d.g->cps_lists;
  const uint32_t n_list = large ? (uint32_t)(lists >> 32) : (uint32_t)lists;
  // statistics (tbg_debug_counters, component windows): [1] wave-decided components, [2] their
  // events, [3] their passes, [4] the most passes one took; one add per block that decided any
  uint32_t n_comp = 0, n_ev = 0, n_pass = 0, mx_pass = 0;
  for (uint32_t x = blockIdx.x; x < n_list; x += gridDim.x) {
    const uint32_t at = large ? E - 1 - x : x;
    const uint32_t n = s.rval_in[at];
    const uint32_t np = cps_component<NT>(d, s, ev, w, L, s.rkey_in[at], n);
    n_comp++;
    n_ev += n;
    n_pass += np;
    mx_pass = np > mx_pass ? np : mx_pass;
  }
  if (threadIdx.x == 0 && n_comp) {
    Globals* g = d.g;
    atomicAdd((unsigned long long*)&g->dbg[1], (unsigned long long)n_comp);
    atomicAdd((unsigned long long*)&g->dbg[2], (unsigned long long)n_ev);
    atomicAdd((unsigned long long*)&g->dbg[3], (unsigned long long)n_pass);
    atomicMax((unsigned long long*)&g->dbg[4], (unsigned long long)mx_pass);
  }
}
