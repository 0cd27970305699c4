// relax.h — exact resolution of balance-limit windows by windowed relaxation (default resolver).
//
// Same class, inputs and outputs as the wait-based walkers of resolver.h (sorted per-account entry
// lists from k_res_keys/k_res_segs; published checks in st[]; per-account effect sums in
// RState::d), but no walker ever waits on another. The sequential semantics (state_machine.zig:
// 1220-1306 calling create_transfer's limit checks :1567-1570) are the unique solution s of
//
//   s[e] = AND over the sides of e that check: amount(e) <= A_side(e)
//   A_x(e) = A_x(start) + sum of effects on x of the committed events before e  (resolver.h header)
//
// because s[e] reads only events before e. The kernel iterates towards that solution:
//  * every hot account is walked by one walker (a whole wave for a heavy one, 64 entries per step
//    with the exclusive-scan-and-correct scheme of resolver.h; a lane for a light one), computing
//    its checks from the other sides' latest published checks (an unpublished check reads as pass);
//  * a published check that changes marks the other side's walker dirty at that entry (atomicMin
//    of the entry index), and records the event position (atomicMin into fc);
//  * walkers walk only entries of events in [clo, chi), chi = clo + chunk, from their first dirty
//    or never-walked entry, with the available balance stored after every entry (racc);
//  * after a grid barrier every wave reads f = first changed position: nothing before f changed in
//    that iteration, so (every status before f being computed from unchanged earlier statuses) the
//    prefix before f is the unique solution and final: clo = f, or chi when nothing changed.
// The position at f is final after the next iteration (its inputs are final), so clo strictly
// advances at least every other iteration; an iteration cap and bounded barrier spins fall back to
// the sequential walker (res_error), as in resolver.h.
//
// k_res_sum then publishes the final checks as st bits, adds each committed entry's amount into its account's four balance fields
// (segmented wave sums + one u128 atomic per segment per wave), and k_res_apply / k_res_final of
// resolver.h finish the window unchanged.
#pragma once
#include "resolver.h"

#define RELAX_THREADS 512
#ifndef RELAX_PROF
#define RELAX_PROF 0  // 1: per-part clock64() sums of the heavy walkers into Globals::dbg (tbg_debug_counters)
#endif
struct RProf {
  uint64_t steps, rounds, t_wait, t_scan, t_corr, t_pub, t_setup;
};
#define RP_T0() const uint64_t _rp0 = RELAX_PROF ? clock64() : 0
#define RP_ADD(f, t0) \
  do {                \
    if (RELAX_PROF) prof.f += clock64() - (t0); \
  } while (0)
#define RELAX_MAX_ITERS 200000u

__device__ inline uint32_t st_pass_bit(uint32_t side) { return side ? ST_CR_PASS : ST_DR_PASS; }

// Grid barrier: per-group arrival counters (group = blockIdx % 8), the last arriver of a group bumps
// the top counter, every block polls the top counter. Counters are monotonic within one launch
// (zeroed by k_res_keys). Returns false if the spin outlived RES_TIMEOUT_TICKS.
__device__ inline bool relax_barrier(Globals* g, uint32_t it) {
  __shared__ uint32_t ok_sh;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t grp = blockIdx.x & 7u;
    const uint32_t nb = gridDim.x;
    const uint32_t in_grp = nb / 8u + ((grp < nb % 8u) ? 1u : 0u);
    const uint32_t ngrp = nb < 8u ? nb : 8u;
    __threadfence();
    const uint32_t old = __hip_atomic_fetch_add(&g->res_bar[grp], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1u == in_grp * (it + 1u))
      __hip_atomic_fetch_add(&g->res_bar_top, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t target = ngrp * (it + 1u);
    const uint64_t t0 = wall_clock64();
    uint32_t ok = 1;
    while (__hip_atomic_load(&g->res_bar_top, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (wall_clock64() - t0 > RES_TIMEOUT_TICKS ||
          __hip_atomic_load(&g->res_error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        __hip_atomic_fetch_or(&g->res_error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __threadfence();
    ok_sh = ok;
  }
  __syncthreads();
  return ok_sh != 0;
}

// Per-entry status words (no walker reads another walker's state through an event index):
//   rown[k] = this entry's own last published check: 0 fail, 1 pass, 2 not yet published
//   roth[k] = the other side's last published check of this entry's event: 0 fail, 1 pass (initially)
// written by that other side's walker through kidx. Every cross-walker word is accessed with
// relaxed agent-scope atomics (sc1: coherent across the XCDs' L2s) and without fences; ordering
// comes from the grid barrier: a change made in iteration `it` marks the reader dirty in
// dirty[it & 1], consumed only after the barrier, so the reader's re-walk sees the new word.
__device__ inline uint32_t at_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Publishes entry k's own check (rown; k_res_sum turns the final values into st bits) and, for a
// semantic change (a reader assuming the old value would be wrong; unpublished reads as pass), the
// other side's roth word and dirty mark. `link` = (other side's entry, its rank), precomputed by
// k_res_links so that no store here waits on a load. Returns true on a semantic change.
__device__ inline bool relax_publish(const Scratch& s, uint32_t k, uint2 link, uint32_t own, bool pass, uint32_t it) {
  s.rown[k] = pass ? 1u : 0u;
  if ((own != 0u) == pass) return false;
  if (link.x != NONE32) {
    __hip_atomic_store(&s.roth[link.x], pass ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_min(&s.rstate[link.y].dirty[it & 1u], link.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return true;
}

// A walker's view of one rank, kept in registers across iterations: hwm = first never-walked entry
// and hwm_e its event (NONE32 at the end). A dirty mark always names an entry of an event walked in
// the previous iteration (< that chi <= this chi), so a marked rank always walks.
struct RSlot {
  uint32_t r, start, end, hwm, hwm_e;
};

__device__ inline RSlot relax_slot(const Scratch& s, uint32_t r) {
  RSlot q;
  q.r = r;
  q.start = s.rstate[r].start;
  q.end = s.rstate[r].end;
  q.hwm = q.start;
  q.hwm_e = s.rmeta[q.start] & RM_EVENT;
  return q;
}

// Consumes rank r's dirty mark of the previous iteration (NONE32 if none).
__device__ inline uint32_t relax_take_mark(const Scratch& s, uint32_t r, uint32_t it, uint32_t seen) {
  if (seen == NONE32) return NONE32;
  return __hip_atomic_exchange(&s.rstate[r].dirty[(it + 1u) & 1u], NONE32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#define RB 4  // steps (64 entries each) per batch of loads in the heavy walker
#define RSLOTS 4  // ranks per heavy wave / light lane kept in registers (more go through memory)

struct RBatch {
  uint32_t meta[RB], oth[RB], own[RB];
  uint2 link[RB];
  u128 amt[RB];
};

__device__ inline void relax_load(const Scratch& s, uint32_t k, uint32_t end, int lane, RBatch& b) {
  // branch-free (indices clamped into the rank's list, end > 0): the loads stay in flight until a
  // step uses them; lanes past the end are masked at use (relax_step)
#pragma unroll
  for (int j = 0; j < RB; j++) {
    const uint32_t kk = min(k + 64u * j + (uint32_t)lane, end - 1u);
    b.meta[j] = s.rmeta[kk];
    b.link[j] = s.rlink[kk];
    b.amt[j] = s.ramt[kk];
    b.oth[j] = at_load(&s.roth[kk]);
    b.own[j] = s.rown[kk];
  }
}

// Wave primitives for the heavy walker's step (DPP row shifts/broadcasts and v_readlane: no LDS
// round trips, unlike __shfl's ds_bpermute).
template <int CTRL, int ROW_MASK>
__device__ inline int64_t dpp_i64(int64_t v) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(uint64_t)v, CTRL, ROW_MASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)((uint64_t)v >> 32), CTRL, ROW_MASK, 0xf, false);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
// Inclusive wave64 scan: row_shr 1/2/4/8 within rows of 16, then row_bcast 15 / 31 across rows.
__device__ inline int64_t wave_incl_scan_i64(int64_t x) {
  x += dpp_i64<0x111, 0xf>(x);
  x += dpp_i64<0x112, 0xf>(x);
  x += dpp_i64<0x114, 0xf>(x);
  x += dpp_i64<0x118, 0xf>(x);
  x += dpp_i64<0x142, 0xa>(x);
  x += dpp_i64<0x143, 0xc>(x);
  return x;
}
__device__ inline int64_t readlane_i64(int64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ inline __int128 readlane_i128(__int128 v, int l) {
  const uint64_t lo = (uint64_t)readlane_i64((int64_t)(uint64_t)v, l);
  const uint64_t hi = (uint64_t)readlane_i64((int64_t)(uint64_t)((unsigned __int128)v >> 64), l);
  return (__int128)(((unsigned __int128)hi << 64) | lo);
}

// RB steps of a heavy walker over the loaded batch `cur` (entries k.., 64 per step).
template <bool SMALL>
__device__ inline void relax_batch(const Scratch& s, const RBatch& cur, uint32_t chi, uint32_t it, uint32_t end, int lane,
                                   uint32_t& k, __int128& A, uint32_t& first_change, bool& done, uint32_t& stop_e,
                                   RProf& prof) {
#pragma unroll
  for (int j = 0; j < RB; j++) {
    if (done) break;
    uint64_t t0 = RELAX_PROF ? clock64() : 0;
    const uint32_t meta = cur.meta[j];
    const uint32_t e = meta & RM_EVENT;
    const bool act = e < chi && k + (uint32_t)lane < end;
    const unsigned long long am = __ballot(act);
    const uint32_t n = (uint32_t)__popcll(am);  // a prefix: entries are sorted by event
    if (n < 64) stop_e = (uint32_t)__builtin_amdgcn_readlane((int)e, (int)n);  // the first entry not walked
    if (n == 0) {
      done = true;
      break;
    }
    RP_ADD(t_wait, t0);
    if (RELAX_PROF) { prof.steps++; t0 = clock64(); }
    const bool check = act && (meta & RM_CHECK);
    const bool opass = !(meta & RM_WAIT) || cur.oth[j] != 0u;
    bool ok = act && opass;
    const uint32_t kk = k + (uint32_t)lane;
    bool pass;
    __int128 after;  // available balance after this entry
    if (SMALL) {
      const int64_t amt = act ? (int64_t)(uint64_t)cur.amt[j] : 0;
      int64_t eff = 0;
      if (ok) eff = check ? -amt : ((meta & RM_ADD) ? amt : 0);
      int64_t pre = wave_incl_scan_i64(eff) - eff;
      RP_ADD(t_scan, t0);
      if (RELAX_PROF) t0 = clock64();
      int floor_lane = -1;
      for (;;) {
        const unsigned long long fm = __ballot(ok && check && lane > floor_lane && (__int128)amt > A + pre);
        if (!fm) break;
        if (RELAX_PROF) prof.rounds++;
        const int jl = __builtin_ctzll(fm);
        const int64_t aj = readlane_i64(amt, jl);
        if (lane > jl) pre += aj;
        if (lane == jl) {
          ok = false;
          eff = 0;
        }
        floor_lane = jl;
      }
      pass = (__int128)amt <= A + pre;
      after = A + (pre + eff);
      A += readlane_i64(pre + eff, (int)n - 1);
      RP_ADD(t_corr, t0);
      if (RELAX_PROF) t0 = clock64();
    } else {
      const __int128 amt = act ? (__int128)cur.amt[j] : (__int128)0;
      __int128 eff = 0;
      if (ok) eff = check ? -amt : ((meta & RM_ADD) ? amt : (__int128)0);
      __int128 x = eff;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const __int128 y = i128_shfl_up(x, o);
        if (lane >= o) x += y;
      }
      __int128 P = x - eff + A;
      int floor_lane = -1;
      for (;;) {
        const unsigned long long fm = __ballot(ok && check && lane > floor_lane && amt > P);
        if (!fm) break;
        const int jl = __builtin_ctzll(fm);
        const __int128 aj = readlane_i128(amt, jl);
        if (lane > jl) P += aj;
        if (lane == jl) {
          ok = false;
          eff = 0;
        }
        floor_lane = jl;
      }
      pass = amt <= P;
      after = P + eff;
      A = readlane_i128(after, (int)n - 1);
    }
    if (check && cur.own[j] != (pass ? 1u : 0u) && relax_publish(s, kk, cur.link[j], cur.own[j], pass, it))
      first_change = min(first_change, e);
    if (act) s.racc[kk] = after;
    k += n;
    if (n < 64) done = true;
    RP_ADD(t_pub, t0);
  }
}

// Heavy walker: the wave walks slot q's entries from entry k (A = available balance before k) while
// their events are < chi, 64 per step, loads issued one batch (RB steps) ahead; updates q.hwm/hwm_e.
// SMALL: the window's amounts sum below 2^62, so every in-step prefix of effects fits an int64
// (available balance = A (i128) + prefix (i64)).
template <bool SMALL>
__device__ inline uint32_t relax_wave(const Scratch& s, RSlot& q, uint32_t k, uint32_t chi, uint32_t it, RProf& prof) {
  const int lane = threadIdx.x & 63;
  uint64_t tp = RELAX_PROF ? clock64() : 0;
  const uint32_t end = q.end;
  __int128 A = k == q.start ? s.rstate[q.r].A : s.racc[k - 1];
  uint32_t first_change = NONE32;
  RBatch b0, b1;
  relax_load(s, k, end, lane, b0);
  RP_ADD(t_setup, tp);
  bool done = false;
  uint32_t stop_e = NONE32;
  // ping-pong: the next batch's loads are in flight while this batch's RB steps run
  for (;;) {
    relax_load(s, k + 64u * RB, end, lane, b1);
    relax_batch<SMALL>(s, b0, chi, it, end, lane, k, A, first_change, done, stop_e, prof);
    if (done) break;
    relax_load(s, k + 64u * RB, end, lane, b0);
    relax_batch<SMALL>(s, b1, chi, it, end, lane, k, A, first_change, done, stop_e, prof);
    if (done) break;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) first_change = min(first_change, (uint32_t)__shfl_xor((int)first_change, o, 64));
  if (k > q.hwm) {
    q.hwm = k;
    q.hwm_e = k < end ? stop_e : NONE32;
  }
  return first_change;
}

// Light walker: this lane walks slot q's entries from entry k (events < chi); updates q.hwm/hwm_e.
__device__ inline uint32_t relax_lane(const Scratch& s, RSlot& q, uint32_t k, uint32_t chi, uint32_t it) {
  const uint32_t end = q.end;
  __int128 A = k == q.start ? s.rstate[q.r].A : s.racc[k - 1];
  uint32_t first_change = NONE32;
  uint32_t meta = s.rmeta[k];
  uint32_t stop_e = NONE32;
  for (;;) {
    const uint32_t e = meta & RM_EVENT;
    const __int128 amt = (__int128)s.ramt[k];
    const bool opass = !(meta & RM_WAIT) || at_load(&s.roth[k]) != 0u;
    if (meta & RM_CHECK) {
      const bool pass = amt <= A;
      const uint32_t own = s.rown[k];
      if (own != (pass ? 1u : 0u) && relax_publish(s, k, s.rlink[k], own, pass, it)) first_change = min(first_change, e);
      if (pass && opass) A -= amt;
    } else if (opass && (meta & RM_ADD)) {
      A += amt;
    }
    s.racc[k] = A;
    k++;
    if (k >= end) break;
    meta = s.rmeta[k];
    if ((meta & RM_EVENT) >= chi) {
      stop_e = meta & RM_EVENT;
      break;
    }
  }
  if (k > q.hwm) {
    q.hwm = k;
    q.hwm_e = stop_e;
  }
  return first_change;
}

// Walks slot q in iteration `it` if it is marked dirty or chi passed its never-walked entries.
template <bool WAVE, bool SMALL>
__device__ inline uint32_t relax_visit(const Scratch& s, RSlot& q, uint32_t mark, uint32_t chi, uint32_t it,
                                       RProf& prof) {
  if (mark == NONE32 && q.hwm_e >= chi) return NONE32;
  uint32_t k = q.hwm;
  if (mark != NONE32) {
    uint32_t m = NONE32;
    if (!WAVE || (threadIdx.x & 63) == 0) m = relax_take_mark(s, q.r, it, mark);
    if (WAVE) m = (uint32_t)__builtin_amdgcn_readfirstlane((int)m);
    k = min(k, m);
  }
  if (WAVE) return relax_wave<SMALL>(s, q, k, chi, it, prof);
  return relax_lane(s, q, k, chi, it);
}

// Persistent relaxation (cooperative launch, one block per CU). Waves [0, Ph) walk the heavy ranks,
// the others the light ranks, one per lane.
__global__ void __launch_bounds__(RELAX_THREADS) k_res_relax(Dev d, Scratch s, uint32_t E, uint32_t chunk) {
  Globals* g = d.g;
  if (g->res_inelig || !g->hot_count || g->res_chunked) return;
  const uint32_t H = g->heavy_count, L = g->light_count;
  const uint32_t P = gridDim.x * (RELAX_THREADS / 64);
  const uint32_t wave = blockIdx.x * (RELAX_THREADS / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t Ph = min(H, L ? P / 2 : P);
  const bool small = !g->batch_huge && g->batch_amount_sum < ((u128)1 << 62);
  // register slots: a heavy wave's first RSLOTS ranks, a light lane's first RSLOTS ranks
  const uint32_t lstride = (P - Ph) * 64, lfirst = (wave - Ph) * 64 + (uint32_t)lane;
  RSlot slot[RSLOTS];
  int nslot = 0;
#pragma unroll
  for (int i = 0; i < RSLOTS; i++) {
    const uint32_t j = wave < Ph ? wave + i * Ph : lfirst + i * lstride;
    if (j < (wave < Ph ? H : L)) {
      slot[i] = relax_slot(s, wave < Ph ? s.heavy[j] : s.light[j]);
      nslot = i + 1;
    } else {
      slot[i] = RSlot{0, 0, 0, 0, NONE32};
    }
  }
  uint32_t clo = 0;
  const uint64_t t_begin = wall_clock64();
  uint64_t t_bar = 0, n_it = 0, n_same = 0, t_work = 0;
  RProf prof = {0, 0, 0, 0, 0, 0, 0};
  for (uint32_t it = 0; clo < E; it++) {
    if (it >= RELAX_MAX_ITERS) {
      if (threadIdx.x == 0) __hip_atomic_fetch_or(&g->res_error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    const uint32_t chi = min(E, clo + chunk);
    uint32_t* fc = &g->res_fc[it % 3u];
    if (blockIdx.x == 0 && threadIdx.x == 0)
      __hip_atomic_store(&g->res_fc[(it + 1u) % 3u], NONE32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t tw0 = wall_clock64();
    uint32_t fch = NONE32;
    if (wave < Ph) {
      // this wave's heavy ranks; the marks of all of them are loaded before any walk
      uint32_t mk[RSLOTS];
#pragma unroll
      for (int i = 0; i < RSLOTS; i++) mk[i] = i < nslot ? at_load(&s.rstate[slot[i].r].dirty[(it + 1u) & 1u]) : NONE32;
#pragma unroll
      for (int i = 0; i < RSLOTS; i++) {
        if (i >= nslot) break;
        const uint32_t m = (uint32_t)__builtin_amdgcn_readfirstlane((int)mk[i]);
        fch = min(fch, small ? relax_visit<true, true>(s, slot[i], m, chi, it, prof)
                             : relax_visit<true, false>(s, slot[i], m, chi, it, prof));
      }
      for (uint32_t j = wave + RSLOTS * Ph; j < H; j += Ph) {  // beyond the register slots
        RSlot q = relax_slot(s, s.heavy[j]);
        q.hwm = q.start + s.rstate[q.r].pos;
        q.hwm_e = q.hwm < q.end ? (s.rmeta[q.hwm] & RM_EVENT) : NONE32;
        const uint32_t m = (uint32_t)__builtin_amdgcn_readfirstlane((int)at_load(&s.rstate[q.r].dirty[(it + 1u) & 1u]));
        fch = min(fch, small ? relax_visit<true, true>(s, q, m, chi, it, prof)
                             : relax_visit<true, false>(s, q, m, chi, it, prof));
        if (lane == 0) s.rstate[q.r].pos = q.hwm - q.start;
      }
    } else {
      uint32_t mk[RSLOTS];
#pragma unroll
      for (int i = 0; i < RSLOTS; i++) mk[i] = i < nslot ? at_load(&s.rstate[slot[i].r].dirty[(it + 1u) & 1u]) : NONE32;
#pragma unroll
      for (int i = 0; i < RSLOTS; i++)
        if (i < nslot) fch = min(fch, relax_visit<false, true>(s, slot[i], mk[i], chi, it, prof));
      for (uint32_t j = lfirst + RSLOTS * lstride; j < L; j += lstride) {
        RSlot q = relax_slot(s, s.light[j]);
        q.hwm = q.start + s.rstate[q.r].pos;
        q.hwm_e = q.hwm < q.end ? (s.rmeta[q.hwm] & RM_EVENT) : NONE32;
        fch = min(fch, relax_visit<false, true>(s, q, at_load(&s.rstate[q.r].dirty[(it + 1u) & 1u]), chi, it, prof));
        s.rstate[q.r].pos = q.hwm - q.start;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) fch = min(fch, (uint32_t)__shfl_xor((int)fch, o, 64));
    if (lane == 0 && fch != NONE32) __hip_atomic_fetch_min(fc, fch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    t_work += wall_clock64() - tw0;
    const uint64_t tb0 = wall_clock64();
    if (!relax_barrier(g, it)) return;
    t_bar += wall_clock64() - tb0;
    const uint32_t f = __hip_atomic_load(fc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    clo = f == NONE32 ? chi : f;
    n_it++;
    n_same += f == NONE32;
  }
  // statistics (tbg_debug_counters): [0] iterations, [1] change-free iterations (block 0); heavy
  // walkers (RELAX_PROF): [2] steps, [3] correction rounds, [4] wait, [5] scan, [6] correction,
  // [7] publish/store clock64 cycles (sums over heavy waves)
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    g->dbg[0] += n_it;
    g->dbg[1] += n_same;
  }
  if (RELAX_PROF && wave < Ph && lane == 0) {
    atomicAdd((unsigned long long*)&g->dbg[2], (unsigned long long)prof.steps);
    atomicAdd((unsigned long long*)&g->dbg[3], (unsigned long long)prof.rounds);
    atomicAdd((unsigned long long*)&g->dbg[4], (unsigned long long)prof.t_wait);
    atomicAdd((unsigned long long*)&g->dbg[5], (unsigned long long)prof.t_scan);
    atomicAdd((unsigned long long*)&g->dbg[6], (unsigned long long)prof.t_corr);
    atomicAdd((unsigned long long*)&g->dbg[7], (unsigned long long)prof.t_pub);
  }
  (void)t_bar;
  (void)t_work;
  (void)t_begin;
}

// Per entry: the other side's entry of the same event and its rank (or NONE when that side is not hot).
__global__ void __launch_bounds__(256) k_res_links(Dev d, Scratch s, uint32_t n) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n || d.g->res_inelig || !d.g->hot_count || d.g->res_chunked) return;
  if (s.rkey[k] == RES_DUMMY) return;
  const uint32_t v = s.rval[k];
  const uint32_t ko = s.kidx[v ^ 1u];
  s.rlink[k] = make_uint2(ko, ko == NONE32 ? NONE32 : s.rkey[ko]);
}

// Per-account effect sums of the committed entries: a committed entry adds its amount to its
// account's field rm_field(meta). Segmented wave sums by key, one u128 atomic per segment.
// CHUNKED (chunks.h): keys are (chunk, rank), rown holds each entry's committed bit, st is written.
template <bool CHUNKED>
__global__ void __launch_bounds__(256) k_res_sum(Dev d, Scratch s, uint32_t n) {
  const Globals* g = d.g;
  if (g->res_inelig || !g->hot_count || g->res_error || (g->res_chunked != 0) != CHUNKED) return;
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const uint32_t dummy = CHUNKED ? RC_DUMMY : RES_DUMMY;
  uint32_t key = dummy;
  u128 v[4] = {0, 0, 0, 0};
  if (k < n) {
    key = s.rkey[k];
    if (key != dummy) {
      const uint32_t meta = s.rmeta[k];
      bool ok = true;
      if (CHUNKED) {
        ok = s.rown[k] != 0u;
      } else {
        const uint32_t e = meta & RM_EVENT;
        const uint32_t side = (meta & RM_SIDE) ? 1u : 0u;
        if (meta & RM_CHECK) {
          const bool pass = s.rown[k] == 1u;
          atomicOr(&s.st[e], st_known(side) | (pass ? st_pass_bit(side) : 0u));  // for k_res_final
          ok = pass;
        }
        if (meta & RM_WAIT) ok = ok && s.roth[k] != 0u;
      }
      if (ok) v[rm_field(meta)] = s.ramt[k];
    }
  }
  // segmented inclusive scan towards higher lanes; the last lane of a segment holds its sum
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t ko = (uint32_t)__shfl_up((int)key, o, 64);
    const bool take = lane >= o && ko == key;
    // take only if every lane between is the same key: keys are sorted, so equality at distance o
    // implies it
#pragma unroll
    for (int f = 0; f < 4; f++) {
      const unsigned long long lo = __shfl_up((unsigned long long)v[f], o, 64);
      const unsigned long long hi = __shfl_up((unsigned long long)(v[f] >> 64), o, 64);
      if (take) v[f] += ((u128)hi << 64) | lo;
    }
  }
  const uint32_t kn = (uint32_t)__shfl_down((int)key, 1, 64);
  const bool last = lane == 63 || kn != key || k + 1 >= n;
  if (key != dummy && k < n && last) {
    RState& rs = s.rstate[CHUNKED ? key & RC_RMASK : key];
#pragma unroll
    for (int f = 0; f < 4; f++)
      if (v[f]) atomic_add_u128((tb_uint128_t*)&rs.d[f], v[f]);
  }
}
