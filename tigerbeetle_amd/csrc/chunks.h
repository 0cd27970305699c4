// chunks.h — chunked exact resolution of balance-limit windows in ONE workgroup (default resolver
// when the window's hot accounts fit its LDS).
//
// Same class, equations and outputs as relax.h (the sequential execution, state_machine.zig:
// 1220-1306 calling create_transfer's limit checks :1567-1570, is the unique solution of
//   s[e] = AND over the sides of e that check: amount(e) <= A_side(e)
//   A_x(e) = A_x(start) + effects on x of the committed events before e), solved chunk by chunk:
//  * the window is cut into aligned chunks of RC_C events; the sorted entries are keyed by
//    (chunk, compact hot rank), so a chunk's entries are contiguous and grouped by account;
//  * one workgroup walks the chunks in order with every hot account's available balance A in LDS
//    (exact at each chunk start); a chunk's entries, statuses and segment table live in LDS;
//  * inside a chunk it iterates: every account segment is walked exactly in event order from A
//    (a wave per long segment: 64-entry exclusive scan, then the first failing check corrected and
//    the rest re-tested, as in relax.h; a lane per short one), reading the other side's check of
//    the previous iteration (initially: pass); when no check that another walker reads changed,
//    the chunk is the unique solution (every status is computed from the statuses it reads), so A
//    advances by each segment's effects and the next chunk starts. Iteration k settles at least the
//    chunk's first k positions, so a chunk needs at most RC_C + 1 iterations.
// Cross-walker traffic is LDS only and a step is a workgroup barrier (sub-microsecond), against a
// grid barrier per relax.h iteration: the cfg3 window (Zipf-hot accounts, ~2.5 % exceeds_credits)
// needs ~2.6 iterations per 1024-event chunk. Eligible: at most RC_MAXR hot accounts after
// k_bind_decide (compact ranks), window amounts below 2^62 (in-chunk sums in int64), E <= 2^20.
// Outputs as relax.h: st[] pass bits (k_res_final), per-entry committed bits in rown[] (k_res_sum
// then sums them per account, k_res_apply applies the sums).
#pragma once
#include "relax.h"

#define RC_T 1024  // threads of the workgroup
#define RC_ME (2 * RC_C)  // entries per chunk at most
#ifndef RC_LONG
#define RC_LONG 8  // longer segments are walked by a whole wave (round 6 A/B on cfg3: 4, 12 and 16 slower)
#endif
// Entry encoding in LDS (k_rc_build): bits 0-10 the (side, event) check slot (side << 10 | event in
// chunk), bit 11 the entry's side checks (a limit), bit 12 a committed entry raises A.
#define RC_EM_IDX 0x7FFu
#define RC_EM_CHECK 0x800u
#define RC_EM_ADD 0x1000u
#ifndef RC_HEAD_SIMD
// 1: the chunk's longest segment walked by wave 0 alone on its SIMD; 2: by wave 0 (others share the
// SIMD); 0: taken from the long queue like any other. Round 6 (cfg3, one box): 0 9.87, 1 9.39,
// 2 6.92 x 10^7 transfers/s — the other segments' walks, not the head's, pace an iteration
// (RC_PROF: the longest wave walk is 0.78 of 1.84 ms of walk phases per window), so no wave sits out.
#define RC_HEAD_SIMD 0
#endif
#ifndef RC_PROF
#define RC_PROF 0  // 1: per-phase clock64() sums of k_rc_run into Globals::dbg (tbg_debug_counters);
                   // profiling only: it adds clock reads and changes no result
#endif
#define RC_NONE 0xFFFFu

// Per chunk, built by k_rc_build (one workgroup per chunk, all chunks at once) so that the single
// workgroup of k_rc_run only copies a chunk's tables into LDS (one barrier per chunk). Chunk c owns
// the entry range [cb, cb + 2 * RC_C), cb = 2 * c * RC_C (its events' two sides), of which the
// first m = rc_cb[c] - cb are its hot entries, grouped by rank, event order inside a rank:
//   rkey/rmeta/ramt[k] entry k: (chunk, rank) key (RC_DUMMY past the hot entries), meta, amount
//   rc_segof[k]        entry k's segment within its chunk
//   rc_seg[cb + c + i] segment i's first entry (i <= nseg; the last = the chunk's entry count)
//   rc_list[cb + i]    segment ids: the > 64-entry segments, then the > RC_LONG ones, then the rest
//   rc_ent[2e + side]  the entry of (event e, side) within its chunk (RC_NONE: that side is not hot)
//   rc_em[k]           entry k's encoding (RC_EM_*)
//   rc_srank[cb + c + i] segment i's compact rank (its A without a load of its first entry's rank)
//   rc_cnt[c]          (nseg, huge, long, some amount >= 2^24)
// and per rank (from the first entry of each (chunk, rank) segment: identical values) its account
// slot and initial A in rstate.
struct RcLds {
  int64_t A[RC_MAXR];          // available balance of every hot rank at the chunk start (clamped, below)
  uint64_t amt[RC_ME];         // the chunk's entries, grouped by rank, event order inside a rank
  int64_t dent[RC_ME];         // per entry: the segment's effects on A before it (last walk)
  int64_t delta[RC_ME];        // per segment: its effects on A (last walk)
  uint16_t em[RC_ME];          // entry encoding (RC_EM_*)
  uint32_t dfrom[RC_ME];       // per segment: first entry whose input changed (RC_NONE: clean)
  uint16_t srank[RC_ME];       // per segment: its account's compact rank (k_rc_build)
  uint16_t segof[RC_ME];       // entry -> segment
  uint16_t seg[RC_ME + 1];     // segment starts (entry index), seg[nseg] = entries
  uint16_t lst[RC_ME];         // segment ids: long ones (the longest first), then short ones
  uint16_t ent[2][RC_C];       // per side and event: its entry (RC_NONE: that side is not hot)
  uint8_t oth[RC_ME];          // per entry: the other side's check as its reader sees it (1 = pass)
  uint8_t cur[2 * RC_C], prv[2][RC_C];  // per (side, event): latest check / the one readers use (1 = pass)
  uint32_t cb[1024];           // every chunk's end of hot entries (no global load on a chunk's critical path)
  uint32_t qlong, qshort, chg[2];
  uint32_t pmax;  // RC_PROF: longest wave walk of the iteration (cycles)
};

// The chunk's (side, event) pairs sorted by (rank, position) in LDS: a 2048-key bitonic sort of
// rank << 11 | position (unique keys, so the order inside a rank is event order, as the stable global
// sort it replaces gave), non-hot sides (rank 0xFFF) last. RC_MAXR = 4095 keeps 0xFFF free.
__global__ void __launch_bounds__(RC_T) k_rc_build(Dev d, Scratch s, uint32_t E) {
  __shared__ uint32_t sk[RC_ME];
  __shared__ uint16_t seg[RC_ME + 1];
  __shared__ uint32_t wcnt[2][RC_T / 64];
  __shared__ uint32_t ncls[3], big, mtot;
  if (!d.g->res_chunked) return;
  const uint32_t c = blockIdx.x, t = threadIdx.x;
  const int lane = t & 63;
  const uint32_t wave = t >> 6;
  const uint32_t c0 = c * RC_C, nev = min((uint32_t)RC_C, E - c0), n = 2 * nev, cb0 = 2 * c0;
  if (t < nev) *(uint32_t*)&s.rc_ent[2 * (c0 + t)] = (RC_NONE << 16) | RC_NONE;
  if (t < 3) ncls[t] = 0;
  if (t == 0) {
    big = 0;
    mtot = 0;
  }
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const uint32_t p = t + (uint32_t)j * RC_T;
    uint32_t v = 0xFFFFFFFFu;
    if (p < n) {
      const uint32_t key = s.rkey_in[cb0 + p];
      v = ((key == RC_DUMMY ? 0xFFFu : (key & RC_RMASK)) << 11) | p;
    }
    sk[p] = v;
  }
  __syncthreads();
  for (uint32_t k = 2; k <= RC_ME; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      const uint32_t i = ((t & ~(j - 1)) << 1) | (t & (j - 1)), l = i + j;
      const uint32_t a = sk[i], b = sk[l];
      if ((a > b) == ((i & k) == 0)) {
        sk[i] = b;
        sk[l] = a;
      }
      __syncthreads();
    }
  }
  // the hot entries: m = the first non-hot position (sorted)
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const uint32_t q = t + (uint32_t)j * RC_T;
    const bool hot = (sk[q] >> 11) < 0xFFFu;
    const bool next_hot = q + 1 < RC_ME && (sk[q + 1] >> 11) < 0xFFFu;
    if (hot && !next_hot) mtot = q + 1;
  }
  __syncthreads();
  const uint32_t m = mtot;
  bool bg = false, f[2];
  uint32_t meta[2];
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const uint32_t q = t + (uint32_t)j * RC_T;
    f[j] = false;
    meta[j] = 0;
    if (q >= n) continue;
    const uint32_t k = cb0 + q;
    if (q >= m) {
      s.rkey[k] = RC_DUMMY;
      continue;
    }
    const uint32_t r = sk[q] >> 11, pos = sk[q] & 0x7FFu;
    const uint32_t e = c0 + (pos >> 1), side = pos & 1u;
    const uint32_t key = (c << RC_RBITS) | r;
    s.rkey[k] = key;
    // entry meta and amount (the relaxation's k_res_segs, chunk layout)
    const uint32_t cls = s.cls[e];
    const bool need_dr = cls & C_READS_DR, need_cr = cls & C_READS_CR;
    const uint32_t slot = side ? s.cr_slot[e] : s.dr_slot[e];
    const tb_account_t& a = d.acc[slot];
    const bool dc = acc_is_dc(a.flags);
    const bool pending = cls & C_PENDING;
    const bool check = side ? need_cr : need_dr;
    const bool add = !check && !pending && (side ? dc : !dc);
    const bool wait = side ? need_dr : need_cr;
    meta[j] = e | (side ? RM_SIDE : 0) | (check ? RM_CHECK : 0) | (wait ? RM_WAIT : 0) | (add ? RM_ADD : 0) |
              (pending ? RM_PEND : 0);
    s.rmeta[k] = meta[j];
    const u128 amt = s.amt[e];
    s.ramt[k] = amt;
    bg = bg || (uint64_t)amt >= (1ull << 24);
    f[j] = q == 0 || (sk[q - 1] >> 11) != r;
    if (f[j]) {
      const __int128 dp = (__int128)U(a.debits_pending), dpo = (__int128)U(a.debits_posted);
      const __int128 cp = (__int128)U(a.credits_pending), cpo = (__int128)U(a.credits_posted);
      RState& rs = s.rstate[r];
      rs.start = 0;
      rs.end = 1;  // k_res_apply: the rank has entries
      rs.slot = slot;
      rs.A = dc ? cpo - dp - dpo : dpo - cp - cpo;
      rs.d[0] = rs.d[1] = rs.d[2] = rs.d[3] = 0;
    }
    s.rc_ent[2 * e + side] = (uint16_t)q;
    s.rc_em[k] = (uint16_t)((side << 10) | (e - c0) | ((meta[j] & RM_CHECK) ? RC_EM_CHECK : 0u) |
                            ((meta[j] & RM_ADD) ? RC_EM_ADD : 0u));
  }
  if (bg) big = 1;
  // segments: their starts, each entry's segment, and the walk lists (huge, long, short)
  const unsigned long long b0 = __ballot(f[0]), b1 = __ballot(f[1]);
  if (lane == 0) {
    wcnt[0][wave] = (uint32_t)__popcll(b0);
    wcnt[1][wave] = (uint32_t)__popcll(b1);
  }
  __syncthreads();
  uint32_t pre0 = 0, tot0 = 0, pre1 = 0, tot1 = 0;
  for (uint32_t w = 0; w < RC_T / 64; w++) {
    const uint32_t a0 = wcnt[0][w], a1 = wcnt[1][w];
    pre0 += w < wave ? a0 : 0u;
    pre1 += w < wave ? a1 : 0u;
    tot0 += a0;
    tot1 += a1;
  }
  const unsigned long long upto = (2ull << lane) - 1ull;  // lanes <= this one
  const uint32_t id0 = pre0 + (uint32_t)__popcll(b0 & upto) - 1u;
  const uint32_t id1 = tot0 + pre1 + (uint32_t)__popcll(b1 & upto) - 1u;
  if (f[0]) {
    seg[id0] = (uint16_t)t;
    s.rc_srank[cb0 + c + id0] = (uint16_t)(sk[t] >> 11);
  }
  if (f[1]) {
    seg[id1] = (uint16_t)(t + RC_T);
    s.rc_srank[cb0 + c + id1] = (uint16_t)(sk[t + RC_T] >> 11);
  }
  if (t < m) s.rc_segof[cb0 + t] = (uint16_t)id0;
  if (t + RC_T < m) s.rc_segof[cb0 + t + RC_T] = (uint16_t)id1;
  const uint32_t nseg = tot0 + tot1;
  if (t == 0) seg[nseg] = (uint16_t)m;
  __syncthreads();
  uint32_t cl[2], idx[2];
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const uint32_t sg = t + (uint32_t)j * RC_T;
    cl[j] = 3;
    if (sg <= nseg) s.rc_seg[cb0 + c + sg] = seg[sg];
    if (sg < nseg) {
      const uint32_t len = (uint32_t)(seg[sg + 1] - seg[sg]);
      cl[j] = len > 64 ? 0u : (len > RC_LONG ? 1u : 2u);
      idx[j] = atomicAdd(&ncls[cl[j]], 1u);
    }
  }
  __syncthreads();
  const uint32_t nh = ncls[0], nl = ncls[1];
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const uint32_t sg = t + (uint32_t)j * RC_T;
    if (cl[j] < 3) s.rc_list[cb0 + (cl[j] == 0 ? 0u : (cl[j] == 1 ? nh : nh + nl)) + idx[j]] = (uint16_t)sg;
  }
  if (t == 0) {
    s.rc_cnt[c] = make_uint4(nseg, nh, nl, big);
    s.rc_cb[c] = cb0 + m;  // the end of the chunk's hot entries
  }
}

// A is the pre-window balance clamped into [-2^62, 2^62] plus the window's effects so far: a check
// fails iff amount > A_exact + P, where P sums effects of other events of the window, and amount + |P|
// is below the window's amount sum < 2^62. So A_exact >= 2^62 never fails and A_exact <= -2^62
// always fails, exactly as the clamped value decides, and A never leaves int64 (the exact balances
// are applied by k_res_sum / k_res_apply, not from A).
__device__ inline int64_t rc_clamp(__int128 a) {
  const __int128 lim = (__int128)1 << 62;
  if (a > lim) return (int64_t)lim;
  if (a < -lim) return -(int64_t)lim;
  return (int64_t)a;
}
__device__ inline int64_t rc_sat_add(int64_t a, int64_t b) {
  int64_t r;
  if (__builtin_add_overflow(a, b, &r)) return a > 0 ? INT64_MAX : INT64_MIN;
  return r;
}

__device__ inline uint32_t rc_uniform(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ inline int64_t rc_uniform64(int64_t v) {
  return (int64_t)(((uint64_t)rc_uniform((uint32_t)((uint64_t)v >> 32)) << 32) | rc_uniform((uint32_t)(uint64_t)v));
}

// Inclusive wave64 scan of int32 (DPP row shifts, row broadcasts).
__device__ inline int32_t wave_incl_scan_i32(int32_t x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
  return x;
}

// One 64-entry step of rc_walk_wave32 from its (already loaded) inputs; advances D.
__device__ __attribute__((always_inline)) inline void rc_step32(RcLds& L, uint32_t k, uint32_t s1, int lane, int64_t A0,
                                                                int64_t& D, uint32_t em, int32_t amt, uint32_t oth,
                                                                uint64_t& rounds, uint64_t* tp) {
  const uint64_t q0 = RC_PROF == 1 ? clock64() : 0;
  const uint32_t kk = k + (uint32_t)lane;
  const bool act = kk < s1;
  const uint32_t n = min(64u, s1 - k);
  const bool check = em & RC_EM_CHECK;
  bool ok = act && oth != 0u;
  int32_t eff = 0;
  if (ok) eff = check ? -amt : ((em & RC_EM_ADD) ? amt : 0);
  int32_t pre = wave_incl_scan_i32(eff) - eff;
  // B = A0 + D clamped into int32 with 32-bit scalar operations (|A0| <= 2^62, |D| < 2^62)
  const int64_t B64 = A0 + D;
  const uint32_t blo = (uint32_t)B64;
  const int32_t bhi = (int32_t)(B64 >> 32);
  const int32_t B = bhi == ((int32_t)blo >> 31) ? (int32_t)blo : (bhi < 0 ? INT32_MIN : INT32_MAX);
  // Failures in lane order: every lane after the last failure found sees the failed amounts so far
  // added back, so the next failure is the first later candidate with amount - pre > B + acc (a
  // uniform threshold: one compare, one find-first and one readlane per failure); the failed
  // amounts are added to the later prefixes once, by a scan, after the last one.
  const int32_t x = amt - pre;
  uint64_t q1 = 0;
  if (RC_PROF == 1) {
    q1 = clock64();
    tp[0] += q1 - q0;
  }
  const unsigned long long cand = __ballot(ok && check);
  unsigned long long fails = 0, after = ~0ull;
  const uint32_t room = (uint32_t)INT32_MAX - (uint32_t)B;  // B + acc stays an int32 below it
  uint32_t acc = 0;
  while (acc < room) {
    const unsigned long long fm = __ballot(x > B + (int32_t)acc) & cand & after;
    if (!fm) break;
    const int jl = __builtin_ctzll(fm);
    if (RC_PROF == 1) rounds++;
    acc += (uint32_t)__builtin_amdgcn_readlane(amt, jl);
    fails |= 1ull << jl;
    after = jl == 63 ? 0ull : ~0ull << (jl + 1);
  }
  if (fails) {
    const bool failed = (fails >> lane) & 1ull;
    const int32_t fa = failed ? amt : 0;
    pre += wave_incl_scan_i32(fa) - fa;
    if (failed) eff = 0;
  }
  if (RC_PROF == 1) tp[1] += clock64() - q1;
  if (act) {
    if (check) L.cur[em & RC_EM_IDX] = amt - pre <= B ? 1 : 0;
    L.dent[kk] = D + pre;
  }
  D += __builtin_amdgcn_readlane(pre + eff, (int)n - 1);
}

// Whole-wave walk of a segment whose amounts are all below 2^24 (the chunk's common case): the
// in-step prefix and amount - prefix fit an int32 (|.| < 65 * 2^24), and a check fails iff
// amount - pre > A0 + D, with A0 + D clamped into int32 without changing any comparison. Same
// outputs as rc_walk_wave.
// Each step's LDS inputs are loaded one step ahead into one of two register sets, alternating (the
// loop is unrolled by two): with a single set the loop-carried copy of the prefetched values at the
// end of each step waited for the loads it had just issued (and for the step's stores).
__device__ inline void rc_walk_wave32(RcLds& L, uint32_t sg, uint32_t kf, int lane, uint64_t& rounds,
                                      uint64_t* tp) {
  const uint64_t e0 = RC_PROF == 2 ? clock64() : 0;
  const uint32_t s0 = rc_uniform(L.seg[sg]), s1 = rc_uniform(L.seg[sg + 1]);
  const int64_t A0 = rc_uniform64(L.A[L.srank[sg]]);
  // a re-walk starts at the first entry whose input changed, from the balance kept before it
  int64_t D = kf == s0 ? 0 : rc_uniform64(L.dent[kf]);
  if (RC_PROF == 2) {  // walks and their set-up cycles
    rounds++;
    tp[1] += clock64() - e0;
  }
  // prefetches are unconditional loads of clamped positions (lanes past the end ignore what they
  // read): a load issued on one path only made the compiler wait for every outstanding LDS op
  uint32_t kk = min(kf + (uint32_t)lane, (uint32_t)RC_ME - 1u);
  uint32_t emA = L.em[kk], emB;
  int32_t amtA = reinterpret_cast<const int32_t*>(L.amt)[2 * kk], amtB;  // the low word (< 2^24)
  uint32_t othA = L.oth[kk], othB;
  for (uint32_t k = kf; k < s1; k += 128) {
    kk = min(k + 64u + (uint32_t)lane, (uint32_t)RC_ME - 1u);
    emB = L.em[kk];
    amtB = reinterpret_cast<const int32_t*>(L.amt)[2 * kk];
    othB = L.oth[kk];
    rc_step32(L, k, s1, lane, A0, D, emA, amtA, othA, rounds, tp);
    if (k + 64u >= s1) break;
    kk = min(k + 128u + (uint32_t)lane, (uint32_t)RC_ME - 1u);
    emA = L.em[kk];
    amtA = reinterpret_cast<const int32_t*>(L.amt)[2 * kk];
    othA = L.oth[kk];
    rc_step32(L, k + 64u, s1, lane, A0, D, emB, amtB, othB, rounds, tp);
  }
  if (lane == 0) L.delta[sg] = D;
}

// Whole-wave walk of segment sg (64 entries per step), any amounts below 2^62. A check passes iff
// amount <= A0 + D + pre, i.e. amount - (pre + D) <= A0.
__device__ inline void rc_walk_wave(RcLds& L, uint32_t sg, uint32_t kf, int lane) {
  // wave-uniform bounds (SGPRs): the step loop and its ballots are uniform control flow
  const uint32_t s0 = rc_uniform(L.seg[sg]), s1 = rc_uniform(L.seg[sg + 1]);
  const int64_t A0 = rc_uniform64(L.A[L.srank[sg]]);
  int64_t D = kf == s0 ? 0 : rc_uniform64(L.dent[kf]);
  for (uint32_t k = kf; k < s1; k += 64) {
    const uint32_t kk = k + (uint32_t)lane;
    const bool act = kk < s1;
    const uint32_t n = min(64u, s1 - k);
    const uint32_t em = act ? L.em[kk] : 0u;
    const int64_t amt = act ? (int64_t)L.amt[kk] : 0;
    const bool check = em & RC_EM_CHECK;
    const bool opass = L.oth[kk & (RC_ME - 1)];  // 1 unless the other side's check failed
    bool ok = act && opass;
    int64_t eff = 0;
    if (ok) eff = check ? -amt : ((em & RC_EM_ADD) ? amt : 0);
    int64_t pre = wave_incl_scan_i64(eff) - eff;
    // failures in lane order against a uniform threshold (rc_walk_wave32)
    const int64_t x = amt - (pre + D);
    const unsigned long long cand = __ballot(ok && check);
    unsigned long long fails = 0, after = ~0ull;
    int64_t thr = A0;
    for (;;) {
      const unsigned long long fm = __ballot(x > thr) & cand & after;
      if (!fm) break;
      const int jl = __builtin_ctzll(fm);
      thr += readlane_i64(amt, jl);
      fails |= 1ull << jl;
      after = jl == 63 ? 0ull : ~0ull << (jl + 1);
    }
    if (fails) {
      const bool failed = (fails >> lane) & 1ull;
      const int64_t fa = failed ? amt : 0;
      pre += wave_incl_scan_i64(fa) - fa;
      if (failed) eff = 0;
    }
    if (act) {
      if (check) L.cur[em & RC_EM_IDX] = amt - (pre + D) <= A0 ? 1 : 0;
      L.dent[kk] = D + pre;
    }
    D += readlane_i64(pre + eff, (int)n - 1);
  }
  if (lane == 0) L.delta[sg] = D;
}

// One lane walks a short segment (at most RC_LONG entries, always from its start: dirty marks of
// short segments are only consumed as "walk it").
__device__ inline void rc_walk_lane(RcLds& L, uint32_t sg) {
  const uint32_t s0 = L.seg[sg], s1 = L.seg[sg + 1];
  const int64_t A0 = L.A[L.srank[sg]];
  int64_t D = 0;
  for (uint32_t k = s0; k < s1; k++) {
    const uint32_t em = L.em[k];
    const int64_t amt = (int64_t)L.amt[k];
    const bool opass = L.oth[k];
    if (em & RC_EM_CHECK) {
      const bool pass = amt - D <= A0;
      L.cur[em & RC_EM_IDX] = pass ? 1 : 0;
      if (opass && pass) D -= amt;
    } else if (opass && (em & RC_EM_ADD)) {
      D += amt;
    }
  }
  L.delta[sg] = D;
}

#define RC_T0() const uint64_t _rc0 = RC_PROF ? clock64() : 0
#define RC_ADD(k, t0)                          \
  do {                                         \
    if (RC_PROF && t == 0) prof[k] += clock64() - (t0); \
  } while (0)

__global__ void __launch_bounds__(RC_T) k_rc_run(Dev d, Scratch s, uint32_t E) {
  __shared__ RcLds L;
  Globals* g = d.g;
  if (!g->res_chunked) return;
  const uint32_t t = threadIdx.x;
  const int lane = t & 63;
  const uint32_t nch = (E + RC_C - 1) / RC_C;
  const uint32_t R = g->hot_live;
  // RC_PROF (thread 0): setup, walk phase, change detection cycles, sum of the longest wave walk per
  // iteration; per wave: load+scan and failure-search cycles, failure rounds
  uint64_t prof[4] = {0, 0, 0, 0};
  uint64_t wrounds = 0, wt[2] = {0, 0}, hz[4] = {0, 0, 0, 0};  // RC_PROF > 1: head walks, other huge walks (cycles, steps)
  for (uint32_t r = t; r < R; r += RC_T) L.A[r] = rc_clamp(s.rstate[r].A);
  for (uint32_t c = t; c < nch; c += RC_T) L.cb[c] = s.rc_cb[c];  // chunk ends (k_rc_build)
  __syncthreads();
  // the next chunk's entries and tables, loaded one chunk ahead (two of each per thread)
  uint32_t pe = 0;
  uint16_t pm[2] = {0, 0};
  uint64_t pa[2] = {0, 0};
  uint16_t ps[2] = {0, 0}, pg[2] = {0, 0}, pl[2] = {0, 0}, pr[2] = {0, 0};
  uint4 pc = make_uint4(0, 0, 0, 0);
  auto fetch = [&](uint32_t c) {
    const uint32_t b0 = 2 * c * RC_C, b1 = L.cb[c];
    pc = s.rc_cnt[c];
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const uint32_t kl = t + (uint32_t)j * RC_T;
      if (b0 + kl < b1) {
        pm[j] = s.rc_em[b0 + kl];
        pa[j] = (uint64_t)s.ramt[b0 + kl];
        ps[j] = s.rc_segof[b0 + kl];
        pl[j] = s.rc_list[b0 + kl];
      }
      if (b0 + kl < b1) pr[j] = s.rc_srank[b0 + c + kl];  // (read past nseg too: unused there)
      if (b0 + kl <= b1) pg[j] = s.rc_seg[b0 + c + kl];
    }
    if (c * RC_C + t < E) pe = *(const uint32_t*)&s.rc_ent[2 * (c * RC_C + t)];
  };
  fetch(0);
  uint64_t iters = 0;
  for (uint32_t c = 0; c < nch; c++) {
    const uint32_t cb0 = 2 * c * RC_C, m = L.cb[c] - cb0;
    const uint32_t c0 = c * RC_C;
    const uint32_t nseg = rc_uniform(pc.x), nhuge = rc_uniform(pc.y), nlong = nhuge + rc_uniform(pc.z);
    const bool big = rc_uniform(pc.w) != 0;
    __syncthreads();  // the previous chunk's LDS is consumed
    const uint64_t tp0 = RC_PROF ? clock64() : 0;
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const uint32_t kl = t + (uint32_t)j * RC_T;
      if (kl < m) {
        L.em[kl] = pm[j];
        L.amt[kl] = pa[j];
        L.segof[kl] = ps[j];
        L.oth[kl] = 1;
      }
      if (kl < nseg) {
        L.lst[kl] = pl[j];
        L.dfrom[kl] = pg[j];  // every segment is walked in the first iteration
        L.srank[kl] = pr[j];
      }
      if (kl <= nseg) L.seg[kl] = pg[j];
    }
    const bool ev = c0 + t < E;
    L.ent[0][t] = ev ? (uint16_t)pe : (uint16_t)RC_NONE;
    L.ent[1][t] = ev ? (uint16_t)(pe >> 16) : (uint16_t)RC_NONE;
    L.cur[t] = L.cur[RC_C + t] = 1;
    L.prv[0][t] = L.prv[1][t] = 1;
    if (t == 0) {
      L.pmax = 0;
      L.qlong = L.qshort = 0;
      L.chg[0] = L.chg[1] = 0;
    }
    if (c + 1 < nch) fetch(c + 1);
    if (m == 0) continue;
    __syncthreads();
    RC_ADD(0, tp0);
    const uint32_t nshort = nseg - nlong;
    // The chunk's longest segment (the Zipf head's: the iteration's critical path) is walked by wave
    // 0 with its SIMD to itself: the other waves of that SIMD (waves 4, 8, 12; waves go to SIMDs
    // round-robin) sit the walk phase out, so the head's steps do not share issue slots.
    uint32_t H = RC_NONE, hlen = 0;
    for (uint32_t j = 0; RC_HEAD_SIMD && j < nhuge; j++) {
      const uint32_t sg = rc_uniform(L.lst[j]);
      const uint32_t len = rc_uniform(L.seg[sg + 1]) - rc_uniform(L.seg[sg]);
      if (len > hlen) {
        hlen = len;
        H = sg;
      }
    }
    const uint32_t wv = t >> 6;
    for (uint32_t it = 0;; it++) {
      if (it > RC_C + 1) {  // cannot happen (see header); the sequential walker takes the window
        if (t == 0) g->res_error = 1;
        return;
      }
      const uint64_t tw0 = RC_PROF ? clock64() : 0;
      uint64_t busy = 0;
      // the dirty segments, from their first changed entry: long ones one per wave (the longest
      // first), short ones one per lane. Every lane of the wave adds 1 (one LDS atomic of 64 after the
      // compiler's wave aggregation): the long queue counts 64 per grab, the short queue hands each
      // lane its own index. No lane-divergent branch around the atomic, so the loops stay
      // wave-uniform (a grab under `if (lane == 0)` let the compiler split the loop per lane).
      if (H != RC_NONE && wv == 0) {
        const uint32_t kf = rc_uniform(L.dfrom[H]);
        if (kf != RC_NONE) {
          L.dfrom[H] = RC_NONE;
          const uint64_t th0 = RC_PROF ? clock64() : 0;
          __builtin_amdgcn_s_setprio(3);
          if (big) rc_walk_wave(L, H, kf, lane);
          else rc_walk_wave32(L, H, kf, lane, wrounds, wt);
          __builtin_amdgcn_s_setprio(0);
          if (RC_PROF > 1) {
            hz[0] += clock64() - th0;
            hz[1] += (rc_uniform(L.seg[H + 1]) - kf + 63) / 64;
          }
        }
      }
      if (RC_PROF == 3) __syncthreads();  // the head walked alone (profiling only)
      const bool sit_out = RC_HEAD_SIMD == 1 && H != RC_NONE && wv != 0 && (wv & 3u) == 0;
      for (; !sit_out;) {
        const uint32_t j = rc_uniform(atomicAdd(&L.qlong, 1u)) >> 6;
        if (j >= nlong) break;
        const uint32_t sg = rc_uniform(L.lst[j]);
        if (sg == H) continue;
        const uint32_t kf = rc_uniform(L.dfrom[sg]);
        if (kf == RC_NONE) continue;
        L.dfrom[sg] = RC_NONE;
        const uint64_t tb0 = RC_PROF ? clock64() : 0;
        // the longest walks (the Zipf head's) are the iteration's critical path: they issue first
        // on their SIMD while other waves walk short segments beside them
        if (j < nhuge) __builtin_amdgcn_s_setprio(3);
        if (big) rc_walk_wave(L, sg, kf, lane);
        else rc_walk_wave32(L, sg, kf, lane, wrounds, wt);
        __builtin_amdgcn_s_setprio(0);
        if (RC_PROF) {
          const uint64_t dt = clock64() - tb0;
          busy += dt;
          if (j < nhuge) {
            hz[2] += dt;
            hz[3] += (rc_uniform(L.seg[sg + 1]) - kf + 63) / 64;
          }
        }
      }
      for (; !sit_out;) {
        const uint32_t j = atomicAdd(&L.qshort, 1u);
        if (rc_uniform(j) >= nshort) break;
        if (j < nshort) {
          const uint32_t sg = L.lst[nlong + j];
          const uint32_t kf = L.dfrom[sg];
          if (kf != RC_NONE) {
            L.dfrom[sg] = RC_NONE;
            rc_walk_lane(L, sg);
          }
        }
      }
      if (RC_PROF && lane == 0) atomicMax(&L.pmax, (uint32_t)busy);
      __syncthreads();
      RC_ADD(1, tw0);
      if (RC_PROF && t == 0) {
        prof[3] += L.pmax;
        L.pmax = 0;
      }
      const uint64_t td0 = RC_PROF ? clock64() : 0;
      // changed checks mark their readers' segments dirty from the reading entry
      if (t == 0) {
        L.qlong = L.qshort = 0;
        L.chg[(it + 1) & 1] = 0;
      }
      bool ch = false;
#pragma unroll
      for (int sd = 0; sd < 2; sd++) {
        const uint8_t v = L.cur[sd * RC_C + t];
        if (v != L.prv[sd][t]) {
          L.prv[sd][t] = v;
          const uint32_t r = L.ent[sd ^ 1][t];
          if (r != RC_NONE) {
            L.oth[r] = v;
            atomicMin(&L.dfrom[L.segof[r]], r);
            ch = true;
          }
        }
      }
      if (ch) L.chg[it & 1] = 1;
      iters++;
      __syncthreads();
      RC_ADD(2, td0);
      if (!L.chg[it & 1]) break;
    }
    // the chunk is final: advance A, publish the statuses and the committed entries
    for (uint32_t sg = t; sg < nseg; sg += RC_T) {
      const uint32_t r = L.srank[sg];
      L.A[r] += L.delta[sg];
    }
    if (c0 + t < E) s.st[c0 + t] = (L.cur[t] ? ST_DR_PASS : 0u) | (L.cur[RC_C + t] ? ST_CR_PASS : 0u);
    // an entry's effect applies iff the other side's check passed and its own (if it checks) did
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const uint32_t kl = t + (uint32_t)j * RC_T;
      if (kl < m) {
        const uint32_t em = L.em[kl];
        s.rown[cb0 + kl] = (L.oth[kl] && (!(em & RC_EM_CHECK) || L.cur[em & RC_EM_IDX])) ? 1u : 0u;
      }
    }
  }
  if (RC_PROF) {
    if (RC_PROF == 1 && lane == 0) atomicAdd((unsigned long long*)&g->dbg[6], (unsigned long long)wt[0]);
    if (lane == 0) atomicAdd((unsigned long long*)&g->dbg[7], (unsigned long long)wt[1]);
    if (lane == 0) atomicAdd((unsigned long long*)&g->dbg[1], (unsigned long long)wrounds);
    if (RC_PROF > 1 && lane == 0) {  // huge-walk split instead of setup / detect / pmax
      atomicAdd((unsigned long long*)&g->dbg[2], (unsigned long long)hz[0]);
      atomicAdd((unsigned long long*)&g->dbg[4], (unsigned long long)hz[1]);
      atomicAdd((unsigned long long*)&g->dbg[5], (unsigned long long)hz[2]);
      atomicAdd((unsigned long long*)&g->dbg[6], (unsigned long long)hz[3]);
    }
  }
  if (t == 0) {
    g->dbg[0] += iters;
    if (RC_PROF == 1)
      for (int k = 0; k < 4; k++) g->dbg[2 + k] += prof[k];
    if (RC_PROF > 1) g->dbg[3] += prof[1];  // the walk phase
    g->res_chunk_windows++;
  }
}

// Chunked windows: each account's committed effects per field, summed per 1024-entry block in LDS
// (the entries are sorted by (chunk, rank): a block holds runs of equal keys; one LDS add per entry,
// then one global add per run and field). Per-wave segment atomics would put every wave of the
// Zipf head's runs on the same four words. Sums stay below 2^62 (rc_eligible), so 64-bit adds.
__global__ void __launch_bounds__(1024) k_rc_sum(Dev d, Scratch s, uint32_t n) {
  __shared__ unsigned long long sums[1024][4];
  __shared__ uint32_t runkey[1024];
  __shared__ uint32_t lds[1024 / 64];
  const Globals* g = d.g;
  if (g->res_inelig || !g->hot_count || g->res_error || !g->res_chunked) return;
  const uint32_t k = blockIdx.x * 1024 + threadIdx.x;
  const uint32_t key = k < n ? s.rkey[k] : RC_DUMMY;
  const bool live = key != RC_DUMMY;
  const bool start = live && (threadIdx.x == 0 || s.rkey[k - 1] != key);
  uint32_t nrun;
  const uint32_t excl = block_excl<1024 / 64>(start ? 1u : 0u, lds, &nrun);
  const uint32_t run = excl + (start ? 1u : 0u) - 1u;  // live entries: the run they belong to
  if (start) runkey[run] = key;
  if (threadIdx.x < nrun) sums[threadIdx.x][0] = sums[threadIdx.x][1] = sums[threadIdx.x][2] = sums[threadIdx.x][3] = 0;
  __syncthreads();
  if (live && s.rown[k] != 0u) {
    const uint32_t meta = s.rmeta[k];
    atomicAdd(&sums[run][rm_field(meta)], (unsigned long long)(uint64_t)s.ramt[k]);
  }
  __syncthreads();
  if (threadIdx.x < nrun) {
    RState& rs = s.rstate[runkey[threadIdx.x] & RC_RMASK];
#pragma unroll
    for (int f = 0; f < 4; f++) {
      const unsigned long long v = sums[threadIdx.x][f];
      if (v) atomic_add_u128((tb_uint128_t*)&rs.d[f], (u128)v);
    }
  }
}
