// resolver.h — account-parallel exact resolution of balance-limit windows.
//
// The sequential walker (walker.h) replays the window's W events one by one. For the common
// order-dependent class — events whose outcome depends on order only through the balance-limit
// checks of create_transfer (debits_must_not_exceed_credits / credits_must_not_exceed_debits,
// state_machine.zig:1567-1570, tigerbeetle.zig:31-39) — the order dependence factors per account:
//
//   a D<=C account's limit test for a debit of `amount` at window position p reads only
//   A(p) = credits_posted - debits_pending - debits_posted of that account just before p, and
//   A(p) is the account's pre-window value plus the effects of the window's earlier committed
//   events on that account (debits: -amount; posted credits: +amount). Symmetrically for C<=D.
//
// So every hot account (one some event's decision reads) walks its own events in window order, and
// an event's outcome is the AND of the checks of
// the (at most two) accounts that read for it. A walker publishes its check of event e in st[e]
// before it needs the other side's check of e, and a check at position p needs only outcomes at
// positions < p, so waits always point to strictly earlier positions: no cycle, every walker
// finishes (all waves are co-resident: cooperative launch; every wait is bounded and falls back to
// the sequential walker if it ever expires). The fixpoint is unique (outcome at p depends only on
// outcomes before p), so the result equals the reference's sequential execution.
//
// Walkers: an account with more than HEAVY_T entries gets a whole wave of its own (64 entries per
// step; it spins when blocked); the others are walked one account per lane, many per wave, each
// lane visiting its accounts round-robin so that a blocked account never holds up another.
// Each walker also sums the window's effects on its account's four balance fields and k_res_apply
// writes them once (no contended atomics on hot accounts); k_final skips the sides so applied.
//
// Within one 64-entry step a heavy wave resolves the recurrence
//   debit check:  pass = amount <= A;  if the event commits: A -= amount
//   posted credit into the account (event commits): A += amount
// by an exclusive 128-bit scan that assumes every check passes, then corrects the first failing
// check, re-tests the lanes after it, and so on (one ballot per failure).
//
// Eligible windows (checked per W event in k_classify): not in overflow mode, 128-bit headroom,
// no linked event, no post/void, no balancing flag, no duplicate / pending-target id. Anything
// else runs on the sequential walker, unchanged.
#pragma once
#include "window.h"

#define RES_KEY_BITS 21
#define RES_DUMMY ((1u << RES_KEY_BITS) - 1)
// chunked mode (chunks.h): keys (1024-event chunk << RC_RBITS | compact rank)
#define RC_C 1024
#define RC_RBITS 12
#define RC_RMASK ((1u << RC_RBITS) - 1u)
#define RC_MAXR RC_RMASK                         // compact ranks 0..RC_MAXR-1
#define RC_DUMMY ((1u << (RC_RBITS + 10)) - 1u)  // sorts after every (chunk < 1024, rank) key
#define RES_SORT_BITS (RC_RBITS + 10)            // the resolver's sort (>= RES_KEY_BITS)
static_assert(RES_SORT_BITS >= RES_KEY_BITS, "sort bits");
#define HEAVY_T 16

enum : uint32_t { ST_DR_KNOWN = 1, ST_DR_PASS = 2, ST_CR_KNOWN = 4, ST_CR_PASS = 8 };
// entry meta: [19:0] event | side | check (this side reads A) | wait (the other side reads) |
// add (a committed event raises A) | pending (the event creates a pending transfer)
enum : uint32_t {
  RM_EVENT = 0xFFFFFu,
  RM_SIDE = 1u << 20,
  RM_CHECK = 1u << 21,
  RM_WAIT = 1u << 22,
  RM_ADD = 1u << 23,
  RM_PEND = 1u << 24,
};

struct __attribute__((aligned(16))) RState {
  uint32_t start, end, pos, slot;
  __int128 A;  // available balance before entry `pos` (see header); relax.h: before entry 0
  u128 d[4];   // committed effects so far: debits_pending, debits_posted, credits_pending, credits_posted
  uint32_t dirty[2];  // relax.h: first entry whose other-side input changed, by iteration parity
  uint32_t pad[2];
};
static_assert(sizeof(RState) == 112, "RState");

__device__ inline bool acc_is_dc(uint16_t flags) { return flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS; }
__device__ inline uint32_t rm_field(uint32_t meta) {
  return ((meta & RM_SIDE) ? 2u : 0u) + ((meta & RM_PEND) ? 0u : 1u);
}
__device__ inline uint32_t st_known(uint32_t side) { return side ? ST_CR_KNOWN : ST_DR_KNOWN; }
__device__ inline uint32_t st_bits(uint32_t side, bool pass) {
  return side ? (ST_CR_KNOWN | (pass ? ST_CR_PASS : 0u)) : (ST_DR_KNOWN | (pass ? ST_DR_PASS : 0u));
}
__device__ inline uint32_t st_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_publish(uint32_t* p, uint32_t bits) {
  __hip_atomic_fetch_or(p, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Chunked mode: every hot account that k_bind_decide kept has a compact rank < RC_MAXR, the
// window's amounts sum below 2^62 (in-chunk int64 sums) and E <= 2^20 (1024 chunks).
__device__ inline bool rc_eligible(const Globals* g, uint32_t E) {
  return !WIN_REJECTED(g) && g->hot_live && g->hot_live <= RC_MAXR && !g->batch_huge &&
         g->batch_amount_sum < ((u128)1 << 62) && E <= 1024u * RC_C;
}

// Keys: one (hot rank, 2*event+side) pair per side of a W event (not failed in validation) whose
// account is hot. Also zeroes the per-event status words and the per-rank segments.
__global__ void __launch_bounds__(256) k_res_keys(Dev d, Scratch s, uint32_t E, uint32_t epoch, uint32_t allow_chunks,
                                                  uint32_t allow_relax) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  Globals* g = d.g;
  if (SP_DONE(g)) return;
  bool active = !g->res_inelig && g->hot_count;
  if (active && i < g->hot_count) {
    s.rstate[i].start = 0;
    s.rstate[i].end = 0;
  }
  if (i < 8) g->res_bar[i] = 0;
  if (i == 0) {
    g->res_bar_top = 0;
    g->res_fc[0] = NONE32;
  }
  // chunked mode (chunks.h): keys (1024-event chunk, compact rank), else (rank)
  const bool chunked = active && allow_chunks && rc_eligible(g, E);
  if (i == 0) g->res_chunked = chunked ? 1u : 0u;
  if (active && !chunked && !allow_relax) {
    // the host did not launch the relaxation (it predicted a chunked window): the sequential walker
    // decides this window; the host's next prediction comes from this window
    if (i == 0) g->res_inelig = 1;
    active = false;
  }
  if (i >= E) return;
  s.kidx[2 * i] = NONE32;
  s.kidx[2 * i + 1] = NONE32;
  s.st[i] = 0;
  const uint32_t dummy = chunked ? RC_DUMMY : RES_DUMMY;
  uint32_t key[2] = {dummy, dummy};
  if (active) {
    const uint32_t cls = s.cls[i];
    if ((cls & C_W) && s.code[i] == TB_CT_OK) {
      const uint32_t dr = s.dr_slot[i], cr = s.cr_slot[i];
      const uint32_t hi = chunked ? (i / RC_C) << RC_RBITS : 0u;
      if (d.hot[dr] == epoch) key[0] = hi | d.hot_rank[dr];
      if (d.hot[cr] == epoch) key[1] = hi | d.hot_rank[cr];
    }
  }
  s.rkey_in[2 * i] = key[0];
  s.rkey_in[2 * i + 1] = key[1];
  s.rval_in[2 * i] = 2 * i;
  s.rval_in[2 * i + 1] = 2 * i + 1;
}

// Sorted pairs -> entries (meta, amount) and per-rank segments with the account's initial A.
__global__ void __launch_bounds__(256) k_res_segs(Dev d, Scratch s, uint32_t n) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n || d.g->res_inelig || !d.g->hot_count || d.g->res_chunked) return;
  const uint32_t key = s.rkey[k];
  if (key == RES_DUMMY) return;
  const uint32_t v = s.rval[k];
  const uint32_t e = v >> 1, side = v & 1;
  const uint32_t cls = s.cls[e];
  const bool need_dr = cls & C_READS_DR, need_cr = cls & C_READS_CR;
  const uint32_t slot = side ? s.cr_slot[e] : s.dr_slot[e];
  const tb_account_t& a = d.acc[slot];
  const bool dc = acc_is_dc(a.flags);
  const bool pending = cls & C_PENDING;
  // D<=C: debits are checked, posted credits raise A. C<=D: credits are checked, posted debits raise A.
  const bool check = side ? need_cr : need_dr;
  const bool add = !check && !pending && (side ? dc : !dc);
  const bool wait = side ? need_dr : need_cr;
  s.kidx[v] = k;
  s.rown[k] = 2u;
  s.roth[k] = 1u;
  s.rmeta[k] = e | (side ? RM_SIDE : 0) | (check ? RM_CHECK : 0) | (wait ? RM_WAIT : 0) | (add ? RM_ADD : 0) |
               (pending ? RM_PEND : 0);
  s.ramt[k] = s.amt[e];
  if (k == 0 || s.rkey[k - 1] != key) {
    const __int128 dp = (__int128)U(a.debits_pending), dpo = (__int128)U(a.debits_posted);
    const __int128 cp = (__int128)U(a.credits_pending), cpo = (__int128)U(a.credits_posted);
    RState& rs = s.rstate[key];
    rs.start = k;
    rs.pos = 0;
    rs.slot = slot;
    rs.A = dc ? cpo - dp - dpo : dpo - cp - cpo;
    rs.d[0] = rs.d[1] = rs.d[2] = rs.d[3] = 0;
    rs.dirty[0] = rs.dirty[1] = NONE32;
  }
  if (k + 1 == n || s.rkey[k + 1] != key) s.rstate[key].end = k + 1;
}

// Splits the hot ranks into heavy (wave-walked) and light (lane-walked) lists.
__global__ void __launch_bounds__(256) k_res_split(Dev d, Scratch s) {
  Globals* g = d.g;
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (g->res_inelig || g->res_chunked || r >= g->hot_count) return;
  const uint32_t len = s.rstate[r].end - s.rstate[r].start;
  if (len == 0) return;
  const bool heavy = len > HEAVY_T;
  const unsigned long long mh = __ballot(heavy), ml = __ballot(!heavy);
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ull << lane) - 1;
  const unsigned long long mine = heavy ? mh : ml;
  const int leader = __builtin_ctzll(mine);
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(heavy ? &g->heavy_count : &g->light_count, (uint32_t)__popcll(mine));
  base = __shfl(base, leader, 64);
  (heavy ? s.heavy : s.light)[base + (uint32_t)__popcll(mine & below)] = r;
}

__device__ inline __int128 i128_shfl(__int128 v, int src) {
  const unsigned long long lo = __shfl((unsigned long long)v, src, 64);
  const unsigned long long hi = __shfl((unsigned long long)((unsigned __int128)v >> 64), src, 64);
  return (__int128)(((unsigned __int128)hi << 64) | lo);
}
__device__ inline __int128 i128_shfl_up(__int128 v, int delta) {
  const unsigned long long lo = __shfl_up((unsigned long long)v, delta, 64);
  const unsigned long long hi = __shfl_up((unsigned long long)((unsigned __int128)v >> 64), delta, 64);
  return (__int128)(((unsigned __int128)hi << 64) | lo);
}
__device__ inline u128 u128_wave_sum(u128 v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long lo = __shfl_xor((unsigned long long)v, o, 64);
    const unsigned long long hi = __shfl_xor((unsigned long long)(v >> 64), o, 64);
    v += ((u128)hi << 64) | lo;
  }
  return v;
}

#define RES_THREADS 256
#ifndef RES_DBG
#define RES_DBG 0  // 1: count steps / blocks / spin time into Globals::dbg (tbg_debug_counters)
#endif
#define DBG_ADD(k, v) \
  do {                                                                             \
    if (RES_DBG) atomicAdd((unsigned long long*)&g->dbg[k], (unsigned long long)(v)); \
  } while (0)
#define DBG_MAX(k, v) \
  do {                                                                             \
    if (RES_DBG) atomicMax((unsigned long long*)&g->dbg[k], (unsigned long long)(v)); \
  } while (0)
#define RES_BUDGET 32
#define RES_LANE_BUDGET 8
#define RES_TIMEOUT_TICKS 20000000ull  // 200 ms of s_memrealtime (100 MHz) without progress

// Gives up (all waves) once any wave has waited RES_TIMEOUT_TICKS without progress.
__device__ inline bool res_stalled(Globals* g, uint64_t last) {
  if (__hip_atomic_load(&g->res_error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return true;
  if (wall_clock64() - last > RES_TIMEOUT_TICKS) {
    __hip_atomic_fetch_or(&g->res_error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  }
  return false;
}

// Heavy walker: the wave advances rank `r` 64 entries per step. `exclusive`: the wave owns no
// other rank, so it waits in place when blocked (bounded); otherwise it returns when blocked.
// Returns false if the resolver gave up.
__device__ inline bool wave_advance(Globals* g, const Scratch& s, uint32_t r, bool exclusive, uint32_t budget,
                                    bool* moved, bool* done) {
  const int lane = threadIdx.x & 63;
  RState* rsp = &s.rstate[r];
  const uint32_t start = rsp->start, end = rsp->end;
  uint32_t pos = rsp->pos;
  __int128 A = rsp->A;
  const uint32_t pos0 = pos;
  u128 acc[4] = {0, 0, 0, 0};
  uint64_t last = wall_clock64();
  // entries of the current step, loaded one step ahead
  uint32_t meta = 0;
  __int128 amt = 0;
  if (start + pos + lane < end) {
    meta = s.rmeta[start + pos + lane];
    amt = (__int128)s.ramt[start + pos + lane];
  }
  for (uint32_t step = 0; (exclusive || step < budget) && start + pos < end; step++) {
    const uint32_t k0 = start + pos;
    const uint32_t n = min(64u, end - k0);
    const bool act = (uint32_t)lane < n;
    const uint32_t e = meta & RM_EVENT;
    const uint32_t side = (meta & RM_SIDE) ? 1u : 0u;
    const bool check = meta & RM_CHECK;
    bool have = true, opass = true;
    uint32_t w = 0;
    if (act && (meta & RM_WAIT)) w = st_load(&s.st[e]);
    // prefetch the next step's entries (used if this step is not blocked)
    uint32_t meta_n = 0;
    __int128 amt_n = 0;
    if (k0 + 64 + lane < end) {
      meta_n = s.rmeta[k0 + 64 + lane];
      amt_n = (__int128)s.ramt[k0 + 64 + lane];
    }
    if (act && (meta & RM_WAIT)) {
      have = w & st_known(side ^ 1);
      opass = w & (side ? ST_DR_PASS : ST_CR_PASS);
    }
    const unsigned long long blocked = __ballot(act && !have);
    const uint32_t lim = blocked ? (uint32_t)__builtin_ctzll(blocked) : n;
    // effects on A assuming every check passes
    bool ok = (uint32_t)lane < lim && opass;
    __int128 eff = 0;
    if (ok) eff = check ? -amt : ((meta & RM_ADD) ? amt : (__int128)0);
    __int128 x = eff;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const __int128 y = i128_shfl_up(x, o);
      if (lane >= o) x += y;
    }
    __int128 P = i128_shfl_up(x, 1);
    if (lane == 0) P = 0;
    P += A;
    // the first failing check fails; re-test the lanes after it; repeat
    int floor_lane = -1;
    for (;;) {
      const unsigned long long fm = __ballot(ok && check && lane > floor_lane && amt > P);
      if (!fm) break;
      const int j = __builtin_ctzll(fm);
      const __int128 aj = i128_shfl(amt, j);
      if (lane > j) P += aj;
      if (lane == j) {
        ok = false;
        eff = 0;
      }
      floor_lane = j;
    }
    if (act && check && (uint32_t)lane <= lim) st_publish(&s.st[e], st_bits(side, amt <= P));
    if (ok) {
      const uint32_t f = rm_field(meta);
      acc[0] += f == 0 ? (u128)amt : (u128)0;
      acc[1] += f == 1 ? (u128)amt : (u128)0;
      acc[2] += f == 2 ? (u128)amt : (u128)0;
      acc[3] += f == 3 ? (u128)amt : (u128)0;
    }
    if (lim > 0) A = i128_shfl(P + eff, (int)lim - 1);
    pos += lim;
    if (lane == 0) DBG_ADD(0, 1);
    if (lim == n) {
      meta = meta_n;
      amt = amt_n;
    } else {
      if (lane == 0) DBG_ADD(1, 1);
      if (!exclusive) break;
      // wait for the blocking lane's other side, then redo the step from there
      const uint32_t eb = (uint32_t)__shfl((int)e, (int)lim, 64);
      const uint32_t sb = (uint32_t)__shfl((int)side, (int)lim, 64);
      if (lim > 0) last = wall_clock64();
      const uint64_t t_spin = wall_clock64();
      while (!(st_load(&s.st[eb]) & st_known(sb ^ 1))) {
        if (res_stalled(g, last)) return false;
        __builtin_amdgcn_s_sleep(1);
      }
      last = wall_clock64();
      if (lane == 0) DBG_ADD(2, last - t_spin);
      meta = 0;
      amt = 0;
      if (start + pos + lane < end) {
        meta = s.rmeta[start + pos + lane];
        amt = (__int128)s.ramt[start + pos + lane];
      }
    }
  }
#pragma unroll
  for (int f = 0; f < 4; f++) acc[f] = u128_wave_sum(acc[f]);
  if (lane == 0) {
    rsp->pos = pos;
    rsp->A = A;
    rsp->d[0] += acc[0];
    rsp->d[1] += acc[1];
    rsp->d[2] += acc[2];
    rsp->d[3] += acc[3];
  }
  *moved = pos != pos0;
  *done = start + pos >= end;
  return true;
}

// Light walker: this lane advances rank `r` one entry at a time until blocked (or budget).
__device__ inline bool lane_advance(const Scratch& s, uint32_t r, uint32_t budget, bool* done) {
  RState* rsp = &s.rstate[r];
  const uint32_t start = rsp->start, end = rsp->end;
  uint32_t pos = rsp->pos;
  const uint32_t pos0 = pos;
  __int128 A = rsp->A;
  u128 d0 = rsp->d[0], d1 = rsp->d[1], d2 = rsp->d[2], d3 = rsp->d[3];
  uint32_t meta_n = 0;
  __int128 amt_n = 0;
  if (start + pos < end) {
    meta_n = s.rmeta[start + pos];
    amt_n = (__int128)s.ramt[start + pos];
  }
  for (uint32_t step = 0; step < budget && start + pos < end; step++) {
    const uint32_t k = start + pos;
    const uint32_t meta = meta_n;
    const __int128 amt = amt_n;
    if (k + 1 < end) {
      meta_n = s.rmeta[k + 1];
      amt_n = (__int128)s.ramt[k + 1];
    }
    const uint32_t e = meta & RM_EVENT;
    const uint32_t side = (meta & RM_SIDE) ? 1u : 0u;
    const bool check = meta & RM_CHECK;
    const bool pass = amt <= A;
    bool opass = true;
    if (meta & RM_WAIT) {
      const uint32_t w = st_load(&s.st[e]);
      if (!(w & st_known(side ^ 1))) {
        if (check) st_publish(&s.st[e], st_bits(side, pass));  // the other side may wait on us
        break;
      }
      opass = w & (side ? ST_DR_PASS : ST_CR_PASS);
    }
    bool ok = opass;
    if (check) {
      st_publish(&s.st[e], st_bits(side, pass));
      ok = ok && pass;
      if (ok) A -= amt;
    } else if (ok && (meta & RM_ADD)) {
      A += amt;
    }
    if (ok) {
      const uint32_t f = rm_field(meta);
      if (f == 0) d0 += (u128)amt;
      else if (f == 1) d1 += (u128)amt;
      else if (f == 2) d2 += (u128)amt;
      else d3 += (u128)amt;
    }
    pos++;
  }
  if (pos != pos0) {
    rsp->pos = pos;
    rsp->A = A;
    rsp->d[0] = d0;
    rsp->d[1] = d1;
    rsp->d[2] = d2;
    rsp->d[3] = d3;
  }
  *done = start + pos >= end;
  return pos != pos0;
}

// Persistent walkers (cooperative launch: all waves co-resident). Waves [0, Ph) walk the heavy
// ranks (each its own if there are few enough), the other waves walk the light ranks, one per lane
// (lane-strided, round-robin when a lane owns several).
__global__ void __launch_bounds__(RES_THREADS) k_res_walk(Dev d, Scratch s) {
  Globals* g = d.g;
  if (g->res_inelig || !g->hot_count || g->res_chunked) return;
  const uint32_t H = g->heavy_count, L = g->light_count;
  const uint32_t P = gridDim.x * (RES_THREADS / 64);
  const uint32_t wave = blockIdx.x * (RES_THREADS / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const uint32_t Ph = min(H, L ? P / 2 : P);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    DBG_ADD(5, H);
    DBG_ADD(6, L);
  }
  uint64_t last = wall_clock64();
  const uint64_t t_begin = last;
  if (wave < Ph) {
    const bool exclusive = H <= Ph;
    for (;;) {
      bool any_left = false, any_moved = false;
      for (uint32_t j = wave; j < H; j += Ph) {
        const uint32_t r = s.heavy[j];
        const RState* rsp = &s.rstate[r];
        if (rsp->start + rsp->pos >= rsp->end) continue;
        bool moved = false, done = false;
        if (!wave_advance(g, s, r, exclusive, RES_BUDGET, &moved, &done)) return;
        any_moved |= moved;
        any_left |= !done;
      }
      if (!any_left) {
        if (lane == 0) DBG_MAX(3, wall_clock64() - t_begin);
        return;
      }
      if (any_moved) {
        last = wall_clock64();
      } else {
        if (res_stalled(g, last)) return;
        __builtin_amdgcn_s_sleep(2);
      }
    }
  }
  const uint32_t PL = P - Ph;
  const uint32_t first = (wave - Ph) * 64 + lane;
  const uint32_t stride = PL * 64;
  for (;;) {
    bool left = false, moved = false;
    for (uint32_t j = first; j < L; j += stride) {
      const uint32_t r = s.light[j];
      const RState* rsp = &s.rstate[r];
      if (rsp->start + rsp->pos >= rsp->end) continue;
      bool done = false;
      if (lane_advance(s, r, RES_LANE_BUDGET, &done)) moved = true;
      if (!done) left = true;
    }
    const bool any_left = __any(left), any_moved = __any(moved);
    if (lane == 0) DBG_ADD(7, 1);
    if (!any_left) {
      if (lane == 0) DBG_MAX(4, wall_clock64() - t_begin);
      return;
    }
    if (any_moved) {
      last = wall_clock64();
    } else {
      if (res_stalled(g, last)) return;
      __builtin_amdgcn_s_sleep(2);
    }
  }
}

// Writes each walked account's summed effects (one owner per account: plain read-modify-write).
__global__ void __launch_bounds__(256) k_res_apply(Dev d, Scratch s) {
  const Globals* g = d.g;
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (g->res_inelig || g->res_error || r >= g->hot_count) return;
  const RState& rs = s.rstate[r];
  if (rs.end == rs.start) return;
  tb_account_t& a = d.acc[rs.slot];
  a.debits_pending = W(U(a.debits_pending) + rs.d[0]);
  a.debits_posted = W(U(a.debits_posted) + rs.d[1]);
  a.credits_pending = W(U(a.credits_pending) + rs.d[2]);
  a.credits_posted = W(U(a.credits_posted) + rs.d[3]);
}

// Final outcomes of the W events from the published checks (unless a wave gave up), folded into
// the per-segment failure / insert counts (a 256-event block lies inside one 1024-event segment).
__global__ void __launch_bounds__(256) k_res_final(Dev d, Scratch s, uint32_t E, uint32_t epoch) {
  __shared__ uint32_t nbad, nins;
  Globals* g = d.g;
  if (g->res_inelig || !g->hot_count || g->res_error) return;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) g->res_done = 1;
  if (threadIdx.x == 0) nbad = nins = 0;
  __syncthreads();
  uint32_t cls = i < E ? s.cls[i] : 0u;
  if (cls & C_W) {
    uint32_t code = s.code[i];
    if (code == TB_CT_OK && (cls & (C_READS_DR | C_READS_CR))) {
      const uint32_t w = s.st[i];
      if ((cls & C_READS_DR) && !(w & ST_DR_PASS))
        code = TB_CT_EXCEEDS_CREDITS;
      else if ((cls & C_READS_CR) && !(w & ST_CR_PASS))
        code = TB_CT_EXCEEDS_DEBITS;
      s.code[i] = code;
    }
    const bool ok = code == TB_CT_OK;
    const bool ins = ok && (cls & C_INSERT);
    s.ins[i] = ins ? 1 : 0;
    cls = (cls & ~C_W) | (ok ? C_COMMIT : 0u) | (ins ? C_INSERTED : 0u);
    if (ok) {
      if (d.hot[s.dr_slot[i]] == epoch) cls |= C_RES_DR;
      if (d.hot[s.cr_slot[i]] == epoch) cls |= C_RES_CR;
    }
    s.cls[i] = cls;
    if (!ok) atomicAdd(&nbad, 1u);
    if (ins) atomicAdd(&nins, 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0 && (nbad | nins)) {
    const uint32_t seg = (blockIdx.x * blockDim.x) / SEG;
    if (nbad) atomicAdd(&s.cnt_bad[seg], nbad);
    if (nins) atomicAdd(&s.cnt_ins[seg], nins);
  }
}
