// cpw.h — component-parallel walking of W (windows where no decision reads a balance).
//
// When no event of the window reads an account balance (no hot account: no limit flag and no
// balancing among the events that reach the balance checks) and the window is overflow-free, the
// only order dependences between W events are through
//   - linked chains (consecutive events, state_machine.zig:1236-1300),
//   - transfer ids: duplicate ids (the exists check, :1487-1490) and pending ids (post/void of a
//     pending transfer created in the window or posted/voided several times, :1616-1680).
// Those links partition W into connected components that are mutually independent: the reference's
// sequential loop restricted to one component yields the same outcomes as the whole loop. Balance
// effects are commutative adds (nothing reads them), applied atomically.
//
// So: union-find over the links (events as nodes; a key's first claimant in the window key map
// stands for the key), a stable sort of W by component root (window order inside a component is
// kept), then one walker thread per component (walker.h in atomic-balance mode, with a private undo
// region). The window's sequential walker is skipped; k_walk only folds the outcomes.
#pragma once
#include "walker.h"
#ifndef CPS_PROF
#define CPS_PROF_WALK_OFF 0
#else
#define CPS_PROF_WALK_OFF CPS_PROF
#endif

__device__ inline bool cpw_active(const Globals* g) {
  // windows with history rows need the exact balances after each event: sequential walker
  return !WIN_REJECTED(g) && !SP_DONE(g) && !g->hot_count && !window_ovf_mode(g) && !(g->win_flags & 16u);
}

__device__ inline uint32_t cc_find(const uint32_t* parent, uint32_t x) {
  for (;;) {
    const uint32_t p = __hip_atomic_load(&parent[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (p == x) return x;
    x = p;
  }
}

// Hooks the larger root under the smaller one (CAS on the root's parent word; retries on races).
__device__ inline void cc_union(uint32_t* parent, uint32_t a, uint32_t b) {
  for (;;) {
    a = cc_find(parent, a);
    b = cc_find(parent, b);
    if (a == b) return;
    if (a < b) {
      const uint32_t t = a;
      a = b;
      b = t;
    }
    if (atomicCAS(&parent[a], a, b) == a) return;
  }
}

__global__ void __launch_bounds__(256) k_cc_init(Dev d, Scratch s, uint32_t E) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    d.g->cc_count = 0;
    d.g->cps_lists = 0;
    d.g->cpw_want &= ~2u;  // (k_cc_walk: a component above CPS_NMAX this window)
  }
  if (i >= E || !cpw_active(d.g)) return;
  s.cc_parent[i] = i;
  s.rkey_in[i] = 0;  // (grouped form: the per-root counts)
}

__global__ void __launch_bounds__(256) k_cc_link(Dev d, Scratch s, WinDesc w, uint32_t epoch) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= w.E || !cpw_active(d.g)) return;
  const uint32_t cls = s.cls[i];
  if (!(cls & C_W)) return;
  if ((cls & C_LINKED) && i + 1 < w.off[s.batch[i] + 1]) cc_union(s.cc_parent, i, i + 1);
  if (!(cls & C_REACH)) return;
  const uint64_t k = s.bmap[s.id_ent[i]].key;
  if (bk_epoch(k) == epoch && bk_owner(k) != i) cc_union(s.cc_parent, i, bk_owner(k));
  if (cls & C_POSTVOID) {
    const uint64_t kp = s.bmap[s.pid_ent[i]].key;
    if (bk_epoch(kp) == epoch && bk_owner(kp) != i) cc_union(s.cc_parent, i, bk_owner(kp));
  }
}

// Sort keys: the component root of each W event (others: past the end).
__global__ void __launch_bounds__(256) k_cc_keys(Dev d, Scratch s, uint32_t E) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= E) return;
  const bool on = cpw_active(d.g) && (s.cls[i] & C_W);
  s.rkey_in[i] = on ? cc_find(s.cc_parent, i) : RES_DUMMY;
  s.rval_in[i] = i;
}

// Component starts in the sorted order, and each component's last sorted position by root
// (Scratch::light: no resolver runs in a component-walked window).
// One counter atomic per 1024-thread block: same-address atomics serialize at the memory side
// (~140K component starts in a cfg4 window; even one per wave cost ~90 us).
__global__ void __launch_bounds__(1024) k_cc_segs(Dev d, Scratch s, uint32_t E) {
  __shared__ uint32_t lds[1024 / 64];
  __shared__ uint32_t base;
  if (!cpw_active(d.g)) return;
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  bool start = false;
  if (k < E) {
    const uint32_t key = s.rkey[k];
    start = key != RES_DUMMY && (k == 0 || s.rkey[k - 1] != key);
    if (key != RES_DUMMY && (k + 1 == E || s.rkey[k + 1] != key)) s.light[key] = k;  // (root < E)
  }
  uint32_t tot;
  const uint32_t r = block_excl<1024 / 64>(start ? 1u : 0u, lds, &tot);
  if (tot == 0) return;
  if (threadIdx.x == 0) base = atomicAdd(&d.g->cc_count, tot);
  __syncthreads();
  if (start) s.cc_list[base + r] = k;
}

// Grouping W by component without a sort (the form used while cps.h takes the long components):
// the W events counted per root, the roots' offsets from one scan, the events scattered to their
// root's segment. A segment's order is then arbitrary; its walker (up to CC_REG events, in registers)
// or its solver (in LDS) orders it by window position before walking. The onesweep sort this
// replaces cost ~170 us per 1M-event window with its fills (k_cc_keys + sort + k_cc_segs).
#define CC_REG 16
__global__ void __launch_bounds__(256) k_cc_count(Dev d, Scratch s, uint32_t E) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= E || !cpw_active(d.g) || !(s.cls[i] & C_W)) return;
  const uint32_t r = cc_find(s.cc_parent, i);
  s.rkey[i] = r;
  atomicAdd(&s.rkey_in[r], 1u);
}

// Per 1024 roots: the number of W events and of components (packed: events | components << 21).
__global__ void __launch_bounds__(1024) k_cc_bsum(Dev d, Scratch s, uint32_t E) {
  __shared__ uint32_t lds[1024 / 64];
  if (!cpw_active(d.g)) return;
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t c = r < E ? s.rkey_in[r] : 0u;
  const uint32_t v = block_sum<1024 / 64>(c | (c ? 1u << 21 : 0u), lds);
  if (threadIdx.x == 0) s.rval_in[E + blockIdx.x] = v;
}

// Each root's segment offset (left in rkey_in as the scatter's cursor) and, per component in root
// order, its start (cc_list) and length (Scratch::light, by component: no resolver runs in a
// component-walked window).
__global__ void __launch_bounds__(1024) k_cc_place(Dev d, Scratch s, uint32_t E) {
  __shared__ uint32_t lds[1024 / 64];
  if (!cpw_active(d.g)) return;
  uint32_t pe = 0, pc = 0;  // W events and components of the earlier blocks' roots
  for (uint32_t b = threadIdx.x; b < blockIdx.x; b += blockDim.x) {
    const uint32_t v = s.rval_in[E + b];
    pe += v & 0x1FFFFFu;
    pc += v >> 21;
  }
  pe = block_sum<1024 / 64>(pe, lds);
  pc = block_sum<1024 / 64>(pc, lds);
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t c = r < E ? s.rkey_in[r] : 0u;
  uint32_t tot;
  const uint32_t ex = block_excl<1024 / 64>(c | (c ? 1u << 21 : 0u), lds, &tot);
  const uint32_t off = pe + (ex & 0x1FFFFFu);
  if (c) {
    const uint32_t j = pc + (ex >> 21);
    s.cc_list[j] = off;
    s.light[j] = c;
    s.rkey_in[r] = off;
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) d.g->cc_count = pc + (tot >> 21);
}

__global__ void __launch_bounds__(256) k_cc_scatter(Dev d, Scratch s, uint32_t E) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= E || !cpw_active(d.g) || !(s.cls[i] & C_W)) return;
  s.rval[atomicAdd(&s.rkey_in[s.rkey[i]], 1u)] = i;
}

// A grouped segment in window order, by its walker thread: up to CC_REG events sorted in registers,
// longer ones (components the solver does not take) by an in-place heap sort.
__device__ inline void cc_order(uint32_t* seg, uint32_t len) {
  if (len <= CC_REG) {
    uint32_t v[CC_REG];
#pragma unroll
    for (int k = 0; k < CC_REG; k++) v[k] = (uint32_t)k < len ? seg[k] : 0xFFFFFFFFu;
#pragma unroll
    for (int size = 2; size <= CC_REG; size <<= 1)
#pragma unroll
      for (int stride = size >> 1; stride > 0; stride >>= 1)
#pragma unroll
        for (int x = 0; x < CC_REG / 2; x++) {
          const int lo = 2 * stride * (x / stride) + (x % stride), hi = lo + stride;
          const bool up = (lo & size) == 0;
          const uint32_t a = v[lo], b = v[hi];
          const bool sw = (a > b) == up;
          v[lo] = sw ? b : a;
          v[hi] = sw ? a : b;
        }
#pragma unroll
    for (int k = 0; k < CC_REG; k++)
      if ((uint32_t)k < len) seg[k] = v[k];
    return;
  }
  auto sift = [&](uint32_t root, uint32_t n) {
    for (;;) {
      uint32_t c = 2 * root + 1;
      if (c >= n) return;
      if (c + 1 < n && seg[c + 1] > seg[c]) c++;
      if (seg[root] >= seg[c]) return;
      const uint32_t t = seg[root];
      seg[root] = seg[c];
      seg[c] = t;
      root = c;
    }
  };
  for (uint32_t r = len / 2; r-- > 0;) sift(r, len);
  for (uint32_t n = len; n > 1; n--) {
    const uint32_t t = seg[0];
    seg[0] = seg[n - 1];
    seg[n - 1] = t;
    sift(0, n - 1);
  }
}

// One walker per component: events rval[start .. start + len), undo records from 5 * start (the
// length from the component's last sorted position, k_cc_segs: no scan of the sorted keys).
// Components of more than solve_min and at most solve_max events are cps.h's (solve_min 0: none).
// grouped: the segments came from k_cc_place / k_cc_scatter (length in light[j], order by cc_order).
template <bool XFER>
__global__ void __launch_bounds__(256) k_cc_walk(Dev d, Scratch s, const uint8_t* ev, WinDesc w, uint32_t epoch,
                                                 uint32_t solve_min, uint32_t solve_max, uint32_t grouped) {
  Globals* g = d.g;
  if (!cpw_active(g)) return;
  __shared__ uint2 pcache[256 * WCACHE];
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j == 0) g->cpw_done = 1;
  const bool on = j < g->cc_count;
  uint32_t start = 0, len = 0;
  if (on) {
    start = s.cc_list[j];
    len = grouped ? s.light[j] : s.light[s.rkey[start]] + 1 - start;
  }
  // statistics (tbg_debug_counters): [5] longest component, [6] components, [7] W events walked;
  // one lane per block adds (same-address atomics from every wave serialize at the memory side)
  __shared__ uint32_t st_mx, st_n, st_sum;
  if (threadIdx.x == 0) st_mx = st_n = st_sum = 0;
  __syncthreads();
  uint32_t mx = len, sum = len;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t y = __shfl_xor(mx, o, 64);
    mx = y > mx ? y : mx;
    sum += __shfl_xor(sum, o, 64);
  }
  const uint32_t n_on = (uint32_t)__popcll(__ballot(on));
  if ((threadIdx.x & 63) == 0 && n_on) {
    atomicMax(&st_mx, mx);
    atomicAdd(&st_n, n_on);
    atomicAdd(&st_sum, sum);
  }
  __syncthreads();
  if (threadIdx.x == 0 && st_n && !CPS_PROF_WALK_OFF) {
    atomicMax((unsigned long long*)&g->dbg[5], (unsigned long long)st_mx);
    atomicAdd((unsigned long long*)&g->dbg[6], (unsigned long long)st_n);
    atomicAdd((unsigned long long*)&g->dbg[7], (unsigned long long)st_sum);
  }
  // a component too long for the solver: the host groups the next window by the sort (its segments
  // come ordered), so a run of such windows pays cc_order's heap sort at most once
  if (on && len > solve_max) atomicOr(&g->cpw_want, 2u);
  if (!on || (solve_min && len > solve_min && len <= solve_max)) return;
  if (grouped) cc_order(s.rval + start, len);
  uint2* mine = pcache + threadIdx.x * WCACHE;
  for (int k = 0; k < WCACHE; k++) mine[k] = make_uint2(NONE32, 0);
  Walker wk;
  wk.pcache = mine;
  wk.d = d;
  wk.s = s;
  wk.s.undo = s.undo + 5ull * start;
  wk.ev = ev;
  wk.w = &w;
  wk.epoch = epoch;
  wk.atomic_bal = true;
  wk.rows = XFER;
  wk.small_bal = g->small_win != 0;  // k_prep_reduce
  wk.template run<XFER>(s.rval + start, len);
}

