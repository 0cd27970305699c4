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
  if (i == 0) d.g->cc_count = 0;
  if (i >= E || !cpw_active(d.g)) return;
  s.cc_parent[i] = i;
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

// One walker per component: events rval[start .. start + len), undo records from 5 * start (the
// length from the component's last sorted position, k_cc_segs: no scan of the sorted keys).
template <bool XFER>
__global__ void __launch_bounds__(256) k_cc_walk(Dev d, Scratch s, const uint8_t* ev, WinDesc w, uint32_t epoch) {
  Globals* g = d.g;
  if (!cpw_active(g)) return;
  __shared__ uint2 pcache[256 * WCACHE];
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j == 0) g->cpw_done = 1;
  const bool on = j < g->cc_count;
  uint32_t start = 0, len = 0;
  if (on) {
    start = s.cc_list[j];
    len = s.light[s.rkey[start]] + 1 - start;
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
  if (threadIdx.x == 0 && st_n) {
    atomicMax((unsigned long long*)&g->dbg[5], (unsigned long long)st_mx);
    atomicAdd((unsigned long long*)&g->dbg[6], (unsigned long long)st_n);
    atomicAdd((unsigned long long*)&g->dbg[7], (unsigned long long)st_sum);
  }
  if (!on) return;
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

