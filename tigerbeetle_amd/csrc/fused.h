// fused.h — one pass over an order-free create_transfers window (the cfg1 / cfg2 shape: plain
// single-phase transfers with strictly increasing ids between unlimited accounts).
//
// The general path (k_ct_prep -> k_prep_reduce -> k_classify -> k_wlist -> k_walk -> k_final) writes
// ~72 B of scratch columns per event and reads ~40 B of them back, in seven launches. For a window in
// which every outcome is order-free that traffic buys nothing: k_ct_fused decides each event
// (state_machine.zig:1462-1507 validation, lookups, ledgers, create_transfer_exists :1587-1606; the
// balance tail :1509-1547 cannot fail, below), applies its balance effects (:1549-1575) and writes its
// reply and record, in one launch. Ranks (reply slot, record slot) come from a decoupled look-back
// over per-block status words instead of scratch columns.
//
// Simple = every event of the window is either decided statically (validation, lookups, ledgers,
// exists) or is a plain create (no linked / pending / post / void / balancing flag) whose accounts
// carry no limit and no history flag, every id is below 2^64 and strictly increasing over the window
// (so no id repeats: the window is claim-free), and every amount reaching the account checks is below
// 2^43 with the overflow bound below 2^63 (so no balance field leaves its low 64-bit word: the
// overflow checks of :1532-1545 cannot fail, and the balance adds are exact no-return 64-bit adds).
// Then every outcome is a function of the pre-window state and the event alone.
//
// Speculation. Each block applies its balance adds as soon as its own events are simple; whether the
// whole window is simple is known only to the window's last block (its inclusive look-back). If it is
// not, k_fu_post subtracts the adds of every block that applied (recomputing the same decisions from
// the same unchanged inputs: nothing the decisions read is written here), and the general path runs
// the window as if this kernel had not (its record, reply and status stores are all rewritten or
// beyond the store's end). Globals::sp_done tells the general path's kernels to return at once when the
// fused pass committed the window. A window that is not simple backs the speculation off
// exponentially (Globals::sp_skip windows, k_final counts them down).
#pragma once

#define FU_T 256
#define FU_AMOUNT_MAX (1ull << 43)  // per-event amount bound: 2^20 events x 2^43 <= 2^63
// Globals::sp_state after a fused launch (read by k_fu_post)
enum : uint32_t { FU_STATE_NONE = 0, FU_STATE_UNDO = 1, FU_STATE_INSERT = 2 };
// look-back status word per block: [63:32] window epoch | [31:30] state | [29] not simple | [20:0] failures
enum : uint32_t { FU_AGG = 1u, FU_INC = 2u };
#define FU_SPIN_MAX (1u << 22)  // bounded look-back wait (a stuck predecessor fails the speculation)

__device__ __forceinline__ unsigned long long fu_word(uint32_t epoch, uint32_t state, bool not_simple, uint32_t bad) {
  return ((unsigned long long)epoch << 32) | ((unsigned long long)state << 30) | (not_simple ? (1ull << 29) : 0ull) |
         (unsigned long long)(bad & 0x1FFFFFu);
}
__device__ __forceinline__ uint32_t fu_state(unsigned long long w) { return (uint32_t)(w >> 30) & 3u; }
__device__ __forceinline__ bool fu_not_simple(unsigned long long w) { return (w >> 29) & 1ull; }
__device__ __forceinline__ uint32_t fu_bad(unsigned long long w) { return (uint32_t)w & 0x1FFFFFu; }

__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long y = __shfl_xor(v, o, 64);
    v = y > v ? y : v;
  }
  return v;
}

// One event's decision on the fused path. `simple` is cleared when the event puts the window outside
// the class; then the other outputs are meaningless. `ok` events insert and apply `amount` to the
// debit account's debits_posted and the credit account's credits_posted (:1569-1575).
struct FuEv {
  uint32_t code, dr, cr;
  unsigned long long amount;  // C_REACH events: the amount (every one counts toward the overflow bound)
  unsigned long long id_key;  // C_REACH events: the id (x_id_max bound)
  bool simple, reach;
};

__device__ __forceinline__ void fu_decide(const Dev& d, const tb_transfer_t* __restrict__ ev, uint32_t i,
                                          const tb_transfer_t& t, uint64_t x_id_max, uint64_t P, FuEv* o) {
  const uint16_t f = t.flags;
  o->dr = o->cr = NONE32;
  o->amount = 0;
  o->id_key = 0;
  o->reach = false;
  // claim-free: ids strictly increasing over the window, below 2^64, no post/void (k_ct_prep's test)
  bool simple = !(f & TB_TRANSFER_LINKED) && t.id.hi == 0 && !(f & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING));
  if (i > 0) simple = simple && t.id.lo > ev[i - 1].id.lo;
  uint32_t code;
  if (t.timestamp != 0) {
    code = TB_CT_TIMESTAMP_MUST_BE_ZERO;  // :1251
  } else {
    code = ct_head(t);
    if (code == CONT) {
      if (f & (TB_TRANSFER_PENDING | TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING | TB_TRANSFER_BALANCING_DEBIT |
               TB_TRANSFER_BALANCING_CREDIT)) {
        simple = false;
      } else {
        code = ct_validate(t);
        if (code == CONT) {
          // three independent probes in flight together (k_ct_prep)
          const uint64_t hd = hash_id(t.debit_account_id.lo, t.debit_account_id.hi) & d.acc_mask;
          const uint64_t hc = hash_id(t.credit_account_id.lo, t.credit_account_id.hi) & d.acc_mask;
          const bool mx = x_may_exist(t.id, x_id_max);
          const uint64_t hx = hash_id(t.id.lo, t.id.hi);
          const AccEntry ed = d.acc_tab[hd], ec = d.acc_tab[hc];
          const XEntry ex = mx ? d.x_tab[hx & d.x_mask] : X_EMPTY;
          AccEntry de, ce;
          o->dr = acc_probe_from(d.acc_tab, d.acc_mask, hd, ed, t.debit_account_id, &de);
          o->cr = acc_probe_from(d.acc_tab, d.acc_mask, hc, ec, t.credit_account_id, &ce);
          if (o->dr == NONE32)
            code = TB_CT_DEBIT_ACCOUNT_NOT_FOUND;
          else if (o->cr == NONE32)
            code = TB_CT_CREDIT_ACCOUNT_NOT_FOUND;
          else
            code = ct_ledgers(t, de.ledger, ce.ledger);
          if (code == CONT) {
            o->reach = true;
            o->amount = t.amount.lo;
            o->id_key = t.id.lo;
            // a limit or history flag reads (or records) balances in order: not order-free
            if (((de.flags | ce.flags) & TB_ACCOUNT_HISTORY) || (de.flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) ||
                (ce.flags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS) || t.amount.hi != 0 || t.amount.lo >= FU_AMOUNT_MAX)
              simple = false;
            uint32_t xs = mx ? x_probe_from(d.x_tab, d.xr, d.x_mask, hx, ex, t.id) : NONE32;
            if (xs == NONE32 && mx) xs = x_prefix_find(d.xr, P, t.id);
            // :1506-1507; a plain create with timeout 0 cannot overflow the timeout (:1543)
            code = xs != NONE32 ? ct_exists(t, d.xr[xs]) : (uint32_t)TB_CT_OK;
          }
        }
      }
    }
  }
  o->code = code;
  o->simple = simple;
}

// Scratch of the fused pass (per 256-event block; per 64-event wave).
struct FuScratch {
  unsigned long long* st;   // look-back status words
  unsigned long long* pay;  // per block: [4k] aggregate sum, [4k+1] aggregate id max, [4k+2..3] inclusive
  uint8_t* applied;         // per block: its balance adds were applied (k_fu_post undoes them)
  unsigned long long* ok;   // per wave: ok-event bitmap (k_fu_post indexes a non-prefix window's ids)
};

__global__ void __launch_bounds__(FU_T) k_ct_fused(Dev d, FuScratch fs, const tb_transfer_t* __restrict__ ev,
                                                   WinDesc w, uint32_t epoch, FinalOut o) {
  __shared__ uint4 stage[FU_T * 4];     // half of each inserted record per round (16 KiB)
  __shared__ uint32_t lds[FU_T / 64];
  __shared__ unsigned long long ldsu[2 * (FU_T / 64)];
  __shared__ uint32_t sh_ex_bad, sh_ns;
  Globals* g = d.g;
  if (WIN_REJECTED(g)) return;
  if (g->sp_skip) {  // backed off: the general path decides this window
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      g->sp_done = 0;
      g->sp_state = FU_STATE_NONE;
    }
    return;
  }
  const uint32_t k = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t i = k * FU_T + threadIdx.x;
  const uint32_t E = w.E;
  const uint64_t base = g->x_count, x_id_max = g->x_id_max, P = g->x_sorted;
  const u128 ovf = g->ovf_bound;
  // window-level conditions: the balance fields stay below 2^64 (ovf + 2^20 x 2^43 < 2^64)
  const bool glob_ok = (uint64_t)(ovf >> 64) == 0 && (uint64_t)ovf < (1ull << 63) && !g->batch_huge;
  // the window extends the sorted prefix (claim-free when simple; first id above every stored id)
  const bool prefix_win = P == base && ev[0].id.hi == 0 && ev[0].id.lo > x_id_max;
  const bool aborted = __hip_atomic_load(&g->fu_abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;

  tb_transfer_t t;
  FuEv fe;
  fe.simple = true;
  fe.reach = false;
  fe.code = TB_CT_OK;
  fe.amount = fe.id_key = 0;
  fe.dr = fe.cr = NONE32;
  uint32_t b = 0;
  if (i < E && !aborted) {
    t = ev[i];
    b = win_batch(w, i);
    fu_decide(d, ev, i, t, x_id_max, P, &fe);
    t.timestamp = win_ts(w, b, i);  // :1253 (the record as inserted)
  }
  const bool blk_simple = __syncthreads_and(fe.simple) && glob_ok && !aborted;
  const bool ok = i < E && fe.code == TB_CT_OK;
  if (blk_simple && ok) {
    // no-return 64-bit adds: every field stays below 2^64 this window (glob_ok, FU_AMOUNT_MAX)
    (void)atomicAdd(reinterpret_cast<unsigned long long*>(&d.acc[fe.dr].debits_posted), fe.amount);
    (void)atomicAdd(reinterpret_cast<unsigned long long*>(&d.acc[fe.cr].credits_posted), fe.amount);
  }
  if (threadIdx.x == 0) {
    fs.applied[k] = blk_simple ? 1 : 0;
    if (!blk_simple && !aborted) __hip_atomic_store(&g->fu_abort, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const unsigned long long okm = __ballot(ok);
  if (lane == 0 && i < E) fs.ok[i >> 6] = okm;

  // this block's aggregate: failures, the reaching amounts' sum and the largest reaching id
  const bool bad = i < E && !ok;
  const uint32_t inc = wave_incl_scan(bad ? 1u : 0u);
  const unsigned long long wsum = wave_sum_u64(fe.reach ? fe.amount : 0ull);
  const unsigned long long wmax = wave_max_u64(fe.reach ? fe.id_key : 0ull);
  if (lane == 63) lds[wave] = inc;
  if (lane == 0) {
    ldsu[2 * wave] = wsum;
    ldsu[2 * wave + 1] = wmax;
  }
  __syncthreads();
  uint32_t wp = 0, nbad = 0;
  unsigned long long bsum = 0, bmax = 0;
#pragma unroll
  for (uint32_t q = 0; q < FU_T / 64; q++) {
    if (q < wave) wp += lds[q];
    nbad += lds[q];
    bsum += ldsu[2 * q];
    bmax = ldsu[2 * q + 1] > bmax ? ldsu[2 * q + 1] : bmax;
  }

  // Decoupled look-back (wave 0): publish the aggregate, then fold predecessors until an inclusive
  // one. A block outside the class publishes "not simple" as its inclusive state at once (absorbing).
  if (wave == 0) {
    uint32_t ex_bad = 0;
    unsigned long long ex_sum = 0, ex_max = 0;
    bool ns = !blk_simple;
    if (k > 0 && blk_simple) {
      if (lane == 0) {
        st_agent(&fs.pay[4 * k], bsum);
        st_agent(&fs.pay[4 * k + 1], bmax);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // payload before the status word
        st_agent(&fs.st[k], fu_word(epoch, FU_AGG, false, nbad));
      }
      int32_t pos = (int32_t)k - 1;
      uint32_t spins = 0;
      for (;;) {
        const int32_t j = pos - (int32_t)lane;
        const unsigned long long wd = j >= 0 ? ld_agent(&fs.st[j]) : fu_word(epoch, FU_INC, false, 0);
        const bool ready = (uint32_t)(wd >> 32) == epoch && fu_state(wd) != 0;
        const unsigned long long mready = __ballot(ready);
        const unsigned long long minc = __ballot(ready && fu_state(wd) == FU_INC);
        const uint32_t nready = mready == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~mready);
        const unsigned long long in_prefix = nready == 64u ? ~0ull : ((1ull << nready) - 1ull);
        if (minc & in_prefix) {
          const uint32_t f = (uint32_t)__builtin_ctzll(minc & in_prefix);
          const bool take = lane <= f;
          if (__ballot(take && fu_not_simple(wd))) {
            ns = true;
          } else {
            uint32_t vb = take ? fu_bad(wd) : 0u;
            unsigned long long vs = 0, vm = 0;
            if (take && j >= 0) {
              const uint32_t off = lane == f ? 2u : 0u;  // the inclusive payload of the closest inclusive
              vs = ld_agent(&fs.pay[4 * j + off]);
              vm = ld_agent(&fs.pay[4 * j + off + 1]);
            }
            ex_bad += wave_sum(vb);
            ex_sum += wave_sum_u64(vs);
            const unsigned long long mm = wave_max_u64(vm);
            ex_max = mm > ex_max ? mm : ex_max;
          }
          break;
        }
        if (nready == 64u) {  // 64 aggregates: fold them and look further back
          if (__ballot(fu_not_simple(wd))) {
            ns = true;
            break;
          }
          const unsigned long long vs = ld_agent(&fs.pay[4 * j]), vm = ld_agent(&fs.pay[4 * j + 1]);
          ex_bad += wave_sum(fu_bad(wd));
          ex_sum += wave_sum_u64(vs);
          const unsigned long long mm = wave_max_u64(vm);
          ex_max = mm > ex_max ? mm : ex_max;
          pos -= 64;
          continue;
        }
        if (++spins > FU_SPIN_MAX) {  // never expected: fail the speculation instead of hanging
          ns = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (lane == 0) {
      const uint32_t tot_bad = ex_bad + nbad;
      if (!ns) {
        st_agent(&fs.pay[4 * k + 2], ex_sum + bsum);
        st_agent(&fs.pay[4 * k + 3], ex_max > bmax ? ex_max : bmax);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      st_agent(&fs.st[k], fu_word(epoch, FU_INC, ns, tot_bad));
      sh_ex_bad = ex_bad;
      sh_ns = ns ? 1u : 0u;
      if (k == gridDim.x - 1) {
        // the window's last block: its inclusive state is the window's
        if (!ns) {
          const uint32_t total_ins = E - tot_bad;
          for (int32_t bb = (int32_t)w.nb; bb >= 0 && w.off[bb] == E; bb--) o.batch_base[bb] = tot_bad;
          if (o.out_count) *o.out_count = tot_bad;
          g->result_count = tot_bad;
          g->base = base;
          if (prefix_win) g->x_sorted = base + total_ins;
          g->x_count = base + total_ins;
          g->win_flags = 1u | (prefix_win ? 2u : 0u);
          g->mono_prev = 1;
          g->ovf_bound = ovf + (u128)(ex_sum + bsum);
          const unsigned long long idm = ex_max > bmax ? ex_max : bmax;
          if (idm > g->x_id_max) g->x_id_max = idm;
          g->windows_applied++;
          g->events_total += E;
          g->w_count = 0;
          g->cpw_want = 0;
          g->rc_last = 0;
          g->sp_done = 1;
          g->sp_fails = 0;
          g->sp_state = prefix_win ? FU_STATE_NONE : FU_STATE_INSERT;
          g->fu_windows++;
        } else {
          g->sp_done = 0;
          g->sp_state = FU_STATE_UNDO;
          const uint32_t fails = g->sp_fails + 1;
          g->sp_fails = fails;
          g->sp_skip = fails >= 12 ? 4096u : (1u << fails);
        }
      }
    }
  }
  __syncthreads();
  if (sh_ns) return;  // not simple so far: the general path rewrites everything this window

  // Replies and records at their ranks (every event either fails or inserts).
  const uint32_t rbad = sh_ex_bad + wp + inc - (bad ? 1u : 0u);
  const uint32_t rins = i - rbad;
  if (i < E) {
    if (i == w.off[b]) {
      // event i opens batch b and every empty batch just before it
      for (int32_t bb = (int32_t)b; bb >= 0 && w.off[bb] == i; bb--) o.batch_base[bb] = rbad;
    }
    if (bad) {
      tb_create_result_t r;
      r.index = i - w.off[b];
      r.result = fe.code;
      o.results[rbad] = r;
    }
    if (ok) d.xstatus[base + rins] = 0;
  }
  // this wave's inserted records as one contiguous run through LDS, in two halves of 64 B
  if (okm) {
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)rins, (int)__builtin_ctzll(okm));
    const uint32_t nins = (uint32_t)__popcll(okm);
    const uint32_t pos = ok ? (uint32_t)__popcll(okm & ((1ull << lane) - 1ull)) : 0u;
    uint4* ws = stage + wave * 256;
    const uint4* src = reinterpret_cast<const uint4*>(&t);
    uint4* dst = reinterpret_cast<uint4*>(d.xr + (base + r0));
#pragma unroll
    for (int half = 0; half < 2; half++) {
      wave_sync();
      if (ok) {
#pragma unroll
        for (int q = 0; q < 4; q++) ws[pos * 4 + q] = src[half * 4 + q];
      }
      wave_sync();
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const uint32_t idx = c * 64 + lane, r = idx >> 2, q = idx & 3;
        if (r < nins) st_stream(dst + r * 8 + half * 4 + q, ws[idx]);
      }
    }
  }
}

// After k_ct_fused (same grid): a window outside the class gets the balance adds of every block that
// applied them subtracted (the same decisions from the same inputs); a committed window whose records
// do not extend the sorted prefix gets its ids indexed.
__global__ void __launch_bounds__(FU_T) k_fu_post(Dev d, FuScratch fs, const tb_transfer_t* __restrict__ ev,
                                                  uint32_t E, uint32_t epoch) {
  Globals* g = d.g;
  if (WIN_REJECTED(g)) return;
  const uint32_t state = g->sp_state;
  if (state == FU_STATE_NONE) return;
  const uint32_t k = blockIdx.x, i = k * FU_T + threadIdx.x;
  if (state == FU_STATE_UNDO) {
    if (!fs.applied[k] || i >= E) return;
    FuEv fe;
    fu_decide(d, ev, i, ev[i], g->x_id_max, g->x_sorted, &fe);
    if (fe.code == TB_CT_OK) {
      (void)atomicAdd(reinterpret_cast<unsigned long long*>(&d.acc[fe.dr].debits_posted), 0ull - fe.amount);
      (void)atomicAdd(reinterpret_cast<unsigned long long*>(&d.acc[fe.cr].credits_posted), 0ull - fe.amount);
    }
    return;
  }
  // FU_STATE_INSERT: ranks from the look-back's inclusive failure counts
  __shared__ uint32_t lds[FU_T / 64];
  const bool ok = i < E && ((fs.ok[i >> 6] >> (threadIdx.x & 63)) & 1ull);
  const uint32_t ex_bad = k ? fu_bad(fs.st[k - 1]) : 0u;
  uint32_t tot;
  const uint32_t rb = block_excl<FU_T / 64>((i < E && !ok) ? 1u : 0u, lds, &tot);
  if (ok) x_insert(d.x_tab, d.x_mask, ev[i].id, (uint32_t)(g->base + (i - ex_bad - rb)));
}
