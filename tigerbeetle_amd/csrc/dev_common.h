// dev_common.h — device-side layout of the engine's HBM state and the shared primitives.
//
// HBM layout (one engine per GPU):
//   acc_tab  AccEntry[acc_cap]   open-addressing id -> slot table, 32 B entries (id, slot, ledger,
//                                flags): the transfer path resolves an account and checks ledger and
//                                limit flags from this one line, never touching the 128 B record.
//   acc      tb_account_t[]      dense Account records in creation (= timestamp) order.
//   x_tab    XEntry[x_cap]       id -> slot table for transfers, 8 B entries {fingerprint, slot}: one
//                                64-bit CAS inserts; a fingerprint hit is confirmed against the
//                                stored record's id (the caller reads that record anyway).
//   xr       tb_transfer_t[]     dense Transfer records in commit (= timestamp) order.
//   xstatus  u8[]                TransferPending.status per transfer slot (0 = none). Keyed by slot
//                                instead of by timestamp: slot order == timestamp order, 1:1.
//   exp/alt  ExpEntry[]          live pending-with-timeout list (the `expires_at` index).
// Capacities are powers of two with load factor <= 1/2.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tb_types.h"

typedef unsigned __int128 u128;

#define NONE32 0xFFFFFFFFu
#define CONT 0xFFFFFFFFu  // "no result yet, keep evaluating"

static constexpr u128 MAX128 = ~(u128)0;

struct __attribute__((aligned(32))) AccEntry {
  uint64_t id_lo, id_hi;
  uint32_t slot;  // NONE32 = empty
  uint32_t ledger;
  uint16_t flags;
  uint16_t pad0;
  uint32_t pad1;
};
static_assert(sizeof(AccEntry) == 32, "AccEntry");

typedef unsigned long long XEntry;  // [63:32] high half of the id hash, [31:0] record slot
#define X_EMPTY 0xFFFFFFFFFFFFFFFFull  // slot NONE32 never occurs in a live entry

// Window-local key map. Entries are epoch-tagged (the window number), so a stale entry from an
// earlier window reads as empty and nothing is ever reset. Keys are never stored: `key` names the
// first event that claimed the entry (bit 20 says whether the key is that event's id or its
// pending_id), and claims compare against the immutable input events, so there is no
// reader/writer race on a 128-bit key. One 64-bit CAS claims an entry and bumps its counts.
//   key:    [63:32] epoch | [24:23] pid_count (sat. 3) | [22:21] id_count (sat. 3) | [20] pid | [19:0] owner
//   commit: [63:32] epoch | [31:0] walker: index of the in-window event holding this id
struct __attribute__((aligned(16))) BEntry {
  unsigned long long key;
  unsigned long long commit;
};
static_assert(sizeof(BEntry) == 16, "BEntry");

__host__ __device__ inline uint32_t bk_epoch(unsigned long long k) { return (uint32_t)(k >> 32); }
__host__ __device__ inline uint32_t bk_owner(unsigned long long k) { return (uint32_t)k & 0xFFFFFu; }
__host__ __device__ inline uint32_t bk_is_pid(unsigned long long k) { return ((uint32_t)k >> 20) & 1u; }
__host__ __device__ inline uint32_t bk_idc(unsigned long long k) { return ((uint32_t)k >> 21) & 3u; }
__host__ __device__ inline uint32_t bk_pidc(unsigned long long k) { return ((uint32_t)k >> 23) & 3u; }

struct __attribute__((aligned(16))) ExpEntry {
  uint64_t expires_at;
  uint32_t slot;
  uint32_t pad;
};

// Device-global scalars (one cache line each group).
struct __attribute__((aligned(64))) Globals {
  uint64_t acc_count;
  uint64_t x_count;
  uint64_t exp_count;
  uint64_t pulse_next;  // ExpirePendingTransfers.pulse_next_timestamp, exact (k_pn)
  u128 ovf_bound;       // >= every account's dp+dpo and cp+cpo (overflow-free batch test)
  // per batch
  u128 batch_amount_sum;
  uint32_t batch_huge;
  uint32_t epoch;
  uint32_t result_count;
  uint32_t insert_count;
  uint32_t w_count;
  // bit 0: a window was rejected whole because a pulse with expiries would fall due inside it
  // (sticky: every later window is skipped until tbg_sync reports and clears it); bit 1: sharded
  // window outside the class; bit 2: index guard; bit 3: a fused-only window left the class (host.inc
  // settle() replays it and the windows after it)
  uint32_t window_error;
  uint64_t base;  // acc_count / x_count at batch start (captured by the scan kernel)
  // pulse
  uint32_t cand_count;
  uint32_t alt_count;
  uint32_t expired_count;
  uint32_t pulse_done;  // k_pulse blocks finished (the last one runs the pulse's tail), reset by it
  uint64_t next_min;
  // walker statistics (cumulative)
  uint64_t w_events_total;
  uint64_t events_total;
  // account-parallel resolver (resolver.h), per window; reset by k_final's last event
  uint32_t hot_count;   // hot accounts this window (dense ranks 0..hot_count-1)
  uint32_t res_inelig;  // some W event is outside the resolver's class
  uint32_t res_error;   // a resolver wave gave up (bounded spin): the sequential walker runs instead
  uint32_t res_done;    // the resolver decided every W event
  uint32_t heavy_count; // hot ranks walked by a whole wave (long entry lists)
  uint32_t light_count; // hot ranks walked by one lane
  uint64_t res_events_total;  // cumulative W events decided by the resolver
  uint64_t limited_accounts;  // accounts created with a balance-limit flag (cumulative)
  uint64_t dbg[8];            // resolver instrumentation (tbg_debug_counters)
  uint32_t res_bar[8];        // relax.h grid barrier: per-group arrivals (zeroed per window)
  uint32_t res_bar_top;       // groups arrived
  uint32_t res_fc[3];         // first changed event position per iteration (rotating)
  // component-parallel walker (cpw.h), per window; reset by k_final's last event
  uint32_t cc_count;    // components of W
  uint32_t cpw_done;    // the component walkers decided every W event
  uint64_t cpw_events_total;  // cumulative W events decided by component walkers
  uint32_t small_win;   // this window: ovf_bound + window amounts < 2^64 (set by k_walk; k_final reads it)
  uint32_t cold_count;  // hot ranks found non-binding this window (k_bind_decide; k_bind_finish resets)
  // Sorted transfer prefix: records [0, x_sorted) have ids strictly increasing (u128 order) with the
  // slot, and are found by binary search (x_prefix_find; the hash table holds some of them too when a
  // claim-mode fused window extended the prefix: the same slots either way). A window whose
  // ids are strictly increasing and above every stored id extends it instead of hashing its inserts
  // (monotonic ids, the form TigerBeetle recommends); the first other window freezes it.
  uint64_t x_sorted;
  uint32_t win_flags;   // this transfer window (k_prep_reduce): bit 0 claim-free, bit 1 extends the prefix
  uint32_t mono_prev;   // the previous transfer window was claim-free (k_ct_prep's speculation)
  u128 x_id_max;        // >= every stored transfer id (u128 order): an id above it cannot exist, so its
                        // table probe is skipped (strictly increasing ids, 64- or 128-bit)
  uint64_t windows_applied;  // create_* windows applied (rejected windows excluded), cumulative
  uint32_t final_done;  // k_final blocks finished in a window with pulse_next ops (the last runs k_pn)
  uint32_t pad4;
  // chunked resolver (chunks.h), per window: hot accounts left after k_bind_decide (compact ranks
  // 0..hot_live-1) and whether this window's resolver runs in chunked mode
  uint32_t hot_live;
  uint32_t res_chunked;
  uint64_t res_chunk_windows;  // cumulative windows the chunked resolver decided
  uint32_t cpw_want;  // last window: W events in a window the component walkers could take (host readback)
  uint32_t rc_last;   // last window: the chunked resolver decided it (host readback, read with cpw_want)
  // fused pass (fused.h): sp_done = the fused pass committed the current window (the general path's
  // kernels return at once); sp_skip =
  // transfer windows left before the next speculation (exponential back-off after sp_fails misses);
  // fu_abort = epoch of the window a block found outside the class (later blocks skip their work)
  uint32_t sp_done;
  uint32_t sp_skip;
  uint32_t sp_fails;
  uint32_t fu_abort;
  uint32_t fu_epoch;    // the window k_ct_fused ran for (not backed off)
  uint32_t fu_prefix;   // that window extends the sorted prefix (captured before k_fu_final updates it)
  uint64_t fu_base;     // that window's first record slot
  uint64_t cps_lists;  // cps.h this window: components listed, small class | large class << 32 (k_cc_init resets)
  uint64_t fu_windows;  // cumulative windows committed by the fused pass
  uint32_t fu_fail_epoch;  // the fused-only window that left the class (window_error bit 3)
  uint32_t sh_mis;         // sharded: this shard's ledger-mismatch slots used this window (shard.h)
  uint32_t sh_unsup;       // sharded: a home event outside the class this window (k_sh_reply -> trailer 2)
  uint64_t ovf_rescans;    // times ovf_bound was re-tightened to the accounts' largest balance sum (restore.h)
  uint32_t fu_nonmono;     // the epoch of a fused window whose ids did not all rise (claim mode, fused.h)
  uint32_t pad6;
  // fused pass: exp_count as k_ct_fused saw it; the window's live expiry entries go after it
  // (reserved per block in FuScratch::slots, written by k_fu_final)
  uint64_t fu_exp_base;
  uint32_t sh_cap_bad;  // sharded order-free window: some shard's store lacks room for its inserts (k_sh_decide)
  uint32_t fu_done;     // blocks of k_fu_final<true> finished (the last copies the reply out, fused.h)
  uint32_t fu_claim;    // the fused window ran in claim mode (its events claimed their ids in the table)
  uint32_t pad9;
};

// The fused pass (fused.h) committed this window: the general path's kernels return at once.
#define SP_DONE(g) ((g)->sp_done != 0)

// Whether this block is the last of its grid to arrive (every thread of every block calls it once).
// Every thread's earlier writes are released device-wide first, so the last block, after its
// acquire, sees all of them; it resets the counter for the next launch. Costs an agent-scope fence
// per block (an L2 writeback across the XCDs): only for rare paths.
__device__ inline bool last_block_done(uint32_t* counter, uint32_t* flag_lds) {
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t prev = atomicAdd(counter, 1u);
    *flag_lds = prev == gridDim.x - 1 ? 1u : 0u;
    if (*flag_lds) *counter = 0;
  }
  __syncthreads();
  const bool last = *flag_lds != 0;
  if (last) __threadfence();
  return last;
}

// A rejected window (Globals::window_error bit 0) is skipped by every kernel that could change
// state, and so is every window queued after it, until the host has seen the error (tbg_sync). Bit 3:
// a fused-only window left the class (fused.h): every later window is skipped until settle() replays
// them.
#define WIN_REJECTED(g) (__builtin_expect(((g)->window_error & 9u) != 0, 0))

// Per-event class bits (scratch `cls`).
enum : uint32_t {
  C_STATIC = 1u << 0,      // code is final regardless of order/state (validation-stage result)
  C_REACH = 1u << 1,       // reaches the exists check: id entered into the batch map
  C_U = 1u << 2,           // order/state dependent: needs the sequential walker
  C_W = 1u << 3,           // processed by the walker (U, touches a hot account, or chained with one)
  C_LINKED = 1u << 4,
  C_TSNZ = 1u << 5,        // event.timestamp != 0
  C_INSERT = 1u << 6,      // static path: the event inserts its record if it executes (ok or quirk)
  C_PENDING = 1u << 7,     // creates a pending transfer
  C_POSTVOID = 1u << 8,
  C_POST = 1u << 9,
  C_READS_DR = 1u << 10,   // decision reads the debit account's balances
  C_READS_CR = 1u << 11,
  C_PV_PREBATCH = 1u << 12,// post/void whose pending transfer was found in the pre-batch table
  C_COMMIT = 1u << 13,     // final: effects persist (set by the scan kernel)
  C_INSERTED = 1u << 14,   // final: record inserted (ok, or the expired-post quirk)
  C_BAL = 1u << 15,        // balancing_debit or balancing_credit
  C_RES_DR = 1u << 16,     // final: the resolver applied this event's debit-account effects
  C_RES_CR = 1u << 17,     // final: the resolver applied this event's credit-account effects
  C_OWN = 1u << 18,        // sharded: this shard owns the event's id (it inserts the record)
  C_PNOP = 1u << 19,       // pulse_next op candidate (scratch pnv): a pending create with a timeout, or
                           // a post/void of a pending transfer with a timeout (state_machine.zig:1576-1581,
                           // 1704-1708); applies if the event ran ok, even if its chain is rolled back
  C_RANOK = 1u << 20,      // ran ok, then rolled back with its chain (code back-filled linked_event_failed)
  C_HIST = 1u << 21,       // touches an account with flags.history: its history row needs the balances
                           // after it in order, so it runs on the sequential walker
  C_PREP_REC = 1u << 22,   // k_ct_prep stored the stamped record at slot base + i (k_final keeps it if final)
  C_IDALONE = 1u << 23,    // W, transfers: no other event of the window carries this id (k_classify; the
                           // walker skips looking up an earlier commit of it)
};

__host__ __device__ inline uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}
__host__ __device__ inline uint64_t hash_id(uint64_t lo, uint64_t hi) {
  return mix64(lo ^ mix64(hi + 0x9e3779b97f4a7c15ull));
}

__device__ inline u128 U(const tb_uint128_t& v) { return ((u128)v.hi << 64) | v.lo; }
__device__ inline tb_uint128_t W(u128 v) {
  tb_uint128_t r;
  r.lo = (uint64_t)v;
  r.hi = (uint64_t)(v >> 64);
  return r;
}
__device__ inline bool ovf128(u128 a, u128 b) { return a + b < a; }
__device__ inline bool ovf64(uint64_t a, uint64_t b) { return a + b < a; }

// 128-bit atomic add from two 64-bit atomics: the carry out of the low word is computed from the
// value the low-word atomic returned, so concurrent adds compose to the exact 128-bit sum.
__device__ inline void atomic_add_u128(tb_uint128_t* p, u128 v) {
  unsigned long long* w = reinterpret_cast<unsigned long long*>(p);
  const unsigned long long lo = (unsigned long long)v, hi = (unsigned long long)(v >> 64);
  const unsigned long long old = atomicAdd(w, lo);
  const unsigned long long carry = (old + lo) < old ? 1ull : 0ull;
  if (hi + carry) atomicAdd(w + 1, hi + carry);
}
__device__ inline void atomic_sub_u128(tb_uint128_t* p, u128 v) { atomic_add_u128(p, (u128)0 - v); }

// ------------------------------------------------------------------------------------------------
// Table probes (linear probing; thread-per-query; one 32 B entry per probe).
// ------------------------------------------------------------------------------------------------
__device__ inline uint32_t acc_find(const AccEntry* __restrict__ tab, uint64_t mask, tb_uint128_t id,
                                    AccEntry* out) {
  if ((id.lo | id.hi) == 0) return NONE32;
  uint64_t h = hash_id(id.lo, id.hi) & mask;
  for (;;) {
    const AccEntry e = tab[h];
    if (e.slot == NONE32) return NONE32;
    if (e.id_lo == id.lo && e.id_hi == id.hi) {
      *out = e;
      return e.slot;
    }
    h = (h + 1) & mask;
  }
}

// Continues a transfer-id probe whose first entry `e` (at h & mask) is already loaded.
__device__ inline uint32_t x_probe_from(const XEntry* __restrict__ tab, const tb_transfer_t* __restrict__ xr,
                                        uint64_t mask, uint64_t h, XEntry e, tb_uint128_t id) {
  const uint32_t fp = (uint32_t)(h >> 32);
  uint64_t pos = h & mask;
  for (;;) {
    if (e == X_EMPTY) return NONE32;
    if ((uint32_t)(e >> 32) == fp) {
      const tb_uint128_t k = xr[(uint32_t)e].id;
      if (k.lo == id.lo && k.hi == id.hi) return (uint32_t)e;
    }
    pos = (pos + 1) & mask;
    e = tab[pos];
  }
}

__device__ inline uint32_t x_find(const XEntry* __restrict__ tab, const tb_transfer_t* __restrict__ xr, uint64_t mask,
                                  tb_uint128_t id) {
  if ((id.lo | id.hi) == 0) return NONE32;
  const uint64_t h = hash_id(id.lo, id.hi);
  return x_probe_from(tab, xr, mask, h, tab[h & mask], id);
}

__device__ inline double u128_to_double(u128 v) {
  return (double)(uint64_t)(v >> 64) * 18446744073709551616.0 + (double)(uint64_t)v;
}

// Search of the sorted transfer prefix [0, P) (Globals::x_sorted), in u128 id order. The prefix's ids
// are mostly dense runs (sequential ids; time-based ids spread evenly within a millisecond), so a few
// interpolation steps narrow the range to the key's neighbourhood (one step for a dense run) before a
// binary search: a post/void of a prefix transfer no longer pays ~log2(P) dependent loads. Each step
// keeps the invariant that the key, if present, is in [lo, hi).
__device__ inline uint32_t x_prefix_find(const tb_transfer_t* __restrict__ xr, uint64_t P, tb_uint128_t id) {
  if (P == 0) return NONE32;
  const u128 key = U(id);
  u128 a = U(xr[0].id), b = U(xr[P - 1].id);
  if (key < a || key > b) return NONE32;
  if (key == a) return 0;
  if (key == b) return (uint32_t)(P - 1);
  uint64_t lo = 1, hi = P - 1;  // a < key < b
  for (int it = 0; it < 4 && hi - lo > 16; it++) {
    const double f = u128_to_double(key - a) / u128_to_double(b - a);
    uint64_t mid = lo + (uint64_t)(f * (double)(hi - lo));
    if (mid >= hi) mid = hi - 1;
    const u128 km = U(xr[mid].id);
    if (km == key) return (uint32_t)mid;
    if (km < key) {
      lo = mid + 1;
      a = km;
    } else {
      hi = mid;
      b = km;
    }
  }
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (U(xr[mid].id) < key)
      lo = mid + 1;
    else
      hi = mid;
  }
  return (lo < P && U(xr[lo].id) == key) ? (uint32_t)lo : NONE32;
}

// Whether `id` can be in the transfer table (x_id_max bounds every stored id).
__device__ inline bool x_may_exist(const tb_uint128_t& id, u128 x_id_max) { return U(id) <= x_id_max; }
__device__ inline u128 umax128(u128 a, u128 b) { return a > b ? a : b; }
// Wave-wide max of a u128 (every lane gets it).
__device__ inline u128 wave_max_u128(u128 v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t lo = __shfl_xor((unsigned long long)v, o, 64), hi = __shfl_xor((unsigned long long)(v >> 64), o, 64);
    const u128 y = ((u128)hi << 64) | lo;
    v = y > v ? y : v;
  }
  return v;
}

// Inserts of distinct, absent keys: claim by CAS on the slot word, then publish the key. Readers
// run in later kernels only.
__device__ inline void acc_insert(AccEntry* tab, uint64_t mask, tb_uint128_t id, uint32_t slot, uint32_t ledger,
                                  uint16_t flags) {
  uint64_t h = hash_id(id.lo, id.hi) & mask;
  for (;;) {
    if (atomicCAS(&tab[h].slot, NONE32, slot) == NONE32) {
      tab[h].id_lo = id.lo;
      tab[h].id_hi = id.hi;
      tab[h].ledger = ledger;
      tab[h].flags = flags;
      return;
    }
    h = (h + 1) & mask;
  }
}

// Inserts a distinct, absent id whose record is already stored at xr[slot] (readers run in later
// kernels): one 64-bit CAS.
// The fused pass's claim of a transfer id (fused.h, claim mode): walks the id's probe sequence from
// entry e at h. A stored transfer with the id (slot below `base`) is returned; an entry of this
// window's own events (slot base + j, compared against the request's event j) marks an in-window
// duplicate (*dup); at the sequence's first empty entry the event claims it for its own record
// (fp | base + i) when `insert`, and NONE32 is returned.
// *cpos: the position of the event's claim (NONE32: none), where k_fu_final finds it again.
__device__ inline uint32_t x_probe_claim(XEntry* tab, const tb_transfer_t* __restrict__ xr,
                                         const tb_transfer_t* __restrict__ ev, uint64_t mask, uint64_t h, XEntry e,
                                         tb_uint128_t id, uint64_t base, uint32_t i, uint32_t E, bool insert,
                                         bool* dup, uint32_t* cpos) {
  const uint32_t fp = (uint32_t)(h >> 32);
  uint64_t pos = h & mask;
  *dup = false;
  *cpos = NONE32;
  for (;;) {
    if (e == X_EMPTY) {
      if (!insert) return NONE32;
      const XEntry mine = ((unsigned long long)fp << 32) | (uint32_t)(base + i);
      const XEntry seen = atomicCAS(&tab[pos], X_EMPTY, mine);
      if (seen == X_EMPTY) {
        *cpos = (uint32_t)pos;
        return NONE32;
      }
      e = seen;  // another claim took it first: examine that one
      continue;
    }
    if ((uint32_t)(e >> 32) == fp) {
      const uint32_t slot = (uint32_t)e;
      if (slot < base) {
        const tb_uint128_t k = xr[slot].id;
        if (k.lo == id.lo && k.hi == id.hi) return slot;
      } else if (slot - base < E) {
        const tb_uint128_t k = ev[slot - base].id;
        if (k.lo == id.lo && k.hi == id.hi) {
          *dup = true;
          return NONE32;
        }
      }
    }
    pos = (pos + 1) & mask;
    e = tab[pos];
  }
}

__device__ inline void x_insert(XEntry* tab, uint64_t mask, tb_uint128_t id, uint32_t slot) {
  const uint64_t h = hash_id(id.lo, id.hi);
  const XEntry v = ((unsigned long long)(uint32_t)(h >> 32) << 32) | slot;
  uint64_t pos = h & mask;
  for (;;) {
    if (atomicCAS(&tab[pos], X_EMPTY, v) == X_EMPTY) return;
    pos = (pos + 1) & mask;
  }
}

// Block-wide max of a u64 (one LDS word per wave), result valid in every thread.
template <int NWAVES>
__device__ inline unsigned long long block_max_u64(unsigned long long v, unsigned long long* lds) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long y = __shfl_xor(v, o, 64);
    v = y > v ? y : v;
  }
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  unsigned long long m = 0;
#pragma unroll
  for (int k = 0; k < NWAVES; k++) m = lds[k] > m ? lds[k] : m;
  __syncthreads();
  return m;
}
