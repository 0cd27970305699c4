// window.h — a commit window: up to MAXB consecutive prepared batches processed by one pass of the
// kernels (super-batching). Batches keep their own commit timestamp T_b (events stamped
// T_b - n_b + j + 1, state_machine.zig:1253), their own chain structure (chains never cross a batch
// end: the last linked event of a batch is linked_event_chain_open, :1247) and their own reply
// (results are emitted per batch in ascending event order, :1289-1290).
#pragma once
#include "dev_common.h"

#define MAXB 128
#define SEG 1024          // events per segment = threads per segment block (one event each)

struct WinDesc {
  uint32_t nb;             // batches in the window
  uint32_t E;              // events in the window
  uint32_t off[MAXB + 1];  // event offset of each batch; off[nb] = E
  uint32_t xwin;           // pulses inside the window are modelled (xwin.h): it spans >= 1 s
  uint32_t log;            // TBG_WINDOW_LOG: batches from a replica's log, no pulse between them
  uint32_t bsz;            // nonzero: every batch but the last has bsz events, the last at most bsz
  uint64_t T[MAXB];        // commit timestamp of each batch
};

// WinDesc::bsz from the offsets (host): the common shape of a window of full batches, so that an
// event's batch is a division rather than a binary search over off[] (eight dependent loads from the
// kernel arguments per event).
inline void win_set_bsz(WinDesc* w) {
  w->bsz = 0;
  const uint32_t n0 = w->off[1] - w->off[0];
  if (n0 == 0) return;
  for (uint32_t b = 1; b + 1 < w->nb; b++)
    if (w->off[b + 1] - w->off[b] != n0) return;
  if (w->E - w->off[w->nb - 1] > n0) return;
  w->bsz = n0;
}

// The first batch of the window whose pulse check (T_b >= expires_at) finds an entry due: the pulse
// that expires it (xwin.h; MAXB = window's nb when none).
__device__ inline uint32_t xw_due(const WinDesc& w, uint64_t expires_at) {
  uint32_t lo = 0, hi = w.nb;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (w.T[mid] >= expires_at) hi = mid; else lo = mid + 1;
  }
  return lo;
}

__device__ inline uint32_t win_batch(const WinDesc& w, uint32_t i) {
  if (w.bsz) {
    const uint32_t b = i / w.bsz;
    return b < w.nb ? b : w.nb - 1;
  }
  uint32_t lo = 0, hi = w.nb - 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (w.off[mid] <= i)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

__device__ inline uint64_t win_ts(const WinDesc& w, uint32_t b, uint32_t i) {
  const uint32_t n = w.off[b + 1] - w.off[b];
  return w.T[b] - n + (i - w.off[b]) + 1;
}

enum : uint32_t { UNDO_BAL = 1, UNDO_XST, UNDO_BST, UNDO_COMMIT, UNDO_INS, UNDO_ADD };
struct __attribute__((aligned(16))) UndoRec {
  uint32_t kind, a, pad0, pad1;
  u128 old[4];
};

// account_balances groove row (state_machine.zig:296-315) of one transfer, beside its record: the
// dr and cr accounts' balances after the transfer (historical_balance, :1806-1841); Dev::hist_side
// says which sides are present (bit 0 dr, bit 1 cr: the accounts with flags.history).
struct HistRow {
  u128 dr[4];  // debits_pending, debits_posted, credits_pending, credits_posted
  u128 cr[4];
};
static_assert(sizeof(HistRow) == 128, "HistRow");

struct Dev {
  AccEntry* acc_tab;
  uint64_t acc_mask;
  tb_account_t* acc;
  uint32_t* hot;  // per account slot: epoch of the last window that marked it hot
  uint32_t* hot_rank;  // per account slot: its dense rank among this window's hot accounts
  XEntry* x_tab;
  uint64_t x_mask;
  tb_transfer_t* xr;
  uint8_t* xstatus;
  ExpEntry* exp[2];
  uint32_t* exp_cur;  // device word selecting the live expiry buffer
  Globals* g;
  uint64_t acc_max, x_max;  // store capacities (records)
  HistRow* hist;            // per transfer slot (unsharded engines)
  uint8_t* hist_side;       // per transfer slot: sides present in hist (0 = no row)
};

struct Scratch {
  uint32_t *code, *cls, *dr_slot, *cr_slot, *id_tslot, *p_tslot, *id_ent, *pid_ent, *wlist;
  // create_transfers: the columns a walker reads per event, also as one 32 B row (k_ct_prep,
  // k_claim_fix): {code, id_tslot, id_ent, pid_ent}, {dr_slot, cr_slot, p_tslot, batch}. A component
  // walker reads each event's row with one request instead of eight column loads.
  uint4* wrow;
  uint16_t* batch;
  uint8_t *ins, *bstatus;
  u128 *amt, *pamt;
  tb_transfer_t* t2;
  BEntry* bmap;
  uint32_t bmask;
  UndoRec* undo;
  uint32_t *cnt_w, *cnt_bad, *cnt_ins;  // per segment
  // per-block partials reduced by one small kernel (no same-address atomics across blocks)
  u128* blk_amt;                   // prep blocks: sum of the window's amounts
  uint32_t* blk_aux;               // prep blocks: bit 0 huge amount, bit 1 unsupported (sharded), own << 2
  u128* blk_idmax;                 // prep blocks: largest id that reaches the exists check (x_id_max)
  ExpEntry* cand;
  // account-parallel resolver (resolver.h)
  uint32_t *rkey_in, *rval_in, *rkey, *rval;  // (hot rank, 2*event+side) pairs, then sorted by rank
  uint32_t* rmeta;                            // sorted entries: event | side | check | wait
  u128* ramt;                                 // sorted entries: amount
  struct RState* rstate;                      // per hot rank: segment, cursor, available balance
  uint32_t* st;                               // per event: published limit-check outcomes
  __int128* racc;                             // relax.h: available balance after each sorted entry
  uint32_t* kidx;                             // relax.h: per (event, side): its sorted entry (or NONE)
  uint32_t *rown, *roth;                      // relax.h: per sorted entry: own / other side's check
  uint2* rlink;                               // relax.h: per sorted entry: other side's entry and rank
  uint32_t *heavy, *light;                    // hot ranks by walker kind
  uint32_t *cc_parent, *cc_list;              // component-parallel walker (cpw.h)
  // non-binding limits (k_bind_*): per hot rank its account slot and the adverse sum of the window
  // (debits of a debits<=credits account, credits of a credits<=debits one; bit 63 = must stay hot)
  uint32_t* bind_slot;
  unsigned long long* bind_adv;
  // chunked resolver (chunks.h): the end of each 1024-event chunk's hot entries, and the per-chunk
  // tables k_rc_build builds (segment of each entry, segment starts, walk lists, entry of each event
  // side, counts)
  uint32_t* rc_cb;
  uint16_t *rc_segof, *rc_seg, *rc_srank, *rc_list, *rc_ent, *rc_em;
  uint4* rc_cnt;
  // pulse_next (k_pn): per event the op's value (C_PNOP) and, for a walker post/void of a pending
  // transfer created in the window, that transfer's event index; per segment the min creation value
  // and the count of resets among the events that ran ok
  uint64_t* pnv;
  uint32_t* pn_src;
  // history rows of the walker's inserts (k_final copies them to Dev::hist)
  HistRow* hrow;
  uint8_t* hside;
  // windows with pulses inside (xwin.h): per in-window pending creation, the batch of the committed
  // post/void that removed it; per batch: due counts, minimum live expires_at after its pulse
  // (segment tree over MAXB leaves), minimum creation expiry and reset candidate
  uint16_t* pn_rb;
  uint32_t* xw_cnt;             // [MAXB]
  unsigned long long* xw_tree;  // [2 * MAXB]
  unsigned long long* xw_minx;  // [MAXB]
  unsigned long long* xw_ccnt;  // [MAXB] reset candidates per batch (k_xwin_pm)
  unsigned long long* xw_miny;  // [MAXB]
  uint64_t* pn_min;
  uint32_t* pn_res;
  void* sort_tmp;
  size_t sort_tmp_bytes;
};

// Wave-scope LDS ordering: this wave's LDS writes are visible to all of its lanes after the call.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ------------------------------------------------------------------------------------------------
// Scan helpers (wave64 shuffles + one LDS word per wave).
// ------------------------------------------------------------------------------------------------
// Inclusive wave64 scan with DPP row shifts and row broadcasts (six VALU adds, no LDS round trip:
// a __shfl is a ds_bpermute through the LDS unit).
__device__ inline uint32_t wave_incl_scan(uint32_t v) {
  int32_t x = (int32_t)v;
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return (uint32_t)x;
}

__device__ inline uint32_t wave_sum(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(v), 63);
}

// Exclusive prefix over the threads of a block of `nwaves` waves; *total = block sum.
template <int NWAVES>
__device__ inline uint32_t block_excl(uint32_t v, uint32_t* lds, uint32_t* total) {
  const uint32_t inc = wave_incl_scan(v);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 63) lds[wave] = inc;
  __syncthreads();
  uint32_t wp = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < NWAVES; k++) {
    const uint32_t x = lds[k];
    if (k < wave) wp += x;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return wp + inc - v;
}

template <int NWAVES>
__device__ inline uint32_t block_sum(uint32_t v, uint32_t* lds) {
  v = wave_sum(v);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) lds[wave] = v;
  __syncthreads();
  uint32_t tot = 0;
#pragma unroll
  for (int k = 0; k < NWAVES; k++) tot += lds[k];
  __syncthreads();
  return tot;
}

// Sum of per-segment counts cnt[0..seg) (the segment's global exclusive offset), for a block of
// NTHREADS threads.
template <int NTHREADS>
__device__ inline uint32_t seg_prefix(const uint32_t* cnt, uint32_t seg, uint32_t* lds) {
  uint32_t v = 0;
  for (uint32_t j = threadIdx.x; j < seg; j += NTHREADS) v += cnt[j];
  return block_sum<NTHREADS / 64>(v, lds);
}
