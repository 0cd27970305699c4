// route.h — hash-sharded commit with partitioned ingestion: each GPU takes only its home slice of a
// window, and three all-to-alls over xGMI carry what the other shards must know ("scatter
// half-events to dr-owner / cr-owner / id-owner; owners evaluate their side's checks; all-to-all back;
// commit: owners apply only admitted events").
//
// Ownership as in shard.h: an account lives on shard_of(account id), a transfer on shard_of(transfer
// id). Shard r is the HOME of the contiguous batches [hb[r], hb[r+1]) of the window (rank order =
// batch order) and holds only their events. Per window:
//
//   k_rt_route1   home, one event per thread: timestamp stamped (state_machine.zig:1253), the
//                 validation that needs no state (:1424-1439, 1465-1489), the owners of the id and of
//                 both accounts; per block the messages per destination shard
//   k_rt_scan     home, one workgroup: every destination's message offsets per block (order-preserving),
//                 the A headers (message counts, the slice's first and last id), the home verdicts
//   k_rt_route2   home: the messages, in event order per destination: the stamped 128 B record to the
//                 id owner, a 32 B side {account id, amount, side} to each account owner
//   (caller)      exchange A: all-to-all of the message blocks (RCCL grouped send/recv over xGMI)
//   k_rt_own      owner, one message per thread: the id owner claims the id when the window's ids are
//                 not known to rise (in-window duplicates) and compares it with a stored transfer or
//                 account (`exists`, :1506-1507, 1450-1460); an account owner resolves the account (found,
//                 its ledger, a limit or history flag) and keeps its slot. One reply per message
//   (caller)      exchange B: all-to-all of the replies back to the homes (1 B per id, 8 B per side)
//   k_rt_decide   home: every home event's code from its replies, in the reference's order (account
//                 lookups :1496-1497, ledgers :1503-1504, exists :1506-1507), linked chains
//                 (:1240-1300; a chain never crosses a batch, so never a home); one commit byte per
//                 message and, per destination, the committed records per 1024-message chunk
//   (caller)      exchange C: all-to-all of the commit bytes to the owners
//   k_rt_apply    home replies (ascending index per batch); owners: balance adds of committed sides,
//                 committed records appended in (home, event) order = timestamp order
//
// Every header carries a verdict word; each home ORs every owner's verdict (B) with its own into its C
// header, and every shard ORs the G C headers it receives: the same verdict everywhere before anything
// is applied. The class is shard.h's order-free one (no limit/history flag on a committed event's
// accounts, no balancing / pending / post / void, no in-window duplicate id, amounts below 2^64, no
// bound overflow, room in every store, every destination block within its capacity). A window outside
// it changes nothing on any shard (TBG_E_UNSUPPORTED at tbg_sync); the caller gathers the whole window
// and commits it through the general path.
#pragma once
#include "shard.h"

#define RT_MAXG 16
#define RT_T 1024       // k_rt_apply's block (= SEG: the home replies' segments); k_rt_own / k_rt_decide use 256
#define RT_RT 256       // k_rt_route1 / k_rt_route2's block (small blocks: a shard's slice fills the chip)
#define RT_CHUNK 1024   // committed-record counts per chunk of id messages (one k_rt_apply block each)
#define RT_HDR_A 256u   // bytes
#define RT_HDR_B 64u
#define RT_HDR_C 64u

// Verdict bits (headers; any bit on any shard rejects the window on every shard).
enum : uint32_t {
  RV_DUP = 1,       // in-window duplicate id
  RV_CAP = 2,       // a store without room, or a destination block past its capacity
  RV_OVF = 4,       // the overflow bound could not hold the window
  RV_UNSUP = 8,     // pending / balancing / post / void, or a committed event reading a balance
  RV_HUGE = 16,     // an amount of 2^64 or more
  RV_PULSE = 32,    // a pulse falls due inside the window
};

// Block header of exchange A (home s -> owner), 256 B.
struct RtHdrA {
  uint32_t n_id, n_side;  // messages in the block
  uint32_t n_home;        // events of the sender's home slice
  uint32_t flags;         // bit 0: the slice's ids are not strictly increasing; bit 1: the slice is not empty
  uint64_t first_lo, first_hi, last_lo, last_hi;  // the slice's first and last transfer id
};
enum : uint32_t { RH_NONMONO = 1, RH_NONEMPTY = 2 };

// Side message (home -> account owner), 32 B.
struct RtSide {
  uint64_t id_lo, id_hi;
  uint64_t amount;  // the class keeps every amount below 2^64 (RV_HUGE otherwise)
  uint32_t side;    // 0 debit, 1 credit
  uint32_t pad;
};
static_assert(sizeof(RtSide) == 32, "RtSide");
// Its reply (owner -> home), 8 B: the account's ledger and state.
enum : uint32_t { RS_FOUND = 1, RS_LIMIT = 2 };  // RS_LIMIT: the side's limit flag or flags.history
// id reply byte: 1 + code (bits 0-5), RI_DUP: an earlier message of the window claimed the id
enum : uint32_t { RI_CODE = 0x3F, RI_DUP = 0x40 };

// The window's geometry, the same on every shard: per shard (as a home) its events and its per-destination
// capacities. Everything else (block sizes, offsets) derives from these.
struct RtLayout {
  uint32_t G, me;
  uint32_t xfer;
  uint32_t own_j;        // received messages per k_rt_own thread (1 or RT_OWN_J; local to the shard)
  uint32_t n[RT_MAXG];   // home events
  uint32_t c1[RT_MAXG];  // id messages per destination block (capacity)
  uint32_t c2[RT_MAXG];  // side messages per destination block
};

__host__ __device__ inline uint64_t rt_al16(uint64_t x) { return (x + 15) & ~15ull; }
__host__ __device__ inline uint32_t rt_cap1(uint32_t n, uint32_t G) {
  if (n == 0) return 0;
  const uint64_t c = (uint64_t)n / G + (uint64_t)n / (8ull * G) + 256;
  return (uint32_t)rt_al16(c < n ? c : n);
}
__host__ __device__ inline uint32_t rt_cap2(uint32_t n, uint32_t G, bool xfer) {
  if (!xfer || n == 0) return 0;
  const uint64_t c = 2ull * n / G + 2ull * n / (8ull * G) + 256;
  return (uint32_t)rt_al16(c < 2ull * n ? c : 2ull * n);
}
__host__ __device__ inline uint32_t rt_nch(uint32_t c1) { return (c1 + RT_CHUNK - 1) / RT_CHUNK; }
// Block bytes of the three exchanges, by the HOME shard s they belong to.
__host__ __device__ inline uint64_t rt_blk_a(const RtLayout& L, uint32_t s) {
  return RT_HDR_A + (uint64_t)L.c1[s] * 128 + (uint64_t)L.c2[s] * 32;
}
__host__ __device__ inline uint64_t rt_b_side(const RtLayout& L, uint32_t s) { return RT_HDR_B + rt_al16(L.c1[s]); }
__host__ __device__ inline uint64_t rt_blk_b(const RtLayout& L, uint32_t s) { return rt_b_side(L, s) + (uint64_t)L.c2[s] * 8; }
__host__ __device__ inline uint64_t rt_c_hdr(const RtLayout& L, uint32_t s) { return RT_HDR_C + rt_al16(4ull * rt_nch(L.c1[s])); }
__host__ __device__ inline uint64_t rt_c_side(const RtLayout& L, uint32_t s) { return rt_c_hdr(L, s) + rt_al16(L.c1[s]); }
__host__ __device__ inline uint64_t rt_blk_c(const RtLayout& L, uint32_t s) { return rt_c_side(L, s) + rt_al16(L.c2[s]); }
// Offsets of the blocks from / to shard s where the blocks are concatenated in shard order and belong to
// different homes (A recv, B send, C recv): sum of the earlier homes' block sizes.
__host__ __device__ inline uint64_t rt_off_a(const RtLayout& L, uint32_t s) {
  uint64_t o = 0;
  for (uint32_t k = 0; k < s; k++) o += rt_blk_a(L, k);
  return o;
}
__host__ __device__ inline uint64_t rt_off_b(const RtLayout& L, uint32_t s) {
  uint64_t o = 0;
  for (uint32_t k = 0; k < s; k++) o += rt_blk_b(L, k);
  return o;
}
__host__ __device__ inline uint64_t rt_off_c(const RtLayout& L, uint32_t s) {
  uint64_t o = 0;
  for (uint32_t k = 0; k < s; k++) o += rt_blk_c(L, k);
  return o;
}
// Flat indices of the messages an owner receives: src s's ids at [id_base(s), + c1[s]), sides likewise.
__host__ __device__ inline uint32_t rt_id_base(const RtLayout& L, uint32_t s) {
  uint32_t o = 0;
  for (uint32_t k = 0; k < s; k++) o += L.c1[k];
  return o;
}
__host__ __device__ inline uint32_t rt_side_base(const RtLayout& L, uint32_t s) {
  uint32_t o = 0;
  for (uint32_t k = 0; k < s; k++) o += L.c2[k];
  return o;
}

// The engine's routed-commit buffers (allocated at the first routed window, sized for window_events_max).
struct RtBufs {
  uint8_t *a_send, *a_recv, *b_send, *b_recv, *c_send, *c_recv;
  uint32_t* cnt;    // [nblk][RT_MAXG][2] messages per destination and kind, per k_rt_route1 block
  uint32_t* boff;   // the same, exclusive offsets (k_rt_scan)
  uint32_t* aux;    // per k_rt_route1 block: verdict bits | RH_NONMONO << 8
  uint32_t* side_slot;      // owner: per received side message, the account slot (NONE32: missing)
  unsigned long long* claim;  // owner: in-window duplicate ids, {epoch, flat id message}
  uint32_t claim_mask;
  unsigned long long* amt;  // owner: 64 slots x {low 32 bits, the rest} of the received amounts' sum
  uint32_t* hv;             // [0] the home verdict (k_rt_scan -> k_rt_decide)
  u128* imax;               // owner: per k_rt_own id block, the largest received transfer id
};

__device__ inline uint32_t rt_lane_lt(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// Owner-side claim of a transfer / account id among the window's id messages: *dup when an earlier
// claimant (any message of this window: the first to CAS wins, the rest see the duplicate) holds it.
// Entries {epoch << 32 | flat index}; a stale epoch reads as empty.
__device__ inline bool rt_claim(unsigned long long* map, uint32_t mask, uint32_t epoch, uint32_t flat, tb_uint128_t id,
                                const uint8_t* a_recv, const RtLayout& L) {
  uint32_t h = (uint32_t)hash_id(id.lo, id.hi) & mask;
  const unsigned long long mine = ((unsigned long long)epoch << 32) | flat;
  for (;;) {
    unsigned long long old = __hip_atomic_load(&map[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t)(old >> 32) != epoch) {
      const unsigned long long prev = atomicCAS(&map[h], old, mine);
      if (prev == old) return false;
      old = prev;
      if ((uint32_t)(old >> 32) != epoch) continue;  // (another stale value: retry the CAS)
    }
    // an entry of this window: compare its id (the claimant's record in the A recv buffer)
    uint32_t f = (uint32_t)old, s = 0;
    while (s + 1 < L.G && f >= L.c1[s]) f -= L.c1[s++];
    const uint64_t* rec = reinterpret_cast<const uint64_t*>(a_recv + rt_off_a(L, s) + RT_HDR_A + (uint64_t)f * 128);
    if (rec[0] == id.lo && rec[1] == id.hi) return true;
    h = (h + 1) & mask;
  }
}

// ------------------------------------------------------------------------------------------------
// k_rt_route1 (home): stamps, static validation, owners; per block the messages per destination.
// Scratch: code (static code or CONT), cls (owners | flags), id_tslot (the event's ledger).
// ------------------------------------------------------------------------------------------------
enum : uint32_t { RC_REACH = 1u << 12, RC_LINKED = 1u << 13 };

template <bool XFER>
__global__ void __launch_bounds__(RT_RT) k_rt_route1(Dev d, Scratch s, RtBufs rb, const uint8_t* __restrict__ ev_bytes,
                                                     WinDesc w, RtLayout L) {
  __shared__ uint32_t lcnt[RT_MAXG * 2];
  __shared__ uint32_t laux;
  const uint32_t i = blockIdx.x * RT_RT + threadIdx.x;
  const uint32_t G = L.G;
  if (threadIdx.x < RT_MAXG * 2) lcnt[threadIdx.x] = 0;
  if (threadIdx.x == 0) {
    laux = 0;
    if ((i & (SEG - 1)) == 0) s.cnt_bad[i / SEG] = 0;  // this segment's failures (k_rt_decide adds to them)
  }
  __syncthreads();
  bool reach = false;
  uint32_t o_id = 0, o_dr = 0, o_cr = 0, aux = 0;
  if (i < w.E) {
    const uint4* q = reinterpret_cast<const uint4*>(ev_bytes + (size_t)i * 128);
    uint4 r[8];
#pragma unroll
    for (int k = 0; k < 8; k++) r[k] = q[k];
    uint32_t cls = 0, code;
    const uint32_t b = win_batch(w, i);
    const tb_uint128_t id = rw_u128(r[0]);
    if (XFER) {
      tb_transfer_t t = *reinterpret_cast<const tb_transfer_t*>(r);
      bool unsup = false;
      code = sh_static_ct(t, w, b, i, &cls, &reach, &unsup);
      if (unsup) aux |= RV_UNSUP;
      if (reach && (uint64_t)(U(t.amount) >> 64) != 0) aux |= RV_HUGE;
      s.id_tslot[i] = t.ledger;
      if (i > 0 && !(U(id) > U(reinterpret_cast<const tb_transfer_t*>(ev_bytes)[i - 1].id))) aux |= RH_NONMONO << 8;
    } else {
      const tb_account_t a = *reinterpret_cast<const tb_account_t*>(r);
      code = sh_static_ca(a, &cls, &reach);
    }
    if (reach) {
      o_id = shard_of(id.lo, id.hi, G);
      if (XFER) {
        const tb_uint128_t dra = rw_u128(r[1]), cra = rw_u128(r[2]);
        o_dr = shard_of(dra.lo, dra.hi, G);
        o_cr = shard_of(cra.lo, cra.hi, G);
      }
    }
    s.code[i] = reach ? CONT : code;
    s.cls[i] = o_id | (o_dr << 4) | (o_cr << 8) | (reach ? RC_REACH : 0u) | ((cls & C_LINKED) ? RC_LINKED : 0u);
  }
  // per wave and destination: ballots, one LDS add per nonzero count
  for (uint32_t dd = 0; dd < G; dd++) {
    const uint32_t ni = (uint32_t)__popcll(__ballot(reach && o_id == dd));
    const uint32_t ns = XFER ? (uint32_t)(__popcll(__ballot(reach && o_dr == dd)) + __popcll(__ballot(reach && o_cr == dd))) : 0u;
    if ((threadIdx.x & 63) == 0) {
      if (ni) atomicAdd(&lcnt[dd * 2], ni);
      if (ns) atomicAdd(&lcnt[dd * 2 + 1], ns);
    }
  }
  if (aux) atomicOr(&laux, aux);
  __syncthreads();
  if (threadIdx.x < RT_MAXG * 2) rb.cnt[(size_t)blockIdx.x * RT_MAXG * 2 + threadIdx.x] = lcnt[threadIdx.x];
  if (threadIdx.x == 0) rb.aux[blockIdx.x] = laux;
}

// ------------------------------------------------------------------------------------------------
// k_rt_scan (home, one workgroup): per (destination, kind) the exclusive offsets over the route blocks,
// the A headers, the home verdict; zeroes this window's C headers (k_rt_decide adds to them) and the
// owner's amount slots (k_rt_own adds to them).
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) k_rt_scan(Dev d, RtBufs rb, const uint8_t* __restrict__ ev_bytes, uint32_t E,
                                                  uint32_t nblk, RtLayout L, uint64_t t_last, uint64_t first_ts,
                                                  uint32_t multi) {
  __shared__ uint32_t tot[RT_MAXG * 2];
  __shared__ uint32_t seg[1024];  // per (column, segment): the segment's sum, then its exclusive base
  __shared__ uint32_t vbits;
  const uint32_t G = L.G, me = L.me, ncol = 2 * G;
  if (threadIdx.x == 0) vbits = 0;
  // thread t: column t % ncol, segment t / ncol of the route blocks (every load independent: no serial
  // chain of global latencies through one wave)
  const uint32_t nseg = 1024 / ncol, col = threadIdx.x % ncol, sg = threadIdx.x / ncol;
  const uint32_t per = (nblk + nseg - 1) / nseg;
  const uint32_t b0 = sg * per, b1 = min(nblk, b0 + per);
  const bool on = sg < nseg;
  uint32_t sum = 0;
  if (on) {
#pragma unroll 8
    for (uint32_t b = b0; b < b1; b++) sum += rb.cnt[(size_t)b * RT_MAXG * 2 + col];
  }
  seg[threadIdx.x] = sum;
  __syncthreads();
  {  // per column, one wave: the segments' exclusive bases (wave scans, 64 segments a step) and the total
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    for (uint32_t c = wv; c < ncol; c += 1024 / 64) {
      uint32_t carry = 0;
      for (uint32_t k0 = 0; k0 < nseg; k0 += 64) {
        const uint32_t k = k0 + ln;
        const uint32_t v = k < nseg ? seg[k * ncol + c] : 0u;
        const uint32_t inc = wave_incl_scan(v);
        if (k < nseg) seg[k * ncol + c] = carry + inc - v;
        carry += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
      }
      if (ln == 0) tot[c] = carry;
    }
  }
  __syncthreads();
  if (on) {
    uint32_t c = seg[threadIdx.x];
#pragma unroll 8
    for (uint32_t b = b0; b < b1; b++) {
      const size_t k = (size_t)b * RT_MAXG * 2 + col;
      const uint32_t v = rb.cnt[k];
      rb.boff[k] = c;
      c += v;
    }
  }
  uint32_t a = 0;
  for (uint32_t b = threadIdx.x; b < nblk; b += 1024) a |= rb.aux[b];
  if (a) atomicOr(&vbits, a);
  // the C headers and chunk counts of this window (k_rt_decide adds to them), zeroed
  const uint64_t cb = rt_blk_c(L, me), ch = rt_c_hdr(L, me);
  for (uint32_t dd = 0; dd < G; dd++) {
    uint32_t* h = reinterpret_cast<uint32_t*>(rb.c_send + dd * cb);
    for (uint32_t k = threadIdx.x; k < ch / 4; k += 1024) h[k] = 0;
  }
  for (uint32_t k = threadIdx.x; k < 128; k += 1024) rb.amt[k] = 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t v = vbits & 0xFFu;
    const bool nonmono = (vbits >> 8) & RH_NONMONO;
    // a pulse due inside the window (the caller ran the one before its first batch): outside the class
    if (t_last >= d.g->pulse_next || (multi && t_last >= first_ts + TB_NS_PER_S)) v |= RV_PULSE;
    uint64_t f0 = 0, f1 = 0, l0 = 0, l1 = 0;
    if (E) {
      const uint64_t* fr = reinterpret_cast<const uint64_t*>(ev_bytes);
      const uint64_t* lr = reinterpret_cast<const uint64_t*>(ev_bytes + (size_t)(E - 1) * 128);
      f0 = fr[0];
      f1 = fr[1];
      l0 = lr[0];
      l1 = lr[1];
    }
    const uint64_t ab = rt_blk_a(L, me);
    for (uint32_t dd = 0; dd < G; dd++) {
      if (tot[dd * 2] > L.c1[me] || tot[dd * 2 + 1] > L.c2[me]) v |= RV_CAP;  // (route2 writes none past it)
      RtHdrA h;
      h.n_id = min(tot[dd * 2], L.c1[me]);
      h.n_side = min(tot[dd * 2 + 1], L.c2[me]);
      h.n_home = E;
      h.flags = (nonmono ? RH_NONMONO : 0u) | (E ? RH_NONEMPTY : 0u);
      h.first_lo = f0;
      h.first_hi = f1;
      h.last_lo = l0;
      h.last_hi = l1;
      *reinterpret_cast<RtHdrA*>(rb.a_send + dd * ab) = h;
    }
    rb.hv[0] = v;
  }
}

// ------------------------------------------------------------------------------------------------
// k_rt_route2 (home): the messages, in event order per destination (block offsets from k_rt_scan, wave
// ranks by ballot). Scratch amt (as uint4): {id message rank, debit side rank, credit side rank}.
// ------------------------------------------------------------------------------------------------
template <bool XFER>
__global__ void __launch_bounds__(RT_RT) k_rt_route2(Dev d, Scratch s, RtBufs rb, const uint8_t* __restrict__ ev_bytes,
                                                     WinDesc w, RtLayout L) {
  __shared__ uint32_t wcnt[RT_RT / 64][RT_MAXG * 2];
  const uint32_t i = blockIdx.x * RT_RT + threadIdx.x;
  const uint32_t G = L.G, me = L.me, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t cls = i < w.E ? s.cls[i] : 0u;
  const bool reach = (cls & RC_REACH) != 0;
  const uint32_t o_id = cls & 15u, o_dr = (cls >> 4) & 15u, o_cr = (cls >> 8) & 15u;
  uint32_t r_id = 0, r_dr = 0, r_cr = 0;
  for (uint32_t dd = 0; dd < G; dd++) {
    const unsigned long long bi = __ballot(reach && o_id == dd);
    if (o_id == dd) r_id = rt_lane_lt(bi);
    uint32_t ns = 0;
    if (XFER) {
      const unsigned long long bd = __ballot(reach && o_dr == dd), bc = __ballot(reach && o_cr == dd);
      const uint32_t before = rt_lane_lt(bd) + rt_lane_lt(bc);
      if (o_dr == dd) r_dr = before;
      if (o_cr == dd) r_cr = before + (o_dr == dd ? 1u : 0u);
      ns = (uint32_t)(__popcll(bd) + __popcll(bc));
    }
    if (lane == 0) {
      wcnt[wave][dd * 2] = (uint32_t)__popcll(bi);
      wcnt[wave][dd * 2 + 1] = ns;
    }
  }
  __syncthreads();
  if (!reach) return;
  const uint32_t* bo = rb.boff + (size_t)blockIdx.x * RT_MAXG * 2;
  uint32_t k_id = bo[o_id * 2] + r_id, k_dr = 0, k_cr = 0;
  for (uint32_t w2 = 0; w2 < wave; w2++) k_id += wcnt[w2][o_id * 2];
  if (XFER) {
    k_dr = bo[o_dr * 2 + 1] + r_dr;
    k_cr = bo[o_cr * 2 + 1] + r_cr;
    for (uint32_t w2 = 0; w2 < wave; w2++) {
      k_dr += wcnt[w2][o_dr * 2 + 1];
      k_cr += wcnt[w2][o_cr * 2 + 1];
    }
  }
  reinterpret_cast<uint4*>(s.amt)[i] = make_uint4(k_id, k_dr, k_cr, 0);
  const uint64_t ab = rt_blk_a(L, me);
  const uint4* q = reinterpret_cast<const uint4*>(ev_bytes + (size_t)i * 128);
  uint4 r[8];
#pragma unroll
  for (int k = 0; k < 8; k++) r[k] = q[k];
  rw_stamp(r, win_ts(w, win_batch(w, i), i));
  if (k_id < L.c1[me]) {
    uint4* dst = reinterpret_cast<uint4*>(rb.a_send + o_id * ab + RT_HDR_A + (uint64_t)k_id * 128);
#pragma unroll
    for (int k = 0; k < 8; k++) dst[k] = r[k];
  }
  if (XFER) {
    const uint64_t amount = rw_u64(r[3].x, r[3].y);
    const uint64_t side0 = RT_HDR_A + (uint64_t)L.c1[me] * 128;
    if (k_dr < L.c2[me]) {  // RtSide: the account id, then {amount, side}
      uint4* m = reinterpret_cast<uint4*>(rb.a_send + o_dr * ab + side0 + (uint64_t)k_dr * 32);
      m[0] = r[1];
      m[1] = make_uint4((uint32_t)amount, (uint32_t)(amount >> 32), 0u, 0u);
    }
    if (k_cr < L.c2[me]) {
      uint4* m = reinterpret_cast<uint4*>(rb.a_send + o_cr * ab + side0 + (uint64_t)k_cr * 32);
      m[0] = r[2];
      m[1] = make_uint4((uint32_t)amount, (uint32_t)(amount >> 32), 1u, 0u);
    }
  }
}

// The global facts every shard derives identically from the G A headers it received: the window's ids
// strictly increasing across the slices (rank order = event order), the first id, the message counts.
// One wave: lane l < G reads header l (all G loads in flight at once; a serial walk over the headers
// put G dependent global latencies in front of every block). Every lane of the wave calls it; `pick`
// (wave-uniform) selects the header whose own counts come back in n_id / n_side (0 past G).
struct RtAFold {
  bool mono;
  tb_uint128_t first;
  uint32_t n_id, n_side;        // header `pick`
  unsigned long long nid, nside;  // over all G headers
};
__device__ inline RtAFold rt_fold_a(const uint8_t* a_recv, const RtLayout& L, uint32_t pick) {
  const uint32_t l = threadIdx.x & 63;
  uint32_t flags = 0, nid = 0, nside = 0;
  unsigned long long f0 = 0, f1 = 0, l0 = 0, l1 = 0;
  if (l < L.G) {
    const RtHdrA* h = reinterpret_cast<const RtHdrA*>(a_recv + rt_off_a(L, l));
    flags = h->flags;
    nid = h->n_id;
    nside = h->n_side;
    f0 = h->first_lo;
    f1 = h->first_hi;
    l0 = h->last_lo;
    l1 = h->last_hi;
  }
  const bool ne = (flags & RH_NONEMPTY) != 0;
  const unsigned long long mne = __ballot(ne);
  const unsigned long long below = mne & ((1ull << l) - 1ull);
  const int prev = below ? 63 - __builtin_clzll(below) : -1;  // the previous non-empty slice
  const int src = prev < 0 ? (int)l : prev;
  const unsigned long long p0 = __shfl(l0, src, 64), p1 = __shfl(l1, src, 64);
  bool bad = false;
  if (ne) {
    if (flags & RH_NONMONO) bad = true;
    if (prev >= 0 && !((((u128)f1 << 64) | f0) > (((u128)p1 << 64) | p0))) bad = true;
  }
  RtAFold r;
  r.mono = __ballot(bad) == 0;
  const int fl = mne ? __builtin_ctzll(mne) : 0;
  const unsigned long long g0 = __shfl(f0, fl, 64), g1 = __shfl(f1, fl, 64);
  r.first.lo = mne ? g0 : 0;
  r.first.hi = mne ? g1 : 0;
  r.n_id = (uint32_t)__shfl((int)nid, (int)pick, 64);
  r.n_side = (uint32_t)__shfl((int)nside, (int)pick, 64);
  unsigned long long a = nid, b = nside;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  r.nid = a;
  r.nside = b;
  return r;
}

// ------------------------------------------------------------------------------------------------
// k_rt_own (owner, after exchange A): J received messages per thread (their loads, and the
// first table probe of every side, issued together: the kernel is a chain of dependent random reads,
// so it is paced by how many are in flight). Blocks: for each source shard its id messages
// (ceil(c1 / (256 J)) blocks), then for each its side messages.
// ------------------------------------------------------------------------------------------------
#define RT_OWN_T 256
#define RT_OWN_J 4  // (four per thread when one per thread would take more than two rounds of resident blocks)
__host__ __device__ inline uint32_t rt_own_blocks(const RtLayout& L, uint32_t* id_blocks) {
  const uint32_t M = RT_OWN_T * (L.own_j ? L.own_j : 1u);
  uint32_t a = 0, b = 0;
  for (uint32_t sg = 0; sg < L.G; sg++) {
    a += (L.c1[sg] + M - 1) / M;
    b += (L.c2[sg] + M - 1) / M;
  }
  if (id_blocks) *id_blocks = a;
  return a + b;
}

// acc_find (dev_common.h) continued from its first entry `e` at `h`, already loaded
__device__ inline uint32_t rt_acc_probe_from(const AccEntry* __restrict__ tab, uint64_t mask, tb_uint128_t id, uint64_t h,
                                             AccEntry e, AccEntry* out) {
  if ((id.lo | id.hi) == 0) return NONE32;
  for (;;) {
    if (e.slot == NONE32) return NONE32;
    if (e.id_lo == id.lo && e.id_hi == id.hi) {
      *out = e;
      return e.slot;
    }
    h = (h + 1) & mask;
    e = tab[h];
  }
}

template <bool XFER, uint32_t J>
__global__ void __launch_bounds__(RT_OWN_T) k_rt_own(Dev d, RtBufs rb, RtLayout L, uint32_t epoch) {
  __shared__ uint32_t sh_n, sh_claim;
  __shared__ unsigned long long ared[RT_OWN_T / 64][2];
  Globals* g = d.g;
  const uint32_t G = L.G;
  // this block's source shard and first message (kernel arguments only: the same in every thread)
  uint32_t b = blockIdx.x, side = 0, sg = 0;
  for (; sg < G; sg++) {
    const uint32_t nb = (L.c1[sg] + (RT_OWN_T * J) - 1) / (RT_OWN_T * J);
    if (b < nb) break;
    b -= nb;
  }
  if (sg == G) {
    side = 1;
    for (sg = 0; sg < G; sg++) {
      const uint32_t nb = (L.c2[sg] + (RT_OWN_T * J) - 1) / (RT_OWN_T * J);
      if (b < nb) break;
      b -= nb;
    }
  }
  if (threadIdx.x < 64) {
    const RtAFold f = rt_fold_a(rb.a_recv, L, sg);
    if (threadIdx.x == 0) {
      sh_n = side ? f.n_side : f.n_id;
      sh_claim = (!XFER || !f.mono) ? 1u : 0u;
    }
    if (blockIdx.x == 0) {
      // static verdicts of this owner (the same arithmetic wherever it runs): room, overflow bound
      uint32_t v = 0;
      if (f.nid > (XFER ? d.x_max - g->x_count : d.acc_max - g->acc_count)) v |= RV_CAP;
      if (XFER && f.nside && g->ovf_bound > MAX128 - ((u128)f.nside << 64)) v |= RV_OVF;
      if (threadIdx.x < G) *reinterpret_cast<uint32_t*>(rb.b_send + rt_off_b(L, threadIdx.x)) = v;
      if (threadIdx.x == 0) {
        // the apply's insert base and whether the window extends this shard's sorted prefix (its records
        // rise across the whole window and start above every id it stores)
        g->base = XFER ? g->x_count : g->acc_count;
        if (XFER) g->win_flags = (f.mono && f.nid && U(f.first) > g->x_id_max && g->x_sorted == g->x_count) ? 2u : 0u;
        // (mono: the first message's id is the window's first; an owner whose first record comes later
        // still sees it above: the ids rise)
      }
    }
  }
  __syncthreads();
  if (sg >= G) return;
  const uint32_t k0 = b * (RT_OWN_T * J) + threadIdx.x, n = sh_n;
  if (!side) {
    // ---- id messages: claim (ids not known to rise), exists against a stored record ----
    const uint8_t* base = rb.a_recv + rt_off_a(L, sg) + RT_HDR_A;
    tb_uint128_t ids[J];
#pragma unroll
    for (uint32_t j = 0; j < J; j++) {
      // the id only (16 B): the rest of the record is read when a stored one must be compared
      const uint32_t k = k0 + j * RT_OWN_T;
      ids[j] = k < n ? rw_u128(*reinterpret_cast<const uint4*>(base + (uint64_t)k * 128)) : tb_uint128_t{0, 0};
    }
    u128 idm = 0;
    const bool claim = sh_claim != 0;
#pragma unroll
    for (uint32_t j = 0; j < J; j++) {
      const uint32_t k = k0 + j * RT_OWN_T;
      if (k >= n) continue;
      const tb_uint128_t id = ids[j];
      const uint8_t* rec = base + (uint64_t)k * 128;
      uint32_t code;
      bool dup = false;
      if (claim) dup = rt_claim(rb.claim, rb.claim_mask, epoch, rt_id_base(L, sg) + k, id, rb.a_recv, L);
      if (XFER) {
        idm = umax128(idm, U(id));
        uint32_t xs = NONE32;
        if (x_may_exist(id, g->x_id_max)) {
          xs = x_find(d.x_tab, d.xr, d.x_mask, id);
          if (xs == NONE32) xs = x_prefix_find(d.xr, g->x_sorted, id);
        }
        code = xs == NONE32 ? (uint32_t)TB_CT_OK : ct_exists(*reinterpret_cast<const tb_transfer_t*>(rec), d.xr[xs]);
      } else {
        AccEntry ae;
        const uint32_t slot = acc_find(d.acc_tab, d.acc_mask, id, &ae);
        code = slot == NONE32 ? (uint32_t)TB_CA_OK : ca_exists(*reinterpret_cast<const tb_account_t*>(rec), d.acc[slot]);
      }
      rb.b_send[rt_off_b(L, sg) + RT_HDR_B + k] = (uint8_t)((1u + code) | (dup ? RI_DUP : 0u));
    }
    if (XFER) {
      // the block's largest received id, for the apply's bound on the stored ids (a bound over every
      // received id holds over the committed ones; one plain store per block, no same-word atomics)
      __shared__ u128 wmax[RT_OWN_T / 64];
      idm = wave_max_u128(idm);
      if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = idm;
      __syncthreads();
      if (threadIdx.x == 0) {
        u128 mx = 0;
        for (int w2 = 0; w2 < RT_OWN_T / 64; w2++) mx = umax128(mx, wmax[w2]);
        rb.imax[blockIdx.x] = mx;
      }
    }
  } else {
    // ---- side messages: the account's slot (kept for the apply), ledger and limit / history flag ----
    const uint8_t* base = rb.a_recv + rt_off_a(L, sg) + RT_HDR_A + (uint64_t)L.c1[sg] * 128;
    uint4 mid[J], mam[J];  // RtSide {id}, {amount, side, pad}
#pragma unroll
    for (uint32_t j = 0; j < J; j++) {
      const uint32_t k = k0 + j * RT_OWN_T;
      const uint4* m = reinterpret_cast<const uint4*>(base + (uint64_t)k * 32);
      mid[j] = k < n ? m[0] : make_uint4(0, 0, 0, 0);
      mam[j] = k < n ? m[1] : make_uint4(0, 0, 0, 0);
    }
    uint64_t hh[J];
    AccEntry e0[J];
#pragma unroll
    for (uint32_t j = 0; j < J; j++) {
      const tb_uint128_t id = rw_u128(mid[j]);
      hh[j] = hash_id(id.lo, id.hi) & d.acc_mask;
      if (k0 + j * RT_OWN_T < n) e0[j] = d.acc_tab[hh[j]];
    }
    unsigned long long alo = 0, ahi = 0;
#pragma unroll
    for (uint32_t j = 0; j < J; j++) {
      const uint32_t k = k0 + j * RT_OWN_T;
      if (k >= n) continue;
      AccEntry e;
      const uint32_t slot = rt_acc_probe_from(d.acc_tab, d.acc_mask, rw_u128(mid[j]), hh[j], e0[j], &e);
      rb.side_slot[rt_side_base(L, sg) + k] = slot;
      uint32_t st = 0, ledger = 0;
      if (slot != NONE32) {
        st = RS_FOUND;
        ledger = e.ledger;
        const uint16_t lim = mam[j].z ? TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS : TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS;
        if (e.flags & (lim | TB_ACCOUNT_HISTORY)) st |= RS_LIMIT;
      }
      *reinterpret_cast<uint2*>(rb.b_send + rt_off_b(L, sg) + rt_b_side(L, sg) + (uint64_t)k * 8) = make_uint2(ledger, st);
      alo += mam[j].x;  // the amount's low and high 32 bits
      ahi += mam[j].y;
    }
    // the received amounts' sum (a bound on this window's balance growth here): 64 slots, no-return adds
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      alo += __shfl_xor(alo, o, 64);
      ahi += __shfl_xor(ahi, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
      ared[threadIdx.x >> 6][0] = alo;
      ared[threadIdx.x >> 6][1] = ahi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long l = 0, h = 0;
      for (int w2 = 0; w2 < RT_OWN_T / 64; w2++) {
        l += ared[w2][0];
        h += ared[w2][1];
      }
      if (l | h) {
        (void)atomicAdd(&rb.amt[(blockIdx.x & 63) * 2], l);
        (void)atomicAdd(&rb.amt[(blockIdx.x & 63) * 2 + 1], h);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// k_rt_decide (home, after exchange B): codes, chains, commit bytes, committed records per chunk.
// ------------------------------------------------------------------------------------------------
#define RT_DEC_T 256
template <bool XFER>
__device__ inline uint32_t rt_code(const Scratch& s, const RtBufs& rb, const RtLayout& L, uint32_t j, uint32_t* verdict,
                                   bool* lim) {
  const uint32_t c0 = s.code[j];
  *lim = false;
  if (c0 != CONT) return c0;
  const uint32_t cls = s.cls[j];
  const uint4 pos = reinterpret_cast<const uint4*>(s.amt)[j];
  const uint32_t me = L.me;
  if (pos.x >= L.c1[me] || (XFER && (pos.y >= L.c2[me] || pos.z >= L.c2[me]))) {
    *verdict |= RV_CAP;  // a message past its block's capacity was never sent (k_rt_scan set RV_CAP too)
    return XFER ? (uint32_t)TB_CT_OK : (uint32_t)TB_CA_OK;
  }
  const uint64_t bb = rt_blk_b(L, me);
  const uint32_t idr = rb.b_recv[(cls & 15u) * bb + RT_HDR_B + pos.x];
  if (idr & RI_DUP) *verdict |= RV_DUP;
  const uint32_t idcode = (idr & RI_CODE) - 1u;
  if (!XFER) return idcode;
  const uint64_t so = rt_b_side(L, me);
  const uint2 dr = *reinterpret_cast<const uint2*>(rb.b_recv + ((cls >> 4) & 15u) * bb + so + (uint64_t)pos.y * 8);
  const uint2 cr = *reinterpret_cast<const uint2*>(rb.b_recv + ((cls >> 8) & 15u) * bb + so + (uint64_t)pos.z * 8);
  if (!(dr.y & RS_FOUND)) return TB_CT_DEBIT_ACCOUNT_NOT_FOUND;   // :1496-1497
  if (!(cr.y & RS_FOUND)) return TB_CT_CREDIT_ACCOUNT_NOT_FOUND;
  if (dr.x != cr.x) return TB_CT_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER;  // :1503-1504
  if (s.id_tslot[j] != dr.x) return TB_CT_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS;
  *lim = ((dr.y | cr.y) & RS_LIMIT) != 0;
  return idcode;  // exists* or ok (:1506-1507)
}

template <bool XFER>
__global__ void __launch_bounds__(RT_DEC_T) k_rt_decide(Dev d, Scratch s, RtBufs rb, WinDesc w, RtLayout L) {
  __shared__ uint32_t nbad, vsh;
  __shared__ uint32_t cmin[RT_MAXG], ccnt[RT_MAXG][2];  // per destination: the block's first chunk, counts
  const uint32_t G = L.G, me = L.me;
  const uint64_t cb = rt_blk_c(L, me), ch = rt_c_hdr(L, me), cs = rt_c_side(L, me);
  if (threadIdx.x == 0) {
    nbad = 0;
    vsh = 0;
  }
  if (threadIdx.x < RT_MAXG) {
    cmin[threadIdx.x] = NONE32;
    ccnt[threadIdx.x][0] = ccnt[threadIdx.x][1] = 0;
  }
  if (blockIdx.x == 0 && threadIdx.x < 64) {
    // the owners' verdicts (B headers, one lane each) and this home's (k_rt_scan), into every C header
    uint32_t v = threadIdx.x < G ? *reinterpret_cast<const uint32_t*>(rb.b_recv + threadIdx.x * rt_blk_b(L, me)) : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v |= (uint32_t)__shfl_xor((int)v, o, 64);
    v |= rb.hv[0];
    if (v && threadIdx.x < G) atomicOr(reinterpret_cast<uint32_t*>(rb.c_send + threadIdx.x * cb), v);
  }
  __syncthreads();
  const uint32_t i = blockIdx.x * RT_DEC_T + threadIdx.x, seg = i / SEG;
  uint32_t lbad = 0, verdict = 0;
  uint32_t cdst = NONE32, cchunk = 0;  // a committed id message: its destination and chunk
  if (i < w.E) {
    const uint32_t b = win_batch(w, i);
    const uint32_t first = w.off[b], last = w.off[b + 1] - 1;
    const bool head = i == first || !(s.cls[i - 1] & RC_LINKED);
    if (head) {
      uint32_t end = i, f = NONE32;
      for (uint32_t j = i;; j++) {
        const bool lj = (s.cls[j] & RC_LINKED) != 0;
        bool lim;
        uint32_t code = rt_code<XFER>(s, rb, L, j, &verdict, &lim);
        if (lj && j == last) code = XFER ? (uint32_t)TB_CT_LINKED_EVENT_CHAIN_OPEN : (uint32_t)TB_CA_LINKED_EVENT_CHAIN_OPEN;
        s.code[j] = code;
        // a committed event reading a balance (limit) or writing a history row: outside the class
        if (XFER && code == TB_CT_OK && lim) verdict |= RV_UNSUP;
        if (code != TB_CT_OK && f == NONE32) f = j;
        end = j;
        if (!lj || j == last) break;
      }
      for (uint32_t j = i; j <= end; j++) {
        const bool commit = f == NONE32;
        if (!commit && j != f && !((s.cls[j] & RC_LINKED) && j == last))
          s.code[j] = XFER ? (uint32_t)TB_CT_LINKED_EVENT_FAILED : (uint32_t)TB_CA_LINKED_EVENT_FAILED;
        const uint32_t cls = s.cls[j];
        if (cls & RC_REACH) {
          const uint4 pos = reinterpret_cast<const uint4*>(s.amt)[j];
          const uint32_t oi = cls & 15u;
          if (pos.x < L.c1[me]) rb.c_send[oi * cb + ch + pos.x] = commit ? 1 : 0;
          if (XFER) {
            if (pos.y < L.c2[me]) rb.c_send[((cls >> 4) & 15u) * cb + cs + pos.y] = commit ? 1 : 0;
            if (pos.z < L.c2[me]) rb.c_send[((cls >> 8) & 15u) * cb + cs + pos.z] = commit ? 1 : 0;
          }
          if (commit && pos.x < L.c1[me]) {
            if (j == i) {
              cdst = oi;
              cchunk = pos.x / RT_CHUNK;
            } else {
              atomicAdd(reinterpret_cast<uint32_t*>(rb.c_send + oi * cb + RT_HDR_C) + pos.x / RT_CHUNK, 1u);
            }
          }
        }
        if (!commit) {
          if (j / SEG == seg) lbad++;
          else atomicAdd(&s.cnt_bad[j / SEG], 1u);  // (a chain running into the next segment)
        }
      }
    }
  }
  // committed id messages per (destination, chunk), counted in LDS and added once per block: a block's
  // messages to one destination are consecutive, so they span at most two chunks (one global add per
  // wave and key had ~128 waves adding to each counter: same-address atomics serialize)
  if (cdst != NONE32) atomicMin(&cmin[cdst], cchunk);
  __syncthreads();
  const uint32_t key = cdst == NONE32 ? NONE32 : (cdst << 24) | cchunk;
  unsigned long long pend = __ballot(key != NONE32);
  while (pend) {
    const uint32_t leader = (uint32_t)__builtin_ctzll(pend);
    const uint32_t lk = (uint32_t)__builtin_amdgcn_readlane((int)key, (int)leader);
    const unsigned long long m = __ballot(key == lk);
    if ((threadIdx.x & 63) == leader) {
      const uint32_t dd = lk >> 24, rel = (lk & 0xFFFFFFu) - cmin[dd];
      if (rel < 2) atomicAdd(&ccnt[dd][rel], (uint32_t)__popcll(m));
      else atomicAdd(reinterpret_cast<uint32_t*>(rb.c_send + dd * cb + RT_HDR_C) + (lk & 0xFFFFFFu), (uint32_t)__popcll(m));
    }
    pend &= ~m;
  }
  const uint32_t wb = wave_sum(lbad);
  if ((threadIdx.x & 63) == 0 && wb) atomicAdd(&nbad, wb);
  if (verdict) atomicOr(&vsh, verdict);
  __syncthreads();
  if (threadIdx.x < 2 * RT_MAXG) {
    const uint32_t dd = threadIdx.x >> 1, rel = threadIdx.x & 1, c = ccnt[dd][rel];
    if (c) atomicAdd(reinterpret_cast<uint32_t*>(rb.c_send + dd * cb + RT_HDR_C) + cmin[dd] + rel, c);
  }
  if (threadIdx.x == 0 && nbad) atomicAdd(&s.cnt_bad[seg], nbad);
  if (vsh && threadIdx.x < G) atomicOr(reinterpret_cast<uint32_t*>(rb.c_send + threadIdx.x * cb), vsh);
}

// ------------------------------------------------------------------------------------------------
// k_rt_apply (after exchange C): blocks [0, nh) the home replies; then per source shard its side
// messages' balance adds, then per source shard its committed records (one block per 1024-message chunk).
// The last block closes the window. Nothing is applied when any shard's verdict is set.
// ------------------------------------------------------------------------------------------------
__host__ __device__ inline uint32_t rt_apply_blocks(const RtLayout& L, uint32_t nh, uint32_t* side_blocks) {
  uint32_t a = 0, b = 0;
  for (uint32_t sg = 0; sg < L.G; sg++) {
    a += (L.c2[sg] + RT_T - 1) / RT_T;
    b += rt_nch(L.c1[sg]);
  }
  if (side_blocks) *side_blocks = a;
  return nh + a + b;
}

template <bool XFER>
__global__ void __launch_bounds__(RT_T) k_rt_apply(Dev d, Scratch s, RtBufs rb, WinDesc w, RtLayout L, uint32_t nh,
                                                   FinalOut o, ChgLog chg, uint32_t chg_epoch, uint32_t b_off,
                                                   uint32_t nblk) {
  // (b_off / nblk: the grid may be launched in parts, one per role — TBG_RT_SPLIT, a profiling aid)
  const uint32_t bid = blockIdx.x + b_off;
  __shared__ uint32_t lds[RT_T / 64];
  __shared__ uint32_t f_v, sh_base, sh_total;
  __shared__ unsigned long long f_amt[2];
  __shared__ uint32_t f_cnt[RT_T / 64][2];
  __shared__ u128 sh_imax[RT_T / 64];
  Globals* g = d.g;
  const uint32_t G = L.G;
  // this block's role, source shard and first message (kernel arguments only: the same in every thread)
  uint32_t b = bid, role = 0, sg = 0, k0 = 0, my_flat = 0;
  if (b >= nh) {
    b -= nh;
    role = 1;
    for (sg = 0; sg < G; sg++) {
      const uint32_t nb = (L.c2[sg] + RT_T - 1) / RT_T;
      if (b < nb) break;
      b -= nb;
    }
    k0 = b * RT_T;
    if (sg == G) {
      role = 2;
      my_flat = b;  // (the id blocks are the chunks in (source, chunk) order: this one's flat index)
      for (sg = 0; sg < G; sg++) {
        const uint32_t nb = rt_nch(L.c1[sg]);
        if (b < nb) break;
        b -= nb;
      }
      k0 = b * RT_CHUNK;
    }
  }
  const bool last = bid == nblk - 1;
  const RtHdrA* hdr = role && sg < G ? reinterpret_cast<const RtHdrA*>(rb.a_recv + rt_off_a(L, sg)) : nullptr;
  const uint32_t n_msg = hdr ? (role == 1 ? hdr->n_side : hdr->n_id) : 0u;
  // what a block folds from the G C headers, in parallel: the verdict (every block); the committed
  // records before its chunk ((source, chunk) order: id blocks) and in all (the last block); whether
  // the received amounts keep every balance field below 2^64 (side blocks)
  if (threadIdx.x == 0) {
    f_v = 0;
    f_amt[0] = f_amt[1] = 0;
  }
  __syncthreads();
  if (threadIdx.x < G) atomicOr(&f_v, *reinterpret_cast<const uint32_t*>(rb.c_recv + rt_off_c(L, threadIdx.x)));
  const bool counts = role == 2 || last;
  if (counts) {
    // one count per thread and source (a source has at most RT_T chunks unless its capacity passes 1M
    // messages: the loop after takes the rest); the G loads are issued before any is used
    uint32_t before = 0, all = 0;
    uint32_t v[RT_MAXG], fl[RT_MAXG];
    uint32_t flat0 = 0;
    uint64_t off = 0;
#pragma unroll
    for (uint32_t s2 = 0; s2 < RT_MAXG; s2++) {
      v[s2] = 0;
      fl[s2] = flat0 + threadIdx.x;
      if (s2 < G) {
        const uint32_t nch = rt_nch(L.c1[s2]);
        if (threadIdx.x < nch) v[s2] = reinterpret_cast<const uint32_t*>(rb.c_recv + off + RT_HDR_C)[threadIdx.x];
        flat0 += nch;
        off += rt_blk_c(L, s2);
      }
    }
#pragma unroll
    for (uint32_t s2 = 0; s2 < RT_MAXG; s2++) {
      all += v[s2];
      if (fl[s2] < my_flat) before += v[s2];
    }
    if (flat0 > RT_T) {
      flat0 = 0;
      for (uint32_t s2 = 0; s2 < G; s2++) {
        const uint32_t nch = rt_nch(L.c1[s2]);
        const uint32_t* cnt = reinterpret_cast<const uint32_t*>(rb.c_recv + rt_off_c(L, s2) + RT_HDR_C);
        for (uint32_t q = threadIdx.x + RT_T; q < nch; q += RT_T) {
          all += cnt[q];
          if (flat0 + q < my_flat) before += cnt[q];
        }
        flat0 += nch;
      }
    }
    before = wave_sum(before);
    all = wave_sum(all);
    if ((threadIdx.x & 63) == 0) {
      f_cnt[threadIdx.x >> 6][0] = before;
      f_cnt[threadIdx.x >> 6][1] = all;
    }
  }
  if (XFER && role == 1 && threadIdx.x < 64) {
    unsigned long long lo = rb.amt[threadIdx.x * 2], hi = rb.amt[threadIdx.x * 2 + 1];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lo += __shfl_xor(lo, o, 64);
      hi += __shfl_xor(hi, o, 64);
    }
    if (threadIdx.x == 0) {
      f_amt[0] = lo;
      f_amt[1] = hi;
    }
  }
  __syncthreads();
  if (counts && threadIdx.x == 0) {
    uint32_t before = 0, all = 0;
    for (int w2 = 0; w2 < RT_T / 64; w2++) {
      before += f_cnt[w2][0];
      all += f_cnt[w2][1];
    }
    sh_base = before;
    sh_total = all;
  }
  bool small = false;
  if (XFER && role == 1) {
    const u128 tot = (u128)f_amt[0] + ((u128)f_amt[1] << 32);
    const u128 top = g->ovf_bound + tot;
    small = top >= g->ovf_bound && (uint64_t)(top >> 64) == 0;
  }
  if (counts) __syncthreads();
  if (f_v) {
    if (last && threadIdx.x == 0) atomicOr(&g->window_error, 2u);
    return;
  }
  if (role == 0) {
    // ---- home replies (batch_base relative to the home's first batch, indices batch-relative) ----
    const uint32_t i = bid * RT_T + threadIdx.x;
    const bool home = i < w.E;
    const uint32_t code = home ? s.code[i] : (uint32_t)TB_CT_OK;
    const uint32_t bad = home && code != TB_CT_OK ? 1u : 0u;
    uint32_t tot;
    const uint32_t rbad = seg_prefix<SEG>(s.cnt_bad, bid, lds) + block_excl<SEG / 64>(bad, lds, &tot);
    if (home) {
      const uint32_t b = win_batch(w, i);
      if (i == w.off[b])
        for (int32_t bb = (int32_t)b; bb >= 0 && w.off[bb] == i; bb--) o.batch_base[bb] = rbad;
      if (bad && sh_guard(g, rbad < w.E, 2, rbad)) {
        tb_create_result_t r;
        r.index = i - w.off[b];
        r.result = code;
        o.results[rbad] = r;
      }
      if (i == w.E - 1) {
        const uint32_t total_bad = rbad + bad;
        for (int32_t bb = (int32_t)w.nb; bb >= 0 && w.off[bb] == w.E; bb--) o.batch_base[bb] = total_bad;
        g->result_count = total_bad;
      }
    }
  } else if (role == 1) {
    // ---- account owner: the committed sides' balance adds ----
    const uint32_t k = k0 + threadIdx.x;
    if (XFER && k < n_msg) {
      // the commit byte, the slot and the message's {amount, side} half loaded together (no chain)
      const uint8_t commit = rb.c_recv[rt_off_c(L, sg) + rt_c_side(L, sg) + k];
      const uint32_t slot = rb.side_slot[rt_side_base(L, sg) + k];
      const uint4 m = reinterpret_cast<const uint4*>(rb.a_recv + rt_off_a(L, sg) + RT_HDR_A +
                                                     (uint64_t)L.c1[sg] * 128 + (uint64_t)k * 32)[1];
      if (commit) {
        if (sh_guard(g, slot < d.acc_max, 3, slot)) {
          const uint64_t amount = (uint64_t)m.x | ((uint64_t)m.y << 32);  // RtSide {id, amount, side, pad}
          const uint32_t side = m.z;
          Add128 a;
          a.issue(side ? &d.acc[slot].credits_posted : &d.acc[slot].debits_posted, (u128)amount, small);
          if (chg.mark) chg.mark[slot] = chg_epoch;
          a.finish();
        }
      }
    }
  } else {
    // ---- id owner: committed records appended at base + rank, (source, message) order ----
    const uint32_t k = k0 + threadIdx.x;
    const bool live = k < n_msg;
    const uint8_t* cc = rb.c_recv + rt_off_c(L, sg) + rt_c_hdr(L, sg);
    const bool ins = live && cc[k] != 0;
    uint32_t tot;
    const uint32_t rank = sh_base + block_excl<RT_T / 64>(ins ? 1u : 0u, lds, &tot);
    const uint64_t slot = g->base + rank;
    const uint4* src = reinterpret_cast<const uint4*>(rb.a_recv + rt_off_a(L, sg) + RT_HDR_A + (uint64_t)k * 128);
    if (XFER) {
      const bool prefix_win = (g->win_flags & 2u) != 0;
      const unsigned long long ml = __ballot(live), mi = __ballot(ins);
      const uint32_t n = (uint32_t)__popcll(ml), lane = threadIdx.x & 63;
      const uint64_t slot0 = g->base + (uint32_t)__builtin_amdgcn_readlane((int)rank, 0);
      if (prefix_win && mi == ml && slot0 + n <= d.x_max) {
        // every live message of this wave commits and the window appends above every stored id (no
        // table insert): the wave's records are one run in the A buffer and one in the store, copied
        // as 16 B words lane by lane, so each load / store instruction covers one contiguous KiB (a
        // record per lane put 64 lines into every instruction, and every store was a partial line)
        const uint4* src0 = reinterpret_cast<const uint4*>(rb.a_recv + rt_off_a(L, sg) + RT_HDR_A + (uint64_t)(k - lane) * 128);
        uint4* dst0 = reinterpret_cast<uint4*>(d.xr + slot0);
        uint4 v[8];
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) v[j] = lane + 64 * j < n * 8 ? src0[lane + 64 * j] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (uint32_t j = 0; j < 8; j++)
          if (lane + 64 * j < n * 8) st_stream(dst0 + lane + 64 * j, v[j]);
        if (ins) d.xstatus[slot] = 0;
      } else if (ins && sh_guard(g, slot < d.x_max, 5, slot)) {
        uint4 r[8];
#pragma unroll
        for (int q = 0; q < 8; q++) r[q] = src[q];
        uint4* dst = reinterpret_cast<uint4*>(d.xr + slot);
#pragma unroll
        for (int q = 0; q < 8; q++) st_stream(dst + q, r[q]);
        if (!prefix_win) x_insert(d.x_tab, d.x_mask, rw_u128(r[0]), (uint32_t)slot);
        d.xstatus[slot] = 0;
      }
    } else if (ins && sh_guard(g, slot < d.acc_max, 6, slot)) {
      uint4 r[8];
#pragma unroll
      for (int q = 0; q < 8; q++) r[q] = src[q];
      uint4* dst = reinterpret_cast<uint4*>(d.acc + slot);
#pragma unroll
      for (int q = 0; q < 8; q++) dst[q] = r[q];
      d.hot[slot] = 0;
      acc_insert(d.acc_tab, d.acc_mask, rw_u128(r[0]), (uint32_t)slot, r[7].x, (uint16_t)(r[7].y >> 16));
    }
  }
  // the last block closes the window (the others read Globals::base, captured by k_rt_own, never the
  // counts written here)
  if (bid != nblk - 1) return;
  u128 mx = 0;
  if (XFER) {
    // the bound on the stored ids: the largest id k_rt_own's blocks received (an upper bound: it can
    // only disable a prefix extension), folded by this block
    uint32_t id_blocks = 0;
    (void)rt_own_blocks(L, &id_blocks);
    for (uint32_t q = threadIdx.x; q < id_blocks; q += RT_T) mx = umax128(mx, rb.imax[q]);
    mx = wave_max_u128(mx);
    if ((threadIdx.x & 63) == 0) sh_imax[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0)
      for (int w2 = 0; w2 < RT_T / 64; w2++) mx = umax128(mx, sh_imax[w2]);
  }
  if (threadIdx.x != 0) return;
  if (XFER && mx > g->x_id_max) g->x_id_max = mx;
  const uint64_t total = g->base + sh_total;
  g->events_total += w.E;
  g->windows_applied++;
  if (XFER) {
    if (g->win_flags & 2u) g->x_sorted = total;
    g->x_count = total;
    u128 tot = 0;
    for (int q = 0; q < 64; q++) tot += (u128)rb.amt[q * 2] + ((u128)rb.amt[q * 2 + 1] << 32);
    const u128 sum = g->ovf_bound + tot;
    g->ovf_bound = sum < g->ovf_bound ? MAX128 : sum;
  } else {
    g->acc_count = total;
  }
}
