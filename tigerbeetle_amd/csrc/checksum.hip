// checksum.hip — TigerBeetle's checksum (vsr/checksum.zig:38-85) for many messages at once.
//
// checksum(source) is AEGIS-128L as a MAC with a zero key and nonce: the source absorbed as
// associated data in 32-byte blocks (last block zero-padded), finalization with (len_bits, 0), tag
// S0 ^ .. ^ S6 as a little-endian u128. One message is a sequential chain of AES rounds, so the GPU
// parallelises across messages (the bodies of a commit window, an AOF's prepares, a window's replies)
// and, inside one message, across the eight state blocks of an update:
//   - 8 lanes per message, lane j holding state block S_j as four 32-bit column words;
//   - one update S'_j = AESRound(S_{j-1}, S_j) (^ M0 on S_0, ^ M1 on S_4): S_{j-1} arrives from the
//     neighbour lane by two DPP row shifts (no LDS round trip), the round is 16 lookups of one
//     1 KiB T-table in LDS (the other three tables are byte rotations of it) and xors;
//   - message bytes are staged through LDS in 1 KiB-per-message chunks (32 updates), loaded with
//     coalesced 16-byte loads one chunk ahead so the loads of chunk c + 1 overlap the rounds of c.
// No AES instructions on CDNA4: the T-table round is the whole cost (16 LDS reads per lane-update,
// 4 per message byte); see DESIGN.md §5 for the measured rate.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tbg.h"

namespace {

__constant__ uint8_t kSbox[256] = {
    0x63, 0x7c, 0x77, 0x7b, 0xf2, 0x6b, 0x6f, 0xc5, 0x30, 0x01, 0x67, 0x2b, 0xfe, 0xd7, 0xab, 0x76,
    0xca, 0x82, 0xc9, 0x7d, 0xfa, 0x59, 0x47, 0xf0, 0xad, 0xd4, 0xa2, 0xaf, 0x9c, 0xa4, 0x72, 0xc0,
    0xb7, 0xfd, 0x93, 0x26, 0x36, 0x3f, 0xf7, 0xcc, 0x34, 0xa5, 0xe5, 0xf1, 0x71, 0xd8, 0x31, 0x15,
    0x04, 0xc7, 0x23, 0xc3, 0x18, 0x96, 0x05, 0x9a, 0x07, 0x12, 0x80, 0xe2, 0xeb, 0x27, 0xb2, 0x75,
    0x09, 0x83, 0x2c, 0x1a, 0x1b, 0x6e, 0x5a, 0xa0, 0x52, 0x3b, 0xd6, 0xb3, 0x29, 0xe3, 0x2f, 0x84,
    0x53, 0xd1, 0x00, 0xed, 0x20, 0xfc, 0xb1, 0x5b, 0x6a, 0xcb, 0xbe, 0x39, 0x4a, 0x4c, 0x58, 0xcf,
    0xd0, 0xef, 0xaa, 0xfb, 0x43, 0x4d, 0x33, 0x85, 0x45, 0xf9, 0x02, 0x7f, 0x50, 0x3c, 0x9f, 0xa8,
    0x51, 0xa3, 0x40, 0x8f, 0x92, 0x9d, 0x38, 0xf5, 0xbc, 0xb6, 0xda, 0x21, 0x10, 0xff, 0xf3, 0xd2,
    0xcd, 0x0c, 0x13, 0xec, 0x5f, 0x97, 0x44, 0x17, 0xc4, 0xa7, 0x7e, 0x3d, 0x64, 0x5d, 0x19, 0x73,
    0x60, 0x81, 0x4f, 0xdc, 0x22, 0x2a, 0x90, 0x88, 0x46, 0xee, 0xb8, 0x14, 0xde, 0x5e, 0x0b, 0xdb,
    0xe0, 0x32, 0x3a, 0x0a, 0x49, 0x06, 0x24, 0x5c, 0xc2, 0xd3, 0xac, 0x62, 0x91, 0x95, 0xe4, 0x79,
    0xe7, 0xc8, 0x37, 0x6d, 0x8d, 0xd5, 0x4e, 0xa9, 0x6c, 0x56, 0xf4, 0xea, 0x65, 0x7a, 0xae, 0x08,
    0xba, 0x78, 0x25, 0x2e, 0x1c, 0xa6, 0xb4, 0xc6, 0xe8, 0xdd, 0x74, 0x1f, 0x4b, 0xbd, 0x8b, 0x8a,
    0x70, 0x3e, 0xb5, 0x66, 0x48, 0x03, 0xf6, 0x0e, 0x61, 0x35, 0x57, 0xb9, 0x86, 0xc1, 0x1d, 0x9e,
    0xe1, 0xf8, 0x98, 0x11, 0x69, 0xd9, 0x8e, 0x94, 0x9b, 0x1e, 0x87, 0xe9, 0xce, 0x55, 0x28, 0xdf,
    0x8c, 0xa1, 0x89, 0x0d, 0xbf, 0xe6, 0x42, 0x68, 0x41, 0x99, 0x2d, 0x0f, 0xb0, 0x54, 0xbb, 0x16,
};

// AEGIS-128L constants C0, C1 as little-endian column words.
__constant__ uint32_t kC0[4] = {0x02010100u, 0x0d080503u, 0x59372215u, 0x6279e990u};
__constant__ uint32_t kC1[4] = {0x55183ddbu, 0xf12fc26du, 0x42311120u, 0xdd28b573u};

#define CK_LANES 64
#define CK_MSGS (CK_LANES / 8)  // messages per wave
#define CK_CHUNK 1024           // bytes per message per staged chunk (32 updates)

struct Blk {
  uint32_t w[4];
};

__device__ inline uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }

// MixColumns(ShiftRows(SubBytes(in))) ^ rk with T0[x] = (2s, s, s, 3s) and Tr = rotl(T0, 8r).
__device__ inline Blk aes_round(const uint32_t* T, const Blk& in, const Blk& rk) {
  Blk o;
#pragma unroll
  for (int c = 0; c < 4; c++) {
    o.w[c] = T[in.w[c] & 0xFF] ^ rotl32(T[(in.w[(c + 1) & 3] >> 8) & 0xFF], 8) ^
             rotl32(T[(in.w[(c + 2) & 3] >> 16) & 0xFF], 16) ^ rotl32(T[in.w[(c + 3) & 3] >> 24], 24) ^ rk.w[c];
  }
  return o;
}

// The previous state block S_{j-1} (lane j - 1 of the 8-lane group, lane 7 for lane 0): DPP
// row_shr:1 for lanes 1..7, row_shl:7 for lane 0 (8-lane groups sit inside 16-lane DPP rows).
__device__ inline uint32_t prev_word(uint32_t v, bool first) {
  const uint32_t a = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
  const uint32_t b = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x107, 0xF, 0xF, false);  // row_shl:7
  return first ? b : a;
}

__device__ inline Blk update(const uint32_t* T, const Blk& S, const Blk& m, bool first, bool inject) {
  Blk p;
#pragma unroll
  for (int c = 0; c < 4; c++) p.w[c] = prev_word(S.w[c], first);
  Blk o = aes_round(T, p, S);
  if (inject) {
#pragma unroll
    for (int c = 0; c < 4; c++) o.w[c] ^= m.w[c];
  }
  return o;
}

// Loads piece `p` (16 bytes) of a message into registers, zero past its end.
__device__ inline uint4 load_piece(const uint8_t* msg, uint32_t len, uint32_t p) {
  const uint64_t off = (uint64_t)p * 16;
  if (off >= len) return make_uint4(0, 0, 0, 0);
  if (off + 16 <= len && (((uintptr_t)(msg + off)) & 15) == 0) return *reinterpret_cast<const uint4*>(msg + off);
  uint32_t w[4] = {0, 0, 0, 0};
  for (uint32_t k = 0; k < 16 && off + k < len; k++) w[k >> 2] |= (uint32_t)msg[off + k] << (8 * (k & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__global__ void __launch_bounds__(CK_LANES) k_checksum(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets,
                                                       const uint32_t* __restrict__ sizes, uint32_t n,
                                                       uint8_t* __restrict__ out) {
  __shared__ uint32_t T[256];
  __shared__ uint4 buf[2][CK_MSGS][CK_CHUNK / 16];
  const uint32_t lane = threadIdx.x;
  const uint32_t g = lane >> 3, j = lane & 7;
  for (uint32_t x = lane; x < 256; x += CK_LANES) {
    const uint32_t s = kSbox[x];
    const uint32_t s2 = ((s << 1) ^ ((s >> 7) * 0x1b)) & 0xFF;
    T[x] = s2 | (s << 8) | (s << 16) | ((s2 ^ s) << 24);
  }
  const uint32_t msg_id = blockIdx.x * CK_MSGS + g;
  const bool live = msg_id < n;
  const uint8_t* msg = live ? base + offsets[msg_id] : base;
  const uint32_t len = live ? sizes[msg_id] : 0;
  const uint32_t nblocks = (len + 31) / 32;
  // the wave runs to its longest message; shorter ones keep their state (masked updates)
  uint32_t wave_blocks = nblocks;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wave_blocks = max(wave_blocks, (uint32_t)__shfl_xor((int)wave_blocks, o, 64));

  // state init: key = nonce = 0 -> S = (0, C1, C0, C1, 0, C0, C1, C0), then 10 updates with M = 0
  Blk S;
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const uint32_t c0 = kC0[c], c1 = kC1[c];
    S.w[c] = (j == 0 || j == 4) ? 0u : (j == 1 || j == 3 || j == 6) ? c1 : c0;
  }
  __syncthreads();  // T ready
  const bool first = j == 0;
  const Blk zero = {{0, 0, 0, 0}};
  for (int r = 0; r < 10; r++) S = update(T, S, zero, first, false);

  // chunks of 32 updates: pieces of chunk c are loaded one chunk ahead (8 lanes x 8 pieces x 16 B)
  const uint32_t n_chunks = (wave_blocks * 32 + CK_CHUNK - 1) / CK_CHUNK;
  uint4 pre[8];
#pragma unroll
  for (int k = 0; k < 8; k++) pre[k] = load_piece(msg, len, (uint32_t)k * 8 + j);
  for (uint32_t c = 0; c < n_chunks; c++) {
    const uint32_t sb = c & 1;
#pragma unroll
    for (int k = 0; k < 8; k++) buf[sb][g][k * 8 + j] = pre[k];
    __syncthreads();
    if (c + 1 < n_chunks) {
      const uint32_t p0 = (c + 1) * (CK_CHUNK / 16);
#pragma unroll
      for (int k = 0; k < 8; k++) pre[k] = load_piece(msg, len, p0 + (uint32_t)k * 8 + j);
    }
    const uint32_t b0 = c * (CK_CHUNK / 32);
    const uint32_t steps = min((uint32_t)(CK_CHUNK / 32), wave_blocks - b0);
    for (uint32_t s = 0; s < steps; s++) {
      // lanes 0..3 read M0 (bytes 0-15 of the block), lanes 4..7 M1; lanes 0 and 4 inject it
      const uint4 mv = buf[sb][g][2 * s + (j >> 2)];
      const Blk m = {{mv.x, mv.y, mv.z, mv.w}};
      const Blk t = update(T, S, m, first, (j & 3) == 0);
      if (b0 + s < nblocks) S = t;
    }
  }
  // finalization: t = S2 ^ (LE64(len * 8) || LE64(0)), 7 updates with M0 = M1 = t
  Blk t;
  const uint64_t bits = (uint64_t)len * 8;
#pragma unroll
  for (int c = 0; c < 4; c++) {
    uint32_t v = (uint32_t)__shfl((int)S.w[c], (int)(lane & ~7u) + 2, 64);
    if (c == 0) v ^= (uint32_t)bits;
    if (c == 1) v ^= (uint32_t)(bits >> 32);
    t.w[c] = v;
  }
  for (int r = 0; r < 7; r++) S = update(T, S, t, first, (j & 3) == 0);
  // tag = S0 ^ .. ^ S6
  Blk x = S;
  if (j == 7) x = zero;
#pragma unroll
  for (int c = 0; c < 4; c++) {
    uint32_t v = x.w[c];
    v ^= (uint32_t)__shfl_xor((int)v, 1, 64);
    v ^= (uint32_t)__shfl_xor((int)v, 2, 64);
    v ^= (uint32_t)__shfl_xor((int)v, 4, 64);
    x.w[c] = v;
  }
  if (live && j == 0) *reinterpret_cast<uint4*>(out + (size_t)msg_id * 16) = make_uint4(x.w[0], x.w[1], x.w[2], x.w[3]);
}

}  // namespace

extern "C" int tbg_checksum(const void* d_base, const uint64_t* d_offsets, const uint32_t* d_sizes, uint32_t n,
                            void* d_out, void* stream) {
  if (n == 0) return TBG_OK;
  if (!d_base || !d_offsets || !d_sizes || !d_out || ((uintptr_t)d_out & 15)) return TBG_E_INVALID;
  const uint32_t blocks = (n + CK_MSGS - 1) / CK_MSGS;
  hipLaunchKernelGGL(k_checksum, dim3(blocks), dim3(CK_LANES), 0, (hipStream_t)stream, (const uint8_t*)d_base,
                     d_offsets, d_sizes, n, (uint8_t*)d_out);
  return hipGetLastError() == hipSuccess ? TBG_OK : TBG_E_DEVICE;
}
