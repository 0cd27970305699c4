// Microbenchmark of the chunked resolver's wave-walk step (chunks.h rc_step32) in isolation: one
// workgroup of one wave walks a synthetic 2048-entry segment in LDS many times; clock64() around the
// whole loop only. Variants: 0 = full step, 1 = no failure search, 2 = scan + balance update only,
// 3 = scan only (the balance chain kept by a readlane), 4/5 = one ballot for any failure before
// the rounds (5: one round), 6 = scan + status + dent stores, 7 = scan + clamped threshold + dent. Prints cycles per 64-entry step.
// Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/ubench_walk tools/ubench_walk.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define N 2048

__device__ inline int32_t scan32(int32_t x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
  return x;
}

template <int V>
__global__ void __launch_bounds__(64) k_walk(const uint32_t* g_em, const int32_t* g_amt, int reps,
                                             unsigned long long* out, int64_t* sink) {
  __shared__ uint16_t em[N];
  __shared__ int32_t amt[N];
  __shared__ uint8_t oth[N], cur[N];
  __shared__ int64_t dent[N];
  const int lane = threadIdx.x;
  for (int k = lane; k < N; k += 64) {
    em[k] = (uint16_t)g_em[k];
    amt[k] = g_amt[k];
    oth[k] = 1;
  }
  __syncthreads();
  const int64_t A0 = 1 << 20;
  int64_t D = 0;
  const uint64_t t0 = clock64();
  for (int r = 0; r < reps; r++) {
    uint32_t emA = em[lane], emB;
    int32_t amtA = amt[lane], amtB;
    uint32_t othA = oth[lane], othB;
    D = D & 0xFFFF;
    for (uint32_t k = 0; k < N; k += 128) {
      const uint32_t kb = min(k + 64u + lane, (uint32_t)N - 1u);
      emB = em[kb];
      amtB = amt[kb];
      othB = oth[kb];
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const uint32_t e = h ? emB : emA;
        const int32_t a = h ? amtB : amtA;
        const uint32_t o = h ? othB : othA;
        const uint32_t kk = k + 64u * h + lane;
        const bool check = e & 0x800u;
        const bool ok = o != 0u;
        int32_t eff = ok ? (check ? -a : ((e & 0x1000u) ? a : 0)) : 0;
        int32_t pre = scan32(eff) - eff;
        if (V <= 1 || V == 4 || V == 5) {
          const int64_t B64 = A0 + D;
          const int32_t B = B64 > INT32_MAX ? INT32_MAX : (B64 < INT32_MIN ? INT32_MIN : (int32_t)B64);
          const int32_t x = a - pre;
          if (V == 4 || V == 5) {
            // fast path: one ballot for "any failure"; the rounds only when there is one
            const bool cnd = ok && check;
            unsigned long long fm = __ballot(cnd && x > B);
            if (fm) {
              unsigned long long fails = 0;
              uint32_t acc = 0;
              const unsigned long long cand = __ballot(cnd);
              for (;;) {
                const int jl = __builtin_ctzll(fm);
                acc += (uint32_t)__builtin_amdgcn_readlane(a, jl);
                fails |= 1ull << jl;
                const unsigned long long after = jl == 63 ? 0ull : ~0ull << (jl + 1);
                if (V == 5 || (uint32_t)B + acc >= (uint32_t)INT32_MAX) break;
                fm = __ballot(x > B + (int32_t)acc) & cand & after;
                if (!fm) break;
              }
              const bool failed = (fails >> lane) & 1ull;
              const int32_t fa = failed ? a : 0;
              pre += scan32(fa) - fa;
              if (failed) eff = 0;
            }
          }
          if (V == 0) {
            const unsigned long long cand = __ballot(ok && check);
            unsigned long long fails = 0, after = ~0ull;
            uint32_t acc = 0;
            const uint32_t room = (uint32_t)INT32_MAX - (uint32_t)B;
            while (acc < room) {
              const unsigned long long fm = __ballot(x > B + (int32_t)acc) & cand & after;
              if (!fm) break;
              const int jl = __builtin_ctzll(fm);
              acc += (uint32_t)__builtin_amdgcn_readlane(a, jl);
              fails |= 1ull << jl;
              after = jl == 63 ? 0ull : ~0ull << (jl + 1);
            }
            if (fails) {
              const bool failed = (fails >> lane) & 1ull;
              const int32_t fa = failed ? a : 0;
              pre += scan32(fa) - fa;
              if (failed) eff = 0;
            }
          }
          if (check) cur[e & 0x7FFu] = x <= B ? 1 : 0;
          dent[kk] = D + pre;
        }
        if (V == 2) dent[kk] = D + pre;
        if (V == 6) {
          if (check) cur[e & 0x7FFu] = a <= pre ? 1 : 0;
          dent[kk] = D + pre;
        }
        if (V == 7) {
          const int64_t B64 = A0 + D;
          const int32_t B = B64 > INT32_MAX ? INT32_MAX : (B64 < INT32_MIN ? INT32_MIN : (int32_t)B64);
          dent[kk] = D + pre + B;
        }
        D += __builtin_amdgcn_readlane(pre + eff, 63);
      }
      if (k + 128u < N) {
        const uint32_t ka = k + 128u + lane;
        emA = em[ka];
        amtA = amt[ka];
        othA = oth[ka];
      }
    }
  }
  const uint64_t t1 = clock64();
  if (lane == 0) {
    out[V] = t1 - t0;
    sink[0] = D + dent[5] + cur[7];
  }
}

int main() {
  uint32_t h_em[N];
  int32_t h_amt[N];
  uint32_t s = 12345;
  for (int k = 0; k < N; k++) {
    s = s * 1664525u + 1013904223u;
    const bool check = (s >> 8) % 2 == 0;
    h_em[k] = (uint32_t)(k & 0x3FF) | (check ? 0x800u : 0x1000u);
    h_amt[k] = 1 + (int32_t)((s >> 12) % 1000);
  }
  uint32_t* d_em;
  int32_t* d_amt;
  unsigned long long* d_out;
  int64_t* d_sink;
  (void)hipMalloc(&d_em, sizeof h_em);
  (void)hipMalloc(&d_amt, sizeof h_amt);
  (void)hipMalloc(&d_out, 8 * sizeof(unsigned long long));
  (void)hipMalloc(&d_sink, 8);
  (void)hipMemcpy(d_em, h_em, sizeof h_em, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_amt, h_amt, sizeof h_amt, hipMemcpyHostToDevice);
  const int reps = 200;
  for (int pass = 0; pass < 2; pass++) {
    k_walk<0><<<1, 64>>>(d_em, d_amt, reps, d_out, d_sink);
    k_walk<1><<<1, 64>>>(d_em, d_amt, reps, d_out, d_sink);
    k_walk<2><<<1, 64>>>(d_em, d_amt, reps, d_out, d_sink);
    k_walk<3><<<1, 64>>>(d_em, d_amt, reps, d_out, d_sink);
    k_walk<4><<<1, 64>>>(d_em, d_amt, reps, d_out, d_sink);
    k_walk<5><<<1, 64>>>(d_em, d_amt, reps, d_out, d_sink);
    k_walk<6><<<1, 64>>>(d_em, d_amt, reps, d_out, d_sink);
    k_walk<7><<<1, 64>>>(d_em, d_amt, reps, d_out, d_sink);
    if (hipDeviceSynchronize() != hipSuccess) {
      printf("error\n");
      return 1;
    }
  }
  unsigned long long h_out[8];
  (void)hipMemcpy(h_out, d_out, sizeof h_out, hipMemcpyDeviceToHost);
  const double steps = (double)reps * (N / 64);
  const char* names[8] = {"full step", "no failure search", "scan + dent store", "scan only",
                          "fast-path failures", "fast-path, 1 round", "scan + cur + dent", "scan + B + dent"};
  for (int v = 0; v < 8; v++) printf("%-20s %8.1f cycles per 64-entry step\n", names[v], h_out[v] / steps);
  return 0;
}
