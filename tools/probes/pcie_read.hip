// Probe: device-initiated reads of mapped pinned host memory (the synchronous commit reads its request
// this way, host.inc request_src) against a copy-engine H2D, for a 1 MiB request. Prints one JSON line.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstring>
#include <algorithm>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int U>
__global__ void __launch_bounds__(256) k_read(uint4* __restrict__ dst, const uint4* __restrict__ src, uint32_t n16) {
  const uint32_t stride = gridDim.x * 256;
  for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < n16; k += stride * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) if (k + u * stride < n16) v[u] = src[k + u * stride];
#pragma unroll
    for (int u = 0; u < U; u++) if (k + u * stride < n16) dst[k + u * stride] = v[u];
  }
}

int main() {
  const size_t bytes = 1 << 20;
  const uint32_t n16 = bytes / 16;
  void* h;
  void* hd;
  void* d;
  CK(hipHostMalloc(&h, bytes, hipHostMallocMapped));
  CK(hipHostGetDevicePointer(&hd, h, 0));
  CK(hipMalloc(&d, bytes));
  memset(h, 1, bytes);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int reps = 50;
  printf("{");
  auto timeit = [&](const char* name, auto launch, bool comma) -> int {
    for (int i = 0; i < 5; i++) launch();
    CK(hipStreamSynchronize(s));
    std::vector<float> t;
    for (int i = 0; i < reps; i++) {
      CK(hipEventRecord(a, s));
      launch();
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      t.push_back(ms * 1000.f);
    }
    std::sort(t.begin(), t.end());
    printf("\"%s\": %.1f%s", name, t[reps / 2], comma ? ", " : "");
    fflush(stdout);
    return 0;
  };
  timeit("sdma_us", [&] { (void)hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s); }, true);
  for (uint32_t g : {32u, 64u, 128u, 256u, 512u, 1024u}) {
    char name[64];
    snprintf(name, sizeof name, "kern_g%u_u1_us", g);
    timeit(name, [&] { k_read<1><<<g, 256, 0, s>>>((uint4*)d, (const uint4*)hd, n16); }, true);
    snprintf(name, sizeof name, "kern_g%u_u4_us", g);
    timeit(name, [&] { k_read<4><<<g, 256, 0, s>>>((uint4*)d, (const uint4*)hd, n16); }, true);
  }
  // writes to host (the reply path)
  timeit("kern_write_g256_us", [&] { k_read<1><<<256, 256, 0, s>>>((uint4*)hd, (const uint4*)d, n16); }, true);
  timeit("empty_kernel_us", [&] { k_read<1><<<1, 256, 0, s>>>((uint4*)d, (const uint4*)d, 0); }, false);
  printf("}\n");
  return 0;
}
