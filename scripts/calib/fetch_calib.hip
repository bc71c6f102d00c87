// FETCH_SIZE calibration for the access shapes of K2 (diagnostic, scripts/gpu_calib.sh).
//
// MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reports 1/2 of the bytes of a wide coalesced
// streaming read; other widths are uncalibrated.  K2's traffic is divergent 16-byte row
// gathers, so this measures FETCH_SIZE per launch for a known access count:
//   stream   : S bytes read as 16 B / lane, fully coalesced (the guide's calibrated case)
//   gather16 : G random 16-byte loads, each in its own 128-byte line of a 4 GiB table
//              (> 256 MiB Infinity Cache: every load misses to HBM)
//   gather16x2: the same lines loaded twice in one launch by different waves (L2 reuse)
// Each kernel's line of output: name, loads, bytes requested, expected distinct lines, ms.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void k_stream(const uint4* __restrict__ a, uint64_t n, uint4* __restrict__ out) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) out[0] = acc;
}

__global__ void k_gather(const uint4* __restrict__ tab, const uint32_t* __restrict__ idx, uint64_t n,
                         uint4* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 v = tab[(uint64_t)idx[i] * 8u];   // line idx (128 B = 8 rows of 16 B)
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9e3779b9u) out[0] = v;
}

int main() {
  const uint64_t tab_bytes = 4ull << 30, lines = tab_bytes / 128;
  const uint64_t G = 8ull << 20;    // gathers per launch
  uint4 *tab = nullptr, *out = nullptr;
  uint32_t* idx = nullptr;
  CK(hipMalloc(&tab, tab_bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMalloc(&idx, G * 2 * 4));
  CK(hipMemset(tab, 1, tab_bytes));
  std::vector<uint32_t> h(G * 2);
  uint64_t s = 88172645463325252ull;
  for (uint64_t i = 0; i < G; ++i) {   // distinct random lines (a random permutation prefix)
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    h[i] = (uint32_t)(s % lines);
  }
  for (uint64_t i = 0; i < G; ++i) h[G + i] = h[(i * 2654435761ull) % G];   // second visit, other order
  std::vector<uint32_t> srt(h.begin(), h.begin() + G);
  std::sort(srt.begin(), srt.end());
  const uint64_t distinct = (uint64_t)(std::unique(srt.begin(), srt.end()) - srt.begin());
  CK(hipMemcpy(idx, h.data(), G * 2 * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  float ms = 0.f;
  // warm-up
  hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, 0, tab, tab_bytes / 16, out);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, 0, tab, tab_bytes / 16, out);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
  std::printf("stream loads=%llu bytes=%llu lines=%llu ms=%.3f GBps=%.0f\n", (unsigned long long)(tab_bytes / 16),
              (unsigned long long)tab_bytes, (unsigned long long)(tab_bytes / 128), ms, tab_bytes / ms / 1e6);
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(k_gather, dim3((uint32_t)(G / 256)), dim3(256), 0, 0, tab, idx, G, out);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
  std::printf("gather16 loads=%llu bytes=%llu lines=%llu ms=%.3f lines_per_s=%.3g\n", (unsigned long long)G,
              (unsigned long long)(G * 16), (unsigned long long)distinct, ms, distinct / ms * 1e3);
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(k_gather, dim3((uint32_t)(2 * G / 256)), dim3(256), 0, 0, tab, idx, 2 * G, out);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
  std::printf("gather16x2 loads=%llu bytes=%llu lines=%llu ms=%.3f\n", (unsigned long long)(2 * G),
              (unsigned long long)(2 * G * 16), (unsigned long long)distinct, ms);
  CK(hipFree(tab)); CK(hipFree(out)); CK(hipFree(idx));
  return 0;
}
