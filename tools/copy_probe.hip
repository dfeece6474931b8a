// HBM copy-kernel probe (bench.py's measured peak, mfg_hbm_copy): read+write GB/s of several 16-B-per-lane copy forms
// over 2 GiB, best of 10 after a warm-up. usage: build/tools/copy_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef unsigned v4u __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) k_flat(uint4* __restrict__ d, const uint4* __restrict__ s, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) d[i] = s[i];
}
__global__ void __launch_bounds__(256) k_flat_nt(uint4* __restrict__ d, const uint4* __restrict__ s, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load((const v4u*)&s[i]), (v4u*)&d[i]);
}
template <int U>
__global__ void __launch_bounds__(256) k_unroll(uint4* __restrict__ d, const uint4* __restrict__ s, long long n) {
  // each block copies U * 256 consecutive uint4, lane-strided (coalesced per instruction)
  const long long b = (long long)blockIdx.x * (U * 256) + threadIdx.x;
  uint4 v[U];
#pragma unroll
  for (int u = 0; u < U; u++) v[u] = b + u * 256 < n ? s[b + u * 256] : make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int u = 0; u < U; u++) if (b + u * 256 < n) d[b + u * 256] = v[u];
}
template <int U>
__global__ void __launch_bounds__(256) k_unroll_nt(uint4* __restrict__ d, const uint4* __restrict__ s, long long n) {
  const long long b = (long long)blockIdx.x * (U * 256) + threadIdx.x;
  v4u v[U];
#pragma unroll
  for (int u = 0; u < U; u++) v[u] = b + u * 256 < n ? __builtin_nontemporal_load((const v4u*)&s[b + u * 256]) : v4u{0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < U; u++) if (b + u * 256 < n) __builtin_nontemporal_store(v[u], (v4u*)&d[b + u * 256]);
}
__global__ void __launch_bounds__(256) k_grid(uint4* __restrict__ d, const uint4* __restrict__ s, long long n) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const uint4 a = s[i], b = s[i + stride], c = s[i + 2 * stride], e = s[i + 3 * stride];
    d[i] = a; d[i + stride] = b; d[i + 2 * stride] = c; d[i + 3 * stride] = e;
  }
  for (; i < n; i += stride) d[i] = s[i];
}

int main() {
  const size_t bytes = 2ull << 30;
  const long long n = (long long)(bytes / 16);
  uint4 *a, *b;
  if (hipMalloc(&a, bytes) || hipMalloc(&b, bytes)) { printf("alloc failed\n"); return 1; }
  hipMemset(a, 1, bytes);
  hipMemset(b, 0, bytes);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int ncu = 256;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  auto run = [&](const char* name, auto launch) {
    launch();
    float best = 1e30f;
    for (int r = 0; r < 10; r++) {
      hipEventRecord(e0, 0);
      launch();
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    printf("%-16s %8.1f GB/s  (%.3f ms)\n", name, 2.0 * bytes / (best * 1e-3) / 1e9, best);
  };
  const unsigned g1 = (unsigned)((n + 255) / 256);
  run("flat", [&] { hipLaunchKernelGGL(k_flat, dim3(g1), dim3(256), 0, 0, b, a, n); });
  run("flat_nt", [&] { hipLaunchKernelGGL(k_flat_nt, dim3(g1), dim3(256), 0, 0, b, a, n); });
  run("unroll4", [&] { hipLaunchKernelGGL(k_unroll<4>, dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, 0, b, a, n); });
  run("unroll4_nt", [&] { hipLaunchKernelGGL(k_unroll_nt<4>, dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, 0, b, a, n); });
  run("unroll8_nt", [&] { hipLaunchKernelGGL(k_unroll_nt<8>, dim3((unsigned)((n + 2047) / 2048)), dim3(256), 0, 0, b, a, n); });
  run("unroll2", [&] { hipLaunchKernelGGL(k_unroll<2>, dim3((unsigned)((n + 511) / 512)), dim3(256), 0, 0, b, a, n); });
  run("grid8/CU", [&] { hipLaunchKernelGGL(k_grid, dim3(8 * ncu), dim3(256), 0, 0, b, a, n); });
  run("grid32/CU", [&] { hipLaunchKernelGGL(k_grid, dim3(32 * ncu), dim3(256), 0, 0, b, a, n); });
  run("hipMemcpy", [&] { hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0); });
  return 0;
}
