// LDS cost probe for k_replay's access patterns (measurement tool, not part of the engine).
// Every wave of a full grid (8 waves per SIMD) issues blocks of 8 independent LDS instructions of one pattern and
// waits once per block, so the LDS array, not the latency, sets the time; the result is CU-cycles per
// wave-instruction (throughput). Round-3 finding from the first (latency-bound) form: 64 lanes on ONE dword with
// ds_mskor_rtn_b32 cost 128 cycles per instruction (same-address atomics serialise ~2 cycles per lane).
// build: hipcc --offload-arch=gfx950 -O3 -o build/lds_probe tools/lds_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 1024  // blocks of 8 instructions per wave
#define SLICE 4096  // bytes of LDS per wave
#define WPB 4

__device__ __forceinline__ uint32_t xs(uint32_t x) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; return x; }

#define MSK8(A, M, D)                                                                                      \
  asm volatile(                                                                                            \
      "ds_mskor_rtn_b32 %0, %8, %16, %17\n\tds_mskor_rtn_b32 %1, %9, %16, %17\n\t"                       \
      "ds_mskor_rtn_b32 %2, %10, %16, %17\n\tds_mskor_rtn_b32 %3, %11, %16, %17\n\t"                     \
      "ds_mskor_rtn_b32 %4, %12, %16, %17\n\tds_mskor_rtn_b32 %5, %13, %16, %17\n\t"                     \
      "ds_mskor_rtn_b32 %6, %14, %16, %17\n\tds_mskor_rtn_b32 %7, %15, %16, %17\n\ts_waitcnt lgkmcnt(0)" \
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7]) \
      : "v"(A[0]), "v"(A[1]), "v"(A[2]), "v"(A[3]), "v"(A[4]), "v"(A[5]), "v"(A[6]), "v"(A[7]), "v"(M), "v"(D) \
      : "memory")
#define RD8(OP, A)                                                                                        \
  asm volatile(OP " %0, %8\n\t" OP " %1, %9\n\t" OP " %2, %10\n\t" OP " %3, %11\n\t" OP " %4, %12\n\t" OP \
                  " %5, %13\n\t" OP " %6, %14\n\t" OP " %7, %15\n\ts_waitcnt lgkmcnt(0)"                   \
               : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]), \
                 "=&v"(r[7])                                                                               \
               : "v"(A[0]), "v"(A[1]), "v"(A[2]), "v"(A[3]), "v"(A[4]), "v"(A[5]), "v"(A[6]), "v"(A[7]) \
               : "memory")
#define WR8(OP, A, D)                                                                                     \
  asm volatile(OP " %0, %8\n\t" OP " %1, %8\n\t" OP " %2, %8\n\t" OP " %3, %8\n\t" OP " %4, %8\n\t" OP      \
                  " %5, %8\n\t" OP " %6, %8\n\t" OP " %7, %8\n\ts_waitcnt lgkmcnt(0)"                      \
               :                                                                                          \
               : "v"(A[0]), "v"(A[1]), "v"(A[2]), "v"(A[3]), "v"(A[4]), "v"(A[5]), "v"(A[6]), "v"(A[7]), "v"(D) \
               : "memory")

// patterns (all lanes issue unless noted; "acc" = ~72% of lanes, fixed per lane):
//  0 mskor consecutive dwords         1 mskor random dwords            2 mskor random acc, u16 sink pairs rest
//  3 mskor random acc, rest exec off  4 mskor random acc, dword sinks  5 mskor u16 i-range (ptop - A) pairs
//  10 read_u16 i-range                11 read_u16 acc i-range, u16 sink pairs rest   12 read_b32 consecutive
//  13 read_u16 i-range incl. rejected lanes (same address as the next accepted lane)
//  20 write_b16 i-range acc, sinks    21 write_b16 i-range acc, rest exec off        22 write_b32 consecutive
__global__ void __launch_bounds__(WPB * 64) k_probe(int pattern, uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  uint8_t* base = smem + wid * SLICE;
  const uint32_t b = (uint32_t)(uintptr_t)base;
  for (int i = 0; i < SLICE / 4 / 64; i++) ((uint32_t*)base)[i * 64 + lane] = lane;
  __builtin_amdgcn_wave_barrier();
  uint32_t s = 0x9e3779b9u * (blockIdx.x * 256 + threadIdx.x + 1);
  s = xs(s);
  const bool acc = (s & 1023) < 737;
  const uint64_t m = __ballot(acc);
  const int A = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
  uint32_t a[8];
  const uint32_t ptop = b + 2048, sink16 = b + 2 * lane, sink32 = b + 4 * lane;
  for (int k = 0; k < 8; k++) {
    s = xs(s);
    const uint32_t rnd = b + 256 + 4 * ((s >> 8) % 896);
    const uint32_t i16 = ptop - 2 * A - 128 * k;
    switch (pattern) {
      case 0: case 12: case 22: a[k] = b + 4 * lane + 256 * (k & 3); break;
      case 1: case 3: a[k] = rnd; break;
      case 2: a[k] = acc ? rnd : (sink16 & ~3u); break;
      case 4: a[k] = acc ? rnd : sink32; break;
      case 5: a[k] = i16 & ~3u; break;
      case 10: case 13: a[k] = i16; break;
      case 11: case 20: a[k] = acc ? i16 : sink16; break;
      case 21: a[k] = i16; break;
    }
  }
  uint32_t r[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t tot = 0;
  const uint32_t M = 0xffffu, D = lane;
  for (int it = 0; it < ITERS; it++) {
    switch (pattern) {
      case 0: case 1: case 2: case 4: case 5: MSK8(a, M, D); break;
      case 3: if (acc) MSK8(a, M, D); break;
      case 10: case 11: case 13: RD8("ds_read_u16", a); break;
      case 12: RD8("ds_read_b32", a); break;
      case 20: WR8("ds_write_b16", a, D); break;
      case 21: if (acc) WR8("ds_write_b16", a, D); break;
      case 22: WR8("ds_write_b32", a, D); break;
    }
    tot += r[0] ^ r[7];
  }
  if (tot == 0x12345678u) out[0] = tot;
}

int main() {
  uint32_t* out;
  (void)hipMalloc(&out, 4);
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const int blocks = cus * 8;  // 32 waves per CU at WPB 4
  const int pats[] = {0, 1, 2, 3, 4, 5, 10, 11, 12, 13, 20, 21, 22};
  hipEvent_t ea, ee;
  (void)hipEventCreate(&ea);
  (void)hipEventCreate(&ee);
  for (int pi = 0; pi < (int)(sizeof(pats) / sizeof(pats[0])); pi++) {
    const int pat = pats[pi];
    hipLaunchKernelGGL(k_probe, dim3(blocks), dim3(WPB * 64), WPB * SLICE, 0, pat, out);
    (void)hipEventRecord(ea, 0);
    for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k_probe, dim3(blocks), dim3(WPB * 64), WPB * SLICE, 0, pat, out);
    (void)hipEventRecord(ee, 0);
    (void)hipEventSynchronize(ee);
    float ms;
    (void)hipEventElapsedTime(&ms, ea, ee);
    const double ops_per_cu = 3.0 * 32 * ITERS * 8;  // wave-instructions per CU
    printf("pattern %2d: %.3f ms, %.2f CU-cycles per wave-instruction\n", pat, ms, ms * 1e-3 * 2.4e9 / ops_per_cu);
  }
  return 0;
}
