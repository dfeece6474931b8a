// issue_probe.hip — issue rates and latencies of the instruction kinds in k_replay's chunk on gfx950, the question
// behind its per-chunk cost: SALU vs VALU issue (do they co-issue?), the cost of taken / not-taken scalar branches,
// and the dependent latencies of the chunk's serial links (VALU, SALU, VALU->SGPR->SALU, the Jacobi round, LDS).
// Throughput kernels run ITER iterations of a 32-instruction body per wave (independent chains) with 8 waves per SIMD;
// latency kernels run one dependent chain with 1 wave per SIMD. Time per kernel from HIP events.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/issue_probe tools/issue_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITER 4096
#define S8(x) x x x x x x x x
// (every asm block that writes SCC declares it: the loop's own s_cmp/s_cbranch must not see a clobbered SCC)
__global__ void k_salu(int* out, int seed) {
  int a = seed, b = seed + 1, c = seed + 2, d = seed + 3;
#pragma nounroll
  for (int i = 0; i < ITER; i++) {
    asm volatile(S8("s_add_u32 %0, %0, 3\n\ts_add_u32 %1, %1, 5\n\ts_add_u32 %2, %2, 7\n\ts_add_u32 %3, %3, 9\n\t")
                 : "+s"(a), "+s"(b), "+s"(c), "+s"(d) : : "scc");  // s_add_u32 writes SCC
  }
  if (threadIdx.x == 0 && (a ^ b ^ c ^ d) == 0x12345) out[blockIdx.x] = 1;  // vector store, keeps the values
}
__global__ void k_valu(int* out, int seed) {
  int a = seed + threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITER; i++) {
    asm volatile(S8("v_add_u32 %0, %0, 3\n\tv_add_u32 %1, %1, 5\n\tv_add_u32 %2, %2, 7\n\tv_add_u32 %3, %3, 9\n\t")
                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
  }
  if ((a ^ b ^ c ^ d) == 0x12345) out[blockIdx.x] = 1;
}
// 16 SALU + 16 VALU per body (the same 32 instructions): co-issue gives max(), no co-issue gives the sum
__global__ void k_mixed(int* out, int seed) {
  int sa = seed, sb = seed + 1, va = seed + threadIdx.x, vb = va + 1;
#pragma nounroll
  for (int i = 0; i < ITER; i++) {
    asm volatile(S8("s_add_u32 %0, %0, 3\n\tv_add_u32 %2, %2, 7\n\ts_add_u32 %1, %1, 5\n\tv_add_u32 %3, %3, 9\n\t")
                 : "+s"(sa), "+s"(sb), "+v"(va), "+v"(vb) : : "scc");
  }
  if ((sa ^ sb ^ va ^ vb) == 0x12345) out[blockIdx.x] = 1;
}
// 32 s_cmp_lg_u32 + s_cselect pairs as in the replay's chunk control (SOPC + SOP2)
__global__ void k_scmp(int* out, int seed) {
  int a = seed, b = seed + 1, c = seed + 2, d = seed + 3;
#pragma nounroll
  for (int i = 0; i < ITER; i++) {
    asm volatile(S8("s_cmp_lg_u32 %0, 17\n\ts_cselect_b32 %1, %1, %2\n\ts_cmp_lg_u32 %2, 19\n\ts_cselect_b32 %3, %3, %0\n\t")
                 : "+s"(a), "+s"(b), "+s"(c), "+s"(d) : : "scc");
  }
  if (threadIdx.x == 0 && (a ^ b ^ c ^ d) == 0x12345) out[blockIdx.x] = 1;
}
// 8 x (s_cmp + not-taken s_cbranch_scc1 + 2 VALU): against k_valu's 32 VALU, the price of a not-taken branch
__global__ void k_br_nt(int* out, int seed) {
  int a = seed + threadIdx.x, b = a + 1, s = seed | 1;
#pragma nounroll
  for (int i = 0; i < ITER; i++) {
    asm volatile(S8("s_cmp_eq_u32 %2, 0\n\ts_cbranch_scc1 2f\n\tv_add_u32 %0, %0, 3\n\tv_add_u32 %1, %1, 5\n2:\n\t")
                 : "+v"(a), "+v"(b) : "s"(s) : "scc");
  }
  if ((a ^ b) == 0x12345) out[blockIdx.x] = 1;
}
// 8 x (taken s_branch to the next instruction + 2 VALU)
__global__ void k_br_t(int* out, int seed) {
  int a = seed + threadIdx.x, b = a + 1;
#pragma nounroll
  for (int i = 0; i < ITER; i++) {
    asm volatile(S8("s_branch 3f\n3:\n\tv_add_u32 %0, %0, 3\n\tv_add_u32 %1, %1, 5\n\t") : "+v"(a), "+v"(b));
  }
  if ((a ^ b) == 0x12345) out[blockIdx.x] = 1;
}
// the same 16 VALU alone (k_br_* minus their branches)
__global__ void k_valu16(int* out, int seed) {
  int a = seed + threadIdx.x, b = a + 1;
#pragma nounroll
  for (int i = 0; i < ITER; i++) {
    asm volatile(S8("v_add_u32 %0, %0, 3\n\tv_add_u32 %1, %1, 5\n\t") : "+v"(a), "+v"(b));
  }
  if ((a ^ b) == 0x12345) out[blockIdx.x] = 1;
}
// ---- dependent latencies (1 wave per SIMD): 32 links of one chain per iteration ----
__global__ void k_lat_valu(int* out, int seed) {
  int a = seed + threadIdx.x;
#pragma nounroll
  for (int i = 0; i < ITER; i++) asm volatile(S8("v_add_u32 %0, %0, 3\n\tv_add_u32 %0, %0, 5\n\tv_add_u32 %0, %0, 7\n\tv_add_u32 %0, %0, 9\n\t") : "+v"(a));
  if (a == 0x12345) out[blockIdx.x] = 1;
}
__global__ void k_lat_salu(int* out, int seed) {
  int a = seed;
#pragma nounroll
  for (int i = 0; i < ITER; i++) asm volatile(S8("s_add_u32 %0, %0, 3\n\ts_add_u32 %0, %0, 5\n\ts_add_u32 %0, %0, 7\n\ts_add_u32 %0, %0, 9\n\t") : "+s"(a) : : "scc");
  if (threadIdx.x == 0 && a == 0x12345) out[blockIdx.x] = 1;
}
// VALU -> SGPR -> SALU -> VALU: v_cmp (to an SGPR pair), s_bcnt1, v_add of the count; 32 links = 32 x 3 instructions
__global__ void k_lat_vsv(int* out, int seed) {
  int v = seed + threadIdx.x;
  uint64_t m;
  int s;
#pragma nounroll
  for (int i = 0; i < ITER; i++)
    asm volatile(S8("v_cmp_gt_u32 %1, %0, 40\n\ts_bcnt1_i32_b64 %2, %1\n\tv_add_u32 %0, %2, %0\n\t"
                    "v_cmp_gt_u32 %1, %0, 40\n\ts_bcnt1_i32_b64 %2, %1\n\tv_add_u32 %0, %2, %0\n\t"
                    "v_cmp_gt_u32 %1, %0, 40\n\ts_bcnt1_i32_b64 %2, %1\n\tv_add_u32 %0, %2, %0\n\t"
                    "v_cmp_gt_u32 %1, %0, 40\n\ts_bcnt1_i32_b64 %2, %1\n\tv_add_u32 %0, %2, %0\n\t")
                 : "+v"(v), "=s"(m), "=s"(s) : : "scc");
  if (v == 0x12345) out[blockIdx.x] = 1;
}
// the Jacobi round of the chunk: m -> mbcnt_lo, mbcnt_hi, v_cmp_le (to m); 32 rounds
__device__ __forceinline__ uint64_t jround(uint64_t m, int c) {
  const int a = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  return __builtin_amdgcn_ballot_w64(a <= c);
}
__global__ void k_lat_jacobi(int* out, int seed) {
  const int c = (int)threadIdx.x - 3 + (seed & 1);
  uint64_t m = ~0ull;
#pragma nounroll
  for (int i = 0; i < ITER; i++) {
#pragma unroll
    for (int k = 0; k < 32; k++) m = jround(m, c + (k & 1));
  }
  if ((int)m == 0x12345) out[blockIdx.x] = 1;
}
// LDS round trip: a dependent ds_read_b32 chain (each read's value is the next address)
__global__ void k_lat_lds(int* out, int seed) {
  __shared__ uint32_t buf[64];
  buf[threadIdx.x] = ((threadIdx.x + 1 + (seed & 1)) & 63) * 4;
  __syncthreads();
  uint32_t p = threadIdx.x * 4;
#pragma nounroll
  for (int i = 0; i < ITER; i++)
    asm volatile(S8("ds_read_b32 %0, %0\n\ts_waitcnt lgkmcnt(0)\n\tds_read_b32 %0, %0\n\ts_waitcnt lgkmcnt(0)\n\t"
                    "ds_read_b32 %0, %0\n\ts_waitcnt lgkmcnt(0)\n\tds_read_b32 %0, %0\n\ts_waitcnt lgkmcnt(0)\n\t")
                 : "+v"(p) : : "memory");
  if (p == 0x12345) out[blockIdx.x] = 1;
}

int main() {
  int* out = nullptr;
  if (hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  // links: instructions per body counted for the per-instruction figure (throughput) or links per body (latency)
  struct K { const char* name; void (*f)(int*, int); int waves_per_simd; int per_body; };
  K ks[] = {{"salu", k_salu, 8, 32}, {"valu", k_valu, 8, 32}, {"mixed", k_mixed, 8, 32}, {"scmp_cselect", k_scmp, 8, 32},
            {"valu16", k_valu16, 8, 16}, {"br_nottaken_body", k_br_nt, 8, 16}, {"br_taken_body", k_br_t, 8, 16},
            {"lat_valu", k_lat_valu, 1, 32}, {"lat_salu", k_lat_salu, 1, 32}, {"lat_v_s_v_link", k_lat_vsv, 1, 32},
            {"lat_jacobi_round", k_lat_jacobi, 1, 32}, {"lat_lds_read", k_lat_lds, 1, 32},
            {"jacobi_8w", k_lat_jacobi, 8, 32}, {"v_s_v_8w", k_lat_vsv, 8, 32}};
  for (int rep = 0; rep < 2; rep++)
    for (auto& k : ks) {
      const int blocks = ncu * 4 * k.waves_per_simd;  // single-wave workgroups
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, out, rep);
      hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, out, rep);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double cyc = ms * 1e-3 * 2.4e9;  // cycles at 2.4 GHz
      // throughput: cycles per wave-body-unit per SIMD; latency (1 wave/SIMD): cycles per link
      const double per = cyc / (ITER * (double)k.per_body * k.waves_per_simd);
      if (rep) printf("%-18s %2d w/SIMD %.3f ms  %.3f cycles per %s\n", k.name, k.waves_per_simd, ms, per,
                      k.waves_per_simd == 1 ? "link (latency)" : "unit per SIMD");
    }
  hipFree(out);
  return 0;
}
