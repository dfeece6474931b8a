// wcal.hip — calibration of rocprofv3's WRITE_SIZE / FETCH_SIZE on the store and load widths k_logic uses
// (MI355X_MICROARCH.md, HBM: WRITE_SIZE is calibrated only for 16-B-per-lane streaming stores). Each kernel writes
// (or reads) a known byte count with one wave per "env" (65,536 waves, the C3 batch), like k_logic's outputs:
//   w_u8_lane0    done[B]: lane 0 of each wave stores 1 byte            (65,536 B)
//   w_u8_x8       ev_act[B][8]: lanes 0..7 store 1 byte each            (524,288 B)
//   w_f64_x8      reward[B][8]: lanes 0..7 store 8 bytes each           (4,194,304 B)
//   w_i32_x12     ev_misc[B][12]: lanes 0..11 store 4 bytes each        (3,145,728 B)
//   w_rec16_x10   10 scattered 16-B chunks of a 5,280-B record per wave (10,485,760 B), like k_logic's write-back
//   w_16b_stream  16 B per lane, contiguous (the guide's calibrated form: 16,777,216 B)
//   r_rec496      the 496-B step prefix of each 5,280-B record, 16 B per lane (32,505,856 B)
// Build: hipcc --offload-arch=gfx950 -O3 -o build/wcal tools/wcal.hip
// Run:   rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/wcal_w -o run --output-format csv -- build/wcal
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define B 65536
#define REC 5280

__global__ void w_u8_lane0(uint8_t* d) { if (threadIdx.x == 0) d[blockIdx.x] = (uint8_t)blockIdx.x; }
__global__ void w_u8_x8(uint8_t* d) { if (threadIdx.x < 8) d[blockIdx.x * 8 + threadIdx.x] = (uint8_t)threadIdx.x; }
__global__ void w_f64_x8(double* d) { if (threadIdx.x < 8) d[blockIdx.x * 8 + threadIdx.x] = 1.0 + threadIdx.x; }
__global__ void w_i32_x12(int* d) { if (threadIdx.x < 12) d[blockIdx.x * 12 + threadIdx.x] = threadIdx.x; }
__global__ void w_rec16_x10(uint8_t* rec) {
  // chunks 0, 2, 5, 6, 9, 12, 17, 20, 25, 30 of the record's 16-B chunks (header, counters, agents, doors, battery)
  const int ch[10] = {0, 2, 5, 6, 9, 12, 17, 20, 25, 30};
  if (threadIdx.x < 10) ((uint4*)(rec + (size_t)blockIdx.x * REC))[ch[threadIdx.x]] = make_uint4(1, 2, 3, threadIdx.x);
}
__global__ void w_16b_stream(uint4* d) { d[(size_t)blockIdx.x * 64 + threadIdx.x] = make_uint4(1, 2, 3, threadIdx.x); }
__global__ void r_rec496(const uint8_t* rec, int* out) {
  uint4 v = make_uint4(0, 0, 0, 0);
  if (threadIdx.x < 31) v = ((const uint4*)(rec + (size_t)blockIdx.x * REC))[threadIdx.x];
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x7FFFFFFF) out[0] = 1;  // keeps the load
}

int main() {
  uint8_t* buf = nullptr;
  int* flag = nullptr;
  const size_t bytes = (size_t)B * REC;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&flag, 4) != hipSuccess) return 1;
  hipMemset(buf, 0, bytes);
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(w_u8_lane0, dim3(B), dim3(64), 0, 0, buf);
    hipLaunchKernelGGL(w_u8_x8, dim3(B), dim3(64), 0, 0, buf);
    hipLaunchKernelGGL(w_f64_x8, dim3(B), dim3(64), 0, 0, (double*)buf);
    hipLaunchKernelGGL(w_i32_x12, dim3(B), dim3(64), 0, 0, (int*)buf);
    hipLaunchKernelGGL(w_rec16_x10, dim3(B), dim3(64), 0, 0, buf);
    hipLaunchKernelGGL(w_16b_stream, dim3(B / 4), dim3(64), 0, 0, (uint4*)buf);
    hipLaunchKernelGGL(r_rec496, dim3(B), dim3(64), 0, 0, buf, flag);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("wcal: bytes written per launch: u8_lane0 %d, u8_x8 %d, f64_x8 %d, i32_x12 %d, rec16_x10 %d, 16b_stream %d; "
         "read rec496 %d\n", B, B * 8, B * 64, B * 48, B * 160, B / 4 * 1024, B * 496);
  hipFree(buf);
  hipFree(flag);
  return 0;
}
