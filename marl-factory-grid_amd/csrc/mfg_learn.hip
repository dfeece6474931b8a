// Learner-side kernels of the on-GPU A2C loop (mfg_amd/marl.py): the elementwise half of one
// GRU step of the learner's window, forward and backward, each as ONE kernel instead of the ~10 / ~15 PyTorch
// elementwise launches per step and GRU (the window's GEMMs stay library calls). PyTorch gate order r, z, n
// (torch.nn.GRU, layer 0), the same formulas in the same evaluation order as _GRUWindow's tensor code
// (marl.py), fp32; -ffp-contract=off keeps the products and sums separately rounded as in that code.
// Rows i < n, columns j < hd; one thread per (i, j). Pointers are pre-offset to step s; *_row are row strides in
// elements (views of [n, t, ...] buffers).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/mfg_learn.h"

namespace {

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// h' = n + z (hp - n), hp = h keep, r = s(gi_r + gh_r), z = s(gi_z + gh_z), n = tanh(gi_n + r gh_n),
// gh = keep (h W_hh^T) + b_hh (gh0 = h W_hh^T without bias: keep in {0, 1} commutes with the GEMM)
__global__ void __launch_bounds__(256) k_gru_fwd(const float* __restrict__ gi, int64_t gi_row,
                                                 const float* __restrict__ gh0, const float* __restrict__ bh,
                                                 const float* __restrict__ h, int64_t h_row,
                                                 const float* __restrict__ keep, int64_t keep_row,
                                                 float* __restrict__ h_out, int64_t ho_row, float* __restrict__ hp_o,
                                                 float* __restrict__ r_o, float* __restrict__ z_o,
                                                 float* __restrict__ n_o, float* __restrict__ ghn_o, int64_t sv_row,
                                                 int64_t n, int hd) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n * hd) return;
  const int64_t i = k / hd;
  const int j = (int)(k - i * hd);
  const float kp = keep[i * keep_row];
  const float* g = gi + i * gi_row;
  const float* q = gh0 + i * (int64_t)(3 * hd);
  const float hp = h ? h[i * h_row + j] * kp : 0.0f;
  const float ar = q[j] * kp + bh[j], az = q[hd + j] * kp + bh[hd + j], ghn = q[2 * hd + j] * kp + bh[2 * hd + j];
  const float r = sigm(g[j] + ar);
  const float z = sigm(g[hd + j] + az);
  const float nn = tanhf(g[2 * hd + j] + r * ghn);
  h_out[i * ho_row + j] = nn + z * (hp - nn);
  const int64_t o = i * sv_row + j;
  hp_o[o] = hp; r_o[o] = r; z_o[o] = z; n_o[o] = nn; ghn_o[o] = ghn;
}

// dh = dout + keep_next dhp_next; dn = dh (1 - z) (1 - n^2); dz = dh (hp - n) z (1 - z); dr = dn ghn r (1 - r);
// dgi = [dr, dz, dn], dgh = [dr, dz, dn r], dhz = dh z (the recurrent GEMM then adds dgh W_hh)
__global__ void __launch_bounds__(256) k_gru_bwd(const float* __restrict__ dout, int64_t do_row,
                                                 const float* __restrict__ dhp, const float* __restrict__ keep_nx,
                                                 int64_t keep_row, const float* __restrict__ r_s,
                                                 const float* __restrict__ z_s, const float* __restrict__ n_s,
                                                 const float* __restrict__ ghn_s, const float* __restrict__ hp_s,
                                                 int64_t sv_row, float* __restrict__ dgi, int64_t dgi_row,
                                                 float* __restrict__ dgh, int64_t dgh_row, float* __restrict__ dhz,
                                                 int64_t n, int hd) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n * hd) return;
  const int64_t i = k / hd;
  const int j = (int)(k - i * hd);
  float dh = 0.0f;
  if (dhp) dh = dhp[i * hd + j] * keep_nx[i * keep_row];
  if (dout) dh = dout[i * do_row + j] + dh;
  const int64_t o = i * sv_row + j;
  const float r = r_s[o], z = z_s[o], nn = n_s[o], ghn = ghn_s[o], hp = hp_s[o];
  const float dn = dh * (1.0f - z) * (1.0f - nn * nn);
  const float dz = dh * (hp - nn) * z * (1.0f - z);
  const float dr = dn * ghn * r * (1.0f - r);
  float* a = dgi + i * dgi_row;
  float* b = dgh + i * dgh_row;
  a[j] = dr; a[hd + j] = dz; a[2 * hd + j] = dn;
  b[j] = dr; b[hd + j] = dz; b[2 * hd + j] = dn * r;
  dhz[i * hd + j] = dh * z;
}

int grid_for(int64_t n, int hd) { return (int)((n * hd + 255) / 256); }

}  // namespace

extern "C" int mfg_gru_fwd_step(const float* gi, int64_t gi_row, const float* gh0, const float* bh, const float* h,
                                int64_t h_row, const float* keep, int64_t keep_row, float* h_out, int64_t ho_row,
                                float* hp_out, float* r_out, float* z_out, float* n_out, float* ghn_out,
                                int64_t sv_row, int64_t n, int hd, void* stream) {
  if (n <= 0 || hd <= 0 || n * hd > (int64_t)INT32_MAX * 256) return -1;
  hipLaunchKernelGGL(k_gru_fwd, dim3(grid_for(n, hd)), dim3(256), 0, (hipStream_t)stream, gi, gi_row, gh0, bh, h,
                     h_row, keep, keep_row, h_out, ho_row, hp_out, r_out, z_out, n_out, ghn_out, sv_row, n, hd);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mfg_gru_bwd_step(const float* dout, int64_t do_row, const float* dhp_next, const float* keep_next,
                                int64_t keep_row, const float* r_s, const float* z_s, const float* n_s,
                                const float* ghn_s, const float* hp_s, int64_t sv_row, float* dgi, int64_t dgi_row,
                                float* dgh, int64_t dgh_row, float* dhz, int64_t n, int hd, void* stream) {
  if (n <= 0 || hd <= 0 || n * hd > (int64_t)INT32_MAX * 256) return -1;
  hipLaunchKernelGGL(k_gru_bwd, dim3(grid_for(n, hd)), dim3(256), 0, (hipStream_t)stream, dout, do_row, dhp_next,
                     keep_next, keep_row, r_s, z_s, n_s, ghn_s, hp_s, sv_row, dgi, dgi_row, dgh, dgh_row, dhz, n, hd);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
