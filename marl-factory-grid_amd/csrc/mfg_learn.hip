// Learner-side kernels of the on-GPU A2C loop (mfg_amd/marl.py): the elementwise half of one
// GRU step of the learner's window, forward and backward, each as ONE kernel instead of the ~10 / ~15 PyTorch
// elementwise launches per step and GRU (the window's GEMMs stay library calls). PyTorch gate order r, z, n
// (torch.nn.GRU, layer 0), the same formulas in the same evaluation order as _GRUWindow's tensor code
// (marl.py), fp32; -ffp-contract=off keeps the products and sums separately rounded as in that code.
// Rows i < n, columns j < hd; one thread per (i, j). Pointers are pre-offset to step s; *_row are row strides in
// elements (views of [n, t, ...] buffers).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
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

// ---- packed rows to dense: out[r][:k] = the row with val[j] at idx[j] and zeros elsewhere (the learner's dense obs
// rows for the obs_proj weight-gradient GEMM). One wave per row through a wave-private LDS row: zero it, store the
// entries (distinct positions), read it back and store it coalesced; LDS instructions of one wave complete in
// issue order, so no barrier is needed between the phases (a wave barrier keeps the compiler from moving them).
__global__ void __launch_bounds__(256) k_packed_densify(const uint16_t* __restrict__ idx, const float* __restrict__ val,
                                                        int64_t m, int cap, int k, float* __restrict__ out,
                                                        int64_t out_row) {
  extern __shared__ float rowbuf[];  // [4][k]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* rb = rowbuf + wv * k;
  for (int64_t r = (int64_t)blockIdx.x * 4 + wv; r < m; r += (int64_t)gridDim.x * 4) {
    for (int c = lane; c < k; c += 64) rb[c] = 0.0f;
    __builtin_amdgcn_wave_barrier();
    for (int j = lane; j < cap; j += 64) {
      const float v = val[r * cap + j];
      const int kk = idx[r * cap + j];
      if (v != 0.0f && kk < k) rb[kk] = v;
    }
    __builtin_amdgcn_wave_barrier();
    float* o = out + r * out_row;
    for (int c = lane; c < k; c += 64) o[c] = rb[c];
    __builtin_amdgcn_wave_barrier();
  }
}

// ---- packed-row projection: out[r] = bias + sum_j val_j wt[idx_j] (obs_proj on packed rows, the same sum the
// render's fused projection forms); one wave per row, lanes on the e_dim columns (two passes past 64)
__global__ void __launch_bounds__(256) k_packed_project(const uint16_t* __restrict__ idx,
                                                        const float* __restrict__ val, int64_t m, int cap,
                                                        const float* __restrict__ wt, const float* __restrict__ bias,
                                                        int e_dim, int k, float* __restrict__ out, int64_t out_row) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= m) return;
  for (int c0 = 0; c0 < e_dim; c0 += 64) {
    const int c = c0 + lane;
    const bool on = c < e_dim;
    float acc = 0.0f;
    for (int j0 = 0; j0 < cap; j0 += 64) {
      const bool in = j0 + lane < cap;
      const uint32_t my_i = in ? idx[r * cap + j0 + lane] : 0u;
      const float my_v = in ? val[r * cap + j0 + lane] : 0.0f;
      uint64_t nz = __ballot(my_v != 0.0f);
      const bool more = nz == ~0ull;
      while (nz) {
        const int j = __builtin_ctzll(nz);
        nz &= nz - 1;
        const int kk = __builtin_amdgcn_readlane((int)my_i, j);
        const float v = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_v), j));
        if (on && kk < k) acc += v * wt[(int64_t)kk * e_dim + c];
      }
      if (!more) break;
    }
    if (on) out[r * out_row + c] = bias[c] + acc;
  }
}

// ---- categorical sampling: a ~ softmax(logits[r]) by inversion of the CDF at u[r] * sum (u uniform in [0, 1)):
// max, exp-sum and search in one pass per row (one thread per row; n_act is small)
__global__ void __launch_bounds__(256) k_sample_cat(const float* __restrict__ logits, int64_t lrow, int n_act,
                                                    const float* __restrict__ u, int64_t n, int32_t* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const float* l = logits + r * lrow;
  float mx = l[0];
  for (int a = 1; a < n_act; a++) mx = fmaxf(mx, l[a]);
  float s = 0.0f;
  for (int a = 0; a < n_act; a++) s += expf(l[a] - mx);
  if (!(s > 0.0f) || isinf(s)) {  // non-finite logits (NaN / inf): no distribution; -1 lets the caller report it
    out[r] = -1;
    return;
  }
  const float thr = u[r] * s;
  float c = 0.0f;
  int pick = n_act - 1;  // rounding past the last bin picks the last action
  for (int a = 0; a < n_act; a++) {
    c += expf(l[a] - mx);
    if (thr < c) { pick = a; break; }
  }
  out[r] = pick;
}

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

extern "C" int mfg_packed_densify(const uint16_t* idx, const float* val, int64_t m, int cap, int k, float* out,
                                  int64_t out_row, void* stream) {
  if (m <= 0 || cap <= 0 || k <= 0 || out_row < k || (size_t)k * 4 * sizeof(float) > 65536) return -1;
  const int64_t nb = std::min<int64_t>((m + 3) / 4, 8192);
  hipLaunchKernelGGL(k_packed_densify, dim3((unsigned)nb), dim3(256), (size_t)k * 4 * sizeof(float),
                     (hipStream_t)stream, idx, val, m, cap, k, out, out_row);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mfg_packed_project(const uint16_t* idx, const float* val, int64_t m, int cap, const float* wt,
                                  const float* bias, int e_dim, int k, float* out, int64_t out_row, void* stream) {
  if (m <= 0 || cap <= 0 || e_dim <= 0 || k <= 0 || out_row < e_dim) return -1;
  hipLaunchKernelGGL(k_packed_project, dim3((unsigned)((m + 3) / 4)), dim3(256), 0, (hipStream_t)stream, idx, val, m,
                     cap, wt, bias, e_dim, k, out, out_row);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mfg_sample_categorical(const float* logits, int64_t logit_row, int n_act, const float* u, int64_t n,
                                      int32_t* out, void* stream) {
  if (n <= 0 || n_act <= 0 || logit_row < n_act) return -1;
  hipLaunchKernelGGL(k_sample_cat, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, logits,
                     logit_row, n_act, u, n, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
