/* mfg_learn.h — learner-side helpers of the on-GPU A2C loop (mfg_amd/marl.py BatchedA2C).
 *
 * Not part of the Factory.step boundary (include/mfg.h): the elementwise half of one GRU step of the learner's
 * window (torch.nn.GRU layer 0, gate order r, z, n), forward and backward, as one kernel each. They replace the
 * ~10 / ~15 PyTorch elementwise launches per step and GRU of the reference learner's recurrent pass
 * (algorithms/marl/networks.py:50-69 forward, autograd backward; base_ac.py:200-225 update). fp32, device
 * pointers pre-offset to step s, *_row = row strides in elements, launched on `stream` (a hipStream_t);
 * return 0, or -1 on a bad size or launch error. */
#ifndef MFG_LEARN_H
#define MFG_LEARN_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* h_out = n + z (hp - n) with hp = h keep (h NULL: zero state), gh = keep gh0 + bh, gh0 = h W_hh^T [n, 3hd]
 * contiguous, gi [n, 3hd] = x W_ih^T + b_ih; also stores hp, r, z, n, gh_n (the backward's inputs). */
int mfg_gru_fwd_step(const float* gi, int64_t gi_row, const float* gh0, const float* bh, const float* h,
                     int64_t h_row, const float* keep, int64_t keep_row, float* h_out, int64_t ho_row,
                     float* hp_out, float* r_out, float* z_out, float* n_out, float* ghn_out, int64_t sv_row,
                     int64_t n, int hd, void* stream);

/* dh = dout + keep_next dhp_next (either NULL: absent); writes dgi = [dr, dz, dn], dgh = [dr, dz, dn r] and
 * dhz = dh z [n, hd] contiguous (dhp of this step = dhz + dgh W_hh, a GEMM by the caller). */
int mfg_gru_bwd_step(const float* dout, int64_t do_row, const float* dhp_next, const float* keep_next,
                     int64_t keep_row, const float* r_s, const float* z_s, const float* n_s, const float* ghn_s,
                     const float* hp_s, int64_t sv_row, float* dgi, int64_t dgi_row, float* dgh, int64_t dgh_row,
                     float* dhz, int64_t n, int hd, void* stream);

/* the packed rows (idx u16 / val f32 [m, cap], a row's entries distinct, zero vals ignored) as dense f32 rows
 * out [m][k] (row stride out_row >= k; k <= 4096): the learner's D for obs_proj's weight gradient D^T g (replaces a
 * zero fill + scatter_add; marl.py _packed_grads). */
int mfg_packed_densify(const uint16_t* idx, const float* val, int64_t m, int cap, int k, float* out, int64_t out_row,
                       void* stream);

/* out[r][:e_dim] = bias + sum_j val[r][j] wt[idx[r][j]] for the packed rows (wt [k][e_dim] = obs_proj.weight^T), the
 * projection the render fuses (mfg_packed_obs.emb), for rows held outside a render (the learner's window slide). */
int mfg_packed_project(const uint16_t* idx, const float* val, int64_t m, int cap, const float* wt, const float* bias,
                       int e_dim, int k, float* out, int64_t out_row, void* stream);

/* out[r] ~ Categorical(logits = logits[r][:n_act]) by inversion at u[r] in [0, 1) (the acting step's
 * Categorical(logits).sample(), base_ac.py:74-76, with the uniforms drawn by the caller); -1 for a row whose
 * logits are not finite (torch.distributions would raise there) */
int mfg_sample_categorical(const float* logits, int64_t logit_row, int n_act, const float* u, int64_t n, int32_t* out,
                           void* stream);

#ifdef __cplusplus
}
#endif
#endif
