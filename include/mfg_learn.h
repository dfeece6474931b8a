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

#ifdef __cplusplus
}
#endif
#endif
