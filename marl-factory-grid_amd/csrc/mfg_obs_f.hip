// mfg_obs_f.hip — the long-ray observation render (k_obs_lr, MP = 0: rays of 65..255 points, see mfg_kernels.h):
// pomdp_r 32..126 and full observability on levels whose shorter side is 64..254 cells.
#define MFG_OBS_UNIT
#include "mfg_kernels.h"

MFG_DEFINE_LAUNCH_OBS
MFG_INSTANTIATE_OBS(0)
