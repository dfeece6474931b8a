// mfg_obs_e.hip — observation-render instantiations for ray lengths 48, 64 (see mfg_kernels.h): pomdp_r 16..31 and
// full observability on levels whose shorter side is 32..63 cells (64-bit point masks).
#define MFG_OBS_UNIT
#include "mfg_kernels.h"

MFG_DEFINE_LAUNCH_OBS
MFG_INSTANTIATE_OBS(48)
MFG_INSTANTIATE_OBS(64)
