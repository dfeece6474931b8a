// mfg_obs_d.hip — observation-render instantiations for ray lengths 24, 32 (see mfg_kernels.h).
#define MFG_OBS_UNIT
#include "mfg_kernels.h"

MFG_DEFINE_LAUNCH_OBS
MFG_INSTANTIATE_OBS(24)
MFG_INSTANTIATE_OBS(32)
