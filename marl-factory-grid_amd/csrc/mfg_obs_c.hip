// mfg_obs_c.hip — observation-render instantiations for ray lengths 16, 18 (see mfg_kernels.h).
#define MFG_OBS_UNIT
#include "mfg_kernels.h"

MFG_DEFINE_LAUNCH_OBS
MFG_INSTANTIATE_OBS(16)
MFG_INSTANTIATE_OBS(18)
