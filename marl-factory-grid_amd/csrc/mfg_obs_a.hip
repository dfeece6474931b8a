// mfg_obs_a.hip — observation-render instantiations for ray lengths 4, 6, 8 (see mfg_kernels.h).
#define MFG_OBS_UNIT
#include "mfg_kernels.h"

MFG_DEFINE_LAUNCH_OBS
MFG_INSTANTIATE_OBS(4)
MFG_INSTANTIATE_OBS(6)
MFG_INSTANTIATE_OBS(8)
