// mfg_obs_b.hip — observation-render instantiations for ray lengths 10, 12, 14 (see mfg_kernels.h).
#define MFG_OBS_UNIT
#include "mfg_kernels.h"

MFG_DEFINE_LAUNCH_OBS
MFG_INSTANTIATE_OBS(10)
MFG_INSTANTIATE_OBS(12)
MFG_INSTANTIATE_OBS(14)
