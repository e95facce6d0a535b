// kp_ffd_pref.hip — Solve kernel entry points: preference relaxation / MIN_VALUES_POLICY=BestEffort (each with and without topology groups, and
// with the slice arrays in LDS or HBM).  ffd_solve is in kp_ffd.h; the launcher is kp_launch_ffd (kp_kernels.hip).
#include "kp_ffd.h"

__global__ __launch_bounds__(KP_NWAVES * 64) void ffd_pref_kernel(KpDev d) { ffd_solve<false, false, true>(d); }
__global__ __launch_bounds__(KP_NWAVES * 64) void ffd_pref_hbm_kernel(KpDev d) { ffd_solve<false, false, true, true>(d); }
