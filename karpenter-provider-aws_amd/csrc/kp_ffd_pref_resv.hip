// kp_ffd_pref_resv.hip — Solve kernel entry points: preference relaxation with reserved offerings (each with and without topology groups, and
// with the slice arrays in LDS or HBM).  ffd_solve is in kp_ffd.h; the launcher is kp_launch_ffd (kp_kernels.hip).
#include "kp_ffd.h"

__global__ __launch_bounds__(KP_NWAVES * 64) void ffd_pref_resv_kernel(KpDev d) { ffd_solve<true, false, true>(d); }
__global__ __launch_bounds__(KP_NWAVES * 64) void ffd_pref_resv_hbm_kernel(KpDev d) { ffd_solve<true, false, true, true>(d); }
