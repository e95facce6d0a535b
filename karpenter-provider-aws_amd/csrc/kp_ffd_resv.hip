// kp_ffd_resv.hip — Solve kernel entry points: reserved offerings (ReservationManager) (each with and without topology groups, and
// with the slice arrays in LDS or HBM).  ffd_solve is in kp_ffd.h; the launcher is kp_launch_ffd (kp_kernels.hip).
#include "kp_ffd.h"

__global__ __launch_bounds__(KP_NWAVES * 64) void ffd_resv_kernel(KpDev d) { ffd_solve<true, false, false>(d); }
__global__ __launch_bounds__(KP_NWAVES * 64) void ffd_resv_hbm_kernel(KpDev d) { ffd_solve<true, false, false, true>(d); }
