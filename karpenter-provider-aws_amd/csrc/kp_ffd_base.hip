// kp_ffd_base.hip — Solve kernel entry points: no reserved offerings, no preference relaxation (each with and without topology groups, and
// with the slice arrays in LDS or HBM).  ffd_solve is in kp_ffd.h; the launcher is kp_launch_ffd (kp_kernels.hip).
#include "kp_ffd.h"

// One named entry point per feature instantiation, so kernel traces (rocprofv3 --stats) report the common case
// (ffd_kernel: no topology groups, no reserved offerings) separately from the topology / reservation variants.
__global__ __launch_bounds__(KP_NWAVES * 64) void ffd_kernel(KpDev d) { ffd_solve<false, false, false>(d); }
__global__ __launch_bounds__(KP_NWAVES * 64) void ffd_hbm_kernel(KpDev d) { ffd_solve<false, false, false, true>(d); }
