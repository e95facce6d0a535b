// kp_ffd_pref_resv_topo.hip — the topology instantiations of kp_ffd_pref_resv.hip, built with KP_NWAVES_TOPO waves: the
// topology path's registers spill at 8 waves (256 VGPRs each), at 4 they fit (512 per wave, the rest in AGPRs), and the
// serial chain runs faster for it (config 3: 745 -> 700 ms) while the other solves keep 8 waves (config 2: 94 vs 104 ms).
// The launcher (kp_launch_ffd) and the LDS plan (kp_ffd_plan_lds: kp_ffd_shared_bytes_topo) use the same count.
#ifndef KP_NWAVES_TOPO
#define KP_NWAVES_TOPO 4  // kp_layout.h
#endif
#define KP_NWAVES KP_NWAVES_TOPO
#include "kp_ffd.h"

__global__ __launch_bounds__(KP_NWAVES * 64) void ffd_pref_resv_topo_kernel(KpDev d) { ffd_solve<true, true, true>(d); }
__global__ __launch_bounds__(KP_NWAVES * 64) void ffd_pref_resv_topo_hbm_kernel(KpDev d) { ffd_solve<true, true, true, true>(d); }
