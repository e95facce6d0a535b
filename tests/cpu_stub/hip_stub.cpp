// TEST INFRASTRUCTURE — CPU stand-ins for the HIP runtime calls and the kernel launchers that kp_host.cpp links against
// (see hip/hip_runtime.h).  The launchers do not schedule anything: they write deterministic placeholder results so the
// host layer's encoding, buffer management, multi-device sharding and decoding run end to end under ThreadSanitizer.
//   ffd / finalize : every pod unschedulable, no NodeClaims;
//   consolidate    : probe i (global index probe0 + i) reports n_pods = i, decision = i % 3, candidate_price = i;
//   queue sort     : identity permutation.
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>

#include "hip/hip_runtime.h"
#include "../../karpenter-provider-aws_amd/csrc/kp_cons.h"
#include "../../karpenter-provider-aws_amd/csrc/kp_launch.h"
#include "../../karpenter-provider-aws_amd/csrc/kp_layout.h"

static thread_local int t_device = 0;
static int n_devices() {
    const char* e = getenv("KP_STUB_DEVICES");
    return e ? atoi(e) : 2;
}
struct ihipStream_t {
    int device;
};
struct ihipEvent_t {
    std::atomic<int64_t> ns{0};
};

hipError_t hipGetDeviceCount(int* n) {
    *n = n_devices();
    return hipSuccess;
}
hipError_t hipSetDevice(int d) {
    if (d < 0 || d >= n_devices()) return hipErrorInvalidDevice;
    t_device = d;
    return hipSuccess;
}
hipError_t hipGetDeviceProperties(hipDeviceProp_t* p, int d) {
    if (d < 0 || d >= n_devices()) return hipErrorInvalidDevice;
    memset(p, 0, sizeof *p);
    strcpy(p->name, "cpu stub");
    strcpy(p->gcnArchName, "gfx950:sramecc+:xnack-");
    p->totalGlobalMem = (size_t)1 << 34;
    p->multiProcessorCount = 256;
    return hipSuccess;
}
const char* hipGetErrorString(hipError_t e) { return e == hipSuccess ? "hipSuccess" : "stub error"; }
hipError_t hipMalloc(void** p, size_t bytes) {
    *p = calloc(1, bytes ? bytes : 1);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void* p) {
    free(p);
    return hipSuccess;
}
hipError_t hipHostMalloc(void** p, size_t bytes, unsigned) { return hipMalloc(p, bytes); }
hipError_t hipHostFree(void* p) { return hipFree(p); }
hipError_t hipMemcpy(void* dst, const void* src, size_t bytes, hipMemcpyKind) {
    if (bytes) memmove(dst, src, bytes);
    return hipSuccess;
}
hipError_t hipMemcpyAsync(void* dst, const void* src, size_t bytes, hipMemcpyKind k, hipStream_t) {
    return hipMemcpy(dst, src, bytes, k);
}
hipError_t hipMemsetAsync(void* dst, int v, size_t bytes, hipStream_t) {
    if (bytes) memset(dst, v, bytes);
    return hipSuccess;
}
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned) {
    *s = new ihipStream_t{t_device};
    return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) {
    delete s;
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipEventCreate(hipEvent_t* e) {
    *e = new ihipEvent_t;
    return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t e) {
    delete e;
    return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t e, hipStream_t) {
    e->ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
    return hipSuccess;
}
hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
hipError_t hipEventElapsedTime(float* ms, hipEvent_t a, hipEvent_t b) {
    *ms = (float)((b->ns - a->ns) * 1e-6);
    return hipSuccess;
}

// ---- kernel launchers (the real ones live in kp_kernels.hip / kp_consolidate.hip / kp_launch.hip) ----
size_t kp_ffd_shared_bytes() { return 0; }
size_t kp_ffd_shared_bytes_topo() { return 0; }
bool kp_ffd_plan_lds(KpDev& d, int) {
    d.lds_ncmax = d.NCcap < KP_MAX_NC ? d.NCcap : KP_MAX_NC;
    d.lds_tpad = (d.T + 63) / 64 * 64;
    d.lds_A = 0;
    d.lds_nq = 0;
    d.lds_bytes = 0;
    return true;
}
hipError_t kp_launch_class_mask(const KpDev&, hipStream_t) { return hipSuccess; }
hipError_t kp_launch_template_init(const KpDev&, hipStream_t) { return hipSuccess; }
hipError_t kp_launch_existing(const KpDev&, hipStream_t) { return hipSuccess; }
hipError_t kp_launch_ffd(const KpDev& d, hipStream_t) {
    for (int p = 0; p < d.P; p++) {
        d.pod_result[p] = -1;
        d.pod_order[p] = -1;
    }
    d.nc_count[0] = 0;
    d.err[0] = 0;
    return hipSuccess;
}
hipError_t kp_ffd_set_attributes() { return hipSuccess; }
hipError_t kp_cons_set_attributes() { return hipSuccess; }
hipError_t kp_launch_finalize(const KpDev&, int, hipStream_t) { return hipSuccess; }
bool kp_cons_plan_lds(const KpDev&, KpCons& k, int) {
    k.lds_bytes = 1024;
    return true;
}
hipError_t kp_launch_select_kernel(const KpLaunch&, hipStream_t) { return hipSuccess; }
hipError_t kp_launch_consolidate(const KpDev&, const KpCons& k, int, hipStream_t, KpDev*, KpCons*) {
    for (int i = 0; i < k.n_probes; i++) {
        const int g = k.probe0 + i;
        kp_probe_result o{};
        o.decision = g % 3;
        o.valid = o.decision != 0;
        o.n_pods = g;
        o.candidate_price = g;
        k.out[i] = o;
    }
    k.stats[CS_PROBES] += k.n_probes;
    return hipSuccess;
}
hipError_t kp_launch_cons_prep(const int32_t*, int, int32_t*, const int32_t*, int, uint64_t*, hipStream_t) {
    return hipSuccess;
}
hipError_t kp_launch_cons_chunk_max(const KpDev&, int64_t*, hipStream_t) { return hipSuccess; }
hipError_t kp_launch_multi_union(const KpCons&, int, uint64_t*, int32_t*, int2*, int32_t*, const int32_t*, hipStream_t) {
    return hipSuccess;
}
hipError_t kp_queue_sort(const int64_t* fields, int n, int32_t* perm_a, int32_t*, uint64_t*, uint64_t*, void*,
                         size_t* temp_bytes, hipStream_t, int32_t** result) {
    if (!fields) {
        *temp_bytes = 16;
        return hipSuccess;
    }
    for (int i = 0; i < n; i++) perm_a[i] = i;
    *result = perm_a;
    return hipSuccess;
}
