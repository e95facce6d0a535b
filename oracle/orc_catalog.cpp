// ORACLE — test infrastructure only (see oracle/README.md). Never linked into libkpsim.
//
// CPU restatement of the instance-type resource arithmetic in
//   pkg/providers/instancetype/types.go
//     NewInstanceType :123-155 (overhead wiring, PrivateIPv4Address for Windows :151-153)
//     computeCapacity :320-338, cpu :340-342, memory :344-354 (arm64 −64 MiB, VM overhead ceil),
//     ephemeralStorage :357-392 (RAID0 → TotalSizeInGB "G"; default EBS 20Gi), awsPodENI :395-402,
//     nvidia/amd/neuron/neuroncore/habana/efa :404-466, ENILimitedPods :468-482,
//     privateIPv4Address :484-491, kubeReservedResources :499-529, evictionThreshold :531-558, pods :560-575
//   with AMI feature flags from pkg/providers/amifamily/resolver.go:102-119 (DefaultFamily),
//   bottlerocket.go:126-131, windows.go:101-107, and DefaultEBS (resolver.go:40-43).
// Floating-point steps are evaluated in IEEE double in Go's operand order (compile with -ffp-contract=off).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "gosort.h"
#include "orc_api.h"

static const int64_t Mi = 1024LL * 1024LL;
static const int64_t Gi = 1024LL * Mi;

struct Flags {
    bool eni_limited_memory_overhead, pods_per_core_enabled, eviction_soft_enabled, eni_limited_pod_density;
};

static Flags flags_for(int fam) {
    switch (fam) {
        case ORC_AMI_BOTTLEROCKET: return {false, false, false, true};
        case ORC_AMI_WINDOWS: return {false, true, true, false};
        default: return {true, true, true, true};  // DefaultFamily (AL2, AL2023, Custom, Ubuntu)
    }
}

// ENILimitedPods(ctx, info, reservedENIs)
static int64_t eni_limited_pods(const orc_ec2_info* info, int reserved) {
    int64_t usable = std::max<int64_t>((int64_t)info->default_card_max_enis - reserved, 0);
    if (usable == 0) return 0;
    return usable * ((int64_t)info->ipv4_per_eni - 1) + 2;
}

extern "C" void orc_instance_type_resources(const orc_ec2_info* info, const orc_type_opts* o, int64_t* cap,
                                            int64_t* kube, int64_t* evict, int64_t* alloc) {
    Flags f = flags_for(o->ami_family);
    for (int r = 0; r < ORC_R_COUNT; r++) cap[r] = kube[r] = evict[r] = alloc[r] = 0;
    // cpu
    int64_t cpu_milli = (int64_t)info->vcpus * 1000;
    cap[ORC_R_CPU] = cpu_milli;
    // memory(): arm64 −64Mi, then − ceil(value * pct / 1024 / 1024) Mi
    int64_t mib = info->memory_mib;
    if (info->arm64) mib -= 64;
    int64_t mem_bytes = mib * Mi;
    double ovh = (double)mem_bytes * o->vm_memory_overhead_pct / 1024 / 1024;
    mem_bytes -= (int64_t)std::ceil(ovh) * Mi;
    cap[ORC_R_MEMORY] = mem_bytes * 1000;
    // ephemeralStorage(): RAID0 with instance storage → "%dG"; otherwise the AMI family's ephemeral block device default:
    // 20Gi (DefaultEBS, amifamily/resolver.go:40-43), 50Gi for Windows' /dev/sda1 (amifamily/windows.go:88-99)
    int64_t eph_bytes = o->ami_family == ORC_AMI_WINDOWS ? 50 * Gi : 20 * Gi;
    if (o->raid0 && info->instance_storage_gb >= 0) eph_bytes = info->instance_storage_gb * 1000000000LL;
    cap[ORC_R_EPHEMERAL] = eph_bytes * 1000;
    // pods()
    int64_t pods;
    if (o->max_pods >= 0)
        pods = o->max_pods;
    else if (f.eni_limited_pod_density)
        pods = eni_limited_pods(info, o->reserved_enis);
    else
        pods = 110;
    if (o->pods_per_core > 0 && f.pods_per_core_enabled) pods = std::min<int64_t>((int64_t)o->pods_per_core * info->vcpus, pods);
    cap[ORC_R_PODS] = pods * 1000;
    cap[ORC_R_POD_ENI] = (info->has_limits && info->limits_trunking) ? (int64_t)info->limits_branch * 1000 : 0;
    cap[ORC_R_NVIDIA] = (int64_t)info->nvidia_gpus * 1000;
    cap[ORC_R_AMD] = (int64_t)info->amd_gpus * 1000;
    cap[ORC_R_NEURON] = (int64_t)info->neuron_devices * 1000;
    cap[ORC_R_NEURONCORE] = (int64_t)info->neuron_cores * 1000;
    cap[ORC_R_GAUDI] = (int64_t)info->habana_gpus * 1000;
    cap[ORC_R_EFA] = (int64_t)info->efa * 1000;
    // PrivateIPv4Address only on Windows-compatible types (os In [windows] requires an amd64 Windows AMI)
    if (o->ami_family == ORC_AMI_WINDOWS && info->amd64)
        cap[ORC_R_PRIVATE_IPV4] = info->has_limits ? (int64_t)(info->limits_ipv4_per_eni - 1) * 1000 : 0;

    // kubeReservedResources(cpu, pods', nil): memory (11*pods + 255)Mi, ephemeral 1Gi, cpu by ranges
    int64_t kpods = f.eni_limited_memory_overhead ? eni_limited_pods(info, 0) : pods;
    kube[ORC_R_MEMORY] = (11 * kpods + 255) * Mi * 1000;
    kube[ORC_R_EPHEMERAL] = 1 * Gi * 1000;
    struct Range {
        int64_t start, end;
        double pct;
    } ranges[] = {{0, 1000, 0.06}, {1000, 2000, 0.01}, {2000, 4000, 0.005}, {4000, 1LL << 31, 0.0025}};
    int64_t kcpu = 0;
    for (auto& rg : ranges) {
        if (cpu_milli >= rg.start) {
            double r = (double)(rg.end - rg.start);
            if (cpu_milli < rg.end) r = (double)(cpu_milli - rg.start);
            kcpu += (int64_t)(r * rg.pct);
        }
    }
    kube[ORC_R_CPU] = kcpu;
    // evictionThreshold(): memory 100Mi, ephemeral ceil(storage/100*10) (no kubelet overrides)
    evict[ORC_R_MEMORY] = 100 * Mi * 1000;
    evict[ORC_R_EPHEMERAL] = (int64_t)std::ceil((double)eph_bytes / 100 * 10) * 1000;
    for (int r = 0; r < ORC_R_COUNT; r++) alloc[r] = cap[r] - kube[r] - evict[r];
}

struct IntKeyAdaptor {
    const int64_t* keys;
    int32_t* perm;
    int n;
    int size() const { return n; }
    bool less(int i, int j) const { return keys[perm[i]] < keys[perm[j]]; }
    void swap(int i, int j) { std::swap(perm[i], perm[j]); }
};

extern "C" void orc_go_sort_slice_ints(const int64_t* keys_by_id, int32_t* perm, int32_t n) {
    IntKeyAdaptor a{keys_by_id, perm, n};
    orc::go_sort_slice(a);
}
