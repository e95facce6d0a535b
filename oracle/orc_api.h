/* ORACLE — test infrastructure only.  C-ABI of liboracle.so (CPU restatement of the reference path).
 * Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker.
 * Inputs use the product's view structs (include/kpsim.h) so both sides see byte-identical inputs;
 * everything behind them is an independent implementation. */
#ifndef ORC_API_H_
#define ORC_API_H_
#include <stdint.h>

#include "../include/kpsim.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_result orc_result;

kp_status orc_solve(const kp_catalog_view* cat, const kp_solve_input* in, kp_solve_output* out, orc_result** res);
/* orc_solve with the context's solver parameters (kp_device_opts.preference_policy); opts NULL = defaults */
kp_status orc_solve_opts(const kp_catalog_view* cat, const kp_solve_input* in, const kp_device_opts* opts,
                         kp_solve_output* out, orc_result** res);
kp_status orc_result_nodeclaim_requirements(const orc_result* res, int32_t nc, char* buf, int64_t cap, int64_t* needed);
void orc_result_free(orc_result* res);

/* Consolidation probes (SimulateScheduling + computeConsolidation), same probe numbering as kp_consolidate;
 * probes are spread over n_threads std::threads (the cpu_baseline leg of config 4). */
int32_t orc_consolidate_probe_count(const kp_consolidate_input* in);
kp_status orc_consolidate(const kp_catalog_view* cat, const kp_consolidate_input* in, kp_probe_result* results,
                          int32_t cap_results, int32_t n_threads);
/* ... with the context's solver parameters (kp_device_opts.preference_policy; the cluster's min_values_policy) */
kp_status orc_consolidate_opts(const kp_catalog_view* cat, const kp_consolidate_input* in, const kp_device_opts* opts,
                               kp_probe_result* results, int32_t cap_results, int32_t n_threads);
double orc_consolidate_last_probe_seconds(void);
/* kp_consolidate_command's restatement: the decision loops replayed over every probe, the replacement of a REPLACE. */
kp_status orc_consolidate_command(const kp_catalog_view* cat, const kp_consolidate_input* in, int32_t mode,
                                  kp_consolidation_command* out, int32_t n_threads);
kp_status orc_consolidate_command_opts(const kp_catalog_view* cat, const kp_consolidate_input* in,
                                       const kp_device_opts* opts, int32_t mode, kp_consolidation_command* out,
                                       int32_t n_threads);
kp_status orc_consolidate_replacement_opts(const kp_catalog_view* cat, const kp_consolidate_input* in,
                                           const kp_device_opts* opts, int32_t mode, int32_t probe,
                                           kp_consolidation_command* out);

/* Launch-time selection (filter.go chain + Truncate + getCapacityType + getOverrides' offering side), same
 * contract as kp_launch_select. */
kp_status orc_launch_select(const kp_catalog_view* cat, int32_t n, const kp_launch_request* requests, int32_t M,
                            kp_launch_result* results, int32_t* type_ids, int32_t cap_type_ids,
                            int32_t* override_offerings, int32_t cap_overrides);

/* pkg/providers/instancetype/types.go:123-155,320-605 — capacity / overhead / allocatable arithmetic.
 * Resource axes (milli-units), fixed order ORC_R_*. */
enum {
    ORC_R_CPU = 0, ORC_R_MEMORY, ORC_R_EPHEMERAL, ORC_R_PODS, ORC_R_POD_ENI, ORC_R_NVIDIA, ORC_R_AMD,
    ORC_R_NEURON, ORC_R_NEURONCORE, ORC_R_GAUDI, ORC_R_EFA, ORC_R_PRIVATE_IPV4, ORC_R_COUNT
};
enum { ORC_AMI_AL2023 = 0, ORC_AMI_AL2 = 1, ORC_AMI_BOTTLEROCKET = 2, ORC_AMI_WINDOWS = 3, ORC_AMI_CUSTOM = 4 };

typedef struct orc_ec2_info {
    int32_t vcpus;                     /* VCpuInfo.DefaultVCpus */
    int64_t memory_mib;                /* MemoryInfo.SizeInMiB */
    int32_t arm64;                     /* ProcessorInfo.SupportedArchitectures[0] == "arm64" */
    int32_t amd64;                     /* an x86_64 architecture is supported (getArchitecture) */
    int32_t default_card_max_enis;     /* NetworkCards[DefaultNetworkCardIndex].MaximumNetworkInterfaces */
    int32_t ipv4_per_eni;              /* NetworkInfo.Ipv4AddressesPerInterface */
    int64_t instance_storage_gb;       /* InstanceStorageInfo.TotalSizeInGB, < 0 if none */
    int32_t nvidia_gpus, amd_gpus, habana_gpus, neuron_devices, neuron_cores, efa;
    int32_t has_limits;                /* entry exists in zz_generated.vpclimits.go Limits */
    int32_t limits_trunking, limits_branch, limits_ipv4_per_eni;
} orc_ec2_info;

typedef struct orc_type_opts {
    double vm_memory_overhead_pct;     /* options.VMMemoryOverheadPercent (test default 0.075) */
    int32_t reserved_enis;             /* options.ReservedENIs */
    int32_t ami_family;                /* ORC_AMI_* */
    int32_t max_pods;                  /* kubelet maxPods, < 0: nil */
    int32_t pods_per_core;             /* kubelet podsPerCore, <= 0: nil */
    int32_t raid0;                     /* instanceStorePolicy == RAID0 */
} orc_type_opts;

void orc_instance_type_resources(const orc_ec2_info* info, const orc_type_opts* opts, int64_t* capacity,
                                 int64_t* kube_reserved, int64_t* eviction, int64_t* allocatable);

/* Go sort.Slice permutation of integer keys under less(i,j) = key[i] < key[j]; perm[] is permuted in place. */
void orc_go_sort_slice_ints(const int64_t* keys_by_id, int32_t* perm, int32_t n);

#ifdef __cplusplus
}
#endif
#endif
