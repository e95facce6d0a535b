/*
 * kpsim.h — C-ABI of the MI355X-native Karpenter scheduling-simulation library (libkpsim.so).
 *
 * This is the drop-in boundary for the ONE hot path of jonathan-innis/karpenter-provider-aws that is
 * accelerated here: the provisioning scheduling simulation (core `scheduling.Scheduler.Solve`) and
 * its consolidation re-simulation, fed by the AWS provider's instance-type catalog.
 *
 * Reference interfaces each entry point replaces (paths relative to the reference root; `[core]` =
 * sigs.k8s.io/karpenter v1.6.1-0.20250908174930-91341612ebc6, go.mod:49, not vendored):
 *
 *   kp_ctx_create / kp_ctx_destroy
 *       — process-wide provider wiring: cmd/controller/main.go:30-85 (CloudProvider construction),
 *         solver options from pkg/operator/options/options.go:36-58 and core settings
 *         (MIN_VALUES_POLICY, website/content/en/preview/reference/settings.md:39).
 *   kp_catalog_upload
 *       — the `[]*cloudprovider.InstanceType` snapshot returned by
 *         CloudProvider.GetInstanceTypes (pkg/cloudprovider/cloudprovider.go:181-197) →
 *         instancetype.DefaultProvider.List (pkg/providers/instancetype/instancetype.go:123-165),
 *         including Offerings injected by offering.InjectOfferings
 *         (pkg/providers/instancetype/offering/offering.go:70-196).  `epoch` mirrors the List cache
 *         key (instancetype.go:219-229) plus ICE seqnums (pkg/cache/unavailableofferings.go:76-83).
 *   kp_catalog_patch_avail / kp_catalog_patch_price
 *       — ICE marks (pkg/cache/unavailableofferings.go:93-120) and price refreshes
 *         (pkg/providers/pricing/pricing.go:379-423) as table deltas.
 *   kp_solve
 *       — [core] provisioning.Scheduler.Solve (pkg/controllers/provisioning/scheduling/scheduler.go),
 *         reached today from the provisioner batch loop registered at cmd/controller/main.go:50-58,
 *         followed by [core] Results.TruncateInstanceTypes (InstanceTypes.Truncate, called at
 *         pkg/providers/instance/instance.go:293 with maxInstanceTypes = 60, instance.go:62).
 *   kp_result_nodeclaim_requirements
 *       — read-back of NodeClaim.Requirements for instanceToNodeClaim-style write-back
 *         (pkg/cloudprovider/cloudprovider.go:381-444).
 *
 * Conventions
 *   - Every function is extern "C", noexcept, and returns kp_status.
 *   - Inputs are borrowed for the duration of the call; outputs go into caller-allocated buffers
 *     (KP_E_BUFFER + required sizes when they are too small).  No pointer to library memory escapes.
 *   - Quantities are int64 MILLI-units of the Kubernetes resource.Quantity (Quantity.MilliValue()):
 *     cpu in millicores, memory/ephemeral-storage in milli-bytes, counts ×1000.
 *   - Strings are NUL-terminated UTF-8; they are interned at catalog upload / solve time.
 *   - A kp_ctx is single-threaded: concurrent callers use one ctx each (the reference calls List()
 *     from many goroutines, pkg/providers/instancetype/suite_test.go:2857-2891; each ctx owns its
 *     own device stream and buffers).  The catalog is immutable per epoch.
 */
#ifndef KPSIM_H_
#define KPSIM_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t kp_status;
enum {
    KP_OK = 0,
    KP_E_INVALID = 1,                /* malformed input view */
    KP_E_BUFFER = 2,                 /* output buffer too small; required sizes written back */
    KP_E_DEVICE = 3,                 /* HIP runtime error or no gfx950 device */
    KP_E_INSUFFICIENT_CAPACITY = 4,  /* cloudprovider.NewInsufficientCapacityError (cloudprovider.go:96, instance.go:283) */
    KP_E_NODECLASS_NOT_READY = 5,    /* cloudprovider.go:104 */
    KP_E_CREATE = 6,                 /* cloudprovider.go:118, instance.go:295 */
    KP_E_UNSUPPORTED = 7,            /* input uses a feature this build does not implement (never silently ignored) */
    KP_E_STATE = 8                   /* call order violated (e.g. solve before catalog upload) */
};

/* corev1.NodeSelectorOperator */
enum { KP_OP_IN = 0, KP_OP_NOT_IN = 1, KP_OP_EXISTS = 2, KP_OP_DOES_NOT_EXIST = 3, KP_OP_GT = 4, KP_OP_LT = 5 };

/* core MIN_VALUES_POLICY */
enum { KP_MIN_VALUES_STRICT = 0, KP_MIN_VALUES_BEST_EFFORT = 1 };

/* scheduling.Requirement as built by NewRequirementWithFlexibility / NewNodeSelectorRequirementsWithMinValues. */
typedef struct kp_requirement {
    const char* key;
    int32_t op;                      /* KP_OP_* */
    int32_t n_values;
    const char* const* values;       /* In/NotIn: the set; Gt/Lt: values[0] is the integer bound */
    int32_t min_values;              /* < 0 : nil */
} kp_requirement;

typedef struct kp_taint {
    const char* key;
    const char* value;
    const char* effect;              /* "NoSchedule" | "PreferNoSchedule" | "NoExecute" */
} kp_taint;

enum { KP_TOL_EQUAL = 0, KP_TOL_EXISTS = 1 };
typedef struct kp_toleration {
    const char* key;                 /* "" matches every key (only with Exists) */
    int32_t op;                      /* KP_TOL_* */
    const char* value;
    const char* effect;              /* "" matches every effect */
} kp_toleration;

/* Per (type, label key) and (offering, label key) state of InstanceType.Requirements. */
enum { KP_LABEL_ABSENT = 0, KP_LABEL_DOES_NOT_EXIST = 1, KP_LABEL_IN = 2 };

/*
 * The cloudprovider.InstanceType catalog as SoA (one row per instance type as returned by
 * GetInstanceTypes; rows from different EC2NodeClasses may share a name).
 */
typedef struct kp_catalog_view {
    int32_t n_types;                         /* T */
    int32_t n_resources;                     /* R */
    const char* const* resource_names;       /* [R] corev1.ResourceName */
    const char* const* type_names;           /* [T] */
    const int64_t* capacity;                 /* [T*R] InstanceType.Capacity (milli) */
    const int64_t* allocatable;              /* [T*R] InstanceType.Allocatable() = Capacity − Overhead.Total() */

    int32_t n_label_keys;                    /* K */
    const char* const* label_keys;           /* [K] */
    const int8_t* label_state;               /* [T*K] KP_LABEL_* */
    const int32_t* label_offsets;            /* [T*K+1] CSR offsets into label_values (used when KP_LABEL_IN) */
    const char* const* label_values;

    int32_t n_offerings;                     /* O, rows grouped by type (offering_type non-decreasing) */
    const int32_t* offering_type;            /* [O] */
    const double* offering_price;            /* [O] Offering.Price */
    const uint8_t* offering_available;       /* [O] Offering.Available */
    const int32_t* offering_reservation_capacity; /* [O] Offering.ReservationCapacity (0 for od/spot) */
    int32_t n_offering_keys;                 /* KO: keys of Offering.Requirements */
    const char* const* offering_keys;        /* [KO] */
    const int8_t* offering_label_state;      /* [O*KO] KP_LABEL_* (single value when IN) */
    const char* const* offering_label_values;/* [O*KO] value when KP_LABEL_IN, else ignored */
} kp_catalog_view;

/* A NodePool as the scheduler sees it: NodeClaimTemplate (core scheduling/nodeclaimtemplate.go). */
typedef struct kp_nodepool {
    const char* name;
    int32_t weight;                          /* .spec.weight (templates ordered weight desc, name asc) */
    int32_t n_requirements;                  /* template Requirements: spec requirements + template labels */
    const kp_requirement* requirements;      /*   + karpenter.sh/nodepool In [name] */
    int32_t n_taints;
    const kp_taint* taints;
    const int64_t* daemon_overhead;          /* [R] or NULL: daemonset overhead added to every new NodeClaim */
    const uint8_t* limit_set;                /* [R] or NULL: resources that carry a NodePool limit */
    const int64_t* limit_remaining;          /* [R] remaining = limits − capacity of this pool's existing nodes */
    int32_t n_types;                         /* GetInstanceTypes(nodepool) rows; < 0 means all catalog rows */
    const int32_t* type_index;
} kp_nodepool;

/*
 * Topology terms of a pod class: corev1.TopologySpreadConstraint and PodAffinityTerm as [core]
 * scheduling/topology.go (newForTopologies / newForAffinities / updateInverseAntiAffinity) turns them into
 * TopologyGroups (topologygroup.go).  Semantics restated in oracle/orc_solve.cpp (Topology) and DESIGN.md §4.
 */
enum { KP_TOPO_SPREAD = 0, KP_TOPO_AFFINITY = 1, KP_TOPO_ANTI_AFFINITY = 2 };
enum { KP_POLICY_IGNORE = 0, KP_POLICY_HONOR = 1 };        /* corev1.NodeInclusionPolicy */
enum { KP_DO_NOT_SCHEDULE = 0, KP_SCHEDULE_ANYWAY = 1 };   /* corev1.UnsatisfiableConstraintAction */
typedef struct kp_topology_term {
    int32_t type;                            /* KP_TOPO_* */
    const char* topology_key;                /* e.g. topology.kubernetes.io/zone, kubernetes.io/hostname */
    int32_t max_skew;                        /* spread */
    int32_t min_domains;                     /* spread; <= 0: nil */
    int32_t when_unsatisfiable;              /* spread: KP_DO_NOT_SCHEDULE, or KP_SCHEDULE_ANYWAY (a preference) */
    int32_t node_affinity_policy;            /* spread: KP_POLICY_* (Kubernetes default Honor) */
    int32_t node_taints_policy;              /* spread: KP_POLICY_* (Kubernetes default Ignore) */
    int32_t weight;                          /* (anti-)affinity: 0 = requiredDuringScheduling, > 0 = preferred weight */
    int32_t n_selector;                      /* LabelSelector over pod labels as requirements (matchLabels k=v → In [v];
                                                matchExpressions In/NotIn/Exists/DoesNotExist); < 0: nil (selects nothing) */
    const kp_requirement* selector;
    int32_t n_namespaces;                    /* (anti-)affinity term namespaces; 0: the pod's own namespace */
    const char* const* namespaces;
} kp_topology_term;

/* corev1.NodeSelectorTerm (required node affinity) or PreferredSchedulingTerm (preferred node affinity). */
typedef struct kp_node_selector_term {
    int32_t weight;                          /* PreferredSchedulingTerm.Weight (required terms: ignored) */
    int32_t n_requirements;                  /* MatchExpressions */
    const kp_requirement* requirements;
} kp_node_selector_term;

/*
 * A pod class: pods that share scheduling constraints (podData.Requirements, tolerations, labels, topology).
 * Preferences ([core] scheduling/preferences.go Relax, applied per pod when it fails to schedule, PREFERENCE_POLICY
 * Respect): the heaviest preferred node-affinity term and every preferred pod (anti-)affinity / ScheduleAnyway spread
 * constrain the pod until relaxed one at a time, in the order: the first of several required node-affinity terms,
 * the heaviest preferred pod-affinity term, the heaviest preferred anti-affinity term, the heaviest preferred
 * node-affinity term, the first ScheduleAnyway spread, then (when a NodePool carries a PreferNoSchedule taint) a
 * toleration of PreferNoSchedule taints.  A relaxed pod is re-queued with Queue.Push(pod, relaxed = true).
 */
typedef struct kp_pod_class {
    int32_t n_requirements;                  /* nodeSelector ∪ requiredDuringScheduling term[0]; with n_required_terms
                                                > 0: the nodeSelector only */
    const kp_requirement* requirements;
    int32_t n_tolerations;
    const kp_toleration* tolerations;
    const char* namespace_name;              /* metadata.namespace (NULL: "default") */
    int32_t n_labels;                        /* metadata.labels (topology selectors match these) */
    const char* const* label_keys;
    const char* const* label_values;
    int32_t n_topology;
    const kp_topology_term* topology;
    int32_t n_required_terms;                /* nodeAffinity.requiredDuringScheduling NodeSelectorTerms (ORed; tried in
                                                order as relaxation removes the first); 0: folded into requirements */
    const kp_node_selector_term* required_terms;
    int32_t n_preferred_terms;               /* nodeAffinity.preferredDuringScheduling terms (<= 12) */
    const kp_node_selector_term* preferred_terms;
} kp_pod_class;

typedef struct kp_pods_view {
    int32_t n_pods;                          /* P */
    const int32_t* class_id;                 /* [P] */
    const int64_t* requests;                 /* [P*R] resources.RequestsForPods (incl. pods = 1000 milli) */
    const int64_t* creation_ns;              /* [P] CreationTimestamp (queue tie-break) */
    const char* const* uids;                 /* [P] UID (final queue tie-break) */
} kp_pods_view;

/* An existing (or in-flight real) node: ExistingNode in core scheduling/existingnode.go. */
typedef struct kp_existing_node {
    const char* name;
    int32_t n_labels;                        /* node labels (each becomes `key In [value]`) */
    const char* const* label_keys;
    const char* const* label_values;
    int32_t n_taints;
    const kp_taint* taints;
    const int64_t* available;                /* [R] StateNode.Available() */
    const int64_t* requests;                 /* [R] remaining daemonset requests (initial n.requests) */
} kp_existing_node;

typedef struct kp_solve_input {
    int32_t n_nodepools;
    const kp_nodepool* nodepools;
    int32_t n_classes;
    const kp_pod_class* classes;
    kp_pods_view pods;
    int32_t n_existing;
    const kp_existing_node* existing;        /* in scheduling order (initialized first, core sorts stably) */
    int32_t max_instance_types;              /* 60 (instance.go:62); <= 0 disables truncation */
    int32_t min_values_policy;               /* KP_MIN_VALUES_* */
    /* pods already bound to existing nodes: topology.go countDomains (spread / affinity counts) and
       updateInverseAffinities (their required anti-affinity terms); pods being scheduled must not be listed */
    int32_t n_bound;
    const int32_t* bound_node;               /* [n_bound] index into existing */
    const int32_t* bound_class;              /* [n_bound] index into classes (labels, namespace, terms) */
} kp_solve_input;

/* Per-solve counters: evaluation counts feed the algorithmic-bytes roofline. */
typedef struct kp_solve_stats {
    int64_t pods_popped;                     /* queue pops incl. retries */
    int64_t nodeclaim_evals;                 /* NodeClaim.Add attempts */
    int64_t nodeclaim_candidates_scanned;    /* Σ_steps N_t (rows in the sorted in-flight list per step) */
    int64_t template_evals;                  /* new-NodeClaim attempts */
    int64_t existing_evals;
    int64_t sorts_fast;                      /* sort.Slice emulations resolved on the fast path */
    int64_t sorts_full;                      /* ... needing the full pdqsort emulation */
    double  ns_host_prep;
    double  ns_device_solve;
    double  ns_device_finalize;
    double  ns_total;
} kp_solve_stats;

/* pod_result encoding */
#define KP_POD_UNSCHEDULABLE (-1)            /* pod has an entry in Results.PodErrors */
#define KP_POD_EXISTING(j) (-2 - (j))        /* scheduled onto existing node j */

typedef struct kp_solve_output {
    /* capacities, set by the caller */
    int32_t cap_nodeclaims;
    int32_t cap_type_ids;
    /* results */
    int32_t n_nodeclaims;                    /* Results.NewNodeClaims (creation order) */
    int32_t n_type_ids;                      /* entries written to type_ids */
    int32_t* nodeclaim_nodepool;             /* [cap_nodeclaims] index into input nodepools */
    int32_t* nodeclaim_n_pods;               /* [cap_nodeclaims] */
    int32_t* nodeclaim_slice_pos;            /* [cap_nodeclaims] position in s.newNodeClaims at the end of Solve */
    int32_t* nodeclaim_n_options;            /* [cap_nodeclaims] InstanceTypeOptions before truncation */
    int32_t* nodeclaim_type_offset;          /* [cap_nodeclaims+1] into type_ids */
    int32_t* type_ids;                       /* [cap_type_ids] truncated, price-ordered catalog rows */
    int32_t* pod_result;                     /* [P] >= 0 nodeclaim index, KP_POD_EXISTING(j), KP_POD_UNSCHEDULABLE */
    int32_t* pod_order;                      /* [P] queue position of the pod's final placement (-1 if none) */
    kp_solve_stats stats;
} kp_solve_output;

/* core PREFERENCE_POLICY (website/content/en/preview/reference/settings.md:40) */
enum { KP_PREFERENCE_RESPECT = 0, KP_PREFERENCE_IGNORE = 1 };

/* Context options: devices and the solver parameters core reads from its operator options
   (settings.md:13-42, pkg/operator/options/options.go:36-58). */
typedef struct kp_device_opts {
    int32_t device;                          /* HIP device ordinal (the ctx's primary device) */
    int32_t n_devices;                       /* > 1: a multi-device ctx over devices[0..n) (devices[0] is the primary;
                                                `device` is ignored).  Catalog uploads / patches and
                                                kp_consolidate_prepare are applied on every device (one host thread
                                                each); kp_consolidate_execute / kp_consolidate split the probe range into
                                                one contiguous shard per device and gather the results (SURVEY §8b(4):
                                                kp_consolidate runs multi-GPU internally).  Solve and launch selection
                                                run on the primary. */
    const int32_t* devices;
    int32_t preference_policy;               /* KP_PREFERENCE_*: Respect relaxes preferences (ScheduleAnyway spreads,
                                                preferred affinities); Ignore drops them before scheduling */
    int32_t reserved_capacity;               /* feature gate ReservedCapacity: reserved offerings join Solve */
} kp_device_opts;

typedef struct kp_ctx kp_ctx;

kp_status kp_ctx_create(const kp_device_opts* opts, kp_ctx** out);
kp_status kp_ctx_destroy(kp_ctx* ctx);
const char* kp_last_error(const kp_ctx* ctx);
const char* kp_version(void);

kp_status kp_catalog_upload(kp_ctx* ctx, const kp_catalog_view* catalog, uint64_t epoch);
/* ICE / availability delta: available[o] for every offering row, same order as the upload. */
kp_status kp_catalog_patch_avail(kp_ctx* ctx, const uint8_t* available, int32_t n_offerings, uint64_t epoch);
/* price delta: price of offering rows idx[i] becomes price[i]. */
kp_status kp_catalog_patch_price(kp_ctx* ctx, const int32_t* idx, const double* price, int32_t n, uint64_t epoch);

/* Solve = kp_solve_prepare + kp_solve_execute + kp_solve_fetch.  In-flight NodeClaims per solve: up to 65,535 (u16 ids).
 * The prepare plans for 4096, or from the start for more when the pods' self-selecting hostname anti-affinity / spread
 * terms need more (one NodeClaim per pod / per maxSkew pods): such node-dense solves run one execute, with the slice
 * arrays in HBM once they outgrow LDS (~11k NodeClaims).  A solve that still overflows its plan surfaces as
 * KP_E_UNSUPPORTED from kp_solve_fetch; the next prepare of that ctx (only that one) then plans for every pod, and
 * kp_solve does that one re-run itself.  Later solves on the ctx start from the first plan again. */
kp_status kp_solve(kp_ctx* ctx, const kp_solve_input* in, kp_solve_output* out);

/* kp_solve split into its phases (kp_solve == prepare + execute + fetch):
 *   prepare — intern strings into the catalog dictionaries, encode digests, upload inputs to HBM;
 *   execute — all scheduling work on the device (queue sort, class masks, template filter, FFD, Truncate),
 *             synchronous; inputs are HBM-resident when it starts;
 *   fetch   — download and decode results into the caller's buffers. */
kp_status kp_solve_prepare(kp_ctx* ctx, const kp_solve_input* in);
kp_status kp_solve_execute(kp_ctx* ctx);
kp_status kp_solve_fetch(kp_ctx* ctx, kp_solve_output* out);

/* Device time (ms, HIP events on the ctx stream) of the last kp_solve_execute, per phase:
 * [0] queue sort, [1] class masks, [2] template filter, [3] FFD solve kernel, [4] finalize/Truncate;
 * then (after kp_solve_fetch, KPSIM_PROFILE=1 in the environment at prepare) FFD-kernel shader-clock counters
 * [5..10]: wave-0 fast loop, its sort.Slice share, slow-path NodeClaim.Add rounds, new-NodeClaim templates, -,
 * full-pdqsort share; [11..16] per-stage evaluation cycles; then event counts [17] quick accepts, [18] slow-path
 * pods, [19] witness misses (slow-path evaluations of a NodeClaim whose class repeats), [20..23] fast-loop
 * cycles: pop, scan, quick check, quick commit; [24..34] fast-loop event counts; [35] topology quick accepts, [36..37]
 * topology prefilter setup / scan cycles; [38..41] failed NodeClaim.Add evaluations by stage: requirement merge,
 * topology narrowing, no instance type left, minValues (n up to 42). */
kp_status kp_last_kernel_times(kp_ctx* ctx, double* ms, int32_t n);

/*
 * Consolidation re-simulation — replaces the scheduling simulation of [core] pkg/controllers/disruption:
 * SimulateScheduling (helpers.go) + consolidation.computeConsolidation (consolidation.go), driven by
 * SingleNodeConsolidation (singlenodeconsolidation.go: first valid candidate in disruption-cost order) and
 * MultiNodeConsolidation.firstNConsolidationOption (multinodeconsolidation.go: binary search over the prefix
 * length).  Reached today from the disruption controller registered at cmd/controller/main.go:50-58; the decision
 * semantics are restated from the un-vendored core module and are marked "recalled" in DESIGN.md.
 *
 * A probe is one SimulateScheduling call: the pods of its candidates (plus pending pods) are rescheduled onto every
 * other existing node, the in-flight NodeClaims it creates and the NodePools.
 *   single mode: probe i = { candidates[i] }                       (i = 0 .. n_candidates-1)
 *   multi mode:  probe i = { candidates[0 .. i+2) }                (firstNConsolidationOption's mid = i+1: prefix
 *                sizes 2 .. n when n <= max_candidates, else 2 .. max_candidates+1)
 * Probes are independent, so [probe_begin, probe_end) may be any shard of them (one shard per GPU); the caller replays
 * the single-node scan (first valid probe) or the multi-node binary search over the results, which is exact because
 * every probe the sequential search would visit has been evaluated.
 * cluster.existing must be in NewScheduler's order (initialized nodes first, then by name); probes keep that order
 * with the candidates removed.  Candidate prices must be >= 0 (getCandidatePrices fails otherwise).
 *
 * Caller-side, outside this entry point (website/content/en/preview/concepts/disruption.md):
 *   - Empty Node Consolidation (:94-97) deletes nodes with no reschedulable pods without any simulation, so empty
 *     nodes need no probe;
 *   - NodePool disruption budgets (:274-285) cap how many candidates may be disrupted.  The caller drops candidates
 *     whose NodePool has no allowed disruptions left before building `candidates`, as the disruption controller does
 *     when it lists them;
 *   - consolidationPolicy / consolidateAfter decide which nodes are candidates at all.
 */
enum { KP_CONSOLIDATE_SINGLE = 0, KP_CONSOLIDATE_MULTI = 1,
       KP_CONSOLIDATE_BOTH = 2 };  /* both probe lists in one pass: the multi-node probes, then the single-node probes
                                      (one device launch; the longest multi-node prefixes are started first, the
                                      single-node probes fill the remaining compute units) */
enum { KP_DECISION_NONE = 0, KP_DECISION_DELETE = 1, KP_DECISION_REPLACE = 2 };
enum { KP_CT_ON_DEMAND = 0, KP_CT_SPOT = 1, KP_CT_RESERVED = 2 };

typedef struct kp_candidate {
    int32_t node;                    /* index into cluster.existing */
    int32_t n_pods;                  /* Candidate.ReschedulablePods, indices into cluster.pods */
    const int32_t* pods;
    double price;                    /* getCandidatePrices term: cheapest offering compatible with the node's labels */
    int32_t capacity_type;           /* KP_CT_* of the node */
    int32_t instance_type;           /* catalog row of the node's instance type (filterOutSameInstanceType), -1 */
    int32_t nodepool;                /* index into cluster.nodepools, -1 */
    const int64_t* capacity;         /* [R] node capacity, added back to its NodePool's remaining limits, or NULL */
} kp_candidate;

typedef struct kp_consolidate_input {
    kp_solve_input cluster;          /* nodepools, classes, pods (pending + reschedulable), existing = all state nodes */
    const uint8_t* initialized;      /* [n_existing] StateNode.Initialized(); NULL: all initialized */
    int32_t n_pending;               /* provisioner.GetPendingPods, indices into cluster.pods */
    const int32_t* pending;
    int32_t n_candidates;            /* in disruption-cost order */
    const kp_candidate* candidates;
    int32_t mode;                    /* KP_CONSOLIDATE_* */
    int32_t max_candidates;          /* multi: 100 */
    int32_t probe_begin, probe_end;  /* shard of the probe list; probe_end <= 0: to the end */
    int32_t spot_to_spot;            /* feature gate SpotToSpotConsolidation */
} kp_consolidate_input;

typedef struct kp_probe_result {
    int32_t decision;                /* KP_DECISION_* of computeConsolidation */
    int32_t valid;                   /* single: decision != NONE; multi: DELETE, or REPLACE with options left by
                                        filterOutSameInstanceType (the binary search's test) */
    int32_t all_scheduled;           /* Results.AllNonPendingPodsScheduled; uninitialized-node placements are errors */
    int32_t n_new_nodeclaims;        /* valid new NodeClaims, capped at 2 (the device stops a probe at its second
                                        NodeClaim, after which the decision is NONE and all_scheduled is undefined) */
    int32_t n_replacement_types;     /* replacement options of the command (REPLACE; spot-to-spot single: at most 15;
                                        multi: after filterOutSameInstanceType) */
    int32_t n_pods;                  /* pods the probe rescheduled */
    double candidate_price;          /* Σ candidate prices */
    double replacement_price;        /* cheapest WorstLaunchPrice among the replacement options (REPLACE), else 0 */
} kp_probe_result;

/* Number of probes of an input (mode, n_candidates, max_candidates). */
int32_t kp_consolidate_probe_count(const kp_consolidate_input* in);
/* Evaluates probes [probe_begin, probe_end) on the ctx's device; results[i] is probe probe_begin + i. */
kp_status kp_consolidate(kp_ctx* ctx, const kp_consolidate_input* in, kp_probe_result* results, int32_t cap_results);
/* Split form (inputs resident on the device between calls): prepare encodes and uploads the cluster and candidates
 * of `in` (its mode and probe range are ignored); execute evaluates probes [probe_begin, probe_end) of `mode` over the
 * prepared pass (probe_end <= 0: to the end).  kp_consolidate = prepare + execute of in->mode / in's range.
 * Any kp_solve_prepare or catalog upload on the ctx invalidates the prepared pass (KP_E_STATE). */
kp_status kp_consolidate_prepare(kp_ctx* ctx, const kp_consolidate_input* in);
kp_status kp_consolidate_execute(kp_ctx* ctx, int32_t mode, int32_t probe_begin, int32_t probe_end,
                                 kp_probe_result* results, int32_t cap_results);
/*
 * The consolidation command of a prepared pass — replaces the decision loops of [core] disruption
 * (SingleNodeConsolidation.ComputeCommand, singlenodeconsolidation.go: the first candidate in disruption-cost order whose
 * computeConsolidation is not a no-op; MultiNodeConsolidation.firstNConsolidationOption, multinodeconsolidation.go: the
 * binary search over the prefix length, a prefix kept when DELETE or a REPLACE with options left after
 * filterOutSameInstanceType) and their Command (consolidation.go computeConsolidation: delete set + replacement
 * NodeClaim).  One call evaluates every probe the loop could visit (one device pass, sharded over a multi-device ctx)
 * unless the last kp_consolidate_execute of the prepared pass already evaluated them all (a full pass of `mode`, or of
 * KP_CONSOLIDATE_BOTH): then it replays that pass.  It replays the loop over the rows on the host, then re-runs the
 * chosen probe on the primary device to read back its replacement NodeClaim (kept with the prepared pass: a repeated
 * call, e.g. after KP_E_BUFFER, copies it) — the NodeClaim CloudProvider.Create (pkg/cloudprovider/cloudprovider.go:90-137)
 * is later called with:
 *   type_ids      its InstanceTypeOptions after RemoveInstanceTypeOptionsByPriceAndMinValues (or the spot-to-spot cut
 *                 to max(15, minNeeded) cheapest) and, for multi-node, filterOutSameInstanceType; OrderByPrice order;
 *   requirements  its Requirements (FinalizeScheduling's reservation-id In [held IDs] included; capacity-type narrowed to
 *                 spot when the replacement was priced as spot), kp_result_nodeclaim_requirements' text format.
 * mode: KP_CONSOLIDATE_SINGLE, _MULTI, or _BOTH = the disruption controller's method order (multi-node, then single-node
 * when the multi-node search finds no command), evaluated in one pass.
 */
typedef struct kp_consolidation_command {
    /* caller-set buffers */
    int32_t cap_type_ids;
    int32_t* type_ids;               /* [cap_type_ids] catalog rows */
    int64_t cap_requirements;
    char* requirements;              /* [cap_requirements] bytes incl. NUL */
    /* results */
    int32_t decision;                /* KP_DECISION_*; NONE: no command */
    int32_t mode;                    /* KP_CONSOLIDATE_SINGLE / _MULTI: the method that produced the command */
    int32_t probe;                   /* index of the chosen probe in that method's probe list, -1 */
    int32_t first_candidate;         /* delete set: candidates[first_candidate, first_candidate + n_candidates) */
    int32_t n_candidates;
    int32_t nodepool;                /* REPLACE: the replacement's NodePool (index into cluster.nodepools), else -1 */
    int32_t n_type_ids;              /* REPLACE: number of options (written up to cap_type_ids) */
    int32_t n_reserved;              /* REPLACE: reservation IDs the replacement holds */
    int64_t requirements_needed;     /* REPLACE: bytes incl. NUL of the requirements text */
    kp_probe_result result;          /* the chosen probe's row */
} kp_consolidation_command;

/* KP_E_BUFFER (with n_type_ids / requirements_needed set) when a replacement does not fit the caller's buffers. */
kp_status kp_consolidate_command(kp_ctx* ctx, int32_t mode, kp_consolidation_command* out);
/* The command of one given probe of a prepared pass (mode KP_CONSOLIDATE_SINGLE or _MULTI, probe index in that mode's
 * list): its row and, for a REPLACE, the replacement NodeClaim as kp_consolidate_command returns it.  For callers that
 * replay the decision loops themselves over probe rows gathered from several processes (one GPU per process,
 * kpsim.consolidation.compute_command with a torch.distributed group). */
kp_status kp_consolidate_replacement(kp_ctx* ctx, int32_t mode, int32_t probe, kp_consolidation_command* out);

/* Diagnostics of the last kp_consolidate: ms[3] = {device prep (queue sort, masks), probe kernel, whole call};
 * counters[18] = {pods popped, existing-node slots examined, NodeClaim evaluations, template evaluations, probes,
 * queue-bitmap words scanned, existing-node placements, new NodeClaims, node chunks loaded, cached-chunk hits, then
 * with KPSIM_PROFILE set: s_memtime cycles of queue build, existing-node scans, NodeClaim/template evaluation,
 * decision, whole probe (summed over probes); then chunks the headroom summary skipped, preference relaxations,
 * probes run with per-probe node requirement copies (pods whose NotIn / DoesNotExist requirements change nodes)};
 * counters[18..19] = {probe passes launched, replacement read-backs run} since the last kp_consolidate_prepare. */
kp_status kp_consolidate_stats(kp_ctx* ctx, double* ms, int64_t* counters, int32_t n_counters);

/*
 * Launch-time instance-type selection — replaces the pure-function part of CloudProvider.Create
 * (pkg/cloudprovider/cloudprovider.go:90-137) → instance.DefaultProvider.Create (pkg/providers/instance/instance.go:132-137):
 *   filterInstanceTypes (instance.go:270-298): the filter chain of pkg/providers/instance/filter/filter.go
 *     CompatibleAvailableFilter :39-64, CapacityReservationTypeFilter :73-157, CapacityBlockFilter :163-221,
 *     ReservedOfferingFilter :230-270, ExoticInstanceTypeFilter :279-318, SpotInstanceFilter :328-386
 *     (a filter leaving no type → KP_E_INSUFFICIENT_CAPACITY, instance.go:281-284), then
 *     [core] InstanceTypes.Truncate(reqs, max_instance_types) (instance.go:293; minValues failure → KP_E_CREATE :295);
 *   getCapacityType (instance.go:532-546): reserved > spot > on-demand;
 *   the offering side of getOverrides (instance.go:420-467): per kept type, its Available offerings Compatible with the
 *     requirements narrowed to the chosen capacity type (the caller maps each offering's zone to a subnet).
 * One request = one NodeClaim (Spec.Requirements with minValues, Spec.Resources.Requests) against the whole uploaded
 * catalog (instanceTypeProvider.List, cloudprovider.go:116).  Requests are independent: a batch is evaluated in parallel.
 * Order conventions where the reference iterates Go maps (filter.go:115,156,263: lo.Values): catalog row order for
 * types and view row order for offerings.  The truncated list is ordered by (cheapest compatible available price, name).
 */
enum {
    KP_FILTER_COMPATIBLE_AVAILABLE = 0, KP_FILTER_CAPACITY_RESERVATION_TYPE = 1, KP_FILTER_CAPACITY_BLOCK = 2,
    KP_FILTER_RESERVED_OFFERING = 3, KP_FILTER_EXOTIC = 4, KP_FILTER_SPOT = 5, KP_N_FILTERS = 6
};

typedef struct kp_launch_request {
    int32_t n_requirements;                  /* NodeClaim.Spec.Requirements (NewNodeSelectorRequirementsWithMinValues) */
    const kp_requirement* requirements;
    const int64_t* requests;                 /* [R] Spec.Resources.Requests (milli); 0 = resource not requested */
} kp_launch_request;

typedef struct kp_launch_result {
    int32_t status;                          /* KP_OK | KP_E_INSUFFICIENT_CAPACITY | KP_E_CREATE */
    int32_t failed_filter;                   /* KP_FILTER_* that left no type (ICE), else -1 */
    int32_t capacity_type;                   /* KP_CT_* (getCapacityType) */
    int32_t n_types;                         /* truncated, price-ordered types */
    int32_t type_offset;                     /* into type_ids */
    int32_t n_overrides;                     /* offering rows (catalog view order) of the kept types */
    int32_t override_offset;                 /* into override_offerings */
    int32_t n_options;                       /* types left by the filter chain, before Truncate */
    int32_t rejected[KP_N_FILTERS];          /* types each filter rejected */
    int32_t fleet_pick;                      /* the override offering row a lowest-price CreateFleet launches (SURVEY §8f
                                                row 4, the kwok fake EC2: kwok/ec2/ec2.go:432-461 lo.MinBy over the
                                                overrides in order, scored by kwok/strategy/strategy.go:45-60 — the spot
                                                price of (type, zone) for a spot launch, else the type's on-demand price;
                                                a missing price scores MaxFloat64, a zero score never wins); -1 on error */
} kp_launch_result;

/* Evaluates n requests on the ctx's device.  type_ids / override_offerings receive the concatenated lists
 * (KP_E_BUFFER with results[*] offsets still valid up to the capacity when a buffer is too small). */
kp_status kp_launch_select(kp_ctx* ctx, int32_t n, const kp_launch_request* requests, int32_t max_instance_types,
                           kp_launch_result* results, int32_t* type_ids, int32_t cap_type_ids,
                           int32_t* override_offerings, int32_t cap_overrides);
/* Of the last kp_launch_select: ms[0] = launch kernel time (HIP events on the ctx stream, summed over the call's
 * sub-batches), ms[1] = whole call; host phases ms[2] = request encoding, ms[3] = table merge + upload, ms[4] = waits
 * for kernel + result download, ms[5] = result expansion; ms[6] = number of sub-batches, ms[7] = device busy time (union
 * of the sub-batch kernels, which overlap on two streams).  A batch of >= 4096 requests is cut into 2 sub-batches on two
 * streams (even sub-batches on the ctx stream, odd ones on a second stream) so that encoding and expansion on the host
 * overlap the kernels; the KPSIM_LAUNCH_SUB environment variable overrides the count (diagnostics, capped at
 * KL_MAX_SUB). */
kp_status kp_launch_stats(kp_ctx* ctx, double* ms, int32_t n);

/*
 * NodeClaim write-back for a launched instance — replaces CloudProvider.instanceToNodeClaim's label and status-resource
 * rules (pkg/cloudprovider/cloudprovider.go:381-444) for an instance of catalog row type_index launched through offering
 * row `offering` (CreateFleet's pick among kp_launch_select's overrides: the instance's zone, capacity type and
 * capacity reservation):
 *   labels: every single-valued requirement of the instance type (Requirement.Len() == 1) except the
 *           capacity-reservation id / type keys; topology.kubernetes.io/zone; topology.k8s.aws/zone-id (zone_id, the
 *           EC2NodeClass subnet's ZoneID, or when NULL the offering's own zone-id); karpenter.sh/capacity-type; for a
 *           reserved instance its reservation id and type; karpenter.sh/nodepool (nodepool, the instance tag, if given).
 *           Written as "key 	 value 
" lines sorted by key (*needed = bytes incl. NUL).
 *   capacity / allocatable [R] (optional): InstanceType.Capacity / Allocatable() with zero quantities dropped (0) and
 *           vpc.amazonaws.com/efa kept only when efa_enabled (the launch asked for EFA interfaces).
 */
kp_status kp_nodeclaim_labels(kp_ctx* ctx, int32_t type_index, int32_t offering, const char* zone_id,
                              const char* nodepool, int32_t efa_enabled, char* buf, int64_t cap, int64_t* needed,
                              int64_t* capacity, int64_t* allocatable);

/*
 * Catalog ingestion — replaces instancetype.DefaultProvider.List's construction of the
 * `[]*cloudprovider.InstanceType` (pkg/providers/instancetype/instancetype.go:123-165) from raw EC2 data:
 *   NewInstanceType (pkg/providers/instancetype/types.go:123-155) = computeRequirements (:158-299),
 *     computeCapacity (:320-338: cpu, memory − VM overhead, ephemeral storage from the block device mappings / AMI
 *     family defaults, pods, pod-eni, GPUs, neuron, gaudi, efa), PrivateIPv4Address for Windows-compatible types
 *     (:151-153), Overhead = kubeReservedResources (:493-530) + systemReservedResources (:487-491) +
 *     evictionThreshold (:532-560, computeEvictionSignal :598-615); Allocatable = Capacity − Overhead.Total();
 *     AMI family feature flags (pkg/providers/amifamily/resolver.go:102-119, bottlerocket.go:126-131,
 *     windows.go:101-107) and default block devices (al2023.go:99-108, bottlerocket.go:95-112, windows.go:88-99,
 *     custom.go:48-58, resolver.go:40-43);
 *   offering.DefaultProvider.InjectOfferings / createOfferings (pkg/providers/instancetype/offering/offering.go:70-196):
 *     one offering per (zone of all_zones, capacity type on-demand|spot of the type), Available = !ICE && hasPrice &&
 *     zone ∈ the type's zones (:148), zone-id when the NodeClass maps the zone (:151-153); with the ReservedCapacity
 *     gate, one reserved offering per capacity reservation of the type, price = on-demand / 1e7 (:176), Available =
 *     count ≠ 0 && zone ok && not expiring (:187).
 * The resulting kp_catalog is a host object; kp_catalog_get_view exposes it as a kp_catalog_view (resource axes in the
 * order of kp_catalog_resource_name) that stays valid until kp_catalog_free, ready for kp_catalog_upload.  Go iterates
 * the allZones set in map order (offering.go:135); here offerings follow all_zones order, types follow input order.
 */
enum { KP_AMI_AL2 = 0, KP_AMI_AL2023 = 1, KP_AMI_BOTTLEROCKET = 2, KP_AMI_WINDOWS2019 = 3, KP_AMI_WINDOWS2022 = 4,
       KP_AMI_CUSTOM = 5 };
#define KP_CATALOG_R 12                      /* resource axes of a built catalog */

typedef struct kp_ec2_device {               /* GpuDeviceInfo / InferenceDeviceInfo / NeuronDeviceInfo */
    const char* name;
    const char* manufacturer;
    int32_t count;
    int32_t memory_mib;                      /* GPUs: MemoryInfo.SizeInMiB */
    int32_t cores;                           /* neuron: CoreInfo.Count */
} kp_ec2_device;

/* ec2types.InstanceTypeInfo fields the provider reads, plus the per-name tables it joins
   (zz_generated.vpclimits.go Limits, zz_generated.bandwidth.go InstanceTypeBandwidthMegabits). */
typedef struct kp_ec2_instance_type {
    const char* name;                        /* InstanceType */
    int32_t default_vcpus;                   /* VCpuInfo.DefaultVCpus */
    int64_t memory_mib;                      /* MemoryInfo.SizeInMiB */
    int32_t n_architectures;                 /* ProcessorInfo.SupportedArchitectures ("x86_64", "arm64", ...) */
    const char* const* architectures;
    int32_t has_processor_info;              /* ProcessorInfo != nil */
    const char* cpu_manufacturer;            /* ProcessorInfo.Manufacturer (NULL: nil) */
    double sustained_clock_ghz;              /* ProcessorInfo.SustainedClockSpeedInGhz (NaN: nil) */
    int32_t n_usage_classes;                 /* SupportedUsageClasses */
    const char* const* usage_classes;
    const char* hypervisor;                  /* Hypervisor (NULL: "") */
    int32_t encryption_in_transit;           /* NetworkInfo.EncryptionInTransitSupported */
    int32_t n_network_cards;                 /* NetworkInfo.NetworkCards[].MaximumNetworkInterfaces */
    const int32_t* card_max_interfaces;
    int32_t default_card;                    /* NetworkInfo.DefaultNetworkCardIndex */
    int32_t max_network_interfaces;          /* used only when n_network_cards == 0 */
    int32_t ipv4_per_interface;              /* NetworkInfo.Ipv4AddressesPerInterface */
    int32_t efa_max;                         /* NetworkInfo.EfaInfo.MaximumEfaInterfaces (0: nil) */
    int64_t instance_storage_gb;             /* InstanceStorageInfo.TotalSizeInGB (< 0: nil) */
    const char* nvme_support;                /* InstanceStorageInfo.NvmeSupport (NULL: nil) */
    int32_t n_gpus;                          /* GpuInfo.Gpus */
    const kp_ec2_device* gpus;
    int32_t n_accelerators;                  /* InferenceAcceleratorInfo.Accelerators (< 0: nil) */
    const kp_ec2_device* accelerators;
    int32_t n_neuron;                        /* NeuronInfo.NeuronDevices (< 0: NeuronInfo nil) */
    const kp_ec2_device* neuron;
    int64_t ebs_max_bandwidth_mbps;          /* EbsInfo.EbsOptimizedInfo.MaximumBandwidthInMbps (< 0: nil) */
    const char* ebs_optimized_support;       /* EbsInfo.EbsOptimizedSupport */
    int32_t has_vpc_limits;                  /* Limits[name] present */
    int32_t vpc_trunking;                    /*   .IsTrunkingCompatible */
    int32_t vpc_branch_interface;            /*   .BranchInterface */
    int32_t vpc_ipv4_per_interface;          /*   .IPv4PerInterface */
    int64_t network_bandwidth_mbps;          /* InstanceTypeBandwidthMegabits[name] (< 0: absent) */
} kp_ec2_instance_type;

typedef struct kp_string_pair { const char* key; const char* value; } kp_string_pair;   /* map[string]string entry */
typedef struct kp_zone_info { const char* zone; const char* zone_id; } kp_zone_info;    /* v1.ZoneInfo */
typedef struct kp_block_device_mapping {     /* v1.BlockDeviceMapping */
    const char* device_name;
    int32_t root_volume;
    const char* volume_size;                 /* EBS.VolumeSize quantity ("100Gi"), NULL: nil */
} kp_block_device_mapping;
typedef struct kp_capacity_reservation {     /* v1.CapacityReservation (EC2NodeClass status) */
    const char* id;
    const char* instance_type;
    const char* availability_zone;
    const char* reservation_type;            /* "default" | "capacity-block" */
    int32_t expiring;                        /* State == expiring */
    int32_t available_count;                 /* capacityReservationProvider.GetAvailableInstanceCount(id) */
} kp_capacity_reservation;

/* The EC2NodeClass (resolved kubelet configuration included) and the provider options the catalog depends on. */
typedef struct kp_nodeclass_view {
    int32_t ami_family;                      /* KP_AMI_* (amifamily.GetAMIFamily) */
    const char* region;
    int32_t n_zones;                         /* nodeClass.ZoneInfo(): subnet zones and their zone ids */
    const kp_zone_info* zones;
    int32_t n_block_device_mappings;
    const kp_block_device_mapping* block_device_mappings;
    int32_t instance_store_raid0;            /* InstanceStorePolicy == RAID0 */
    int32_t max_pods;                        /* kubelet maxPods (< 0: nil) */
    int32_t pods_per_core;                   /* kubelet podsPerCore (<= 0: nil) */
    int32_t n_kube_reserved;                 /* kubelet kubeReserved / systemReserved (resource → quantity) */
    const kp_string_pair* kube_reserved;
    int32_t n_system_reserved;
    const kp_string_pair* system_reserved;
    int32_t n_eviction_hard;                 /* kubelet evictionHard / evictionSoft (signal → quantity or "N%") */
    const kp_string_pair* eviction_hard;
    int32_t n_eviction_soft;
    const kp_string_pair* eviction_soft;
    int32_t n_capacity_reservations;         /* nodeClass.CapacityReservations() */
    const kp_capacity_reservation* capacity_reservations;
    double vm_memory_overhead_percent;       /* options.VMMemoryOverheadPercent (0.075) */
    int32_t reserved_enis;                   /* options.ReservedENIs */
    int32_t reserved_capacity;               /* feature gate ReservedCapacity */
} kp_nodeclass_view;

/* Prices and the ICE cache as createOfferings reads them (pricing.OnDemandPrice / SpotPrice, IsUnavailable). */
typedef struct kp_offering_source {
    int32_t n_zones;                         /* allZones: every zone with an instance-type offering */
    const char* const* zones;
    const char* const* type_zones;           /* [n_types] per type: its offering zones, '\n'-separated
                                                (DescribeInstanceTypeOfferings) */
    const double* od_price;                  /* [n_types] on-demand price, NaN: no price */
    const double* spot_price;                /* [n_types * n_zones] spot price per zone, NaN: no price */
    const uint8_t* unavailable;              /* [n_types * n_zones * 2] ICE (zone-major, then od/spot), NULL: none */
} kp_offering_source;

typedef struct kp_catalog kp_catalog;
kp_status kp_catalog_build(int32_t n_types, const kp_ec2_instance_type* types, const kp_nodeclass_view* nodeclass,
                           const kp_offering_source* offerings, kp_catalog** out);
/* A view of the built catalog (borrowed from `cat`, valid until kp_catalog_free). */
kp_status kp_catalog_get_view(const kp_catalog* cat, kp_catalog_view* view);
/* Overhead.Total() of type t ([KP_CATALOG_R]) and the resource-axis names. */
kp_status kp_catalog_overhead(const kp_catalog* cat, int32_t t, int64_t* overhead);
const char* kp_catalog_resource_name(int32_t r);
kp_status kp_catalog_free(kp_catalog* cat);

/*
 * Requirements of NodeClaim `nc` from the last kp_solve on this ctx (hostname removed as in
 * FinalizeScheduling), one line per key, lines sorted:
 *   "key \t complement(0|1) \t gt|- \t lt|- \t minValues|- \t v1 \x1f v2 ..."   (values sorted)
 * Writes at most cap bytes (incl. NUL); *needed receives the full size.
 */
kp_status kp_result_nodeclaim_requirements(kp_ctx* ctx, int32_t nc, char* buf, int64_t cap, int64_t* needed);

#ifdef __cplusplus
}
#endif
#endif /* KPSIM_H_ */
