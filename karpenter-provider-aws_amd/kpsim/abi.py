"""ctypes mirror of include/kpsim.h plus marshaling of the Python model into the C views.

The same views are handed to libkpsim.so (the product) and, in tests only, to the CPU oracle, so both
sides see byte-identical inputs.
"""
import ctypes as C

import numpy as np

c_int8_p = C.POINTER(C.c_int8)
c_uint8_p = C.POINTER(C.c_uint8)
c_int32_p = C.POINTER(C.c_int32)
c_int64_p = C.POINTER(C.c_int64)
c_double_p = C.POINTER(C.c_double)
c_char_pp = C.POINTER(C.c_char_p)

KP_OK, KP_E_INVALID, KP_E_BUFFER, KP_E_DEVICE, KP_E_INSUFFICIENT_CAPACITY, KP_E_NODECLASS_NOT_READY, \
    KP_E_CREATE, KP_E_UNSUPPORTED, KP_E_STATE = range(9)
STATUS_NAMES = {0: "KP_OK", 1: "KP_E_INVALID", 2: "KP_E_BUFFER", 3: "KP_E_DEVICE", 4: "KP_E_INSUFFICIENT_CAPACITY",
                5: "KP_E_NODECLASS_NOT_READY", 6: "KP_E_CREATE", 7: "KP_E_UNSUPPORTED", 8: "KP_E_STATE"}

OPS = {"In": 0, "NotIn": 1, "Exists": 2, "DoesNotExist": 3, "Gt": 4, "Lt": 5}
KP_TOL_EQUAL, KP_TOL_EXISTS = 0, 1
KP_LABEL_ABSENT, KP_LABEL_DOES_NOT_EXIST, KP_LABEL_IN = 0, 1, 2
KP_POD_UNSCHEDULABLE = -1


def KP_POD_EXISTING(j):
    return -2 - j


class kp_requirement(C.Structure):
    _fields_ = [("key", C.c_char_p), ("op", C.c_int32), ("n_values", C.c_int32), ("values", c_char_pp),
                ("min_values", C.c_int32)]


class kp_taint(C.Structure):
    _fields_ = [("key", C.c_char_p), ("value", C.c_char_p), ("effect", C.c_char_p)]


class kp_toleration(C.Structure):
    _fields_ = [("key", C.c_char_p), ("op", C.c_int32), ("value", C.c_char_p), ("effect", C.c_char_p)]


class kp_catalog_view(C.Structure):
    _fields_ = [
        ("n_types", C.c_int32), ("n_resources", C.c_int32), ("resource_names", c_char_pp), ("type_names", c_char_pp),
        ("capacity", c_int64_p), ("allocatable", c_int64_p),
        ("n_label_keys", C.c_int32), ("label_keys", c_char_pp), ("label_state", c_int8_p),
        ("label_offsets", c_int32_p), ("label_values", c_char_pp),
        ("n_offerings", C.c_int32), ("offering_type", c_int32_p), ("offering_price", c_double_p),
        ("offering_available", c_uint8_p), ("offering_reservation_capacity", c_int32_p),
        ("n_offering_keys", C.c_int32), ("offering_keys", c_char_pp), ("offering_label_state", c_int8_p),
        ("offering_label_values", c_char_pp),
    ]


class kp_nodepool(C.Structure):
    _fields_ = [
        ("name", C.c_char_p), ("weight", C.c_int32), ("n_requirements", C.c_int32),
        ("requirements", C.POINTER(kp_requirement)), ("n_taints", C.c_int32), ("taints", C.POINTER(kp_taint)),
        ("daemon_overhead", c_int64_p), ("limit_set", c_uint8_p), ("limit_remaining", c_int64_p),
        ("n_types", C.c_int32), ("type_index", c_int32_p),
    ]


KP_TOPO_SPREAD, KP_TOPO_AFFINITY, KP_TOPO_ANTI_AFFINITY = 0, 1, 2
KP_POLICY_IGNORE, KP_POLICY_HONOR = 0, 1
KP_DO_NOT_SCHEDULE, KP_SCHEDULE_ANYWAY = 0, 1
KP_PREFERENCE_RESPECT, KP_PREFERENCE_IGNORE = 0, 1
KP_MIN_VALUES_STRICT, KP_MIN_VALUES_BEST_EFFORT = 0, 1


class kp_topology_term(C.Structure):
    _fields_ = [("type", C.c_int32), ("topology_key", C.c_char_p), ("max_skew", C.c_int32), ("min_domains", C.c_int32),
                ("when_unsatisfiable", C.c_int32), ("node_affinity_policy", C.c_int32),
                ("node_taints_policy", C.c_int32), ("weight", C.c_int32), ("n_selector", C.c_int32),
                ("selector", C.POINTER(kp_requirement)), ("n_namespaces", C.c_int32), ("namespaces", c_char_pp)]


class kp_node_selector_term(C.Structure):
    _fields_ = [("weight", C.c_int32), ("n_requirements", C.c_int32), ("requirements", C.POINTER(kp_requirement))]


class kp_pod_class(C.Structure):
    _fields_ = [("n_requirements", C.c_int32), ("requirements", C.POINTER(kp_requirement)),
                ("n_tolerations", C.c_int32), ("tolerations", C.POINTER(kp_toleration)),
                ("namespace_name", C.c_char_p), ("n_labels", C.c_int32), ("label_keys", c_char_pp),
                ("label_values", c_char_pp), ("n_topology", C.c_int32), ("topology", C.POINTER(kp_topology_term)),
                ("n_required_terms", C.c_int32), ("required_terms", C.POINTER(kp_node_selector_term)),
                ("n_preferred_terms", C.c_int32), ("preferred_terms", C.POINTER(kp_node_selector_term))]


class kp_pods_view(C.Structure):
    _fields_ = [("n_pods", C.c_int32), ("class_id", c_int32_p), ("requests", c_int64_p), ("creation_ns", c_int64_p),
                ("uids", c_char_pp)]


class kp_existing_node(C.Structure):
    _fields_ = [("name", C.c_char_p), ("n_labels", C.c_int32), ("label_keys", c_char_pp), ("label_values", c_char_pp),
                ("n_taints", C.c_int32), ("taints", C.POINTER(kp_taint)), ("available", c_int64_p),
                ("requests", c_int64_p)]


class kp_solve_input(C.Structure):
    _fields_ = [("n_nodepools", C.c_int32), ("nodepools", C.POINTER(kp_nodepool)),
                ("n_classes", C.c_int32), ("classes", C.POINTER(kp_pod_class)),
                ("pods", kp_pods_view),
                ("n_existing", C.c_int32), ("existing", C.POINTER(kp_existing_node)),
                ("max_instance_types", C.c_int32), ("min_values_policy", C.c_int32),
                ("n_bound", C.c_int32), ("bound_node", c_int32_p), ("bound_class", c_int32_p)]


class kp_solve_stats(C.Structure):
    _fields_ = [("pods_popped", C.c_int64), ("nodeclaim_evals", C.c_int64), ("nodeclaim_candidates_scanned", C.c_int64),
                ("template_evals", C.c_int64), ("existing_evals", C.c_int64), ("sorts_fast", C.c_int64),
                ("sorts_full", C.c_int64), ("ns_host_prep", C.c_double), ("ns_device_solve", C.c_double),
                ("ns_device_finalize", C.c_double), ("ns_total", C.c_double)]


class kp_solve_output(C.Structure):
    _fields_ = [("cap_nodeclaims", C.c_int32), ("cap_type_ids", C.c_int32), ("n_nodeclaims", C.c_int32),
                ("n_type_ids", C.c_int32), ("nodeclaim_nodepool", c_int32_p), ("nodeclaim_n_pods", c_int32_p),
                ("nodeclaim_slice_pos", c_int32_p), ("nodeclaim_n_options", c_int32_p),
                ("nodeclaim_type_offset", c_int32_p), ("type_ids", c_int32_p), ("pod_result", c_int32_p),
                ("pod_order", c_int32_p), ("stats", kp_solve_stats)]


KP_CONSOLIDATE_SINGLE, KP_CONSOLIDATE_MULTI, KP_CONSOLIDATE_BOTH = 0, 1, 2
KP_DECISION_NONE, KP_DECISION_DELETE, KP_DECISION_REPLACE = 0, 1, 2
KP_CT_ON_DEMAND, KP_CT_SPOT, KP_CT_RESERVED = 0, 1, 2


class kp_candidate(C.Structure):
    _fields_ = [("node", C.c_int32), ("n_pods", C.c_int32), ("pods", c_int32_p), ("price", C.c_double),
                ("capacity_type", C.c_int32), ("instance_type", C.c_int32), ("nodepool", C.c_int32),
                ("capacity", c_int64_p)]


class kp_consolidate_input(C.Structure):
    _fields_ = [("cluster", kp_solve_input), ("initialized", c_uint8_p), ("n_pending", C.c_int32),
                ("pending", c_int32_p), ("n_candidates", C.c_int32), ("candidates", C.POINTER(kp_candidate)),
                ("mode", C.c_int32), ("max_candidates", C.c_int32), ("probe_begin", C.c_int32),
                ("probe_end", C.c_int32), ("spot_to_spot", C.c_int32)]


class kp_probe_result(C.Structure):
    _fields_ = [("decision", C.c_int32), ("valid", C.c_int32), ("all_scheduled", C.c_int32),
                ("n_new_nodeclaims", C.c_int32), ("n_replacement_types", C.c_int32), ("n_pods", C.c_int32),
                ("candidate_price", C.c_double), ("replacement_price", C.c_double)]


class kp_consolidation_command(C.Structure):
    _fields_ = [("cap_type_ids", C.c_int32), ("type_ids", c_int32_p), ("cap_requirements", C.c_int64),
                ("requirements", C.c_char_p), ("decision", C.c_int32), ("mode", C.c_int32), ("probe", C.c_int32),
                ("first_candidate", C.c_int32), ("n_candidates", C.c_int32), ("nodepool", C.c_int32),
                ("n_type_ids", C.c_int32), ("n_reserved", C.c_int32), ("requirements_needed", C.c_int64),
                ("result", kp_probe_result)]


PROBE_DTYPE = np.dtype([("decision", np.int32), ("valid", np.int32), ("all_scheduled", np.int32),
                        ("n_new_nodeclaims", np.int32), ("n_replacement_types", np.int32), ("n_pods", np.int32),
                        ("candidate_price", np.float64), ("replacement_price", np.float64)])
assert PROBE_DTYPE.itemsize == C.sizeof(kp_probe_result)


KP_FILTER_NAMES = ["compatible-available-filter", "capacity-reservation-type-filter", "capacity-block-filter",
                   "reserved-offering-filter", "exotic-instance-filter", "spot-instance-filter"]  # filter.go Name()
KP_N_FILTERS = 6
(KP_FILTER_COMPATIBLE_AVAILABLE, KP_FILTER_CAPACITY_RESERVATION_TYPE, KP_FILTER_CAPACITY_BLOCK,
 KP_FILTER_RESERVED_OFFERING, KP_FILTER_EXOTIC, KP_FILTER_SPOT) = range(6)


class kp_launch_request(C.Structure):
    _fields_ = [("n_requirements", C.c_int32), ("requirements", C.POINTER(kp_requirement)),
                ("requests", C.POINTER(C.c_int64))]


class kp_launch_result(C.Structure):
    _fields_ = [("status", C.c_int32), ("failed_filter", C.c_int32), ("capacity_type", C.c_int32),
                ("n_types", C.c_int32), ("type_offset", C.c_int32), ("n_overrides", C.c_int32),
                ("override_offset", C.c_int32), ("n_options", C.c_int32), ("rejected", C.c_int32 * KP_N_FILTERS),
                ("fleet_pick", C.c_int32)]


LAUNCH_DTYPE = np.dtype([("status", np.int32), ("failed_filter", np.int32), ("capacity_type", np.int32),
                         ("n_types", np.int32), ("type_offset", np.int32), ("n_overrides", np.int32),
                         ("override_offset", np.int32), ("n_options", np.int32), ("rejected", np.int32, KP_N_FILTERS),
                         ("fleet_pick", np.int32)])
assert LAUNCH_DTYPE.itemsize == C.sizeof(kp_launch_result)


class kp_device_opts(C.Structure):
    _fields_ = [("device", C.c_int32), ("n_devices", C.c_int32), ("devices", c_int32_p),
                ("preference_policy", C.c_int32), ("reserved_capacity", C.c_int32)]


# ------------------------------------------------------------------------------------------------
# marshaling helpers — a Keep object owns every buffer a view points into
# ------------------------------------------------------------------------------------------------
class Keep:
    def __init__(self):
        self.refs = []

    def hold(self, x):
        self.refs.append(x)
        return x

    def cstrs(self, strs):
        arr = (C.c_char_p * max(1, len(strs)))(*[s.encode() if isinstance(s, str) else s for s in strs])
        return self.hold(arr)

    def np(self, a, dtype):
        a = np.ascontiguousarray(a, dtype=dtype)
        self.hold(a)
        return a

    def ptr(self, a, dtype, ctype):
        a = self.np(a, dtype)
        return a.ctypes.data_as(C.POINTER(ctype))


def requirement_array(keep, reqs):
    """reqs: iterable of model.Requirement -> (n, POINTER(kp_requirement))"""
    reqs = list(reqs)
    arr = (kp_requirement * max(1, len(reqs)))()
    for i, r in enumerate(reqs):
        arr[i].key = r.key.encode()
        arr[i].op = OPS[r.op]
        arr[i].n_values = len(r.values)
        arr[i].values = keep.cstrs(list(r.values))
        arr[i].min_values = -1 if r.min_values is None else int(r.min_values)
    keep.hold(arr)
    return len(reqs), arr


def node_term_array(keep, terms):
    """terms: iterable of (weight, [model.Requirement]) -> (n, POINTER(kp_node_selector_term))"""
    terms = list(terms)
    arr = (kp_node_selector_term * max(1, len(terms)))()
    for i, (w, reqs) in enumerate(terms):
        arr[i].weight = int(w)
        arr[i].n_requirements, arr[i].requirements = requirement_array(keep, reqs)
    keep.hold(arr)
    return len(terms), arr


def taint_array(keep, taints):
    taints = list(taints)
    arr = (kp_taint * max(1, len(taints)))()
    for i, t in enumerate(taints):
        arr[i].key = t.key.encode()
        arr[i].value = (t.value or "").encode()
        arr[i].effect = t.effect.encode()
    keep.hold(arr)
    return len(taints), arr


def toleration_array(keep, tols):
    tols = list(tols)
    arr = (kp_toleration * max(1, len(tols)))()
    for i, t in enumerate(tols):
        arr[i].key = (t.key or "").encode()
        arr[i].op = KP_TOL_EXISTS if t.operator == "Exists" else KP_TOL_EQUAL
        arr[i].value = (t.value or "").encode()
        arr[i].effect = (t.effect or "").encode()
    keep.hold(arr)
    return len(tols), arr


def topology_array(keep, terms):
    """terms: iterable of model.TopologyTerm -> (n, POINTER(kp_topology_term))"""
    from kpsim.model import TOPO_KIND
    terms = list(terms)
    arr = (kp_topology_term * max(1, len(terms)))()
    pol = {"Ignore": KP_POLICY_IGNORE, "Honor": KP_POLICY_HONOR}
    for i, t in enumerate(terms):
        x = arr[i]
        x.type = TOPO_KIND[t.kind]
        x.topology_key = t.key.encode()
        x.max_skew = int(t.max_skew)
        x.min_domains = int(t.min_domains) if t.min_domains else 0
        x.when_unsatisfiable = KP_SCHEDULE_ANYWAY if t.when_unsatisfiable == "ScheduleAnyway" else KP_DO_NOT_SCHEDULE
        x.node_affinity_policy = pol[t.node_affinity_policy]
        x.node_taints_policy = pol[t.node_taints_policy]
        x.weight = int(t.weight)
        if t.selector is None:
            x.n_selector = -1
            x.selector = (kp_requirement * 1)()
            keep.hold(x.selector)
        else:
            x.n_selector, x.selector = requirement_array(keep, t.selector)
        x.n_namespaces = len(t.namespaces)
        x.namespaces = keep.cstrs(list(t.namespaces))
    keep.hold(arr)
    return len(terms), arr
