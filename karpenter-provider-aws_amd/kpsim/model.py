"""Python mirror of the reference's scheduling inputs/outputs and their marshaling into kpsim C views.

Types mirror the Go types they stand for:
  Requirement   -> karpv1.NodeSelectorRequirementWithMinValues / scheduling.Requirement
  Offering      -> cloudprovider.Offering (pkg/providers/instancetype/offering/offering.go:140-152,179-192)
  InstanceType  -> cloudprovider.InstanceType (Requirements, Capacity, Overhead→Allocatable, Offerings)
  NodePool      -> karpv1.NodePool as a NodeClaimTemplate (weight, template requirements/labels, taints, limits)
  PodClass/Pods -> corev1.Pod scheduling constraints (nodeSelector, required affinity term 0, tolerations)
  Results       -> scheduling.Results (NewNodeClaims, ExistingNodes, PodErrors) after TruncateInstanceTypes(60)
"""
import ctypes as C
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import abi

# Resource axes of the catalog view (types.go computeCapacity :320-338 + PrivateIPv4Address :151-153).
RESOURCES = [
    "cpu", "memory", "ephemeral-storage", "pods", "vpc.amazonaws.com/pod-eni", "nvidia.com/gpu", "amd.com/gpu",
    "aws.amazon.com/neuron", "aws.amazon.com/neuroncore", "habana.ai/gaudi", "vpc.amazonaws.com/efa",
    "vpc.amazonaws.com/PrivateIPv4Address",
]
R = len(RESOURCES)
RIDX = {r: i for i, r in enumerate(RESOURCES)}

# Well-known label keys
ZONE = "topology.kubernetes.io/zone"
ZONE_ID = "topology.k8s.aws/zone-id"
CAPACITY_TYPE = "karpenter.sh/capacity-type"
NODEPOOL = "karpenter.sh/nodepool"
INSTANCE_TYPE = "node.kubernetes.io/instance-type"
ARCH = "kubernetes.io/arch"
OS = "kubernetes.io/os"
RESERVATION_ID = "karpenter.k8s.aws/capacity-reservation-id"      # cloudprovider.ReservationIDLabel (apis/v1/doc.go:38)
RESERVATION_TYPE = "karpenter.k8s.aws/capacity-reservation-type"
OFFERING_KEYS = [CAPACITY_TYPE, ZONE, RESERVATION_ID, RESERVATION_TYPE, ZONE_ID]


@dataclass
class Requirement:
    key: str
    op: str                       # In | NotIn | Exists | DoesNotExist | Gt | Lt
    values: List[str] = field(default_factory=list)
    min_values: Optional[int] = None


@dataclass
class Taint:
    key: str
    value: str = ""
    effect: str = "NoSchedule"


@dataclass
class Toleration:
    key: str = ""
    operator: str = "Equal"       # Equal | Exists
    value: str = ""
    effect: str = ""


@dataclass
class Offering:
    capacity_type: str
    zone: str
    price: float
    available: bool
    zone_id: Optional[str] = None
    reservation_id: Optional[str] = None
    reservation_type: Optional[str] = None
    reservation_capacity: int = 0

    def label(self, key):
        """(state, value) of Offering.Requirements[key]"""
        if key == CAPACITY_TYPE:
            return abi.KP_LABEL_IN, self.capacity_type
        if key == ZONE:
            return abi.KP_LABEL_IN, self.zone
        if key == RESERVATION_ID:
            return (abi.KP_LABEL_IN, self.reservation_id) if self.reservation_id else (abi.KP_LABEL_DOES_NOT_EXIST, None)
        if key == RESERVATION_TYPE:
            return (abi.KP_LABEL_IN, self.reservation_type) if self.reservation_id else (abi.KP_LABEL_DOES_NOT_EXIST, None)
        if key == ZONE_ID:
            return (abi.KP_LABEL_IN, self.zone_id) if self.zone_id else (abi.KP_LABEL_ABSENT, None)
        raise KeyError(key)


@dataclass
class InstanceType:
    name: str
    labels: Dict[str, Optional[List[str]]]   # key -> values (In), or None for DoesNotExist
    capacity: np.ndarray                      # [R] int64 milli
    allocatable: np.ndarray                   # [R] int64 milli
    offerings: List[Offering] = field(default_factory=list)


@dataclass
class NodePool:
    name: str
    weight: int = 0
    requirements: List[Requirement] = field(default_factory=list)
    labels: Dict[str, str] = field(default_factory=dict)
    taints: List[Taint] = field(default_factory=list)
    daemon_overhead: Optional[np.ndarray] = None      # [R] milli
    limits_remaining: Optional[Dict[str, int]] = None  # resource -> remaining milli
    instance_types: Optional[List[int]] = None         # catalog rows; None = all

    def template_requirements(self):
        """NewNodeClaimTemplate: spec requirements + template labels + karpenter.sh/nodepool In [name]."""
        reqs = list(self.requirements)
        labels = dict(self.labels)
        labels[NODEPOOL] = self.name
        for k, v in labels.items():
            reqs.append(Requirement(k, "In", [v]))
        return reqs


@dataclass
class TopologyTerm:
    """corev1.TopologySpreadConstraint (kind "spread") or a pod (anti-)affinity term (kind "affinity" / "anti"), as
    [core] scheduling/topology.go reads them.  selector: LabelSelector as Requirements over pod labels (None = nil)."""
    kind: str                                   # spread | affinity | anti
    key: str                                    # topologyKey
    selector: Optional[List[Requirement]] = field(default_factory=list)
    max_skew: int = 1
    min_domains: Optional[int] = None
    when_unsatisfiable: str = "DoNotSchedule"   # | ScheduleAnyway
    node_affinity_policy: str = "Honor"
    node_taints_policy: str = "Ignore"
    weight: int = 0                             # (anti-)affinity: 0 = required
    namespaces: List[str] = field(default_factory=list)


TOPO_KIND = {"spread": 0, "affinity": 1, "anti": 2}
HOSTNAME = "kubernetes.io/hostname"


@dataclass
class PodClass:
    """requirements: nodeSelector ∪ required node-affinity term[0], or the nodeSelector alone when required_terms is
    given (the ORed NodeSelectorTerms, relaxed from the front).  preferred_terms: (weight, requirements) of the
    preferred node affinity (kpsim.h kp_pod_class)."""
    requirements: List[Requirement] = field(default_factory=list)
    tolerations: List[Toleration] = field(default_factory=list)
    labels: Dict[str, str] = field(default_factory=dict)
    namespace: str = "default"
    topology: List[TopologyTerm] = field(default_factory=list)
    required_terms: List[List[Requirement]] = field(default_factory=list)
    preferred_terms: List[Tuple[int, List[Requirement]]] = field(default_factory=list)


@dataclass
class Pods:
    class_id: np.ndarray      # [P] int32
    requests: np.ndarray      # [P, R] int64 milli (incl. pods = 1000)
    creation_ns: np.ndarray   # [P] int64
    uids: List[str]

    @property
    def n(self):
        return int(self.class_id.shape[0])


@dataclass
class ExistingNode:
    name: str
    labels: Dict[str, str]
    available: np.ndarray
    requests: Optional[np.ndarray] = None
    taints: List[Taint] = field(default_factory=list)


@dataclass
class Problem:
    catalog: List[InstanceType]
    nodepools: List[NodePool]
    classes: List[PodClass]
    pods: Pods
    existing: List[ExistingNode] = field(default_factory=list)
    max_instance_types: int = 60
    min_values_policy: int = 0
    bound: List[tuple] = field(default_factory=list)   # (existing node, class) of pods already bound (topology counts)


@dataclass
class Candidate:
    """disruption.Candidate: a state node considered for consolidation."""
    node: int                       # index into ConsolidationProblem.cluster.existing
    pods: np.ndarray                # reschedulable pods, indices into cluster.pods
    price: float                    # cheapest offering of its instance type compatible with the node's labels
    capacity_type: int = abi.KP_CT_ON_DEMAND
    instance_type: int = -1         # catalog row
    nodepool: int = -1              # index into cluster.nodepools
    capacity: Optional[np.ndarray] = None  # [R] node capacity (returns to the NodePool's limits)


@dataclass
class ConsolidationProblem:
    """Cluster state of one consolidation pass: the Problem's existing nodes are ALL state nodes in NewScheduler
    order (initialized first, then by name); its pods are the pending pods plus every candidate's pods."""
    cluster: Problem
    candidates: List[Candidate]
    pending: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    initialized: Optional[np.ndarray] = None  # [E] uint8


def consolidation_probe_count(n_candidates, mode, max_candidates=100):
    """Same numbering as kp_consolidate_probe_count (include/kpsim.h); KP_CONSOLIDATE_BOTH: multi then single."""
    if mode == abi.KP_CONSOLIDATE_SINGLE:
        return n_candidates
    nm = 0 if n_candidates < 2 else (n_candidates - 1 if n_candidates <= max_candidates else max_candidates)
    return nm + n_candidates if mode == abi.KP_CONSOLIDATE_BOTH else nm


# ------------------------------------------------------------------------------------------------
# views
# ------------------------------------------------------------------------------------------------
class CatalogView:
    """kp_catalog_view over a list of InstanceType (buffers owned by self.keep)."""

    def __init__(self, catalog: List[InstanceType]):
        k = self.keep = abi.Keep()
        T = len(catalog)
        keys = []
        kidx = {}
        for it in catalog:
            for key in it.labels:
                if key not in kidx:
                    kidx[key] = len(keys)
                    keys.append(key)
        K = len(keys)
        state = np.zeros((T, K), np.int8)
        offsets = np.zeros(T * K + 1, np.int32)
        vals = []
        for t, it in enumerate(catalog):
            for key, v in it.labels.items():
                state[t, kidx[key]] = abi.KP_LABEL_DOES_NOT_EXIST if v is None else abi.KP_LABEL_IN
        # CSR in (t, k) order
        pos = 0
        for t, it in enumerate(catalog):
            for j, key in enumerate(keys):
                offsets[t * K + j] = pos
                v = it.labels.get(key)
                if v is not None and state[t, j] == abi.KP_LABEL_IN:
                    vals.extend(v)
                    pos += len(v)
        offsets[T * K] = pos
        cap = np.stack([it.capacity for it in catalog]).astype(np.int64) if T else np.zeros((0, R), np.int64)
        alloc = np.stack([it.allocatable for it in catalog]).astype(np.int64) if T else np.zeros((0, R), np.int64)
        otype, oprice, oavail, ocap, ostate, ovals = [], [], [], [], [], []
        for t, it in enumerate(catalog):
            for o in it.offerings:
                otype.append(t)
                oprice.append(o.price)
                oavail.append(1 if o.available else 0)
                ocap.append(o.reservation_capacity)
                for key in OFFERING_KEYS:
                    st, v = o.label(key)
                    ostate.append(st)
                    ovals.append(v or "")
        v = self.view = abi.kp_catalog_view()
        v.n_types = T
        v.n_resources = R
        v.resource_names = k.cstrs(RESOURCES)
        v.type_names = k.cstrs([it.name for it in catalog])
        v.capacity = k.ptr(cap, np.int64, C.c_int64)
        v.allocatable = k.ptr(alloc, np.int64, C.c_int64)
        v.n_label_keys = K
        v.label_keys = k.cstrs(keys)
        v.label_state = k.ptr(state.reshape(-1), np.int8, C.c_int8)
        v.label_offsets = k.ptr(offsets, np.int32, C.c_int32)
        v.label_values = k.cstrs(vals)
        v.n_offerings = len(otype)
        v.offering_type = k.ptr(np.array(otype, np.int32), np.int32, C.c_int32)
        v.offering_price = k.ptr(np.array(oprice, np.float64), np.float64, C.c_double)
        v.offering_available = k.ptr(np.array(oavail, np.uint8), np.uint8, C.c_uint8)
        v.offering_reservation_capacity = k.ptr(np.array(ocap, np.int32), np.int32, C.c_int32)
        v.n_offering_keys = len(OFFERING_KEYS)
        v.offering_keys = k.cstrs(OFFERING_KEYS)
        v.offering_label_state = k.ptr(np.array(ostate, np.int8), np.int8, C.c_int8)
        v.offering_label_values = k.cstrs(ovals)
        self.n_offerings = len(otype)


class SolveInputView:
    """kp_solve_input for a Problem (buffers owned by self.keep)."""

    def __init__(self, prob: Problem):
        k = self.keep = abi.Keep()
        nps = (abi.kp_nodepool * max(1, len(prob.nodepools)))()
        for i, np_ in enumerate(prob.nodepools):
            x = nps[i]
            x.name = np_.name.encode()
            x.weight = int(np_.weight)
            x.n_requirements, x.requirements = abi.requirement_array(k, np_.template_requirements())
            x.n_taints, x.taints = abi.taint_array(k, np_.taints)
            if np_.daemon_overhead is not None:
                x.daemon_overhead = k.ptr(np_.daemon_overhead, np.int64, C.c_int64)
            if np_.limits_remaining:
                ls = np.zeros(R, np.uint8)
                lr = np.zeros(R, np.int64)
                for res, q in np_.limits_remaining.items():
                    ls[RIDX[res]] = 1
                    lr[RIDX[res]] = q
                x.limit_set = k.ptr(ls, np.uint8, C.c_uint8)
                x.limit_remaining = k.ptr(lr, np.int64, C.c_int64)
            if np_.instance_types is None:
                x.n_types = -1
            else:
                x.n_types = len(np_.instance_types)
                x.type_index = k.ptr(np.array(np_.instance_types, np.int32), np.int32, C.c_int32)
        k.hold(nps)
        cls = (abi.kp_pod_class * max(1, len(prob.classes)))()
        for i, pc in enumerate(prob.classes):
            cls[i].n_requirements, cls[i].requirements = abi.requirement_array(k, pc.requirements)
            cls[i].n_tolerations, cls[i].tolerations = abi.toleration_array(k, pc.tolerations)
            cls[i].namespace_name = pc.namespace.encode()
            cls[i].n_labels = len(pc.labels)
            cls[i].label_keys = k.cstrs(list(pc.labels.keys()))
            cls[i].label_values = k.cstrs(list(pc.labels.values()))
            cls[i].n_topology, cls[i].topology = abi.topology_array(k, pc.topology)
            cls[i].n_required_terms, cls[i].required_terms = abi.node_term_array(k, [(0, t) for t in pc.required_terms])
            cls[i].n_preferred_terms, cls[i].preferred_terms = abi.node_term_array(k, pc.preferred_terms)
        k.hold(cls)
        ex = (abi.kp_existing_node * max(1, len(prob.existing)))()
        for i, e in enumerate(prob.existing):
            ex[i].name = e.name.encode()
            ex[i].n_labels = len(e.labels)
            ex[i].label_keys = k.cstrs(list(e.labels.keys()))
            ex[i].label_values = k.cstrs(list(e.labels.values()))
            ex[i].n_taints, ex[i].taints = abi.taint_array(k, e.taints)
            ex[i].available = k.ptr(e.available, np.int64, C.c_int64)
            if e.requests is not None:
                ex[i].requests = k.ptr(e.requests, np.int64, C.c_int64)
        k.hold(ex)
        v = self.view = abi.kp_solve_input()
        v.n_nodepools = len(prob.nodepools)
        v.nodepools = nps
        v.n_classes = len(prob.classes)
        v.classes = cls
        p = prob.pods
        v.pods.n_pods = p.n
        v.pods.class_id = k.ptr(p.class_id, np.int32, C.c_int32)
        v.pods.requests = k.ptr(p.requests.reshape(-1), np.int64, C.c_int64)
        v.pods.creation_ns = k.ptr(p.creation_ns, np.int64, C.c_int64)
        v.pods.uids = k.cstrs(p.uids)
        v.n_existing = len(prob.existing)
        v.existing = ex
        v.max_instance_types = prob.max_instance_types
        v.min_values_policy = prob.min_values_policy
        v.n_bound = len(prob.bound)
        if prob.bound:
            b = np.array(prob.bound, np.int32).reshape(-1, 2)
            v.bound_node = k.ptr(b[:, 0].copy(), np.int32, C.c_int32)
            v.bound_class = k.ptr(b[:, 1].copy(), np.int32, C.c_int32)


@dataclass
class Results:
    """scheduling.Results after TruncateInstanceTypes, in canonical-comparable form."""
    nodeclaim_nodepool: np.ndarray
    nodeclaim_n_pods: np.ndarray
    nodeclaim_slice_pos: np.ndarray
    nodeclaim_n_options: np.ndarray
    nodeclaim_types: List[List[int]]
    pod_result: np.ndarray
    pod_order: np.ndarray
    stats: dict

    @property
    def n_nodeclaims(self):
        return len(self.nodeclaim_types)


class OutputBuffers:
    def __init__(self, n_pods, cap_nodeclaims, cap_type_ids):
        self.keep = abi.Keep()
        k = self.keep
        self.arrays = {}
        o = self.view = abi.kp_solve_output()
        o.cap_nodeclaims = cap_nodeclaims
        o.cap_type_ids = cap_type_ids

        def buf(name, n):
            a = np.full(max(1, n), -7, np.int32)
            self.arrays[name] = a
            k.hold(a)
            setattr(o, name, a.ctypes.data_as(abi.c_int32_p))

        buf("nodeclaim_nodepool", cap_nodeclaims)
        buf("nodeclaim_n_pods", cap_nodeclaims)
        buf("nodeclaim_slice_pos", cap_nodeclaims)
        buf("nodeclaim_n_options", cap_nodeclaims)
        buf("nodeclaim_type_offset", cap_nodeclaims + 1)
        buf("type_ids", cap_type_ids)
        buf("pod_result", n_pods)
        buf("pod_order", n_pods)
        self.n_pods = n_pods

    def results(self) -> Results:
        o = self.view
        n = o.n_nodeclaims
        a = self.arrays
        off = a["nodeclaim_type_offset"]
        types = [a["type_ids"][off[i]:off[i + 1]].tolist() for i in range(n)]
        st = {f: getattr(o.stats, f) for f, _ in abi.kp_solve_stats._fields_}
        return Results(a["nodeclaim_nodepool"][:n].copy(), a["nodeclaim_n_pods"][:n].copy(),
                       a["nodeclaim_slice_pos"][:n].copy(), a["nodeclaim_n_options"][:n].copy(), types,
                       a["pod_result"][:self.n_pods].copy(), a["pod_order"][:self.n_pods].copy(), st)


def parse_requirements_blob(s: str):
    """kp_result_nodeclaim_requirements serialization -> {key: (complement, gt, lt, min, tuple(values))}"""
    out = {}
    for line in s.split("\n"):
        if not line:
            continue
        key, comp, gt, lt, mn, vals = line.split("\t")
        out[key] = (comp == "1", gt, lt, mn, tuple(v for v in vals.split("\x1f") if v != "") if vals else ())
    return out


class ConsolidateInputView:
    """kp_consolidate_input for a ConsolidationProblem, probes [probe_begin, probe_end)."""

    def __init__(self, cp: ConsolidationProblem, mode, probe_begin=0, probe_end=0, spot_to_spot=False,
                 max_candidates=100, cluster_view: Optional[SolveInputView] = None):
        self.cluster_view = cluster_view or SolveInputView(cp.cluster)
        k = self.keep = abi.Keep()
        v = self.view = abi.kp_consolidate_input()
        v.cluster = self.cluster_view.view
        if cp.initialized is not None:
            v.initialized = k.ptr(cp.initialized, np.uint8, C.c_uint8)
        v.n_pending = len(cp.pending)
        v.pending = k.ptr(cp.pending, np.int32, C.c_int32)
        cands = (abi.kp_candidate * max(1, len(cp.candidates)))()
        for i, c in enumerate(cp.candidates):
            x = cands[i]
            x.node = int(c.node)
            x.n_pods = len(c.pods)
            x.pods = k.ptr(c.pods, np.int32, C.c_int32)
            x.price = float(c.price)
            x.capacity_type = int(c.capacity_type)
            x.instance_type = int(c.instance_type)
            x.nodepool = int(c.nodepool)
            if c.capacity is not None:
                x.capacity = k.ptr(c.capacity, np.int64, C.c_int64)
        k.hold(cands)
        v.n_candidates = len(cp.candidates)
        v.candidates = cands
        v.mode = int(mode)
        v.max_candidates = int(max_candidates)
        v.probe_begin = int(probe_begin)
        v.probe_end = int(probe_end)
        v.spot_to_spot = 1 if spot_to_spot else 0


@dataclass
class LaunchRequest:
    """A NodeClaim as CloudProvider.Create sees it (pkg/providers/instance/instance.go:132): Spec.Requirements (with
    minValues) and Spec.Resources.Requests (milli, RESOURCES order; 0 = not requested)."""
    requirements: List[Requirement]
    requests: np.ndarray


class LaunchBatchView:
    """kp_launch_request[n] (buffers owned by self.keep)."""

    def __init__(self, reqs: List[LaunchRequest]):
        k = self.keep = abi.Keep()
        self.n = len(reqs)
        arr = (abi.kp_launch_request * max(1, self.n))()
        for i, lr in enumerate(reqs):
            nr, ra = abi.requirement_array(k, lr.requirements)
            arr[i].n_requirements = nr
            arr[i].requirements = ra
            arr[i].requests = k.ptr(np.asarray(lr.requests, np.int64), np.int64, C.c_int64)
        k.hold(arr)
        self.array = arr


@dataclass
class LaunchResults:
    """Per request: LAUNCH_DTYPE rows, plus the concatenated type ids and override offering rows."""
    rows: np.ndarray
    type_ids: np.ndarray
    overrides: np.ndarray

    def types(self, i):
        r = self.rows[i]
        return self.type_ids[r["type_offset"]:r["type_offset"] + r["n_types"]]

    def offerings(self, i):
        r = self.rows[i]
        return self.overrides[r["override_offset"]:r["override_offset"] + r["n_overrides"]]


def launch_buffers(n, M, catalog_view):
    rows = np.zeros(max(1, n), abi.LAUNCH_DTYPE)
    tids = np.zeros(max(1, n * M), np.int32)
    ovs = np.zeros(max(1, n * M * 64), np.int32)
    return rows, tids, ovs


def launch_call(fn, cv, batch: LaunchBatchView, M):
    """Runs fn(n, requests, M, results, type_ids, cap, overrides, cap) (kp_launch_select or its oracle)."""
    rows, tids, ovs = launch_buffers(batch.n, M, cv)
    st = fn(batch.n, batch.array, M, rows.ctypes.data_as(C.POINTER(abi.kp_launch_result)),
            tids.ctypes.data_as(C.POINTER(C.c_int32)), len(tids), ovs.ctypes.data_as(C.POINTER(C.c_int32)), len(ovs))
    return st, LaunchResults(rows[:batch.n], tids, ovs)
