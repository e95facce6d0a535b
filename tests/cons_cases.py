"""Consolidation scenarios of the reference's e2e suites, as ConsolidationProblems over the golden catalog.

Each builder returns (cp, expect) where expect holds the reference's asserted outcome for the command
(kp_consolidate_command / orc_consolidate_command).  Cluster shapes follow the suites' setup (NodePool requirements,
deployment pod specs, the nodes the first provisioning round launched); quantities the e2e environment supplies at run
time (daemonset overhead, node allocatable) come from the golden catalog.

  reserved_into        test/suites/consolidation/suite_test.go:915-957  "should consolidate into a reserved offering"
  reserved_between     test/suites/consolidation/suite_test.go:958-1001 "should consolidate between reserved offerings"
"""
import copy

import numpy as np

from kpsim import abi, model, synth
from kpsim.model import CAPACITY_TYPE, INSTANCE_TYPE, RESERVATION_ID, RESERVATION_TYPE

ZA = "test-zone-1a"


def row(catalog, name):
    return next(i for i, it in enumerate(catalog) if it.name == name)


def add_reservation(catalog, name, rid, zone=ZA, capacity=1, rtype="default"):
    """A capacity reservation of `name` in `zone` (offering.go:164-194): price = odPrice / 1e7, Available iff
    capacity != 0, and computeRequirements' capacity-type / reservation labels (types.go:181-234)."""
    it = catalog[row(catalog, name)]
    od = next(o for o in it.offerings if o.capacity_type == "on-demand" and o.zone == zone)
    it.offerings.append(model.Offering("reserved", zone, od.price / 10_000_000.0, capacity != 0, zone_id=od.zone_id,
                                       reservation_id=rid, reservation_type=rtype, reservation_capacity=capacity))
    res = [o for o in it.offerings if o.capacity_type == "reserved"]
    cts = list(it.labels.get(CAPACITY_TYPE) or [])
    if "reserved" not in cts:
        it.labels[CAPACITY_TYPE] = cts + ["reserved"]
    it.labels[RESERVATION_ID] = sorted({o.reservation_id for o in res})
    it.labels[RESERVATION_TYPE] = sorted({o.reservation_type for o in res})
    return it


def _reserved_pool():
    # suite_test.go:891-913: capacity-type In [on-demand, reserved]
    return model.NodePool("default", requirements=[model.Requirement(CAPACITY_TYPE, "In", ["on-demand", "reserved"])])


def _one_pod_node(catalog, name, ct, labels_extra=None):
    it = catalog[row(catalog, name)]
    pods = synth.pods_from_specs([(0, {"cpu": "100m", "memory": "128Mi"})])
    labels = synth.node_labels(it, ZA, ct, "default")
    labels.update(labels_extra or {})
    avail = np.array(it.allocatable, np.int64) - pods.requests[0]
    node = model.ExistingNode("node-0", labels, avail, np.zeros(model.R, np.int64))
    return it, pods, labels, node


def _dep_class():
    # the deployment's pods: node.kubernetes.io/instance-type In [m5.large, m5.xlarge] (suite_test.go:917-927)
    return model.PodClass(requirements=[model.Requirement(INSTANCE_TYPE, "In", ["m5.large", "m5.xlarge"])],
                          labels={"app": "dep"})


def reserved_into(golden):
    """An m5.large on-demand node; a reservation of m5.xlarge (capacity 1) appears: the node is replaced by an m5.xlarge
    in that reservation ("We should prioritize the reserved instance since it's already been paid for")."""
    cat = copy.deepcopy(golden)
    add_reservation(cat, "m5.xlarge", "cr-xlarge")
    it, pods, labels, node = _one_pod_node(cat, "m5.large", "on-demand")
    prob = model.Problem(cat, [_reserved_pool()], [_dep_class()], pods, [node])
    cand = model.Candidate(node=0, pods=np.array([0], np.int32), price=synth.candidate_price(it, labels),
                           capacity_type=abi.KP_CT_ON_DEMAND, instance_type=row(cat, "m5.large"), nodepool=0,
                           capacity=np.array(it.capacity, np.int64))
    cp = model.ConsolidationProblem(prob, [cand], np.zeros(0, np.int32), np.ones(1, np.uint8))
    return cp, dict(decision=abi.KP_DECISION_REPLACE, types=["m5.xlarge"], reservation="cr-xlarge")


def reserved_between(golden):
    """An m5.xlarge node in reservation cr-xlarge (its only instance: available count 0); a reservation of m5.large
    (capacity 1) appears: the node is replaced by an m5.large in cr-large."""
    cat = copy.deepcopy(golden)
    add_reservation(cat, "m5.xlarge", "cr-xlarge", capacity=0)
    add_reservation(cat, "m5.large", "cr-large", capacity=1)
    it, pods, labels, node = _one_pod_node(cat, "m5.xlarge", "reserved",
                                           {RESERVATION_ID: "cr-xlarge", RESERVATION_TYPE: "default"})
    prob = model.Problem(cat, [_reserved_pool()], [_dep_class()], pods, [node])
    price = synth.candidate_price(it, labels)
    assert price is not None and price < 1e-6
    cand = model.Candidate(node=0, pods=np.array([0], np.int32), price=price, capacity_type=abi.KP_CT_RESERVED,
                           instance_type=row(cat, "m5.xlarge"), nodepool=0, capacity=np.array(it.capacity, np.int64))
    cp = model.ConsolidationProblem(prob, [cand], np.zeros(0, np.int32), np.ones(1, np.uint8))
    return cp, dict(decision=abi.KP_DECISION_REPLACE, types=["m5.large"], reservation="cr-large")


def req_lines(text):
    """kp_result_nodeclaim_requirements text -> {key: (complement, values)}"""
    out = {}
    for line in text.splitlines():
        if not line:
            continue
        key, cmp_, _gt, _lt, _mv, vals = line.split("\t")
        out[key] = (cmp_ == "1", vals.split("\x1f") if vals else [])
    return out


def check_expect(cmd, cp, expect):
    """The reference's asserted outcome of a scenario, on a kpsim.consolidation.Command."""
    cat = cp.cluster.catalog
    assert cmd.decision == expect["decision"], cmd
    if "types" in expect:
        assert [cat[t].name for t in cmd.type_ids] == expect["types"]
    if "reservation" in expect:
        reqs = req_lines(cmd.requirements)
        assert reqs[RESERVATION_ID] == (False, [expect["reservation"]])
        assert cmd.n_reserved == 1


SCENARIOS = {"reserved_into": reserved_into, "reserved_between": reserved_between}


def shared_identity_cluster(golden, pending_a, selection=False):
    """Two m5.2xlarge nodes (1a, 1b), each a candidate holding one pod of test_topology_cpu.shared_filter_problem's
    Deployments (one spread identity, Honor filters zone In [1a, 1b] vs [1b, 1c]); a third node (1c) with room.  Each
    single-node probe's NewTopology sees only its own candidate's pod (and the pending pods), so without a pending pod
    the two probes create the group from different owners: kp_consolidate refuses that.  pending_a adds a pending pod
    of A's Deployment, which every probe sees first.  Without one, each probe starts with its own first owner's variant
    group born (kp_consolidate_prepare).  selection: A's selector is app In [web] twice — hashstructure folds the pair
    away (SlicesAsSets XOR), so it hashes like B's empty selector, which also selects a third class (app=db): one
    identity, two selections, which variant groups do not cover — refused."""
    import test_topology_cpu as TC
    prob = TC.shared_filter_problem(golden, True)
    if selection:
        web = model.Requirement("app", "In", ["web"])
        prob.classes[0].topology = [model.TopologyTerm("spread", model.ZONE, [web, web], max_skew=1)]
        prob.classes[1].topology = [model.TopologyTerm("spread", model.ZONE, [], max_skew=1)]
        prob.classes.append(model.PodClass(labels={"app": "db"}))
    it = golden[row(golden, "m5.2xlarge")]
    specs = [(0, {"cpu": "1", "memory": "1Gi"}), (1, {"cpu": "1", "memory": "1Gi"})]
    if pending_a:
        specs.append((0, {"cpu": "1", "memory": "1Gi"}))
    pods = synth.pods_from_specs(specs)
    nodes, cands = [], []
    for j, zone in enumerate(["test-zone-1a", "test-zone-1b", "test-zone-1c"]):
        labels = synth.node_labels(it, zone, "on-demand", "default")
        avail = np.array(it.allocatable, np.int64) - (pods.requests[j] if j < 2 else 0)
        nodes.append(model.ExistingNode("node-%d" % j, labels, avail, np.zeros(model.R, np.int64)))
        if j < 2:
            cands.append(model.Candidate(node=j, pods=np.array([j], np.int32), price=synth.candidate_price(it, labels),
                                         capacity_type=abi.KP_CT_ON_DEMAND, instance_type=row(golden, "m5.2xlarge"),
                                         nodepool=0, capacity=np.array(it.capacity, np.int64)))
    cluster = model.Problem(golden, prob.nodepools, prob.classes, pods, nodes)
    pending = np.array([2] if pending_a else [], np.int32)
    return model.ConsolidationProblem(cluster, cands, pending, np.ones(3, np.uint8))
