"""CPU: the oracle's restatement of [core] topology (scheduling/topology.go, topologygroup.go) against the reference's
own expectations and hand-computed cases.

Reference-pinned cases (e2e suites; the core module itself is not vendored):
  * test/suites/scheduling/suite_test.go:443-470   three pods, zonal spread maxSkew 1 minDomains 3 → three nodes
  * test/suites/scheduling/suite_test.go:421-442   two pods with hostname self-affinity → one node
  * test/suites/scale/provisioning_test.go:76-122  node-dense: 500 pods with hostname anti-affinity → 500 nodes
  * test/suites/scale/provisioning_test.go:123-178 the same with minValues 30 on instance-type → 500 nodes
  * test/suites/scale/provisioning_test.go:179-214 pod-dense: 6,600 pods, maxPods 110 + DaemonSets, size large → 60
"""
import copy

import numpy as np
import pytest

import pyoracle
from kpsim import abi, model, synth
from kpsim.model import HOSTNAME, ZONE, PodClass, Requirement, TopologyTerm

AWS = "karpenter.k8s.aws/"


def solve(prob, **kw):
    o = pyoracle.solve(prob, **kw)
    reqs = [model.parse_requirements_blob(o.requirements(i)) for i in range(o.results.n_nodeclaims)]
    return o.results, reqs


def deployment(n, labels, terms, cpu="10m", mem="50Mi", requirements=()):
    pc = PodClass(list(requirements), labels=dict(labels), topology=list(terms))
    return pc, synth.pods_from_specs([(0, {"cpu": cpu, "memory": mem})] * n)


def sel(labels):
    return [Requirement(k, "In", [v]) for k, v in labels.items()]


def zone_of(reqs):
    z = reqs.get(ZONE)
    return z[4] if z and not z[0] else None


def test_zonal_spread_three_nodes(golden):
    """scheduling/suite_test.go:443-470: one pod per zone, three NodeClaims (one zone each)."""
    lab = {"test": "zonal-spread"}
    pc, pods = deployment(3, lab, [TopologyTerm("spread", ZONE, sel(lab), max_skew=1, min_domains=3)])
    r, q = solve(model.Problem(golden, [synth.default_nodepool()], [pc], pods))
    assert r.n_nodeclaims == 3 and (r.pod_result >= 0).all()
    assert sorted(zone_of(x) for x in q) == [("test-zone-1a",), ("test-zone-1b",), ("test-zone-1c",)]


def test_self_affinity_one_node(golden):
    """scheduling/suite_test.go:421-442: two pods with hostname self-affinity land on one NodeClaim."""
    lab = {"test": "self-affinity"}
    pc, pods = deployment(2, lab, [TopologyTerm("affinity", HOSTNAME, sel(lab))])
    r, _ = solve(model.Problem(golden, [synth.default_nodepool()], [pc], pods))
    assert r.n_nodeclaims == 1 and list(r.nodeclaim_n_pods) == [2]


def e2e_nodepool(min_values=None):
    reqs = [Requirement(AWS + "instance-category", "In", ["c", "m", "r"]),
            Requirement(AWS + "instance-generation", "Gt", ["2"])]
    if min_values:
        reqs.append(Requirement(model.INSTANCE_TYPE, "Exists", [], min_values=min_values))
    return synth.default_nodepool(requirements=reqs)


@pytest.mark.parametrize("min_values", [None, 30])
def test_node_dense_hostname_anti_affinity(golden, min_values):
    """scale/provisioning_test.go:76-178: 500 replicas with hostname anti-affinity → 500 NodeClaims, one pod each."""
    lab = {"app": "node-dense"}
    pc, pods = deployment(500, lab, [TopologyTerm("anti", HOSTNAME, sel(lab))])
    r, _ = solve(model.Problem(golden, [e2e_nodepool(min_values)], [pc], pods))
    assert r.n_nodeclaims == 500 and (r.nodeclaim_n_pods == 1).all() and (r.pod_result >= 0).all()
    if min_values:
        assert all(len(ts) >= 30 for ts in r.nodeclaim_types)


def test_pod_dense_sixty_nodes(golden):
    """scale/provisioning_test.go:179-214: 60 × 110 pods (10m / 50Mi), kubelet maxPods = 110 + DaemonSet count, sizes
    `large` only → 60 NodeClaims of 110 pods (maxPods is the binding axis: types.go pods() returns maxPods)."""
    ds = 3
    cat = copy.deepcopy(golden)
    for it in cat:
        it.capacity[model.RIDX["pods"]] = (110 + ds) * 1000
        it.allocatable[model.RIDX["pods"]] = (110 + ds) * 1000
    daemon = np.zeros(model.R, np.int64)
    daemon[model.RIDX["cpu"]] = 150
    daemon[model.RIDX["memory"]] = 200 * 2 ** 20 * 1000
    daemon[model.RIDX["pods"]] = ds * 1000
    np_ = synth.default_nodepool(requirements=[Requirement(AWS + "instance-size", "In", ["large"])],
                                 daemon_overhead=daemon)
    pods = synth.pods_from_specs([(0, {"cpu": "10m", "memory": "50Mi"})] * 6600)
    r, _ = solve(model.Problem(cat, [np_], [PodClass()], pods))
    assert r.n_nodeclaims == 60 and (r.nodeclaim_n_pods == 110).all()


def test_hostname_spread_max_skew_two(golden):
    """Hostname spread: domainMinCount is 0 for hostname keys, so maxSkew 2 allows two selected pods per node."""
    lab = {"app": "h"}
    pc, pods = deployment(10, lab, [TopologyTerm("spread", HOSTNAME, sel(lab), max_skew=2)])
    r, _ = solve(model.Problem(golden, [synth.default_nodepool()], [pc], pods))
    assert r.n_nodeclaims == 5 and (r.nodeclaim_n_pods == 2).all()


def _bound_zone_problem(golden, n_pending):
    """Two existing nodes in test-zone-1a carrying two bound pods of the class; pending pods spread over the zones."""
    lab = {"app": "z"}
    pc, pods = deployment(n_pending, lab, [TopologyTerm("spread", ZONE, sel(lab), max_skew=1)])
    it = golden[0]
    nodes = []
    for j in range(2):
        labels = synth.node_labels(it, "test-zone-1a", "on-demand", "default")
        avail = np.zeros(model.R, np.int64)  # full: pending pods cannot land here
        nodes.append(model.ExistingNode("node-%d" % j, labels, avail))
    return model.Problem(golden, [synth.default_nodepool()], [pc], pods, nodes, bound=[(0, 0), (1, 0)])


def test_zonal_spread_counts_bound_pods(golden):
    """countDomains: two bound pods in 1a.  Pending pods go to 1b, then 1c (1a is 2 ahead), then join the 1b and 1c
    NodeClaims in slice order as the minimum rises: two NodeClaims of two pods, zones 1b and 1c."""
    r, q = solve(_bound_zone_problem(golden, 4))
    assert r.n_nodeclaims == 2 and list(r.nodeclaim_n_pods) == [2, 2]
    assert [zone_of(x) for x in q] == [("test-zone-1b",), ("test-zone-1c",)]


def test_anti_affinity_inverse_group(golden):
    """updateInverseAntiAffinity: pod A (app=a, anti-affinity to app=b on hostname) is placed first (larger cpu); the
    app=b pods, which carry no terms themselves, may not join A's node and share a second NodeClaim."""
    a = PodClass(labels={"app": "a"}, topology=[TopologyTerm("anti", HOSTNAME, sel({"app": "b"}))])
    b = PodClass(labels={"app": "b"})
    pods = synth.pods_from_specs([(0, {"cpu": "2", "memory": "1Gi"}), (1, {"cpu": "1", "memory": "1Gi"}),
                                  (1, {"cpu": "1", "memory": "1Gi"})])
    r, _ = solve(model.Problem(golden, [synth.default_nodepool()], [a, b], pods))
    assert r.n_nodeclaims == 2 and list(r.pod_result) == [0, 1, 1]


def test_zonal_anti_affinity_blocks_every_possible_zone(golden):
    """Zonal self anti-affinity on a NodeClaim whose zone is not pinned: AddRequirements narrows it to the empty zones
    (all three) and Record blocks out every zone the pod could land in (topology.go Record, anti-affinity branch), so
    the other replicas find no empty zone in this Solve."""
    lab = {"app": "za"}
    pc, pods = deployment(4, lab, [TopologyTerm("anti", ZONE, sel(lab))])
    r, q = solve(model.Problem(golden, [synth.default_nodepool()], [pc], pods))
    assert r.n_nodeclaims == 1 and int((r.pod_result == -1).sum()) == 3
    assert zone_of(q[0]) == ("test-zone-1a", "test-zone-1b", "test-zone-1c")


def test_zonal_anti_affinity_pinned_zones(golden):
    """With the zone pinned per replica (a zone nodeSelector per class, same anti-affinity selector), each zone holds
    one replica and a second replica for an occupied zone is unschedulable."""
    lab = {"app": "za"}
    term = TopologyTerm("anti", ZONE, sel(lab))
    classes = [PodClass([Requirement(ZONE, "In", [z])], labels=lab, topology=[term])
               for z in ("test-zone-1a", "test-zone-1b", "test-zone-1c", "test-zone-1a")]
    pods = synth.pods_from_specs([(c, {"cpu": "1", "memory": "1Gi"}) for c in range(4)])
    r, q = solve(model.Problem(golden, [synth.default_nodepool()], classes, pods))
    assert r.n_nodeclaims == 3 and list(r.pod_result) == [0, 1, 2, -1]


def test_spread_selecting_another_class(golden):
    """A spread whose selector matches a different class: the selected pods (no terms of their own) are counted where
    they land.  The owner does not select itself (no +1): with one web pod in 1a it may still join 1a's NodeClaim
    (1 - 0 <= 1); with two it may not (2 - 0 > 1) and opens a NodeClaim in the emptiest zone, 1b by name."""
    other = PodClass(labels={"app": "web"}, requirements=[Requirement(ZONE, "In", ["test-zone-1a"])])
    owner = PodClass(labels={"app": "probe"}, topology=[TopologyTerm("spread", ZONE, sel({"app": "web"}), max_skew=1)])
    for n_web, want in ((1, 1), (2, 2)):
        pods = synth.pods_from_specs([(0, {"cpu": "2", "memory": "1Gi"})] * n_web + [(1, {"cpu": "1", "memory": "1Gi"})])
        r, q = solve(model.Problem(golden, [synth.default_nodepool()], [other, owner], pods))
        assert r.n_nodeclaims == want
        assert zone_of(q[r.pod_result[-1]]) == (("test-zone-1a",) if want == 1 else ("test-zone-1b",))


def test_preferences_respect_spreads_ignore_drops(golden):
    """ScheduleAnyway spreads are preferences: PREFERENCE_POLICY=Ignore drops them (same result as no term); Respect
    treats them as DoNotSchedule until relaxed (one pod per NodeClaim here, every NodeClaim unconstrained)."""
    lab = {"app": "p"}
    pc, pods = deployment(6, lab, [TopologyTerm("spread", HOSTNAME, sel(lab), when_unsatisfiable="ScheduleAnyway")])
    prob = model.Problem(golden, [synth.default_nodepool()], [pc], pods)
    resp, _ = solve(prob)
    assert resp.n_nodeclaims == 6 and (resp.pod_result >= 0).all()
    ign, _ = solve(prob, preference_policy=abi.KP_PREFERENCE_IGNORE)
    plain, _ = solve(model.Problem(golden, [synth.default_nodepool()], [PodClass(labels=lab)], pods))
    np.testing.assert_array_equal(ign.pod_result, plain.pod_result)


def test_config3_small_runs(golden):
    """config 3's generator (five weighted NodePools with limits, topology terms) on a 2,000-pod sample: every
    hostname-constrained class has at most one pod per NodeClaim and zonal-spread classes stay within skew 1 over
    the zones they use (computed from the NodeClaim zone requirements)."""
    prob = synth.subsample(synth.config3(catalog=golden), 2000)
    r, q = solve(prob)
    assert r.n_nodeclaims > 0
    cls = prob.pods.class_id
    for c, pc in enumerate(prob.classes):
        placed = np.nonzero((cls == c) & (r.pod_result >= 0))[0]
        if any(t.key == HOSTNAME for t in pc.topology):
            assert len(set(r.pod_result[placed].tolist())) == len(placed)


def node_dense(cat, n_pods):
    """The scale suite's node-dense Deployment (test/suites/scale/provisioning_test.go:76-136: hostname anti-affinity on
    its own label) at n_pods: one NodeClaim per pod.  At 10k it exceeds the FFD kernel's first slice plan (KP_NC_FIRST);
    tests/golden/gen_scale_digest.py node_dense_10k holds the oracle's digest of it."""
    lab = {"app": "node-dense"}
    pc, pods = deployment(n_pods, lab, [model.TopologyTerm("anti", model.HOSTNAME, sel(lab))])
    return model.Problem(cat, [e2e_nodepool(None)], [pc], pods)


# ---- one group per TopologyGroup.Hash() identity: the first owner's node filter and minDomains ([core] topology.go
# Update keeps topologyGroups[hash]; hashstructure skips Requirement values and minDomains, topologygroup.go Hash) ----

def _web_spread(min_domains=None):
    lab = {"app": "web"}
    return lab, TopologyTerm("spread", ZONE, sel(lab), max_skew=1, min_domains=min_domains, node_affinity_policy="Honor")


def shared_filter_problem(golden, a_first):
    """Two Deployments share an app label and a zonal spread (website scheduling.md:347-372), one pinned to zones 1a/1b,
    the other to 1b/1c, under nodeAffinityPolicy Honor: one identity, two node filters.  A's pods (2 cpu) are
    scheduled before B's (1 cpu) either way; a_first puts A's pods first in the input (NewTopology's order)."""
    lab, term = _web_spread()
    a = PodClass([Requirement(ZONE, "In", ["test-zone-1a", "test-zone-1b"])], labels=lab, topology=[term])
    b = PodClass([Requirement(ZONE, "In", ["test-zone-1b", "test-zone-1c"])], labels=lab, topology=[term])
    pa, pb = [(0, {"cpu": "2", "memory": "1Gi"})] * 3, [(1, {"cpu": "1", "memory": "1Gi"})] * 3
    pods = synth.pods_from_specs(pa + pb if a_first else pb + pa)
    return model.Problem(golden, [synth.default_nodepool()], [a, b], pods)


def shared_min_domains_problem(golden, a_first):
    """Two Deployments with one zonal spread identity, A's with minDomains 4 (more than the 3 zones: the global
    minimum counts as 0, faq.md:180-182), B's without; A's pods (2 cpu) schedule first."""
    lab, _ = _web_spread()
    a = PodClass(labels=lab, topology=[_web_spread(4)[1]])
    b = PodClass(labels=lab, topology=[_web_spread()[1]])
    pa, pb = [(0, {"cpu": "2", "memory": "1Gi"})] * 2, [(1, {"cpu": "1", "memory": "1Gi"})] * 3
    pods = synth.pods_from_specs(pa + pb if a_first else pb + pa)
    return model.Problem(golden, [synth.default_nodepool()], [a, b], pods)


# hand-derived placements (pod_result in input order, NodeClaim zones in creation order):
# filter A {1a,1b}: A → 1a, 1b (1a is 1 ahead), 1a; B pods land in 1c and are never counted (A's filter excludes 1c),
#   so 1b stays one ahead of 1c and all three B pods share the 1c NodeClaim.
# filter B {1b,1c}: A's pods in 1a are never counted, so all three share the 1a NodeClaim; B → 1b, 1c, then 1b again.
SHARED_FILTER_WANT = {
    True: ([0, 1, 0, 2, 2, 2], ["test-zone-1a", "test-zone-1b", "test-zone-1c"]),
    False: ([1, 2, 1, 0, 0, 0], ["test-zone-1a", "test-zone-1b", "test-zone-1c"]),
}
# minDomains 4 (A first): every zone may hold one selected pod (min is 0 with 3 < 4 domains) → A 1a, A 1b, B 1c, then
#   two B pods unschedulable.  No minDomains (B first): A 1a, A 1b, B 1c, then B joins the first NodeClaims in slice order.
SHARED_MIN_DOMAINS_WANT = {
    True: [0, 1, 2, -1, -1],
    False: [2, 0, 1, 0, 1],
}


@pytest.mark.parametrize("a_first", [True, False])
def test_shared_identity_first_owner_filter(golden, a_first):
    r, q = solve(shared_filter_problem(golden, a_first))
    want, zones = SHARED_FILTER_WANT[a_first]
    assert list(r.pod_result) == want
    assert [zone_of(x) for x in q] == [(z,) for z in zones]


@pytest.mark.parametrize("a_first", [True, False])
def test_shared_identity_first_owner_min_domains(golden, a_first):
    r, _ = solve(shared_min_domains_problem(golden, a_first))
    assert list(r.pod_result) == SHARED_MIN_DOMAINS_WANT[a_first]


def relaxed_only_shared_problem(golden, a_big=True):
    """Two Deployments with ORed required node-affinity terms whose first term no type satisfies: after Relax drops it,
    each spread's node filter is its second term, zone In [1a, 1b] vs zone In [1b, 1c] — one identity that only relaxed
    pods create, with two filters.  Topology.Update creates it from whichever pod relaxes first: the bigger pods (2 cpu)
    pop and relax first, A's when a_big (the device keeps one variant group per filter and births the first one)."""
    lab, term = _web_spread()
    nothing = [Requirement(AWS + "instance-category", "In", ["zz"])]
    a = PodClass(labels=lab, topology=[term],
                 required_terms=[nothing, [Requirement(ZONE, "In", ["test-zone-1a", "test-zone-1b"])]])
    b = PodClass(labels=lab, topology=[term],
                 required_terms=[nothing, [Requirement(ZONE, "In", ["test-zone-1b", "test-zone-1c"])]])
    big, small = {"cpu": "2", "memory": "1Gi"}, {"cpu": "1", "memory": "1Gi"}
    pods = synth.pods_from_specs([(0, big if a_big else small)] * 3 + [(1, small if a_big else big)] * 3)
    return model.Problem(golden, [synth.default_nodepool()], [a, b], pods)


# A relaxes first: A's filter {1a,1b} (as SHARED_FILTER_WANT[True]).  B relaxes first: B's filter {1b,1c}; B → 1b, 1c,
# 1b; A's pods in 1a are never counted, so all three share a 1a NodeClaim.
RELAXED_ONLY_WANT = {True: [0, 1, 0, 2, 2, 2], False: [2, 2, 2, 0, 1, 0]}


@pytest.mark.parametrize("a_big", [True, False])
def test_relaxed_only_shared_identity_oracle(golden, a_big):
    """The oracle creates the relaxed identity from the first pod that relaxes into it (Solver::birth)."""
    r, _ = solve(relaxed_only_shared_problem(golden, a_big))
    assert list(r.pod_result) == RELAXED_ONLY_WANT[a_big]
