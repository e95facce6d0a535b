"""Preference relaxation (PREFERENCE_POLICY) and MIN_VALUES_POLICY=BestEffort cases, shared by the CPU (oracle) and
GPU (device) tests.  Each case is a Solve problem + the solver parameters + a check of the values the semantics fix.

Pinned by the reference where it holds an answer:
  * test/suites/scheduling/suite_test.go:107-133 and :134-200 — pods whose nodeSelector / required node affinity are
    repeated as preferred terms schedule onto one node;
  * test/suites/scheduling/suite_test.go:366-400 — a NodePool `instance-type In [c5.large, invalid-1, invalid-2]`
    with minValues 3: Strict leaves the pod pending with no NodeClaim; BestEffort creates one NodeClaim whose
    instance-type requirement is In [c5.large] with minValues relaxed to 1.
The relaxation order and the Queue.Push(pod, relaxed) semantics are [core] scheduling/preferences.go and queue.go,
recalled (not vendored); those cases are hand-computed from that restatement ("parity unpinned" beyond the oracle).
"""
from dataclasses import dataclass, field

import numpy as np
from typing import Callable, List

from kpsim import abi, catalog, model, synth
from kpsim.model import INSTANCE_TYPE, ZONE, PodClass, Requirement, Taint, Toleration, TopologyTerm

import kat_cases as KC

HOST = model.HOSTNAME
Z1A, Z1B, Z1C = "test-zone-1a", "test-zone-1b", "test-zone-1c"


@dataclass
class PrefCase:
    name: str
    ref: str
    problem: model.Problem
    check: Callable                      # check(problem, results, nodeclaim requirements)
    preference_policy: int = abi.KP_PREFERENCE_RESPECT
    opts: dict = field(default_factory=dict)


CASES: List[Callable] = []


def case(fn):
    CASES.append(fn)
    return fn


def ids():
    return [f.__name__ for f in CASES]


def _prob(cat, nps, classes, specs, **kw):
    p = model.Problem(cat, nps, classes, synth.pods_from_specs(specs))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _scheduled(res):
    assert (res.pod_result >= 0).all(), res.pod_result


@case
def e2e_preferences_repeat_selector(fx):
    """scheduling/suite_test.go:107-133: nodeSelector = required = preferred node affinity → one node."""
    cat = catalog.fake_catalog(fx=fx)
    reqs = KC.sel_map(KC.G4DN_LABELS)
    pc = PodClass(KC.sel_map(KC.G4DN_LABELS), required_terms=[reqs], preferred_terms=[(1, reqs)])
    prob = _prob(cat, [synth.default_nodepool()], [pc], [(0, {})])

    def check(prob, res, q):
        _scheduled(res)
        assert res.n_nodeclaims == 1
        assert KC.names(cat, res.nodeclaim_types[0]) == ["g4dn.8xlarge"]
    return PrefCase("e2e_preferences_repeat_selector", "test/suites/scheduling/suite_test.go:107-133", prob, check)


@case
def e2e_preferred_gt(fx):
    """scheduling/suite_test.go:150-172: instance-local-nvme Gt 0 both preferred and required → one node with nvme."""
    cat = catalog.fake_catalog(fx=fx)
    r = [Requirement(KC.AWS + "instance-local-nvme", "Gt", ["0"])]
    pc = PodClass([], required_terms=[r], preferred_terms=[(1, r)])
    prob = _prob(cat, [synth.default_nodepool()], [pc], [(0, {})])

    def check(prob, res, q):
        _scheduled(res)
        assert res.n_nodeclaims == 1
        for t in res.nodeclaim_types[0]:
            assert int(cat[t].labels[KC.AWS + "instance-local-nvme"][0]) > 0
    return PrefCase("e2e_preferred_gt", "test/suites/scheduling/suite_test.go:150-172", prob, check)


@case
def preferred_unsatisfiable_relaxed(fx):
    """A preferred node-affinity term no type satisfies: the pod fails, Relax drops the term, the pod schedules and its
    NodeClaim carries no trace of the preference."""
    cat = catalog.fake_catalog(fx=fx)
    pc = PodClass([], preferred_terms=[(10, [Requirement(INSTANCE_TYPE, "In", ["no-such-type"])])])
    prob = _prob(cat, [synth.default_nodepool()], [pc], [(0, {"cpu": "1"})] * 3)

    def check(prob, res, q):
        _scheduled(res)
        assert res.n_nodeclaims == 1
        assert INSTANCE_TYPE not in q[0] or "no-such-type" not in q[0][INSTANCE_TYPE][4]
    return PrefCase("preferred_unsatisfiable_relaxed", "[core] preferences.go removePreferredNodeAffinityTerm", prob, check)


@case
def heaviest_preference_first(fx):
    """newPodRequirements treats the heaviest preferred term as required: zone 1b (weight 50) over zone 1a (weight 1)."""
    cat = catalog.fake_catalog(fx=fx)
    pc = PodClass([], preferred_terms=[(1, [Requirement(ZONE, "In", [Z1A])]), (50, [Requirement(ZONE, "In", [Z1B])])])
    prob = _prob(cat, [synth.default_nodepool()], [pc], [(0, {"cpu": "1"})])

    def check(prob, res, q):
        _scheduled(res)
        assert q[0][ZONE][4] == (Z1B,)
    return PrefCase("heaviest_preference_first", "[core] scheduling/requirements.go newPodRequirements", prob, check)


@case
def required_terms_relaxed_in_order(fx):
    """Required node-affinity terms are ORed: the first (no such type) fails, Relax removes it, the second (zone 1c)
    places the pod."""
    cat = catalog.fake_catalog(fx=fx)
    pc = PodClass([], required_terms=[[Requirement(INSTANCE_TYPE, "In", ["no-such-type"])],
                                      [Requirement(ZONE, "In", [Z1C])]])
    prob = _prob(cat, [synth.default_nodepool()], [pc], [(0, {"cpu": "1"})])

    def check(prob, res, q):
        _scheduled(res)
        assert q[0][ZONE][4] == (Z1C,)
    return PrefCase("required_terms_relaxed_in_order", "[core] preferences.go removeRequiredNodeAffinityTerm", prob, check)


def _self_terms(kind, **kw):
    return [TopologyTerm(kind, HOST, selector=[Requirement("app", "In", ["web"])], **kw)]


@case
def schedule_anyway_spread_respected(fx):
    """A ScheduleAnyway hostname spread (maxSkew 1) is honoured while it can be: three pods, three NodeClaims."""
    cat = catalog.fake_catalog(fx=fx)
    pc = PodClass([], labels={"app": "web"}, topology=_self_terms("spread", when_unsatisfiable="ScheduleAnyway"))
    prob = _prob(cat, [synth.default_nodepool()], [pc], [(0, {"cpu": "1"})] * 3)

    def check(prob, res, q):
        _scheduled(res)
        assert res.n_nodeclaims == 3
    return PrefCase("schedule_anyway_spread_respected", "[core] topology.go newForTopologies (Respect)", prob, check)


@case
def schedule_anyway_spread_ignored(fx):
    """PREFERENCE_POLICY=Ignore drops the ScheduleAnyway spread: one NodeClaim for the three pods."""
    c = schedule_anyway_spread_respected(fx)

    def check(prob, res, q):
        _scheduled(res)
        assert res.n_nodeclaims == 1
    return PrefCase("schedule_anyway_spread_ignored", "settings.md:40 PREFERENCE_POLICY", c.problem, check,
                    preference_policy=abi.KP_PREFERENCE_IGNORE)


@case
def preferred_anti_affinity_relaxed_at_limit(fx):
    """Preferred hostname anti-affinity is required until relaxed: the NodePool's cpu limit admits one m5.large, so
    pods 2 and 3 fail, drop the term (Relax) and join the first NodeClaim."""
    cat = catalog.fake_catalog(fx=fx)
    m5 = [i for i, it in enumerate(cat) if it.name == "m5.large"]
    np_ = synth.default_nodepool(instance_types=m5, limits_remaining={"cpu": 3000})
    pc = PodClass([], labels={"app": "web"}, topology=_self_terms("anti", weight=10))
    prob = _prob(cat, [np_], [pc], [(0, {"cpu": "100m"})] * 3)

    def check(prob, res, q):
        _scheduled(res)
        assert res.n_nodeclaims == 1 and int(res.nodeclaim_n_pods[0]) == 3
    return PrefCase("preferred_anti_affinity_relaxed_at_limit", "[core] preferences.go removePreferredPodAntiAffinityTerm",
                    prob, check)


@case
def prefer_no_schedule_tolerated_after_relax(fx):
    """A NodePool tainted PreferNoSchedule: the pod does not tolerate it, fails, and Relax adds the PreferNoSchedule
    toleration (toleratePreferNoSchedule is on because a NodePool carries such a taint)."""
    cat = catalog.fake_catalog(fx=fx)
    np_ = synth.default_nodepool(taints=[Taint("example.com/soft", "", "PreferNoSchedule")])
    prob = _prob(cat, [np_], [PodClass([])], [(0, {"cpu": "1"})] * 2)

    def check(prob, res, q):
        _scheduled(res)
        assert res.n_nodeclaims == 1
    return PrefCase("prefer_no_schedule_tolerated_after_relax", "[core] preferences.go toleratePreferNoScheduleTaints",
                    prob, check)


@case
def prefer_no_schedule_already_tolerated(fx):
    """The same NodePool, a pod that already tolerates PreferNoSchedule taints: scheduled without relaxation."""
    c = prefer_no_schedule_tolerated_after_relax(fx)
    c.problem.classes = [PodClass([], tolerations=[Toleration("", "Exists", "", "PreferNoSchedule")])]
    return PrefCase("prefer_no_schedule_already_tolerated", c.ref, c.problem, c.check)


@case
def preferred_zone_term_strict_pod_domains(fx):
    """A preferred zone term on a zone spread's key: the NodeClaim's requirements take the preference (zone In [1a]) but
    podDomains come from the strict requirements (NewStrictPodRequirements: every zone), so the skew counts the empty
    zones.  Pod 1 lands in 1a; pods 2-3 see 1a at skew 2, fail, drop the preference and open 1b and 1c; pod 4 (skew 1
    again) joins 1a.  Pod domains taken from the preference would put all four pods in 1a."""
    cat = catalog.fake_catalog(fx=fx)
    pc = PodClass([], labels={"app": "web"},
                  topology=[TopologyTerm("spread", ZONE, selector=[Requirement("app", "In", ["web"])])],
                  preferred_terms=[(10, [Requirement(ZONE, "In", [Z1A])])])
    prob = _prob(cat, [synth.default_nodepool()], [pc], [(0, {"cpu": "100m"})] * 4)

    def check(prob, res, q):
        _scheduled(res)
        assert res.n_nodeclaims == 3
        assert sorted(q[i][ZONE][4] for i in range(3)) == [(Z1A,), (Z1B,), (Z1C,)]
        assert sorted(int(n) for n in res.nodeclaim_n_pods[:3]) == [1, 1, 2]
    return PrefCase("preferred_zone_term_strict_pod_domains", "[core] nodeclaim.go CanAdd (podData.StrictRequirements)",
                    prob, check)


@case
def honor_spread_filter_ignores_preference(fx):
    """nodeAffinityPolicy Honor with a preferred node-affinity term: MakeTopologyNodeFilter takes the nodeSelector and
    the required terms only, so two bound pods on t3.large nodes in zone 1a count although the pod prefers m5.large; the
    pod's NodeClaim (m5.large by preference) avoids 1a.  A filter carrying the preference would count nothing there and
    pick 1a (smallest domain name)."""
    cat = catalog.fake_catalog(fx=fx)
    t3 = next(it for it in cat if it.name == "t3.large")
    sel = [Requirement("app", "In", ["web"])]
    pc = PodClass([], labels={"app": "web"}, topology=[TopologyTerm("spread", ZONE, selector=sel)],
                  preferred_terms=[(10, [Requirement(INSTANCE_TYPE, "In", ["m5.large"])])])
    nodes = [model.ExistingNode("t3-%d" % j, synth.node_labels(t3, Z1A, "on-demand"), np.zeros(model.R, np.int64))
             for j in range(2)]
    prob = _prob(cat, [synth.default_nodepool()], [pc], [(0, {"cpu": "100m"})], existing=nodes, bound=[(0, 0), (1, 0)])

    def check(prob, res, q):
        _scheduled(res)
        assert res.n_nodeclaims == 1
        assert q[0][ZONE][4] == (Z1B,)
        assert q[0][INSTANCE_TYPE][4] == ("m5.large",)
    return PrefCase("honor_spread_filter_ignores_preference", "[core] topologynodefilter.go MakeTopologyNodeFilter",
                    prob, check)


@case
def relaxed_spec_spread_group_created_late(fx):
    """Topology.Update creates the spread group of a relaxed spec (its node filter keeps the remaining required terms,
    so it hashes apart from the first spec's group) when the first pod relaxes, counting only bound pods from then on.
    Required terms [t3.large] | [m5.large, amd64], zone spread (maxSkew 1, nodeAffinityPolicy Ignore): pods 1-2 take
    t3.large in 1a / 1b; pods 3-4 cannot reach 1c with t3.large, relax, and the new group (empty) spreads them over
    m5.large in 1a then 1b.  A group counting since the start would send pod 3 to 1c and pod 4 after it (3 NodeClaims)."""
    cat = catalog.fake_catalog(fx=fx)
    sel = [Requirement("app", "In", ["web"])]
    pc = PodClass([], labels={"app": "web"},
                  topology=[TopologyTerm("spread", ZONE, selector=sel, node_affinity_policy="Ignore")],
                  required_terms=[[Requirement(INSTANCE_TYPE, "In", ["t3.large"])],
                                  [Requirement(INSTANCE_TYPE, "In", ["m5.large"]), Requirement(model.ARCH, "In", ["amd64"])]])
    prob = _prob(cat, [synth.default_nodepool()], [pc], [(0, {"cpu": "100m"})] * 4)

    def check(prob, res, q):
        _scheduled(res)
        assert res.n_nodeclaims == 4
        got = sorted((q[i][INSTANCE_TYPE][4], q[i][ZONE][4]) for i in range(4))
        assert got == [(("m5.large",), (Z1A,)), (("m5.large",), (Z1B,)), (("t3.large",), (Z1A,)), (("t3.large",), (Z1B,))], got
    return PrefCase("relaxed_spec_spread_group_created_late", "[core] topology.go Update (countDomains for a new hash)",
                    prob, check)


@case
def honor_spread_several_required_terms(fx):
    """nodeAffinityPolicy Honor with ORed required terms: the node filter matches a node compatible with ANY remaining
    term.  Two bound pods on t3.large nodes in 1a count for the spread of a pod whose first term (t3.large) fails;
    after Relax its spec's group is new (late) and also counts them (countDomains at creation), so the m5.large
    NodeClaim goes to 1b."""
    cat = catalog.fake_catalog(fx=fx)
    t3 = next(it for it in cat if it.name == "t3.large")
    sel = [Requirement("app", "In", ["web"])]
    pc = PodClass([], labels={"app": "web"}, topology=[TopologyTerm("spread", ZONE, selector=sel)],
                  required_terms=[[Requirement(INSTANCE_TYPE, "In", ["no-such-type"])],
                                  [Requirement(INSTANCE_TYPE, "In", ["m5.large", "t3.large"])]])
    nodes = [model.ExistingNode("t3-%d" % j, synth.node_labels(t3, Z1A, "on-demand"), np.zeros(model.R, np.int64))
             for j in range(2)]
    prob = _prob(cat, [synth.default_nodepool()], [pc], [(0, {"cpu": "100m"})], existing=nodes, bound=[(0, 0), (1, 0)])

    def check(prob, res, q):
        _scheduled(res)
        assert res.n_nodeclaims == 1
        assert q[0][ZONE][4] == (Z1B,)
    return PrefCase("honor_spread_several_required_terms", "[core] topologynodefilter.go MatchesRequirements", prob, check)


def _best_effort_problem(golden, policy):
    np_ = synth.default_nodepool(requirements=[Requirement(INSTANCE_TYPE, "In",
                                                           ["c5.large", "invalid-instance-type-1", "invalid-instance-type-2"],
                                                           min_values=3)])
    return _prob(golden, [np_], [PodClass([])], [(0, {})], min_values_policy=policy)


@case
def e2e_min_values_strict(fx):
    """scheduling/suite_test.go:386-400 (Strict): the pod stays pending, no NodeClaim."""
    golden = catalog.golden_catalog(fx=fx)

    def check(prob, res, q):
        assert res.n_nodeclaims == 0 and (res.pod_result == -1).all()
    return PrefCase("e2e_min_values_strict", "test/suites/scheduling/suite_test.go:366-400",
                    _best_effort_problem(golden, abi.KP_MIN_VALUES_STRICT), check)


@case
def e2e_min_values_best_effort(fx):
    """scheduling/suite_test.go:380-385 (BestEffort): one NodeClaim, instance-type In [c5.large] with minValues 1."""
    golden = catalog.golden_catalog(fx=fx)

    def check(prob, res, q):
        _scheduled(res)
        assert res.n_nodeclaims == 1
        assert KC.names(golden, res.nodeclaim_types[0]) == ["c5.large"]
        assert q[0][INSTANCE_TYPE][3] == "1", q[0][INSTANCE_TYPE]
    return PrefCase("e2e_min_values_best_effort", "test/suites/scheduling/suite_test.go:366-385",
                    _best_effort_problem(golden, abi.KP_MIN_VALUES_BEST_EFFORT), check)
