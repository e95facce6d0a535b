"""GPU: preference relaxation (PREFERENCE_POLICY) and MIN_VALUES_POLICY=BestEffort on the device (libkpsim), bit-exact
with the oracle: the cases of tests/pref_cases.py (their known answers asserted on the device result too) and seeded
fuzz problems that mix preferred / required node-affinity terms, ScheduleAnyway spreads, preferred pod
(anti-)affinity, PreferNoSchedule taints, NodePool limits and minValues."""
import numpy as np
import pytest

import parity
import pref_cases as PC
import pyoracle
from kpsim import abi, model, native, synth
from kpsim.model import PodClass, Requirement, Taint, TopologyTerm

pytestmark = pytest.mark.gpu


def _ctx(policy):
    return native.Context(0, preference_policy=policy)


def _oracle(prob, policy):
    o = pyoracle.solve(prob, preference_policy=policy)
    return o.results, [model.parse_requirements_blob(o.requirements(i)) for i in range(o.results.n_nodeclaims)]


@pytest.mark.parametrize("mk", PC.CASES, ids=PC.ids())
def test_pref_case_device(fx, mk):
    c = mk(fx)
    ctx = _ctx(c.preference_policy)
    try:
        dev = parity.run_device(ctx, c.problem)
    finally:
        ctx.close()
    parity.assert_same(dev, _oracle(c.problem, c.preference_policy))
    c.check(c.problem, dev[0], dev[1])


AWS = "karpenter.k8s.aws/"


def fuzz_problem(golden, seed):
    rng = np.random.Generator(np.random.PCG64(7000 + seed))
    prob = synth.subsample(synth.config2(catalog=golden, seed=synth.SEED + seed), int(rng.integers(300, 900)))
    cats = ["c", "m", "r", "t", "g", "i"]
    for ci, pc in enumerate(prob.classes):
        u = rng.random()
        lab = {"app": "a%d" % (ci % 40)}  # a handful of classes per selector (the device's per-class group limits)
        pc.labels.update(lab)
        if u < 0.25:
            pc.preferred_terms = [(int(rng.integers(1, 100)),
                                   [Requirement(AWS + "instance-category", "In",
                                                list(rng.choice(cats, size=int(rng.integers(1, 3)), replace=False)))])
                                  for _ in range(int(rng.integers(1, 4)))]
        elif u < 0.4:
            pc.required_terms = [[Requirement(AWS + "instance-category", "In", [str(rng.choice(cats))])],
                                 [Requirement("kubernetes.io/arch", "In", [str(rng.choice(["amd64", "arm64"]))])]]
        v = rng.random()
        if v < 0.2:
            pc.topology = [TopologyTerm("spread", model.HOSTNAME if rng.random() < 0.5 else model.ZONE,
                                        selector=[Requirement("app", "In", [lab["app"]])],
                                        max_skew=int(rng.integers(1, 3)), when_unsatisfiable="ScheduleAnyway",
                                        node_affinity_policy="Ignore")]
        elif v < 0.35:
            pc.topology = [TopologyTerm("anti", model.HOSTNAME, selector=[Requirement("app", "In", [lab["app"]])],
                                        weight=int(rng.integers(1, 100)))]
        elif v < 0.42:
            pc.topology = [TopologyTerm("affinity", model.ZONE, selector=[Requirement("app", "In", [lab["app"]])],
                                        weight=int(rng.integers(1, 100)))]
    if seed % 3 == 0:
        prob.nodepools[0].taints = list(prob.nodepools[0].taints) + [Taint("example.com/soft", "", "PreferNoSchedule")]
    if seed % 2 == 1:
        for np_ in prob.nodepools:
            np_.limits_remaining = {"cpu": int(rng.integers(40, 400)) * 1000}
    if seed % 4 == 2:
        prob.min_values_policy = abi.KP_MIN_VALUES_BEST_EFFORT
        prob.nodepools[0].requirements = list(prob.nodepools[0].requirements) + [
            Requirement(AWS + "instance-family", "Exists", [], min_values=int(rng.integers(20, 120)))]
    return prob


@pytest.mark.parametrize("seed", range(16))
def test_preference_fuzz(golden, seed):
    prob = fuzz_problem(golden, seed)
    for policy in (abi.KP_PREFERENCE_RESPECT, abi.KP_PREFERENCE_IGNORE):
        ctx = _ctx(policy)
        try:
            dev = parity.run_device(ctx, prob)
        finally:
            ctx.close()
        parity.assert_same(dev, _oracle(prob, policy))


@pytest.mark.parametrize("seed", list(range(12)) + [2058, 2233])  # + tools/soak.py topo_pref 58 / 233
def test_topology_preference_fuzz(golden, seed):
    """Preferred node-affinity terms on pods with topology terms over a cluster (fuzzgen.add_topology_preferences after
    fuzz_topology_existing_problem): preferences on the zone / capacity-type topology keys (podDomains from the strict
    requirements) and nodeAffinityPolicy Honor spreads whose node filter leaves the preference out."""
    import fuzzgen
    rng = np.random.Generator(np.random.PCG64(7300 + seed))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(80, 300)), replace=False))]
    prob = fuzzgen.fuzz_topology_existing_problem(sub, 7300 + seed, n_pods=int(rng.integers(100, 400)))
    fuzzgen.add_topology_preferences(rng, prob)
    assert any(pc.preferred_terms for pc in prob.classes)
    for policy in (abi.KP_PREFERENCE_RESPECT, abi.KP_PREFERENCE_IGNORE):
        ctx = _ctx(policy)
        try:
            dev = parity.run_device(ctx, prob)
        finally:
            ctx.close()
        parity.assert_same(dev, _oracle(prob, policy))


@pytest.mark.parametrize("seed", range(6))
def test_many_preferred_terms_fuzz(golden, seed):
    """More than 12 preferred node-affinity terms with tied weights: newPodRequirements' sort.Slice is Go's pdqsort
    (unstable), so which tied term is tried first follows its exact swap sequence (kp_gosort_host.h on the host,
    oracle/gosort.h in the oracle); Relax then walks that order."""
    rng = np.random.Generator(np.random.PCG64(7800 + seed))
    prob = synth.subsample(synth.config2(catalog=golden, seed=synth.SEED + seed), int(rng.integers(200, 600)))
    cats = ["c", "m", "r", "t", "g", "i", "x", "z"]
    zones = sorted({o.zone for it in golden for o in it.offerings})
    for pc in prob.classes:
        if rng.random() < 0.5:
            continue
        terms = []
        for _ in range(int(rng.integers(13, 40))):
            if rng.random() < 0.5:
                r = Requirement(AWS + "instance-category", "In", [str(rng.choice(cats))])
            else:
                r = Requirement(model.ZONE, "In", [str(rng.choice(zones))])
            terms.append((int(rng.choice([1, 5, 5, 10, 10, 10, 50])), [r]))
        pc.preferred_terms = terms
    ctx = _ctx(abi.KP_PREFERENCE_RESPECT)
    try:
        dev = parity.run_device(ctx, prob)
    finally:
        ctx.close()
    parity.assert_same(dev, _oracle(prob, abi.KP_PREFERENCE_RESPECT))


def relaxing_topology_problem(golden, seed):
    import fuzzgen
    rng = np.random.Generator(np.random.PCG64(7600 + seed))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(80, 300)), replace=False))]
    prob = fuzzgen.fuzz_topology_existing_problem(sub, 7600 + seed, n_pods=int(rng.integers(100, 400)))
    return fuzzgen.add_relaxing_topology(rng, prob)


@pytest.mark.parametrize("seed", range(12))
def test_relaxing_topology_fuzz(golden, seed):
    """Relaxations that change a spread group's TopologyGroup.Hash() (ORed required terms under both
    nodeAffinityPolicies, the PreferNoSchedule toleration): the relaxed spec's groups are created when the first pod
    relaxes into it and count only the bound pods until then (fuzzgen.add_relaxing_topology; seeds 6, 7 and 11 decide
    differently if those groups count from the start, ORC_NO_LATE)."""
    prob = relaxing_topology_problem(golden, seed)
    for policy in (abi.KP_PREFERENCE_RESPECT, abi.KP_PREFERENCE_IGNORE):
        ctx = _ctx(policy)
        try:
            dev = parity.run_device(ctx, prob)
        finally:
            ctx.close()
        parity.assert_same(dev, _oracle(prob, policy))


def test_repeated_execute_restores_classes(golden):
    """kp_solve_execute twice on one prepare: relaxed pods start again from their input classes."""
    prob = fuzz_problem(golden, 1)
    ctx = _ctx(abi.KP_PREFERENCE_RESPECT)
    try:
        a = parity.run_device(ctx, prob)
        ctx.execute()
        out = model.OutputBuffers(prob.pods.n, prob.pods.n + 16, (prob.pods.n + 16) * 60)
        ctx.fetch(out)
        b = out.results()
        np.testing.assert_array_equal(a[0].pod_result, b.pod_result)
        np.testing.assert_array_equal(a[0].pod_order, b.pod_order)
    finally:
        ctx.close()
