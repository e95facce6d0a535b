"""GPU: topology spread, pod affinity and anti-affinity on the device (topo_narrow / topo_record in csrc/kp_eval.h)
against the oracle's restatement of [core] topology.go — bit-exact, plus the reference's own expectations.

Reference-pinned: test/suites/scheduling/suite_test.go:421-470 (self-affinity → 1 node, zonal spread → 3 nodes) and
test/suites/scale/provisioning_test.go:76-214 (node-dense 500 nodes with and without minValues, pod-dense 60 nodes).
"""
import json
import os

import numpy as np
import pytest

import fuzzgen
import parity
from kpsim import abi, model, synth
import test_topology_cpu as TC

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from kpsim import native
    c = native.Context(0)
    yield c
    c.close()


def same(ctx, prob):
    dev = parity.run_device(ctx, prob)
    parity.assert_same(dev, parity.run_oracle(prob))
    return dev


def test_zonal_spread_three_nodes(ctx, golden):
    lab = {"test": "zonal-spread"}
    pc, pods = TC.deployment(3, lab, [model.TopologyTerm("spread", model.ZONE, TC.sel(lab), max_skew=1, min_domains=3)])
    r, q = same(ctx, model.Problem(golden, [synth.default_nodepool()], [pc], pods))
    assert r.n_nodeclaims == 3
    assert sorted(TC.zone_of(x) for x in q) == [("test-zone-1a",), ("test-zone-1b",), ("test-zone-1c",)]


def test_self_affinity_one_node(ctx, golden):
    lab = {"test": "self-affinity"}
    pc, pods = TC.deployment(2, lab, [model.TopologyTerm("affinity", model.HOSTNAME, TC.sel(lab))])
    r, _ = same(ctx, model.Problem(golden, [synth.default_nodepool()], [pc], pods))
    assert r.n_nodeclaims == 1


@pytest.mark.parametrize("min_values", [None, 30])
def test_node_dense(ctx, golden, min_values):
    lab = {"app": "node-dense"}
    pc, pods = TC.deployment(500, lab, [model.TopologyTerm("anti", model.HOSTNAME, TC.sel(lab))])
    r, _ = same(ctx, model.Problem(golden, [TC.e2e_nodepool(min_values)], [pc], pods))
    assert r.n_nodeclaims == 500 and (r.nodeclaim_n_pods == 1).all()


def test_hostname_spread_and_inverse_anti_affinity(ctx, golden):
    lab = {"app": "h"}
    pc, pods = TC.deployment(10, lab, [model.TopologyTerm("spread", model.HOSTNAME, TC.sel(lab), max_skew=2)])
    r, _ = same(ctx, model.Problem(golden, [synth.default_nodepool()], [pc], pods))
    assert r.n_nodeclaims == 5
    a = model.PodClass(labels={"app": "a"}, topology=[model.TopologyTerm("anti", model.HOSTNAME, TC.sel({"app": "b"}))])
    b = model.PodClass(labels={"app": "b"})
    pods = synth.pods_from_specs([(0, {"cpu": "2", "memory": "1Gi"}), (1, {"cpu": "1", "memory": "1Gi"}),
                                  (1, {"cpu": "1", "memory": "1Gi"})])
    r, _ = same(ctx, model.Problem(golden, [synth.default_nodepool()], [a, b], pods))
    assert list(r.pod_result) == [0, 1, 1]


def test_zonal_anti_affinity_and_foreign_selector(ctx, golden):
    lab = {"app": "za"}
    pc, pods = TC.deployment(4, lab, [model.TopologyTerm("anti", model.ZONE, TC.sel(lab))])
    r, _ = same(ctx, model.Problem(golden, [synth.default_nodepool()], [pc], pods))
    assert r.n_nodeclaims == 1 and int((r.pod_result == -1).sum()) == 3
    other = model.PodClass(labels={"app": "web"}, requirements=[model.Requirement(model.ZONE, "In", ["test-zone-1a"])])
    owner = model.PodClass(labels={"app": "probe"},
                           topology=[model.TopologyTerm("spread", model.ZONE, TC.sel({"app": "web"}), max_skew=1)])
    pods = synth.pods_from_specs([(0, {"cpu": "2", "memory": "1Gi"})] * 2 + [(1, {"cpu": "1", "memory": "1Gi"})])
    r, _ = same(ctx, model.Problem(golden, [synth.default_nodepool()], [other, owner], pods))
    assert r.n_nodeclaims == 2


def test_preference_policy_ignore(golden):
    """PREFERENCE_POLICY=Ignore (kp_device_opts.preference_policy) drops ScheduleAnyway spreads; Respect honours them
    until relaxed (one pod per NodeClaim here), both bit-exact with the oracle."""
    from kpsim import native
    lab = {"app": "p"}
    pc, pods = TC.deployment(6, lab, [model.TopologyTerm("spread", model.HOSTNAME, TC.sel(lab),
                                                         when_unsatisfiable="ScheduleAnyway")])
    prob = model.Problem(golden, [synth.default_nodepool()], [pc], pods)
    c = native.Context(0, preference_policy=abi.KP_PREFERENCE_IGNORE)
    try:
        dev = parity.run_device(c, prob)
        o = __import__("pyoracle").solve(prob, preference_policy=abi.KP_PREFERENCE_IGNORE)
        np.testing.assert_array_equal(dev[0].pod_result, o.results.pod_result)
    finally:
        c.close()
    r = native.Context(0)
    try:
        dev = parity.run_device(r, prob)
        o = __import__("pyoracle").solve(prob)
        np.testing.assert_array_equal(dev[0].pod_result, o.results.pod_result)
        assert dev[0].n_nodeclaims == 6
    finally:
        r.close()


@pytest.mark.parametrize("seed", range(24))
def test_fuzz_topology(ctx, golden, seed):
    """Random spread / affinity / anti-affinity terms (zone, hostname, capacity-type; selectors on the class itself,
    other classes, everything or nothing; namespaces; minDomains; node filter policies) over fuzzed requirements,
    taints, weighted NodePools with limits and minValues."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=160, replace=False))]
    same(ctx, fuzzgen.fuzz_topology_problem(sub, seed, n_pods=int(rng.integers(50, 300))))


@pytest.mark.parametrize("n", [500, 3000])
def test_config3_sample(ctx, golden, n):
    same(ctx, synth.subsample(synth.config3(catalog=golden), n))


def test_config3_full_digest(ctx, golden):
    """BASELINE configs[2] at full size (50k pods): every output field equals the oracle's committed digest
    (tests/golden/gen_scale_digest.py config3_50k; the oracle needs ~1 min here)."""
    with open(os.path.join(os.path.dirname(__file__), "golden", "scale_digests.json")) as f:
        want = json.load(f)["config3_50k"]
    prob = synth.config3(catalog=golden, n_pods=want["n_pods"])
    got = parity.result_digest(parity.run_device(ctx, prob))
    assert got == {k: v for k, v in want.items() if k != "n_pods"}


def test_bound_pods_zonal_spread(ctx, golden):
    """countDomains: two bound pods in test-zone-1a push the pending pods to 1b and 1c (test_topology_cpu's case)."""
    r, q = same(ctx, TC._bound_zone_problem(golden, 4))
    assert r.n_nodeclaims == 2 and list(r.nodeclaim_n_pods) == [2, 2]


def test_existing_nodes_hostname_anti_affinity(ctx, golden):
    """Existing nodes with room: a hostname self-anti-affinity deployment takes one pod per existing node (bound pods of
    the class block their nodes), then one NodeClaim per remaining pod."""
    lab = {"app": "spread-me"}
    pc, pods = TC.deployment(8, lab, [model.TopologyTerm("anti", model.HOSTNAME, TC.sel(lab))])
    it = golden[0]
    nodes = []
    for j in range(4):
        labels = synth.node_labels(it, "test-zone-1%s" % "abc"[j % 3], "on-demand", "default")
        nodes.append(model.ExistingNode("node-%d" % j, labels, np.array(it.allocatable, np.int64)))
    prob = model.Problem(golden, [synth.default_nodepool()], [pc], pods, nodes, bound=[(1, 0)])
    r, _ = same(ctx, prob)
    assert sorted(int(x) for x in r.pod_result if x < -1) == [-5, -4, -2]   # nodes 0, 2, 3 (node 1 holds one already)
    assert r.n_nodeclaims == 5


def _hostname_affinity_problem(golden, op, hosts, bound_on):
    """a self-selecting hostname pod affinity whose pod requires the hostname (op hosts); a selected pod is bound on
    node `bound_on` of three existing nodes"""
    lab = {"app": "ha", "tier": "web"}
    pc = model.PodClass(labels=lab, requirements=[model.Requirement(model.HOSTNAME, op, hosts)],
                        topology=[model.TopologyTerm("affinity", model.HOSTNAME, TC.sel({"tier": "web"}))])
    pods = synth.pods_from_specs([(0, {"cpu": "1", "memory": "1Gi"})] * 2)
    it = next(t for t in golden if t.name == "m5.2xlarge")
    nodes = [model.ExistingNode("node-%d" % j, synth.node_labels(it, "test-zone-1a", "on-demand", "default"),
                                np.array(it.allocatable, np.int64)) for j in range(3)]
    return model.Problem(golden, [synth.default_nodepool()], [pc], pods, nodes, bound=[(bound_on, 0)])


@pytest.mark.parametrize("op,hosts,bound_on,want", [
    ("In", ["node-1"], 0, [-3, -3]),             # the positive host is outside podDomains: bootstrap on node-1
    ("In", ["node-0", "node-1"], 0, [-2, -2]),   # a positive host inside podDomains: only it
    ("NotIn", ["node-0"], 0, [-3, -3]),          # every positive host excluded: bootstrap on the first node left
    ("NotIn", ["node-2"], 0, [-2, -2]),
    ("In", ["node-2", "node-7"], 1, [-4, -4]),   # a name no node carries
])
def test_hostname_affinity_pod_domains(ctx, golden, op, hosts, bound_on, want):
    """nextDomainAffinity counts only the positive domains the pod's own requirements admit (soak: many_groups 199):
    a pod requiring hostname In [node-1] with a selected pod bound elsewhere bootstraps on node-1."""
    r, _ = same(ctx, _hostname_affinity_problem(golden, op, hosts, bound_on))
    assert list(r.pod_result) == want


def _sort_skipped_problem(golden):
    """four self-spread pods fill NodeClaims 0 and 1 (two each; the slice is [1, 0] after the fourth), a plain pod joins
    NodeClaim 1 (a sort pending: 3 pods ahead of 2), and the last pod — a topology pod only the tainted existing node accepts — never reaches sort.Slice"""
    sp = model.PodClass(labels={"app": "s"}, topology=[model.TopologyTerm("spread", model.HOSTNAME, TC.sel({"app": "s"}),
                                                                         max_skew=2)])
    plain = model.PodClass(labels={"app": "y"})
    tp = model.PodClass(labels={"app": "t"}, requirements=[model.Requirement("team", "In", ["a"])],
                        tolerations=[model.Toleration("dedicated", "Exists")],
                        topology=[model.TopologyTerm("anti", model.HOSTNAME, TC.sel({"app": "nobody"}))])
    pods = synth.pods_from_specs([(0, {"cpu": "2", "memory": "1Gi"})] * 4 + [(1, {"cpu": "1500m", "memory": "1Gi"}),
                                                                          (2, {"cpu": "1", "memory": "1Gi"})])
    it = next(t for t in golden if t.name == "m5.2xlarge")
    labels = dict(synth.node_labels(it, "test-zone-1a", "on-demand", "default"), team="a")
    node = model.ExistingNode("node-0", labels, np.array(it.allocatable, np.int64),
                              taints=[model.Taint("dedicated", "x", "NoSchedule")])
    return model.Problem(golden, [synth.default_nodepool()], [sp, plain, tp], pods, [node])


def _eager_move_problem(golden):
    """_sort_skipped_problem with the plain pod a topology pod too: the block commits it and moves its NodeClaim ahead
    of the sort (the eager move), which the last pod's add() — taken by the existing node — must not adopt"""
    prob = _sort_skipped_problem(golden)
    prob.classes[1].topology = [model.TopologyTerm("anti", model.HOSTNAME, TC.sel({"app": "nobody"}))]
    return prob


@pytest.mark.parametrize("mk", [_sort_skipped_problem, _eager_move_problem])
def test_existing_node_takes_topology_pod_before_sort(ctx, golden, mk):
    """add() tries the existing nodes before sort.Slice(newNodeClaims): a topology pod an existing node takes leaves the
    slice unsorted (soak: topo_pref 58 — the device sorted for it, then placed it on the node)."""
    r, _ = same(ctx, mk(golden))
    assert list(r.pod_result) == [0, 0, 1, 1, 1, -2]
    assert list(r.nodeclaim_slice_pos) == [1, 0]


@pytest.mark.parametrize("seed", range(24))
def test_fuzz_topology_existing(ctx, golden, seed):
    """Topology terms over a cluster: existing nodes (placement order, headroom, taints, team labels, hostname /
    team requirements on the pods) and bound pods (countDomains, inverse anti-affinity), bit-exact with the oracle."""
    rng = np.random.Generator(np.random.PCG64(seed + 1000))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=160, replace=False))]
    same(ctx, fuzzgen.fuzz_topology_existing_problem(sub, seed, n_pods=int(rng.integers(50, 300)),
                                                     n_existing=int(rng.integers(4, 40))))


def test_node_dense_10k_beyond_first_slice_plan(golden):
    """10,000-pod node-dense Deployment (hostname anti-affinity): 10,000 in-flight NodeClaims, beyond the first slice
    plan (KP_NC_FIRST = 4096).  The prepare plans for them from the pods' self-selecting anti-affinity (allocatable read
    from HBM); every output field equals the oracle's committed digest (tests/golden/gen_scale_digest.py node_dense_10k;
    ~1 min of oracle time)."""
    from kpsim import native
    with open(os.path.join(os.path.dirname(__file__), "golden", "scale_digests.json")) as f:
        want = json.load(f)["node_dense_10k"]
    c = native.Context(0)  # its own ctx: the grown capacity stays with it
    try:
        dev = parity.run_device(c, TC.node_dense(golden, want["n_pods"]))
        assert dev[0].n_nodeclaims == 10_000 and (dev[0].nodeclaim_n_pods == 1).all()
        assert parity.result_digest(dev) == {k: v for k, v in want.items() if k != "n_pods"}
    finally:
        c.close()


def _split_solve(ctx, prob):
    """prepare + execute + fetch (one execute: an overflow would surface as KP_E_UNSUPPORTED from fetch)."""
    cv = model.CatalogView(prob.catalog)
    ctx.upload_catalog(cv)
    ctx.prepare(model.SolveInputView(prob))
    ctx.execute()
    cap_nc = max(16, prob.pods.n + 1)
    out = model.OutputBuffers(prob.pods.n, cap_nc, cap_nc * prob.max_instance_types)
    ctx.fetch(out)
    r = out.results()
    return r, [model.parse_requirements_blob(ctx.nodeclaim_requirements(i)) for i in range(r.n_nodeclaims)]


def test_node_dense_20k_one_execute(golden):
    """20,000-pod node-dense Deployment: planned for 20k NodeClaims at prepare (no overflow re-run: the split calls
    succeed), slice arrays in HBM beyond the LDS slice; equal to the oracle's committed digest (node_dense_20k)."""
    from kpsim import native
    with open(os.path.join(os.path.dirname(__file__), "golden", "scale_digests.json")) as f:
        want = json.load(f)["node_dense_20k"]
    c = native.Context(0)
    try:
        dev = _split_solve(c, TC.node_dense(golden, want["n_pods"]))
        assert dev[0].n_nodeclaims == 20_000 and (dev[0].nodeclaim_n_pods == 1).all()
        assert parity.result_digest(dev) == {k: v for k, v in want.items() if k != "n_pods"}
    finally:
        c.close()


def test_scheduler_solve_grows_output_buffers(golden):
    """kpsim.scheduler.Scheduler.Solve (the reference-shaped entry point) over the 10k node-dense Deployment: its first
    output buffers hold 8,192 NodeClaims; kp_solve reports KP_E_BUFFER with the sizes and the scheduler re-fetches the
    executed solve into buffers of that size (one execute).  The raw result equals the oracle's committed digest."""
    from kpsim import native, scheduler
    with open(os.path.join(os.path.dirname(__file__), "golden", "scale_digests.json")) as f:
        want = json.load(f)["node_dense_10k"]
    prob = TC.node_dense(golden, want["n_pods"])
    c = native.Context(0)
    try:
        s = scheduler.Scheduler(prob.catalog, ctx=c)
        res = s.Solve(prob)
        assert len(res.new_nodeclaims) == 10_000 and not res.pod_errors
        assert all(len(nc.pods) == 1 for nc in res.new_nodeclaims)
        reqs = [model.parse_requirements_blob(c.nodeclaim_requirements(i)) for i in range(res.raw.n_nodeclaims)]
        assert parity.result_digest((res.raw, reqs)) == {k: v for k, v in want.items() if k != "n_pods"}
    finally:
        c.close()


def test_node_dense_does_not_stick_to_ctx(golden):
    """A node-dense solve does not leave its large plan on the ctx: a config-2 solve after it on the same
    ctx takes the same quick-accept path (counters) and result as on a fresh ctx."""
    from kpsim import native
    prob = synth.subsample(synth.config2(catalog=golden), 4000)
    fresh = native.Context(0)
    used = native.Context(0)
    try:
        want = parity.run_device(fresh, prob)
        qa_want = fresh.ffd_cycles()[12]
        parity.run_device(used, TC.node_dense(golden, 6000))
        got = parity.run_device(used, prob)
        parity.assert_same(got, want)
        assert used.ffd_cycles()[12] == qa_want  # quick accepts
    finally:
        fresh.close()
        used.close()


def test_overflow_rerun_once(golden):
    """In-flight NodeClaims the prepare cannot foresee (pods that each need most of a node, no topology terms): the first
    plan overflows, kp_solve re-runs once planned for every pod, and the result equals the oracle."""
    big = [it for it in golden if it.name.startswith("m5.") or it.name.startswith("m6i.")]
    pc = model.PodClass(requirements=[model.Requirement("node.kubernetes.io/instance-type", "In", ["m5.large"])])
    pods = synth.pods_from_specs([(0, {"cpu": "1500m", "memory": "1Gi"})] * 4500)
    prob = model.Problem(big, [synth.default_nodepool()], [pc], pods)
    from kpsim import native
    c = native.Context(0)
    try:
        dev = parity.run_device(c, prob)
        assert dev[0].n_nodeclaims == 4500
        parity.assert_same(dev, parity.run_oracle(prob))
    finally:
        c.close()


@pytest.mark.parametrize("seed", list(range(8)) + [1872, 1899])  # + tools/soak.py many_groups 172 / 199
def test_fuzz_many_groups(ctx, golden, seed):
    """More than 8 topology groups constraining a class and more than 16 counting it (fuzzgen.add_many_groups): up to
    KP_MAX_TOPO = 32 / KP_MAX_TOPO_REC = 64 per class, over a cluster with bound pods."""
    rng = np.random.Generator(np.random.PCG64(seed + 8100))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=200, replace=False))]
    prob = fuzzgen.fuzz_topology_existing_problem(sub, seed + 8100, n_pods=int(rng.integers(100, 400)),
                                                  n_existing=int(rng.integers(4, 40)))
    fuzzgen.add_many_groups(rng, prob, n_terms=int(rng.integers(10, 18)))  # 8-13 constraining, up to 27 counting
    same(ctx, prob)


# ---- one group per TopologyGroup.Hash() identity, with the first owner's node filter / minDomains (row N1) ----

@pytest.mark.parametrize("a_first", [True, False])
def test_shared_identity_first_owner_filter(ctx, golden, a_first):
    """Equal identities, Honor node filters zone In [1a, 1b] vs [1b, 1c]: the first pod in input order decides the
    group's filter (hand-derived placements in test_topology_cpu.SHARED_FILTER_WANT)."""
    r, q = same(ctx, TC.shared_filter_problem(golden, a_first))
    want, zones = TC.SHARED_FILTER_WANT[a_first]
    assert list(r.pod_result) == want
    assert [TC.zone_of(x) for x in q] == [(z,) for z in zones]


@pytest.mark.parametrize("a_first", [True, False])
def test_shared_identity_first_owner_min_domains(ctx, golden, a_first):
    """Equal identities, minDomains 4 vs none: the first pod in input order decides the group's minDomains."""
    r, _ = same(ctx, TC.shared_min_domains_problem(golden, a_first))
    assert list(r.pod_result) == TC.SHARED_MIN_DOMAINS_WANT[a_first]


@pytest.mark.parametrize("a_big", [True, False])
def test_shared_identity_relaxed_only(ctx, golden, a_big):
    """An identity with two filters that only relaxed pods create: one variant group per filter, the first relaxation
    births its own (KpDev.late_sib), and every owner's constraint routes to it (hand-derived placements in
    test_topology_cpu.RELAXED_ONLY_WANT)."""
    r, _ = same(ctx, TC.relaxed_only_shared_problem(golden, a_big))
    assert list(r.pod_result) == TC.RELAXED_ONLY_WANT[a_big]


@pytest.mark.parametrize("seed", range(16))
def test_fuzz_shared_identity(ctx, golden, seed):
    """fuzzgen.add_shared_identities over the topology fuzz families (odd seeds: with existing nodes and bound pods):
    sibling classes whose terms hash equal while their Honor filter values and minDomains differ, pods of a family
    interleaved in input order."""
    rng = np.random.Generator(np.random.PCG64(seed + 500))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=160, replace=False))]
    same(ctx, fuzzgen.fuzz_shared_identity_problem(sub, seed, n_pods=int(rng.integers(80, 300)),
                                                   n_existing=(seed % 2) * 20))


@pytest.mark.parametrize("seed", range(10))
def test_fuzz_shared_identity_relaxed(ctx, golden, seed):
    """fuzzgen.add_relaxed_shared on top: families whose shared spread identity only relaxation creates (variant
    groups, the first relaxation births its own) next to families whose first input pod decides."""
    rng = np.random.Generator(np.random.PCG64(seed + 700))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=160, replace=False))]
    prob = fuzzgen.fuzz_shared_identity_problem(sub, seed + 700, n_pods=int(rng.integers(80, 300)),
                                                n_existing=(seed % 2) * 20)
    same(ctx, fuzzgen.add_relaxed_shared(rng, prob))


@pytest.mark.parametrize("seed", range(8))
def test_fuzz_more_than_16_constraining_groups(ctx, golden, seed):
    """add_many_groups with 36-47 terms: classes constrained by 17-24 topology groups (KP_MAX_TOPO = 32; beyond the
    8-row prefilter snapshot, read from the global counters) and counted by up to 50, over clusters with bound pods."""
    rng = np.random.Generator(np.random.PCG64(seed + 8300))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=200, replace=False))]
    prob = fuzzgen.fuzz_topology_existing_problem(sub, seed + 8300, n_pods=int(rng.integers(100, 300)),
                                                  n_existing=int(rng.integers(4, 40)))
    fuzzgen.add_many_groups(rng, prob, n_terms=int(rng.integers(36, 48)))
    same(ctx, prob)
