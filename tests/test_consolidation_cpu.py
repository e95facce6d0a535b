"""CPU: consolidation decisions of the oracle on hand-built clusters, the command replay, and rank sharding (gloo).

Known answers follow [core] pkg/controllers/disruption (computeConsolidation, computeSpotToSpotConsolidation,
filterOutSameInstanceType, SimulateScheduling's uninitialized-node errors, NodePool limits recomputed without the
candidates).  The core module is not in the reference tree, so these cases are built from its recalled semantics and
the reference's documentation (designs/consolidation.md, website disruption.md); the decision layer is "parity
unpinned" in DESIGN.md, while the Solve underneath it is pinned by the reference KATs.
"""
import os

import numpy as np
import pytest

import pyoracle
from kpsim import abi, consolidation, model
from kpsim.model import ARCH, CAPACITY_TYPE, INSTANCE_TYPE, NODEPOOL, ZONE

GI = 2 ** 30 * 1000  # milli-bytes per GiB
ZA = "test-zone-1a"


def _type(name, cpu, mem_gi, od=None, spot=None):
    cap = np.zeros(model.R, np.int64)
    cap[model.RIDX["cpu"]] = cpu * 1000
    cap[model.RIDX["memory"]] = mem_gi * GI
    cap[model.RIDX["pods"]] = 110_000
    offs = []
    if od is not None:
        offs.append(model.Offering("on-demand", ZA, od, True))
    if spot is not None:
        offs.append(model.Offering("spot", ZA, spot, True))
    return model.InstanceType(name, {INSTANCE_TYPE: [name], ARCH: ["amd64"]}, cap, cap.copy(), offs)


def _node(name, it, cpu_avail, ct="on-demand", pool="default"):
    avail = np.array(it.allocatable, np.int64).copy()
    avail[model.RIDX["cpu"]] = cpu_avail
    labels = {INSTANCE_TYPE: it.name, ARCH: "amd64", ZONE: ZA, CAPACITY_TYPE: ct, NODEPOOL: pool}
    return model.ExistingNode(name=name, labels=labels, available=avail)


def _pods(cpus):
    from kpsim import synth
    return synth.pods_from_specs([(0, {"cpu": str(c)}) for c in cpus])


def _pool(cts=("on-demand",), limits=None):
    return model.NodePool("default", requirements=[model.Requirement(CAPACITY_TYPE, "In", list(cts))],
                          limits_remaining=limits)


def _cand(node, pods, price, ct=abi.KP_CT_ON_DEMAND, it=-1, pool=-1, cap=None):
    return model.Candidate(node=node, pods=np.array(pods, np.int32), price=price, capacity_type=ct, instance_type=it,
                           nodepool=pool, capacity=cap)


def _one(cp, mode=abi.KP_CONSOLIDATE_SINGLE, spot_to_spot=False):
    return pyoracle.consolidate(cp, mode, spot_to_spot=spot_to_spot)


CAT = [_type("small", 2, 4, od=0.1, spot=0.05), _type("medium", 4, 8, od=0.2, spot=0.1),
       _type("large", 8, 16, od=0.4, spot=0.2)]


def test_delete_when_pods_fit_elsewhere():
    prob = model.Problem(CAT, [_pool()], [model.PodClass()], _pods([1]),
                         existing=[_node("n0", CAT[1], 3000), _node("n1", CAT[1], 4000)])
    cp = model.ConsolidationProblem(prob, [_cand(0, [0], 0.2, it=1)])
    r = _one(cp)[0]
    assert (r["decision"], r["valid"], r["all_scheduled"], r["n_new_nodeclaims"]) == (abi.KP_DECISION_DELETE, 1, 1, 0)


def test_replace_with_cheaper_type_and_price_filter():
    prob = model.Problem(CAT, [_pool()], [model.PodClass()], _pods([3]),
                         existing=[_node("n0", CAT[2], 5000), _node("n1", CAT[1], 1000)])
    r = _one(model.ConsolidationProblem(prob, [_cand(0, [0], 0.4, it=2)]))[0]
    # medium (0.2) fits 3 cpu and is cheaper; large's worst launch price 0.4 is not < 0.4
    assert (r["decision"], r["valid"], r["n_new_nodeclaims"], r["n_replacement_types"]) == (abi.KP_DECISION_REPLACE, 1, 1, 1)
    assert r["replacement_price"] == 0.2 and r["candidate_price"] == 0.4
    r = _one(model.ConsolidationProblem(prob, [_cand(0, [0], 0.15, it=2)]))[0]
    assert r["decision"] == abi.KP_DECISION_NONE and r["n_new_nodeclaims"] == 1


def test_two_replacements_is_no_op():
    prob = model.Problem(CAT, [_pool()], [model.PodClass()], _pods([7, 7]),
                         existing=[_node("n0", CAT[2], 0), _node("n1", CAT[1], 1000)])
    r = _one(model.ConsolidationProblem(prob, [_cand(0, [0, 1], 5.0, it=2)]))[0]
    assert r["decision"] == abi.KP_DECISION_NONE and r["n_new_nodeclaims"] == 2 and r["all_scheduled"] == 1


def test_uninitialized_node_placement_is_an_error():
    prob = model.Problem(CAT, [_pool(limits={"cpu": 0})], [model.PodClass()], _pods([1]),
                         existing=[_node("n0", CAT[1], 3000), _node("n1", CAT[1], 4000)])
    init = np.array([1, 0], np.uint8)
    r = _one(model.ConsolidationProblem(prob, [_cand(0, [0], 0.2, it=1)], initialized=init))[0]
    assert r["decision"] == abi.KP_DECISION_NONE and r["all_scheduled"] == 0
    # a pending pod on the uninitialized node is not an error
    prob2 = model.Problem(CAT, [_pool(limits={"cpu": 0})], [model.PodClass()], _pods([1, 1]),
                          existing=[_node("n0", CAT[1], 3000), _node("n1", CAT[1], 4000)])
    cp = model.ConsolidationProblem(prob2, [_cand(0, [], 0.2, it=1)], pending=np.array([0, 1], np.int32),
                                    initialized=init)
    assert _one(cp)[0]["decision"] == abi.KP_DECISION_DELETE


def test_candidate_capacity_returns_to_nodepool_limits():
    # the pool's remaining cpu is 2: without the candidate's 8 cpu back, no NodeClaim can be launched
    prob = model.Problem(CAT, [_pool(limits={"cpu": 2000})], [model.PodClass()], _pods([3]),
                         existing=[_node("n0", CAT[2], 5000)])
    r = _one(model.ConsolidationProblem(prob, [_cand(0, [0], 0.4, it=2)]))[0]
    assert r["decision"] == abi.KP_DECISION_NONE and r["all_scheduled"] == 0
    r = _one(model.ConsolidationProblem(prob, [_cand(0, [0], 0.4, it=2, pool=0, cap=CAT[2].capacity)]))[0]
    assert r["decision"] == abi.KP_DECISION_REPLACE and r["n_replacement_types"] == 1


def _spot_catalog(n):
    return [_type("t%02d" % i, 4 + i % 3, 16, od=1.0 + i, spot=0.01 * (i + 1)) for i in range(n)]


@pytest.mark.parametrize("n_types,gate,expect", [(20, False, (abi.KP_DECISION_NONE, 0)),
                                                  (20, True, (abi.KP_DECISION_REPLACE, 15)),
                                                  (14, True, (abi.KP_DECISION_NONE, 0))])
def test_spot_to_spot(n_types, gate, expect):
    cat = _spot_catalog(n_types)
    prob = model.Problem(cat, [_pool(("spot", "on-demand"))], [model.PodClass()], _pods([3]),
                         existing=[_node("n0", cat[0], 4000, ct="spot")])
    cp = model.ConsolidationProblem(prob, [_cand(0, [0], 0.5, ct=abi.KP_CT_SPOT, it=0)])
    r = _one(cp, spot_to_spot=gate)[0]
    assert (r["decision"], r["n_replacement_types"]) == expect


def test_od_candidate_replacement_keeps_spot_price_filter():
    # an on-demand candidate with a spot/on-demand pool: worst launch price uses the spot offerings (precedence
    # reserved > spot > on-demand), so a type whose on-demand price is above the candidate's still qualifies
    cat = [_type("a", 4, 16, od=5.0, spot=0.1), _type("b", 8, 16, od=0.3, spot=None)]
    prob = model.Problem(cat, [_pool(("spot", "on-demand"))], [model.PodClass()], _pods([3]),
                         existing=[_node("n0", cat[1], 4000)])
    r = _one(model.ConsolidationProblem(prob, [_cand(0, [0], 0.2, it=1)]))[0]
    assert r["decision"] == abi.KP_DECISION_REPLACE and r["n_replacement_types"] == 1 and r["replacement_price"] == 0.1


def test_multi_filter_out_same_instance_type():
    cat = [_type("medium", 4, 8, od=0.2), _type("large", 8, 16, od=0.35)]
    nodes = [_node("n0", cat[1], 5500), _node("n1", cat[0], 1500), _node("n2", cat[0], 0)]
    prob = model.Problem(cat, [_pool()], [model.PodClass()], _pods([2.5, 2.5]), existing=nodes)
    # candidates: large (0.35) + medium (0.2); the replacement large is not cheaper than the candidate large
    cp = model.ConsolidationProblem(prob, [_cand(0, [0], 0.35, it=1), _cand(1, [1], 0.2, it=0)])
    r = _one(cp, abi.KP_CONSOLIDATE_MULTI)
    assert len(r) == 1
    assert (r[0]["decision"], r[0]["valid"]) == (abi.KP_DECISION_REPLACE, 0)
    # two mediums: large (0.35 < 0.4) is a valid replacement of a type not being removed
    nodes2 = [_node("n0", cat[0], 1500), _node("n1", cat[0], 1500), _node("n2", cat[0], 0)]
    prob2 = model.Problem(cat, [_pool()], [model.PodClass()], _pods([2.5, 2.5]), existing=nodes2)
    cp2 = model.ConsolidationProblem(prob2, [_cand(0, [0], 0.2, it=0), _cand(1, [1], 0.2, it=0)])
    r2 = _one(cp2, abi.KP_CONSOLIDATE_MULTI)[0]
    assert (r2["decision"], r2["valid"], r2["n_replacement_types"]) == (abi.KP_DECISION_REPLACE, 1, 1)


def test_probe_numbering_matches_firstn_search_space():
    for n, mx, want in [(0, 100, 0), (1, 100, 0), (2, 100, 1), (50, 100, 49), (100, 100, 99), (101, 100, 100),
                        (5000, 100, 100)]:
        assert model.consolidation_probe_count(n, abi.KP_CONSOLIDATE_MULTI, mx) == want
    assert model.consolidation_probe_count(7, abi.KP_CONSOLIDATE_SINGLE) == 7


def _sequential_multi(valid, n, mx=100):
    """firstNConsolidationOption as written (binary search calling computeConsolidation on demand)."""
    if n < 2:
        return -1
    lo, hi = 1, mx if n > mx else n - 1
    best = -1
    while lo <= hi:
        mid = (lo + hi) // 2
        if valid(mid + 1):  # prefix candidates[0 : mid+1]
            best, lo = mid + 1, mid + 1
        else:
            hi = mid - 1
    return best


def test_replay_equals_sequential_search():
    rng = np.random.Generator(np.random.PCG64(5))
    for _ in range(300):
        n = int(rng.integers(0, 160))
        cnt = model.consolidation_probe_count(n, abi.KP_CONSOLIDATE_MULTI)
        res = np.zeros(cnt, abi.PROBE_DTYPE)
        res["valid"] = rng.random(cnt) < rng.random()
        seq = _sequential_multi(lambda size: bool(res["valid"][size - 2]), n)
        got = consolidation.replay_multi(res, n)
        assert (got + 2 if got >= 0 else -1) == seq


def _fuzz_cp(seed):
    import fuzzgen
    from kpsim import catalog
    gold = catalog.golden_catalog()
    rng = np.random.Generator(np.random.PCG64(seed))
    sub = [gold[int(i)] for i in sorted(rng.choice(len(gold), size=100, replace=False))]
    return fuzzgen.fuzz_consolidation(sub, seed, n_nodes=30, n_pods=120, n_candidates=12)


def _rank_main(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = []
        for seed in SHARD_SEEDS:
            cp = _fuzz_cp(seed)
            fn = lambda c, m, b0, b1: pyoracle.consolidate(c, m, b0, b1)  # noqa: E731
            for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
                cmd = consolidation.compute_command(cp, mode, fn, group=dist.group.WORLD,
                                                    replacement_fn=pyoracle.consolidate_replacement)
                out.append(_cmd_fields(cmd))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


SHARD_SEEDS = (3, 4, 8, 11)


def _cmd_fields(cmd):
    return (cmd.decision, tuple(cmd.candidates), cmd.n_replacement_types, cmd.candidate_price, cmd.replacement_price,
            cmd.mode, cmd.probe, cmd.nodepool, tuple(cmd.type_ids), cmd.requirements, cmd.n_reserved)


def test_sharded_command_equals_single_rank_gloo():
    """compute_command over a world-size-2 gloo group (probes sharded, one all_gather, the replacement read back on every
    rank) returns the whole Command — delete set, prices, the replacement's NodePool, price-ordered type ids,
    requirements and held reservations — equal to the single-process command (orc_consolidate_command)."""
    import multiprocessing as mp
    import socket
    want = []
    n_replace = 0
    for seed in SHARD_SEEDS:
        cp = _fuzz_cp(seed)
        for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
            cmd = pyoracle.consolidate_command(cp, mode)
            want.append(_cmd_fields(cmd))
            n_replace += cmd.decision == abi.KP_DECISION_REPLACE and len(cmd.type_ids) > 0
    assert n_replace >= 1
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(60)
    assert got[0] == want and got[1] == want


# ------------------------------------------------------------------------------------------------
# the command (orc_consolidate_command, the restatement kp_consolidate_command is checked against)
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", sorted(__import__("cons_cases").SCENARIOS))
@pytest.mark.parametrize("mode", [abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_BOTH])
def test_command_reference_scenarios(golden, name, mode):
    """The reference's e2e consolidation outcomes (tests/cons_cases.py) from the oracle's command."""
    import cons_cases
    cp, expect = cons_cases.SCENARIOS[name](golden)
    cmd = pyoracle.consolidate_command(cp, mode)
    cons_cases.check_expect(cmd, cp, expect)
    assert cmd.mode == abi.KP_CONSOLIDATE_SINGLE and cmd.candidates == [0]


def _both(cp, fn, s2s):
    m = consolidation.compute_command(cp, abi.KP_CONSOLIDATE_MULTI, fn)
    return m if m.decision != abi.KP_DECISION_NONE else consolidation.compute_command(cp, abi.KP_CONSOLIDATE_SINGLE, fn)


@pytest.mark.parametrize("seed", range(6))
def test_command_equals_probe_replay(seed):
    """orc_consolidate_command = the Python replay (first valid single / firstNConsolidationOption) over the oracle's
    probe rows; BOTH = multi-node, else single-node (the disruption controller's method order)."""
    cp = _fuzz_cp(40 + seed)
    s2s = seed % 2 == 0
    fn = lambda c, m, b0, b1: pyoracle.consolidate(c, m, b0, b1, spot_to_spot=s2s)  # noqa: E731
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI, abi.KP_CONSOLIDATE_BOTH):
        want = _both(cp, fn, s2s) if mode == abi.KP_CONSOLIDATE_BOTH else consolidation.compute_command(cp, mode, fn)
        got = pyoracle.consolidate_command(cp, mode, spot_to_spot=s2s)
        assert (got.decision, got.candidates, got.n_replacement_types, got.candidate_price, got.replacement_price) == \
            (want.decision, want.candidates, want.n_replacement_types, want.candidate_price, want.replacement_price)
        if got.decision == abi.KP_DECISION_REPLACE:
            assert len(got.type_ids) == got.n_replacement_types and got.nodepool >= 0 and got.requirements
        else:
            assert got.type_ids == [] and got.nodepool == -1


# ------------------------------------------------------------------------------------------------
# the reference's e2e disruption scenarios on the cluster emulator, oracle backend (tests/e2e_cases.py)
# ------------------------------------------------------------------------------------------------
def _oracle_backend():
    import cluster_sim
    return cluster_sim.OracleBackend()


@pytest.mark.parametrize("spot", [False, True])
def test_e2e_replace_hostname_spread(golden, spot):
    import e2e_cases
    sim = e2e_cases.replace_hostname_spread(golden, _oracle_backend(), spot)
    assert [c.decision for c in sim.commands] == [abi.KP_DECISION_REPLACE] * 3 + [abi.KP_DECISION_NONE]


def test_e2e_od_to_spot(golden):
    import e2e_cases
    e2e_cases.od_to_spot(golden, _oracle_backend())


@pytest.mark.parametrize("spot", [False, True])
def test_e2e_delete_utilization(golden, spot):
    import e2e_cases
    e2e_cases.delete_utilization(golden, _oracle_backend(), spot)


def test_e2e_anti_affinity_replace(golden):
    import e2e_cases
    e2e_cases.anti_affinity_replace(golden, _oracle_backend(), n_nodes=8)


def test_e2e_multi_delete(golden):
    import e2e_cases
    sim = e2e_cases.multi_delete(golden, _oracle_backend(), n_nodes=50)
    assert sim.commands[0].mode == abi.KP_CONSOLIDATE_MULTI


@pytest.mark.parametrize("name", ["reserved_into", "reserved_between"])
def test_command_reference_scenarios_best_effort(golden, name):
    """suite_test.go's reserved scenarios run under MIN_VALUES_POLICY BestEffort too (the Describe's Entries,
    :1002-1004): without minValues the simulation is the Strict one."""
    import cons_cases
    cp, expect = cons_cases.SCENARIOS[name](golden)
    cp.cluster.min_values_policy = 1
    cons_cases.check_expect(pyoracle.consolidate_command(cp, abi.KP_CONSOLIDATE_BOTH), cp, expect)


@pytest.mark.parametrize("policy", [0, 1])
def test_e2e_preferred_anti_affinity_replace(golden, policy):
    import cluster_sim
    import e2e_cases
    e2e_cases.preferred_anti_affinity_replace(golden, cluster_sim.OracleBackend(policy), n_nodes=6, respect=policy == 0)


def test_e2e_preferred_affinity_delete(golden):
    import e2e_cases
    e2e_cases.preferred_affinity_delete(golden, _oracle_backend())


@pytest.mark.parametrize("name", ["budget_empty_delete", "budget_nonempty_delete", "budget_replace", "budget_blocking"])
def test_e2e_budgets(golden, name):
    """test/suites/consolidation/suite_test.go:188-453 (NodePool disruption budgets, filtered caller-side) on the
    emulator, oracle backend: the reference's per-step disruption bound and end state."""
    import e2e_cases
    getattr(e2e_cases, name)(golden, _oracle_backend())
