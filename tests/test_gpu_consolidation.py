"""GPU: consolidation probes on the gfx950 path (kp_consolidate) against the CPU oracle (orc_consolidate).

Per probe: decision, validity (the multi-node search test), new NodeClaims (capped at 2), replacement option count,
candidate / replacement prices (exact doubles), pods rescheduled; all_scheduled wherever the probe ran to completion
(fewer than two new NodeClaims).  Sizes are those the oracle finishes in seconds; config 4 at full size is checked
by properties (every probe evaluated, DELETE-dominated at 40-60% utilisation, shard-invariance).
"""
import numpy as np
import pytest

import fuzzgen
import pyoracle
from kpsim import abi, consolidation, model, synth

pytestmark = pytest.mark.gpu

FIELDS = ["decision", "valid", "n_new_nodeclaims", "n_replacement_types", "n_pods", "candidate_price",
          "replacement_price"]


@pytest.fixture(scope="module")
def ctx():
    from kpsim import native
    c = native.Context(0)
    yield c
    c.close()


def device_probes(ctx, cp, mode, spot_to_spot=False, begin=0, end=0):
    ctx.upload_catalog(model.CatalogView(cp.cluster.catalog))
    return ctx.consolidate(model.ConsolidateInputView(cp, mode, begin, end, spot_to_spot))


def assert_probes_equal(dev, orc):
    assert len(dev) == len(orc)
    for f in FIELDS:
        np.testing.assert_array_equal(dev[f], orc[f], err_msg=f)
    done = orc["n_new_nodeclaims"] < 2
    np.testing.assert_array_equal(dev["all_scheduled"][done], orc["all_scheduled"][done], err_msg="all_scheduled")


@pytest.mark.parametrize("seed", range(24))
def test_fuzz_consolidation(ctx, golden, seed):
    rng = np.random.Generator(np.random.PCG64(500 + seed))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(60, 300)), replace=False))]
    cp = fuzzgen.fuzz_consolidation(sub, 500 + seed, n_nodes=int(rng.integers(4, 80)),
                                    n_pods=int(rng.integers(20, 300)), all_spot=seed % 4 == 0)
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        s2s = seed % 2 == 0
        assert_probes_equal(device_probes(ctx, cp, mode, s2s), pyoracle.consolidate(cp, mode, spot_to_spot=s2s))


@pytest.mark.parametrize("seed", range(20))
def test_fuzz_consolidation_mutating(ctx, golden, seed):
    """ExistingNode.Add's requirement merge changes nodes (the MUT probes): the GPU-avoidance pattern (instance-gpu-count
    DoesNotExist / NotIn pods next to Gt 0 / Exists pods; non-GPU nodes lack the label) and the mixed node-group pattern
    (karpenter.sh/nodepool DoesNotExist pods; managed-node-group nodes lack the label) over fuzzed clusters, plus the
    fuzz generator's own NotIn / DoesNotExist custom-label and hostname requirements.  Probes of both modes and the
    command against the oracle, and the pass really ran MUT probes."""
    rng = np.random.Generator(np.random.PCG64(6100 + seed))
    gpus = [it for it in golden if it.labels.get(fuzzgen.GPU_COUNT) not in (None, [], "")]
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(60, 250)), replace=False))]
    sub += [g for g in gpus[::max(1, len(gpus) // 12)] if g not in sub]
    cp = fuzzgen.fuzz_consolidation(sub, 6100 + seed, n_nodes=int(rng.integers(6, 70)),
                                    n_pods=int(rng.integers(30, 260)), all_spot=seed % 4 == 0,
                                    with_min=seed % 5 == 3)
    fuzzgen.add_mutators(rng, cp, gpus)
    s2s = seed % 2 == 0
    n_mut = 0
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode, s2s), pyoracle.consolidate(cp, mode, spot_to_spot=s2s))
        n_mut += ctx.consolidate_stats()[1][17]  # probes the MUT variant ran
    assert n_mut > 0
    assert_commands_equal(device_command(ctx, cp, abi.KP_CONSOLIDATE_BOTH, s2s),
                          pyoracle.consolidate_command(cp, abi.KP_CONSOLIDATE_BOTH, spot_to_spot=s2s))


@pytest.mark.parametrize("seed", range(8))
def test_fuzz_consolidation_mutating_topology(ctx, golden, seed):
    """The mutating shapes over topology-constrained clusters (per-probe domain counts, ExistingNode.Add's topology step
    on the probes' node copies) and over preferences that relax into them."""
    rng = np.random.Generator(np.random.PCG64(6300 + seed))
    gpus = [it for it in golden if it.labels.get(fuzzgen.GPU_COUNT) not in (None, [], "")]
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(60, 250)), replace=False))]
    sub += [g for g in gpus[::max(1, len(gpus) // 12)] if g not in sub]
    cp = fuzzgen.fuzz_topology_consolidation(sub, 6300 + seed, n_nodes=int(rng.integers(6, 50)),
                                             n_pods=int(rng.integers(30, 200)), all_spot=seed % 4 == 0)
    fuzzgen.add_mutators(rng, cp, gpus)
    s2s = seed % 2 == 1
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode, s2s), pyoracle.consolidate(cp, mode, spot_to_spot=s2s))
    assert_commands_equal(device_command(ctx, cp, abi.KP_CONSOLIDATE_BOTH, s2s),
                          pyoracle.consolidate_command(cp, abi.KP_CONSOLIDATE_BOTH, spot_to_spot=s2s))


@pytest.mark.parametrize("seed", range(16))
def test_fuzz_consolidation_min_values(ctx, golden, seed):
    """NodePools with minValues on instance-family: the probes' NodeClaim.Add minValues filter, TruncateInstanceTypes'
    minValues check (a dropped NodeClaim: NONE, or DELETE when only pending pods rode on it) and
    RemoveInstanceTypeOptionsByPriceAndMinValues / the spot-to-spot max(15, minNeeded) cut, against the oracle."""
    rng = np.random.Generator(np.random.PCG64(900 + seed))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(60, 300)), replace=False))]
    cp = fuzzgen.fuzz_consolidation(sub, 900 + seed, n_nodes=int(rng.integers(4, 80)),
                                    n_pods=int(rng.integers(20, 300)), all_spot=seed % 3 == 0,
                                    with_min=True)
    for np_ in cp.cluster.nodepools:  # minValues on every pool, sometimes beyond what a truncated list can hold
        if not any(r.min_values for r in np_.requirements):
            np_.requirements.append(model.Requirement("karpenter.k8s.aws/instance-family", "Exists", [],
                                                      int(rng.choice([1, 2, 5, 20, 40]))))
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        s2s = seed % 2 == 0
        assert_probes_equal(device_probes(ctx, cp, mode, s2s), pyoracle.consolidate(cp, mode, spot_to_spot=s2s))


def test_shard_ranges_concatenate(ctx, golden):
    cp = fuzzgen.fuzz_consolidation(golden[:200], 77, n_nodes=60, n_pods=250, n_candidates=40)
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        full = device_probes(ctx, cp, mode)
        n = len(full)
        parts = []
        for r in range(3):
            b0, b1 = consolidation.shard_range(n, r, 3)
            parts.append(device_probes(ctx, cp, mode, begin=b0, end=b1))
        assert_probes_equal(np.concatenate(parts), full)


def test_config4_small_parity(ctx, golden):
    cp = synth.config4(n_nodes=400, catalog=golden, n_pending=50)
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode), pyoracle.consolidate(cp, mode, n_threads=8))


def test_config4_full_size_properties(ctx, golden):
    """5k nodes / ~100k pods (BASELINE configs[3]): every probe of both modes against the oracle."""
    cp = synth.config4(catalog=golden)
    dev = device_probes(ctx, cp, abi.KP_CONSOLIDATE_SINGLE)
    assert len(dev) == len(cp.candidates)
    assert (dev["n_pods"] == np.array([len(c.pods) for c in cp.candidates])).all()
    assert_probes_equal(dev, pyoracle.consolidate(cp, abi.KP_CONSOLIDATE_SINGLE, n_threads=8))
    multi = device_probes(ctx, cp, abi.KP_CONSOLIDATE_MULTI)
    assert_probes_equal(multi, pyoracle.consolidate(cp, abi.KP_CONSOLIDATE_MULTI, n_threads=8))


@pytest.mark.parametrize("n_nodes", [600, 5000])
def test_config4_replace_parity(ctx, golden, n_nodes):
    """config4 with 2% node headroom (synth.config4(headroom=0.02), the bench's replace leg): the candidates' pods mostly
    miss the other nodes, so the probes scan the whole cluster, then run NodeClaim.Add / the templates and produce
    REPLACE decisions.  Every probe of both modes against the oracle, and the mix of decisions the leg exists for."""
    cp = synth.config4(n_nodes=n_nodes, catalog=golden, headroom=0.02)
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        dev = device_probes(ctx, cp, mode)
        assert_probes_equal(dev, pyoracle.consolidate(cp, mode, n_threads=8))
        assert (dev["decision"] == abi.KP_DECISION_REPLACE).sum() > len(dev) // 3


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_multi_device_ctx(golden, devices):
    """kp_device_opts.devices: one ctx over several device streams (the same ordinal repeated on a
    one-GPU box) shards the probe range internally and gathers the shards; equal to the single-device evaluation,
    also over a sub-range, and the summed counters cover every probe."""
    from kpsim import native
    cp = synth.config4(n_nodes=400, catalog=golden, n_pending=50)
    one = native.Context(0)
    multi = native.Context(devices=devices)
    try:
        for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
            want = device_probes(one, cp, mode)
            got = device_probes(multi, cp, mode)
            assert_probes_equal(got, want)
            _, cst = multi.consolidate_stats()
            assert cst[4] == len(want)  # probes evaluated, summed over the devices
            n = len(want)
            assert_probes_equal(device_probes(multi, cp, mode, begin=n // 3, end=n - 2), want[n // 3:n - 2])
        # KP_CONSOLIDATE_BOTH (the pass bench.py times): the multi-node and single-node parts are sharded separately;
        # the full range and sub-ranges inside / straddling the multi-node part, against the one-device pass and the
        # oracle
        n_s = model.consolidation_probe_count(len(cp.candidates), abi.KP_CONSOLIDATE_SINGLE)
        n_m = model.consolidation_probe_count(len(cp.candidates), abi.KP_CONSOLIDATE_MULTI)
        for c in (one, multi):
            c.upload_catalog(model.CatalogView(cp.cluster.catalog))
            c.consolidate_prepare(model.ConsolidateInputView(cp, abi.KP_CONSOLIDATE_SINGLE))
        want = one.consolidate_execute(abi.KP_CONSOLIDATE_BOTH, n_m + n_s)
        assert_probes_equal(multi.consolidate_execute(abi.KP_CONSOLIDATE_BOTH, n_m + n_s), want)
        assert multi.consolidate_stats()[1][4] == n_m + n_s
        for b, e in ((n_m // 2, n_m + 37), (3, n_m - 5), (n_m + 11, n_m + n_s - 9)):
            assert_probes_equal(multi.consolidate_execute(abi.KP_CONSOLIDATE_BOTH, n_m + n_s, b, e), want[b:e])
        assert_probes_equal(want[:n_m], pyoracle.consolidate(cp, abi.KP_CONSOLIDATE_MULTI, n_threads=8))
        assert_probes_equal(want[n_m:], pyoracle.consolidate(cp, abi.KP_CONSOLIDATE_SINGLE, n_threads=8))
        # split form: prepare once (every device), execute twice
        multi.consolidate_prepare(model.ConsolidateInputView(cp, abi.KP_CONSOLIDATE_SINGLE))
        n_s = model.consolidation_probe_count(len(cp.candidates), abi.KP_CONSOLIDATE_SINGLE)
        a = multi.consolidate_execute(abi.KP_CONSOLIDATE_SINGLE, n_s)
        assert_probes_equal(a, device_probes(one, cp, abi.KP_CONSOLIDATE_SINGLE))
    finally:
        multi.close()
        one.close()


def test_multi_device_state_errors(golden):
    """A solve prepare on the primary invalidates the multi-device pass (KP_E_STATE), like the single-device ctx."""
    from kpsim import native
    cp = synth.config4(n_nodes=100, catalog=golden, n_pending=0)
    multi = native.Context(devices=[0, 0])
    try:
        multi.upload_catalog(model.CatalogView(cp.cluster.catalog))
        multi.consolidate_prepare(model.ConsolidateInputView(cp, abi.KP_CONSOLIDATE_SINGLE))
        multi.prepare(model.SolveInputView(cp.cluster))
        with pytest.raises(native.KpError) as e:
            multi.consolidate_execute(abi.KP_CONSOLIDATE_SINGLE, len(cp.candidates))
        assert e.value.status == abi.KP_E_STATE
    finally:
        multi.close()


def _reserved_consolidation(golden, seed, full_cluster=False):
    """fuzz_consolidation over a catalog with reserved offerings (config5_catalog on the subsample: ODCR default and
    capacity-block reservations of capacity 1-20, some expiring) and NodePools that admit capacity-type reserved."""
    rng = np.random.Generator(np.random.PCG64(1300 + seed))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(80, 240)), replace=False))]
    cat = synth.config5_catalog(sub, n_default=min(44, len(sub) // 2), n_block=min(20, len(sub) // 6), seed=1300 + seed)
    cp = fuzzgen.fuzz_consolidation(cat, 1300 + seed, n_nodes=int(rng.integers(4, 60)),
                                    n_pods=int(rng.integers(20, 250)), all_spot=seed % 4 == 0,
                                    pending_frac=0.0 if full_cluster else 0.15)
    for np_ in cp.cluster.nodepools:
        for r in np_.requirements:
            if r.key == model.CAPACITY_TYPE and r.op == "In" and rng.random() < 0.8:
                r.values = sorted(set(r.values) | {"reserved"})
    if full_cluster:  # no headroom anywhere: every probe's pods need a new NodeClaim (REPLACE / NONE decisions)
        for n in cp.cluster.existing:
            n.available = np.minimum(n.available, 0)
    return cp


@pytest.mark.parametrize("seed", range(16))
def test_fuzz_consolidation_reserved(ctx, golden, seed):
    """Reserved offerings in the probes (ReservedOfferingModeFallback): NodeClaim.Add reserves compatible reserved
    offerings while the probe's capacities last but never fails for want of one, FinalizeScheduling's reservation-id
    requirement, reserved prices in OrderByPrice and first in WorstLaunchPrice — against the oracle."""
    cp = _reserved_consolidation(golden, seed, full_cluster=seed % 2 == 0)
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        s2s = seed % 2 == 1
        assert_probes_equal(device_probes(ctx, cp, mode, s2s), pyoracle.consolidate(cp, mode, spot_to_spot=s2s))


def _reserved_replace_case(golden, rcap, expiring=False, n_cands=1, ct="on-demand"):
    """One NodePool admitting on-demand + reserved, a catalog whose reserved offerings have capacity rcap, candidates
    each carrying one small pod on otherwise full nodes: the probe's NodeClaim reserves while capacity lasts."""
    cat = synth.config5_catalog(golden[:120], n_default=60, n_block=0, seed=3, expiring_frac=1.0 if expiring else 0.0)
    for it in cat:
        for o in it.offerings:
            if o.capacity_type == "reserved":
                o.reservation_capacity = rcap
                o.available = o.available and rcap != 0
    np_ = synth.default_nodepool()
    np_.requirements = [model.Requirement(model.CAPACITY_TYPE, "In", ["on-demand", "reserved"])]
    pods = synth.pods_from_specs([(0, {"cpu": "100m", "memory": "128Mi"})] * n_cands)
    nodes = []
    for j in range(n_cands):
        it = cat[j]
        nodes.append(model.ExistingNode("node-%d" % j, synth.node_labels(it, "test-zone-1a", ct, "default"),
                                        np.zeros(model.R, np.int64)))
    prob = model.Problem(cat, [np_], [model.PodClass()], pods, nodes)
    cands = [model.Candidate(node=j, pods=np.array([j], np.int32), price=5.0,
                             capacity_type=abi.KP_CT_SPOT if ct == "spot" else abi.KP_CT_ON_DEMAND, instance_type=j,
                             nodepool=0, capacity=None) for j in range(n_cands)]
    return model.ConsolidationProblem(prob, cands, np.zeros(0, np.int32), np.ones(n_cands, np.uint8))


@pytest.mark.parametrize("rcap,expiring", [(3, False), (1, False), (0, False), (5, True)])
def test_reserved_replacement(ctx, golden, rcap, expiring):
    """A REPLACE onto reserved capacity is priced at odPrice / 1e7 (offering.go:176) and is WorstLaunchPrice's first
    choice; with no capacity (or expiring reservations) the probe falls back to on-demand."""
    cp = _reserved_replace_case(golden, rcap, expiring, n_cands=3)
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        dev = device_probes(ctx, cp, mode)
        assert_probes_equal(dev, pyoracle.consolidate(cp, mode))
        assert (dev["decision"] == abi.KP_DECISION_REPLACE).all()
        if rcap > 0 and not expiring:
            assert (dev["replacement_price"] < 1e-6).all()
        else:
            assert (dev["replacement_price"] > 1e-6).all()


@pytest.mark.parametrize("seed", range(6))
def test_both_modes_one_pass(ctx, golden, seed):
    """KP_CONSOLIDATE_BOTH: one pass returns the multi-node probes then the single-node probes, each equal to its own
    mode's pass (and shards of the combined list concatenate to it)."""
    rng = np.random.Generator(np.random.PCG64(700 + seed))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(60, 300)), replace=False))]
    cp = fuzzgen.fuzz_consolidation(sub, 700 + seed, n_nodes=int(rng.integers(4, 80)), n_pods=int(rng.integers(20, 300)))
    ctx.upload_catalog(model.CatalogView(cp.cluster.catalog))
    ctx.consolidate_prepare(model.ConsolidateInputView(cp, abi.KP_CONSOLIDATE_SINGLE))
    nc = len(cp.candidates)
    n_s = model.consolidation_probe_count(nc, abi.KP_CONSOLIDATE_SINGLE)
    n_m = model.consolidation_probe_count(nc, abi.KP_CONSOLIDATE_MULTI)
    both = ctx.consolidate_execute(abi.KP_CONSOLIDATE_BOTH, n_m + n_s)
    assert_probes_equal(both[:n_m], ctx.consolidate_execute(abi.KP_CONSOLIDATE_MULTI, n_m))
    assert_probes_equal(both[n_m:], ctx.consolidate_execute(abi.KP_CONSOLIDATE_SINGLE, n_s))
    assert_probes_equal(both[:n_m], pyoracle.consolidate(cp, abi.KP_CONSOLIDATE_MULTI))
    cut = (n_m + n_s) // 3
    parts = [ctx.consolidate_execute(abi.KP_CONSOLIDATE_BOTH, n_m + n_s, b, e)
             for b, e in ((0, cut), (cut, 2 * cut), (2 * cut, n_m + n_s))]
    assert_probes_equal(np.concatenate(parts), both)


# ------------------------------------------------------------------------------------------------
# kp_consolidate_command: the decision loops replayed in the library + the replacement NodeClaim read-back
# ------------------------------------------------------------------------------------------------
CMD_FIELDS = ("decision", "mode", "probe", "candidates", "n_replacement_types", "candidate_price", "replacement_price",
              "nodepool", "type_ids", "requirements", "n_reserved")


def device_command(ctx, cp, mode, spot_to_spot=False):
    ctx.upload_catalog(model.CatalogView(cp.cluster.catalog))
    ctx.consolidate_prepare(model.ConsolidateInputView(cp, abi.KP_CONSOLIDATE_SINGLE, spot_to_spot=spot_to_spot))
    return ctx.consolidate_command(mode)


def assert_commands_equal(dev, orc):
    for f in CMD_FIELDS:
        assert getattr(dev, f) == getattr(orc, f), (f, dev, orc)


def _command_cases(golden):
    """(cp, spot_to_spot) over the fuzz generators: plain, minValues, reserved (REPLACE-heavy full clusters)."""
    out = []
    for seed in range(8):
        rng = np.random.Generator(np.random.PCG64(2500 + seed))
        sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(60, 300)), replace=False))]
        cp = fuzzgen.fuzz_consolidation(sub, 2500 + seed, n_nodes=int(rng.integers(4, 60)),
                                        n_pods=int(rng.integers(20, 250)), all_spot=seed % 4 == 0,
                                        with_min=seed % 3 == 0)
        out.append((cp, seed % 2 == 0))
    for seed in range(8):
        out.append((_reserved_consolidation(golden, 40 + seed, full_cluster=seed % 2 == 0), seed % 2 == 1))
    return out


def test_command_parity(ctx, golden):
    """kp_consolidate_command = orc_consolidate_command for SINGLE / MULTI / BOTH: the chosen method, probe and
    delete set, the probe row, and for a REPLACE the replacement's NodePool, price-ordered options, requirements text
    (capacity-type narrowed to spot, reservation-id of the held reservations) and held-reservation count."""
    n_replace = 0
    for cp, s2s in _command_cases(golden):
        for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI, abi.KP_CONSOLIDATE_BOTH):
            dev = device_command(ctx, cp, mode, s2s)
            assert_commands_equal(dev, pyoracle.consolidate_command(cp, mode, spot_to_spot=s2s))
            n_replace += dev.decision == abi.KP_DECISION_REPLACE and len(dev.type_ids) > 1
    assert n_replace >= 4


def test_command_costs_one_pass(ctx, golden):
    """kp_consolidate_command after kp_consolidate_execute of the same prepared pass replays that pass (no probe launch)
    and reads the replacement back once; a KP_E_BUFFER retry and a repeated call copy it; a BOTH pass serves a SINGLE or
    MULTI command; a new prepare starts over (kp_consolidate_stats counters 18-19: passes launched, read-backs run)."""
    n_seen = 0
    for cp, s2s in _command_cases(golden):
        ctx.upload_catalog(model.CatalogView(cp.cluster.catalog))
        ctx.consolidate_prepare(model.ConsolidateInputView(cp, abi.KP_CONSOLIDATE_SINGLE, spot_to_spot=s2s))
        nc = len(cp.candidates)
        n = model.consolidation_probe_count(nc, abi.KP_CONSOLIDATE_SINGLE) + \
            model.consolidation_probe_count(nc, abi.KP_CONSOLIDATE_MULTI)
        ctx.consolidate_execute(abi.KP_CONSOLIDATE_BOTH, n)
        want = pyoracle.consolidate_command(cp, abi.KP_CONSOLIDATE_BOTH, spot_to_spot=s2s)
        rb = 1 if want.decision == abi.KP_DECISION_REPLACE else 0
        tiny = consolidation.command_call(
            lambda cc: ctx.L.kp_consolidate_command(ctx.h, abi.KP_CONSOLIDATE_BOTH, __import__("ctypes").byref(cc)),
            cap_types=1, cap_req=4)[1]  # first try KP_E_BUFFER for a REPLACE, then the grown buffers
        cmd = ctx.consolidate_command(abi.KP_CONSOLIDATE_BOTH)
        assert_commands_equal(tiny, want)
        assert_commands_equal(cmd, want)
        ct = ctx.consolidate_stats()[1]
        assert (ct[18], ct[19]) == (1, rb), (ct[18], ct[19])
        single = pyoracle.consolidate_command(cp, abi.KP_CONSOLIDATE_SINGLE, spot_to_spot=s2s)
        assert_commands_equal(ctx.consolidate_command(abi.KP_CONSOLIDATE_SINGLE), single)
        assert ctx.consolidate_stats()[1][18] == 1  # served by the BOTH pass
        # a fresh prepare: the command runs its own pass
        ctx.consolidate_prepare(model.ConsolidateInputView(cp, abi.KP_CONSOLIDATE_SINGLE, spot_to_spot=s2s))
        assert_commands_equal(ctx.consolidate_command(abi.KP_CONSOLIDATE_BOTH), want)
        ct = ctx.consolidate_stats()[1]
        assert (ct[18], ct[19]) == (1, rb)
        n_seen += rb
    assert n_seen >= 2


def test_consolidator_command_has_replacement(golden):
    """kpsim.consolidation.Consolidator.compute_command (the per-process path; with a torch.distributed group each rank
    evaluates a shard) returns the whole Command, the replacement NodeClaim included (kp_consolidate_replacement), equal
    to the oracle's command of that method."""
    from kpsim import native
    n_rep = 0
    for cp, s2s in _command_cases(golden):
        con = consolidation.Consolidator(cp.cluster.catalog, ctx=native.Context(0), spot_to_spot=s2s)
        try:
            for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
                got = con.compute_command(cp, mode)
                assert_commands_equal(got, pyoracle.consolidate_command(cp, mode, spot_to_spot=s2s))
                n_rep += got.decision == abi.KP_DECISION_REPLACE
        finally:
            con.ctx.close()
    assert n_rep >= 2


@pytest.mark.parametrize("name", ["reserved_into", "reserved_between"])
def test_command_reference_scenarios(ctx, golden, name):
    """test/suites/consolidation/suite_test.go:915-1001 through the library: the on-demand m5.large is replaced by the
    m5.xlarge in the new reservation; the m5.xlarge reserved node moves to the m5.large reservation."""
    import cons_cases
    cp, expect = cons_cases.SCENARIOS[name](golden)
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_BOTH):
        cmd = device_command(ctx, cp, mode)
        cons_cases.check_expect(cmd, cp, expect)
        assert_commands_equal(cmd, pyoracle.consolidate_command(cp, mode))


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_command_multi_device(golden, devices):
    """The command over a multi-device ctx (probes sharded, the read-back on the primary) equals one device's."""
    from kpsim import native
    one = native.Context(0)
    multi = native.Context(devices=devices)
    try:
        for cp, s2s in _command_cases(golden)[::3]:
            for mode in (abi.KP_CONSOLIDATE_MULTI, abi.KP_CONSOLIDATE_BOTH):
                assert_commands_equal(device_command(multi, cp, mode, s2s), device_command(one, cp, mode, s2s))
    finally:
        multi.close()
        one.close()


# ------------------------------------------------------------------------------------------------
# consolidation over topology-constrained clusters (per-probe domain counts)
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("seed", range(24))
def test_fuzz_consolidation_topology(ctx, golden, seed):
    """Probes over pods with zonal / hostname / capacity-type spread, anti-affinity and zonal affinity, bound pods
    counted: every probe's counts = the cluster's bound pods minus the pods it reschedules, against the oracle's
    recount; and the command."""
    rng = np.random.Generator(np.random.PCG64(3100 + seed))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(60, 300)), replace=False))]
    cp = fuzzgen.fuzz_topology_consolidation(sub, 3100 + seed, n_nodes=int(rng.integers(4, 60)),
                                             n_pods=int(rng.integers(20, 250)), all_spot=seed % 4 == 0)
    s2s = seed % 2 == 0
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode, s2s), pyoracle.consolidate(cp, mode, spot_to_spot=s2s))
    assert_commands_equal(device_command(ctx, cp, abi.KP_CONSOLIDATE_BOTH, s2s),
                          pyoracle.consolidate_command(cp, abi.KP_CONSOLIDATE_BOTH, spot_to_spot=s2s))


def test_consolidation_hostname_affinity_case(ctx, golden):
    """Required hostname pod affinity in the probes: a self-selecting class bootstraps a hostname domain only while no
    domain holds a selected pod, counted per probe (the candidates' pods come off)."""
    cp = fuzzgen.fuzz_topology_consolidation(golden[:100], 11, n_nodes=10, n_pods=40)
    cp.cluster.classes[0].topology = [model.TopologyTerm("affinity", model.HOSTNAME, [model.Requirement("app", "Exists")])]
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode), pyoracle.consolidate(cp, mode))
    assert_commands_equal(device_command(ctx, cp, abi.KP_CONSOLIDATE_BOTH),
                          pyoracle.consolidate_command(cp, abi.KP_CONSOLIDATE_BOTH))


@pytest.mark.parametrize("seed", range(12))
def test_fuzz_consolidation_hostname_affinity(ctx, golden, seed):
    """fuzz_topology_consolidation with hostname pod affinity kept (self-selecting and cross-class selectors, bound pods
    holding some domains): probes of both modes and the command against the oracle."""
    rng = np.random.Generator(np.random.PCG64(3700 + seed))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(60, 300)), replace=False))]
    cp = fuzzgen.fuzz_topology_consolidation(sub, 3700 + seed, n_nodes=int(rng.integers(4, 60)),
                                             n_pods=int(rng.integers(20, 250)), all_spot=seed % 4 == 0, host_affinity=True,
                                             n_bound=int(rng.integers(0, 40)))
    s2s = seed % 2 == 0
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode, s2s), pyoracle.consolidate(cp, mode, spot_to_spot=s2s))
    assert_commands_equal(device_command(ctx, cp, abi.KP_CONSOLIDATE_BOTH, s2s),
                          pyoracle.consolidate_command(cp, abi.KP_CONSOLIDATE_BOTH, spot_to_spot=s2s))


def hostname_pod_domains_consolidation(golden, seed):
    """fuzz_topology_consolidation with hostname pod affinity, and hostname requirements (In / NotIn a few node names,
    candidates among them) on the classes with a hostname affinity term: the bootstrap counts only the positive hosts
    the pod admits, a candidate's node counting what its reschedulable pods leave (KpTopoCons.hdom)"""
    rng = np.random.Generator(np.random.PCG64(3900 + seed))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(60, 300)), replace=False))]
    cp = fuzzgen.fuzz_topology_consolidation(sub, 3900 + seed, n_nodes=int(rng.integers(4, 40)),
                                             n_pods=int(rng.integers(20, 200)), host_affinity=True,
                                             n_bound=int(rng.integers(0, 40)))
    names = [e.name for e in cp.cluster.existing]
    for pc in cp.cluster.classes:
        if not any(t.kind == "affinity" and t.key == model.HOSTNAME for t in pc.topology) or rng.random() < 0.3:
            continue
        pick = sorted(set(str(names[int(i)]) for i in rng.integers(0, len(names), size=int(rng.integers(1, 5)))))
        pc.requirements = [r for r in pc.requirements if r.key != model.HOSTNAME]
        pc.requirements.append(model.Requirement(model.HOSTNAME, "In" if rng.random() < 0.5 else "NotIn", pick))
    return cp


@pytest.mark.parametrize("seed", range(12))
def test_fuzz_consolidation_hostname_pod_domains(ctx, golden, seed):
    """Probes and the command over hostname_pod_domains_consolidation against the oracle."""
    cp = hostname_pod_domains_consolidation(golden, seed)
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode), pyoracle.consolidate(cp, mode))
    assert_commands_equal(device_command(ctx, cp, abi.KP_CONSOLIDATE_BOTH),
                          pyoracle.consolidate_command(cp, abi.KP_CONSOLIDATE_BOTH))


# ------------------------------------------------------------------------------------------------
# consolidation over pods with preferences (PREFERENCE_POLICY Respect / Ignore) and MIN_VALUES_POLICY=BestEffort
# ------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def pctx():
    from kpsim import native
    cs = {p: native.Context(0, preference_policy=p) for p in (abi.KP_PREFERENCE_RESPECT, abi.KP_PREFERENCE_IGNORE)}
    yield cs
    for c in cs.values():
        c.close()


@pytest.mark.parametrize("seed", range(16))
@pytest.mark.parametrize("policy", ["respect", "ignore"])
def test_fuzz_consolidation_preferences(pctx, golden, seed, policy):
    """Probes whose pods carry preferred node affinity, ORed required terms, ScheduleAnyway spreads and preferred pod
    (anti-)affinity (fuzzgen.add_preferences), some under MIN_VALUES_POLICY=BestEffort with minValues a NodeClaim can
    miss, some with minValues on the zone label: each probe relaxes a failing pod's preferences one at a time and
    re-queues it (Queue.Push(pod, relaxed) clears lastLen), as the Solve does.  Probes of both modes and the command."""
    pol = abi.KP_PREFERENCE_RESPECT if policy == "respect" else abi.KP_PREFERENCE_IGNORE
    ctx = pctx[pol]
    rng = np.random.Generator(np.random.PCG64(4100 + seed))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(60, 300)), replace=False))]
    cp = fuzzgen.fuzz_preference_consolidation(sub, 4100 + seed, n_nodes=int(rng.integers(4, 60)),
                                               n_pods=int(rng.integers(20, 250)), all_spot=seed % 4 == 0,
                                               best_effort=seed % 3 == 1, zone_min=seed % 4 == 2)
    s2s = seed % 2 == 1
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode, s2s),
                            pyoracle.consolidate(cp, mode, spot_to_spot=s2s, preference_policy=pol))
    assert_commands_equal(device_command(ctx, cp, abi.KP_CONSOLIDATE_BOTH, s2s),
                          pyoracle.consolidate_command(cp, abi.KP_CONSOLIDATE_BOTH, spot_to_spot=s2s, preference_policy=pol))


@pytest.mark.parametrize("seed", range(10))
def test_fuzz_consolidation_topology_preferences(pctx, golden, seed):
    """Probes over pods with topology terms and preferred node-affinity terms (fuzzgen.add_topology_preferences):
    preferences on topology keys and nodeAffinityPolicy Honor spreads, under Respect."""
    ctx = pctx[abi.KP_PREFERENCE_RESPECT]
    rng = np.random.Generator(np.random.PCG64(4300 + seed))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(60, 300)), replace=False))]
    cp = fuzzgen.fuzz_topology_consolidation(sub, 4300 + seed, n_nodes=int(rng.integers(4, 50)),
                                             n_pods=int(rng.integers(20, 200)), all_spot=seed % 4 == 0)
    fuzzgen.add_topology_preferences(rng, cp.cluster)
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode),
                            pyoracle.consolidate(cp, mode, preference_policy=abi.KP_PREFERENCE_RESPECT))


@pytest.mark.parametrize("seed", range(10))
def test_fuzz_consolidation_relaxing_topology(pctx, golden, seed):
    """Probes whose pods relax into specs with new spread groups (fuzzgen.add_relaxing_topology): each probe's
    NewTopology creates the groups its own pods own; a relaxed pod's Topology.Update creates the rest."""
    ctx = pctx[abi.KP_PREFERENCE_RESPECT]
    rng = np.random.Generator(np.random.PCG64(4500 + seed))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(60, 300)), replace=False))]
    cp = fuzzgen.fuzz_topology_consolidation(sub, 4500 + seed, n_nodes=int(rng.integers(4, 50)),
                                             n_pods=int(rng.integers(20, 200)), all_spot=seed % 4 == 0)
    fuzzgen.add_relaxing_topology(rng, cp.cluster)
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode),
                            pyoracle.consolidate(cp, mode, preference_policy=abi.KP_PREFERENCE_RESPECT))


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_consolidation_many_groups(ctx, golden, seed):
    """Probes over classes constrained by more than 8 topology groups and counted by more than 16 (add_many_groups)."""
    rng = np.random.Generator(np.random.PCG64(4700 + seed))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(60, 300)), replace=False))]
    cp = fuzzgen.fuzz_topology_consolidation(sub, 4700 + seed, n_nodes=int(rng.integers(4, 50)),
                                             n_pods=int(rng.integers(20, 200)), all_spot=seed % 4 == 0)
    fuzzgen.add_many_groups(rng, cp.cluster, n_terms=int(rng.integers(14, 30)))
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode), pyoracle.consolidate(cp, mode))


def test_preference_relaxations_in_probes(pctx, golden):
    """The fuzz above relaxes preferences inside the probes (kp_consolidate_stats counter 16): under Respect every
    preference kind; under Ignore only the ORed required node-affinity terms (removeRequiredNodeAffinityTerm)."""
    tot = {}
    for pol in (abi.KP_PREFERENCE_RESPECT, abi.KP_PREFERENCE_IGNORE):
        tot[pol] = 0
        for seed in range(6):
            rng = np.random.Generator(np.random.PCG64(4100 + seed))
            sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(60, 300)), replace=False))]
            cp = fuzzgen.fuzz_preference_consolidation(sub, 4100 + seed, n_nodes=int(rng.integers(4, 60)),
                                                       n_pods=int(rng.integers(20, 250)), all_spot=seed % 4 == 0,
                                                       best_effort=seed % 3 == 1, zone_min=seed % 4 == 2)
            device_probes(pctx[pol], cp, abi.KP_CONSOLIDATE_SINGLE)
            tot[pol] += pctx[pol].consolidate_stats()[1][16]
    assert tot[abi.KP_PREFERENCE_RESPECT] > tot[abi.KP_PREFERENCE_IGNORE], tot


@pytest.mark.parametrize("policy", ["respect", "ignore"])
def test_e2e_preferred_anti_affinity_replace(pctx, golden, policy):
    """Preferred hostname anti-affinity through Solve + consolidation: under Respect each node is replaced and every pod
    keeps a node of its own; under Ignore the Deployment packs onto one node.  Same trajectory as the oracle."""
    import cluster_sim
    import e2e_cases
    pol = abi.KP_PREFERENCE_RESPECT if policy == "respect" else abi.KP_PREFERENCE_IGNORE
    kw = dict(n_nodes=8, respect=policy == "respect")
    dev = e2e_cases.preferred_anti_affinity_replace(golden, cluster_sim.DeviceBackend(pctx[pol]), **kw)
    orc = e2e_cases.preferred_anti_affinity_replace(golden, cluster_sim.OracleBackend(pol), **kw)
    assert _trajectory(dev) == _trajectory(orc)


def test_e2e_preferred_affinity_delete(ctx, golden):
    """Pods preferring an instance category no NodePool offers: the probes relax the preference, then the pods fit the
    remaining nodes (DELETE), until utilisation > 0.6; same trajectory as the oracle."""
    import e2e_cases
    _e2e(ctx, golden, e2e_cases.preferred_affinity_delete)


# ------------------------------------------------------------------------------------------------
# the reference's e2e disruption scenarios (tests/e2e_cases.py) driven through the library: Solve for provisioning,
# kp_consolidate_command for disruption; the reference's end state, and the same command trajectory as the oracle
# ------------------------------------------------------------------------------------------------
def _trajectory(sim):
    return [(c.decision, c.mode, c.candidates, c.type_ids, c.requirements, c.nodepool) for c in sim.commands]


def _e2e(ctx, golden, fn, **kw):
    import cluster_sim
    dev = fn(golden, cluster_sim.DeviceBackend(ctx), **kw)
    orc = fn(golden, cluster_sim.OracleBackend(), **kw)
    assert _trajectory(dev) == _trajectory(orc)
    return dev


@pytest.mark.parametrize("spot", [False, True])
def test_e2e_replace_hostname_spread(ctx, golden, spot):
    """suite_test.go:574-729: 3 x 2xlarge (hostname spread) -> 3 x .large, one single-node REPLACE at a time."""
    import e2e_cases
    sim = _e2e(ctx, golden, e2e_cases.replace_hostname_spread, spot=spot)
    assert [c.decision for c in sim.commands] == [abi.KP_DECISION_REPLACE] * 3 + [abi.KP_DECISION_NONE]


def test_e2e_od_to_spot(ctx, golden):
    """suite_test.go:730-860: on-demand nodes replaced by spot (replacement requirements narrowed to spot)."""
    import e2e_cases
    sim = _e2e(ctx, golden, e2e_cases.od_to_spot)
    assert all("karpenter.sh/capacity-type\t0\t-\t-\t-\tspot\n" in c.requirements for c in sim.commands[:-1])


@pytest.mark.parametrize("spot", [False, True])
def test_e2e_delete_utilization(ctx, golden, spot):
    """suite_test.go:491-573: 100 pods scaled to 40, consolidation deletes nodes until utilisation > 0.6."""
    import e2e_cases
    _e2e(ctx, golden, e2e_cases.delete_utilization, spot=spot)


def test_e2e_anti_affinity_replace(ctx, golden):
    """deprovisioning_test.go:454-523: 20 nodes with hostname anti-affinity, each replaced once the size requirement
    goes (20 deleted, 20 remain)."""
    import e2e_cases
    _e2e(ctx, golden, e2e_cases.anti_affinity_replace, n_nodes=20)


def test_e2e_multi_delete(ctx, golden):
    """deprovisioning_test.go:399-453: 200 nodes at 20 pods, scaled to 20%: 160 deleted by multi-node consolidation."""
    import e2e_cases
    sim = _e2e(ctx, golden, e2e_cases.multi_delete, n_nodes=200)
    assert sim.commands[0].mode == abi.KP_CONSOLIDATE_MULTI and len(sim.nodes) == 40


@pytest.mark.parametrize("name", ["budget_empty_delete", "budget_nonempty_delete", "budget_replace", "budget_blocking"])
def test_e2e_budgets(ctx, golden, name):
    """test/suites/consolidation/suite_test.go:188-453: NodePool disruption budgets filter the candidates caller-side
    (Emptiness, then MultiNodeConsolidation over the budget-capped prefix, then SingleNodeConsolidation); the device
    command trajectory equals the oracle's and meets the reference's per-step bound and end state."""
    import e2e_cases
    _e2e(ctx, golden, getattr(e2e_cases, name))


@pytest.mark.parametrize("seed", range(3))
def test_consolidation_many_nodepools(ctx, golden, seed):
    """40-60 NodePools: candidates' capacity back into their own pool's limits, replacements from any pool."""
    rng = np.random.Generator(np.random.PCG64(5300 + seed))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=200, replace=False))]
    cp = fuzzgen.fuzz_consolidation(sub, 5300 + seed, n_nodes=40, n_pods=200,
                                    n_pools=int(rng.integers(40, 61)))
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode), pyoracle.consolidate(cp, mode))


@pytest.mark.parametrize("seed", range(8))
def test_consolidation_wide_axes(ctx, golden, seed):
    """Pods requesting 7-9 resource axes (pod ENIs, EFA, GPUs, Neuron, Gaudi besides cpu / memory / pods): the probes
    check the axes past their registers per candidate node from HBM; probes of both modes and the command vs the
    oracle."""
    rng = np.random.Generator(np.random.PCG64(5500 + seed))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(100, 300)), replace=False))]
    cp = fuzzgen.fuzz_consolidation(sub, 5500 + seed, n_nodes=int(rng.integers(10, 80)),
                                    n_pods=int(rng.integers(50, 300)), all_spot=seed % 4 == 0)
    fuzzgen.add_extra_resources(rng, cp.cluster)
    active = (cp.cluster.pods.requests != 0).any(0).sum()
    assert active > 6, active
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode), pyoracle.consolidate(cp, mode))
    assert_commands_equal(device_command(ctx, cp, abi.KP_CONSOLIDATE_BOTH),
                          pyoracle.consolidate_command(cp, abi.KP_CONSOLIDATE_BOTH))


def test_consolidation_wide_catalog(ctx, golden):
    """Probes over a 1,300-type catalog (32 option words; OrderByPrice / Truncate over the wider option set)."""
    cat = synth.widen_catalog(golden, 1300)
    for seed in range(2):
        cp = fuzzgen.fuzz_consolidation(cat, 5700 + seed, n_nodes=40, n_pods=200, all_spot=seed == 1)
        for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
            assert_probes_equal(device_probes(ctx, cp, mode), pyoracle.consolidate(cp, mode))


# ---- topology groups shared by TopologyGroup.Hash() identity in the probes (row N1): each probe's NewTopology creates
# the group from the first of its pods (pending, then its candidates' pods) that owns it ----

@pytest.mark.parametrize("pending_a", [True, False])
def test_shared_identity_probes(ctx, golden, pending_a):
    """pending_a: a pending pod of A's Deployment comes first in every probe, so the group is A's (filter zone In
    [1a, 1b]) in all of them.  Without it probe 0 creates the group from A's pod and probe 1 from B's: one variant group
    per filter, each probe starting with its own first owner's variant born.  Probes and command against the oracle."""
    import cons_cases
    cp = cons_cases.shared_identity_cluster(golden, pending_a)
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode), pyoracle.consolidate(cp, mode))
    assert_commands_equal(device_command(ctx, cp, abi.KP_CONSOLIDATE_BOTH),
                          pyoracle.consolidate_command(cp, abi.KP_CONSOLIDATE_BOTH))


def test_shared_identity_selection_refused(ctx, golden):
    """One identity whose owners select different pods (a selector pair hashstructure folds away) and whose first owner
    differs between probes: variant groups need one selection, so the pass is refused (KP_E_UNSUPPORTED)."""
    import cons_cases
    from kpsim import native
    cp = cons_cases.shared_identity_cluster(golden, pending_a=False, selection=True)
    with pytest.raises(native.KpError) as e:
        device_probes(ctx, cp, abi.KP_CONSOLIDATE_SINGLE)
    assert e.value.status == abi.KP_E_UNSUPPORTED and "different selections" in str(e.value)


@pytest.mark.parametrize("seed", range(12))
def test_fuzz_consolidation_shared_identity(ctx, golden, seed):
    """fuzzgen.fuzz_shared_identity_consolidation: sibling Deployments with equal spread identities and different Honor
    filter values / minDomains over topology-constrained clusters; even seeds put a pod of each family first among the
    pending pods (one first owner for every probe), odd seeds leave the first owner to each probe (variant groups).
    Both modes and the command against the oracle."""
    rng = np.random.Generator(np.random.PCG64(4500 + seed))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(60, 300)), replace=False))]
    cp = fuzzgen.fuzz_shared_identity_consolidation(sub, 4500 + seed, n_nodes=int(rng.integers(4, 50)),
                                                    n_pods=int(rng.integers(20, 200)), pending_owner=seed % 2 == 0)
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode), pyoracle.consolidate(cp, mode))
    assert_commands_equal(device_command(ctx, cp, abi.KP_CONSOLIDATE_BOTH),
                          pyoracle.consolidate_command(cp, abi.KP_CONSOLIDATE_BOTH))


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_consolidation_more_than_16_constraining_groups(ctx, golden, seed):
    """Probes over classes constrained by more than 16 topology groups (add_many_groups with 36-47 terms)."""
    rng = np.random.Generator(np.random.PCG64(4800 + seed))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(60, 300)), replace=False))]
    cp = fuzzgen.fuzz_topology_consolidation(sub, 4800 + seed, n_nodes=int(rng.integers(4, 50)),
                                             n_pods=int(rng.integers(20, 200)), all_spot=seed % 4 == 0)
    fuzzgen.add_many_groups(rng, cp.cluster, n_terms=int(rng.integers(36, 48)))
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode), pyoracle.consolidate(cp, mode))
