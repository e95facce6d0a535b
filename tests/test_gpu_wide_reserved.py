"""GPU: catalogs with more reserved offerings than one 64-bit word (up to KP_MAX_RO = 1024) — Solve's ReservationManager
and FinalizeScheduling, and the consolidation probes' reservations, over multi-word reservation tables (ResvTab.w words
per row, reservation capacities by dense reservation id), bit-identical to the oracle."""
import numpy as np
import pytest

import fuzzgen
import kat_cases as KC
import parity
import pyoracle
from kpsim import abi, model, native, synth
from test_gpu_consolidation import assert_commands_equal, assert_probes_equal, device_command, device_probes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = native.Context(0)
    yield c
    c.close()


def _n_reserved(cat):
    return sum(1 for it in cat for o in it.offerings if o.capacity_type == "reserved")


def _held(reqs):
    return sum(1 for q in reqs if KC.RESVID in q and not q[KC.RESVID][0])


@pytest.fixture(scope="module")
def cat200(golden):
    return synth.wide_reservation_catalog(golden, 200)


@pytest.mark.parametrize("n", [500, 5000, 20000])
def test_wide_config5_parity(ctx, cat200, n):
    """config 5's workload over a 200-reservation catalog (76 types, up to 4 reservations each)."""
    assert _n_reserved(cat200) == 200
    prob = synth.config5(n_pods=n, catalog=cat200)
    cv = model.CatalogView(cat200)
    dev = parity.run_device(ctx, prob, cv)
    parity.assert_same(dev, parity.run_oracle(prob, cv))
    assert _held(dev[1]) > 0


def wide_scarce_problem(golden, seed, n_pods=1500):
    """65-700 reservations of capacity 0-3: strict-mode failures, releases and re-reservations across words."""
    rng = np.random.Generator(np.random.PCG64(2000 + seed))
    n_res = int(rng.choice([65, 128, 300, 700]))
    cat = synth.wide_reservation_catalog(golden, n_res, max_per_type=int(rng.integers(1, 6)), seed=synth.SEED + seed,
                                         expiring_frac=0.2, rcap=(0, 4))
    for it in cat:
        for o in it.offerings:
            if o.capacity_type == "reserved":
                o.available = o.available and o.reservation_capacity > 0
    prob = synth.config2(n_pods=n_pods, n_classes=60, catalog=cat, seed=synth.SEED + seed)
    cts = [["reserved"], ["reserved", "on-demand"], ["reserved", "spot", "on-demand"], ["spot", "on-demand"]]
    for np_ in prob.nodepools:
        np_.requirements = [r for r in np_.requirements if r.key != model.CAPACITY_TYPE]
        np_.requirements.append(model.Requirement(model.CAPACITY_TYPE, "In", cts[int(rng.integers(len(cts)))]))
    return prob


@pytest.mark.parametrize("seed", range(10))
def test_wide_reservation_fuzz(ctx, golden, seed):
    prob = wide_scarce_problem(golden, seed)
    assert _n_reserved(prob.catalog) > 64
    cv = model.CatalogView(prob.catalog)
    parity.assert_same(parity.run_device(ctx, prob, cv), parity.run_oracle(prob, cv))


def _wide_consolidation(golden, seed, full_cluster=False):
    rng = np.random.Generator(np.random.PCG64(2300 + seed))
    sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(120, 300)), replace=False))]
    cat = synth.wide_reservation_catalog(sub, int(rng.integers(65, 260)), max_per_type=4, seed=2300 + seed,
                                         rcap=(0, 6))
    cp = fuzzgen.fuzz_consolidation(cat, 2300 + seed, n_nodes=int(rng.integers(4, 60)),
                                    n_pods=int(rng.integers(20, 250)), all_spot=seed % 4 == 0,
                                    pending_frac=0.0 if full_cluster else 0.15)
    for np_ in cp.cluster.nodepools:
        for r in np_.requirements:
            if r.key == model.CAPACITY_TYPE and r.op == "In" and rng.random() < 0.8:
                r.values = sorted(set(r.values) | {"reserved"})
    if full_cluster:
        for n in cp.cluster.existing:
            n.available = np.minimum(n.available, 0)
    return cp


@pytest.mark.parametrize("seed", range(10))
def test_wide_consolidation_fuzz(ctx, golden, seed):
    cp = _wide_consolidation(golden, seed, full_cluster=seed % 2 == 0)
    assert _n_reserved(cp.cluster.catalog) > 64
    s2s = seed % 3 == 1
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode, s2s), pyoracle.consolidate(cp, mode, spot_to_spot=s2s))


def test_wide_consolidation_command(ctx, golden):
    """kp_consolidate_command's replacement over a wide catalog: the reservation-id requirement lists the held
    reservations (any of the catalog's words)."""
    n_replace = n_held = 0
    for seed in range(14):
        cp = _wide_consolidation(golden, 50 + seed, full_cluster=True)
        for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
            dev = device_command(ctx, cp, mode, False)
            assert_commands_equal(dev, pyoracle.consolidate_command(cp, mode))
            n_replace += dev.decision == abi.KP_DECISION_REPLACE
            n_held += dev.decision == abi.KP_DECISION_REPLACE and dev.n_reserved > 0
    assert n_replace >= 4 and n_held >= 3


def test_wide_reservation_id_requirement(ctx, cat200):
    """A pod requirement on karpenter.k8s.aws/capacity-reservation-id over a catalog with more reservation IDs than one
    64-value word: the key's per-type values are the type's ResvTab rows (KF_RESV_ROWS), bit-exact with the oracle."""
    prob = synth.config5(n_pods=2000, catalog=cat200)
    rid = next(o.reservation_id for it in cat200 for o in it.offerings if o.capacity_type == "reserved")
    prob.classes[0].requirements = list(prob.classes[0].requirements) + [
        model.Requirement(model.RESERVATION_ID, "In", [rid])]
    cv = model.CatalogView(cat200)
    dev = parity.run_device(ctx, prob, cv)
    parity.assert_same(dev, parity.run_oracle(prob, cv))
    placed = dev[0].pod_result[prob.pods.class_id == 0]
    assert (placed >= 0).any()


@pytest.mark.parametrize("n", [2000, 20000])
def test_wide_reservation_id_selection_config5(ctx, cat200, n):
    """config 5 over the 200-reservation catalog with pods and NodePools selecting reservations by ID (In / NotIn /
    Exists / DoesNotExist; website odcrs.md:53-57), at 2k and 20k pods."""
    prob = synth.config5(n_pods=n, catalog=cat200)
    fuzzgen.add_reservation_id_requirements(np.random.Generator(np.random.PCG64(77 + n)), prob)
    cv = model.CatalogView(cat200)
    dev = parity.run_device(ctx, prob, cv)
    parity.assert_same(dev, parity.run_oracle(prob, cv))
    assert _held(dev[1]) > 0


@pytest.mark.parametrize("seed", range(10))
def test_wide_reservation_id_fuzz(ctx, golden, seed):
    """wide_scarce_problem (65-700 reservations, capacity 0-3) with reservation-ID selections on pods and NodePools."""
    prob = wide_scarce_problem(golden, 40 + seed)
    fuzzgen.add_reservation_id_requirements(np.random.Generator(np.random.PCG64(4100 + seed)), prob)
    cv = model.CatalogView(prob.catalog)
    parity.assert_same(parity.run_device(ctx, prob, cv), parity.run_oracle(prob, cv))


@pytest.mark.parametrize("seed", range(8))
def test_wide_reservation_id_consolidation_fuzz(ctx, golden, seed):
    """Consolidation probes and the command over 65-260 reservations with reservation-ID selections."""
    cp = _wide_consolidation(golden, 60 + seed, full_cluster=seed % 2 == 0)
    fuzzgen.add_reservation_id_requirements(np.random.Generator(np.random.PCG64(4200 + seed)), cp.cluster)
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode), pyoracle.consolidate(cp, mode))
    assert_commands_equal(device_command(ctx, cp, abi.KP_CONSOLIDATE_BOTH),
                          pyoracle.consolidate_command(cp, abi.KP_CONSOLIDATE_BOTH))


def test_over_max_reserved_offerings_refused(ctx, golden):
    """More than KP_MAX_RO (1024) reserved offerings: refused loudly."""
    cat = synth.wide_reservation_catalog(golden, 1100, max_per_type=4)
    ctx.upload_catalog(model.CatalogView(cat))
    prob = synth.config2(n_pods=200, catalog=cat)
    with pytest.raises(native.KpError) as e:
        ctx.prepare(model.SolveInputView(prob))
    assert e.value.status == abi.KP_E_UNSUPPORTED
