"""GPU: reserved capacity in Solve — the ReservationManager (strict mode) and FinalizeScheduling's reservation-id
requirement on the device, bit-identical to the oracle (config 5 and seeded reservation-scarce problems)."""
import numpy as np
import pytest

import kat_cases as KC
import parity
from kpsim import model, native, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = native.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def cat5(golden):
    return synth.config5_catalog(golden)


def _held(reqs):
    return sum(1 for q in reqs if KC.RESVID in q and not q[KC.RESVID][0])


@pytest.mark.parametrize("n", [300, 3000, 20000])
def test_config5_parity(ctx, cat5, n):
    prob = synth.config5(n_pods=n, catalog=cat5)
    cv = model.CatalogView(cat5)
    dev = parity.run_device(ctx, prob, cv)
    orc = parity.run_oracle(prob, cv)
    parity.assert_same(dev, orc)
    assert _held(dev[1]) > 0


def scarce_problem(golden, seed, n_pods=1500):
    """Few reservations with capacities 1-3 on popular types, every NodePool admitting reserved capacity: strict-mode
    failures, releases (a NodeClaim narrowed off its reserved types) and re-reservations all occur."""
    rng = np.random.Generator(np.random.PCG64(1000 + seed))
    cat = synth.config5_catalog(golden, n_default=int(rng.integers(4, 12)), n_block=int(rng.integers(0, 6)),
                                seed=synth.SEED + seed, expiring_frac=0.2)
    for it in cat:
        for o in it.offerings:
            if o.capacity_type == "reserved":
                o.reservation_capacity = int(rng.integers(0, 4))
                o.available = o.available and o.reservation_capacity > 0
    prob = synth.config2(n_pods=n_pods, n_classes=60, catalog=cat, seed=synth.SEED + seed)
    cts = [["reserved"], ["reserved", "on-demand"], ["reserved", "spot", "on-demand"], ["spot", "on-demand"]]
    for i, np_ in enumerate(prob.nodepools):
        np_.requirements = [r for r in np_.requirements if r.key != model.CAPACITY_TYPE]
        np_.requirements.append(model.Requirement(model.CAPACITY_TYPE, "In", cts[int(rng.integers(len(cts)))]))
    return prob


@pytest.mark.parametrize("seed", range(12))
def test_reservation_fuzz(ctx, golden, seed):
    prob = scarce_problem(golden, seed)
    cv = model.CatalogView(prob.catalog)
    parity.assert_same(parity.run_device(ctx, prob, cv), parity.run_oracle(prob, cv))


def test_reserved_capacity_gate_off(golden):
    """FEATURE_GATES ReservedCapacity=false: no reservations are tracked (offeringsToReserve returns nothing)."""
    import pyoracle
    prob = scarce_problem(golden, 3)
    cv = model.CatalogView(prob.catalog)
    c = native.Context(0, reserved_capacity=0)
    try:
        dev = parity.run_device(c, prob, cv)
    finally:
        c.close()
    o = pyoracle.solve(prob, cv, reserved_capacity=0)
    orc = (o.results, [model.parse_requirements_blob(o.requirements(i)) for i in range(o.results.n_nodeclaims)])
    parity.assert_same(dev, orc)
    assert _held(dev[1]) == 0


def test_config5_200k_digest(ctx, golden):
    """BASELINE configs[4] at full size (200k pods): every output field equals the committed oracle digest
    (tests/golden/gen_scale_digest.py config5_200k; the oracle needs ~15 min at this size)."""
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "scale_digests.json")) as f:
        want = json.load(f)["config5_200k"]
    prob = synth.config5(n_pods=want["n_pods"], golden=golden)
    got = parity.result_digest(parity.run_device(ctx, prob))
    for k, v in got.items():
        assert v == want[k], k
