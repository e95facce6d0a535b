"""CPU: the oracle (Solve, then launch where the It inspects CreateFleet) against the reference suites' known answers
(tests/kat_cases.py), and the catalog builder's labels / capacity-block offerings against the Its that inspect them."""
import pytest

import kat_cases as KC
import parity
import pyoracle
from kpsim import abi, catalog, model
from kpsim.model import CAPACITY_TYPE, RESERVATION_ID, RESERVATION_TYPE, ZONE


def run_kat_oracle(k):
    res, reqs = parity.run_oracle(k.problem)
    k.check(k.problem, res, reqs)
    lres = None
    if k.launch_check:
        lreqs = KC.nodeclaim_launch_requests(k.problem, res, reqs)
        st, lres = pyoracle.launch_select(model.CatalogView(k.problem.catalog), model.LaunchBatchView(lreqs), 60)
        assert st == abi.KP_OK
        k.launch_check(k.problem.catalog, lreqs, lres)
    return res, reqs, lres


@pytest.mark.parametrize("mk", KC.CASES, ids=KC.ids())
def test_kat_oracle(fx, mk):
    run_kat_oracle(mk(fx))


def _row(cat, name):
    return next(it for it in cat if it.name == name)


LABEL_ALIASES = {"failure-domain.beta.kubernetes.io/region", "failure-domain.beta.kubernetes.io/zone",
                 "beta.kubernetes.io/arch", "beta.kubernetes.io/os", "beta.kubernetes.io/instance-type",
                 "topology.ebs.csi.aws.com/zone", model.NODEPOOL, CAPACITY_TYPE, ZONE, "topology.k8s.aws/zone-id"}


@pytest.mark.parametrize("name,labels", [("g4dn.8xlarge", KC.G4DN_LABELS), ("inf2.xlarge", KC.INF2_LABELS)])
def test_compute_requirements_label_rows(fx, name, labels):
    """computeRequirements (types.go:158-299) on the pkg/fake type yields every instance-type label value the label Its
    select on (suite_test.go:220-394); offering-level keys (zone, zone-id, capacity type) come from the offerings."""
    it = _row(catalog.fake_catalog(fx=fx), name)
    for k, v in labels.items():
        if k in LABEL_ALIASES:
            continue
        assert it.labels.get(k) == [v], (k, it.labels.get(k), v)
    assert Z1A_OFFER(it)


def Z1A_OFFER(it):
    return any(o.zone == KC.Z1A and o.zone_id == "tstz1-1a" and o.capacity_type == "on-demand" and o.available
               for o in it.offerings)


def test_g4dn_has_no_accelerator_labels(fx):
    """The TODO at suite_test.go:251: the accelerator selectors are satisfied by another type, not by g4dn."""
    it = _row(catalog.fake_catalog(fx=fx), "g4dn.8xlarge")
    assert it.labels.get(KC.AWS + "instance-accelerator-name") is None


def test_windows_rows(fx):
    win = catalog.fake_catalog(fx=fx, opts=catalog.TypeOptions(ami_family="Windows2022"))
    m5 = _row(win, "m5.large")
    assert m5.labels["kubernetes.io/os"] == ["windows"]
    assert m5.labels["node.kubernetes.io/windows-build"] == ["10.0.20348"]
    assert _row(win, "c6g.large").labels["kubernetes.io/os"] is None   # arm64: getOS → [] (types.go:301-309)
    lin = catalog.fake_catalog(fx=fx)
    assert _row(lin, "m5.large").labels["node.kubernetes.io/windows-build"] is None


@pytest.mark.parametrize("state", ["active", "expiring"])
def test_capacity_block_offering(fx, state):
    """suite_test.go:2892-2947: exactly one reserved offering for c6g.large, with the reservation's zone, type, id and
    capacity; available unless the block is expiring."""
    it = _row(KC.capacity_block_catalog(fx, state), "c6g.large")
    res = [o for o in it.offerings if o.capacity_type == "reserved"]
    assert len(res) == 1
    o = res[0]
    assert o.zone == KC.Z1A and o.reservation_type == "capacity-block" and o.reservation_id == "cr-123"
    assert o.label(RESERVATION_ID) == (abi.KP_LABEL_IN, "cr-123")
    assert o.label(RESERVATION_TYPE) == (abi.KP_LABEL_IN, "capacity-block")
    assert o.available == (state != "expiring") and o.reservation_capacity == 1
    assert it.labels[CAPACITY_TYPE] == ["on-demand", "spot", "reserved"]


@pytest.mark.parametrize("state", ["active", "expiring"])
def test_capacity_block_launch_oracle(fx, state):
    """A reserved NodeClaim for c6g.large launches into the block while it is active, and is an ICE once it expires."""
    cat = KC.capacity_block_catalog(fx, state)
    rq = model.LaunchRequest([model.Requirement(CAPACITY_TYPE, "In", ["reserved"]),
                              model.Requirement(model.INSTANCE_TYPE, "In", ["c6g.large"])],
                             __import__("numpy").zeros(len(model.RESOURCES), "int64"))
    st, lres = pyoracle.launch_select(model.CatalogView(cat), model.LaunchBatchView([rq]), 60)
    assert st == abi.KP_OK
    row = lres.rows[0]
    if state == "active":
        assert int(row["status"]) == abi.KP_OK and int(row["capacity_type"]) == abi.KP_CT_RESERVED
        assert [(n, z, ct) for n, z, ct, _ in KC.overrides(cat, lres, 0)] == [("c6g.large", KC.Z1A, "reserved")]
    else:
        assert int(row["status"]) == abi.KP_E_INSUFFICIENT_CAPACITY


@pytest.mark.parametrize("mk", KC.RESV_CASES, ids=KC.resv_ids())
def test_kat_reserved_oracle(fx, mk):
    run_kat_oracle(mk(fx))
