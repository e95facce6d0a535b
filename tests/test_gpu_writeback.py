"""GPU ctx: the NodeClaim write-back of a launched instance (kp_nodeclaim_labels = CloudProvider.instanceToNodeClaim,
pkg/cloudprovider/cloudprovider.go:381-444), chained after kp_launch_select and the kwok CreateFleet pick.

Reference-pinned: pkg/cloudprovider/suite_test.go:289-303 (the zone-id label is the zone's subnet ZoneID),
:1409-1440 (vpc.amazonaws.com/efa is advertised only when the NodeClaim requested it), :1472-1480 (a reserved launch
carries its reservation).  The label rule (single-valued requirements only, reservation keys excluded) is checked
against a restatement over the catalog model on every type of the envtest catalog."""
import numpy as np
import pytest

from kpsim import abi, catalog, launch, model, native, synth
from kpsim.model import CAPACITY_TYPE, INSTANCE_TYPE, RESERVATION_ID, RESERVATION_TYPE, ZONE, ZONE_ID, Requirement

pytestmark = pytest.mark.gpu
EFA = "vpc.amazonaws.com/efa"


@pytest.fixture(scope="module")
def ctx():
    c = native.Context(0)
    yield c
    c.close()


def expected_labels(it, o, nodepool=None, zone_id=None):
    """instanceToNodeClaim's labels restated over the catalog model."""
    want = {k: v[0] for k, v in it.labels.items()
            if v is not None and len(v) == 1 and k not in (RESERVATION_ID, RESERVATION_TYPE)}
    want[ZONE] = o.zone
    if zone_id or o.zone_id:
        want[ZONE_ID] = zone_id or o.zone_id
    want[CAPACITY_TYPE] = o.capacity_type
    if o.capacity_type == "reserved":
        want[RESERVATION_ID] = o.reservation_id
        want[RESERVATION_TYPE] = o.reservation_type
    if nodepool:
        want[model.NODEPOOL] = nodepool
    return want


def rows_of(cat):
    rows, r = [], 0
    for t, it in enumerate(cat):
        for o in it.offerings:
            rows.append((t, o, r))
            r += 1
    return rows


def test_labels_every_offering(ctx, fx):
    cat = catalog.fake_catalog(fx=fx)
    ctx.upload_catalog(model.CatalogView(cat))
    for t, o, r in rows_of(cat):
        got, cap, alloc = ctx.nodeclaim_labels(t, r, nodepool="default")
        assert got == expected_labels(cat[t], o, "default"), (cat[t].name, o)
        nz = cat[t].allocatable != 0
        efa = model.RIDX[EFA]
        nz[efa] = False
        np.testing.assert_array_equal(alloc[nz], cat[t].allocatable[nz])
        assert alloc[efa] == 0 and cap[efa] == 0


def test_zone_id_is_the_subnet_zone_id(ctx, fx):
    """suite_test.go:289-303: the launched zone's subnet ZoneID (envtest subnets test-zone-1a → tstz1-1a)."""
    cat = catalog.fake_catalog(fx=fx)
    ctx.upload_catalog(model.CatalogView(cat))
    n = 0
    for t, o, r in rows_of(cat):
        if not o.zone_id:  # e.g. a local zone without an envtest subnet: the type's own label (if single) stays
            continue
        n += 1
        got, _, _ = ctx.nodeclaim_labels(t, r)
        assert got[ZONE] == o.zone and got[ZONE_ID] == o.zone_id and o.zone_id.startswith("tstz1-")
        got, _, _ = ctx.nodeclaim_labels(t, r, zone_id="use1-az9")  # the EC2NodeClass status subnet wins
        assert got[ZONE_ID] == "use1-az9"
    assert n > 12


@pytest.mark.parametrize("efa_requested", [True, False])
def test_efa_only_when_requested(ctx, fx, efa_requested):
    """suite_test.go:1409-1440: dl1.24xlarge, EFA advertised in Allocatable only if the NodeClaim requested it."""
    cat = catalog.fake_catalog(fx=fx)
    cv = model.CatalogView(cat)
    ctx.upload_catalog(cv)
    rq = np.zeros(model.R, np.int64)
    if efa_requested:
        rq[model.RIDX[EFA]] = 1000
    req = model.LaunchRequest([Requirement(INSTANCE_TYPE, "In", ["dl1.24xlarge"])], rq)
    res = ctx.launch_select(model.LaunchBatchView([req]), 60)
    assert int(res.rows[0]["status"]) == abi.KP_OK
    t, row = launch.fleet_pick(cat, res, 0)
    assert cat[t].name == "dl1.24xlarge" and cat[t].allocatable[model.RIDX[EFA]] > 0
    _, cap, alloc = ctx.nodeclaim_labels(t, row, efa_enabled=efa_requested)
    assert (alloc[model.RIDX[EFA]] > 0) == efa_requested and (cap[model.RIDX[EFA]] > 0) == efa_requested


def test_reserved_launch_carries_its_reservation(ctx, golden):
    """suite_test.go:1472-1480: a reserved launch's NodeClaim is labelled with its reservation id and type; on-demand
    and spot launches of the same type are not (the type's reservation-id requirement lists every reservation)."""
    cat = synth.config5_catalog(golden)
    ctx.upload_catalog(model.CatalogView(cat))
    seen = 0
    for t, o, r in rows_of(cat):
        if not any(x.capacity_type == "reserved" for x in cat[t].offerings):
            continue
        got, _, _ = ctx.nodeclaim_labels(t, r)
        assert got == expected_labels(cat[t], o)
        assert (RESERVATION_ID in got) == (o.capacity_type == "reserved")
        seen += o.capacity_type == "reserved"
    assert seen >= 40


def test_bad_indices(ctx, fx):
    cat = catalog.fake_catalog(fx=fx)
    ctx.upload_catalog(model.CatalogView(cat))
    with pytest.raises(native.KpError):
        ctx.nodeclaim_labels(0, len(cat[0].offerings))  # an offering row of type 1
    with pytest.raises(native.KpError):
        ctx.nodeclaim_labels(len(cat), 0)
