"""GPU: the reference suites' known answers (tests/kat_cases.py) through the device — kp_solve, then kp_launch_select
on the device's own NodeClaims — asserting the Its' expected values, and bit-identical to the oracle."""
import numpy as np
import pytest

import kat_cases as KC
import launch_cases as LC
import parity
import pyoracle
from kpsim import abi, model, native

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = native.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("mk", KC.CASES + KC.RESV_CASES, ids=KC.ids() + KC.resv_ids())
def test_kat_device(ctx, fx, mk):
    k = mk(fx)
    cv = model.CatalogView(k.problem.catalog)
    dev = parity.run_device(ctx, k.problem, cv)
    k.check(k.problem, *dev)
    parity.assert_same(dev, parity.run_oracle(k.problem, cv))
    if k.launch_check:
        lreqs = KC.nodeclaim_launch_requests(k.problem, *dev)
        b = model.LaunchBatchView(lreqs)
        lres = ctx.launch_select(b, 60)
        k.launch_check(k.problem.catalog, lreqs, lres)
        st, orc = pyoracle.launch_select(cv, b, 60)
        assert st == abi.KP_OK
        LC.assert_same(lres, orc)


@pytest.mark.parametrize("state", ["active", "expiring"])
def test_capacity_block_launch_device(ctx, fx, state):
    cat = KC.capacity_block_catalog(fx, state)
    ctx.upload_catalog(model.CatalogView(cat))
    rq = model.LaunchRequest([model.Requirement(model.CAPACITY_TYPE, "In", ["reserved"]),
                              model.Requirement(model.INSTANCE_TYPE, "In", ["c6g.large"])],
                             np.zeros(len(model.RESOURCES), np.int64))
    lres = ctx.launch_select(model.LaunchBatchView([rq]), 60)
    row = lres.rows[0]
    if state == "active":
        assert int(row["status"]) == abi.KP_OK and int(row["capacity_type"]) == abi.KP_CT_RESERVED
        assert [(n, z, c) for n, z, c, _ in KC.overrides(cat, lres, 0)] == [("c6g.large", KC.Z1A, "reserved")]
    else:
        assert int(row["status"]) == abi.KP_E_INSUFFICIENT_CAPACITY
