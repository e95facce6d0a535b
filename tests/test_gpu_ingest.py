"""GPU: Solve over a catalog built by the library's ingestion path (kp_catalog_build → kp_catalog_upload).

The reference's label / packing known answers (tests/kat_cases.py) whose catalog is the plain envtest catalog run on the
ingested catalog: the device must reach the Its' expected values and be bit-identical to the oracle run on the Python
host builder's catalog — so ingestion → upload → Solve is exact end to end."""
import numpy as np
import pytest

import kat_cases as KC
import parity
from kpsim import ingest, model, native, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = native.Context(0)
    yield c
    c.close()


def _same_catalog(a, b):
    if [x.name for x in a] != [x.name for x in b]:
        return False
    for x, y in zip(a, b):
        lx = {k: sorted(v) if v else None for k, v in x.labels.items()}
        ly = {k: sorted(v) if v else None for k, v in y.labels.items()}
        if lx != ly or not (x.capacity == y.capacity).all() or not (x.allocatable == y.allocatable).all():
            return False
        ox = [(o.capacity_type, o.zone, o.price, o.available, o.zone_id) for o in x.offerings]
        oy = [(o.capacity_type, o.zone, o.price, o.available, o.zone_id) for o in y.offerings]
        if ox != oy:
            return False
    return True


@pytest.mark.parametrize("mk", KC.ENVTEST_CASES, ids=[c.__name__ for c in KC.ENVTEST_CASES])
def test_kat_on_ingested_catalog(ctx, fx, mk):
    """Every known answer over the envtest catalog, that catalog built by kp_catalog_build with the case's own edits
    (ICE marks, spot prices, MakeInstances types, the Windows NodeClass; kat_cases.native_catalog): the device reaches
    the It's expected values and equals the oracle over the host builder's catalog."""
    k = mk(fx)
    nats, types = KC.native_catalog(k.problem.catalog)
    assert _same_catalog(types, k.problem.catalog)
    view = nats[0] if len(nats) == 1 else model.CatalogView(types)  # several NodeClasses: the built types, merged
    dev = parity.run_device(ctx, k.problem, view)
    k.check(k.problem, *dev)
    parity.assert_same(dev, parity.run_oracle(k.problem, model.CatalogView(k.problem.catalog)))


@pytest.mark.parametrize("fam", ["AL2023", "Bottlerocket", "Windows2022"])
def test_seeded_solve_on_ingested_catalog(ctx, fx, fam):
    """A seeded config-2-style pod mix over the ingested envtest catalog equals the oracle over the host builder's."""
    from kpsim import catalog
    nat = ingest.fake_catalog(fx, nodeclass=ingest.NodeClass(ami_family=fam))
    py = catalog.fake_catalog(fx=fx, opts=catalog.TypeOptions(ami_family=fam))
    assert _same_catalog(nat.instance_types(), py)
    prob = synth.subsample(synth.config2(n_pods=3000, catalog=py), 600)
    dev = parity.run_device(ctx, prob, nat)
    parity.assert_same(dev, parity.run_oracle(prob, model.CatalogView(py)))
    assert int((dev[0].pod_result == -1).sum()) < prob.pods.n
