"""Launch-time selection (filter.go chain + Truncate + getCapacityType): the oracle against the reference's own
filter_test.go cases (tests/launch_cases.py), plus properties of the instancetype suite on the golden catalog."""
import numpy as np
import pytest

import launch_cases as LC
import pyoracle
from kpsim import abi, model, synth


@pytest.mark.parametrize("mk", LC.CASES, ids=[getattr(c, "__name__", "case%d" % i) for i, c in enumerate(LC.CASES)])
def test_oracle_filter_cases(mk):
    cat, reqs, expect = mk()
    st, res = pyoracle.launch_select(model.CatalogView(cat), model.LaunchBatchView(reqs), 60)
    assert st == abi.KP_OK
    LC.check(cat, res, expect)


def test_oracle_golden_properties(golden):
    """instancetype/suite_test.go:409-453 (≤ 60 overrides, all among the cheapest) and :454-525 (every spot offering
    launched is no dearer than the cheapest on-demand one) on the golden catalog."""
    cat = golden
    reqs = [LC.req(LC.ct("spot", "on-demand"), cpu=2000), LC.req(LC.ct("on-demand"), cpu=1000)]
    cv = model.CatalogView(cat)
    st, res = pyoracle.launch_select(cv, model.LaunchBatchView(reqs), 60)
    assert st == abi.KP_OK
    rows = [(t, o) for t in range(len(cat)) for o in cat[t].offerings]
    for i, cts in enumerate([("spot", "on-demand"), ("on-demand",)]):
        assert res.rows[i]["status"] == abi.KP_OK and res.rows[i]["n_types"] == 60
        prices = [min(o.price for o in cat[int(t)].offerings if o.available and o.capacity_type in cts)
                  for t in res.types(i)]
        assert prices == sorted(prices)
    spot = [rows[int(o)][1] for o in res.offerings(0)]
    assert res.rows[0]["capacity_type"] == abi.KP_CT_SPOT and all(o.capacity_type == "spot" for o in spot)


def test_oracle_config5_batch_runs(golden):
    cat = synth.config5_catalog(golden)
    reqs = synth.launch_requests(cat, n=50)
    st, res = pyoracle.launch_select(model.CatalogView(cat), model.LaunchBatchView(reqs), 60)
    assert st == abi.KP_OK
    assert (res.rows["status"] == abi.KP_OK).sum() > 20
    assert (res.rows["capacity_type"] == abi.KP_CT_RESERVED).sum() > 0
