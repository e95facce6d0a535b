"""GPU parity of kp_launch_select (launch-time filter chain + Truncate + getCapacityType + overrides) against the
oracle: the ported filter_test.go cases, a seeded config-5 batch over the golden catalog with reserved offerings, and
ICE / price deltas applied through kp_catalog_patch_*."""
import numpy as np
import pytest

import launch_cases as LC
import parity
import pyoracle
from kpsim import abi, model, native, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = native.Context(0)
    yield c
    c.close()


def _both(ctx, cat, reqs, M=60):
    cv = model.CatalogView(cat)
    ctx.upload_catalog(cv)
    b = model.LaunchBatchView(reqs)
    dev = ctx.launch_select(b, M)
    st, orc = pyoracle.launch_select(cv, b, M)
    assert st == abi.KP_OK
    return dev, orc


@pytest.mark.parametrize("mk", LC.CASES, ids=[getattr(c, "__name__", "case%d" % i) for i, c in enumerate(LC.CASES)])
def test_filter_cases(ctx, mk):
    cat, reqs, expect = mk()
    dev, orc = _both(ctx, cat, reqs)
    LC.check(cat, dev, expect)
    LC.assert_same(dev, orc)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_config5_batch_parity(ctx, golden, seed):
    cat = synth.config5_catalog(golden, seed=synth.SEED + seed)
    reqs = synth.launch_requests(cat, n=600, seed=synth.SEED + seed)
    dev, orc = _both(ctx, cat, reqs)
    LC.assert_same(dev, orc)
    assert (dev.rows["capacity_type"] == abi.KP_CT_RESERVED).sum() > 0
    # fleet emulation folded into the launch result: kwok's CreateFleet pick per request
    from kpsim import launch
    for i in range(len(reqs)):
        want = launch.fleet_pick(cat, dev, i)
        assert int(dev.rows[i]["fleet_pick"]) == (want[1] if want else -1), i
    assert (dev.rows["status"] == abi.KP_E_INSUFFICIENT_CAPACITY).sum() > 0


def test_pipelined_batch_parity(ctx, golden):
    """A batch of >= 4096 requests is evaluated as sub-batches (host encoding and expansion overlap the kernel): equal
    to the oracle, and to the same requests selected in small single-launch calls (offsets rebased per call)."""
    cat = synth.config5_catalog(golden, seed=synth.SEED + 5)
    reqs = synth.launch_requests(cat, n=6200, seed=synth.SEED + 5)
    cv = model.CatalogView(cat)
    ctx.upload_catalog(cv)
    dev = ctx.launch_select(model.LaunchBatchView(reqs), 60)
    assert ctx.launch_stats(7)[6] == 2
    st, orc = pyoracle.launch_select(cv, model.LaunchBatchView(reqs[2000:4000]), 60)
    assert st == abi.KP_OK
    for j in range(2000):  # requests 2000..3999: the sub-batch boundary (3100) lies inside
        i = 2000 + j
        for f in ("status", "failed_filter", "n_types", "n_options", "n_overrides"):
            assert int(dev.rows[i][f]) == int(orc.rows[j][f]), (i, f)
        assert list(dev.rows[i]["rejected"]) == list(orc.rows[j]["rejected"]), i
        if int(dev.rows[i]["status"]) == abi.KP_OK:
            assert int(dev.rows[i]["capacity_type"]) == int(orc.rows[j]["capacity_type"]), i
        assert list(dev.types(i)) == list(orc.types(j)), i
        assert list(dev.offerings(i)) == list(orc.offerings(j)), i
    for b0 in range(0, len(reqs), 1000):
        part = ctx.launch_select(model.LaunchBatchView(reqs[b0:b0 + 1000]), 60)
        assert ctx.launch_stats(7)[6] == 1
        for i in range(len(part.rows)):
            for f in ("status", "failed_filter", "n_types", "n_options", "n_overrides", "capacity_type"):
                assert int(part.rows[i][f]) == int(dev.rows[b0 + i][f]), (b0 + i, f)
            assert list(part.types(i)) == list(dev.types(b0 + i)), b0 + i
            assert list(part.offerings(i)) == list(dev.offerings(b0 + i)), b0 + i


def test_patches_reach_launch(ctx, golden):
    """ICE marks and price refreshes (kp_catalog_patch_avail / _price) change the launch result like a re-List."""
    cat = synth.config5_catalog(golden)
    cv = model.CatalogView(cat)
    ctx.upload_catalog(cv)
    reqs = synth.launch_requests(cat, n=200, seed=7)
    b = model.LaunchBatchView(reqs)
    rng = np.random.Generator(np.random.PCG64(3))
    avail = np.array([o.available for it in cat for o in it.offerings], np.uint8)
    avail[rng.random(len(avail)) < 0.3] = 0
    ctx.patch_avail(avail, 2)
    idx = rng.choice(len(avail), size=500, replace=False).astype(np.int32)
    price = rng.random(500) * 3
    ctx.patch_price(idx, price, 3)
    dev = ctx.launch_select(b, 60)
    flat = [o for it in cat for o in it.offerings]
    for j, o in enumerate(flat):
        o.available = bool(avail[j])
    for i, p in zip(idx, price):
        flat[int(i)].price = float(p)
    st, orc = pyoracle.launch_select(model.CatalogView(cat), b, 60)
    assert st == abi.KP_OK
    LC.assert_same(dev, orc)


def test_solve_over_64_reserved_offerings(ctx, golden):
    """Solve keeps the reserved offerings in multi-word rows (ResvTab.w words): a 70-reservation catalog solves
    bit-identically to the oracle (tests/test_gpu_wide_reserved.py covers up to 700)."""
    cat = synth.config5_catalog(golden, n_default=50, n_block=20)
    cv = model.CatalogView(cat)
    prob = synth.config2(n_pods=200, catalog=cat)
    parity.assert_same(parity.run_device(ctx, prob, cv), parity.run_oracle(prob, cv))


def test_empty_batch(ctx, golden):
    ctx.upload_catalog(model.CatalogView(golden))
    res = ctx.launch_select(model.LaunchBatchView([]), 60)
    assert len(res.rows) == 0


def test_wide_catalog_launch(ctx, golden):
    """Launch selection over a 1,800-type catalog with reserved offerings (Truncate ranks up to 2048 types)."""
    cat = synth.config5_catalog(synth.widen_catalog(golden, 1800), seed=synth.SEED + 9)
    reqs = synth.launch_requests(cat, n=400, seed=synth.SEED + 9)
    dev, orc = _both(ctx, cat, reqs)
    LC.assert_same(dev, orc)
