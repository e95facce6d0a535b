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


def _launch_rank_main(rank, world, port, q):
    import os
    import torch.distributed as dist
    from kpsim import catalog, launch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cat = synth.config5_catalog(catalog.golden_catalog())
        cv = model.CatalogView(cat)
        reqs = synth.launch_requests(cat, n=45, seed=11)
        fn = lambda b: pyoracle.launch_select(cv, b, 60)[1]  # noqa: E731
        q.put((rank, launch.select_sharded(reqs, fn, group=dist.group.WORLD)))
    finally:
        dist.destroy_process_group()


def test_sharded_launch_equals_single_rank_gloo(golden):
    """Rank slices of a launch batch (bench.py's launch leg at N>1) gathered over gloo equal the whole-batch result."""
    import multiprocessing as mp
    import socket
    from kpsim import launch
    cat = synth.config5_catalog(golden)
    cv = model.CatalogView(cat)
    reqs = synth.launch_requests(cat, n=45, seed=11)
    want = launch.select_sharded(reqs, lambda b: pyoracle.launch_select(cv, b, 60)[1])
    assert len(want) == 45 and any(r[0] == abi.KP_OK for r in want)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_launch_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(60)
    assert got[0] == want and got[1] == want


@pytest.mark.parametrize("scores,want", [([3.0, 1.0, 2.0], 1), ([1.0, 1.0], 0), ([0.0, 5.0, 3.0], 2),
                                         ([5.0, 0.0, 3.0], 2), ([0.0, 0.0], 1), ([], -1)])
def test_fleet_min_by_score(scores, want):
    """lo.MinBy with kwok's comparator (kwok/ec2/ec2.go:432-461), including its zero-score (lo.IsEmpty) branches."""
    from kpsim import launch
    assert launch.min_by_score(scores) == want


def test_fleet_pick_config5(golden):
    """The kwok CreateFleet pick over the oracle's launch result: one of the overrides, of minimal score, the first
    such override, and of the launch's capacity type (reserved launches pick reserved offerings)."""
    from kpsim import launch
    cat = synth.config5_catalog(golden)
    cv = model.CatalogView(cat)
    b = model.LaunchBatchView(synth.launch_requests(cat, n=40, seed=5))
    st, res = pyoracle.launch_select(cv, b, 60)
    assert st == abi.KP_OK
    flat = [o for it in cat for o in it.offerings]
    ct_name = {abi.KP_CT_ON_DEMAND: "on-demand", abi.KP_CT_SPOT: "spot", abi.KP_CT_RESERVED: "reserved"}
    n_ok = 0
    for i in range(b.n):
        pick = launch.fleet_pick(cat, res, i)
        if int(res.rows[i]["status"]) != abi.KP_OK:
            assert pick is None
            continue
        n_ok += 1
        t, row = pick
        rows = [int(x) for x in res.offerings(i)]
        assert row in rows and t in list(res.types(i))
        assert flat[row].capacity_type == ct_name[int(res.rows[i]["capacity_type"])]
        # the pick is the first override of minimal LowestPrice score (kwok/strategy/strategy.go:45-60)
        scores = [_lowest_price_score(cat, r, int(res.rows[i]["capacity_type"]) == abi.KP_CT_SPOT) for r in rows]
        k = rows.index(row)
        assert scores[k] == min(scores)
        assert all(s != scores[k] for s in scores[:k])
        # the oracle's restatement inside orc_launch_select (kp_launch_result.fleet_pick) agrees
        assert int(res.rows[i]["fleet_pick"]) == row
    assert n_ok > 0


def _lowest_price_score(cat, row, spot):
    """strategy.go LowestPrice score of an offering row: SpotPrice(type, zone) for spot fleets, OnDemandPrice(type)
    otherwise, MaxFloat64 when the pricing provider has no price."""
    from kpsim import launch
    owner = [(t, o) for t, it in enumerate(cat) for o in it.offerings]
    t, o = owner[row]
    want = "spot" if spot else "on-demand"
    for x in cat[t].offerings:
        if x.capacity_type == want and (not spot or x.zone == o.zone):
            return x.price
    return launch.MAX_FLOAT64


def _one_request_result(overrides, ct):
    rows = np.zeros(1, abi.LAUNCH_DTYPE)
    rows[0]["status"] = abi.KP_OK
    rows[0]["capacity_type"] = ct
    rows[0]["n_overrides"] = len(overrides)
    return model.LaunchResults(rows, np.zeros(1, np.int32), np.array(overrides, np.int32))


def test_fleet_pick_hand_cases():
    """Hand-computed picks (kwok/ec2/ec2.go:432-461 + strategy.go:45-60): a spot price tie across zones keeps the
    earlier override; a type without a spot price in that zone scores MaxFloat64 and loses to any priced override; an
    on-demand fleet scores every zone of a type with the same OD price, so the first override of the cheapest type wins."""
    from kpsim import launch
    O = model.Offering
    mk = lambda name, offs: model.InstanceType(name, {}, np.zeros(model.R, np.int64), np.zeros(model.R, np.int64), offs)  # noqa: E731
    cat = [mk("a.large", [O("spot", "z1", 0.05, True), O("spot", "z2", 0.05, True), O("on-demand", "z1", 0.2, True)]),
           mk("b.large", [O("on-demand", "z1", 0.1, True), O("on-demand", "z2", 0.1, True)]),
           mk("c.large", [O("spot", "z3", 0.01, True)])]
    # rows: a/z1-spot 0, a/z2-spot 1, a/z1-od 2, b/z1-od 3, b/z2-od 4, c/z3-spot 5
    assert launch.fleet_pick(cat, _one_request_result([1, 0], abi.KP_CT_SPOT), 0) == (0, 1)   # tie: first listed
    assert launch.fleet_pick(cat, _one_request_result([3, 0, 5], abi.KP_CT_SPOT), 0) == (2, 5)  # b has no spot price
    assert launch.fleet_pick(cat, _one_request_result([3, 1], abi.KP_CT_SPOT), 0) == (0, 1)
    assert launch.fleet_pick(cat, _one_request_result([2, 4, 3], abi.KP_CT_ON_DEMAND), 0) == (1, 4)
    # c.large has no on-demand price: MaxFloat64 never beats a priced override, and only it → it is still picked
    assert launch.fleet_pick(cat, _one_request_result([5, 3], abi.KP_CT_ON_DEMAND), 0) == (1, 3)
    assert launch.fleet_pick(cat, _one_request_result([5], abi.KP_CT_ON_DEMAND), 0) == (2, 5)
