"""Launch-selection cases shared by the CPU (oracle) and GPU (device) tests.

Each case ports a Describe/It of pkg/providers/instance/filter/filter_test.go:47-631 to the whole chain that
instance.go:270-298 runs (kp_launch_select evaluates the chain, not one filter).  Where a later filter of the chain
changes the single-filter expectation the case says so.  Offerings need a zone and a capacity type in the catalog view:
where the Go test leaves the zone empty, the case uses one zone ("zone-1a"), which keeps every per-zone grouping of
the Go test intact.  makeInstanceType/makeOffering: filter_test.go:667-760.
"""
import numpy as np

from kpsim import abi, model
from kpsim.model import CAPACITY_TYPE, ZONE, Requirement

R = len(model.RESOURCES)
RI = {r: i for i, r in enumerate(model.RESOURCES)}
Z = "zone-1a"


def it(name, labels=None, cpu=None, res=None, offerings=()):
    cap = np.zeros(R, np.int64)
    if cpu is not None:
        cap[RI["cpu"]] = cpu
    for k, v in (res or {}).items():
        cap[RI[k]] = v
    return model.InstanceType(name, dict(labels or {}), cap, cap.copy(), list(offerings))


def off(ct, available=True, zone=Z, price=0.0, crt=None, rid=None, rcap=0):
    if crt is not None and rid is None:
        rid = "cr-" + crt
    return model.Offering(ct, zone, price, available, reservation_id=rid, reservation_type=crt, reservation_capacity=rcap)


def req(*reqs, cpu=0, min_values=None):
    rq = np.zeros(R, np.int64)
    rq[RI["cpu"]] = cpu
    return model.LaunchRequest(list(reqs), rq)


def ct(*vals, op="In"):
    return Requirement(CAPACITY_TYPE, op, list(vals))


CASES = []


def case(fn):
    CASES.append(fn)
    return fn


# Each case returns (catalog, [LaunchRequest], expect) with expect = per request
# {"types": [names in price order] | None, "status": kp status, "ct": KP_CT_*, "failed": filter, "offer_rids": ...}

@case
def compatible_by_requirements():  # filter_test.go:49-73
    cat = [it("compatible-instance", {ZONE: [Z]}, cpu=2000, offerings=[off("on-demand")]),
           it("incompatible-instance", {ZONE: ["zone-1b"]}, cpu=2000, offerings=[off("on-demand", zone="zone-1b")])]
    return cat, [req(Requirement(ZONE, "In", [Z]), cpu=1000)], [{"types": ["compatible-instance"]}]


@case
def compatible_by_requests():  # filter_test.go:74-98
    cat = [it("compatible-instance", {ZONE: [Z]}, cpu=2000, offerings=[off("on-demand")]),
           it("incompatible-instance", {ZONE: [Z]}, cpu=500, offerings=[off("on-demand")])]
    return cat, [req(Requirement(ZONE, "In", [Z]), cpu=1000)], [{"types": ["compatible-instance"]}]


@case
def compatible_available():  # filter_test.go:99-127
    cat = [it("available-instance", {ZONE: [Z]}, cpu=2000, offerings=[off("on-demand")]),
           it("unavailable-instance", {ZONE: [Z]}, cpu=2000, offerings=[off("on-demand", available=False)])]
    return cat, [req(Requirement(ZONE, "In", [Z]), cpu=1000)], [{"types": ["available-instance"]}]


@case
def all_unavailable_is_ice():  # instance.go:281-284
    cat = [it("a", cpu=2000, offerings=[off("on-demand", available=False)])]
    return cat, [req(cpu=1000)], [{"status": abi.KP_E_INSUFFICIENT_CAPACITY, "failed": abi.KP_FILTER_COMPATIBLE_AVAILABLE}]


def _crt_cheapest(sel):  # filter_test.go:131-178 (chain: a capacity-block selection is then narrowed by CapacityBlockFilter)
    other = "capacity-block" if sel == "default" else "default"
    cat = [it("cheap-instance-" + sel, offerings=[off("reserved", crt=sel, price=5.0)]),
           it("expensive-instance-" + sel, offerings=[off("reserved", crt=sel, price=10.0)]),
           it("expensive-instance-" + other, offerings=[
               off("reserved", crt=other, price=10.0),
               off("reserved", available=False, crt=other, price=1.0, rid="cr-x1"),
               off("reserved", crt=other, price=1.0, zone="zone-1b", rid="cr-x2")])]
    want = ["cheap-instance-" + sel] + (["expensive-instance-" + sel] if sel == "default" else [])
    return cat, [req(ct("reserved"), Requirement(ZONE, "In", [Z]))], [{"types": want, "ct": abi.KP_CT_RESERVED}]


@case
def crt_cheapest_default():
    return _crt_cheapest("default")


@case
def crt_cheapest_capacity_block():
    return _crt_cheapest("capacity-block")


@case
def crt_tie_prefers_default():  # filter_test.go:179-212 (priority default < capacity-block, filter.go:93-97)
    cat = [it("default", offerings=[off("reserved", crt="default", price=5.0)]),
           it("capacity-block", offerings=[off("reserved", crt="capacity-block", price=5.0)])]
    return cat, [req(ct("reserved"))], [{"types": ["default"], "ct": abi.KP_CT_RESERVED}]


@case
def crt_not_reserved():  # filter_test.go:244-259 (capacity-type NotIn reserved: nothing filtered)
    cat = [it("%s-instance" % t, offerings=[off("on-demand"), off("reserved", crt=t, price=1.0)])
           for t in ("default", "capacity-block")]
    return cat, [req(ct("reserved", op="NotIn"))], [{"types": ["capacity-block-instance", "default-instance"],
                                                     "ct": abi.KP_CT_ON_DEMAND}]


@case
def capacity_block_cheapest():  # filter_test.go:262-277
    cat = [it("cheap-instance", offerings=[off("reserved", crt="capacity-block", price=1.0, rid="a1"),
                                           off("reserved", crt="capacity-block", price=10.0, rid="a2")]),
           it("expensive-instance", offerings=[off("reserved", crt="capacity-block", price=2.0, rid="b1"),
                                               off("reserved", crt="capacity-block", price=10.0, rid="b2")])]
    return cat, [req(Requirement(CAPACITY_TYPE, "Exists"))], [{"types": ["cheap-instance"], "ct": abi.KP_CT_RESERVED,
                                                               "offer_rids": ["a1"]}]


@case
def capacity_block_not_for_default():  # filter_test.go:278-300
    cat = [it("cheap-instance", offerings=[off("reserved", crt="default", price=1.0, rid="a1"),
                                           off("reserved", crt="default", price=10.0, rid="a2")]),
           it("expensive-instance", offerings=[off("reserved", crt="default", price=2.0, rid="b1"),
                                               off("reserved", crt="default", price=10.0, rid="b2")])]
    return cat, [req(Requirement(CAPACITY_TYPE, "Exists"))], [{"types": ["cheap-instance", "expensive-instance"],
                                                               "ct": abi.KP_CT_RESERVED}]


@case
def reserved_one_offering_per_pool():  # filter_test.go:321-354 (the chain's partition filter rejects the od/spot type)
    cat = [it("non-reserved-instance", offerings=[off("on-demand", zone="1"), off("spot", zone="1")]),
           it("reserved-instance-a", offerings=[
               off("on-demand", zone="1"), off("spot", zone="1"),
               off("reserved", zone="1", crt="default", rid="kept", rcap=5),
               off("reserved", zone="2", crt="default", rid="kept", rcap=6),
               off("reserved", zone="2", crt="default", rid="rejected", rcap=5)]),
           it("reserved-instance-b", offerings=[
               off("on-demand", zone="1"), off("spot", zone="1"),
               off("reserved", zone="1", crt="default", rid="kept", rcap=1),
               off("reserved", available=False, zone="1", crt="default", rid="rejected", rcap=2)])]
    return cat, [req(Requirement(CAPACITY_TYPE, "Exists"))], [{"types": ["reserved-instance-a", "reserved-instance-b"],
                                                               "ct": abi.KP_CT_RESERVED,
                                                               "offer_rids": ["kept", "kept", "kept"]}]


@case
def reserved_no_available():  # filter_test.go:306-320
    cat = [it("non-reserved-instance", offerings=[off("on-demand", price=1.0), off("spot", price=0.5)]),
           it("reserved-instance", offerings=[off("on-demand", price=1.0), off("spot", price=0.5),
                                              off("reserved", available=False, crt="default")])]
    return cat, [req(Requirement(CAPACITY_TYPE, "Exists"))], [{"types": ["non-reserved-instance", "reserved-instance"],
                                                               "ct": abi.KP_CT_SPOT}]


def _exotic(resource=None, size=None):  # filter_test.go:386-431
    labels = {"karpenter.k8s.aws/instance-size": [size]} if size else {}
    cat = [it("generic-instance-type", {"karpenter.k8s.aws/instance-size": ["large"]}, offerings=[off("on-demand")]),
           it("exotic-instance-type", labels, res={resource: 1000} if resource else None, offerings=[off("on-demand")])]
    return cat, [req()], [{"types": ["generic-instance-type"]}]


for _r in ("aws.amazon.com/neuron", "aws.amazon.com/neuroncore", "amd.com/gpu", "nvidia.com/gpu", "habana.ai/gaudi"):
    CASES.append(lambda r=_r: _exotic(resource=r))
CASES.append(lambda: _exotic(size="metal"))
CASES.append(lambda: _exotic(size="metal-24xl"))


@case
def exotic_only_exotic_kept():  # filter.go:313-316: no generic type → nothing filtered
    cat = [it("g4dn.xlarge", res={"nvidia.com/gpu": 1000}, offerings=[off("on-demand")])]
    return cat, [req()], [{"types": ["g4dn.xlarge"]}]


@case
def exotic_skipped_with_min_values():  # filter.go:290-292
    cat = [it("a", {"karpenter.k8s.aws/instance-family": ["a"]}, offerings=[off("on-demand", price=2.0)]),
           it("b-metal", {"karpenter.k8s.aws/instance-family": ["b"], "karpenter.k8s.aws/instance-size": ["metal"]},
              offerings=[off("on-demand", price=1.0)])]
    r = req(Requirement("karpenter.k8s.aws/instance-family", "Exists", [], min_values=2))
    return cat, [r], [{"types": ["b-metal", "a"]}]


@case
def spot_cheaper_than_cheapest_od():  # filter.go:339-386, instancetype/suite_test.go:454-525
    cat = [it("a", offerings=[off("on-demand", price=1.0), off("spot", price=0.5)]),
           it("b", offerings=[off("spot", price=2.0)]),
           it("c", offerings=[off("on-demand", price=3.0)]),
           it("d", offerings=[off("spot", price=1.0)])]
    return cat, [req(ct("spot", "on-demand"))], [{"types": ["a", "d", "c"], "ct": abi.KP_CT_SPOT}]


@case
def spot_filter_needs_both_capacity_types():  # filter.go:343-345
    cat = [it("a", offerings=[off("on-demand", price=1.0), off("spot", price=0.5)]),
           it("b", offerings=[off("spot", price=2.0)])]
    return cat, [req(ct("spot"))], [{"types": ["a", "b"], "ct": abi.KP_CT_SPOT}]


@case
def truncate_orders_by_price_then_name():  # [core] OrderByPrice + Truncate(60), instance.go:293
    cat = [it("t%03d" % i, offerings=[off("on-demand", price=float(100 - i // 2))]) for i in range(100)]
    want = sorted(["t%03d" % i for i in range(100)], key=lambda n: (100 - int(n[1:]) // 2, n))[:60]
    return cat, [req(ct("on-demand"))], [{"types": want}]


@case
def truncate_min_values_failure():  # Truncate → SatisfiesMinValues error → CreateError (instance.go:294-296)
    cat = [it("t%03d" % i, {"karpenter.k8s.aws/instance-family": ["f%03d" % i]},
              offerings=[off("on-demand", price=float(i))]) for i in range(100)]
    r = req(ct("on-demand"), Requirement("karpenter.k8s.aws/instance-family", "Exists", [], min_values=61))
    return cat, [r], [{"status": abi.KP_E_CREATE}]


@case
def capacity_type_preference():  # getCapacityType: reserved > spot > on-demand (instance.go:532-546)
    cat = [it("a", offerings=[off("on-demand", price=1.0), off("spot", price=0.4)]),
           it("b", offerings=[off("on-demand", price=2.0)])]
    return cat, [req(ct("spot", "on-demand")), req(ct("on-demand")), req(ct("reserved", "on-demand"))], [
        {"types": ["a", "b"], "ct": abi.KP_CT_SPOT}, {"types": ["a", "b"], "ct": abi.KP_CT_ON_DEMAND},
        {"types": ["a", "b"], "ct": abi.KP_CT_ON_DEMAND}]


for _sel in ("default", "capacity-block"):
    def _crt_pins(sel=_sel):  # filter_test.go:213-243 (chain: a capacity-block pin is then narrowed to the cheapest type)
        cat = [it("pin-instance", offerings=[off("reserved", crt=sel, price=1.0, rid="pin")]),
               it("filter-instance", offerings=[off("reserved", crt=t, price=5.0, rid="f-" + t)
                                                for t in ("default", "capacity-block")])]
        want = ["pin-instance"] + (["filter-instance"] if sel == "default" else [])
        rids = ["pin"] + (["f-" + sel] if sel == "default" else [])
        return cat, [req(ct("reserved"))], [{"types": want, "ct": abi.KP_CT_RESERVED, "offer_rids": rids}]
    _crt_pins.__name__ = "crt_pins_selected_" + _sel.replace("-", "_")
    CASES.append(_crt_pins)


@case
def reserved_filter_not_reserved():  # filter_test.go:373-397 (NotIn reserved: both types kept, od+spot offerings)
    cat = [it("non-reserved-instance", offerings=[off("on-demand"), off("spot")]),
           it("reserved-instance", offerings=[off("on-demand"), off("spot"), off("reserved", zone="1", crt="default")])]
    return cat, [req(ct("reserved", op="NotIn"))], [{"types": ["non-reserved-instance", "reserved-instance"],
                                                     "ct": abi.KP_CT_SPOT}]


def _spot_zones(with_reserved):  # filter_test.go:513-583
    zs = lambda *o: list(o)  # noqa: E731
    kept = [it("expensive-od-instance", offerings=zs(off("on-demand", price=15.0, zone="zone-1a"),
                                                     off("on-demand", price=15.0, zone="zone-1b"))),
            it("od-instance", offerings=zs(off("on-demand", price=5.0, zone="zone-1a"),
                                           off("on-demand", price=10.0, zone="zone-1b"))),
            it("cheap-spot-instance", offerings=zs(off("spot", price=1.0, zone="zone-1a"),
                                                   off("spot", price=2.0, zone="zone-1b"))),
            it("mixed-spot-instance", offerings=zs(off("spot", price=1.0, zone="zone-1a"),
                                                   off("spot", price=10.0, zone="zone-1b"))),
            it("mixed-compatible-available-spot-instance", offerings=zs(off("spot", price=1.0, zone="zone-1a"),
                                                                        off("spot", price=10.0, zone="zone-1c")))]
    rejected = [it("mixed-unavailable-spot-instance", offerings=zs(off("spot", False, price=1.0, zone="zone-1a"),
                                                                   off("spot", price=10.0, zone="zone-1b"))),
                it("mixed-compatible-unavailable-spot-instance", offerings=zs(off("spot", price=10.0, zone="zone-1a"),
                                                                              off("spot", price=1.0, zone="zone-1c"))),
                it("expensive-spot-instance", offerings=zs(off("spot", price=10.0, zone="zone-1a"),
                                                           off("spot", price=10.0, zone="zone-1b")))]
    cat = kept + rejected
    r = req(Requirement(CAPACITY_TYPE, "Exists"), Requirement(ZONE, "In", ["zone-1a", "zone-1b"]))
    if not with_reserved:
        return cat, [r], [{"type_set": [x.name for x in kept], "ct": abi.KP_CT_SPOT}]
    # the single-filter It also keeps a type with a reserved offering; in the chain the reserved-offering filter runs
    # before the spot filter (instance.go:270-298) and keeps only that type
    cat.append(it("reserved-instance", offerings=zs(off("spot", price=10.0, zone="zone-1a"),
                                                     off("spot", price=10.0, zone="zone-1b"),
                                                     off("reserved", zone="zone-1b", crt="default"))))
    return cat, [r], [{"types": ["reserved-instance"], "ct": abi.KP_CT_RESERVED}]


@case
def spot_filter_compatible_zones():
    return _spot_zones(False)


@case
def spot_filter_compatible_zones_with_reserved():
    return _spot_zones(True)


def _three_spot():
    # the instance-type label (absent on filter_test's mocks) lets the chain's Truncate count minValues
    return [it(n, {"node.kubernetes.io/instance-type": [n]}, offerings=[off(c, price=p)])
            for n, c, p in (("od-instance", "on-demand", 5.0), ("cheap-spot-instance", "spot", 1.0),
                            ("expensive-spot-instance", "spot", 10.0))]


@case
def spot_filter_only_spot_compatible():  # filter_test.go:584-603 (od-instance then fails the compatible filter)
    return _three_spot(), [req(ct("spot"))], [{"types": ["cheap-spot-instance", "expensive-spot-instance"],
                                               "ct": abi.KP_CT_SPOT}]


@case
def spot_filter_min_values():  # filter_test.go:604-631
    r = req(Requirement(CAPACITY_TYPE, "Exists"), Requirement("node.kubernetes.io/instance-type", "Exists", [], min_values=2))
    return _three_spot(), [r], [{"types": ["cheap-spot-instance", "od-instance", "expensive-spot-instance"],
                                 "ct": abi.KP_CT_SPOT}]


def check(cat, res, expect):
    """Asserts a model.LaunchResults against a case's expectations."""
    for i, e in enumerate(expect):
        row = res.rows[i]
        assert int(row["status"]) == e.get("status", abi.KP_OK), (i, row)
        if "failed" in e:
            assert int(row["failed_filter"]) == e["failed"]
        if "type_set" in e:
            assert sorted(cat[int(t)].name for t in res.types(i)) == sorted(e["type_set"]), i
        if e.get("types") is not None:
            assert [cat[int(t)].name for t in res.types(i)] == e["types"], (i, [cat[int(t)].name for t in res.types(i)])
        if "ct" in e:
            assert int(row["capacity_type"]) == e["ct"]
        if "offer_rids" in e:
            rows = []
            for t in range(len(cat)):
                rows.extend([(t, o) for o in cat[t].offerings])
            assert [rows[int(o)][1].reservation_id for o in res.offerings(i)] == e["offer_rids"]


def assert_same(a, b):
    """Device vs oracle: every result field, type list and override list identical."""
    assert len(a.rows) == len(b.rows)
    for i in range(len(a.rows)):
        ra, rb = a.rows[i], b.rows[i]
        for f in ("status", "failed_filter", "n_types", "n_options", "n_overrides"):
            assert int(ra[f]) == int(rb[f]), (i, f, ra, rb)
        assert list(ra["rejected"]) == list(rb["rejected"]), (i, ra, rb)
        if int(ra["status"]) == abi.KP_OK:
            assert int(ra["capacity_type"]) == int(rb["capacity_type"]), (i, ra, rb)
            assert list(a.types(i)) == list(b.types(i)), i
            assert list(a.offerings(i)) == list(b.offerings(i)), i
            assert int(ra["fleet_pick"]) == int(rb["fleet_pick"]), (i, ra, rb)
