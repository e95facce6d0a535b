"""CPU: catalog ingestion through the C-ABI (kp_catalog_build, csrc/kp_ingest.cpp).

The library's NewInstanceType / createOfferings restatement is a host function, so these tests call libkpsim.so on the
CPU.  They pin it to:
  * the reference's golden instance-type doc (allocatable cpu / memory / pods / ephemeral-storage, 915 types);
  * the Overhead / max-pods / ENI / eviction known-answer tests of pkg/providers/instancetype/suite_test.go
    (expected values transcribed below with their file:line);
  * the Python host builder kpsim.catalog (labels, capacity, allocatable, offerings) and the C++ oracle's resource
    arithmetic on the pkg/fake catalog, over several EC2NodeClass settings.
"""
import math

import numpy as np
import pytest

import pyoracle
from kpsim import abi, catalog, ingest, model
from kpsim.native import KpError

RI = model.RIDX
Mi, Gi = 1024 ** 2, 1024 ** 3


def _info(fx, name):
    return next(i for i in fx["fake"]["instance_types"] if i["name"] == name)


def _one(fx, name, nc):
    """NewInstanceType of one pkg/fake type (offering zones = the suite's subnets)."""
    info = _info(fx, name)
    zones = ["test-zone-1a", "test-zone-1b", "test-zone-1c"]
    cat = ingest.build_catalog([info], nc, zones, [zones], [fx["prices"].get(name)], vpclimits=fx["vpclimits"],
                               bandwidth=fx["bandwidth"])
    return cat, cat.instance_types()[0]


def test_golden_doc_allocatable(fx):
    """instance-types.md allocatable (AL2023, default options) for every type with VPC limits."""
    rows = [r for r in fx["golden"] if r["name"] in fx["vpclimits"]]
    assert len(rows) == 915
    infos = [catalog.golden_info(r, fx["vpclimits"]) for r in rows]
    cat = ingest.build_catalog(infos, ingest.NodeClass(), ["z"], [["z"]] * len(infos), [1.0] * len(infos),
                               vpclimits=fx["vpclimits"], bandwidth=fx["bandwidth"])
    its = cat.instance_types()
    bad = []
    for row, it in zip(rows, its):
        for res in ("cpu", "memory", "pods", "ephemeral-storage"):
            if it.allocatable[RI[res]] != catalog.parse_quantity_milli(row["allocatable"][res]):
                bad.append((row["name"], res))
    assert bad == []


NODECLASSES = [
    ingest.NodeClass(),
    ingest.NodeClass(ami_family="AL2", raid0=True),
    ingest.NodeClass(ami_family="Bottlerocket", pods_per_core=2),
    ingest.NodeClass(ami_family="Windows2022"),
    ingest.NodeClass(ami_family="Windows2019", max_pods=30),
    ingest.NodeClass(ami_family="Custom", reserved_enis=1, pods_per_core=1),
]
OPTS = [catalog.TypeOptions(), catalog.TypeOptions(ami_family="AL2", raid0=True),
        catalog.TypeOptions(ami_family="Bottlerocket", pods_per_core=2), catalog.TypeOptions(ami_family="Windows2022"),
        catalog.TypeOptions(ami_family="Windows2019", max_pods=30),
        catalog.TypeOptions(ami_family="Custom", reserved_enis=1, pods_per_core=1)]


@pytest.mark.parametrize("i", range(len(NODECLASSES)))
def test_fake_catalog_matches_host_builder(fx, i):
    """Labels, capacity, allocatable and offerings of all 17 pkg/fake types equal kpsim.catalog.fake_catalog's."""
    got = ingest.fake_catalog(fx, nodeclass=NODECLASSES[i]).instance_types()
    want = catalog.fake_catalog(fx=fx, opts=OPTS[i])
    assert [g.name for g in got] == [w.name for w in want]
    for g, w in zip(got, want):
        gl = {k: (sorted(v) if v is not None else None) for k, v in g.labels.items()}
        wl = {k: (sorted(v) if v is not None else None) for k, v in w.labels.items()}
        assert gl == wl, g.name
        assert (g.capacity == w.capacity).all(), (g.name, g.capacity, w.capacity)
        assert (g.allocatable == w.allocatable).all(), g.name
        assert [(o.capacity_type, o.zone, o.price, o.available, o.zone_id, o.reservation_id) for o in g.offerings] == \
               [(o.capacity_type, o.zone, o.price, o.available, o.zone_id, o.reservation_id) for o in w.offerings], g.name


@pytest.mark.parametrize("fam,oracle_fam", [("AL2023", 0), ("Bottlerocket", 2), ("Windows2022", 3)])
def test_fake_catalog_matches_oracle_arithmetic(fx, fam, oracle_fam):
    """Capacity and allocatable equal the C++ oracle's restatement (orc_instance_type_resources)."""
    its = ingest.fake_catalog(fx, nodeclass=ingest.NodeClass(ami_family=fam)).instance_types()
    opts = catalog.TypeOptions(ami_family=fam)
    for it in its:
        capo, _, _, alloc = pyoracle.instance_type_resources(_info(fx, it.name), opts, fx["vpclimits"])
        assert (capo == it.capacity).all() and (alloc == it.allocatable).all(), it.name


# ---- pkg/providers/instancetype/suite_test.go known-answer tests (m5.xlarge unless stated) ----

def _ovh(cat):
    return cat.overhead(0)


def test_kat_default_overhead(fx):
    """:1104-1112 system reserved 0; :1130-1136 kube reserved 80m / 893Mi / 1Gi; :1467-1474 eviction 100Mi, ~2Gi."""
    cat, it = _one(fx, "m5.xlarge", ingest.NodeClass())
    o = _ovh(cat)
    ev_eph = math.ceil(20 * Gi / 100 * 10)
    assert o[RI["cpu"]] == 80
    assert o[RI["memory"]] == (893 + 100) * Mi * 1000
    assert o[RI["ephemeral-storage"]] == (1 * Gi + ev_eph) * 1000


def test_kat_system_reserved_override(fx):
    """:1113-1128 systemReserved cpu 2, memory 20Gi, ephemeral 10Gi."""
    nc = ingest.NodeClass(system_reserved={"cpu": "2", "memory": "20Gi", "ephemeral-storage": "10Gi"})
    cat, _ = _one(fx, "m5.xlarge", nc)
    base, _ = _one(fx, "m5.xlarge", ingest.NodeClass())
    d = _ovh(cat) - _ovh(base)
    assert d[RI["cpu"]] == 2000 and d[RI["memory"]] == 20 * Gi * 1000 and d[RI["ephemeral-storage"]] == 10 * Gi * 1000


def test_kat_kube_reserved_override(fx):
    """:1137-1158 kubeReserved cpu 2, memory 10Gi, ephemeral 2Gi (systemReserved 1 / 20Gi / 1Gi alongside)."""
    nc = ingest.NodeClass(system_reserved={"cpu": "1", "memory": "20Gi", "ephemeral-storage": "1Gi"},
                          kube_reserved={"cpu": "2", "memory": "10Gi", "ephemeral-storage": "2Gi"})
    cat, _ = _one(fx, "m5.xlarge", nc)
    o = _ovh(cat)
    ev_eph = math.ceil(20 * Gi / 100 * 10)
    assert o[RI["cpu"]] == 3000
    assert o[RI["memory"]] == (30 * Gi + 100 * Mi) * 1000
    assert o[RI["ephemeral-storage"]] == (3 * Gi + ev_eph) * 1000


EVICTION = [  # (evictionHard, evictionSoft, AMI family, expected memory eviction threshold; None: 10% / 5% of capacity)
    ({"memory.available": "500Mi"}, None, "AL2023", 500 * Mi, ":1167-1180"),
    ({"memory.available": "10%"}, None, "AL2023", 0.10, ":1181-1194"),
    ({"memory.available": "100%"}, None, "AL2023", 0, ":1195-1208"),
    (None, {"memory.available": "50Mi"}, "AL2023", 50 * Mi, ":1209-1222"),
    (None, {"memory.available": "500Mi"}, "AL2023", 500 * Mi, ":1225-1238"),
    ({"memory.available": "5%"}, {"memory.available": "10%"}, "AL2023", 0.10, ":1239-1255"),
    (None, {"memory.available": "100%"}, "AL2023", 0, ":1256-1269"),
    ({"memory.available": "1Gi"}, {"memory.available": "10Gi"}, "Bottlerocket", 1 * Gi, ":1270-1288"),
    ({"memory.available": "1Gi"}, {"memory.available": "3Gi"}, "AL2023", 3 * Gi, ":1296-1312"),
    ({"memory.available": "5%"}, {"memory.available": "2%"}, "AL2023", 0.05, ":1313-1329"),
    ({"memory.available": "1Gi"}, {"memory.available": "10%"}, "AL2023", 0.10, ":1330-1346"),
]


@pytest.mark.parametrize("hard,soft,fam,want,line", EVICTION)
def test_kat_eviction_threshold(fx, hard, soft, fam, want, line):
    """Eviction Thresholds context (VMMemoryOverheadPercent 0; systemReserved memory 20Gi, kubeReserved memory 10Gi)."""
    nc = ingest.NodeClass(ami_family=fam, vm_memory_overhead_pct=0.0, system_reserved={"memory": "20Gi"},
                          kube_reserved={"memory": "10Gi"}, eviction_hard=hard, eviction_soft=soft)
    cat, it = _one(fx, "m5.xlarge", nc)
    ev = _ovh(cat)[RI["memory"]] - 30 * Gi * 1000
    cap_mem = it.capacity[RI["memory"]] // 1000
    if isinstance(want, float):
        assert abs(ev / 1000 - cap_mem * want) <= 10, line
    else:
        assert ev == want * 1000, line


def test_kat_pods_eni_and_max_pods(fx):
    """:1590-1607 t3.large 35 / m6idn.32xlarge 394; :1608-1616 maxPods 10 on every type; :1002-1043 ENI density
    (never 110) vs Windows (110)."""
    infos = fx["fake"]["instance_types"]
    z = ["test-zone-1a"]

    def pods(nc):
        c = ingest.build_catalog(infos, nc, z, [z] * len(infos), [1.0] * len(infos), vpclimits=fx["vpclimits"])
        return {it.name: it.capacity[RI["pods"]] // 1000 for it in c.instance_types()}

    p = pods(ingest.NodeClass())
    assert p["t3.large"] == 35 and p["m6idn.32xlarge"] == 394
    assert all(v != 110 for v in p.values())
    assert set(pods(ingest.NodeClass(max_pods=10)).values()) == {10}
    assert set(pods(ingest.NodeClass(ami_family="Windows2022")).values()) == {110}
    ppc = pods(ingest.NodeClass(pods_per_core=1))                         # :1693-1702
    assert all(ppc[i["name"]] == i["vcpus"] for i in infos)
    both = pods(ingest.NodeClass(pods_per_core=4, max_pods=20))             # :1703-1712
    assert all(both[i["name"]] == min(20, i["vcpus"] * 4) for i in infos)
    br = pods(ingest.NodeClass(ami_family="Bottlerocket", pods_per_core=1))  # :1713-1725 podsPerCore ignored
    assert br == p


MAX_PODS_TABLE = [  # :1617-1645 maxPods 10 on t3.large: (family, pods, kube-reserved memory)
    ("AL2", 10, 640), ("AL2023", 10, 640), ("Bottlerocket", 10, 365), ("Windows2019", 10, 365),
    ("Windows2022", 10, 365), ("Custom", 10, 640)]
RESERVED_ENI_TABLE = [  # :1654-1680 reservedENIs 1 on t3.large
    ("AL2", 24, 640), ("AL2023", 24, 640), ("Bottlerocket", 24, 519), ("Windows2019", 110, 1465),
    ("Windows2022", 110, 1465), ("Custom", 24, 640)]


@pytest.mark.parametrize("fam,pods,mem", MAX_PODS_TABLE)
def test_kat_max_pods_table(fx, fam, pods, mem):
    cat, it = _one(fx, "t3.large", ingest.NodeClass(ami_family=fam, max_pods=10))
    assert it.capacity[RI["pods"]] == pods * 1000
    kube_mem = _ovh(cat)[RI["memory"]] - 100 * Mi * 1000   # minus the default memory eviction threshold
    assert kube_mem == mem * Mi * 1000


@pytest.mark.parametrize("fam,pods,mem", RESERVED_ENI_TABLE)
def test_kat_reserved_enis_table(fx, fam, pods, mem):
    cat, it = _one(fx, "t3.large", ingest.NodeClass(ami_family=fam, reserved_enis=1))
    assert it.capacity[RI["pods"]] == pods * 1000
    assert _ovh(cat)[RI["memory"]] - 100 * Mi * 1000 == mem * Mi * 1000


def test_kat_reserved_enis_floor(fx):
    """:1681-1692 reservedENIs 1,000,000 → 0 pods."""
    _, it = _one(fx, "t3.large", ingest.NodeClass(reserved_enis=1_000_000))
    assert it.capacity[RI["pods"]] == 0


def test_kat_raid0_ephemeral(fx):
    """:973-995 RAID0 instance store: m6idn.32xlarge ephemeral-storage capacity 7600G."""
    _, it = _one(fx, "m6idn.32xlarge", ingest.NodeClass(raid0=True))
    assert it.capacity[RI["ephemeral-storage"]] == catalog.parse_quantity_milli(fx["kats"]["ephemeral_5000Gi"]["raid0_capacity"])


def test_block_device_mappings(fx):
    """ephemeralStorage (types.go:357-392): root volume, the family's ephemeral device, Custom's last mapping, and the
    AMI defaults (Windows /dev/sda1 50Gi, Bottlerocket /dev/xvdb)."""
    def eph(nc):
        return _one(fx, "m5.large", nc)[1].capacity[RI["ephemeral-storage"]] // 1000
    assert eph(ingest.NodeClass()) == 20 * Gi
    assert eph(ingest.NodeClass(ami_family="Windows2022")) == 50 * Gi
    assert eph(ingest.NodeClass(block_device_mappings=[("/dev/xvda", False, "100Gi")])) == 100 * Gi
    assert eph(ingest.NodeClass(block_device_mappings=[("/dev/xvdz", True, "75Gi"), ("/dev/xvda", False, "100Gi")])) == 75 * Gi
    assert eph(ingest.NodeClass(block_device_mappings=[("/dev/xvdz", False, "75Gi")])) == 20 * Gi
    assert eph(ingest.NodeClass(ami_family="Bottlerocket", block_device_mappings=[
        ("/dev/xvda", False, "4Gi"), ("/dev/xvdb", False, "60Gi")])) == 60 * Gi
    assert eph(ingest.NodeClass(ami_family="Custom", block_device_mappings=[
        ("/dev/a", False, "30Gi"), ("/dev/b", False, "40G")])) == 40 * 10 ** 9
    assert eph(ingest.NodeClass(ami_family="Custom", block_device_mappings=[("/dev/a", False, None)])) == 20 * Gi


def test_offerings_ice_spot_and_reservations(fx):
    """createOfferings (offering.go:103-196): ICE and a missing spot price make an offering unavailable; reserved
    offerings only with the ReservedCapacity gate, priced od / 1e7, unavailable when expiring or at capacity 0."""
    zones = ["test-zone-1a", "test-zone-1b"]
    info = _info(fx, "m5.large")
    crs = [{"id": "cr-1", "instance_type": "m5.large", "zone": "test-zone-1a", "type": "default", "capacity": 3},
           {"id": "cr-2", "instance_type": "m5.large", "zone": "test-zone-1b", "type": "capacity-block", "capacity": 2,
            "state": "expiring"},
           {"id": "cr-3", "instance_type": "m5.large", "zone": "test-zone-1a", "type": "default", "capacity": 0},
           {"id": "cr-x", "instance_type": "c6g.large", "zone": "test-zone-1a", "type": "default", "capacity": 5}]
    od = float(fx["prices"]["m5.large"])
    for gate in (False, True):
        nc = ingest.NodeClass(zones=[(z, "id-" + z[-2:]) for z in zones], capacity_reservations=crs,
                              reserved_capacity=gate)
        un = [[[False, False], [True, False]]]                     # ICE on-demand in 1b
        it = ingest.build_catalog([info], nc, zones, [zones], [od], [[0.05, float("nan")]], un,
                                  fx["vpclimits"], fx["bandwidth"]).instance_types()[0]
        assert sorted(it.labels[model.RESERVATION_ID]) == ["cr-1", "cr-2", "cr-3"]
        assert it.labels[model.CAPACITY_TYPE] == ["on-demand", "spot", "reserved"]
        got = [(o.capacity_type, o.zone, o.price, o.available, o.zone_id, o.reservation_id, o.reservation_capacity)
               for o in it.offerings]
        want = [("on-demand", "test-zone-1a", od, True, "id-1a", None, 0), ("spot", "test-zone-1a", 0.05, True, "id-1a", None, 0),
                ("on-demand", "test-zone-1b", od, False, "id-1b", None, 0), ("spot", "test-zone-1b", 0.0, False, "id-1b", None, 0)]
        if gate:
            want += [("reserved", "test-zone-1a", od / 1e7, True, "id-1a", "cr-1", 3),
                     ("reserved", "test-zone-1b", od / 1e7, False, "id-1b", "cr-2", 2),
                     ("reserved", "test-zone-1a", od / 1e7, False, "id-1a", "cr-3", 0)]
        assert got == want


def test_zone_labels_follow_subnets(fx):
    """computeRequirements: zone = offering zones ∩ subnet zones; zone-id only for mapped available zones; a type offered
    outside the subnets has offerings there but they are unavailable (itZones)."""
    info = _info(fx, "m5.large")
    nc = ingest.NodeClass(zones=[("test-zone-1a", "z1")])
    it = ingest.build_catalog([info], nc, ["test-zone-1a", "test-zone-1b"], [["test-zone-1a", "test-zone-1b"]],
                              [0.1]).instance_types()[0]
    assert it.labels[model.ZONE] == ["test-zone-1a"] and it.labels[model.ZONE_ID] == ["z1"]
    assert [(o.zone, o.available, o.zone_id) for o in it.offerings if o.capacity_type == "on-demand"] == \
           [("test-zone-1a", True, "z1"), ("test-zone-1b", False, None)]
    it2 = ingest.build_catalog([info], ingest.NodeClass(zones=[("test-zone-1c", "z3")]), ["test-zone-1a"],
                               [["test-zone-1a"]], [0.1]).instance_types()[0]
    assert it2.labels[model.ZONE] is None and model.ZONE_ID not in it2.labels


def test_invalid_inputs_rejected(fx):
    info = dict(_info(fx, "m5.large"))
    with pytest.raises(KpError):
        ingest.build_catalog([info], ingest.NodeClass(kube_reserved={"memory": "lots"}), ["z"], [["z"]], [1.0])
    with pytest.raises(KpError):
        ingest.build_catalog([info], ingest.NodeClass(eviction_hard={"memory.available": "x%"}), ["z"], [["z"]], [1.0])
    info["default_card"] = 7
    with pytest.raises(KpError):
        ingest.build_catalog([info], ingest.NodeClass(), ["z"], [["z"]], [1.0])


def test_quantity_forms(fx):
    """resource.Quantity forms through kubeReserved: decimal SI, binary SI, exponent, milli, fractions (rounded up)."""
    for q, milli in [("2", 2000), ("500m", 500), ("1.5", 1500), ("1Ki", 1024000), ("1e3", 1000000), ("1E-3", 1),
                     ("0.0001", 1), ("3k", 3000000), ("1.5Gi", int(1.5 * Gi) * 1000)]:
        cat, _ = _one(fx, "m5.xlarge", ingest.NodeClass(kube_reserved={"cpu": q}))
        assert _ovh(cat)[RI["cpu"]] == milli, q


def test_view_uploads_like_the_python_view(fx):
    """The built view carries the resource axes and offering keys kp_catalog_upload expects."""
    cat = ingest.fake_catalog(fx)  # the view borrows the catalog's arrays: keep it alive
    v = cat.view
    assert [v.resource_names[r].decode() for r in range(v.n_resources)] == model.RESOURCES
    assert [v.offering_keys[q].decode() for q in range(v.n_offering_keys)] == model.OFFERING_KEYS
    assert v.n_types == 17 and v.n_offerings > 0


@pytest.mark.parametrize("fam", ["AL2023", "Windows2022"])
def test_oracle_solve_over_ingested_view(fx, fam):
    """The oracle's Solve over the library-built view equals its Solve over the Python builder's view (same dictionaries,
    digests and offerings reach the scheduler)."""
    import parity
    from kpsim import synth
    nat = ingest.fake_catalog(fx, nodeclass=ingest.NodeClass(ami_family=fam))
    py = catalog.fake_catalog(fx=fx, opts=catalog.TypeOptions(ami_family=fam))
    prob = synth.subsample(synth.config2(n_pods=3000, catalog=py), 400)
    a = parity.run_oracle(prob, nat)
    b = parity.run_oracle(prob, model.CatalogView(py))
    parity.assert_same(a, b)
    assert a[0].n_nodeclaims > 0


def test_envtest_kat_catalogs_through_ingestion(fx):
    """Every known-answer case over the envtest catalog (kat_cases.ENVTEST_CASES) rebuilds its catalog — ICE marks, spot
    prices, MakeInstances types, the Windows NodeClass — through kp_catalog_build, equal to the host builder's
    (labels, capacity, allocatable, offerings); test_gpu_ingest.py then runs each through Solve on the device."""
    import kat_cases as KC
    from test_gpu_ingest import _same_catalog
    for mk in KC.ENVTEST_CASES:
        k = mk(fx)
        got = KC.native_catalog(k.problem.catalog)
        assert got is not None, mk.__name__
        assert _same_catalog(got[1], k.problem.catalog), mk.__name__
