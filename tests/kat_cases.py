"""Known-answer cases from the reference's own suites, shared by the CPU (oracle) and GPU (device) tests.

Each case rebuilds one Ginkgo It of the reference as a Solve problem over the envtest catalog (catalog.fake_catalog:
pkg/fake 17 types, subnets test-zone-1a/1b/1c) and asserts the values that It asserts — not only device == oracle.
Where the It also inspects the CreateFleet call, the Solve's NodeClaims are chained into kp_launch_select the way
[core] NodeClaimTemplate.ToNodeClaim hands them to CloudProvider.Create: the NodeClaim requirements, plus
`instance-type In [truncated options]` (with the key's minValues), with the summed pod requests.

An ICE'd pool (fake.CapacityPool / UnavailableOfferings cache) is an unavailable offering: the Its that expect
"not scheduled, then scheduled on the second reconcile" are the second reconcile, after the cache is populated.
Preferred node-affinity terms of the Its are dropped (kp preference policy Ignore: the second reconcile relaxes them
away).  The windows NodePool of :220-281 gets its own catalog rows (AMI family Windows2022 → os
windows, windows-build 10.0.20348, types.go:281-284) through NodePool.instance_types.
"""
import copy
from dataclasses import dataclass, field
from typing import Callable, List, Optional

import numpy as np

from kpsim import abi, catalog, model, synth
from kpsim.model import CAPACITY_TYPE, INSTANCE_TYPE, NODEPOOL, ZONE, PodClass, Requirement

AWS = "karpenter.k8s.aws/"
Z1A, Z1B = "test-zone-1a", "test-zone-1b"


@dataclass
class Kat:
    name: str
    ref: str                                    # reference file:line of the It
    problem: model.Problem
    check: Callable                             # check(problem, results, nodeclaim requirements)
    launch_check: Optional[Callable] = None     # launch_check(catalog, [launch row], LaunchResults)
    extra: dict = field(default_factory=dict)


class Cat(list):
    """A catalog list that remembers how catalog.fake_catalog built it: native_parts = [(fixtures, kwargs)] per
    concatenated part (None: not an envtest build), so tests/test_gpu_ingest.py builds the same catalog through the
    library's ingestion path (kp_catalog_build)."""
    native_parts = None

    def __add__(self, other):
        out = Cat(list.__add__(self, other))
        a, b = self.native_parts, getattr(other, "native_parts", None)
        out.native_parts = a + b if a is not None and b is not None else None
        return out


def envtest(fx, **kw):
    """catalog.fake_catalog(fx=fx, **kw) as a Cat (kw: opts, ice, spot_prices)"""
    c = Cat(catalog.fake_catalog(fx=fx, **kw))
    c.native_parts = [(fx, dict(kw))]
    return c


CASES: List[Callable] = []


def case(fn):
    CASES.append(fn)
    return fn


def pods(n, cls=0, **res):
    return synth.pods_from_specs([(cls, dict(res))] * n)


def problem(cat, nodepools, classes, pod_specs):
    return model.Problem(cat, nodepools, classes, synth.pods_from_specs(pod_specs))


def sel(**kv):
    return [Requirement(k, "In", [v]) for k, v in kv.items()]


def sel_map(d):
    return [Requirement(k, "In", [v]) for k, v in d.items()]


def names(cat, ts):
    return [cat[t].name for t in ts]


# ----------------------------------------------------------------------------------------------------------------------
# chaining Solve → launch
# ----------------------------------------------------------------------------------------------------------------------
def nodeclaim_launch_requests(prob, res, reqs):
    """[core] ToNodeClaim: the Solve's NodeClaim i as CloudProvider.Create receives it."""
    out = []
    for i in range(res.n_nodeclaims):
        rq = []
        it_min = None
        for key, (comp, gt, lt, mn, vals) in reqs[i].items():
            mv = None if mn == "-" else int(mn)
            if key == INSTANCE_TYPE:
                it_min = mv
            if not comp:
                rq.append(Requirement(key, "In", list(vals), mv) if vals else Requirement(key, "DoesNotExist"))
            else:
                rq.append(Requirement(key, "NotIn", list(vals), mv) if vals else Requirement(key, "Exists", [], mv))
                if gt != "-":
                    rq.append(Requirement(key, "Gt", [gt]))
                if lt != "-":
                    rq.append(Requirement(key, "Lt", [lt]))
        rq.append(Requirement(INSTANCE_TYPE, "In", names(prob.catalog, res.nodeclaim_types[i]), it_min))
        total = prob.pods.requests[res.pod_result == i].sum(axis=0)
        np_ = prob.nodepools[int(res.nodeclaim_nodepool[i])]
        if np_.daemon_overhead is not None:
            total = total + np_.daemon_overhead
        out.append(model.LaunchRequest(rq, total.astype(np.int64)))
    return out


def flat_offerings(cat):
    return [(t, o) for t in range(len(cat)) for o in cat[t].offerings]


def overrides(cat, lres, i):
    """[(type name, zone, capacity type, price)] of launch row i's CreateFleet overrides."""
    fo = flat_offerings(cat)
    out = []
    for j in lres.offerings(i):
        t, o = fo[int(j)]
        out.append((cat[t].name, o.zone, o.capacity_type, o.price))
    return out


# ----------------------------------------------------------------------------------------------------------------------
# catalogs
# ----------------------------------------------------------------------------------------------------------------------
def make_instances(fx, names_=None, vcpus=None, spot_prices=None):
    """fake.MakeInstances (pkg/fake/utils.go:185-214) + MakeInstanceOfferings (:238-): one uniform type per static
    price (2 vCPU, 8 GiB, 3 ENIs × 10 IPs), offered in test-zone-1a.  names_/vcpus: MakeUniqueInstancesAndFamilies
    with its VCpuInfo overrides (cloudprovider/suite_test.go:371-374)."""
    infos = []
    for name in (names_ if names_ is not None else fx["prices"]):
        v = (vcpus or {}).get(name, 2)
        infos.append({"name": name, "usage_classes": ["on-demand", "spot"], "architectures": ["x86_64"], "vcpus": v,
                      "memory_mib": 8192, "max_enis": 3, "ipv4_per_eni": 10, "default_card": 0, "cards": [3]})
    fxc = dict(fx)
    fxc["fake"] = {"instance_types": infos, "offerings": [[i["name"], Z1A] for i in infos]}
    return envtest(fxc, spot_prices=spot_prices)


def unique_families(fx, n):
    """MakeUniqueInstancesAndFamilies(MakeInstances(), n) (utils.go:216-236): the first n types of distinct families.
    Go takes them in map order; any such pick satisfies the It, this one takes the names in sorted order."""
    out, fams = [], set()
    for name in sorted(fx["prices"]):
        fam = name.split(".")[0]
        if fam not in fams and "." in name:
            out.append(name)
            fams.add(fam)
            if len(out) == n:
                break
    return out


def spot_half_od(cat):
    """generateSpotPricing (instancetype/suite_test.go:3006-3038): spot = %0.3f of 0.5 × on-demand."""
    sp = {}
    for it in cat:
        od = 1.0
        for o in it.offerings:
            if o.capacity_type == "on-demand":
                od = o.price
        for o in it.offerings:
            if o.capacity_type == "spot":
                sp[(it.name, o.zone)] = float("%0.3f" % (od * 0.5))
    return sp


# ----------------------------------------------------------------------------------------------------------------------
# instancetype/suite_test.go — labels
# ----------------------------------------------------------------------------------------------------------------------
G4DN_LABELS = {
    NODEPOOL: "default", "topology.kubernetes.io/region": "us-west-2", ZONE: Z1A, INSTANCE_TYPE: "g4dn.8xlarge",
    "kubernetes.io/os": "linux", "kubernetes.io/arch": "amd64", CAPACITY_TYPE: "on-demand",
    AWS + "instance-hypervisor": "nitro", AWS + "instance-encryption-in-transit-supported": "true",
    AWS + "instance-category": "g", AWS + "instance-capacity-flex": "false", AWS + "instance-generation": "4",
    AWS + "instance-family": "g4dn", AWS + "instance-size": "8xlarge", AWS + "instance-cpu": "32",
    AWS + "instance-cpu-manufacturer": "intel", AWS + "instance-cpu-sustained-clock-speed-mhz": "2500",
    AWS + "instance-memory": "131072", AWS + "instance-ebs-bandwidth": "9500",
    AWS + "instance-network-bandwidth": "50000", AWS + "instance-gpu-name": "t4",
    AWS + "instance-gpu-manufacturer": "nvidia", AWS + "instance-gpu-count": "1", AWS + "instance-gpu-memory": "16384",
    AWS + "instance-local-nvme": "900", "topology.k8s.aws/zone-id": "tstz1-1a",
    "failure-domain.beta.kubernetes.io/region": "us-west-2", "failure-domain.beta.kubernetes.io/zone": Z1A,
    "beta.kubernetes.io/arch": "amd64", "beta.kubernetes.io/os": "linux",
    "beta.kubernetes.io/instance-type": "g4dn.8xlarge", "topology.ebs.csi.aws.com/zone": Z1A,
}
# the accelerator and windows-build selectors of :251-263, each on its own pod
G4DN_EXTRA = {AWS + "instance-accelerator-name": "inferentia2", AWS + "instance-accelerator-manufacturer": "aws",
              AWS + "instance-accelerator-count": "1", "node.kubernetes.io/windows-build": "10.0.20348"}
INF2_LABELS = {
    NODEPOOL: "default", "topology.kubernetes.io/region": "us-west-2", ZONE: Z1A, INSTANCE_TYPE: "inf2.xlarge",
    "kubernetes.io/os": "linux", "kubernetes.io/arch": "amd64", CAPACITY_TYPE: "on-demand",
    AWS + "instance-hypervisor": "nitro", AWS + "instance-encryption-in-transit-supported": "true",
    AWS + "instance-category": "inf", AWS + "instance-capacity-flex": "false", AWS + "instance-generation": "2",
    AWS + "instance-family": "inf2", AWS + "instance-size": "xlarge", AWS + "instance-cpu": "4",
    AWS + "instance-cpu-sustained-clock-speed-mhz": "3600", AWS + "instance-cpu-manufacturer": "amd",
    AWS + "instance-memory": "16384", AWS + "instance-ebs-bandwidth": "10000",
    AWS + "instance-network-bandwidth": "2083", AWS + "instance-accelerator-name": "inferentia2",
    AWS + "instance-accelerator-manufacturer": "aws", AWS + "instance-accelerator-count": "1",
    "topology.k8s.aws/zone-id": "tstz1-1a",
    "failure-domain.beta.kubernetes.io/region": "us-west-2", "failure-domain.beta.kubernetes.io/zone": Z1A,
    "beta.kubernetes.io/arch": "amd64", "beta.kubernetes.io/os": "linux",
    "beta.kubernetes.io/instance-type": "inf2.xlarge", "topology.ebs.csi.aws.com/zone": Z1A,
}


def _all_scheduled(prob, res, reqs):
    assert (res.pod_result >= 0).all(), res.pod_result


@case
def labels_individual(fx):
    """Every well-known label as its own nodeSelector; all pods schedule (default + windows NodePools)."""
    lin = envtest(fx)
    win = envtest(fx, opts=catalog.TypeOptions(ami_family="Windows2022"))
    cat = lin + win
    nps = [synth.default_nodepool("default", instance_types=list(range(len(lin)))),
           synth.default_nodepool("windows", instance_types=list(range(len(lin), len(cat))))]
    sels = dict(G4DN_LABELS)
    sels.update(G4DN_EXTRA)
    classes = [PodClass(sel_map({k: v})) for k, v in sels.items()]
    prob = problem(cat, nps, classes, [(c, {}) for c in range(len(classes))])

    def check(prob, res, reqs):
        _all_scheduled(prob, res, reqs)
        keys = list(sels)
        wb = keys.index("node.kubernetes.io/windows-build")
        assert int(res.nodeclaim_nodepool[res.pod_result[wb]]) == 1   # the windows NodePool
    return Kat("labels_individual", "pkg/providers/instancetype/suite_test.go:220-281", prob, check)


@case
def labels_combined(fx):
    cat = envtest(fx)
    prob = problem(cat, [synth.default_nodepool()], [PodClass(sel_map(G4DN_LABELS))], [(0, {})])

    def check(prob, res, reqs):
        _all_scheduled(prob, res, reqs)
        assert names(cat, res.nodeclaim_types[0]) == ["g4dn.8xlarge"]
        assert reqs[0][ZONE][4] == (Z1A,)
    return Kat("labels_combined", "pkg/providers/instancetype/suite_test.go:282-338", prob, check)


@case
def labels_accelerator(fx):
    cat = envtest(fx)
    prob = problem(cat, [synth.default_nodepool()], [PodClass(sel_map(INF2_LABELS))], [(0, {})])

    def check(prob, res, reqs):
        _all_scheduled(prob, res, reqs)
        assert names(cat, res.nodeclaim_types[0]) == ["inf2.xlarge"]
    return Kat("labels_accelerator", "pkg/providers/instancetype/suite_test.go:339-394", prob, check)


# ----------------------------------------------------------------------------------------------------------------------
# instancetype/suite_test.go — price ordering, exotic types
# ----------------------------------------------------------------------------------------------------------------------
@case
def spot_cheaper_than_cheapest_od(fx):
    base = make_instances(fx)
    cat = make_instances(fx, spot_prices=spot_half_od(base))
    prob = problem(cat, [synth.default_nodepool(capacity_types=("spot", "on-demand"))], [PodClass()],
                   [(0, {"cpu": "1"})])

    def launch_check(cat, lreqs, lres):
        ov = overrides(cat, lres, 0)
        assert int(lres.rows[0]["capacity_type"]) == abi.KP_CT_SPOT and ov
        od = {it.name: min(o.price for o in it.offerings if o.capacity_type == "on-demand") for it in cat}
        cheapest_od = min(od[n] for n, _, _, _ in ov)
        for n, z, ct, price in ov:
            assert ct == "spot" and price < cheapest_od, (n, price, cheapest_od)
    return Kat("spot_cheaper_than_cheapest_od", "pkg/providers/instancetype/suite_test.go:454-525", prob,
               _all_scheduled, launch_check)


@case
def metal_kept_with_min_values(fx):
    cat = envtest(fx)
    np_ = model.NodePool("default", requirements=[Requirement(CAPACITY_TYPE, "In", ["spot"], 1)])
    prob = problem(cat, [np_], [PodClass()], [(0, {"cpu": "1"})])

    def launch_check(cat, lreqs, lres):
        assert any("metal" in n for n, _, _, _ in overrides(cat, lres, 0))
    return Kat("metal_kept_with_min_values", "pkg/providers/instancetype/suite_test.go:526-562", prob,
               _all_scheduled, launch_check)


@case
def deprioritize_metal_and_gpu(fx):
    cat = envtest(fx)
    prob = problem(cat, [synth.default_nodepool()], [PodClass()], [(0, {"cpu": "1"})])

    def launch_check(cat, lreqs, lres):
        ov = overrides(cat, lres, 0)
        assert ov
        for n, _, _, _ in ov:
            assert "metal" not in n and not n.startswith("g"), n
    return Kat("deprioritize_metal_and_gpu", "pkg/providers/instancetype/suite_test.go:563-600", prob,
               _all_scheduled, launch_check)


@case
def launch_on_metal(fx):
    cat = envtest(fx)
    np_ = synth.default_nodepool(requirements=[Requirement(INSTANCE_TYPE, "Exists")])
    prob = problem(cat, [np_], [PodClass(sel(**{AWS + "instance-size": "metal"}))], [(0, {"cpu": "1"})])

    def check(prob, res, reqs):
        _all_scheduled(prob, res, reqs)
        assert names(cat, res.nodeclaim_types[0]) == ["m5.metal"]

    def launch_check(cat, lreqs, lres):
        assert {n for n, _, _, _ in overrides(cat, lres, 0)} == {"m5.metal"}
    return Kat("launch_on_metal", "pkg/providers/instancetype/suite_test.go:601-621", prob, check, launch_check)


@case
def flex_instance_type(fx):
    cat = envtest(fx)
    prob = problem(cat, [synth.default_nodepool()], [PodClass(sel(**{AWS + "instance-capacity-flex": "true"}))],
                   [(0, {})])

    def check(prob, res, reqs):
        _all_scheduled(prob, res, reqs)
        assert all("flex" in n for n in names(cat, res.nodeclaim_types[0]))
    return Kat("flex_instance_type", "pkg/providers/instancetype/suite_test.go:639-650", prob, check)


@case
def flex_disallowed(fx):
    cat = envtest(fx)
    np_ = synth.default_nodepool(requirements=[Requirement(AWS + "instance-capacity-flex", "NotIn", ["true"])])
    prob = problem(cat, [np_], [PodClass(sel(**{AWS + "instance-capacity-flex": "true"}))], [(0, {})])

    def check(prob, res, reqs):
        assert (res.pod_result == -1).all()
    return Kat("flex_disallowed", "pkg/providers/instancetype/suite_test.go:651-665", prob, check)


# ----------------------------------------------------------------------------------------------------------------------
# instancetype/suite_test.go — Insufficient Capacity Error cache (:2039-2215)
# ----------------------------------------------------------------------------------------------------------------------
def _inf2_pair(fx, ice):
    cat = envtest(fx, ice=ice)
    cls = [PodClass(sel(**{ZONE: Z1A}))]
    return cat, problem(cat, [synth.default_nodepool()], cls, [(0, {"aws.amazon.com/neuron": "1"})] * 2)


@case
def ice_inf2_fallback(fx):
    cat, prob = _inf2_pair(fx, {("on-demand", "inf2.24xlarge", Z1A)})

    def check(prob, res, reqs):
        _all_scheduled(prob, res, reqs)
        assert res.n_nodeclaims == 2 and res.pod_result[0] != res.pod_result[1]
        for ts in res.nodeclaim_types:
            assert "inf2.24xlarge" not in names(cat, ts)

    def launch_check(cat, lreqs, lres):
        for i in range(len(lres.rows)):
            ov = overrides(cat, lres, i)
            cheapest = min(ov, key=lambda x: (x[3], x[0]))[0]
            it = next(x for x in cat if x.name == cheapest)
            assert it.labels[AWS + "instance-accelerator-name"] == ["inferentia2"], cheapest
    return Kat("ice_inf2_fallback", "pkg/providers/instancetype/suite_test.go:2040-2072", prob, check, launch_check)


@case
def ice_inf2_first_attempt(fx):
    """The same Its' first reconcile (no ICE yet): both pods pack onto one inf2.24xlarge."""
    cat, prob = _inf2_pair(fx, ())

    def check(prob, res, reqs):
        _all_scheduled(prob, res, reqs)
        assert res.n_nodeclaims == 1 and names(cat, res.nodeclaim_types[0]) == ["inf2.24xlarge"]
    return Kat("ice_inf2_first_attempt", "pkg/providers/instancetype/suite_test.go:2059-2060", prob, check)


def _zone_fallback(fx, typ, resource, lines):
    cat = envtest(fx, ice={("on-demand", typ, Z1A)})
    prob = problem(cat, [synth.default_nodepool()], [PodClass(sel(**{INSTANCE_TYPE: typ}))], [(0, {resource: "1"})])

    def check(prob, res, reqs):
        _all_scheduled(prob, res, reqs)
        assert names(cat, res.nodeclaim_types[0]) == [typ]

    def launch_check(cat, lreqs, lres):
        ov = overrides(cat, lres, 0)
        assert ov and all(n == typ and z == Z1B for n, z, _, _ in ov), ov
    return Kat("ice_zone_fallback_" + typ, "pkg/providers/instancetype/suite_test.go:" + lines, prob, check,
               launch_check)


@case
def ice_zone_fallback_p3(fx):
    return _zone_fallback(fx, "p3.8xlarge", "nvidia.com/gpu", "2073-2099")


@case
def ice_zone_fallback_dl1(fx):
    return _zone_fallback(fx, "dl1.24xlarge", "habana.ai/gaudi", "2153-2179")


def _m5_pair(fx, ice):
    cat = envtest(fx, ice=ice)
    np_ = synth.default_nodepool(requirements=[Requirement(INSTANCE_TYPE, "In", ["m5.large", "m5.xlarge"])])
    return cat, problem(cat, [np_], [PodClass(sel(**{ZONE: Z1A}))], [(0, {"cpu": "1"})] * 2)


@case
def ice_smaller_instances(fx):
    cat, prob = _m5_pair(fx, {("on-demand", "m5.xlarge", Z1A)})

    def check(prob, res, reqs):
        _all_scheduled(prob, res, reqs)
        assert res.n_nodeclaims == 2
        assert [names(cat, ts) for ts in res.nodeclaim_types] == [["m5.large"], ["m5.large"]]
    return Kat("ice_smaller_instances", "pkg/providers/instancetype/suite_test.go:2100-2133", prob, check)


@case
def ice_smaller_first_attempt(fx):
    cat, prob = _m5_pair(fx, ())

    def check(prob, res, reqs):
        _all_scheduled(prob, res, reqs)
        assert res.n_nodeclaims == 1 and names(cat, res.nodeclaim_types[0]) == ["m5.xlarge"]
    return Kat("ice_smaller_first_attempt", "pkg/providers/instancetype/suite_test.go:2122-2124", prob, check)


def _expiry(fx, ice):
    cat = envtest(fx, ice=ice)
    return cat, problem(cat, [synth.default_nodepool()], [PodClass(sel(**{INSTANCE_TYPE: "inf2.24xlarge"}))],
                        [(0, {"aws.amazon.com/neuron": "2"})])


@case
def ice_expiry_cached(fx):
    cat, prob = _expiry(fx, {("on-demand", "inf2.24xlarge", Z1A)})

    def check(prob, res, reqs):
        assert (res.pod_result == -1).all()
    return Kat("ice_expiry_cached", "pkg/providers/instancetype/suite_test.go:2134-2145", prob, check)


@case
def ice_expiry_expired(fx):
    cat, prob = _expiry(fx, ())

    def check(prob, res, reqs):
        _all_scheduled(prob, res, reqs)
        assert names(cat, res.nodeclaim_types[0]) == ["inf2.24xlarge"]
    return Kat("ice_expiry_expired", "pkg/providers/instancetype/suite_test.go:2146-2151", prob, check)


@case
def ice_spot_falls_back_to_od(fx):
    fake = envtest(fx)
    ice = {("spot", it.name, Z1A) for it in fake}
    cat = envtest(fx, ice=ice)
    np_ = model.NodePool("default", requirements=[Requirement(CAPACITY_TYPE, "In", ["spot", "on-demand"]),
                                                  Requirement(ZONE, "In", [Z1A])])
    prob = problem(cat, [np_], [PodClass()], [(0, {})])

    def launch_check(cat, lreqs, lres):
        assert int(lres.rows[0]["status"]) == abi.KP_OK
        assert int(lres.rows[0]["capacity_type"]) == abi.KP_CT_ON_DEMAND
        assert all(ct == "on-demand" for _, _, ct, _ in overrides(cat, lres, 0))
    return Kat("ice_spot_falls_back_to_od", "pkg/providers/instancetype/suite_test.go:2180-2215", prob,
               _all_scheduled, launch_check)


# ----------------------------------------------------------------------------------------------------------------------
# instancetype/suite_test.go — CapacityType (:2392-2460)
# ----------------------------------------------------------------------------------------------------------------------
@case
def capacity_type_default_od(fx):
    cat = envtest(fx)
    prob = problem(cat, [synth.default_nodepool()], [PodClass()], [(0, {})])

    def launch_check(cat, lreqs, lres):
        assert int(lres.rows[0]["capacity_type"]) == abi.KP_CT_ON_DEMAND
    return Kat("capacity_type_default_od", "pkg/providers/instancetype/suite_test.go:2393-2399", prob,
               _all_scheduled, launch_check)


@case
def capacity_type_spot_when_flexible(fx):
    cat = envtest(fx)
    prob = problem(cat, [model.NodePool("default", requirements=[Requirement(CAPACITY_TYPE, "In",
                                                                             ["spot", "on-demand"])])],
                   [PodClass()], [(0, {})])

    def launch_check(cat, lreqs, lres):
        assert int(lres.rows[0]["capacity_type"]) == abi.KP_CT_SPOT
    return Kat("capacity_type_spot_when_flexible", "pkg/providers/instancetype/suite_test.go:2400-2408", prob,
               _all_scheduled, launch_check)


def _m5_spot_only_1a(fx, zone_req):
    cat = envtest(fx, spot_prices={("m5.large", Z1A): 0.004})
    reqs = [Requirement(CAPACITY_TYPE, "In", ["spot"]), Requirement(INSTANCE_TYPE, "In", ["m5.large"])]
    if zone_req:
        reqs.append(Requirement(ZONE, "In", [Z1B]))
    return cat, problem(cat, [model.NodePool("default", requirements=reqs)], [PodClass()], [(0, {})])


@case
def capacity_type_no_zonal_spot(fx):
    cat, prob = _m5_spot_only_1a(fx, True)

    def check(prob, res, reqs):
        assert (res.pod_result == -1).all()
    return Kat("capacity_type_no_zonal_spot", "pkg/providers/instancetype/suite_test.go:2409-2434", prob, check)


@case
def capacity_type_zonal_spot(fx):
    cat, prob = _m5_spot_only_1a(fx, False)

    def check(prob, res, reqs):
        _all_scheduled(prob, res, reqs)
        assert reqs[0][NODEPOOL][4] == ("default",)

    def launch_check(cat, lreqs, lres):
        assert overrides(cat, lres, 0) == [("m5.large", Z1A, "spot", 0.004)]
    return Kat("capacity_type_zonal_spot", "pkg/providers/instancetype/suite_test.go:2435-2460", prob, check,
               launch_check)


# ----------------------------------------------------------------------------------------------------------------------
# instancetype/suite_test.go — Capacity Blocks (:2892-2947), through Solve-less launch (config 5 catalog shape)
# ----------------------------------------------------------------------------------------------------------------------
def capacity_block_catalog(fx, state):
    crs = {"c6g.large": [{"id": "cr-123", "zone": Z1A, "type": "capacity-block", "capacity": 1, "state": state}]}
    return catalog.fake_catalog(fx=fx, reservations=crs)


# ----------------------------------------------------------------------------------------------------------------------
# cloudprovider/suite_test.go — MinValues (:365-671)
# ----------------------------------------------------------------------------------------------------------------------
def _min_values_catalog(fx, n, vcpus, prices):
    nm = unique_families(fx, n)
    sp = {(nm[i], Z1A): prices[i] for i in range(n)}
    return nm, make_instances(fx, nm, dict(zip(nm, vcpus)), sp)


def _two_nodeclaims(prob, res, reqs):
    _all_scheduled(prob, res, reqs)
    assert res.n_nodeclaims == 2 and res.pod_result[0] != res.pod_result[1]


@case
def min_values_in_operator(fx):
    nm, cat = _min_values_catalog(fx, 2, (1, 8), (0.002, 0.003))
    np_ = model.NodePool("default", requirements=[Requirement(CAPACITY_TYPE, "In", ["spot"]),
                                                  Requirement(INSTANCE_TYPE, "In", nm, 2)])
    prob = problem(cat, [np_], [PodClass()], [(0, {"cpu": "0.9"})] * 2)

    def launch_check(cat, lreqs, lres):
        assert len(lres.rows) == 2
        for i in range(2):
            assert len({n for n, _, _, _ in overrides(cat, lres, i)}) >= 2
    return Kat("min_values_in_operator", "pkg/cloudprovider/suite_test.go:366-466", prob, _two_nodeclaims,
               launch_check)


@case
def min_values_exists_operator(fx):
    nm, cat = _min_values_catalog(fx, 2, (1, 8), (0.002, 0.003))
    np_ = model.NodePool("default", requirements=[Requirement(INSTANCE_TYPE, "Exists", [], 2),
                                                  Requirement(INSTANCE_TYPE, "In", nm, 1)])
    prob = problem(cat, [np_], [PodClass()], [(0, {"cpu": "0.9"})] * 2)

    def launch_check(cat, lreqs, lres):
        assert len(lres.rows) == 2
        for i in range(2):
            assert len({n for n, _, _, _ in overrides(cat, lres, i)}) >= 2
    return Kat("min_values_exists_operator", "pkg/cloudprovider/suite_test.go:467-564", prob, _two_nodeclaims,
               launch_check)


@case
def min_values_multiple_keys(fx):
    nm, cat = _min_values_catalog(fx, 3, (1, 4, 8), (0.002, 0.003, 0.004))
    fams = sorted({n.split(".")[0] for n in nm})
    np_ = model.NodePool("default", requirements=[Requirement(INSTANCE_TYPE, "In", nm, 2),
                                                  Requirement(AWS + "instance-family", "In", fams, 3)])
    prob = problem(cat, [np_], [PodClass()], [(0, {"cpu": "0.9"})] * 2)

    def launch_check(cat, lreqs, lres):
        assert len(lres.rows) == 2
        for i in range(2):
            ov = {n for n, _, _, _ in overrides(cat, lres, i)}
            assert len(ov) == 3 and len({n.split(".")[0] for n in ov}) == 3, ov
    return Kat("min_values_multiple_keys", "pkg/cloudprovider/suite_test.go:565-671", prob, _two_nodeclaims,
               launch_check)


# ----------------------------------------------------------------------------------------------------------------------
# test/suites/scheduling/suite_test.go — provisioning end to end (Solve → CreateFleet overrides → kwok's lowest-price
# override pick), over the golden catalog (test-zone-1a/1b/1c = zone ids use1-az1 / use1-az2 / use1-az4)
# ----------------------------------------------------------------------------------------------------------------------
def _env_default_pool(*replace):
    """env.DefaultNodePool (test/pkg/environment/common/environment.go:133-177) + test.ReplaceRequirements."""
    reqs = [Requirement("kubernetes.io/os", "In", ["linux"]), Requirement(CAPACITY_TYPE, "In", ["on-demand"]),
            Requirement(AWS + "instance-category", "In", ["c", "m", "r"]),
            Requirement(AWS + "instance-generation", "Gt", ["4"]), Requirement(AWS + "instance-family", "NotIn", ["a1"])]
    keys = {r.key for r in replace}
    return model.NodePool("default", requirements=[r for r in reqs if r.key not in keys] + list(replace))


def picked(cat, lres, i):
    """(type name, offering) of kwok CreateFleet's pick for launch row i."""
    row = int(lres.rows[i]["fleet_pick"])  # kp_launch_result.fleet_pick (device) / its oracle restatement
    t, o = flat_offerings(cat)[row]
    return cat[t].name, o


@case
def e2e_nodepool_weight(fx):
    """A pod against NodePools of weight 10 (instance-type In [t3.nano]) and 100 (In [c5.large]): one node, a c5.large
    from the high-priority pool."""
    cat = catalog.golden_catalog(fx=fx)
    low = model.NodePool("low", weight=10, requirements=[Requirement("kubernetes.io/os", "In", ["linux"]),
                                                         Requirement(INSTANCE_TYPE, "In", ["t3.nano"])])
    high = model.NodePool("high", weight=100, requirements=[Requirement("kubernetes.io/os", "In", ["linux"]),
                                                            Requirement(INSTANCE_TYPE, "In", ["c5.large"])])
    prob = problem(cat, [low, high], [PodClass()], [(0, {})])

    def check(prob, res, reqs):
        assert res.n_nodeclaims == 1 and (res.pod_result == 0).all()
        assert prob.nodepools[int(res.nodeclaim_nodepool[0])].name == "high"

    def launch_check(cat, lreqs, lres):
        assert picked(cat, lres, 0)[0] == "c5.large"
    return Kat("e2e_nodepool_weight", "test/suites/scheduling/suite_test.go:471-538", prob, check, launch_check)


@case
def e2e_flex_node(fx):
    """env.DefaultNodePool with instance-capacity-flex In [true]: the pod's node is a flex instance type."""
    cat = catalog.golden_catalog(fx=fx)
    prob = problem(cat, [_env_default_pool(Requirement(AWS + "instance-capacity-flex", "In", ["true"]))], [PodClass()],
                   [(0, {})])

    def launch_check(cat, lreqs, lres):
        assert "flex" in picked(cat, lres, 0)[0]
    return Kat("e2e_flex_node", "test/suites/scheduling/suite_test.go:539-553", prob, _all_scheduled, launch_check)


@case
def e2e_zone_and_zone_id_overlap(fx):
    """zone In [1a, 1b] and zone-id In [az2, az4]: only test-zone-1b / use1-az2 satisfies both — the node lands
    there (offering-level joint compatibility, not per-label)."""
    cat = catalog.golden_catalog(fx=fx)
    cls = PodClass(requirements=[Requirement(ZONE, "In", ["test-zone-1a", "test-zone-1b"]),
                                 Requirement(model.ZONE_ID, "In", ["use1-az2", "use1-az4"])])
    prob = problem(cat, [_env_default_pool()], [cls], [(0, {})])

    def launch_check(cat, lreqs, lres):
        _, o = picked(cat, lres, 0)
        assert (o.zone, o.zone_id) == ("test-zone-1b", "use1-az2")
        assert {(z, c) for _, z, c, _ in overrides(cat, lres, 0)} == {("test-zone-1b", "on-demand")}
    return Kat("e2e_zone_and_zone_id_overlap", "test/suites/scheduling/suite_test.go:692-718", prob, _all_scheduled,
               launch_check)


@case
def e2e_zone_id_correct_zone(fx):
    """A NodePool requiring expected-zone-label Exists; one pod per zone with expected-zone-label In [zone] and
    zone-id In [that zone's id]: three nodes, each in the zone its label names."""
    cat = catalog.golden_catalog(fx=fx)
    zid = {"test-zone-1a": "use1-az1", "test-zone-1b": "use1-az2", "test-zone-1c": "use1-az4"}
    classes = [PodClass(requirements=[Requirement("expected-zone-label", "In", [z]),
                                      Requirement(model.ZONE_ID, "In", [zid[z]])]) for z in sorted(zid)]
    prob = problem(cat, [_env_default_pool(Requirement("expected-zone-label", "Exists"))], classes,
                   [(i, {}) for i in range(3)])

    def check(prob, res, reqs):
        assert res.n_nodeclaims == 3 and (res.pod_result >= 0).all()

    def launch_check(cat, lreqs, lres):
        for i, lr in enumerate(lreqs):
            want = next(r.values[0] for r in lr.requirements if r.key == "expected-zone-label")
            _, o = picked(cat, lres, i)
            assert (o.zone, o.zone_id) == (want, zid[want])
    return Kat("e2e_zone_id_correct_zone", "test/suites/scheduling/suite_test.go:719-768", prob, check, launch_check)


def build(fx, mk):
    return mk(fx)


def ids():
    return [c.__name__ for c in CASES]


# the cases over the envtest catalog (pkg/fake EC2 records: an input of the ingestion path, kp_catalog_build); the e2e
# cases run over the golden-doc catalog, whose labels and allocatable come from the doc, not from EC2 records
ENVTEST_CASES = [c for c in CASES if not c.__name__.startswith("e2e_")]


def native_catalog(cat):
    """The same catalog built by the library's ingestion path: (NativeCatalog views, their InstanceTypes concatenated),
    or None for a catalog not built by envtest()."""
    from kpsim import ingest
    parts = getattr(cat, "native_parts", None)
    if parts is None:
        return None
    nats, types = [], []
    for pfx, kw in parts:
        kw = dict(kw)
        opts = kw.pop("opts", None)
        nc = ingest.NodeClass(ami_family=opts.ami_family) if opts is not None else None
        nat = ingest.fake_catalog(pfx, nodeclass=nc, **kw)
        nats.append(nat)
        types += nat.instance_types()
    return nats, types


def clone_problem(prob):
    return copy.deepcopy(prob)


# ----------------------------------------------------------------------------------------------------------------------
# reserved capacity in Solve: ReservationManager + FinalizeScheduling's reservation-id requirement
# ----------------------------------------------------------------------------------------------------------------------
RESV_CASES: List[Callable] = []


def resv_case(fn):
    RESV_CASES.append(fn)
    return fn


RESVID = "karpenter.k8s.aws/capacity-reservation-id"
RESVTYPE = "karpenter.k8s.aws/capacity-reservation-type"


def _cp_reservations_catalog(fx):
    """cloudprovider/suite_test.go:1444-1465: one m5.large reservation per reservation type in test-zone-1a, 10 each."""
    crs = {"m5.large": [{"id": "cr-m5.large-1a-" + t, "zone": Z1A, "type": t, "capacity": 10, "state": "active"}
                        for t in ("default", "capacity-block")]}
    return catalog.fake_catalog(fx=fx, reservations=crs)


def _reserved_pool():
    return model.NodePool("default", requirements=[Requirement(CAPACITY_TYPE, "In", ["reserved"])])


def _launch_reserved(cat, lres, i, rid):
    ov = overrides(cat, lres, i)
    assert int(lres.rows[i]["capacity_type"]) == abi.KP_CT_RESERVED, lres.rows[i]
    fo = flat_offerings(cat)
    rids = {fo[int(j)][1].reservation_id for j in lres.offerings(i)}
    assert rids == {rid} and ov, (rids, rid)


@resv_case
def resv_marks_launched(fx):
    cat = _cp_reservations_catalog(fx)
    prob = problem(cat, [_reserved_pool()], [PodClass()], [(0, {})])
    ids = ("cr-m5.large-1a-capacity-block", "cr-m5.large-1a-default")

    def check(prob, res, reqs):
        _all_scheduled(prob, res, reqs)
        assert res.n_nodeclaims == 1 and names(cat, res.nodeclaim_types[0]) == ["m5.large"]
        assert reqs[0][RESVID][0] is False and reqs[0][RESVID][4] == ids

    def launch_check(cat, lreqs, lres):
        # both reservations are held; the launch's reservation-type filter prefers default on a price tie
        _launch_reserved(cat, lres, 0, "cr-m5.large-1a-default")
    return Kat("resv_marks_launched", "pkg/cloudprovider/suite_test.go:1472-1480", prob, check, launch_check)


def _resv_labels(fx, crt):
    cat = _cp_reservations_catalog(fx)
    prob = problem(cat, [_reserved_pool()], [PodClass(sel(**{RESVTYPE: crt}))], [(0, {})])
    rid = "cr-m5.large-1a-" + crt

    def check(prob, res, reqs):
        _all_scheduled(prob, res, reqs)
        assert reqs[0][RESVID][4] == (rid,)

    def launch_check(cat, lreqs, lres):
        _launch_reserved(cat, lres, 0, rid)
    return Kat("resv_labels_" + crt, "pkg/cloudprovider/suite_test.go:1501-1524", prob, check, launch_check)


@resv_case
def resv_labels_default(fx):
    return _resv_labels(fx, "default")


@resv_case
def resv_labels_capacity_block(fx):
    return _resv_labels(fx, "capacity-block")


def e2e_reservations(fx, large_cap=1, xlarge_cap=2):
    """test/suites/scheduling/suite_test.go:771-823: m5.large (1 instance) and m5.xlarge (2) ODCRs in the first zone,
    NodePool capacity-type In [on-demand, reserved], os In [linux]."""
    crs = {"m5.large": [{"id": "cr-large", "zone": Z1A, "type": "default", "capacity": large_cap,
                         "state": "active"}],
           "m5.xlarge": [{"id": "cr-xlarge", "zone": Z1A, "type": "default", "capacity": xlarge_cap,
                          "state": "active"}]}
    cat = catalog.fake_catalog(fx=fx, reservations=crs)
    np_ = model.NodePool("default", requirements=[Requirement(CAPACITY_TYPE, "In", ["on-demand", "reserved"]),
                                                  Requirement("kubernetes.io/os", "In", ["linux"])])
    return cat, np_


@resv_case
def resv_specific_id(fx):
    cat, np_ = e2e_reservations(fx)
    prob = problem(cat, [np_], [PodClass([Requirement(RESVID, "In", ["cr-xlarge"])])], [(0, {})])

    def check(prob, res, reqs):
        _all_scheduled(prob, res, reqs)
        assert reqs[0][RESVID][4] == ("cr-xlarge",)
        assert names(cat, res.nodeclaim_types[0]) == ["m5.xlarge"]

    def launch_check(cat, lreqs, lres):
        _launch_reserved(cat, lres, 0, "cr-xlarge")
    return Kat("resv_specific_id", "test/suites/scheduling/suite_test.go:824-847", prob, check, launch_check)


@resv_case
def resv_specific_type(fx):
    cat, np_ = e2e_reservations(fx)
    cls = PodClass([Requirement(RESVTYPE, "In", ["default"]), Requirement(INSTANCE_TYPE, "In", ["m5.xlarge"])])
    prob = problem(cat, [np_], [cls], [(0, {})])

    def check(prob, res, reqs):
        _all_scheduled(prob, res, reqs)
        assert reqs[0][RESVID][4] == ("cr-xlarge",) and reqs[0][RESVTYPE][4] == ("default",)

    def launch_check(cat, lreqs, lres):
        _launch_reserved(cat, lres, 0, "cr-xlarge")
    return Kat("resv_specific_type", "test/suites/scheduling/suite_test.go:850-883", prob, check, launch_check)


def _fallback_pods(cat, np_):
    anti = model.TopologyTerm("anti", model.HOSTNAME, selector=[Requirement("foo", "In", ["bar"])])
    cls = PodClass([Requirement(INSTANCE_TYPE, "In", ["m5.large"])], labels={"foo": "bar"}, topology=[anti])
    return problem(cat, [np_], [cls], [(0, {})] * 2)


@resv_case
def resv_fallback_first_solve(fx):
    """:884-920, first provisioning loop: the first pod reserves the single m5.large instance; the second pod's new
    NodeClaim has a compatible reserved offering it cannot reserve (ReservedOfferingModeStrict) and waits."""
    cat, np_ = e2e_reservations(fx)
    prob = _fallback_pods(cat, np_)

    def check(prob, res, reqs):
        assert res.n_nodeclaims == 1 and sorted(res.pod_result.tolist()) == [-1, 0]
        assert reqs[0][RESVID][4] == ("cr-large",)

    def launch_check(cat, lreqs, lres):
        _launch_reserved(cat, lres, 0, "cr-large")
    return Kat("resv_fallback_first_solve", "test/suites/scheduling/suite_test.go:884-920", prob, check, launch_check)


@resv_case
def resv_fallback_second_solve(fx):
    """:884-920, the next loop: the reservation's available count is 0 (offering.go:187, Available = false), so the
    waiting pod gets an on-demand NodeClaim without a reservation requirement."""
    cat, np_ = e2e_reservations(fx, large_cap=0)
    prob = _fallback_pods(cat, np_)
    prob.pods = synth.pods_from_specs([(0, {})])

    def check(prob, res, reqs):
        _all_scheduled(prob, res, reqs)
        assert RESVID not in reqs[0] or reqs[0][RESVID][0] is True or reqs[0][RESVID][4] != ("cr-large",)

    def launch_check(cat, lreqs, lres):
        assert int(lres.rows[0]["capacity_type"]) == abi.KP_CT_ON_DEMAND
    return Kat("resv_fallback_second_solve", "test/suites/scheduling/suite_test.go:884-920", prob, check, launch_check)


def resv_ids():
    return [c.__name__ for c in RESV_CASES]
