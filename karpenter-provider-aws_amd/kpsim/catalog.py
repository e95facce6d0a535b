"""Catalog construction: the `[]*cloudprovider.InstanceType` that GetInstanceTypes hands the scheduler.

This is the host-side ingestion row: it restates, in Python, how the AWS provider builds
instance types and offerings, so tests and the bench can produce kp_catalog_view inputs from the
reference's committed data (tests/golden/*):

  new_instance_type  — pkg/providers/instancetype/types.go:123-299 (computeRequirements) and
                       :320-605 (computeCapacity, kubeReservedResources, evictionThreshold, pods, ...),
                       AMI feature flags pkg/providers/amifamily/resolver.go:102-119, bottlerocket.go:126-131,
                       windows.go:101-107.  Allocatable = Capacity − Overhead.Total().
  inject_offerings   — pkg/providers/instancetype/offering/offering.go:103-196 (one offering per
                       zone ∈ allZones × capacity type; Available = !ICE && hasPrice && zone ∈ itZones (:148);
                       reserved price = odPrice / 1e7 (:176)).
  golden_catalog     — the 918 types of website/content/en/preview/reference/instance-types.md that have a
                       static us-east-1 price (zz_generated.pricing_aws.go:23), allocatable taken from the doc.
  fake_catalog       — pkg/fake/zz_generated.describe_instance_types.go (17 types) with the envtest defaults of
                       pkg/test/options.go:37-55 and static prices (pricing.go Reset :443-455: spot = OD).

The C++ oracle restates the same resource arithmetic independently (oracle/orc_catalog.cpp); tests check
both against the golden doc.
"""
import gzip
import json
import math
import os
import re
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np

from .model import (ARCH, CAPACITY_TYPE, INSTANCE_TYPE, OS, R, RESERVATION_ID, RESERVATION_TYPE, RIDX,
                    ZONE, ZONE_ID, InstanceType, Offering)

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests", "golden")

Mi = 1024 * 1024
Gi = 1024 * Mi
AWS = "karpenter.k8s.aws/"
REGION = "topology.kubernetes.io/region"
WINDOWS_BUILD = "node.kubernetes.io/windows-build"

# Label keys computeRequirements always sets (types.go:181-234), DoesNotExist unless filled in.
TYPE_LABEL_KEYS = [
    INSTANCE_TYPE, ARCH, OS, ZONE, REGION, WINDOWS_BUILD, CAPACITY_TYPE,
    AWS + "instance-cpu", AWS + "instance-cpu-manufacturer", AWS + "instance-cpu-sustained-clock-speed-mhz",
    AWS + "instance-memory", AWS + "instance-ebs-bandwidth", AWS + "instance-network-bandwidth",
    AWS + "instance-category", AWS + "instance-capacity-flex", AWS + "instance-family", AWS + "instance-generation",
    AWS + "instance-local-nvme", AWS + "instance-size", AWS + "instance-gpu-name", AWS + "instance-gpu-manufacturer",
    AWS + "instance-gpu-count", AWS + "instance-gpu-memory", AWS + "instance-accelerator-name",
    AWS + "instance-accelerator-manufacturer", AWS + "instance-accelerator-count", AWS + "instance-hypervisor",
    AWS + "instance-encryption-in-transit-supported", RESERVATION_ID, RESERVATION_TYPE,
]
WINDOWS_BUILDS = {"Windows2019": "10.0.17763", "Windows2022": "10.0.20348"}   # pkg/apis/v1/labels.go:112-113
INSTANCE_TYPE_SCHEME = re.compile(r"(^[a-z]+)(\-[0-9]+tb)?([0-9]+).*\.")


@dataclass
class TypeOptions:
    """Inputs of NewInstanceType that come from options / EC2NodeClass."""
    vm_memory_overhead_pct: float = 0.075      # pkg/test/options.go:52
    reserved_enis: int = 0
    ami_family: str = "AL2023"                 # AL2023 | AL2 | Bottlerocket | Windows2022 | Custom
    max_pods: Optional[int] = None
    pods_per_core: Optional[int] = None
    raid0: bool = False


def _flags(fam):
    if fam == "Bottlerocket":
        return dict(eni_mem=False, ppc=False, evsoft=False, eni_pods=True)
    if fam.startswith("Windows"):
        return dict(eni_mem=False, ppc=True, evsoft=True, eni_pods=False)
    return dict(eni_mem=True, ppc=True, evsoft=True, eni_pods=True)


def _lower_kabob(s):
    return (s or "").replace(" ", "-").lower()


def _go_round(x):
    # math.Round: half away from zero
    return int(math.floor(abs(x) + 0.5)) * (1 if x >= 0 else -1)


def eni_limited_pods(info, reserved):
    cards = info["cards"]
    ifaces = cards[info["default_card"]] if cards else info["max_enis"]
    usable = max(int(ifaces) - reserved, 0)
    if usable == 0:
        return 0
    return usable * (int(info["ipv4_per_eni"]) - 1) + 2


def instance_resources(info, opts: TypeOptions, vpclimits=None):
    """computeCapacity + Overhead (types.go:320-605).  Returns (capacity, kube_reserved, eviction) [R] milli."""
    f = _flags(opts.ami_family)
    cap = np.zeros(R, np.int64)
    kube = np.zeros(R, np.int64)
    ev = np.zeros(R, np.int64)
    vcpus = int(info["vcpus"])
    cap[RIDX["cpu"]] = vcpus * 1000
    mib = int(info["memory_mib"])
    if info["architectures"] and info["architectures"][0] == "arm64":
        mib -= 64
    mem = mib * Mi
    mem -= int(math.ceil(float(mem) * opts.vm_memory_overhead_pct / 1024 / 1024)) * Mi
    cap[RIDX["memory"]] = mem * 1000
    # the AMI family's ephemeral block device default: 20Gi (resolver.go:40-43), Windows /dev/sda1 50Gi (windows.go:88-99)
    eph = 50 * Gi if opts.ami_family.startswith("Windows") else 20 * Gi
    if opts.raid0 and info.get("instance_storage_gb") is not None:
        eph = int(info["instance_storage_gb"]) * 1000 ** 3
    cap[RIDX["ephemeral-storage"]] = eph * 1000
    if opts.max_pods is not None:
        pods = opts.max_pods
    elif f["eni_pods"]:
        pods = eni_limited_pods(info, opts.reserved_enis)
    else:
        pods = 110
    if (opts.pods_per_core or 0) > 0 and f["ppc"]:
        pods = min(opts.pods_per_core * vcpus, pods)
    cap[RIDX["pods"]] = pods * 1000
    lim = (vpclimits or {}).get(info["name"])
    cap[RIDX["vpc.amazonaws.com/pod-eni"]] = lim["branch_interface"] * 1000 if lim and lim["trunking"] else 0
    gpus = info.get("gpus") or []
    cap[RIDX["nvidia.com/gpu"]] = sum(g["count"] for g in gpus if g["manufacturer"] == "NVIDIA") * 1000
    cap[RIDX["amd.com/gpu"]] = sum(g["count"] for g in gpus if g["manufacturer"] == "AMD") * 1000
    cap[RIDX["habana.ai/gaudi"]] = sum(g["count"] for g in gpus if g["manufacturer"] == "Habana") * 1000
    nd = info.get("neuron_devices")
    if nd:
        cap[RIDX["aws.amazon.com/neuron"]] = sum(d["count"] for d in nd) * 1000
        cap[RIDX["aws.amazon.com/neuroncore"]] = nd[0]["count"] * nd[0]["cores"] * 1000
    cap[RIDX["vpc.amazonaws.com/efa"]] = (info.get("efa_max") or 0) * 1000
    if opts.ami_family.startswith("Windows") and _arch(info) == "amd64":
        cap[RIDX["vpc.amazonaws.com/PrivateIPv4Address"]] = (lim["ipv4_per_interface"] - 1) * 1000 if lim else 0
    kpods = eni_limited_pods(info, 0) if f["eni_mem"] else pods
    kube[RIDX["memory"]] = (11 * kpods + 255) * Mi * 1000
    kube[RIDX["ephemeral-storage"]] = Gi * 1000
    cpu_m = vcpus * 1000
    kcpu = 0
    for start, end, pct in ((0, 1000, 0.06), (1000, 2000, 0.01), (2000, 4000, 0.005), (4000, 1 << 31, 0.0025)):
        if cpu_m >= start:
            r = float(end - start)
            if cpu_m < end:
                r = float(cpu_m - start)
            kcpu += int(r * pct)
    kube[RIDX["cpu"]] = kcpu
    ev[RIDX["memory"]] = 100 * Mi * 1000
    ev[RIDX["ephemeral-storage"]] = int(math.ceil(float(eph) / 100 * 10)) * 1000
    return cap, kube, ev


def _arch(info):
    for a in info["architectures"]:
        if a == "x86_64":
            return "amd64"
        if a == "arm64":
            return "arm64"
    return str(info["architectures"])


def compute_requirements(info, region, offering_zones, subnet_zone_info, opts: TypeOptions, bandwidth,
                         capacity_reservations=()):
    """computeRequirements (types.go:158-299) -> {key: [values] | None(DoesNotExist)}"""
    labels = {k: None for k in TYPE_LABEL_KEYS}
    cts = [u for u in info["usage_classes"] if u in ("on-demand", "spot")]
    if capacity_reservations:
        cts.append("reserved")
    subnet_zones = [z["zone"] for z in subnet_zone_info]
    avail = sorted(set(offering_zones) & set(subnet_zones))
    name = info["name"]
    labels[INSTANCE_TYPE] = [name]
    labels[ARCH] = [_arch(info)]
    if opts.ami_family.startswith("Windows"):
        labels[OS] = ["windows"] if _arch(info) == "amd64" else []
    else:
        labels[OS] = ["linux"]
    labels[ZONE] = avail
    labels[REGION] = [region]
    labels[CAPACITY_TYPE] = cts
    labels[AWS + "instance-cpu"] = [str(int(info["vcpus"]))]
    labels[AWS + "instance-memory"] = [str(int(info["memory_mib"]))]
    labels[AWS + "instance-hypervisor"] = [info.get("hypervisor") or ""]
    labels[AWS + "instance-encryption-in-transit-supported"] = ["true" if info.get("encryption_in_transit") else "false"]
    zone_ids = [z.get("zone_id", "") for z in subnet_zone_info if z["zone"] in avail]
    if zone_ids:
        labels[ZONE_ID] = sorted(set(zone_ids))
    if capacity_reservations:
        labels[RESERVATION_ID] = sorted(set(cr["id"] for cr in capacity_reservations))
        labels[RESERVATION_TYPE] = sorted(set(cr["type"] for cr in capacity_reservations))
    m = INSTANCE_TYPE_SCHEME.search(name)
    if m:
        labels[AWS + "instance-category"] = [m.group(1)]
        labels[AWS + "instance-generation"] = [m.group(3)]
    parts = name.split(".")
    if len(parts) == 2:
        labels[AWS + "instance-family"] = [parts[0]]
        labels[AWS + "instance-size"] = [parts[1]]
    if info.get("instance_storage_gb") is not None and info.get("instance_storage_nvme") != "unsupported":
        labels[AWS + "instance-local-nvme"] = [str(int(info["instance_storage_gb"]))]
    labels[AWS + "instance-capacity-flex"] = ["true" if "-flex" in parts[0] else "false"]
    if name in bandwidth:
        labels[AWS + "instance-network-bandwidth"] = [str(bandwidth[name])]
    gpus = info.get("gpus") or []
    if len(gpus) == 1:
        g = gpus[0]
        labels[AWS + "instance-gpu-name"] = [_lower_kabob(g["name"])]
        labels[AWS + "instance-gpu-manufacturer"] = [_lower_kabob(g["manufacturer"])]
        labels[AWS + "instance-gpu-count"] = [str(g["count"])]
        labels[AWS + "instance-gpu-memory"] = [str(g["memory_mib"])]
    accs = info.get("inference_accelerators")
    if accs and len(accs) == 1 and info.get("neuron_devices") is None:
        a = accs[0]
        labels[AWS + "instance-accelerator-name"] = [_lower_kabob(a["name"])]
        labels[AWS + "instance-accelerator-manufacturer"] = [_lower_kabob(a["manufacturer"])]
        labels[AWS + "instance-accelerator-count"] = [str(a["count"])]
    nd = info.get("neuron_devices")
    if nd and len(nd) == 1:
        labels[AWS + "instance-accelerator-name"] = [_lower_kabob(nd[0]["name"])]
        labels[AWS + "instance-accelerator-manufacturer"] = ["aws"]
        labels[AWS + "instance-accelerator-count"] = [str(nd[0]["count"])]
    if opts.ami_family in WINDOWS_BUILDS:   # types.go:281-284
        labels[WINDOWS_BUILD] = [WINDOWS_BUILDS[opts.ami_family]]
    labels[AWS + "instance-cpu-manufacturer"] = [_lower_kabob(info.get("cpu_manufacturer"))]
    ghz = float(info.get("sustained_clock_ghz") or 0.0)
    labels[AWS + "instance-cpu-sustained-clock-speed-mhz"] = [str(_go_round(ghz * 1000))]
    if info.get("ebs_max_bandwidth_mbps") is not None and info.get("ebs_optimized_support") == "default":
        labels[AWS + "instance-ebs-bandwidth"] = [str(info["ebs_max_bandwidth_mbps"])]
    # an empty In set is DoesNotExist
    return {k: (v if v else None) if v is not None else None for k, v in labels.items()}


def new_instance_type(info, opts: TypeOptions, region, offering_zones, subnet_zone_info, bandwidth, vpclimits,
                      capacity_reservations=()):
    labels = compute_requirements(info, region, offering_zones, subnet_zone_info, opts, bandwidth, capacity_reservations)
    cap, kube, ev = instance_resources(info, opts, vpclimits)
    return InstanceType(info["name"], labels, cap, cap - kube - ev, [])


def inject_offerings(it: InstanceType, all_zones, zone_ids: Dict[str, str], od_price: Optional[float],
                     spot_price, unavailable=lambda ct, zone: False, reservations=()):
    """createOfferings (offering.go:103-196).  spot_price(zone) -> float|None."""
    it_zones = set(it.labels.get(ZONE) or [])
    offs = []
    for zone in all_zones:
        for ct in (it.labels.get(CAPACITY_TYPE) or []):
            if ct == "reserved":
                continue
            if ct == "on-demand":
                price, has = (od_price, True) if od_price is not None else (0.0, False)
            else:
                sp = spot_price(zone)
                price, has = (sp, True) if sp is not None else (0.0, False)
            offs.append(Offering(ct, zone, float(price), (not unavailable(ct, zone)) and has and zone in it_zones,
                                 zone_id=zone_ids.get(zone)))
    for cr in reservations:
        price = od_price / 10_000_000.0 if od_price is not None else 0.0
        offs.append(Offering("reserved", cr["zone"], price,
                             cr["capacity"] != 0 and cr["zone"] in it_zones and cr.get("state") != "expiring",
                             zone_id=zone_ids.get(cr["zone"]), reservation_id=cr["id"],
                             reservation_type=cr["type"], reservation_capacity=cr["capacity"]))
    it.offerings = offs
    return it


# ------------------------------------------------------------------------------------------------
# fixtures
# ------------------------------------------------------------------------------------------------
def _load(name):
    p = os.path.join(GOLDEN_DIR, name)
    if name.endswith(".gz"):
        with gzip.open(p, "rt") as f:
            return json.load(f)
    with open(p) as f:
        return json.load(f)


def load_fixtures():
    return dict(golden=_load("catalog_golden.json.gz"), prices=_load("prices_us_east_1.json"),
                vpclimits=_load("vpclimits.json.gz"), bandwidth=_load("bandwidth.json"), fake=_load("fake_catalog.json"),
                kats=_load("kats.json"))


def parse_quantity_milli(s: str) -> int:
    """resource.Quantity string -> MilliValue() (exact for the forms in the fixtures)."""
    from fractions import Fraction
    m = re.fullmatch(r"([+-]?[0-9.]+)([a-zA-Z]*)", s.strip())
    num, suf = Fraction(m.group(1)), m.group(2)
    mult = {"": 1, "n": Fraction(1, 10 ** 9), "u": Fraction(1, 10 ** 6), "m": Fraction(1, 1000), "k": 10 ** 3,
            "M": 10 ** 6, "G": 10 ** 9, "T": 10 ** 12, "P": 10 ** 15, "E": 10 ** 18, "Ki": 2 ** 10, "Mi": 2 ** 20,
            "Gi": 2 ** 30, "Ti": 2 ** 40, "Pi": 2 ** 50, "Ei": 2 ** 60}[suf]
    v = num * mult * 1000
    return int(math.ceil(v))


def golden_info(row, vpclimits):
    """Reconstruct the EC2 fields the resource arithmetic needs from a golden-doc row + vpclimits."""
    lab = row["labels"]
    lim = vpclimits.get(row["name"])
    arch = lab.get(ARCH, "amd64")
    return {
        "name": row["name"], "vcpus": int(lab[AWS + "instance-cpu"]), "memory_mib": int(lab[AWS + "instance-memory"]),
        "architectures": ["arm64" if arch == "arm64" else "x86_64"],
        "cards": lim["cards"] if lim else [], "default_card": lim["default_card"] if lim else 0,
        "max_enis": lim["interface"] if lim else 0, "ipv4_per_eni": lim["ipv4_per_interface"] if lim else 0,
        "usage_classes": ["on-demand", "spot"], "instance_storage_gb": None,
    }


def golden_catalog(zones=("test-zone-1a", "test-zone-1b", "test-zone-1c"),
                   zone_ids=("use1-az1", "use1-az2", "use1-az4"), region="us-east-1", seed=20250912,
                   ice_fraction=0.02, spot=True, reservations=None, fx=None) -> List[InstanceType]:
    """SURVEY §8d catalog: golden doc ∩ static us-east-1 prices (918 types) × zones × {on-demand, spot}.

    Labels and allocatable come from the golden doc; capacity from the restated arithmetic (cpu/memory/pods/
    ephemeral; other resources have no overhead, so capacity = allocatable).  Spot price (type, zone) =
    round(OD × U(0.25, 0.75), 3); `ice_fraction` of (type, zone, capacity-type) offerings are unavailable.
    `reservations`: {type name: [ {id, zone, type, capacity, state} ]} adds reserved offerings (config 5).
    """
    fx = fx or load_fixtures()
    rng = np.random.Generator(np.random.PCG64(seed))
    prices = fx["prices"]
    zone_id = dict(zip(zones, zone_ids))
    subnet_info = [{"zone": z, "zone_id": zone_id[z]} for z in zones]
    out = []
    for row in fx["golden"]:
        name = row["name"]
        if name not in prices:
            continue
        od = float(prices[name])
        info = golden_info(row, fx["vpclimits"])
        opts = TypeOptions()
        crs = (reservations or {}).get(name, [])
        labels = {k: None for k in TYPE_LABEL_KEYS}
        for k, v in row["labels"].items():
            labels[k] = [v]
        labels[ZONE] = list(zones)
        labels[REGION] = [region]
        labels[CAPACITY_TYPE] = ["on-demand", "spot"] + (["reserved"] if crs else [])
        labels[ZONE_ID] = [zone_id[z] for z in zones]
        labels[AWS + "instance-capacity-flex"] = ["true" if "-flex" in name.split(".")[0] else "false"]
        if crs:
            labels[RESERVATION_ID] = sorted(set(c["id"] for c in crs))
            labels[RESERVATION_TYPE] = sorted(set(c["type"] for c in crs))
        alloc = np.zeros(R, np.int64)
        for res, q in row["allocatable"].items():
            alloc[RIDX[res]] = parse_quantity_milli(q)
        cap_calc, kube, ev = instance_resources(info, opts, fx["vpclimits"])
        cap = alloc.copy()
        for res in ("cpu", "memory", "ephemeral-storage"):
            cap[RIDX[res]] = alloc[RIDX[res]] + kube[RIDX[res]] + ev[RIDX[res]]
        it = InstanceType(name, labels, cap, alloc)
        spot_prices = {z: round(od * rng.uniform(0.25, 0.75), 3) for z in zones}
        ice = {(ct, z): bool(rng.random() < ice_fraction) for z in zones for ct in ("on-demand", "spot")}
        inject_offerings(it, list(zones), zone_id, od, (lambda z: spot_prices[z]) if spot else (lambda z: od),
                         unavailable=lambda ct, z: ice[(ct, z)], reservations=crs)
        out.append(it)
    return out


def fake_catalog(opts: TypeOptions = None, zones=("test-zone-1a", "test-zone-1b", "test-zone-1c"), fx=None,
                 extra_infos=(), extra_offerings=(), ice=(), spot_prices=None, reservations=None) -> List[InstanceType]:
    """The envtest catalog: pkg/fake 17 types, subnets test-zone-1a/1b/1c (instancetype/suite_test.go:119-137),
    static us-east-1 prices with spot = on-demand until a spot refresh (pricing.go:443-455).

    ice: {(capacity type, type name, zone)} marked unavailable (the UnavailableOfferings cache after an ICE,
    fake.CapacityPool).  spot_prices: {(type name, zone): price} after UpdateSpotPricing — pairs without an entry have
    no spot price and so no available spot offering (offering.go:148).  reservations: {type name: [cr dicts]}."""
    fx = fx or load_fixtures()
    opts = opts or TypeOptions()
    fake = fx["fake"]
    infos = list(fake["instance_types"]) + list(extra_infos)
    offerings = list(fake["offerings"]) + list(extra_offerings)
    by_type = {}
    all_zones = []
    for t, z in offerings:
        by_type.setdefault(t, []).append(z)
        if z not in all_zones:
            all_zones.append(z)
    # the suite's EC2NodeClass status subnets (pkg/test/nodeclass.go:103-119): test-zone-1x ↔ tstz1-1x
    subnet_info = [{"zone": z, "zone_id": "tstz1-" + z.rsplit("-", 1)[-1]} for z in zones]
    zone_ids = {s["zone"]: s["zone_id"] for s in subnet_info}
    ice = set(ice)
    out = []
    for info in infos:
        name = info["name"]
        crs = (reservations or {}).get(name, [])
        it = new_instance_type(info, opts, "us-west-2", by_type.get(name, []), subnet_info, fx["bandwidth"],
                               fx["vpclimits"], capacity_reservations=crs)
        od = fx["prices"].get(name)
        od = float(od) if od is not None else None
        if spot_prices is None:
            spot = lambda z, od=od: od   # noqa: E731
        else:
            spot = lambda z, name=name: spot_prices.get((name, z))   # noqa: E731
        inject_offerings(it, all_zones, zone_ids, od, spot, unavailable=lambda ct, z, name=name: (ct, name, z) in ice,
                         reservations=crs)
        out.append(it)
    return out
