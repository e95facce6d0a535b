"""Host mirror of the catalog-ingestion C-ABI (kp_catalog_build, include/kpsim.h).

`build_catalog` marshals raw EC2 instance-type data (the fields of ec2types.InstanceTypeInfo the provider reads, joined
with the vpclimits / bandwidth tables) and an EC2NodeClass into the library, which runs NewInstanceType
(pkg/providers/instancetype/types.go:123-605) and createOfferings (offering/offering.go:103-196) in C++
(csrc/kp_ingest.cpp).  The result is a `NativeCatalog` whose `.view` feeds Context.upload_catalog directly, like
model.CatalogView; `.instance_types()` decodes it back into model.InstanceType rows for inspection and tests.
"""
import ctypes as C
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi, model
from .native import KpError, load

AMI = {"AL2": 0, "AL2023": 1, "Bottlerocket": 2, "Windows2019": 3, "Windows2022": 4, "Custom": 5}
CATALOG_R = 12


class kp_ec2_device(C.Structure):
    _fields_ = [("name", C.c_char_p), ("manufacturer", C.c_char_p), ("count", C.c_int32), ("memory_mib", C.c_int32),
                ("cores", C.c_int32)]


class kp_ec2_instance_type(C.Structure):
    _fields_ = [
        ("name", C.c_char_p), ("default_vcpus", C.c_int32), ("memory_mib", C.c_int64),
        ("n_architectures", C.c_int32), ("architectures", abi.c_char_pp), ("has_processor_info", C.c_int32),
        ("cpu_manufacturer", C.c_char_p), ("sustained_clock_ghz", C.c_double),
        ("n_usage_classes", C.c_int32), ("usage_classes", abi.c_char_pp), ("hypervisor", C.c_char_p),
        ("encryption_in_transit", C.c_int32), ("n_network_cards", C.c_int32), ("card_max_interfaces", abi.c_int32_p),
        ("default_card", C.c_int32), ("max_network_interfaces", C.c_int32), ("ipv4_per_interface", C.c_int32),
        ("efa_max", C.c_int32), ("instance_storage_gb", C.c_int64), ("nvme_support", C.c_char_p),
        ("n_gpus", C.c_int32), ("gpus", C.POINTER(kp_ec2_device)),
        ("n_accelerators", C.c_int32), ("accelerators", C.POINTER(kp_ec2_device)),
        ("n_neuron", C.c_int32), ("neuron", C.POINTER(kp_ec2_device)),
        ("ebs_max_bandwidth_mbps", C.c_int64), ("ebs_optimized_support", C.c_char_p),
        ("has_vpc_limits", C.c_int32), ("vpc_trunking", C.c_int32), ("vpc_branch_interface", C.c_int32),
        ("vpc_ipv4_per_interface", C.c_int32), ("network_bandwidth_mbps", C.c_int64),
    ]


class kp_string_pair(C.Structure):
    _fields_ = [("key", C.c_char_p), ("value", C.c_char_p)]


class kp_zone_info(C.Structure):
    _fields_ = [("zone", C.c_char_p), ("zone_id", C.c_char_p)]


class kp_block_device_mapping(C.Structure):
    _fields_ = [("device_name", C.c_char_p), ("root_volume", C.c_int32), ("volume_size", C.c_char_p)]


class kp_capacity_reservation(C.Structure):
    _fields_ = [("id", C.c_char_p), ("instance_type", C.c_char_p), ("availability_zone", C.c_char_p),
                ("reservation_type", C.c_char_p), ("expiring", C.c_int32), ("available_count", C.c_int32)]


class kp_nodeclass_view(C.Structure):
    _fields_ = [
        ("ami_family", C.c_int32), ("region", C.c_char_p), ("n_zones", C.c_int32), ("zones", C.POINTER(kp_zone_info)),
        ("n_block_device_mappings", C.c_int32), ("block_device_mappings", C.POINTER(kp_block_device_mapping)),
        ("instance_store_raid0", C.c_int32), ("max_pods", C.c_int32), ("pods_per_core", C.c_int32),
        ("n_kube_reserved", C.c_int32), ("kube_reserved", C.POINTER(kp_string_pair)),
        ("n_system_reserved", C.c_int32), ("system_reserved", C.POINTER(kp_string_pair)),
        ("n_eviction_hard", C.c_int32), ("eviction_hard", C.POINTER(kp_string_pair)),
        ("n_eviction_soft", C.c_int32), ("eviction_soft", C.POINTER(kp_string_pair)),
        ("n_capacity_reservations", C.c_int32), ("capacity_reservations", C.POINTER(kp_capacity_reservation)),
        ("vm_memory_overhead_percent", C.c_double), ("reserved_enis", C.c_int32), ("reserved_capacity", C.c_int32),
    ]


class kp_offering_source(C.Structure):
    _fields_ = [("n_zones", C.c_int32), ("zones", abi.c_char_pp), ("type_zones", abi.c_char_pp),
                ("od_price", abi.c_double_p), ("spot_price", abi.c_double_p), ("unavailable", abi.c_uint8_p)]


_bound = False


def lib():
    global _bound
    L = load()
    if not _bound:
        L.kp_catalog_build.argtypes = [C.c_int32, C.POINTER(kp_ec2_instance_type), C.POINTER(kp_nodeclass_view),
                                       C.POINTER(kp_offering_source), C.POINTER(C.c_void_p)]
        L.kp_catalog_get_view.argtypes = [C.c_void_p, C.POINTER(abi.kp_catalog_view)]
        L.kp_catalog_overhead.argtypes = [C.c_void_p, C.c_int32, abi.c_int64_p]
        L.kp_catalog_resource_name.argtypes = [C.c_int32]
        L.kp_catalog_resource_name.restype = C.c_char_p
        L.kp_catalog_free.argtypes = [C.c_void_p]
        for f in ("kp_catalog_build", "kp_catalog_get_view", "kp_catalog_overhead", "kp_catalog_free"):
            getattr(L, f).restype = C.c_int32
        _bound = True
    return L


@dataclass
class NodeClass:
    """EC2NodeClass fields (spec + resolved status) and provider options that NewInstanceType / createOfferings read."""
    ami_family: str = "AL2023"
    region: str = "us-west-2"
    zones: Sequence[Tuple[str, str]] = ()                  # status subnets: (zone, zone id)
    block_device_mappings: Sequence[Tuple[str, bool, Optional[str]]] = ()   # (device name, root volume, volume size)
    raid0: bool = False
    max_pods: Optional[int] = None
    pods_per_core: Optional[int] = None
    kube_reserved: Dict[str, str] = field(default_factory=dict)
    system_reserved: Dict[str, str] = field(default_factory=dict)
    eviction_hard: Optional[Dict[str, str]] = None
    eviction_soft: Optional[Dict[str, str]] = None
    capacity_reservations: Sequence[dict] = ()             # {id, instance_type, zone, type, capacity, state}
    vm_memory_overhead_pct: float = 0.075                  # pkg/test/options.go:52
    reserved_enis: int = 0
    reserved_capacity: bool = True


def ec2_info(k: abi.Keep, info: dict, vpclimits: dict, bandwidth: dict) -> kp_ec2_instance_type:
    """kp_ec2_instance_type from a tests/golden/fake_catalog.json-style record (pkg/fake describe output)."""
    x = kp_ec2_instance_type()
    name = info["name"]
    x.name = name.encode()
    x.default_vcpus = int(info["vcpus"])
    x.memory_mib = int(info["memory_mib"])
    archs = list(info.get("architectures") or [])
    x.n_architectures = len(archs)
    x.architectures = k.cstrs(archs)
    x.has_processor_info = 1
    x.cpu_manufacturer = (info.get("cpu_manufacturer") or "").encode() if info.get("cpu_manufacturer") is not None else None
    ghz = info.get("sustained_clock_ghz")
    x.sustained_clock_ghz = float(ghz) if ghz is not None else math.nan
    uc = list(info.get("usage_classes") or [])
    x.n_usage_classes = len(uc)
    x.usage_classes = k.cstrs(uc)
    x.hypervisor = (info.get("hypervisor") or "").encode()
    x.encryption_in_transit = 1 if info.get("encryption_in_transit") else 0
    cards = list(info.get("cards") or [])
    x.n_network_cards = len(cards)
    x.card_max_interfaces = k.ptr(np.array(cards or [0], np.int32), np.int32, C.c_int32)
    x.default_card = int(info.get("default_card") or 0)
    x.max_network_interfaces = int(info.get("max_enis") or 0)
    x.ipv4_per_interface = int(info.get("ipv4_per_eni") or 0)
    x.efa_max = int(info.get("efa_max") or 0)
    sg = info.get("instance_storage_gb")
    x.instance_storage_gb = int(sg) if sg is not None else -1
    x.nvme_support = info["instance_storage_nvme"].encode() if info.get("instance_storage_nvme") else None

    def devs(lst, n_attr, p_attr, nil_negative):
        if lst is None:
            setattr(x, n_attr, -1 if nil_negative else 0)
            return
        arr = (kp_ec2_device * max(1, len(lst)))()
        for i, d in enumerate(lst):
            arr[i].name = (d.get("name") or "").encode()
            arr[i].manufacturer = (d.get("manufacturer") or "").encode()
            arr[i].count = int(d.get("count") or 0)
            arr[i].memory_mib = int(d.get("memory_mib") or 0)
            arr[i].cores = int(d.get("cores") or 0)
        setattr(x, n_attr, len(lst))
        setattr(x, p_attr, k.hold(arr))

    devs(info.get("gpus") or [], "n_gpus", "gpus", False)
    devs(info.get("inference_accelerators"), "n_accelerators", "accelerators", True)
    devs(info.get("neuron_devices"), "n_neuron", "neuron", True)
    eb = info.get("ebs_max_bandwidth_mbps")
    x.ebs_max_bandwidth_mbps = int(eb) if eb is not None else -1
    x.ebs_optimized_support = (info.get("ebs_optimized_support") or "").encode()
    lim = (vpclimits or {}).get(name)
    x.has_vpc_limits = 1 if lim else 0
    if lim:
        x.vpc_trunking = 1 if lim["trunking"] else 0
        x.vpc_branch_interface = int(lim["branch_interface"])
        x.vpc_ipv4_per_interface = int(lim["ipv4_per_interface"])
    bw = (bandwidth or {}).get(name)
    x.network_bandwidth_mbps = int(bw) if bw is not None else -1
    return x


def _pairs(k, d):
    d = d or {}
    arr = (kp_string_pair * max(1, len(d)))()
    for i, (a, b) in enumerate(d.items()):
        arr[i].key = a.encode()
        arr[i].value = b.encode()
    return len(d), k.hold(arr)


def nodeclass_view(k: abi.Keep, nc: NodeClass) -> kp_nodeclass_view:
    v = kp_nodeclass_view()
    v.ami_family = AMI[nc.ami_family]
    v.region = nc.region.encode()
    zs = (kp_zone_info * max(1, len(nc.zones)))()
    for i, (z, zid) in enumerate(nc.zones):
        zs[i].zone = z.encode()
        zs[i].zone_id = zid.encode() if zid is not None else None
    v.n_zones, v.zones = len(nc.zones), k.hold(zs)
    bd = (kp_block_device_mapping * max(1, len(nc.block_device_mappings)))()
    for i, (dev, root, size) in enumerate(nc.block_device_mappings):
        bd[i].device_name = dev.encode() if dev else None
        bd[i].root_volume = 1 if root else 0
        bd[i].volume_size = size.encode() if size else None
    v.n_block_device_mappings, v.block_device_mappings = len(nc.block_device_mappings), k.hold(bd)
    v.instance_store_raid0 = 1 if nc.raid0 else 0
    v.max_pods = nc.max_pods if nc.max_pods is not None else -1
    v.pods_per_core = nc.pods_per_core if nc.pods_per_core is not None else 0
    v.n_kube_reserved, v.kube_reserved = _pairs(k, nc.kube_reserved)
    v.n_system_reserved, v.system_reserved = _pairs(k, nc.system_reserved)
    if nc.eviction_hard is not None:
        v.n_eviction_hard, v.eviction_hard = _pairs(k, nc.eviction_hard)
    if nc.eviction_soft is not None:
        v.n_eviction_soft, v.eviction_soft = _pairs(k, nc.eviction_soft)
    crs = (kp_capacity_reservation * max(1, len(nc.capacity_reservations)))()
    for i, cr in enumerate(nc.capacity_reservations):
        crs[i].id = cr["id"].encode()
        crs[i].instance_type = cr["instance_type"].encode()
        crs[i].availability_zone = cr["zone"].encode()
        crs[i].reservation_type = cr.get("type", "default").encode()
        crs[i].expiring = 1 if cr.get("state") == "expiring" else 0
        crs[i].available_count = int(cr["capacity"])
    v.n_capacity_reservations, v.capacity_reservations = len(nc.capacity_reservations), k.hold(crs)
    v.vm_memory_overhead_percent = nc.vm_memory_overhead_pct
    v.reserved_enis = nc.reserved_enis
    v.reserved_capacity = 1 if nc.reserved_capacity else 0
    return v


class NativeCatalog:
    """A kp_catalog built by the library; `.view` is its kp_catalog_view (valid while this object lives)."""

    def __init__(self, h):
        self.L = lib()
        self.h = h
        self.view = abi.kp_catalog_view()
        st = self.L.kp_catalog_get_view(self.h, C.byref(self.view))
        if st != abi.KP_OK:
            raise KpError(st, "kp_catalog_get_view")

    def close(self):
        if self.h:
            self.L.kp_catalog_free(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def __len__(self):
        return self.view.n_types

    def overhead(self, t) -> np.ndarray:
        out = np.zeros(CATALOG_R, np.int64)
        st = self.L.kp_catalog_overhead(self.h, t, out.ctypes.data_as(C.POINTER(C.c_int64)))
        if st != abi.KP_OK:
            raise KpError(st, "kp_catalog_overhead")
        return out

    def instance_types(self) -> List[model.InstanceType]:
        """Decode the view into model.InstanceType rows (labels: key -> values or None for DoesNotExist)."""
        v = self.view
        T, K, Rr = v.n_types, v.n_label_keys, v.n_resources
        keys = [v.label_keys[i].decode() for i in range(K)]
        assert [v.resource_names[r].decode() for r in range(Rr)] == model.RESOURCES
        out = []
        for t in range(T):
            labels = {}
            for j in range(K):
                st = v.label_state[t * K + j]
                if st == abi.KP_LABEL_ABSENT:
                    continue
                if st == abi.KP_LABEL_DOES_NOT_EXIST:
                    labels[keys[j]] = None
                else:
                    a, b = v.label_offsets[t * K + j], v.label_offsets[t * K + j + 1]
                    labels[keys[j]] = [v.label_values[i].decode() for i in range(a, b)]
            cap = np.array([v.capacity[t * Rr + r] for r in range(Rr)], np.int64)
            alloc = np.array([v.allocatable[t * Rr + r] for r in range(Rr)], np.int64)
            out.append(model.InstanceType(v.type_names[t].decode(), labels, cap, alloc, []))
        KO = v.n_offering_keys
        okeys = [v.offering_keys[q].decode() for q in range(KO)]
        for o in range(v.n_offerings):
            lab = {}
            for q in range(KO):
                st = v.offering_label_state[o * KO + q]
                lab[okeys[q]] = v.offering_label_values[o * KO + q].decode() if st == abi.KP_LABEL_IN else None
            out[v.offering_type[o]].offerings.append(model.Offering(
                lab[model.CAPACITY_TYPE], lab[model.ZONE], float(v.offering_price[o]), bool(v.offering_available[o]),
                zone_id=lab.get(model.ZONE_ID), reservation_id=lab.get(model.RESERVATION_ID),
                reservation_type=lab.get(model.RESERVATION_TYPE),
                reservation_capacity=int(v.offering_reservation_capacity[o])))
        return out


def build_catalog(infos: Sequence[dict], nodeclass: NodeClass, all_zones: Sequence[str],
                  type_zones: Sequence[Sequence[str]], od_price: Sequence[Optional[float]],
                  spot_price=None, unavailable=None, vpclimits=None, bandwidth=None) -> NativeCatalog:
    """kp_catalog_build over fixture-style EC2 records.

    type_zones[t]: the zones DescribeInstanceTypeOfferings lists for type t; od_price[t]: on-demand price or None;
    spot_price: [T][Z] array (NaN = no price), None = spot priced as on-demand (pricing.go Reset :443-455);
    unavailable: [T][Z][2] ICE bools (od, spot) or None."""
    L = lib()
    k = abi.Keep()
    T, Z = len(infos), len(all_zones)
    arr = (kp_ec2_instance_type * max(1, T))()
    for t, info in enumerate(infos):
        arr[t] = ec2_info(k, info, vpclimits, bandwidth)
    ncv = nodeclass_view(k, nodeclass)
    od = np.array([p if p is not None else np.nan for p in od_price], np.float64)
    if spot_price is None:
        sp = np.repeat(od[:, None], Z, axis=1)
    else:
        sp = np.asarray(spot_price, np.float64).reshape(T, Z)
    src = kp_offering_source()
    src.n_zones = Z
    src.zones = k.cstrs(list(all_zones))
    src.type_zones = k.cstrs(["\n".join(z) for z in type_zones])
    src.od_price = k.ptr(od if T else np.zeros(1), np.float64, C.c_double)
    src.spot_price = k.ptr(sp.reshape(-1) if T else np.zeros(1), np.float64, C.c_double)
    if unavailable is not None:
        src.unavailable = k.ptr(np.asarray(unavailable, np.uint8).reshape(-1), np.uint8, C.c_uint8)
    h = C.c_void_p()
    st = L.kp_catalog_build(T, arr, C.byref(ncv), C.byref(src), C.byref(h))
    if st != abi.KP_OK:
        raise KpError(st, "kp_catalog_build")
    return NativeCatalog(h)


def fake_catalog(fx, nodeclass: Optional[NodeClass] = None, zones=("test-zone-1a", "test-zone-1b", "test-zone-1c"),
                 extra_infos=(), extra_offerings=(), ice=(), spot_prices=None) -> NativeCatalog:
    """The envtest catalog of kpsim.catalog.fake_catalog, built by the library: pkg/fake's 17 types, subnets
    test-zone-1a/1b/1c ↔ tstz1-1a/1b/1c, static prices with spot = on-demand unless spot_prices is given."""
    nc = nodeclass or NodeClass()
    if not nc.zones:
        nc.zones = [(z, "tstz1-" + z.rsplit("-", 1)[-1]) for z in zones]
    infos = list(fx["fake"]["instance_types"]) + list(extra_infos)
    offerings = list(fx["fake"]["offerings"]) + list(extra_offerings)
    by_type, all_zones = {}, []
    for t, z in offerings:
        by_type.setdefault(t, []).append(z)
        if z not in all_zones:
            all_zones.append(z)
    od = [float(fx["prices"][i["name"]]) if i["name"] in fx["prices"] else None for i in infos]
    sp = None
    if spot_prices is not None:
        sp = [[spot_prices.get((i["name"], z), np.nan) for z in all_zones] for i in infos]
    ice = set(ice)
    un = [[[(ct, i["name"], z) in ice for ct in ("on-demand", "spot")] for z in all_zones] for i in infos]
    return build_catalog(infos, nc, all_zones, [by_type.get(i["name"], []) for i in infos], od, sp, un,
                         fx["vpclimits"], fx["bandwidth"])
