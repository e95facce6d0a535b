"""Seeded synthetic workloads for BASELINE.json configs and small KAT problems.

Every generator is deterministic in its seed (PCG64, default 20250912).  Pods carry requests as
resources.RequestsForPods would produce them ([core] pkg/utils/resources: Ceiling(pod).Requests merged,
plus `pods: 1`), creation timestamps and UIDs that make the queue order total.
"""
from typing import Dict, List, Optional

import numpy as np

from .catalog import golden_catalog, parse_quantity_milli
from . import abi, model
from .model import (ARCH, CAPACITY_TYPE, NODEPOOL, R, RIDX, ZONE, Candidate, ConsolidationProblem, ExistingNode,
                    NodePool, PodClass, Pods, Problem, Requirement, Taint, Toleration)

SEED = 20250912
AWS = "karpenter.k8s.aws/"


def requests_vec(req: Dict[str, str]) -> np.ndarray:
    v = np.zeros(R, np.int64)
    for k, q in req.items():
        v[RIDX[k]] = parse_quantity_milli(q) if isinstance(q, str) else int(q)
    v[RIDX["pods"]] += 1000
    return v


def pods_from_specs(specs, t0=1_700_000_000 * 10 ** 9):
    """specs: list of (class_id, {resource: quantity}) in creation order."""
    n = len(specs)
    cls = np.array([c for c, _ in specs], np.int32)
    req = np.stack([requests_vec(r) for _, r in specs]) if n else np.zeros((0, R), np.int64)
    ts = t0 + np.arange(n, dtype=np.int64) * 10 ** 9
    uids = ["%08x-0000-4000-8000-%012x" % (i, i) for i in range(n)]
    return Pods(cls, req, ts, uids)


def default_nodepool(name="default", capacity_types=("on-demand",), **kw) -> NodePool:
    reqs = [Requirement(CAPACITY_TYPE, "In", list(capacity_types))]
    reqs += kw.pop("requirements", [])
    return NodePool(name=name, requirements=reqs, **kw)


# ------------------------------------------------------------------------------------------------
# BASELINE configs
# ------------------------------------------------------------------------------------------------
def config1(n_pods=2000, catalog=None, seed=SEED) -> Problem:
    """2,000 homogeneous pods (cpu 1, memory 1Gi), one NodePool `capacity-type In [on-demand]`."""
    catalog = catalog if catalog is not None else golden_catalog(seed=seed)
    pods = pods_from_specs([(0, {"cpu": "1", "memory": "1Gi"})] * n_pods)
    return Problem(catalog, [default_nodepool()], [PodClass()], pods)


def _classes_config2(rng, n_classes, taint_key):
    """250 pod classes: cpu ∈ {100m..8} weighted small, memory = cpu × {1,2,4,8} GiB, 10% ephemeral-storage (256Mi–4Gi; every type has 17Gi allocatable with the default 20Gi root volume),
    2% nvidia.com/gpu, 30% nodeSelectors over {arch, capacity-type, zone, instance-category, generation Gt 4},
    20% tolerate the tainted template."""
    cpus = np.array([100, 250, 500, 1000, 2000, 4000, 8000])
    cpu_w = np.array([0.22, 0.22, 0.2, 0.16, 0.1, 0.06, 0.04])
    classes, reqs = [], []
    for c in range(n_classes):
        cpu_m = int(rng.choice(cpus, p=cpu_w))
        ratio = int(rng.choice([1, 2, 4, 8]))
        mem = cpu_m * ratio * (1 << 30) // 1000  # bytes
        r = {"cpu": cpu_m, "memory": mem * 1000}
        if rng.random() < 0.10:
            r["ephemeral-storage"] = int(rng.choice([256, 512, 1024, 2048, 4096])) * (1 << 20) * 1000
        if rng.random() < 0.02:
            r["nvidia.com/gpu"] = int(rng.choice([1, 2, 4, 8])) * 1000
        sel = []
        if rng.random() < 0.30:
            kind = int(rng.integers(0, 5))
            if kind == 0:
                sel.append(Requirement(ARCH, "In", [str(rng.choice(["amd64", "arm64"]))]))
            elif kind == 1:
                sel.append(Requirement(CAPACITY_TYPE, "In", [str(rng.choice(["spot", "on-demand"]))]))
            elif kind == 2:
                sel.append(Requirement(ZONE, "In", [str(rng.choice(["test-zone-1a", "test-zone-1b", "test-zone-1c"]))]))
            elif kind == 3:
                sel.append(Requirement(AWS + "instance-category", "In",
                                       sorted(set(rng.choice(["c", "m", "r", "t"], size=2).tolist()))))
            else:
                sel.append(Requirement(AWS + "instance-generation", "Gt", ["4"]))
        tols = []
        if rng.random() < 0.20:
            tols.append(Toleration(key=taint_key, operator="Exists", effect="NoSchedule"))
        classes.append(PodClass(sel, tols))
        reqs.append(r)
    return classes, reqs


def config2(n_pods=50_000, n_classes=250, catalog=None, seed=SEED, deployments=True) -> Problem:
    """50k heterogeneous pods × golden catalog × 3 AZ × {spot, on-demand} (BASELINE configs[1])."""
    rng = np.random.Generator(np.random.PCG64(seed + 2))
    catalog = catalog if catalog is not None else golden_catalog(seed=seed)
    taint_key = "example.com/dedicated"
    classes, creqs = _classes_config2(rng, n_classes, taint_key)
    # Deployments dominate: pods of a class are created together (contiguous timestamps)
    w = rng.dirichlet(np.ones(n_classes) * 0.8)
    counts = rng.multinomial(n_pods, w)
    specs = []
    order = rng.permutation(n_classes) if deployments else None
    if deployments:
        for c in order:
            specs += [(int(c), creqs[c])] * int(counts[c])
    else:
        ids = rng.choice(n_classes, size=n_pods, p=w)
        specs = [(int(c), creqs[c]) for c in ids]
    pods = _pods_from_milli(specs)
    nodepools = [
        default_nodepool("default", capacity_types=("spot", "on-demand"), weight=10),
        NodePool(name="dedicated", weight=50, requirements=[Requirement(CAPACITY_TYPE, "In", ["on-demand"])],
                 taints=[Taint(taint_key, "", "NoSchedule")]),
    ]
    return Problem(catalog, nodepools, classes, pods)


def config3_topology(rng, classes, zonal=0.40, hostname=0.20, anti=0.10):
    """Give every class a Deployment label (app=class-N) and draw its topology terms independently: zonal spread
    (maxSkew 1, DoNotSchedule), hostname spread (maxSkew 1) and required hostname anti-affinity, each selecting the
    class's own pods (the Deployment pattern the reference's scale suite uses, test/suites/scale/provisioning_test.go:91-101)."""
    for c, pc in enumerate(classes):
        app = "class-%d" % c
        pc.labels = {"app": app}
        sel = [Requirement("app", "In", [app])]
        if rng.random() < zonal:
            pc.topology.append(model.TopologyTerm("spread", ZONE, list(sel), max_skew=1))
        if rng.random() < hostname:
            pc.topology.append(model.TopologyTerm("spread", model.HOSTNAME, list(sel), max_skew=1))
        if rng.random() < anti:
            pc.topology.append(model.TopologyTerm("anti", model.HOSTNAME, list(sel)))
    return classes


def config3_nodepools(taint_key="example.com/dedicated"):
    """Five weighted NodePools (weights 100/80/50/20/0) with overlapping requirements and cpu limits
    500 / 2000 / 5000 cores / none / none."""
    AWS_ = AWS
    return [
        NodePool(name="np-100", weight=100, requirements=[Requirement(CAPACITY_TYPE, "In", ["on-demand"]),
                                                         Requirement(AWS_ + "instance-category", "In", ["c", "m"])],
                 limits_remaining={"cpu": 500 * 1000}),
        NodePool(name="np-80", weight=80, requirements=[Requirement(CAPACITY_TYPE, "In", ["spot"]),
                                                       Requirement(AWS_ + "instance-category", "In", ["m", "r"])],
                 limits_remaining={"cpu": 2000 * 1000}),
        NodePool(name="np-50", weight=50, requirements=[Requirement(CAPACITY_TYPE, "In", ["spot", "on-demand"]),
                                                       Requirement(AWS_ + "instance-generation", "Gt", ["5"])],
                 limits_remaining={"cpu": 5000 * 1000}),
        NodePool(name="np-20", weight=20, requirements=[Requirement(CAPACITY_TYPE, "In", ["on-demand"])],
                 taints=[Taint(taint_key, "", "NoSchedule")]),
        default_nodepool("np-0", capacity_types=("spot", "on-demand"), weight=0),
    ]


def config3(n_pods=50_000, n_classes=250, catalog=None, seed=SEED) -> Problem:
    """BASELINE configs[2]: config 2's pod mix with zonal + hostname topology spread and hostname anti-affinity
    (config3_topology) over five weighted NodePools with limits (config3_nodepools)."""
    rng = np.random.Generator(np.random.PCG64(seed + 3))
    catalog = catalog if catalog is not None else golden_catalog(seed=seed)
    taint_key = "example.com/dedicated"
    classes, creqs = _classes_config2(rng, n_classes, taint_key)
    config3_topology(rng, classes)
    w = rng.dirichlet(np.ones(n_classes) * 0.8)
    counts = rng.multinomial(n_pods, w)
    specs = []
    for c in rng.permutation(n_classes):
        specs += [(int(c), creqs[c])] * int(counts[c])
    return Problem(catalog, config3_nodepools(taint_key), classes, _pods_from_milli(specs))


def _pods_from_milli(specs, t0=1_700_000_000 * 10 ** 9):
    n = len(specs)
    cls = np.array([c for c, _ in specs], np.int32)
    req = np.zeros((n, R), np.int64)
    cache = {}
    for i, (c, r) in enumerate(specs):
        if c not in cache:
            v = np.zeros(R, np.int64)
            for k, q in r.items():
                v[RIDX[k]] = q
            v[RIDX["pods"]] += 1000
            cache[c] = v
        req[i] = cache[c]
    ts = t0 + np.arange(n, dtype=np.int64) * 10 ** 6
    uids = ["%08x-0000-4000-8000-%012x" % (i, i) for i in range(n)]
    return Pods(cls, req, ts, uids)


def subsample(prob: Problem, n_pods: int, seed=SEED) -> Problem:
    """A bounded sample of a problem's pods (same catalog/pools/classes), for oracle-sized runs."""
    p = prob.pods
    idx = np.sort(np.random.Generator(np.random.PCG64(seed)).choice(p.n, size=min(n_pods, p.n), replace=False))
    pods = Pods(p.class_id[idx].copy(), p.requests[idx].copy(), p.creation_ns[idx].copy(), [p.uids[i] for i in idx])
    return Problem(prob.catalog, prob.nodepools, prob.classes, pods, prob.existing, prob.max_instance_types,
                   prob.min_values_policy, list(prob.bound))


# ------------------------------------------------------------------------------------------------
# consolidation (BASELINE configs[3])
# ------------------------------------------------------------------------------------------------
def node_labels(it, zone, capacity_type, nodepool=None):
    """Labels of a launched node of type `it`: the type's single-valued labels plus zone / capacity-type."""
    labels = {}
    for k, v in it.labels.items():
        if isinstance(v, (list, tuple)):
            if len(v) == 1:
                labels[k] = str(v[0])
        elif v is not None:
            labels[k] = str(v)
    labels[ZONE] = zone
    labels[CAPACITY_TYPE] = capacity_type
    if nodepool:
        labels[NODEPOOL] = nodepool
    return labels


def candidate_price(it, labels):
    """getCandidatePrices term: Offerings.Compatible(NewLabelRequirements(node labels)).Cheapest().Price over ALL
    offerings of the node's type (an offering matches on capacity-type and zone; reservation keys are DoesNotExist on
    od/spot offerings, zone-id is well-known and undefined on the node).  None when nothing matches."""
    best = None
    for o in it.offerings:
        if o.capacity_type != labels.get(CAPACITY_TYPE) or o.zone != labels.get(ZONE):
            continue
        if o.reservation_id and labels.get(abi_RESERVATION_ID) != o.reservation_id:
            continue
        best = o.price if best is None or o.price < best else best
    return best


abi_RESERVATION_ID = "karpenter.k8s.aws/capacity-reservation-id"


def _selector_ok(req: Requirement, labels):
    v = labels.get(req.key)
    if req.op == "In":
        return v is not None and v in req.values
    if req.op == "NotIn":
        return v is None or v not in req.values
    if req.op == "Exists":
        return v is not None
    if req.op == "DoesNotExist":
        return v is None
    try:
        x = int(v)
    except (TypeError, ValueError):
        return False
    return x > int(req.values[0]) if req.op == "Gt" else x < int(req.values[0])


def config4(n_nodes=5000, pods_per_node=(10, 30), n_classes=250, catalog=None, seed=SEED, n_pending=0,
            util=(0.4, 0.6), headroom=None) -> ConsolidationProblem:
    """5k existing nodes with ~100k bound pods of config-2 classes at 40-60% utilisation (BASELINE configs[3]).

    Each node: a NodePool (80% default spot/on-demand, 20% the tainted on-demand pool), a zone, a capacity type, then
    the smallest catalog type (non-GPU, with an offering in that zone / capacity type) whose cpu and memory put the
    node's pods at the drawn utilisation; its pods are drawn from the classes the node satisfies (selectors,
    tolerations).  available = allocatable - bound pod requests.  Candidates = every node in disruption-cost order
    (fewer pods first, then name); multi-node consolidation takes the first 100.  All nodes initialized.

    headroom = f caps each node's available cpu and memory at f x allocatable (capacity held by pods that are not
    rescheduled, e.g. DaemonSets): with a small f the candidates' pods no longer fit the other nodes and the probes run
    NodeClaim.Add and the templates (REPLACE decisions; the "config4-replace" bench leg)."""
    rng = np.random.Generator(np.random.PCG64(seed + 4))
    catalog = catalog if catalog is not None else golden_catalog(seed=seed)
    taint_key = "example.com/dedicated"
    classes, creqs = _classes_config2(rng, n_classes, taint_key)
    nodepools = [
        default_nodepool("default", capacity_types=("spot", "on-demand"), weight=10),
        NodePool(name="dedicated", weight=50, requirements=[Requirement(CAPACITY_TYPE, "In", ["on-demand"])],
                 taints=[Taint(taint_key, "", "NoSchedule")]),
    ]
    creq_vec = np.zeros((n_classes, R), np.int64)
    for c, r in enumerate(creqs):
        for k, q in r.items():
            creq_vec[c, RIDX[k]] = q
        creq_vec[c, RIDX["pods"]] += 1000
    gpu_free = [c for c in range(n_classes) if creq_vec[c, RIDX["nvidia.com/gpu"]] == 0]
    w = rng.dirichlet(np.ones(n_classes) * 0.8)
    types = [t for t, it in enumerate(catalog)
             if it.allocatable[RIDX["nvidia.com/gpu"]] == 0 and it.allocatable[RIDX["cpu"]] >= 2000]
    cpu_alloc = np.array([catalog[t].allocatable[RIDX["cpu"]] for t in types], np.int64)
    mem_alloc = np.array([catalog[t].allocatable[RIDX["memory"]] for t in types], np.int64)
    pods_alloc = np.array([catalog[t].allocatable[RIDX["pods"]] for t in types], np.int64)
    by_cpu = np.lexsort((mem_alloc, cpu_alloc))
    zones = ["test-zone-1a", "test-zone-1b", "test-zone-1c"]
    nodes, specs, owner, cand_meta = [], [], [], []
    for j in range(n_nodes):
        dedicated = rng.random() < 0.2
        pool = nodepools[1] if dedicated else nodepools[0]
        ct = "on-demand" if dedicated or rng.random() < 0.5 else "spot"
        zone = str(rng.choice(zones))
        n = int(rng.integers(pods_per_node[0], pods_per_node[1] + 1))
        u = float(rng.uniform(*util))
        # draw classes tolerating the pool; selectors are checked once the type is known
        pw = w[gpu_free] / w[gpu_free].sum()
        cls = list(rng.choice(gpu_free, size=n, p=pw))
        need_cpu = int(creq_vec[cls, RIDX["cpu"]].sum() / u)
        need_mem = int(creq_vec[cls, RIDX["memory"]].sum() / u)
        pick = None
        for i in by_cpu:
            if cpu_alloc[i] >= need_cpu and mem_alloc[i] >= need_mem and pods_alloc[i] >= n * 1000:
                it = catalog[types[i]]
                if any(o.zone == zone and o.capacity_type == ct and not o.reservation_id for o in it.offerings):
                    pick = types[i]
                    break
        if pick is None:
            pick = types[int(by_cpu[-1])]
        it = catalog[pick]
        labels = node_labels(it, zone, ct, pool.name)
        ok = [c for c in gpu_free if all(_selector_ok(r, labels) for r in classes[c].requirements) and
              (not dedicated or any(t.key == taint_key for t in classes[c].tolerations))]
        okw = w[ok] / w[ok].sum()
        for q in range(n):
            c = cls[q]
            if c not in ok:
                cls[q] = int(rng.choice(ok, p=okw))
        used = creq_vec[cls].sum(axis=0)
        avail = np.array(it.allocatable, np.int64) - used
        if headroom is not None:
            for r in (RIDX["cpu"], RIDX["memory"]):
                avail[r] = min(avail[r], int(it.allocatable[r] * headroom))
        name = "node-%05d" % j
        nodes.append(ExistingNode(name=name, labels=labels, available=avail, requests=np.zeros(R, np.int64),
                                  taints=list(pool.taints)))
        for c in cls:
            specs.append((int(c), creqs[c]))
            owner.append(j)
        price = candidate_price(it, labels)
        cand_meta.append((n, name, j, price, ct, pick, 1 if dedicated else 0, np.array(it.capacity, np.int64)))
    # pending pods (unbound), created after the bound ones
    for _ in range(n_pending):
        c = int(rng.choice(gpu_free))
        specs.append((c, creqs[c]))
        owner.append(-1)
    pods = _pods_from_milli(specs)
    owner = np.array(owner, np.int64)
    prob = Problem(catalog, nodepools, classes, pods, nodes)
    order = np.argsort(owner[owner >= 0], kind="stable")
    pods_of = np.split(np.nonzero(owner >= 0)[0][order], np.cumsum(np.bincount(owner[owner >= 0], minlength=n_nodes))[:-1])
    cand_meta.sort(key=lambda m: (m[0], m[1]))
    cands = [Candidate(node=m[2], pods=pods_of[m[2]].astype(np.int32), price=m[3],
                       capacity_type=abi.KP_CT_SPOT if m[4] == "spot" else abi.KP_CT_ON_DEMAND, instance_type=m[5],
                       nodepool=m[6], capacity=m[7]) for m in cand_meta]
    return ConsolidationProblem(prob, cands, np.nonzero(owner < 0)[0].astype(np.int32), np.ones(n_nodes, np.uint8))


def config5_catalog(catalog, n_default=40, n_block=20, seed=SEED, expiring_frac=0.10):
    """BASELINE configs[4]'s catalog: the golden catalog plus reserved offerings (offering.go:164-194) for 60 types —
    40 ODCR-default and 20 capacity-block, ReservationCapacity in [1, 20], price = odPrice / 1e7 (offering.go:176),
    10% of reservations expiring (Available = false, offering.go:187).  Returns a new catalog list (types copied)."""
    import copy
    rng = np.random.Generator(np.random.PCG64(seed + 5))
    cat = copy.deepcopy(catalog)
    idx = rng.choice(len(cat), size=n_default + n_block, replace=False)
    for j, t in enumerate(idx):
        it = cat[int(t)]
        od = [o for o in it.offerings if o.capacity_type == "on-demand"]
        if not od:
            continue
        z = od[int(rng.integers(len(od)))]
        rcap = int(rng.integers(1, 21))
        expiring = rng.random() < expiring_frac
        it.offerings.append(model.Offering(
            capacity_type="reserved", zone=z.zone, price=z.price / 10_000_000.0, available=not expiring,
            zone_id=z.zone_id, reservation_id="cr-%05d" % j,
            reservation_type="default" if j < n_default else "capacity-block", reservation_capacity=rcap))
        # computeRequirements for a type with capacity reservations (types.go:181-234): capacity-type gains
        # "reserved", and the reservation ID / type labels list the type's reservations
        res = [o for o in it.offerings if o.capacity_type == "reserved"]
        cts = list(it.labels.get(CAPACITY_TYPE) or [])
        if "reserved" not in cts:
            it.labels[CAPACITY_TYPE] = cts + ["reserved"]
        it.labels[model.RESERVATION_ID] = sorted({o.reservation_id for o in res})
        it.labels[model.RESERVATION_TYPE] = sorted({o.reservation_type for o in res})
    return cat


def wide_reservation_catalog(catalog, n_reservations=200, max_per_type=4, seed=SEED, expiring_frac=0.10,
                             rcap=(1, 21)):
    """A catalog with more capacity reservations than one 64-bit word holds (offering.go:164-194 makes one reserved
    offering per reservation, without bound): n_reservations ODCR-default / capacity-block reservations over types
    drawn from the catalog, 1 to max_per_type reservations per type (in its on-demand zones), ReservationCapacity drawn
    from rcap, price = odPrice / 1e7, some expiring.  Returns a new catalog list (types copied)."""
    import copy
    rng = np.random.Generator(np.random.PCG64(seed + 55))
    cat = copy.deepcopy(catalog)
    cands = [t for t, it in enumerate(cat) if any(o.capacity_type == "on-demand" for o in it.offerings)]
    assert len(cands) * max_per_type >= n_reservations, "catalog too small for %d reservations" % n_reservations
    made = 0
    while made < n_reservations:
        t = int(rng.choice(cands))
        it = cat[t]
        od = [o for o in it.offerings if o.capacity_type == "on-demand"]
        for _ in range(int(rng.integers(1, max_per_type + 1))):
            if made >= n_reservations or sum(o.capacity_type == "reserved" for o in it.offerings) >= max_per_type:
                break
            z = od[int(rng.integers(len(od)))]
            expiring = rng.random() < expiring_frac
            it.offerings.append(model.Offering(
                capacity_type="reserved", zone=z.zone, price=z.price / 10_000_000.0, available=not expiring,
                zone_id=z.zone_id, reservation_id="cr-w%05d" % made,
                reservation_type="default" if rng.random() < 0.7 else "capacity-block",
                reservation_capacity=int(rng.integers(*rcap))))
            made += 1
        res = [o for o in it.offerings if o.capacity_type == "reserved"]
        if res:
            cts = list(it.labels.get(CAPACITY_TYPE) or [])
            if "reserved" not in cts:
                it.labels[CAPACITY_TYPE] = cts + ["reserved"]
            it.labels[model.RESERVATION_ID] = sorted({o.reservation_id for o in res})
            it.labels[model.RESERVATION_TYPE] = sorted({o.reservation_type for o in res})
    return cat


def config5(n_pods=200_000, n_classes=250, catalog=None, golden=None, seed=SEED) -> Problem:
    """BASELINE configs[4] as a Solve: config-2 pods over the reserved-offering catalog (config5_catalog), with the
    ODCR NodePool patterns of designs/odcr.md:140-180 — an ODCR-only NodePool first (capacity-type In [reserved],
    weight 100), a tainted NodePool with on-demand fallback (In [on-demand, reserved]) and the spot/on-demand
    default.  Provisioning runs the ReservationManager in strict mode."""
    if catalog is None:
        catalog = config5_catalog(golden if golden is not None else golden_catalog(seed=seed), seed=seed)
    prob = config2(n_pods=n_pods, n_classes=n_classes, catalog=catalog, seed=seed)
    taint_key = "example.com/dedicated"
    prob.nodepools = [
        NodePool(name="odcr", weight=100, requirements=[Requirement(CAPACITY_TYPE, "In", ["reserved"])]),
        NodePool(name="dedicated", weight=50, requirements=[Requirement(CAPACITY_TYPE, "In", ["on-demand", "reserved"])],
                 taints=[Taint(taint_key, "", "NoSchedule")]),
        default_nodepool("default", capacity_types=("spot", "on-demand"), weight=10),
    ]
    return prob


def launch_requests(catalog, n=1000, seed=SEED, with_min_values=True):
    """Seeded NodeClaims for kp_launch_select: requirement mixes a Solve produces (NodePool capacity types, zones,
    arch, categories, instance-type In [≤ 60 names], occasional minValues) and request totals."""
    rng = np.random.Generator(np.random.PCG64(seed + 6))
    names = [it.name for it in catalog]
    fams = sorted({it.labels.get("karpenter.k8s.aws/instance-family", [None])[0] or "" for it in catalog} - {""})
    ct_sets = [["on-demand"], ["spot"], ["spot", "on-demand"], ["reserved"], ["reserved", "on-demand"],
               ["reserved", "spot", "on-demand"], None]
    out = []
    R = len(model.RESOURCES)
    for i in range(n):
        reqs = []
        cts = ct_sets[int(rng.integers(len(ct_sets)))]
        if cts is not None:
            reqs.append(model.Requirement(model.CAPACITY_TYPE, "In", list(cts)))
        u = rng.random()
        if u < 0.6:
            k = int(rng.integers(5, 120))
            reqs.append(model.Requirement(model.INSTANCE_TYPE, "In",
                                          [names[int(x)] for x in rng.choice(len(names), size=k, replace=False)]))
        elif u < 0.8:
            reqs.append(model.Requirement("karpenter.k8s.aws/instance-family", "In",
                                          [fams[int(x)] for x in rng.choice(len(fams), size=int(rng.integers(1, 12)),
                                                                            replace=False)]))
        if rng.random() < 0.3:
            reqs.append(model.Requirement(model.ZONE, "In", ["test-zone-1%s" % c for c in
                                                             rng.choice(list("abc"), size=int(rng.integers(1, 3)),
                                                                        replace=False)]))
        if rng.random() < 0.3:
            reqs.append(model.Requirement(model.ARCH, "In", [["amd64", "arm64"][int(rng.integers(2))]]))
        if rng.random() < 0.2:
            reqs.append(model.Requirement("karpenter.k8s.aws/instance-category", "NotIn", ["g", "p", "inf", "trn"]))
        if rng.random() < 0.15:
            reqs.append(model.Requirement("karpenter.k8s.aws/instance-generation", "Gt", [str(int(rng.integers(2, 7)))]))
        if with_min_values and rng.random() < 0.1:
            reqs.append(model.Requirement("karpenter.k8s.aws/instance-family", "Exists", [],
                                          min_values=int(rng.integers(1, 40))))
        rq = np.zeros(R, np.int64)
        cpu = int(rng.choice([250, 500, 1000, 2000, 4000, 8000, 16000, 64000]))
        rq[0] = cpu
        rq[1] = cpu * int(rng.choice([1, 2, 4, 8])) * (1 << 30)  # cpu cores x GiB/core, milli-bytes
        rq[3] = int(rng.integers(1, 40)) * 1000
        if rng.random() < 0.03:
            rq[5] = int(rng.choice([1, 2, 4, 8])) * 1000
        out.append(model.LaunchRequest(reqs, rq))
    return out


def widen_catalog(catalog, n_types, seed=SEED):
    """A catalog of n_types rows: the given one plus renamed copies of its types ("<family>w<k>.<size>", the family
    label renamed alike, prices scaled by a seeded factor), standing in for a region whose price table lists more types
    than the golden catalog (the library's limit is KP_MAX_TYPES = 2048)."""
    import copy
    rng = np.random.Generator(np.random.PCG64(seed))
    out = list(catalog)
    fam_key = "karpenter.k8s.aws/instance-family"
    k = 0
    while len(out) < n_types:
        base = catalog[len(out) % len(catalog)]
        k += 1 if len(out) % len(catalog) == 0 else 0
        it = copy.deepcopy(base)
        fam, _, size = base.name.partition(".")
        it.name = "%sw%d.%s" % (fam, k, size)
        labels = dict(it.labels)
        labels["node.kubernetes.io/instance-type"] = [it.name]
        if labels.get(fam_key):
            labels[fam_key] = ["%sw%d" % (labels[fam_key][0], k)]
        it.labels = labels
        f = float(rng.uniform(0.8, 1.25))
        for o in it.offerings:
            o.price = round(o.price * f, 6)
        out.append(it)
    return out
