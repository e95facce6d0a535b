"""Seeded synthetic workloads for BASELINE.json configs and small KAT problems.

Every generator is deterministic in its seed (PCG64, default 20250912).  Pods carry requests as
resources.RequestsForPods would produce them ([core] pkg/utils/resources: Ceiling(pod).Requests merged,
plus `pods: 1`), creation timestamps and UIDs that make the queue order total.
"""
from typing import Dict, List, Optional

import numpy as np

from .catalog import golden_catalog, parse_quantity_milli
from .model import (ARCH, CAPACITY_TYPE, R, RIDX, ZONE, NodePool, PodClass, Pods, Problem, Requirement, Taint,
                    Toleration)

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
                   prob.min_values_policy)
