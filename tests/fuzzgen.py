"""Seeded random scheduling problems that exercise the requirement algebra end to end.

Operators In / NotIn / Exists / DoesNotExist / Gt / Lt over catalog labels (single- and multi-valued), values
absent from the catalog, non-well-known custom keys, taints/tolerations, NodePool weights, limits, daemon
overhead and minValues.  Used by the GPU parity tests (device vs. CPU oracle on identical inputs).
"""
import numpy as np

from kpsim import model
from kpsim.model import (ARCH, CAPACITY_TYPE, INSTANCE_TYPE, NodePool, PodClass, Problem, Requirement, Taint,
                         Toleration, ZONE)

HOSTNAME = "kubernetes.io/hostname"
from kpsim.synth import _pods_from_milli

AWS = "karpenter.k8s.aws/"
ZONES = ["test-zone-1a", "test-zone-1b", "test-zone-1c"]


def _rand_req(rng, catalog):
    it = catalog[int(rng.integers(0, len(catalog)))]
    kind = int(rng.integers(0, 14))
    if kind == 0:
        return Requirement(ARCH, str(rng.choice(["In", "NotIn"])), [str(rng.choice(["amd64", "arm64"]))])
    if kind == 1:
        return Requirement(ZONE, str(rng.choice(["In", "NotIn"])),
                           sorted(set(rng.choice(ZONES + ["us-west-2z"], size=int(rng.integers(1, 3))).tolist())))
    if kind == 2:
        return Requirement(CAPACITY_TYPE, "In", [str(rng.choice(["spot", "on-demand"]))])
    if kind == 3:
        return Requirement(AWS + "instance-category", str(rng.choice(["In", "NotIn"])),
                           sorted(set(rng.choice(["c", "m", "r", "t", "g", "x"], size=int(rng.integers(1, 4))).tolist())))
    if kind == 4:
        return Requirement(AWS + "instance-generation", str(rng.choice(["Gt", "Lt"])), [str(int(rng.integers(2, 8)))])
    if kind == 5:
        return Requirement(AWS + "instance-cpu", str(rng.choice(["Gt", "Lt"])), [str(int(rng.choice([2, 4, 8, 16, 48])))])
    if kind == 6:
        return Requirement(AWS + "instance-gpu-name", str(rng.choice(["Exists", "DoesNotExist"])))
    if kind == 7:
        return Requirement(AWS + "instance-local-nvme", str(rng.choice(["Exists", "DoesNotExist", "NotIn"])),
                           ["1900"] if rng.random() < 0.5 else [])
    if kind == 8:
        return Requirement(INSTANCE_TYPE, "In", sorted(set([it.name] + [catalog[int(i)].name for i in
                                                                         rng.integers(0, len(catalog), size=20)])))
    if kind == 9:
        return Requirement("example.com/team", str(rng.choice(["In", "NotIn", "Exists", "DoesNotExist"])), ["a"])
    if kind == 10:
        return Requirement(AWS + "instance-family", "NotIn", [str(v) for v in (it.labels.get(AWS + "instance-family") or ["m5"])])
    if kind == 11:
        return Requirement(AWS + "instance-memory", str(rng.choice(["Gt", "Lt"])), [str(int(rng.choice([4096, 16384, 65536])))])
    if kind == 12:
        return Requirement(AWS + "instance-hypervisor", "In", [str(rng.choice(["nitro", "xen", ""]))])
    return Requirement(AWS + "instance-size", str(rng.choice(["In", "NotIn"])),
                       sorted(set(rng.choice(["large", "xlarge", "2xlarge", "metal", "medium"], size=2).tolist())))


def existing_nodes(rng, catalog, n_nodes):
    """Existing (in-flight / running) nodes: labels of a catalog type (+ zone, capacity-type, a custom team label),
    available = a fraction of the type's allocatable, daemonset requests, sometimes a taint."""
    nodes = []
    for j in range(n_nodes):
        it = catalog[int(rng.integers(0, len(catalog)))]
        labels = {}
        for k, v in it.labels.items():
            if isinstance(v, (list, tuple)):
                if v:
                    labels[k] = str(v[int(rng.integers(0, len(v)))])
            elif v is not None:
                labels[k] = str(v)
        labels[ZONE] = str(rng.choice(ZONES))
        labels[CAPACITY_TYPE] = str(rng.choice(["spot", "on-demand"]))
        if rng.random() < 0.5:
            labels["example.com/team"] = str(rng.choice(["a", "b"]))
        avail = np.array(it.allocatable, np.int64).copy()
        frac = float(rng.choice([0.0, 0.3, 0.6, 0.9, 1.0]))
        for ax in ("cpu", "memory", "pods"):
            avail[model.RIDX[ax]] = int(avail[model.RIDX[ax]] * (1.0 - frac))
        req = np.zeros(model.R, np.int64)
        if rng.random() < 0.5:
            req[model.RIDX["cpu"]] = 100
            req[model.RIDX["pods"]] = 1000
        taints = [Taint("example.com/gpu", "true", "NoSchedule")] if rng.random() < 0.2 else []
        nodes.append(model.ExistingNode(name="node-%d" % j, labels=labels, available=avail, requests=req, taints=taints))
    return nodes


def _existing_req(rng, n_nodes):
    kind = int(rng.integers(0, 5))
    if kind == 0:
        return Requirement(HOSTNAME, "In", ["node-%d" % int(rng.integers(0, n_nodes))])
    if kind == 1:
        return Requirement(HOSTNAME, "NotIn", ["node-%d" % int(rng.integers(0, n_nodes))])
    if kind == 2:
        return Requirement("example.com/team", str(rng.choice(["NotIn", "DoesNotExist"])), ["a"])
    if kind == 3:
        return Requirement("example.com/team", "In", [str(rng.choice(["a", "b"]))])
    return Requirement(HOSTNAME, "Exists")


def fuzz_problem(catalog, seed, n_pods=300, n_classes=12, n_pools=3, with_min=True, with_limits=True, n_existing=0):
    rng = np.random.Generator(np.random.PCG64(seed))
    T = len(catalog)
    pools = []
    for j in range(n_pools):
        reqs = [Requirement(CAPACITY_TYPE, "In", sorted(set(rng.choice(["spot", "on-demand"], size=2).tolist())))]
        for _ in range(int(rng.integers(0, 3))):
            reqs.append(_rand_req(rng, catalog))
        if with_min and rng.random() < 0.3:
            reqs.append(Requirement(AWS + "instance-family", "Exists", [], int(rng.integers(2, 6))))
        labels = {"example.com/team": "a"} if rng.random() < 0.4 else {}
        taints = [Taint("example.com/gpu", "true", "NoSchedule")] if rng.random() < 0.3 else []
        daemon = np.zeros(model.R, np.int64)
        if rng.random() < 0.5:
            daemon[model.RIDX["cpu"]] = int(rng.choice([100, 250]))
            daemon[model.RIDX["memory"]] = int(rng.choice([128, 512])) * 2 ** 20 * 1000
            daemon[model.RIDX["pods"]] = 2000
        limits = None
        if with_limits and rng.random() < 0.4:
            limits = {"cpu": int(rng.choice([16, 64, 256])) * 1000}
        rows = None
        if rng.random() < 0.3:
            rows = sorted(rng.choice(T, size=max(1, T // 2), replace=False).tolist())
        pools.append(NodePool(name="pool-%d" % j, weight=int(rng.choice([0, 10, 10, 50])), requirements=reqs,
                              labels=labels, taints=taints, daemon_overhead=daemon, limits_remaining=limits,
                              instance_types=rows))
    classes, creqs = [], []
    for c in range(n_classes):
        reqs = [_rand_req(rng, catalog) for _ in range(int(rng.integers(0, 3)))]
        if n_existing and rng.random() < 0.4:
            reqs.append(_existing_req(rng, n_existing))
        tols = [Toleration("example.com/gpu", "Exists", "", "NoSchedule")] if rng.random() < 0.3 else []
        classes.append(PodClass(reqs, tols))
        cpu = int(rng.choice([100, 500, 1000, 2000, 4000]))
        r = {"cpu": cpu, "memory": cpu * int(rng.choice([1, 2, 4])) * (2 ** 30) // 1000 * 1000}
        if rng.random() < 0.1:
            r["nvidia.com/gpu"] = 1000
        creqs.append(r)
    specs = []
    for _ in range(n_pods):
        c = int(rng.integers(0, n_classes))
        specs.append((c, creqs[c]))
    # runs of identical pods (deployments) and some shuffling
    if rng.random() < 0.5:
        specs.sort(key=lambda s: s[0])
    pods = _pods_from_milli(specs)
    if rng.random() < 0.5:  # equal creation times: UID order decides ties
        pods.creation_ns[:] = pods.creation_ns[0]
    existing = existing_nodes(rng, catalog, n_existing) if n_existing else []
    return Problem(catalog, pools, classes, pods, existing)


TOPO_KEYS = [ZONE, HOSTNAME, CAPACITY_TYPE]


def _rand_selector(rng, apps):
    kind = int(rng.integers(0, 6))
    if kind == 0:
        return None  # nil selector: selects nothing
    if kind == 1:
        return []    # empty selector: selects every pod of the namespace(s)
    if kind == 2:
        return [Requirement("app", "NotIn", [str(rng.choice(apps))])]
    if kind == 3:
        return [Requirement("tier", str(rng.choice(["Exists", "DoesNotExist"])))]
    return [Requirement("app", "In", sorted(set(rng.choice(apps, size=int(rng.integers(1, 3))).tolist())))]


def add_topology(rng, prob, p_term=0.6, namespaces=("default", "team-b")):
    """Labels, namespaces and random topology terms on a problem's classes: zonal / hostname / capacity-type spread
    (maxSkew 1-3, minDomains, node-affinity / taint policies), required pod affinity and anti-affinity, selectors that
    match the class itself, other classes, everything or nothing."""
    apps = ["a%d" % i for i in range(max(2, len(prob.classes) // 2))]
    for pc in prob.classes:
        pc.labels = {"app": str(rng.choice(apps))}
        if rng.random() < 0.5:
            pc.labels["tier"] = str(rng.choice(["web", "db"]))
        pc.namespace = str(rng.choice(namespaces)) if rng.random() < 0.25 else "default"
    for pc in prob.classes:
        while rng.random() < p_term and len(pc.topology) < 3:
            key = str(rng.choice(TOPO_KEYS, p=[0.5, 0.35, 0.15]))
            sel = [Requirement("app", "In", [pc.labels["app"]])] if rng.random() < 0.6 else _rand_selector(rng, apps)
            kind = str(rng.choice(["spread", "spread", "anti", "affinity"]))
            if kind == "spread":
                pc.topology.append(model.TopologyTerm(
                    "spread", key, sel, max_skew=int(rng.integers(1, 4)),
                    min_domains=int(rng.integers(1, 5)) if rng.random() < 0.2 else None,
                    node_affinity_policy=str(rng.choice(["Honor", "Honor", "Ignore"])),
                    node_taints_policy=str(rng.choice(["Ignore", "Ignore", "Honor"]))))
            else:
                ns = [str(x) for x in rng.choice(namespaces, size=2, replace=False)] if rng.random() < 0.2 else []
                pc.topology.append(model.TopologyTerm(kind, key, sel, namespaces=ns))
    return prob


def fuzz_topology_problem(catalog, seed, n_pods=200, n_classes=10):
    """fuzz_problem (requirements, taints, pools, limits, minValues) plus topology terms on its classes."""
    prob = fuzz_problem(catalog, seed, n_pods=n_pods, n_classes=n_classes)
    return add_topology(np.random.Generator(np.random.PCG64(seed + 99)), prob)


GPU_COUNT = AWS + "instance-gpu-count"
NODEPOOL = "karpenter.sh/nodepool"


def add_mutators(rng, cp, gpu_catalog=None):
    """The reference's shapes whose ExistingNode.Add merges change a node's requirements (a NotIn / DoesNotExist pod
    requirement on a label the node lacks) in a way later pods see:
      * GPU avoidance: non-GPU instance types carry instance-gpu-count / -name as DoesNotExist
        (pkg/providers/instancetype/types.go:204-210) and only single-valued requirements become node labels
        (pkg/cloudprovider/cloudprovider.go:387-398), so non-GPU nodes lack the labels; "keep off GPU nodes" pods say
        instance-gpu-count DoesNotExist (or NotIn [..]) next to GPU pods selecting instance-gpu-count Gt 0;
      * mixed node groups: pods with karpenter.sh/nodepool DoesNotExist in a cluster whose managed-node-group nodes lack
        the label (website/content/en/preview/getting-started/migrating-from-cas/_index.md:117-123), next to pods
        selecting a NodePool positively.
    Some nodes become GPU nodes (labels of a GPU type from gpu_catalog), some Karpenter nodes (karpenter.sh/nodepool);
    some classes get the negative and some the positive requirements."""
    prob = cp.cluster
    gpus = [it for it in (gpu_catalog or prob.catalog) if it.labels.get(GPU_COUNT) not in (None, [], "")]
    for n in prob.existing:
        if gpus and rng.random() < 0.25:
            it = gpus[int(rng.integers(0, len(gpus)))]
            for k in (GPU_COUNT, AWS + "instance-gpu-name", AWS + "instance-gpu-manufacturer"):
                v = it.labels.get(k)
                if isinstance(v, (list, tuple)):
                    v = v[0] if v else None
                if v is not None:
                    n.labels[k] = str(v)
        if rng.random() < 0.6:
            n.labels[NODEPOOL] = prob.nodepools[int(rng.integers(0, len(prob.nodepools)))].name
    pools = [np_.name for np_ in prob.nodepools]
    for pc in prob.classes:
        u = rng.random()
        reqs = list(pc.requirements)
        if u < 0.25:
            reqs.append(Requirement(GPU_COUNT, "DoesNotExist"))
        elif u < 0.35:
            reqs.append(Requirement(GPU_COUNT, "NotIn", [str(rng.choice(["1", "4", "8"]))]))
        elif u < 0.5:
            reqs.append(Requirement(GPU_COUNT, "Gt", ["0"]))
        elif u < 0.55:
            reqs.append(Requirement(GPU_COUNT, "Exists"))
        v = rng.random()
        if v < 0.3:
            reqs.append(Requirement(NODEPOOL, "DoesNotExist"))
        elif v < 0.4:
            reqs.append(Requirement(NODEPOOL, "NotIn", [str(rng.choice(pools))]))
        elif v < 0.55:
            reqs.append(Requirement(NODEPOOL, "In", sorted(set(rng.choice(pools, size=2).tolist()))))
        elif v < 0.6:
            reqs.append(Requirement(NODEPOOL, "Exists"))
        pc.requirements = reqs
    return cp


def fuzz_consolidation(catalog, seed, n_nodes=40, n_pods=200, n_candidates=None, with_min=False, pending_frac=0.15,
                       all_spot=False, n_pools=3):
    """A consolidation pass over random state: fuzz_problem's classes / pools / existing nodes, NewScheduler node order
    (initialized first, then name), candidates with their bound pods, pending pods, candidate prices around their
    offering price (so REPLACE, price-filtered NONE and DELETE all occur)."""
    from kpsim import abi, synth
    prob = fuzz_problem(catalog, seed, n_pods=n_pods, n_classes=12, with_min=with_min, n_existing=n_nodes, n_pools=n_pools)
    rng = np.random.Generator(np.random.PCG64(seed + 7))
    E = len(prob.existing)
    init = (rng.random(E) < 0.9).astype(np.uint8)
    order = sorted(range(E), key=lambda j: (0 if init[j] else 1, prob.existing[j].name))
    prob.existing = [prob.existing[j] for j in order]
    init = init[order]
    by_name = {it.name: t for t, it in enumerate(catalog)}
    nc = int(n_candidates or rng.integers(2, max(3, min(E, 30))))
    cand_nodes = rng.choice(E, size=min(nc, E), replace=False)
    P = prob.pods.n
    owner = rng.integers(0, len(cand_nodes), size=P)
    owner[rng.random(P) < pending_frac] = -1
    cands = []
    for i, j in enumerate(cand_nodes):
        node = prob.existing[int(j)]
        if all_spot:
            node.labels[CAPACITY_TYPE] = "spot"
        t = by_name.get(node.labels.get(INSTANCE_TYPE), -1)
        price = synth.candidate_price(catalog[t], node.labels) if t >= 0 else None
        if price is None:
            price = float(rng.uniform(0.01, 3.0))
        price *= float(rng.choice([0.3, 1.0, 1.0, 3.0, 20.0]))
        ct = abi.KP_CT_SPOT if node.labels.get(CAPACITY_TYPE) == "spot" else abi.KP_CT_ON_DEMAND
        npool = int(rng.integers(-1, len(prob.nodepools)))
        cap = np.array(catalog[t].capacity, np.int64) if t >= 0 else None
        cands.append(model.Candidate(node=int(j), pods=np.nonzero(owner == i)[0].astype(np.int32), price=price,
                                     capacity_type=ct, instance_type=t, nodepool=npool, capacity=cap))
    return model.ConsolidationProblem(prob, cands, np.nonzero(owner < 0)[0].astype(np.int32), init)


def fuzz_topology_existing_problem(catalog, seed, n_pods=200, n_classes=10, n_existing=24, n_bound=40):
    """fuzz_topology_problem over a cluster: existing nodes (labels with zone / capacity-type / team, partial
    headroom, taints) and pods of the classes already bound to them, whose topology terms count (countDomains) and
    whose required anti-affinity blocks their nodes' domains (updateInverseAffinities)."""
    prob = fuzz_problem(catalog, seed, n_pods=n_pods, n_classes=n_classes, n_existing=n_existing)
    rng = np.random.Generator(np.random.PCG64(seed + 7))
    prob = add_topology(rng, prob)
    prob.bound = [(int(rng.integers(0, n_existing)), int(rng.integers(0, n_classes))) for _ in range(n_bound)]
    return prob


def fuzz_topology_consolidation(catalog, seed, n_nodes=30, n_pods=160, n_bound=40, all_spot=False, host_affinity=False):
    """fuzz_consolidation over pods with topology terms (add_topology: zonal / hostname / capacity-type spread,
    anti-affinity, zonal affinity; hostname pod affinity turned into anti-affinity unless host_affinity) plus
    non-reschedulable pods bound to random nodes (cluster.bound)."""
    cp = fuzz_consolidation(catalog, seed, n_nodes=n_nodes, n_pods=n_pods, all_spot=all_spot)
    rng = np.random.Generator(np.random.PCG64(seed + 123))
    prob = add_topology(rng, cp.cluster, p_term=0.4)
    for pc in prob.classes:
        for t in pc.topology:
            if t.kind == "affinity" and t.key == HOSTNAME and not host_affinity:
                t.kind = "anti"
    E = len(prob.existing)
    prob.bound = [(int(rng.integers(0, E)), int(rng.integers(0, len(prob.classes)))) for _ in range(n_bound)]
    return cp


def add_preferences(rng, prob, p_node=0.45, p_topo=0.6):
    """Preferences on a problem's classes, as the Solve's preference suites draw them: preferred node-affinity terms
    (weights 1-100) and ORed required node-affinity terms over instance-category / arch, ScheduleAnyway spreads (zonal or
    hostname), preferred pod anti-affinity (hostname) and preferred pod affinity (zonal or hostname); a handful of
    classes per selector."""
    cats = ["c", "m", "r", "t", "g", "i"]
    for ci, pc in enumerate(prob.classes):
        app = "p%d" % (ci % 5)
        pc.labels = dict(pc.labels)
        pc.labels["app"] = app
        sel = [Requirement("app", "In", [app])]
        u = rng.random()
        if u < p_node * 0.65:
            pc.preferred_terms = [(int(rng.integers(1, 100)),
                                   [Requirement(AWS + "instance-category", "In",
                                                [str(x) for x in rng.choice(cats, size=int(rng.integers(1, 3)), replace=False)])])
                                  for _ in range(int(rng.integers(1, 4)))]
        elif u < p_node:
            pc.required_terms = [[Requirement(AWS + "instance-category", "In", [str(rng.choice(cats))])],
                                 [Requirement(ARCH, "In", [str(rng.choice(["amd64", "arm64"]))])]]
        v = rng.random()
        if v < p_topo * 0.4:
            pc.topology = [model.TopologyTerm("spread", HOSTNAME if rng.random() < 0.5 else ZONE, selector=sel,
                                              max_skew=int(rng.integers(1, 3)), when_unsatisfiable="ScheduleAnyway",
                                              node_affinity_policy="Ignore")]
        elif v < p_topo * 0.75:
            pc.topology = [model.TopologyTerm("anti", HOSTNAME, selector=sel, weight=int(rng.integers(1, 100)))]
        elif v < p_topo:
            pc.topology = [model.TopologyTerm("affinity", ZONE if rng.random() < 0.6 else HOSTNAME, selector=sel,
                                              weight=int(rng.integers(1, 100)))]
    return prob


def add_topology_preferences(rng, prob, p_pref=0.5):
    """Preferred node-affinity terms next to topology terms (after add_topology): terms on the topology keys themselves
    (zone, capacity-type: the NodeClaim takes the preference, podDomains the strict requirements) and on
    instance-category / arch (outside a nodeAffinityPolicy Honor spread's node filter), weights 1-100."""
    zones = sorted({o.zone for it in prob.catalog for o in it.offerings})
    cats = ["c", "m", "r", "t", "g", "i"]
    for pc in prob.classes:
        if rng.random() >= p_pref:
            continue
        terms = []
        for _ in range(int(rng.integers(1, 4))):
            u = rng.random()
            if u < 0.4:
                r = Requirement(ZONE, "In", sorted(set(rng.choice(zones, size=int(rng.integers(1, 3))).tolist())))
            elif u < 0.55:
                r = Requirement(CAPACITY_TYPE, "In", [str(rng.choice(["spot", "on-demand"]))])
            elif u < 0.85:
                r = Requirement(AWS + "instance-category", "In",
                                sorted(set(rng.choice(cats, size=int(rng.integers(1, 3))).tolist())))
            else:
                r = Requirement(ARCH, "In", [str(rng.choice(["amd64", "arm64"]))])
            terms.append((int(rng.integers(1, 100)), [r]))
        pc.preferred_terms = terms
    return prob


def add_relaxing_topology(rng, prob, p_req=0.5):
    """Pods whose relaxation changes their spread groups' TopologyGroup.Hash() (topology.go Update creates the new
    spec's groups then): ORed required node-affinity terms (instance-category / arch / zone, 2-3 terms, the first often
    unsatisfiable for the pod's spread) next to zonal / hostname spreads under both nodeAffinityPolicies, and sometimes
    a PreferNoSchedule taint on a NodePool (the added toleration is part of the node filter's hash)."""
    zones = sorted({o.zone for it in prob.catalog for o in it.offerings})
    cats = ["c", "m", "r", "t", "g", "i"]
    for pc in prob.classes:
        if rng.random() >= p_req:
            continue
        terms = []
        for _ in range(int(rng.integers(2, 4))):
            u = rng.random()
            if u < 0.4:
                t = [Requirement(ZONE, "In", [str(rng.choice(zones))])]
            elif u < 0.7:
                t = [Requirement(AWS + "instance-category", "In", [str(rng.choice(cats))])]
            else:
                t = [Requirement(AWS + "instance-category", "In", [str(rng.choice(cats))]),
                     Requirement(ARCH, "In", [str(rng.choice(["amd64", "arm64"]))])]
            terms.append(t)
        pc.required_terms = terms
        if not any(t.kind == "spread" for t in pc.topology):
            sel = [Requirement("app", "In", [pc.labels.get("app", "x")])]
            pc.topology = list(pc.topology) + [model.TopologyTerm(
                "spread", ZONE if rng.random() < 0.7 else HOSTNAME, sel, max_skew=int(rng.integers(1, 3)),
                node_affinity_policy=str(rng.choice(["Honor", "Ignore"])))]
    if rng.random() < 0.5:
        np_ = prob.nodepools[int(rng.integers(0, len(prob.nodepools)))]
        np_.taints = list(np_.taints) + [Taint("example.com/soft", "", "PreferNoSchedule")]
    return prob


def add_many_groups(rng, prob, n_terms=24):
    """Many distinct topology groups over one popular label (tier=web): spreads of several keys and maxSkews,
    required anti-affinity (whose inverse groups constrain every pod they select) and affinity, spread over the
    classes, so that the web classes are constrained by more than 8 groups and counted by more than 16."""
    zones_keys = [ZONE, HOSTNAME, CAPACITY_TYPE]
    for pc in prob.classes:
        pc.labels = dict(pc.labels)
        if rng.random() < 0.6:
            pc.labels["tier"] = "web"
    web = [Requirement("tier", "In", ["web"])]
    for i in range(n_terms):
        pc = prob.classes[int(rng.integers(0, len(prob.classes)))]
        key = str(rng.choice(zones_keys, p=[0.45, 0.4, 0.15]))
        u = rng.random()
        if u < 0.5:
            t = model.TopologyTerm("spread", key, web, max_skew=int(rng.integers(1, 40)),
                                   node_affinity_policy=str(rng.choice(["Honor", "Ignore"])))
        elif u < 0.8:
            t = model.TopologyTerm("anti", key, web + [Requirement("app", "NotIn", ["x%d" % i])])
        else:
            t = model.TopologyTerm("affinity", key, web + [Requirement("app", "NotIn", ["y%d" % i])])
        pc.topology = list(pc.topology) + [t]
    return prob


def _revalue(rng, r, zones):
    """the same requirement key and operator with other values (the node filter's hash sees only the key)"""
    if r.key == ZONE and r.op in ("In", "NotIn"):
        return Requirement(ZONE, r.op, sorted(set(rng.choice(zones, size=int(rng.integers(1, 3))).tolist())))
    if r.key == CAPACITY_TYPE and r.op in ("In", "NotIn"):
        return Requirement(CAPACITY_TYPE, r.op, [str(rng.choice(["spot", "on-demand"]))])
    if r.op in ("Gt", "Lt") and r.values and r.values[0].lstrip("-").isdigit():
        return Requirement(r.key, r.op, [str(max(0, int(r.values[0]) + int(rng.integers(-3, 4))))])
    return Requirement(r.key, r.op, list(r.values), r.min_values)


def add_shared_identities(rng, prob, n_families=None, p_move=0.5):
    """Deployments whose topology terms share one TopologyGroup.Hash() identity while what Hash() does not see differs
    ([core] topology.go Update keeps topologyGroups[hash], the first owner's group): a family's base class (one with a
    spread; one is made if none has) gets 1-2 sibling classes — same labels, namespace, tolerations, terms and
    requirement keys — whose requirement values (zone / capacity-type subsets, Gt / Lt bounds: the Honor node filter's
    values) and spread minDomains differ.  A share of the base's pods move to the siblings, so whichever of them comes
    first in input order decides the group's node filter and minDomains (website scheduling.md:347-372, faq.md:180-182)."""
    import copy
    zones = sorted({o.zone for it in prob.catalog for o in it.offerings})
    bases = [c for c, pc in enumerate(prob.classes) if any(t.kind == "spread" for t in pc.topology)]
    if not bases:
        pc = prob.classes[0]
        pc.topology = list(pc.topology) + [model.TopologyTerm(
            "spread", ZONE, [Requirement("app", "In", [pc.labels.get("app", "x")])], max_skew=1)]
        bases = [0]
    rng.shuffle(bases)
    cls = prob.pods.class_id.copy()
    prob.shared_families = []
    for b in bases[:int(n_families or rng.integers(1, 4))]:
        fam = [b]
        base = prob.classes[b]
        if not any(r.key == ZONE for r in base.requirements) and rng.random() < 0.8:
            base.requirements = list(base.requirements) + [
                Requirement(ZONE, "In", sorted(set(rng.choice(zones, size=2).tolist())))]
        for t in base.topology:
            if t.kind == "spread" and rng.random() < 0.5:
                t.node_affinity_policy = "Honor"
        for _ in range(int(rng.integers(1, 3))):
            sib = copy.deepcopy(base)
            sib.requirements = [_revalue(rng, r, zones) for r in base.requirements]
            for t in sib.topology:
                if t.kind == "spread" and rng.random() < 0.5:
                    t.min_domains = int(rng.integers(1, 6)) if rng.random() < 0.7 else None
            prob.classes.append(sib)
            fam.append(len(prob.classes) - 1)
            idx = np.nonzero(cls == b)[0]
            cls[idx[rng.random(len(idx)) < p_move]] = len(prob.classes) - 1
        prob.bound = [(j, (len(prob.classes) - 1 if c == b and rng.random() < p_move else c)) for j, c in prob.bound]
        prob.shared_families.append(fam)
    prob.pods.class_id = cls.astype(prob.pods.class_id.dtype)
    return prob


def add_relaxed_shared(rng, prob, p_family=0.7):
    """Shared identities that only relaxation creates: each family of add_shared_identities gets ORed required
    node-affinity terms [instance-category In [zz]] (no type) then zone In [a per-class subset]; every pod relaxes the
    first term away, and the relaxed spreads' node filters (the zone term alone) hash equal while their values differ.
    Topology.Update creates that group from the first pod to relax (the device: variant groups, KpDev.late_sib)."""
    zones = sorted({o.zone for it in prob.catalog for o in it.offerings})
    nothing = [Requirement(AWS + "instance-category", "In", ["zz"])]
    for fam in getattr(prob, "shared_families", []):
        if rng.random() >= p_family:
            continue
        for c in fam:
            sub = sorted(set(rng.choice(zones, size=int(rng.integers(1, 3))).tolist()))
            prob.classes[c].required_terms = [list(nothing), [Requirement(ZONE, "In", sub)]]
    return prob


def fuzz_shared_identity_problem(catalog, seed, n_pods=200, n_existing=0):
    """fuzz_topology_problem (or its cluster variant with existing nodes and bound pods) plus add_shared_identities."""
    if n_existing:
        prob = fuzz_topology_existing_problem(catalog, seed, n_pods=n_pods, n_existing=n_existing)
    else:
        prob = fuzz_topology_problem(catalog, seed, n_pods=n_pods)
    return add_shared_identities(np.random.Generator(np.random.PCG64(seed + 4242)), prob)


def fuzz_shared_identity_consolidation(catalog, seed, n_nodes=30, n_pods=160, pending_owner=True):
    """fuzz_topology_consolidation plus add_shared_identities.  Every probe's NewTopology runs over the pending pods
    first, so a family with a pending pod has one first owner in every probe.  pending_owner: one pod of each family
    that has none moves from its candidate to the front of the pending pods; otherwise the pending pods of the families
    are dropped, so each probe's first owner is among its own candidates' pods."""
    cp = fuzz_topology_consolidation(catalog, seed, n_nodes=n_nodes, n_pods=n_pods)
    rng = np.random.Generator(np.random.PCG64(seed + 4343))
    prob = add_shared_identities(rng, cp.cluster)
    cls = prob.pods.class_id
    pending = [int(p) for p in cp.pending]
    if not pending_owner:
        fam_cls = {c for fam in prob.shared_families for c in fam}
        cp.pending = np.array([p for p in pending if int(cls[p]) not in fam_cls], np.int32)
        return cp
    for fam in prob.shared_families:
        if any(int(cls[p]) in fam for p in pending):
            continue
        for cd in cp.candidates:
            hit = [int(p) for p in cd.pods if int(cls[p]) in fam]
            if hit:
                cd.pods = np.array([p for p in cd.pods if int(p) != hit[0]], np.int32)
                pending.insert(0, hit[0])
                break
    cp.pending = np.array(pending, np.int32)
    return cp


def add_reservation_id_requirements(rng, prob, p_class=0.35, p_pool=0.5):
    """Pods and NodePools that select capacity reservations by ID (website odcrs.md:53-57: karpenter.k8s.aws/
    capacity-reservation-id as a scheduling constraint): In / NotIn 1-4 IDs of the catalog, Exists, DoesNotExist, on
    some pod classes and NodePools (those NodePools also allow capacity-type reserved)."""
    ids = sorted({o.reservation_id for it in prob.catalog for o in it.offerings if o.capacity_type == "reserved"})
    if not ids:
        return prob
    RID = AWS + "capacity-reservation-id"

    def req():
        u = rng.random()
        if u < 0.55:
            return Requirement(RID, "In", sorted(set(rng.choice(ids, size=int(rng.integers(1, 5))).tolist())))
        if u < 0.75:
            return Requirement(RID, "NotIn", sorted(set(rng.choice(ids, size=int(rng.integers(1, 4))).tolist())))
        return Requirement(RID, "Exists" if u < 0.9 else "DoesNotExist")
    for pc in prob.classes:
        if rng.random() < p_class:
            pc.requirements = list(pc.requirements) + [req()]
    for np_ in prob.nodepools:
        if rng.random() < p_pool:
            np_.requirements = list(np_.requirements) + [req()]
            for r in np_.requirements:
                if r.key == CAPACITY_TYPE and r.op == "In":
                    r.values = sorted(set(r.values) | {"reserved"})
    return prob


def fuzz_preference_consolidation(catalog, seed, n_nodes=30, n_pods=160, n_bound=30, all_spot=False, best_effort=False,
                                  zone_min=False):
    """fuzz_consolidation over pods with preferences to relax (add_preferences), pods of those classes bound to random
    nodes (their selectors count), sometimes a PreferNoSchedule taint on a pool; best_effort: MIN_VALUES_POLICY=BestEffort
    with minValues on instance-family that a NodeClaim may not meet; zone_min: minValues on the zone label."""
    from kpsim import abi
    cp = fuzz_consolidation(catalog, seed, n_nodes=n_nodes, n_pods=n_pods, all_spot=all_spot,
                            with_min=best_effort)
    rng = np.random.Generator(np.random.PCG64(seed + 321))
    prob = add_preferences(rng, cp.cluster)
    E = len(prob.existing)
    prob.bound = [(int(rng.integers(0, E)), int(rng.integers(0, len(prob.classes)))) for _ in range(n_bound)]
    if seed % 3 == 0:
        prob.nodepools[0].taints = list(prob.nodepools[0].taints) + [Taint("example.com/soft", "", "PreferNoSchedule")]
    if best_effort:
        prob.min_values_policy = abi.KP_MIN_VALUES_BEST_EFFORT
        for np_ in prob.nodepools:
            if rng.random() < 0.7:
                np_.requirements = list(np_.requirements) + [
                    Requirement(AWS + "instance-family", "Exists", [], int(rng.choice([2, 5, 20, 60, 150])))]
    if zone_min:
        for np_ in prob.nodepools:
            np_.requirements = [r for r in np_.requirements if r.key != ZONE] + [
                Requirement(ZONE, "Exists", [], int(rng.choice([1, 2, 3])))]
    return cp


WIDE_RESOURCES = ["vpc.amazonaws.com/pod-eni", "vpc.amazonaws.com/efa", "nvidia.com/gpu", "aws.amazon.com/neuron",
                  "amd.com/gpu", "habana.ai/gaudi"]


def add_extra_resources(rng, prob, n_extra=None):
    """Requests of further resources on some classes' pods (pod ENIs, EFA, accelerators), so that more resource axes are
    active than the consolidation probes keep in registers (cpu, memory, pods + these: 7-9 axes)."""
    n_extra = int(n_extra or rng.integers(4, len(WIDE_RESOURCES) + 1))
    req = prob.pods.requests.copy()
    for res in WIDE_RESOURCES[:n_extra]:
        c = int(rng.integers(0, len(prob.classes)))
        req[prob.pods.class_id == c, model.RIDX[res]] = 1000 * int(rng.integers(1, 3))
        for n in prob.existing:  # most nodes carry some of it (device-plugin resources of the cluster's nodes)
            if rng.random() < 0.8:
                n.available = np.array(n.available, np.int64).copy()
                n.available[model.RIDX[res]] = 1000 * int(rng.integers(1, 9))
    prob.pods.requests = req
    return prob
