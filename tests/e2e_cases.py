"""The reference's e2e disruption scenarios replayed on the cluster emulator (tests/cluster_sim.py), each asserting the
end state the reference suite asserts.  Quantities the live environment supplies (daemonset overhead: 0 here; node
allocatable) come from the golden catalog.

  replace_hostname_spread  test/suites/consolidation/suite_test.go:574-729  "should consolidate nodes (replace)"
  od_to_spot               test/suites/consolidation/suite_test.go:730-860  "should consolidate on-demand nodes to spot"
  delete_utilization       test/suites/consolidation/suite_test.go:491-573  "should consolidate nodes (delete)"
  anti_affinity_replace    test/suites/scale/deprovisioning_test.go:454-523 "single consolidation replace"
  multi_delete             test/suites/scale/deprovisioning_test.go:399-453 "multi-consolidation delete"

Preference scenarios (website/content/en/preview/concepts/scheduling.md:217-219: preferences are treated as requirements
"when determining if a pod can be shifted to a new node", relaxed one at a time when they cannot be met; PREFERENCE_POLICY,
reference/settings.md:40):
  preferred_anti_affinity_replace  anti_affinity_replace with a preferred (weight 50) hostname anti-affinity: under
                                   Respect every pod keeps a node of its own through consolidation; under Ignore the
                                   Deployment packs onto one node
  preferred_affinity_delete        delete_utilization with pods preferring an instance category no NodePool offers: every
                                   probe relaxes the preference before the pods fit the remaining nodes

NodePool disruption budgets (test/suites/consolidation/suite_test.go:188-453; budgets filter the candidates caller-side,
cluster_sim.SimCluster.consolidate_once_budgeted; the emulator executes commands synchronously, so "nodes disrupting at
once" is the size of one command):
  budget_empty_delete     :211-247 "should respect budgets for empty delete consolidation" (40%: at most 2 at once)
  budget_nonempty_delete  :248-306 "should respect budgets for non-empty delete consolidation" (50% of 3: at most 2)
  budget_replace          :307-409 "should respect budgets for non-empty replace consolidation" ("3"; 5 replaced)
  budget_blocking         :410-436 "should not allow consolidation if the budget is fully blocking" ("0")
"""
import copy

import numpy as np

from cluster_sim import SimCluster
from kpsim import model
from kpsim.model import CAPACITY_TYPE, HOSTNAME, INSTANCE_TYPE

SIZE = "karpenter.k8s.aws/instance-size"
FAMILY = "karpenter.k8s.aws/instance-family"
HYPERVISOR = "karpenter.k8s.aws/instance-hypervisor"
OS = "kubernetes.io/os"
EXCLUDED_FAMILIES = ["t2", "t3", "c1", "t3a", "t4g", "a1"]


def _spread_class(app):
    return model.PodClass(labels={"app": app}, topology=[model.TopologyTerm(
        "spread", HOSTNAME, selector=[model.Requirement("app", "In", [app])], max_skew=1)])


def _n_nodes_of(sim):
    return len(sim.nodes)


def replace_hostname_spread(golden, backend, spot):
    """3 nodes (a 4-cpu large-app pod + a 1.8-cpu small-app pod each, hostname spread on both); the large deployment
    scales to 0; consolidation replaces each 2xlarge with a .large (utilisation > 0.8, 3 nodes, all .large)."""
    ct = "spot" if spot else "on-demand"
    pool = model.NodePool("default", requirements=[
        model.Requirement(CAPACITY_TYPE, "In", [ct]), model.Requirement(SIZE, "In", ["large", "2xlarge"]),
        model.Requirement(FAMILY, "NotIn", EXCLUDED_FAMILIES), model.Requirement(OS, "In", ["linux"])])
    sim = SimCluster(golden, [pool], [_spread_class("large-app"), _spread_class("small-app")], backend,
                     spot_to_spot=spot)
    large = sim.add_pods(0, 3, {"cpu": "4"})
    sim.add_pods(1, 3, {"cpu": "1800m"})
    sim.provision()
    assert _n_nodes_of(sim) == 3  # "3 nodes due to the anti-affinity rules"
    sim.delete_pods(large)
    assert sim.utilization() < 0.5
    sim.consolidate()
    sizes = [golden[n.type_row].name for n in sim.nodes]
    assert sim.utilization() > 0.8, sizes
    assert len(sizes) == 3 and all(s.endswith(".large") for s in sizes), sizes
    return sim


def od_to_spot(golden, backend):
    """2 on-demand .large nodes (one hostname-spread 1.8-cpu pod each); the NodePool then allows every capacity type:
    both nodes are replaced by spot nodes."""
    pool = model.NodePool("default", requirements=[
        model.Requirement(CAPACITY_TYPE, "In", ["on-demand"]), model.Requirement(SIZE, "In", ["large"]),
        model.Requirement(FAMILY, "NotIn", EXCLUDED_FAMILIES)])
    sim = SimCluster(golden, [pool], [_spread_class("small-app")], backend)
    sim.add_pods(0, 2, {"cpu": "1800m"})
    sim.provision()
    assert _n_nodes_of(sim) == 2 and all(n.capacity_type == "on-demand" for n in sim.nodes)
    _replace(pool, model.Requirement(CAPACITY_TYPE, "Exists"), model.Requirement(SIZE, "In", ["large"]))
    sim.consolidate()
    cts = [n.capacity_type for n in sim.nodes]
    assert cts == ["spot", "spot"], cts
    return sim


def delete_utilization(golden, backend, spot, n_pods=100):
    """100 one-cpu pods over medium / large / xlarge nodes, scaled to 40: consolidation deletes nodes until the
    average cpu utilisation exceeds 0.6."""
    pool = model.NodePool("default", requirements=[
        model.Requirement(CAPACITY_TYPE, "In", ["spot" if spot else "on-demand"]),
        model.Requirement(SIZE, "In", ["medium", "large", "xlarge"]), model.Requirement(FAMILY, "NotIn", EXCLUDED_FAMILIES)])
    cls = model.PodClass(labels={"app": "large-app"})
    sim = SimCluster(golden, [pool], [cls], backend, spot_to_spot=spot)
    pods = sim.add_pods(0, n_pods, {"cpu": "1"})
    sim.provision()
    # scale to 40%: ReplicaSet scale-down takes pods from the nodes with the most replicas first
    keep = int(n_pods * 0.4)
    drop = []
    while len(pods) - len(drop) > keep:
        n = max(sim.nodes, key=lambda x: (len([p for p in x.pods if p not in drop]), x.name))
        drop.append([p for p in n.pods if p not in drop][-1])
    sim.delete_pods(drop)
    assert sim.utilization() < 0.5
    sim.consolidate()
    assert sim.utilization() > 0.6, sim.utilization()
    return sim


def _replace(pool, *reqs):
    """coretest.ReplaceRequirements: requirements on the same keys are replaced, the others kept."""
    keys = {r.key for r in reqs}
    pool.requirements = [r for r in pool.requirements if r.key not in keys] + list(reqs)


def _nitro_pool(size):
    """env.DefaultNodePool (test/pkg/environment/common/environment.go:133-177) with the scale suite's
    ReplaceRequirements (deprovisioning_test.go:88-102): hypervisor nitro, instance-size `size`."""
    pool = model.NodePool("default", requirements=[
        model.Requirement(OS, "In", ["linux"]), model.Requirement(CAPACITY_TYPE, "In", ["on-demand"]),
        model.Requirement("karpenter.k8s.aws/instance-category", "In", ["c", "m", "r"]),
        model.Requirement("karpenter.k8s.aws/instance-generation", "Gt", ["4"]), model.Requirement(FAMILY, "NotIn", ["a1"])])
    _replace(pool, model.Requirement(HYPERVISOR, "In", ["nitro"]), model.Requirement(SIZE, "In", [size]))
    return pool


def anti_affinity_replace(golden, backend, n_nodes=20):
    """20 pods with required hostname anti-affinity on 2xlarge nodes; the instance-size requirement is dropped: every
    node is replaced (20 deleted, 20 remain)."""
    pool = _nitro_pool("2xlarge")
    cls = model.PodClass(labels={"app": "dep"}, topology=[model.TopologyTerm(
        "anti", HOSTNAME, selector=[model.Requirement("app", "In", ["dep"])])])
    sim = SimCluster(golden, [pool], [cls], backend)
    sim.add_pods(0, n_nodes, {"cpu": "10m", "memory": "50Mi"})
    sim.provision()
    first = {n.name for n in sim.nodes}
    assert len(first) == n_nodes
    pool.requirements = [r for r in pool.requirements if r.key != SIZE]
    sim.consolidate()
    assert len(sim.nodes) == n_nodes
    assert not first & {n.name for n in sim.nodes}  # every original node was replaced
    return sim


def multi_delete(golden, backend, n_nodes=200, per_node=20):
    """200 .large nodes at kubelet maxPods = 20 replicas each; the deployment scales to 20%: consolidation deletes 80%
    of the nodes (40 remain, every pod healthy)."""
    cat = copy.deepcopy(golden)
    r = model.RIDX["pods"]
    for it in cat:  # kubelet MaxPods = replicasPerNode + dsCount, the daemonsets' slots taken (no daemonsets here)
        it.capacity = np.array(it.capacity, np.int64).copy()
        it.allocatable = np.array(it.allocatable, np.int64).copy()
        it.capacity[r] = it.allocatable[r] = per_node * 1000
    pool = _nitro_pool("large")
    sim = SimCluster(cat, [pool], [model.PodClass(labels={"app": "dep"})], backend)
    pods = sim.add_pods(0, n_nodes * per_node, {"cpu": "10m", "memory": "50Mi"})
    sim.provision()
    assert len(sim.nodes) == n_nodes
    keep = set()
    for n in sim.nodes:  # ReplicaSet scale-down evens the replicas out: 4 of 20 stay on every node
        keep.update(n.pods[:per_node // 5])
    sim.delete_pods([p for p in pods if p not in keep])
    sim.consolidate()
    assert len(sim.nodes) == n_nodes // 5, len(sim.nodes)
    assert sum(len(n.pods) for n in sim.nodes) == len(keep)
    return sim


def preferred_anti_affinity_replace(golden, backend, n_nodes=10, respect=True):
    pool = _nitro_pool("2xlarge")
    cls = model.PodClass(labels={"app": "dep"}, topology=[model.TopologyTerm(
        "anti", HOSTNAME, selector=[model.Requirement("app", "In", ["dep"])], weight=50)])
    sim = SimCluster(golden, [pool], [cls], backend)
    sim.add_pods(0, n_nodes, {"cpu": "10m", "memory": "50Mi"})
    sim.provision()
    first = {n.name for n in sim.nodes}
    assert len(first) == (n_nodes if respect else 1), len(first)
    pool.requirements = [r for r in pool.requirements if r.key != SIZE]
    sim.consolidate()
    if respect:  # each node replaced by a cheaper one, one pod per node throughout
        assert len(sim.nodes) == n_nodes and not first & {n.name for n in sim.nodes}
        assert all(len(n.pods) == 1 for n in sim.nodes)
    else:
        assert len(sim.nodes) == 1 and not first & {n.name for n in sim.nodes}
    return sim


def preferred_affinity_delete(golden, backend, n_pods=60):
    pool = model.NodePool("default", requirements=[
        model.Requirement(CAPACITY_TYPE, "In", ["on-demand"]), model.Requirement(SIZE, "In", ["medium", "large", "xlarge"]),
        model.Requirement("karpenter.k8s.aws/instance-category", "In", ["c", "m"]),
        model.Requirement(FAMILY, "NotIn", EXCLUDED_FAMILIES)])
    cls = model.PodClass(labels={"app": "dep"}, preferred_terms=[
        (10, [model.Requirement("karpenter.k8s.aws/instance-category", "In", ["r"])])])
    sim = SimCluster(golden, [pool], [cls], backend)
    pods = sim.add_pods(0, n_pods, {"cpu": "1"})
    sim.provision()
    keep = int(n_pods * 0.4)
    drop = []
    while len(pods) - len(drop) > keep:
        n = max(sim.nodes, key=lambda x: (len([p for p in x.pods if p not in drop]), x.name))
        drop.append([p for p in n.pods if p not in drop][-1])
    sim.delete_pods(drop)
    assert sim.utilization() < 0.5
    sim.consolidate()
    assert sim.utilization() > 0.6, sim.utilization()
    assert sum(c.decision == 1 for c in sim.commands) >= 1  # DELETE commands: the relaxed pods fit the other nodes
    return sim


def _default_pool(name="default"):
    """env.DefaultNodePool (test/pkg/environment/common/environment.go:133-177)."""
    return model.NodePool(name, requirements=[
        model.Requirement(OS, "In", ["linux"]), model.Requirement(CAPACITY_TYPE, "In", ["on-demand"]),
        model.Requirement("karpenter.k8s.aws/instance-category", "In", ["c", "m", "r"]),
        model.Requirement("karpenter.k8s.aws/instance-generation", "Gt", ["4"]), model.Requirement(FAMILY, "NotIn", ["a1"])])


def _anti_class(app):
    return model.PodClass(labels={"app": app}, topology=[model.TopologyTerm(
        "anti", HOSTNAME, selector=[model.Requirement("app", "In", [app])])])


def _budget_commands_within(sim, limit):
    for c in sim.commands:
        assert len(c.candidates) <= limit, (len(c.candidates), limit)


def budget_empty_delete(golden, backend):
    sim = SimCluster(golden, [_default_pool()], [_anti_class("regular-app")], backend, budgets={0: ["40%"]})
    pods = sim.add_pods(0, 5, {"cpu": "1"})
    sim.provision()
    assert len(sim.nodes) == 5
    sim.delete_pods(pods[1:])  # replicas 5 -> 1: four empty nodes
    sim.consolidate()
    _budget_commands_within(sim, 2)  # ConsistentlyExpectDisruptionsUntilNoneLeft(5, 2, ...)
    assert [len(c.candidates) for c in sim.commands if c.decision == 1] == [2, 2]
    assert len(sim.nodes) == 1
    return sim


def budget_nonempty_delete(golden, backend):
    pool = _default_pool()
    _replace(pool, model.Requirement(SIZE, "In", ["2xlarge"]))
    sim = SimCluster(golden, [pool], [model.PodClass(labels={"app": "large-app"})], backend, budgets={0: ["50%"]})
    pods = sim.add_pods(0, 9, {"cpu": "2100m"})
    sim.provision()
    assert len(sim.nodes) == 3
    keep = {n.pods[0] for n in sim.nodes}  # replicas 9 -> 3, ForcePodsToSpread: one per node
    sim.delete_pods([p for p in pods if p not in keep])
    sim.consolidate()
    _budget_commands_within(sim, 2)  # ConsistentlyExpectDisruptionsUntilNoneLeft(3, 2, ...)
    assert sim.commands[0].decision == 1 and len(sim.commands[0].candidates) == 2
    assert len(sim.nodes) == 1
    return sim


def budget_replace(golden, backend):
    pool = _default_pool()
    _replace(pool, model.Requirement(SIZE, "In", ["xlarge", "2xlarge"]), model.Requirement("test-partition", "Exists"))
    pool.labels = {"app": "large-app"}
    ds = np.zeros(model.R, np.int64)
    ds[model.RIDX["cpu"]] = 3000  # the 3-cpu daemonset
    pool.daemon_overhead = ds
    classes = [model.PodClass(labels={"app": "large-app"},
                              requirements=[model.Requirement("test-partition", "In", [str(i)])]) for i in range(5)]
    sim = SimCluster(golden, [pool], classes, backend, budgets={0: ["3"]})
    for i in range(5):
        sim.add_pods(i, 1, {"cpu": "3"})
    sim.provision()
    first = {n.name for n in sim.nodes}
    assert len(first) == 5 and all(golden[n.type_row].name.endswith(".2xlarge") for n in sim.nodes)
    pool.daemon_overhead = np.zeros(model.R, np.int64)  # the daemonset is deleted
    sim.consolidate()
    _budget_commands_within(sim, 3)  # ConsistentlyExpectDisruptionsUntilNoneLeft(5, 3, ...)
    assert [c.decision for c in sim.commands] == [2] * 5 + [0]
    assert len(sim.nodes) == 5 and not first & {n.name for n in sim.nodes}  # ExpectNodeCount("==", 5), all rolled
    assert all(golden[n.type_row].name.endswith(".xlarge") for n in sim.nodes)
    return sim


def budget_blocking(golden, backend):
    sim = SimCluster(golden, [_default_pool()], [_anti_class("regular-app")], backend, budgets={0: ["0"]})
    pods = sim.add_pods(0, 5, {"cpu": "1"})
    sim.provision()
    sim.delete_pods(pods[1:])
    sim.consolidate()
    assert [c.decision for c in sim.commands] == [0]  # ConsistentlyExpectNoDisruptions(5, ...)
    assert len(sim.nodes) == 5
    return sim
