"""CPU: the oracle's ExistingNode.Add ([core] scheduling/existingnode.go) on small known cases."""
import numpy as np

import parity
from kpsim import model, synth
from kpsim.abi import KP_POD_EXISTING


def _node(name, fake_it, cpu_m, labels=None, taints=None):
    avail = np.array(fake_it.allocatable, np.int64).copy()
    avail[model.RIDX["cpu"]] = cpu_m
    lab = {model.ZONE: "test-zone-1a", model.CAPACITY_TYPE: "on-demand", model.INSTANCE_TYPE: fake_it.name}
    lab.update(labels or {})
    return model.ExistingNode(name=name, labels=lab, available=avail, taints=taints or [])


def test_existing_first_fit_then_new_nodeclaim(fake):
    it = fake[0]
    pods = synth.pods_from_specs([(0, {"cpu": "1"})] * 5)
    prob = model.Problem(fake, [synth.default_nodepool()], [model.PodClass()], pods,
                         existing=[_node("node-0", it, 1500), _node("node-1", it, 2500)])
    r = parity.run_oracle(prob)[0]
    res = sorted(r.pod_result.tolist())
    # node-0 takes 1 pod (1.5 cpu), node-1 takes 2, the remaining 2 go to one new NodeClaim
    assert res.count(KP_POD_EXISTING(0)) == 1 and res.count(KP_POD_EXISTING(1)) == 2
    assert r.n_nodeclaims == 1 and (r.pod_result >= 0).sum() == 2


def test_existing_hostname_selector_and_taints(fake):
    it = fake[0]
    cls = [model.PodClass([model.Requirement("kubernetes.io/hostname", "In", ["node-1"])]),
           model.PodClass()]
    pods = synth.pods_from_specs([(0, {"cpu": "1"}), (1, {"cpu": "1"})])
    prob = model.Problem(fake, [synth.default_nodepool()], cls, pods,
                         existing=[_node("node-0", it, 8000, taints=[model.Taint("dedicated", "x", "NoSchedule")]),
                                   _node("node-1", it, 8000)])
    r = parity.run_oracle(prob)[0]
    # the hostname selector pins pod 0 to node-1; the tainted node-0 is skipped by the untolerating pod 1
    assert r.pod_result.tolist() == [KP_POD_EXISTING(1), KP_POD_EXISTING(1)]
