"""TEST INFRASTRUCTURE: a small cluster emulator that drives provisioning (Solve) and consolidation (the command) in a
loop, the way the reference's e2e suites drive a real cluster — so their asserted end states (node counts, instance
sizes, capacity types) can be checked against this library.

Backends: `OracleBackend` (CPU restatement) and `DeviceBackend` (libkpsim.so through kpsim.native).  A launched
NodeClaim becomes a node of its cheapest option at the cheapest available offering its requirements admit (CreateFleet
lowest-price, kwok/strategy/strategy.go:45-60); evicted / pending pods are scheduled by a Solve over the remaining nodes
(the provisioner); candidates are every node in disruption-cost order (fewer pods first, then name).
"""
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from kpsim import abi, model, synth
from kpsim.model import CAPACITY_TYPE, RESERVATION_ID, RESERVATION_TYPE, ZONE


@dataclass
class Node:
    name: str
    type_row: int
    zone: str
    capacity_type: str
    nodepool: int
    reservation: str = ""
    pods: List[int] = field(default_factory=list)
    labels: Dict[str, str] = field(default_factory=dict)  # single-valued custom requirements of its NodeClaim


def _admits(reqs, key, value):
    r = reqs.get(key)
    if r is None:
        return True
    cmp_, vals = r
    return (value not in vals) if cmp_ else (value in vals)


def _req_dict(text):
    out = {}
    for line in text.splitlines():
        if line:
            key, cmp_, _gt, _lt, _mv, vals = line.split("\t")
            out[key] = (cmp_ == "1", vals.split("\x1f") if vals else [])
    return out


class OracleBackend:
    def __init__(self, preference_policy=0):
        self.preference_policy = preference_policy  # PREFERENCE_POLICY (the device backend's ctx carries its own)

    def solve(self, prob):
        import pyoracle
        o = pyoracle.solve(prob, preference_policy=self.preference_policy)
        r = o.results
        return r, [o.requirements(i) for i in range(r.n_nodeclaims)]

    def command(self, cp, mode, spot_to_spot=False):
        import pyoracle
        return pyoracle.consolidate_command(cp, mode, spot_to_spot=spot_to_spot, preference_policy=self.preference_policy)


class DeviceBackend:
    def __init__(self, ctx):
        self.ctx = ctx

    def solve(self, prob):
        cv = model.CatalogView(prob.catalog)
        self.ctx.upload_catalog(cv)
        cap_nc = max(16, prob.pods.n + 1)
        out = model.OutputBuffers(prob.pods.n, cap_nc, cap_nc * max(1, prob.max_instance_types))
        self.ctx.solve(model.SolveInputView(prob), out)
        r = out.results()
        return r, [self.ctx.nodeclaim_requirements(i) for i in range(r.n_nodeclaims)]

    def command(self, cp, mode, spot_to_spot=False):
        self.ctx.upload_catalog(model.CatalogView(cp.cluster.catalog))
        self.ctx.consolidate_prepare(model.ConsolidateInputView(cp, abi.KP_CONSOLIDATE_SINGLE, spot_to_spot=spot_to_spot))
        return self.ctx.consolidate_command(mode)


class SimCluster:
    def __init__(self, catalog, nodepools, classes, backend, spot_to_spot=False, min_values_policy=0, budgets=None):
        self.catalog = catalog
        # NodePool disruption budgets (karpv1.Budget.Nodes: "40%", "3", ...) by NodePool index; None: no budgets (the
        # consolidation pass runs both methods over every candidate in one call)
        self.budgets: Optional[Dict[int, List[str]]] = budgets
        self.nodepools = nodepools
        self.classes = classes
        self.backend = backend
        self.spot_to_spot = spot_to_spot
        self.min_values_policy = min_values_policy
        self.pod_class: List[int] = []
        self.pod_req: List[np.ndarray] = []
        self.nodes: List[Node] = []
        self.pending: List[int] = []
        self.n_launched = 0
        self.commands = []

    # ---- pods ----
    def add_pods(self, cls, n, req):
        ids = []
        for _ in range(n):
            v = synth.requests_vec(req)  # incl. pods = 1000
            self.pod_class.append(cls)
            self.pod_req.append(v)
            ids.append(len(self.pod_class) - 1)
        self.pending.extend(ids)
        return ids

    def delete_pods(self, ids):
        ids = set(ids)
        for n in self.nodes:
            n.pods = [p for p in n.pods if p not in ids]
        self.pending = [p for p in self.pending if p not in ids]

    # ---- state views ----
    def _labels(self, n: Node):
        it = self.catalog[n.type_row]
        lab = synth.node_labels(it, n.zone, n.capacity_type, self.nodepools[n.nodepool].name)
        if n.reservation:
            lab[RESERVATION_ID] = n.reservation
            lab[RESERVATION_TYPE] = "default"
        lab.update(n.labels)
        return lab

    def _existing(self, nodes):
        out = []
        for n in nodes:
            it = self.catalog[n.type_row]
            avail = np.array(it.allocatable, np.int64).copy()
            for p in n.pods:
                avail -= self.pod_req[p]
            out.append(model.ExistingNode(n.name, self._labels(n), avail, np.zeros(model.R, np.int64),
                                          list(self.nodepools[n.nodepool].taints)))
        return out

    def _pods(self, ids):
        specs = np.array(ids, np.int64)
        t0 = 1_700_000_000 * 10 ** 9
        return model.Pods(np.array([self.pod_class[p] for p in ids], np.int32),
                          np.array([self.pod_req[p] for p in ids], np.int64).reshape(len(ids), model.R),
                          t0 + specs * 1000, ["pod-%06d" % p for p in ids])

    def _sorted_nodes(self):
        return sorted(self.nodes, key=lambda n: n.name)  # NewScheduler order: all initialized, by name

    # ---- provisioning ----
    def provision(self):
        """Solve the pending pods over the nodes; pods placed on existing nodes bind, new NodeClaims launch."""
        if not self.pending:
            return
        nodes = self._sorted_nodes()
        bound = [(j, self.pod_class[p]) for j, n in enumerate(nodes) for p in n.pods]
        prob = model.Problem(self.catalog, self.nodepools, self.classes, self._pods(self.pending), self._existing(nodes),
                             min_values_policy=self.min_values_policy, bound=bound)
        r, reqs = self.backend.solve(prob)
        launched = {}
        left = []
        for i, p in enumerate(self.pending):
            res = int(r.pod_result[i])
            if res <= -2:
                nodes[-2 - res].pods.append(p)
            elif res >= 0:
                if res not in launched:
                    launched[res] = self.launch(r.nodeclaim_types[res], reqs[res], int(r.nodeclaim_nodepool[res]))
                launched[res].pods.append(p)
            else:
                left.append(p)
        self.pending = left

    def launch(self, type_ids, req_text, nodepool):
        """CreateFleet lowest-price over the NodeClaim's options and the offerings its requirements admit."""
        reqs = _req_dict(req_text)
        best = None
        for t in type_ids:
            for o in self.catalog[t].offerings:
                if not o.available or not _admits(reqs, CAPACITY_TYPE, o.capacity_type) or not _admits(reqs, ZONE, o.zone):
                    continue
                if o.reservation_id and not _admits(reqs, RESERVATION_ID, o.reservation_id):
                    continue
                if best is None or o.price < best[0]:
                    best = (o.price, t, o)
        assert best is not None, "no offering to launch"
        _, t, o = best
        self.n_launched += 1
        n = Node("node-%04d" % self.n_launched, t, o.zone, o.capacity_type, nodepool, o.reservation_id or "")
        # NodeClaim labels from single-valued requirements on keys the instance type does not label (e.g. a custom
        # partition key the pod selected)
        known = set(synth.node_labels(self.catalog[t], o.zone, o.capacity_type, self.nodepools[nodepool].name))
        for key, (cmp_, vals) in reqs.items():
            if not cmp_ and len(vals) == 1 and key not in known and key != RESERVATION_ID:
                n.labels[key] = vals[0]
        if o.reservation_id:
            o.reservation_capacity -= 1
            o.available = o.reservation_capacity != 0
        self.nodes.append(n)
        return n

    # ---- consolidation ----
    def consolidation_problem(self, keep=None):
        """keep(node) -> bool: the candidates offered (disruption budgets); every node stays in the cluster."""
        nodes = self._sorted_nodes()
        pods = [p for n in nodes for p in n.pods]
        pos = {p: i for i, p in enumerate(pods)}
        prob = model.Problem(self.catalog, self.nodepools, self.classes, self._pods(pods), self._existing(nodes),
                             min_values_policy=self.min_values_policy)
        cands = []
        for j, n in enumerate(nodes):
            it = self.catalog[n.type_row]
            ct = {"spot": abi.KP_CT_SPOT, "reserved": abi.KP_CT_RESERVED}.get(n.capacity_type, abi.KP_CT_ON_DEMAND)
            cands.append((len(n.pods), n.name, model.Candidate(
                node=j, pods=np.array([pos[p] for p in n.pods], np.int32),
                price=synth.candidate_price(it, self._labels(n)), capacity_type=ct, instance_type=n.type_row,
                nodepool=n.nodepool, capacity=np.array(it.capacity, np.int64))))
        cands.sort(key=lambda c: (c[0], c[1]))
        if keep is not None:
            cands = [c for c in cands if keep(nodes[c[2].node])]
        cp = model.ConsolidationProblem(prob, [c[2] for c in cands], np.zeros(0, np.int32),
                                        np.ones(len(nodes), np.uint8))
        return cp, nodes

    def allowed_disruptions(self):
        """NodePool → allowed disruptions: the least over its budgets, a percentage of its nodes rounded up
        (Budget.GetAllowedDisruptions, intstr.GetScaledValueFromIntOrPercent(..., roundUp=true)); no disruption is in
        flight between the emulator's synchronous commands."""
        out = {}
        for j in range(len(self.nodepools)):
            specs = (self.budgets or {}).get(j)
            if not specs:
                out[j] = 1 << 30
                continue
            n = sum(1 for x in self.nodes if x.nodepool == j)
            out[j] = min(math.ceil(n * int(b[:-1]) / 100) if b.endswith("%") else int(b) for b in specs)
        return out

    def _execute(self, cp, nodes, cmd):
        self.commands.append(cmd)
        if cmd.decision == abi.KP_DECISION_NONE:
            return cmd
        gone = [nodes[cp.candidates[c].node] for c in cmd.candidates]
        if cmd.decision == abi.KP_DECISION_REPLACE:
            self.launch(cmd.type_ids, cmd.requirements, cmd.nodepool)
        for n in gone:
            if n.reservation:  # the reservation's instance is released
                for o in self.catalog[n.type_row].offerings:
                    if o.reservation_id == n.reservation:
                        o.reservation_capacity += 1
                        o.available = True
            self.pending.extend(n.pods)
            self.nodes.remove(n)
        self.provision()
        assert not self.pending, "pods left pending after executing a consolidation command"
        return cmd

    def consolidate_once_budgeted(self):
        """The disruption controller's methods in order under NodePool budgets, candidates filtered caller-side as the
        controller does (kpsim.h: budgets are outside kp_consolidate): Emptiness deletes empty candidates while their
        NodePool allows (no simulation), then MultiNodeConsolidation over the candidates taken in order while their
        NodePool allows (each taken one counts), then SingleNodeConsolidation over the candidates of NodePools with any
        disruption allowed."""
        from kpsim.consolidation import Command
        allowed = self.allowed_disruptions()
        cp, nodes = self.consolidation_problem()
        left = dict(allowed)
        empty = []
        for ci, c in enumerate(cp.candidates):
            n = nodes[c.node]
            if not n.pods and left[n.nodepool] > 0:
                left[n.nodepool] -= 1
                empty.append(ci)
        if empty:
            return self._execute(cp, nodes, Command(abi.KP_DECISION_DELETE, empty, mode=-1))
        left = dict(allowed)

        def take(n):
            if left[n.nodepool] <= 0:
                return False
            left[n.nodepool] -= 1
            return True

        cp, nodes = self.consolidation_problem(keep=take)
        if cp.candidates:
            cmd = self.backend.command(cp, abi.KP_CONSOLIDATE_MULTI, self.spot_to_spot)
            if cmd.decision != abi.KP_DECISION_NONE:
                return self._execute(cp, nodes, cmd)
        cp, nodes = self.consolidation_problem(keep=lambda n: allowed[n.nodepool] > 0)
        if not cp.candidates:
            return self._execute(cp, nodes, Command(abi.KP_DECISION_NONE, []))
        return self._execute(cp, nodes, self.backend.command(cp, abi.KP_CONSOLIDATE_SINGLE, self.spot_to_spot))

    def consolidate_once(self, mode=abi.KP_CONSOLIDATE_BOTH):
        """One disruption pass: compute the command, then execute it (replacement launched, candidates deleted, their
        pods rescheduled).  Returns the command."""
        if self.budgets is not None:
            return self.consolidate_once_budgeted()
        cp, nodes = self.consolidation_problem()
        return self._execute(cp, nodes, self.backend.command(cp, mode, self.spot_to_spot))

    def consolidate(self, max_rounds=100, mode=abi.KP_CONSOLIDATE_BOTH):
        for _ in range(max_rounds):
            if self.consolidate_once(mode).decision == abi.KP_DECISION_NONE:
                return
        raise AssertionError("consolidation did not converge")

    def utilization(self, resource="cpu"):
        r = model.RIDX[resource]
        used = sum(int(self.pod_req[p][r]) for n in self.nodes for p in n.pods)
        alloc = sum(int(self.catalog[n.type_row].allocatable[r]) for n in self.nodes)
        return used / alloc if alloc else 0.0
