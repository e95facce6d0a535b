"""Reference-shaped entry point: Scheduler.Solve on the gfx950 library.

Mirrors [core] pkg/controllers/provisioning/scheduling/scheduler.go — NewScheduler(nodePools,
instanceTypes, ...) then Solve(pods) -> Results{NewNodeClaims, ExistingNodes, PodErrors} — followed by
Results.TruncateInstanceTypes(maxInstanceTypes=60) as the provisioner does (instance.go:62,293).  The
instance-type catalog is what CloudProvider.GetInstanceTypes returns (pkg/cloudprovider/cloudprovider.go:181).
"""
from dataclasses import dataclass
from typing import Dict, List, Optional

from . import abi, model, native


@dataclass
class NodeClaim:
    """A NewNodeClaim of scheduling.Results."""
    index: int
    nodepool: str
    pods: List[int]
    instance_types: List[str]       # truncated, price-ordered (OrderByPrice, ≤ 60)
    instance_type_rows: List[int]
    n_options: int                  # InstanceTypeOptions before truncation


@dataclass
class SolveResults:
    new_nodeclaims: List[NodeClaim]
    pod_errors: List[int]           # pods with an entry in Results.PodErrors
    existing: Dict[int, int]        # pod -> existing node index
    raw: model.Results


class Scheduler:
    def __init__(self, catalog: List[model.InstanceType], device=0, ctx: Optional[native.Context] = None):
        self.ctx = ctx or native.Context(device)
        self.catalog = catalog
        self.catalog_view = model.CatalogView(catalog)
        self.ctx.upload_catalog(self.catalog_view)

    def solve_raw(self, prob: model.Problem) -> model.Results:
        iv = model.SolveInputView(prob)
        cap_nc = max(16, min(prob.pods.n + 1, 8192))
        m = prob.max_instance_types if prob.max_instance_types > 0 else len(self.catalog)
        out = model.OutputBuffers(prob.pods.n, cap_nc, cap_nc * m)
        try:
            self.ctx.solve(iv, out)
        except native.KpError as e:
            if e.status != abi.KP_E_BUFFER:
                raise
            # more NodeClaims than the first buffers hold (node-dense solves): kp_solve_fetch reported the sizes and can
            # be called again on the executed solve with buffers of exactly that size
            v = out.view
            out = model.OutputBuffers(prob.pods.n, max(1, v.n_nodeclaims), max(1, v.n_type_ids))
            self.ctx.fetch(out)
        return out.results()

    def Solve(self, prob: model.Problem) -> SolveResults:
        r = self.solve_raw(prob)
        by_nc: Dict[int, List[int]] = {}
        existing, errors = {}, []
        for p, res in enumerate(r.pod_result.tolist()):
            if res >= 0:
                by_nc.setdefault(res, []).append(p)
            elif res == -1:
                errors.append(p)
            else:
                existing[p] = -2 - res
        ncs = []
        for i, rows in enumerate(r.nodeclaim_types):
            npi = int(r.nodeclaim_nodepool[i])
            if npi < 0:
                continue
            pods = sorted(by_nc.get(i, []), key=lambda p: r.pod_order[p])
            ncs.append(NodeClaim(i, prob.nodepools[npi].name, pods, [self.catalog[t].name for t in rows], rows,
                                 int(r.nodeclaim_n_options[i])))
        return SolveResults(ncs, errors, existing, r)
