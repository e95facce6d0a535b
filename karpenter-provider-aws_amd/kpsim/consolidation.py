"""Reference-shaped consolidation on the gfx950 library, sharded over ranks.

Mirrors [core] sigs.k8s.io/karpenter pkg/controllers/disruption (recalled):
  SingleNodeConsolidation.ComputeCommand — candidates in disruption-cost order, the first whose
      computeConsolidation is not a no-op wins (singlenodeconsolidation.go);
  MultiNodeConsolidation.firstNConsolidationOption — binary search over the prefix length, a prefix is kept when its
      command is DELETE or a REPLACE whose options survive filterOutSameInstanceType (multinodeconsolidation.go).
Every probe those loops could evaluate is independent, so the probes are evaluated in parallel (kp_consolidate; one
wave per probe; one shard of probes per GPU) and the loops are replayed over the results: the decision is the one
the sequential code would reach.  Across ranks the only exchange is the result vector: an all-reduce MIN of the first
valid single-node index, or an all-gather of the multi-node prefix results.
"""
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import abi, model, native


@dataclass
class Command:
    decision: int                   # abi.KP_DECISION_*
    candidates: list                # indices into ConsolidationProblem.candidates
    n_replacement_types: int = 0
    candidate_price: float = 0.0
    replacement_price: float = 0.0
    # kp_consolidate_command only: the method that produced it, its probe, and the replacement NodeClaim
    mode: int = -1
    probe: int = -1
    nodepool: int = -1
    type_ids: list = field(default_factory=list)  # catalog rows, OrderByPrice order
    requirements: str = ""                         # kp_result_nodeclaim_requirements text
    n_reserved: int = 0


NO_OP = Command(abi.KP_DECISION_NONE, [])


def command_call(fn, cap_types=1024, cap_req=1 << 16):
    """Call fn(kp_consolidation_command) (kp_consolidate_command or the oracle's) with output buffers, growing them on
    KP_E_BUFFER -> (status, Command)."""
    import ctypes as C
    for _ in range(2):
        types = np.zeros(cap_types, np.int32)
        req = C.create_string_buffer(int(cap_req))
        cc = abi.kp_consolidation_command()
        cc.cap_type_ids = cap_types
        cc.type_ids = types.ctypes.data_as(C.POINTER(C.c_int32))
        cc.cap_requirements = cap_req
        cc.requirements = C.cast(req, C.c_char_p)
        st = fn(cc)
        if st == abi.KP_E_BUFFER:
            cap_types = max(cap_types, cc.n_type_ids)
            cap_req = max(cap_req, cc.requirements_needed)
            continue
        break
    if st != abi.KP_OK:
        return st, None
    r = cc.result
    cands = list(range(cc.first_candidate, cc.first_candidate + cc.n_candidates))
    cmd = Command(int(cc.decision), cands, int(r.n_replacement_types), float(r.candidate_price),
                  float(r.replacement_price), int(cc.mode), int(cc.probe), int(cc.nodepool),
                  [int(x) for x in types[:cc.n_type_ids]], req.value.decode() if cc.decision == abi.KP_DECISION_REPLACE
                  else "", int(cc.n_reserved))
    return st, cmd


def first_valid_single(results: np.ndarray, probe0: int = 0) -> int:
    """Index (global probe id) of the first non-NONE single-node probe, or -1."""
    idx = np.nonzero(results["decision"] != abi.KP_DECISION_NONE)[0]
    return int(idx[0]) + probe0 if len(idx) else -1


def replay_multi(results: np.ndarray, n_candidates: int, max_candidates: int = 100) -> int:
    """firstNConsolidationOption's binary search over probe results (probe i = prefix of i+2 candidates).
    Returns the chosen probe index or -1."""
    if n_candidates < 2:
        return -1
    lo, hi = 1, max_candidates
    if n_candidates <= hi:
        hi = n_candidates - 1
    best = -1
    while lo <= hi:
        mid = (lo + hi) // 2
        r = results[mid - 1]
        if r["valid"]:
            best = mid - 1
            lo = mid + 1
        else:
            hi = mid - 1
    return best


def _command(cp, results, probe, mode, replacement_fn=None) -> Command:
    """The Command of the chosen probe; replacement_fn(cp, mode, probe) -> Command (kp_consolidate_replacement on this
    process's device, or the oracle's) supplies a REPLACE's replacement NodeClaim: NodePool, price-ordered options,
    requirements, held reservations."""
    if probe < 0:
        return NO_OP
    r = results[probe]
    cands = [probe] if mode == abi.KP_CONSOLIDATE_SINGLE else list(range(probe + 2))
    cmd = Command(int(r["decision"]), cands, int(r["n_replacement_types"]), float(r["candidate_price"]),
                  float(r["replacement_price"]), mode, probe)
    if cmd.decision == abi.KP_DECISION_REPLACE and replacement_fn is not None:
        rep = replacement_fn(cp, mode, probe)
        if (rep.decision, rep.n_replacement_types, rep.replacement_price) != \
                (cmd.decision, cmd.n_replacement_types, cmd.replacement_price):
            raise RuntimeError("replacement read-back disagrees with the gathered probe row")
        cmd.nodepool, cmd.type_ids, cmd.requirements, cmd.n_reserved = rep.nodepool, rep.type_ids, rep.requirements, \
            rep.n_reserved
    return cmd


def shard_range(n_probes, rank, world):
    """Contiguous probe shard of a rank (disruption-cost order is kept inside each shard)."""
    per = (n_probes + world - 1) // world if world else n_probes
    b0 = min(n_probes, rank * per)
    return b0, min(n_probes, b0 + per)


def compute_command(cp: model.ConsolidationProblem, mode, probe_fn, max_candidates=100, group=None,
                    distributed=True, replacement_fn=None) -> Command:
    """ComputeCommand for one mode.  probe_fn(cp, mode, begin, end) evaluates probes [begin, end) (kp_consolidate on
    this rank's GPU).  With a torch.distributed group the probes are sharded across its ranks and one collective
    carries each rank's result: the first valid single-node probe of the shard, or the shard's multi-node rows.
    distributed=False: probe_fn covers the whole range in this process (a multi-device kp_ctx shards internally).
    replacement_fn(cp, mode, probe): a REPLACE's replacement NodeClaim, read back on every rank from its own prepared
    pass (one probe, no further collective), so every rank returns the whole Command."""
    n = model.consolidation_probe_count(len(cp.candidates), mode, max_candidates)
    if n == 0:
        return NO_OP
    if not distributed or (group is None and not _dist_on()):
        res = probe_fn(cp, mode, 0, 0)
        probe = first_valid_single(res) if mode == abi.KP_CONSOLIDATE_SINGLE else \
            replay_multi(res, len(cp.candidates), max_candidates)
        return _command(cp, res, probe, mode, replacement_fn)
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    b0, b1 = shard_range(n, rank, world)
    res = probe_fn(cp, mode, b0, b1) if b1 > b0 else np.zeros(0, abi.PROBE_DTYPE)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else \
        torch.device("cpu")
    if mode == abi.KP_CONSOLIDATE_SINGLE:
        loc = first_valid_single(res, b0)
        row = np.zeros(1, abi.PROBE_DTYPE)
        if loc >= 0:
            row[0] = res[loc - b0]
        msg = np.concatenate([np.array([loc if loc >= 0 else n], np.int64).view(np.uint8), row.view(np.uint8)])
        t = torch.from_numpy(msg).to(dev)
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t, group=group)
        best, best_row = n, None
        for p_ in parts:
            a = p_.cpu().numpy()
            i = int(a[:8].view(np.int64)[0])
            if i < best:
                best, best_row = i, a[8:].view(abi.PROBE_DTYPE)
        if best >= n:
            return NO_OP
        full = np.zeros(n, abi.PROBE_DTYPE)
        full[best] = best_row[0]
        return _command(cp, full, best, mode, replacement_fn)
    per = (n + world - 1) // world
    pad = np.zeros(per, abi.PROBE_DTYPE)
    pad[:len(res)] = res
    loc = torch.from_numpy(pad.view(np.uint8).copy()).to(dev)
    parts = [torch.empty_like(loc) for _ in range(world)]
    dist.all_gather(parts, loc, group=group)
    full = np.concatenate([p_.cpu().numpy().view(abi.PROBE_DTYPE) for p_ in parts])[:n]
    probe = replay_multi(full, len(cp.candidates), max_candidates)
    return _command(cp, full, probe, mode, replacement_fn)


def _dist_on():
    try:
        import torch.distributed as dist
        return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    except Exception:
        return False


class Consolidator:
    """Evaluates consolidation probes on one GPU (one kp_ctx); under torch.distributed, one rank of the pass."""

    def __init__(self, catalog, device=0, ctx: Optional[native.Context] = None, spot_to_spot=False,
                 max_candidates=100):
        self.ctx = ctx or native.Context(device)
        self.catalog_view = model.CatalogView(catalog)
        self.ctx.upload_catalog(self.catalog_view)
        self.spot_to_spot = spot_to_spot
        self.max_candidates = max_candidates

    def probes(self, cp: model.ConsolidationProblem, mode, begin=0, end=0, cluster_view=None) -> np.ndarray:
        v = model.ConsolidateInputView(cp, mode, begin, end, self.spot_to_spot, self.max_candidates, cluster_view)
        res = self.ctx.consolidate(v)
        self._prepared = (cp, mode, self.ctx.pass_gen, v)  # kp_consolidate leaves the pass prepared on the ctx
        return res

    def replacement(self, cp: model.ConsolidationProblem, mode, probe) -> Command:
        """kp_consolidate_replacement of one probe; prepares the pass first unless the ctx still holds this process's
        pass of (cp, mode): nothing else (a Solve, another pass, a catalog change) ran on the ctx since (pass_gen)."""
        prep = getattr(self, "_prepared", None)
        if prep is None or prep[0] is not cp or prep[1] != mode or prep[2] != self.ctx.pass_gen:
            v = model.ConsolidateInputView(cp, mode, 0, 0, self.spot_to_spot, self.max_candidates)
            self.ctx.consolidate_prepare(v)
            self._prepared = (cp, mode, self.ctx.pass_gen, v)
        return self.ctx.consolidate_replacement(mode, probe)

    def compute_command(self, cp: model.ConsolidationProblem, mode, group=None) -> Command:
        """The Command of one method, with the replacement NodeClaim of a REPLACE (kp_consolidate_replacement over this
        process's prepared pass)."""
        return compute_command(cp, mode, lambda c, m, b0, b1: self.probes(c, m, b0, b1), self.max_candidates, group,
                               replacement_fn=self.replacement)
