"""Launch-time selection over ranks: NodeClaim launch requests are independent (instance.go:132-137 runs once per
NodeClaim), so a batch is split into contiguous slices, one per rank, each selected on its own GPU with
kp_launch_select; one all_gather_object returns every rank's rows.  There is no other exchange."""
from typing import Callable, List, Optional

from kpsim import model
from kpsim.consolidation import shard_range


def canonical(res: model.LaunchResults) -> List[tuple]:
    """Per request: (status, failed_filter, capacity_type, type ids, override offering rows, n_options, rejected)."""
    out = []
    for i in range(len(res.rows)):
        r = res.rows[i]
        ok = int(r["status"]) == 0
        out.append((int(r["status"]), int(r["failed_filter"]), int(r["capacity_type"]) if ok else -1,
                    tuple(int(x) for x in res.types(i)), tuple(int(x) for x in res.offerings(i)),
                    int(r["n_options"]), tuple(int(x) for x in r["rejected"])))
    return out


def select_sharded(requests: List[model.LaunchRequest], select_fn: Callable[[model.LaunchBatchView], model.LaunchResults],
                   group=None) -> List[tuple]:
    """select_fn(batch) runs kp_launch_select (or the oracle) on this rank's slice; returns the whole batch's
    canonical rows in request order."""
    world, rank = 1, 0
    if group is not None:
        import torch.distributed as dist
        world, rank = dist.get_world_size(group), dist.get_rank(group)
    b0, b1 = shard_range(len(requests), rank, world)
    part = canonical(select_fn(model.LaunchBatchView(requests[b0:b1])))
    if group is None:
        return part
    import torch.distributed as dist
    parts: List[Optional[list]] = [None] * world
    dist.all_gather_object(parts, part, group=group)
    return [row for p in parts for row in p]
