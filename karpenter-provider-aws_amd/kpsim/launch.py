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


# ---- Fleet emulation: the kwok fake EC2's CreateFleet override pick ----

MAX_FLOAT64 = 1.7976931348623157e308


def min_by_score(scores: List[float]) -> int:
    """Index lo.MinBy picks in kwok/ec2/ec2.go:432-461: min starts at item 0 and item i replaces it when
    comparison(item, min) holds, where comparison is true if min's score is 0 (lo.IsEmpty), false if the item's score
    is 0, else item < min.  Ties keep the earlier override."""
    if not scores:
        return -1
    best = 0
    for i in range(1, len(scores)):
        a, b = scores[i], scores[best]
        if b == 0.0 or (a != 0.0 and a < b):
            best = i
    return best


def fleet_pick(catalog, res: model.LaunchResults, i: int):
    """(type index, offering row) CreateFleet would launch for request i in the kwok provider, or None.

    Overrides come in getOverrides order (instance.go:420-467: kept types in Truncate order, then each type's
    Available ∧ Compatible offerings; every zone is assumed to have a subnet).  The fleet's target capacity type is spot
    for a spot launch and on-demand otherwise (reserved launches are on-demand fleets); kwok/strategy/strategy.go:45-60
    scores an override by SpotPrice(type, zone) or OnDemandPrice(type), MaxFloat64 when there is no price."""
    r = res.rows[i]
    if int(r["status"]) != 0:
        return None
    from kpsim import abi
    spot = int(r["capacity_type"]) == abi.KP_CT_SPOT
    owner = [t for t, it in enumerate(catalog) for _ in it.offerings]
    flat = [o for it in catalog for o in it.offerings]
    rows = [int(x) for x in res.offerings(i)]

    def score(row):
        it = catalog[owner[row]]
        if spot:
            return next((o.price for o in it.offerings if o.capacity_type == "spot" and o.zone == flat[row].zone),
                        MAX_FLOAT64)
        return next((o.price for o in it.offerings if o.capacity_type == "on-demand"), MAX_FLOAT64)

    k = min_by_score([score(row) for row in rows])
    return None if k < 0 else (owner[rows[k]], rows[k])
