"""CPU: ReservationManager invariants of the oracle's Solve (config 5 and reservation-scarce problems)."""
import collections

import pytest

import kat_cases as KC
import parity
from kpsim import synth


def _check_capacity(prob, reqs):
    cap = {}
    for it in prob.catalog:
        for o in it.offerings:
            if o.capacity_type == "reserved":
                cap[o.reservation_id] = min(cap.get(o.reservation_id, 1 << 30), o.reservation_capacity)
    used = collections.Counter()
    for q in reqs:
        if KC.RESVID in q and not q[KC.RESVID][0]:
            for rid in q[KC.RESVID][4]:
                used[rid] += 1
    for rid, n in used.items():
        assert n <= cap[rid], (rid, n, cap[rid])
    return used


def test_config5_reservations_within_capacity(golden):
    prob = synth.config5(n_pods=4000, golden=golden)
    res, reqs = parity.run_oracle(prob)
    used = _check_capacity(prob, reqs)
    assert sum(used.values()) > 0
    # every NodeClaim of the ODCR-only NodePool holds a reservation
    for i in range(res.n_nodeclaims):
        if prob.nodepools[int(res.nodeclaim_nodepool[i])].name == "odcr":
            assert KC.RESVID in reqs[i] and reqs[i][KC.RESVID][4]


@pytest.mark.parametrize("seed", range(4))
def test_scarce_reservations_within_capacity(golden, seed):
    from test_gpu_reserved import scarce_problem
    prob = scarce_problem(golden, seed)
    res, reqs = parity.run_oracle(prob)
    _check_capacity(prob, reqs)
