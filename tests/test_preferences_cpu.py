"""CPU: the oracle's preference relaxation and BestEffort minValues (tests/pref_cases.py) against the known answers,
and the relaxation-stage restrictions that the device build shares."""
import pytest

import pref_cases as PC
import pyoracle
from kpsim import abi, model


def run_oracle(c):
    o = pyoracle.solve(c.problem, preference_policy=c.preference_policy)
    r = o.results
    return r, [model.parse_requirements_blob(o.requirements(i)) for i in range(r.n_nodeclaims)]


@pytest.mark.parametrize("mk", PC.CASES, ids=PC.ids())
def test_pref_case_oracle(fx, mk):
    c = mk(fx)
    res, reqs = run_oracle(c)
    c.check(c.problem, res, reqs)


def test_preferred_node_term_on_topology_key_unsupported(fx):
    """Pod domains come from the strict requirements (no preference): a preferred term on a topology key of the input is
    refused rather than mis-scheduled (KP_E_UNSUPPORTED, shared with the device build)."""
    c = PC.schedule_anyway_spread_respected(fx)
    c.problem.classes[0].preferred_terms = [(5, [model.Requirement(model.HOSTNAME, "Exists")])]
    with pytest.raises(RuntimeError, match="7"):
        run_oracle(c)
