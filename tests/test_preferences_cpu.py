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
