"""GPU box: re-run failing soak seeds (tools/soak.py) with details: the mismatching pods, their classes and the
class features (topology terms, preferred terms, Honor policies), under the in-tree library and KPSIM_LIB overrides."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("karpenter-provider-aws_amd", "tests", "oracle", "tools"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np  # noqa: E402

import fuzzgen  # noqa: E402
import parity  # noqa: E402
import pyoracle  # noqa: E402
from kpsim import abi, catalog, model, native  # noqa: E402

g = catalog.golden_catalog()


def topo_pref(seed):
    rng = np.random.Generator(np.random.PCG64(9300 + seed))
    sub = [g[int(i)] for i in sorted(rng.choice(len(g), size=int(rng.integers(80, 300)), replace=False))]
    prob = fuzzgen.fuzz_topology_existing_problem(sub, 9300 + seed, n_pods=int(rng.integers(100, 400)))
    fuzzgen.add_topology_preferences(rng, prob)
    return prob


def many(seed):
    rng = np.random.Generator(np.random.PCG64(9800 + seed))
    sub = [g[int(i)] for i in sorted(rng.choice(len(g), size=200, replace=False))]
    prob = fuzzgen.fuzz_topology_existing_problem(sub, 9800 + seed, n_pods=int(rng.integers(100, 400)),
                                                  n_existing=int(rng.integers(4, 40)))
    fuzzgen.add_many_groups(rng, prob, n_terms=int(rng.integers(10, 18)))
    return prob


for name, mk, seeds in (("topo_pref", topo_pref, [58, 233]), ("many", many, [172, 199])):
    for seed in seeds:
        prob = mk(seed)
        for pol in (abi.KP_PREFERENCE_RESPECT, abi.KP_PREFERENCE_IGNORE):
            c = native.Context(0, preference_policy=pol)
            dev = parity.run_device(c, prob)
            c.close()
            o = pyoracle.solve(prob, preference_policy=pol)
            dr, orr = dev[0].pod_result, o.results.pod_result
            bad = np.nonzero(dr != orr)[0]
            print(name, seed, "policy", pol, "mismatching pods", len(bad), flush=True)
            for p in bad[:6]:
                ci = int(prob.pods.class_id[p])
                pc = prob.classes[ci]
                print("  pod %d class %d dev %d orc %d | pref %d terms %s" % (
                    p, ci, dr[p], orr[p], len(pc.preferred_terms),
                    [(t.kind, t.key.split('/')[-1], t.node_affinity_policy, t.node_taints_policy, t.max_skew,
                      t.min_domains, t.when_unsatisfiable, t.weight) for t in pc.topology]))
