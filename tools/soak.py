"""GPU box: parity soak over many more seeds than the -m gpu suite runs — device vs oracle on the round's new shapes
(wide reservation catalogs, preference / topology interplay, relaxing topology, many groups, mutating consolidation,
shared topology identities).
Prints one line per family: seeds run, mismatches (the first failing seeds).  Usage: python tools/soak.py [seeds]"""
import os
import sys
import time
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("karpenter-provider-aws_amd", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))

import numpy as np  # noqa: E402

import fuzzgen  # noqa: E402
import parity  # noqa: E402
import pyoracle  # noqa: E402
from kpsim import abi, catalog, model, native, synth  # noqa: E402
from test_gpu_consolidation import (assert_commands_equal, assert_probes_equal, device_command, device_probes,  # noqa: E402
                                    hostname_pod_domains_consolidation)

N = int(sys.argv[1]) if len(sys.argv) > 1 else 40
REFUSED = []
g = catalog.golden_catalog()
ctx = native.Context(0)
pctx = {p: native.Context(0, preference_policy=p) for p in (abi.KP_PREFERENCE_RESPECT, abi.KP_PREFERENCE_IGNORE)}


def solve_case(prob, policy=abi.KP_PREFERENCE_RESPECT):
    c = pctx[policy]
    dev = parity.run_device(c, prob)
    o = pyoracle.solve(prob, preference_policy=policy)
    parity.assert_same(dev, (o.results, [model.parse_requirements_blob(o.requirements(i)) for i in range(o.results.n_nodeclaims)]))


def fam_wide_resv(seed):
    rng = np.random.Generator(np.random.PCG64(9100 + seed))
    cat = synth.wide_reservation_catalog(g, int(rng.choice([65, 128, 300, 700])), max_per_type=int(rng.integers(1, 6)),
                                         seed=synth.SEED + 100 + seed, expiring_frac=0.2, rcap=(0, 4))
    for it in cat:
        for o in it.offerings:
            if o.capacity_type == "reserved":
                o.available = o.available and o.reservation_capacity > 0
    prob = synth.config2(n_pods=int(rng.integers(500, 3000)), n_classes=60, catalog=cat, seed=synth.SEED + 100 + seed)
    cts = [["reserved"], ["reserved", "on-demand"], ["reserved", "spot", "on-demand"], ["spot", "on-demand"]]
    for np_ in prob.nodepools:
        np_.requirements = [r for r in np_.requirements if r.key != model.CAPACITY_TYPE]
        np_.requirements.append(model.Requirement(model.CAPACITY_TYPE, "In", cts[int(rng.integers(len(cts)))]))
    solve_case(prob)


def fam_topo_pref(seed):
    rng = np.random.Generator(np.random.PCG64(9300 + seed))
    sub = [g[int(i)] for i in sorted(rng.choice(len(g), size=int(rng.integers(80, 300)), replace=False))]
    prob = fuzzgen.fuzz_topology_existing_problem(sub, 9300 + seed, n_pods=int(rng.integers(100, 400)))
    fuzzgen.add_topology_preferences(rng, prob)
    for pol in (abi.KP_PREFERENCE_RESPECT, abi.KP_PREFERENCE_IGNORE):
        solve_case(prob, pol)


def fam_relaxing(seed):
    rng = np.random.Generator(np.random.PCG64(9600 + seed))
    sub = [g[int(i)] for i in sorted(rng.choice(len(g), size=int(rng.integers(80, 300)), replace=False))]
    prob = fuzzgen.fuzz_topology_existing_problem(sub, 9600 + seed, n_pods=int(rng.integers(100, 400)))
    fuzzgen.add_relaxing_topology(rng, prob)
    for pol in (abi.KP_PREFERENCE_RESPECT, abi.KP_PREFERENCE_IGNORE):
        solve_case(prob, pol)


def fam_many_groups(seed):
    rng = np.random.Generator(np.random.PCG64(9800 + seed))
    sub = [g[int(i)] for i in sorted(rng.choice(len(g), size=200, replace=False))]
    prob = fuzzgen.fuzz_topology_existing_problem(sub, 9800 + seed, n_pods=int(rng.integers(100, 400)),
                                                  n_existing=int(rng.integers(4, 40)))
    fuzzgen.add_many_groups(rng, prob, n_terms=int(rng.integers(10, 18)))
    try:
        solve_case(prob)
    except native.KpError as e:
        if e.status != abi.KP_E_UNSUPPORTED:
            raise
        REFUSED.append(seed)  # more than 16 constraining / 64 counting groups: refused by design


def fam_cons_mut_topo(seed):
    rng = np.random.Generator(np.random.PCG64(9900 + seed))
    sub = [g[int(i)] for i in sorted(rng.choice(len(g), size=int(rng.integers(60, 300)), replace=False))]
    cp = fuzzgen.fuzz_topology_consolidation(sub, 9900 + seed, n_nodes=int(rng.integers(4, 50)),
                                             n_pods=int(rng.integers(20, 200)), all_spot=seed % 4 == 0)
    fuzzgen.add_mutators(rng, cp, g)
    if seed % 2:
        fuzzgen.add_relaxing_topology(rng, cp.cluster)
    c = pctx[abi.KP_PREFERENCE_RESPECT]
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(c, cp, mode),
                            pyoracle.consolidate(cp, mode, preference_policy=abi.KP_PREFERENCE_RESPECT))


def fam_cons_wide_resv(seed):
    rng = np.random.Generator(np.random.PCG64(9950 + seed))
    sub = [g[int(i)] for i in sorted(rng.choice(len(g), size=int(rng.integers(120, 300)), replace=False))]
    cat = synth.wide_reservation_catalog(sub, int(rng.integers(65, 260)), max_per_type=4, seed=9950 + seed, rcap=(0, 6))
    cp = fuzzgen.fuzz_consolidation(cat, 9950 + seed, n_nodes=int(rng.integers(4, 60)), n_pods=int(rng.integers(20, 250)),
                                    all_spot=seed % 4 == 0, pending_frac=0.15)
    for np_ in cp.cluster.nodepools:
        for r in np_.requirements:
            if r.key == model.CAPACITY_TYPE and r.op == "In":
                r.values = sorted(set(r.values) | {"reserved"})
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode), pyoracle.consolidate(cp, mode))


def fam_cons_host_domains(seed):
    cp = hostname_pod_domains_consolidation(g, 1000 + seed)
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(ctx, cp, mode), pyoracle.consolidate(cp, mode))
    assert_commands_equal(device_command(ctx, cp, abi.KP_CONSOLIDATE_BOTH),
                          pyoracle.consolidate_command(cp, abi.KP_CONSOLIDATE_BOTH))


def fam_shared_solve(seed):
    rng = np.random.Generator(np.random.PCG64(10100 + seed))
    sub = [g[int(i)] for i in sorted(rng.choice(len(g), size=int(rng.integers(80, 300)), replace=False))]
    prob = fuzzgen.fuzz_shared_identity_problem(sub, 10100 + seed, n_pods=int(rng.integers(80, 400)),
                                                n_existing=(seed % 2) * int(rng.integers(4, 40)))
    if seed % 3 == 0:
        fuzzgen.add_relaxed_shared(rng, prob)
    for pol in (abi.KP_PREFERENCE_RESPECT, abi.KP_PREFERENCE_IGNORE):
        solve_case(prob, pol)


def fam_shared_cons(seed):
    rng = np.random.Generator(np.random.PCG64(10300 + seed))
    sub = [g[int(i)] for i in sorted(rng.choice(len(g), size=int(rng.integers(60, 300)), replace=False))]
    cp = fuzzgen.fuzz_shared_identity_consolidation(sub, 10300 + seed, n_nodes=int(rng.integers(4, 50)),
                                                    n_pods=int(rng.integers(20, 200)), pending_owner=seed % 2 == 0)
    if seed % 3 == 0:
        fuzzgen.add_relaxed_shared(rng, cp.cluster)
    c = pctx[abi.KP_PREFERENCE_RESPECT]
    for mode in (abi.KP_CONSOLIDATE_SINGLE, abi.KP_CONSOLIDATE_MULTI):
        assert_probes_equal(device_probes(c, cp, mode),
                            pyoracle.consolidate(cp, mode, preference_policy=abi.KP_PREFERENCE_RESPECT))


FAMILIES = [("wide reservations (Solve)", fam_wide_resv), ("topology x preferences (Solve, 2 policies)", fam_topo_pref),
            ("relaxing topology (Solve, 2 policies)", fam_relaxing), ("many groups (Solve)", fam_many_groups),
            ("mutators x topology (consolidation)", fam_cons_mut_topo),
            ("wide reservations (consolidation)", fam_cons_wide_resv),
            ("hostname podDomains (consolidation)", fam_cons_host_domains),
            ("shared topology identities (Solve, 2 policies)", fam_shared_solve),
            ("shared topology identities (consolidation)", fam_shared_cons)]

if __name__ == "__main__":
    only = os.environ.get("SOAK_FAMILIES")  # comma-separated substrings of family names
    for name, fn in FAMILIES:
        if only and not any(x in name for x in only.split(",")):
            continue
        t = time.time()
        bad = []
        for seed in range(N):
            try:
                fn(seed)
            except Exception:
                bad.append(seed)
                if len(bad) == 1:
                    traceback.print_exc(limit=3, file=sys.stderr)
        print("%-45s seeds %d, mismatches %d %s, refused %d (%.0f s)" % (name, N, len(bad), bad[:8], len(REFUSED),
                                                                        time.time() - t), flush=True)
        REFUSED.clear()
