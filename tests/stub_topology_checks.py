"""Run by tests/test_topology_host_cpu.py in a child process with KPSIM_LIB = the host layer over the CPU stub
(tests/cpu_stub build/libkpsim_stub.so): kp_solve_prepare / kp_consolidate_prepare's topology build decides, without a
GPU, which inputs it accepts.  Prints one JSON object: case → "ok" or the KP status name and message."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "karpenter-provider-aws_amd"), HERE, os.path.join(HERE, "..", "oracle")]

import numpy as np  # noqa: E402

import cons_cases  # noqa: E402
import fuzzgen  # noqa: E402
import test_topology_cpu as TC  # noqa: E402
from kpsim import abi, catalog, model, native  # noqa: E402


def main():
    golden = catalog.golden_catalog(fx=catalog.load_fixtures())
    ctx = native.Context(0)
    out = {}

    def run(name, fn):
        try:
            fn()
            out[name] = "ok"
        except native.KpError as e:
            out[name] = str(e)

    def solve_prep(prob):
        ctx.upload_catalog(model.CatalogView(prob.catalog))
        ctx.prepare(model.SolveInputView(prob))

    def cons_prep(cp):
        ctx.upload_catalog(model.CatalogView(cp.cluster.catalog))
        ctx.consolidate_prepare(model.ConsolidateInputView(cp, abi.KP_CONSOLIDATE_SINGLE))

    for a_first in (True, False):
        run("filter_%s" % a_first, lambda: solve_prep(TC.shared_filter_problem(golden, a_first)))
        run("min_domains_%s" % a_first, lambda: solve_prep(TC.shared_min_domains_problem(golden, a_first)))
    for a_big in (True, False):
        run("relaxed_only_%s" % a_big, lambda: solve_prep(TC.relaxed_only_shared_problem(golden, a_big)))
    for seed in range(int(sys.argv[1]) if len(sys.argv) > 1 else 8):
        rng = np.random.Generator(np.random.PCG64(seed + 500))
        sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=160, replace=False))]
        prob = fuzzgen.fuzz_shared_identity_problem(sub, seed, n_pods=int(rng.integers(80, 300)),
                                                    n_existing=(seed % 2) * 20)
        run("fuzz_%d" % seed, lambda: solve_prep(prob))
    for pend in (True, False):
        run("cons_pending_%s" % pend, lambda: cons_prep(cons_cases.shared_identity_cluster(golden, pend)))
    run("cons_selection", lambda: cons_prep(cons_cases.shared_identity_cluster(golden, False, selection=True)))
    for seed in range(4):
        rng = np.random.Generator(np.random.PCG64(4500 + seed))
        sub = [golden[int(i)] for i in sorted(rng.choice(len(golden), size=int(rng.integers(60, 300)), replace=False))]
        cp = fuzzgen.fuzz_shared_identity_consolidation(sub, 4500 + seed, n_nodes=int(rng.integers(4, 50)),
                                                        n_pods=int(rng.integers(20, 200)), pending_owner=seed % 2 == 0)
        run("cons_fuzz_%d" % seed, lambda: cons_prep(cp))
    # reserved offerings: one type with 70 reservations (its rows exceed one 64-row ResvTab word) and more than
    # KP_MAX_RO in all are refused with their own reasons
    import copy
    from kpsim import synth
    cat = copy.deepcopy(golden)
    for i in range(70):
        cons_cases.add_reservation(cat, "m5.large", "cr-p%03d" % i)
    run("resv_per_type_70", lambda: solve_prep(synth.config2(n_pods=50, catalog=cat)))
    wide = synth.wide_reservation_catalog(golden, 1100, max_per_type=4)
    run("resv_over_max", lambda: solve_prep(synth.config2(n_pods=50, catalog=wide)))
    # reservation-ID selections over more than 64 reservations: accepted (KF_RESV_ROWS); minValues on the key refused
    cat200 = synth.wide_reservation_catalog(golden, 200)
    prob = synth.config5(n_pods=300, catalog=cat200)
    fuzzgen.add_reservation_id_requirements(np.random.Generator(np.random.PCG64(5)), prob, p_class=1.0, p_pool=1.0)
    run("resv_id_selection", lambda: solve_prep(prob))
    prob2 = synth.config5(n_pods=300, catalog=cat200)
    prob2.nodepools[0].requirements = list(prob2.nodepools[0].requirements) + [
        model.Requirement(model.RESERVATION_ID, "Exists", [], 2)]
    run("resv_id_min_values", lambda: solve_prep(prob2))
    ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
