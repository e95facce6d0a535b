#!/usr/bin/env python3
"""FFD-kernel phase profile of one Solve (KPSIM_PROFILE=1: s_memtime cycle counters inside ffd_kernel).

    KPSIM_PROFILE=1 python tools/prof_solve.py [config2|config3|config5] [n_pods]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "karpenter-provider-aws_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

from kpsim import catalog, model, native, synth  # noqa: E402

NAMES = ["cyc_fast_loop", "cyc_sort", "cyc_slow_eval", "cyc_templates", "-", "cyc_sort_full", "ev_req", "ev_mask",
         "ev_off", "ev_types", "ev_min", "ev_calls", "quick_accepts", "slow_pods", "witness_misses", "cyc_q_pop",
         "cyc_q_scan", "cyc_q_check", "cyc_q_commit", "n_noinv", "n_winmove", "n_ldssort", "n_pivot", "n_winload",
         "n_flush", "n_shape", "n_lds_append", "n_lds_nowin", "n_lds_outside", "n_batches", "topo_quick",
         "cyc_topo_setup", "cyc_topo_scan"]


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "config3"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 50_000
    cat = catalog.golden_catalog()
    if which == "config5":
        cat = synth.config5_catalog(cat)
    prob = getattr(synth, which)(n_pods=n, catalog=cat)
    ctx = native.Context(0)
    ctx.upload_catalog(model.CatalogView(cat))
    iv = model.SolveInputView(prob)
    out = model.OutputBuffers(prob.pods.n, prob.pods.n + 16, (prob.pods.n + 16) * 60)
    import time
    t = time.perf_counter()
    ctx.solve(iv, out)
    wall = (time.perf_counter() - t) * 1e3
    r = out.results()
    kt = ctx.kernel_times_ms()
    print(json.dumps({"config": which, "pods": n, "wall_ms": wall, "kernel_ms": kt, "nodeclaims": r.n_nodeclaims, "stats": r.stats,
                      "ffd": dict(zip(NAMES, ctx.ffd_cycles()))}, indent=1))
    ctx.close()


if __name__ == "__main__":
    main()
