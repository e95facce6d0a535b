#!/usr/bin/env python3
"""Device vs oracle divergence finder for one Solve (GPU box): the first pod, in the oracle's placement order, whose
placement differs, with the NodeClaims involved.   python tools/diff_solve.py config5 20000 [seed]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "karpenter-provider-aws_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

from kpsim import catalog, model, native, synth  # noqa: E402
import parity  # noqa: E402


def build(which, n, golden):
    if which == "config5":
        return synth.config5(n_pods=n, golden=golden)
    if which == "scarce":
        from test_gpu_reserved import scarce_problem
        return scarce_problem(golden, n)
    return getattr(synth, which)(n_pods=n, catalog=golden)


def main():
    which = sys.argv[1]
    sizes = [int(x) for x in sys.argv[2].split(",")]
    golden = catalog.golden_catalog()
    ctx = native.Context(0)
    for n in sizes:
        prob = build(which, n, golden)
        cv = model.CatalogView(prob.catalog)
        (rd, qd) = parity.run_device(ctx, prob, cv)
        (ro, qo) = parity.run_oracle(prob, cv)
        same = rd.n_nodeclaims == ro.n_nodeclaims and (rd.pod_result == ro.pod_result).all() and \
            (rd.pod_order == ro.pod_order).all()
        print("n=%d device ncs=%d oracle ncs=%d same=%s" % (n, rd.n_nodeclaims, ro.n_nodeclaims, same), flush=True)
        if same:
            continue
        order = np.argsort(np.where(ro.pod_order >= 0, ro.pod_order, 1 << 30), kind="stable")
        for k, p in enumerate(order):
            if rd.pod_result[p] != ro.pod_result[p] or rd.pod_order[p] != ro.pod_order[p]:
                c = int(prob.pods.class_id[p])
                print(" first diff at oracle step %d: pod %d class %d req %s" % (k, p, c, prob.pods.requests[p][:3].tolist()))
                print("  device nc=%d order=%d   oracle nc=%d order=%d" % (rd.pod_result[p], rd.pod_order[p],
                                                                           ro.pod_result[p], ro.pod_order[p]))
                print("  class reqs", [(r.key, r.op, r.values) for r in prob.classes[c].requirements])
                for lab, r, q, nc in (("dev", rd, qd, int(rd.pod_result[p])), ("orc", ro, qo, int(ro.pod_result[p]))):
                    for m in {nc, int((ro if lab == "dev" else rd).pod_result[p])}:
                        if 0 <= m < r.n_nodeclaims:
                            print("  %s nc %d: np=%d npods=%d nopts=%d resv=%s ct=%s" % (
                                lab, m, r.nodeclaim_nodepool[m], r.nodeclaim_n_pods[m], r.nodeclaim_n_options[m],
                                q[m].get("karpenter.k8s.aws/capacity-reservation-id"), q[m].get("karpenter.sh/capacity-type")))
                # pods placed before this step on either side that differ
                break
        break
    ctx.close()


if __name__ == "__main__":
    main()
