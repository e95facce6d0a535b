#!/usr/bin/env python3
"""Full-size oracle fixtures too slow to recompute inside a GPU test (one to two minutes of single-thread oracle time):
runs the CPU oracle on seeded BASELINE workloads and writes per-field sha256 digests of its Solve output to
tests/golden/scale_digests.json.  tests/test_gpu_parity.py::test_scale_digest and tests/test_gpu_topology.py compare
the device result with them.

    python tests/golden/gen_scale_digest.py [case ...]     (default: every case; others keep their committed digests)
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "karpenter-provider-aws_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

from kpsim import catalog, synth  # noqa: E402
import parity  # noqa: E402

def node_dense(cat, n_pods):
    import test_topology_cpu as TC
    return TC.node_dense(cat, n_pods)


CASES = {
    "config2_200k": ("config2", dict(n_pods=200_000)),  # BASELINE configs[4]'s pod count over the config-2 pod mix
    "config3_50k": ("config3", dict(n_pods=50_000)),    # BASELINE configs[2]: topology + five weighted NodePools
    "config5_200k": ("config5", dict(n_pods=200_000)),  # BASELINE configs[4]: reserved offerings, ODCR-first NodePools
    "node_dense_10k": (node_dense, dict(n_pods=10_000)),  # 10k in-flight NodeClaims
    "node_dense_20k": (node_dense, dict(n_pods=20_000)),  # 20k: beyond the LDS slice (HBM slice arrays), one execute
}


def main():
    cat = catalog.golden_catalog(fx=catalog.load_fixtures())
    path = os.path.join(HERE, "scale_digests.json")
    out = {}
    if os.path.exists(path):
        with open(path) as f:
            out = json.load(f)
    for name in sys.argv[1:] or list(CASES):
        gen, kw = CASES[name]
        if callable(gen):
            prob = gen(cat, **kw)
        else:
            prob = synth.config5(golden=cat, **kw) if gen == "config5" else getattr(synth, gen)(catalog=cat, **kw)
        t = time.time()
        out[name] = dict(kw, **parity.result_digest(parity.run_oracle(prob)))
        print(name, "%.1f s" % (time.time() - t), out[name]["n_nodeclaims"])
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
