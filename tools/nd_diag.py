"""GPU box diagnostics: node-dense Deployments around the first slice plan (KP_NC_FIRST)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "karpenter-provider-aws_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import parity  # noqa: E402
import test_topology_cpu as TC  # noqa: E402
from kpsim import catalog, native  # noqa: E402

cat = catalog.golden_catalog()
for n in [int(x) for x in sys.argv[1:]]:
    c = native.Context(0)
    try:
        r, _ = parity.run_device(c, TC.node_dense(cat, n))
        print(n, "nodeclaims", r.n_nodeclaims, "unschedulable", int((r.pod_result == -1).sum()), r.stats, flush=True)
    except Exception as e:  # noqa: BLE001
        print(n, "error", e, flush=True)
    finally:
        c.close()
