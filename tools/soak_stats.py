"""GPU box: device vs oracle stats and slice positions for a pickled minimized case (tools/soak_min.py output)."""
import os
import pickle
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("karpenter-provider-aws_amd", "tests", "oracle", "tools"):
    sys.path.insert(0, os.path.join(ROOT, p))
import parity  # noqa: E402
import pyoracle  # noqa: E402
from kpsim import native  # noqa: E402

for path in sys.argv[1:]:
    prob = pickle.load(open(path, "rb"))
    ctx = native.Context(0)
    dev = parity.run_device(ctx, prob)
    o = pyoracle.solve(prob)
    for name, r in (("dev", dev[0]), ("orc", o.results)):
        print(path, name, "pods", list(map(int, r.pod_result)), "order", list(map(int, r.pod_order)),
              "slice", list(map(int, r.nodeclaim_slice_pos)), "npods", list(map(int, r.nodeclaim_n_pods)))
        print("   ", {k: v for k, v in r.stats.items() if not k.startswith("ns_") and not k.startswith("cyc")})
    ctx.close()
