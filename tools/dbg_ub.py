"""Development tool: locate the first pod whose placement differs between the device and the oracle."""
import sys
sys.path[:0] = ["karpenter-provider-aws_amd", "oracle", "tests"]
import numpy as np
import parity
from kpsim import catalog, native, synth

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
cat = catalog.golden_catalog(fx=catalog.load_fixtures())
prob = synth.subsample(synth.config2(catalog=cat), n)
ctx = native.Context(0)
rd = parity.run_device(ctx, prob)[0]
ro = parity.run_oracle(prob)[0]
print("nodeclaims dev/oracle", rd.n_nodeclaims, ro.n_nodeclaims)
key = lambda r: np.argsort(np.where(r.pod_order < 0, 1 << 30, r.pod_order), kind="stable")
od, oo = key(rd), key(ro)
for i in range(len(od)):
    if od[i] != oo[i] or rd.pod_result[od[i]] != ro.pod_result[oo[i]]:
        lo = max(0, i - 6)
        print("first divergence at seq", i)
        for j in range(lo, min(len(od), i + 4)):
            pd, po = od[j], oo[j]
            print("  seq %5d  dev pod %5d cls %3d -> nc %3d | oracle pod %5d cls %3d -> nc %3d" % (
                j, pd, prob.pods.class_id[pd], rd.pod_result[pd], po, prob.pods.class_id[po], ro.pod_result[po]))
        break
print("dev nc pods", list(rd.nodeclaim_n_pods[:40]))
print("orc nc pods", list(ro.nodeclaim_n_pods[:40]))
