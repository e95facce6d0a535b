import sys, time, os
sys.path[:0] = ["karpenter-provider-aws_amd", "oracle", "tests"]
from kpsim import catalog, model, native, synth
g = catalog.golden_catalog()
c5 = synth.config5_catalog(g)
ctx = native.Context(0)
ctx.upload_catalog(model.CatalogView(c5))
for n in (50000, 100000, 200000):
    p = synth.config5(n_pods=n, catalog=c5)
    iv = model.SolveInputView(p)
    out = model.OutputBuffers(p.pods.n, p.pods.n + 16, (p.pods.n + 16) * 60)
    t = time.time(); ctx.solve(iv, out); dt = time.time() - t
    r = out.results()
    print(n, "%.1f ms" % (dt * 1e3), ctx.kernel_times_ms(), r.n_nodeclaims, int((r.pod_result == -1).sum()), r.stats["nodeclaim_evals"], flush=True)
