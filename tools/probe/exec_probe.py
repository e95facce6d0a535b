import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, d) for d in ("karpenter-provider-aws_amd", "tests", "oracle")]
from kpsim import catalog, model, native, synth
g = catalog.golden_catalog()
prob = synth.config2(n_pods=50000, catalog=g)
ctx = native.Context(0)
ctx.upload_catalog(model.CatalogView(g))
iv = model.SolveInputView(prob)
ctx.prepare(iv)
for i in range(4):
    t = time.perf_counter(); ctx.execute(); print("execute %.3f ms" % ((time.perf_counter()-t)*1e3), ctx.kernel_times_ms()[:5], flush=True)
