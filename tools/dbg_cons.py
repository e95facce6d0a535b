import sys, os
sys.path[:0] = ['karpenter-provider-aws_amd', 'oracle', 'tests']
import numpy as np, fuzzgen, pyoracle
from kpsim import catalog, abi, model, native
gold = catalog.golden_catalog()
seed = int(sys.argv[1]); mode = int(sys.argv[2])
rng = np.random.Generator(np.random.PCG64(500 + seed))
sub = [gold[int(i)] for i in sorted(rng.choice(len(gold), size=int(rng.integers(60, 300)), replace=False))]
cp = fuzzgen.fuzz_consolidation(sub, 500 + seed, n_nodes=int(rng.integers(4, 80)), n_pods=int(rng.integers(20, 300)), all_spot=seed % 4 == 0, supported=True)
print("nodes", len(cp.cluster.existing), "pods", cp.cluster.pods.n, "cands", len(cp.candidates), "pending", len(cp.pending), flush=True)
ctx = native.Context(0)
ctx.upload_catalog(model.CatalogView(cp.cluster.catalog))
r = ctx.consolidate(model.ConsolidateInputView(cp, mode, 0, 0, seed % 2 == 0))
print("done", r[:5], ctx.consolidate_stats(), flush=True)
