"""GPU box diagnostics: the consolidation pass split by mode (multi-node prefixes alone, single-node probes alone, both in
one launch) for config 4 and config4-replace, probe kernel ms per mode (KPSIM_PROFILE=1 adds the longest probes)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "karpenter-provider-aws_amd"))
from kpsim import abi, model, native, synth  # noqa: E402

from kpsim import catalog as kcat  # noqa: E402

cat = kcat.golden_catalog(fx=kcat.load_fixtures())
for headroom in (None, 0.02):
    cp = synth.config4(n_nodes=5000, catalog=cat, headroom=headroom)
    n_s = model.consolidation_probe_count(len(cp.candidates), abi.KP_CONSOLIDATE_SINGLE)
    n_m = model.consolidation_probe_count(len(cp.candidates), abi.KP_CONSOLIDATE_MULTI)
    ctx = native.Context(0)
    ctx.upload_catalog(model.CatalogView(cat))
    ctx.consolidate_prepare(model.ConsolidateInputView(cp, abi.KP_CONSOLIDATE_SINGLE))
    for name, mode, n in (("multi", abi.KP_CONSOLIDATE_MULTI, n_m), ("single", abi.KP_CONSOLIDATE_SINGLE, n_s),
                          ("both", abi.KP_CONSOLIDATE_BOTH, n_m + n_s)):
        ks = []
        for _ in range(4):
            ctx.consolidate_execute(mode, n)
            ks.append(ctx.consolidate_stats()[0][1])
        print("headroom", headroom, name, "probe kernel ms", " ".join("%.3f" % x for x in ks[1:]), flush=True)
    ctx.close()
