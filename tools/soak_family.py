"""GPU box: one tools/soak.py family over a seed range, with a fresh Context per seed (fresh) or one reused across
seeds (the soak's way), to tell a decision difference from state left behind by an earlier solve.
Usage: python tools/soak_family.py <family> <first> <last> [fresh]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.argv, args = [sys.argv[0], "0"], sys.argv[1:]
import soak  # noqa: E402  (runs nothing with 0 seeds)
from kpsim import abi, native  # noqa: E402

fam, lo, hi = args[0], int(args[1]), int(args[2])
fresh = len(args) > 3
fn = getattr(soak, "fam_" + fam)
bad = []
for seed in range(lo, hi):
    if fresh:
        for p in list(soak.pctx):
            soak.pctx[p].close()
            soak.pctx[p] = native.Context(0, preference_policy=p)
    try:
        fn(seed)
    except native.KpError as e:
        if e.status != abi.KP_E_UNSUPPORTED:
            bad.append(seed)
    except AssertionError:
        bad.append(seed)
print(fam, lo, hi, "fresh" if fresh else "reused", "mismatches", bad, flush=True)
