"""GPU box: shrink a failing soak case (tools/soak.py family + seed) to a small problem that still mismatches — greedy
delta debugging over pods, existing nodes, bound pods, topology / preferred / required terms and classes — then
print it and pickle it (our own dataclasses) under gpurun_out/ for host-side study.
Usage: python tools/soak_min.py <family> <seed> [policy]  |  <case.pkl> 0 [policy]"""
import copy
import os
import pickle
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("karpenter-provider-aws_amd", "tests", "oracle", "tools"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np  # noqa: E402

import fuzzgen  # noqa: E402
import parity  # noqa: E402
import pyoracle  # noqa: E402
from kpsim import abi, catalog, model, native  # noqa: E402

g = catalog.golden_catalog()


def mk_topo_pref(seed):
    rng = np.random.Generator(np.random.PCG64(9300 + seed))
    sub = [g[int(i)] for i in sorted(rng.choice(len(g), size=int(rng.integers(80, 300)), replace=False))]
    prob = fuzzgen.fuzz_topology_existing_problem(sub, 9300 + seed, n_pods=int(rng.integers(100, 400)))
    fuzzgen.add_topology_preferences(rng, prob)
    return prob


def mk_many_groups(seed):
    rng = np.random.Generator(np.random.PCG64(9800 + seed))
    sub = [g[int(i)] for i in sorted(rng.choice(len(g), size=200, replace=False))]
    prob = fuzzgen.fuzz_topology_existing_problem(sub, 9800 + seed, n_pods=int(rng.integers(100, 400)),
                                                  n_existing=int(rng.integers(4, 40)))
    fuzzgen.add_many_groups(rng, prob, n_terms=int(rng.integers(10, 18)))
    return prob


fam, seed = sys.argv[1], int(sys.argv[2])
policy = int(sys.argv[3]) if len(sys.argv) > 3 else abi.KP_PREFERENCE_RESPECT
if fam.endswith(".pkl"):  # a pickled case (an earlier minimisation)
    prob0 = pickle.load(open(fam, "rb"))
    fam = os.path.basename(fam)[:-4]
else:
    prob0 = {"topo_pref": mk_topo_pref, "many_groups": mk_many_groups}[fam](seed)
ctx = native.Context(0, preference_policy=policy)
NCALL = [0]


def outcome(prob):
    NCALL[0] += 1
    try:
        dev = parity.run_device(ctx, prob)
    except Exception:
        return None
    try:
        o = pyoracle.solve(prob, preference_policy=policy)
    except Exception:
        return None
    orc = (o.results, [model.parse_requirements_blob(o.requirements(i)) for i in range(o.results.n_nodeclaims)])
    return dev, orc


def bad(prob):
    r = outcome(prob)
    if r is None:
        return False
    try:
        parity.assert_same(*r)
    except AssertionError:
        return True
    return False


def keep_pods(prob, keep):
    p = copy.copy(prob)
    keep = np.asarray(sorted(keep), dtype=np.int64)
    P = prob.pods
    p.pods = model.Pods(P.class_id[keep].copy(), P.requests[keep].copy(), P.creation_ns[keep].copy(),
                        [P.uids[i] for i in keep])
    return p


def keep_existing(prob, keep):
    p = copy.copy(prob)
    keep = sorted(keep)
    remap = {e: i for i, e in enumerate(keep)}
    p.existing = [prob.existing[e] for e in keep]
    p.bound = [(remap[b[0]],) + tuple(b[1:]) for b in prob.bound if b[0] in remap]
    return p


def keep_bound(prob, keep):
    p = copy.copy(prob)
    p.bound = [prob.bound[i] for i in sorted(keep)]
    return p


def ddmin(prob, n, apply, what):
    """greedy chunk removal over n items; apply(prob, kept indices) -> problem"""
    base = prob
    items = list(range(n))
    chunk = max(1, len(items) // 2)
    while chunk >= 1 and items:
        i = 0
        progressed = False
        while i < len(items):
            trial = items[:i] + items[i + chunk:]
            cand = apply(base, trial)
            if bad(cand):
                items = trial
                prob = cand
                progressed = True
            else:
                i += chunk
        if not progressed:
            chunk //= 2
    print("  %s: %d -> %d" % (what, n, len(items)), flush=True)
    return prob


def shrink_class_lists(prob):
    """drop topology / preferred / required terms one at a time"""
    for attr in ("topology", "preferred_terms", "required_terms"):
        for ci in range(len(prob.classes)):
            j = 0
            while j < len(getattr(prob.classes[ci], attr)):
                cand = copy.deepcopy(prob)
                lst = getattr(cand.classes[ci], attr)
                del lst[j]
                if bad(cand):
                    prob = cand
                else:
                    j += 1
    return prob


def drop_unused_classes(prob):
    used = sorted(set(int(c) for c in prob.pods.class_id) | set(int(b[1]) for b in prob.bound))
    remap = {c: i for i, c in enumerate(used)}
    cand = copy.copy(prob)
    cand.classes = [prob.classes[c] for c in used]
    P = prob.pods
    cand.pods = model.Pods(np.asarray([remap[int(c)] for c in P.class_id], np.int32), P.requests, P.creation_ns, P.uids)
    cand.bound = [(b[0], remap[int(b[1])]) + tuple(b[2:]) for b in prob.bound]
    return cand if bad(cand) else prob


assert bad(prob0), "the case does not mismatch here"
prob = prob0
for rnd in range(3):
    before = (prob.pods.n, len(prob.existing), len(prob.bound))
    prob = ddmin(prob, prob.pods.n, keep_pods, "pods")
    prob = ddmin(prob, len(prob.existing), keep_existing, "existing")
    prob = ddmin(prob, len(prob.bound), keep_bound, "bound")
    prob = shrink_class_lists(prob)
    prob = drop_unused_classes(prob)
    if (prob.pods.n, len(prob.existing), len(prob.bound)) == before:
        break
print("solves", NCALL[0], flush=True)

dev, orc = outcome(prob)
print("pods", prob.pods.n, "existing", len(prob.existing), "bound", prob.bound, flush=True)
print("dev pod_result", list(dev[0].pod_result), "\norc pod_result", list(orc[0].pod_result))
print("dev order", list(dev[0].pod_order), "\norc order", list(orc[0].pod_order))
try:
    parity.assert_same(dev, orc)
except AssertionError as e:
    print("assert:", str(e)[:1500])
for i, pc in enumerate(prob.classes):
    print("class", i, "ns", pc.namespace, "labels", pc.labels, "reqs", [(r.key.split('/')[-1], r.op, r.values) for r in pc.requirements])
    for t in pc.topology:
        print("   term", t.kind, t.key.split('/')[-1], "sel", [(r.key, r.op, r.values) for r in (t.selector or [])],
              "ns", t.namespaces, "skew", t.max_skew, "mind", t.min_domains, t.when_unsatisfiable,
              t.node_affinity_policy, t.node_taints_policy, "w", t.weight)
    for w, tr in pc.preferred_terms:
        print("   pref", w, [(r.key.split('/')[-1], r.op, r.values) for r in tr])
    for tr in pc.required_terms:
        print("   reqterm", [(r.key.split('/')[-1], r.op, r.values) for r in tr])
print("pods class", list(prob.pods.class_id), "requests", prob.pods.requests.tolist())
for e in prob.existing:
    print("existing", e.name, {k.split('/')[-1]: v for k, v in e.labels.items()}, "avail", e.available.tolist(),
          "taints", [(t.key, t.effect) for t in e.taints])
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", "min_%s_%d.pkl" % (fam, seed)), "wb") as f:
    pickle.dump(prob, f)
