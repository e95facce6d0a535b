"""CPU: pin the oracle (and the host catalog builder) to the reference's own golden vectors.

* website/content/en/preview/reference/instance-types.md (927 types; allocatable cpu/memory/pods/ephemeral)
* pkg/providers/instancetype/suite_test.go KATs (overhead, ENI-limited pods, GPU/accelerator packing,
  RAID0 ephemeral storage, pod-ENI, price ordering)
"""
import numpy as np
import pytest

import pyoracle
from kpsim import catalog as cat
from kpsim import model, synth


def _golden_rows(fx):
    return [r for r in fx["golden"] if r["name"] in fx["vpclimits"]]


def test_golden_allocatable_oracle(fx):
    """types.go arithmetic restated in C++ reproduces the golden doc for every type with VPC limits (915)."""
    opts = cat.TypeOptions()
    rows = _golden_rows(fx)
    assert len(rows) == 915
    bad = []
    for row in rows:
        info = cat.golden_info(row, fx["vpclimits"])
        _, _, _, alloc = pyoracle.instance_type_resources(info, opts, fx["vpclimits"])
        for res in ("cpu", "memory", "pods", "ephemeral-storage"):
            if alloc[model.RIDX[res]] != cat.parse_quantity_milli(row["allocatable"][res]):
                bad.append((row["name"], res))
    assert bad == []


def test_golden_allocatable_host_builder(fx):
    opts = cat.TypeOptions()
    for row in _golden_rows(fx):
        info = cat.golden_info(row, fx["vpclimits"])
        capv, kube, ev = cat.instance_resources(info, opts, fx["vpclimits"])
        alloc = capv - kube - ev
        for res in ("cpu", "memory", "pods", "ephemeral-storage"):
            assert alloc[model.RIDX[res]] == cat.parse_quantity_milli(row["allocatable"][res]), (row["name"], res)


def test_kat_overhead_m5_xlarge(fx):
    """suite_test.go:1160-1181 — kube-reserved cpu 80m, memory 893Mi, ephemeral 1Gi."""
    info = next(i for i in fx["fake"]["instance_types"] if i["name"] == "m5.xlarge")
    _, kube, _, _ = pyoracle.instance_type_resources(info, cat.TypeOptions(), fx["vpclimits"])
    k = fx["kats"]["overhead_m5_xlarge"]["kube_reserved"]
    for res, q in k.items():
        assert kube[model.RIDX[res]] == cat.parse_quantity_milli(q), res


def test_kat_eni_limited_pods(fx):
    """suite_test.go:1595-1639 — t3.large 35 pods, m6idn.32xlarge 394 pods."""
    for name, want in fx["kats"]["eni_limited_pods"]["pods"].items():
        info = next(i for i in fx["fake"]["instance_types"] if i["name"] == name)
        capv, _, _, _ = pyoracle.instance_type_resources(info, cat.TypeOptions(), fx["vpclimits"])
        assert capv[model.RIDX["pods"]] == want * 1000


def test_fake_catalog_arithmetic_oracle_vs_builder(fx):
    for raid0 in (False, True):
        opts = cat.TypeOptions(raid0=raid0)
        for info in fx["fake"]["instance_types"]:
            capo, kube, ev, alloc = pyoracle.instance_type_resources(info, opts, fx["vpclimits"])
            capv, kp, evp = cat.instance_resources(info, opts, fx["vpclimits"])
            assert (capo == capv).all() and (alloc == capv - kp - evp).all(), info["name"]


def _packing_problem(fc, case):
    np_ = synth.default_nodepool()
    if "nodepool_instance_type" in case:
        np_.requirements = [model.Requirement(model.INSTANCE_TYPE, "In", [case["nodepool_instance_type"]])]
    pods = synth.pods_from_specs([(0, {case["resource"]: str(q)}) for q in case["requests"]])
    return model.Problem(fc, [np_], [model.PodClass()], pods)


@pytest.mark.parametrize("i", range(7))
def test_kat_gpu_packing_oracle(fx, fake, i):
    """suite_test.go:753-972 — accelerator requests pack onto the expected type / node count."""
    case = fx["kats"]["gpu_packing"]["cases"][i]
    r = pyoracle.solve(_packing_problem(fake, case)).results
    assert r.n_nodeclaims == case["nodes"]
    assert all(fake[ts[0]].name == case["type"] for ts in r.nodeclaim_types)
    assert (r.pod_result >= 0).all()


def test_kat_ephemeral_raid0_oracle(fx):
    """suite_test.go:973-995 — 5000Gi: unschedulable by default, m6idn.32xlarge (7600G) with RAID0."""
    pods = synth.pods_from_specs([(0, {"ephemeral-storage": "5000Gi"})])
    fc = cat.fake_catalog(fx=fx)
    r = pyoracle.solve(model.Problem(fc, [synth.default_nodepool()], [model.PodClass()], pods)).results
    assert (r.pod_result == -1).all()
    fc = cat.fake_catalog(opts=cat.TypeOptions(raid0=True), fx=fx)
    r = pyoracle.solve(model.Problem(fc, [synth.default_nodepool()], [model.PodClass()], pods)).results
    t = r.nodeclaim_types[0][0]
    assert fc[t].name == "m6idn.32xlarge"
    assert fc[t].capacity[model.RIDX["ephemeral-storage"]] == cat.parse_quantity_milli("7600G")


def test_kat_pod_eni_t3_oracle(fake):
    """suite_test.go:395-408 — t3.large advertises no pod-ENI: unschedulable."""
    pods = synth.pods_from_specs([(0, {"vpc.amazonaws.com/pod-eni": "1"})])
    cls = [model.PodClass([model.Requirement(model.INSTANCE_TYPE, "In", ["t3.large"])])]
    r = pyoracle.solve(model.Problem(fake, [synth.default_nodepool()], cls, pods)).results
    assert (r.pod_result == -1).all()


def make_instances_catalog(fx):
    """fake.MakeInstances (pkg/fake/utils.go:185-214): one uniform type per static price, offered in test-zone-1a."""
    infos = []
    for name in fx["prices"]:
        infos.append({"name": name, "usage_classes": ["on-demand", "spot"], "architectures": ["x86_64"], "vcpus": 2,
                      "memory_mib": 8192, "max_enis": 3, "ipv4_per_eni": 10, "default_card": 0, "cards": [3]})
    fxc = dict(fx)
    fxc["fake"] = {"instance_types": infos, "offerings": [[i["name"], "test-zone-1a"] for i in infos]}
    return cat.fake_catalog(fx=fxc)


def test_kat_price_ordering_oracle(fx):
    """suite_test.go:409-453 — the 60 launched types are all among the 100 cheapest by (price, name)."""
    fc = make_instances_catalog(fx)
    pods = synth.pods_from_specs([(0, {"cpu": "1"})])
    r = pyoracle.solve(model.Problem(fc, [synth.default_nodepool()], [model.PodClass()], pods)).results
    ts = r.nodeclaim_types[0]
    assert len(ts) == 60
    od = lambda it: min(o.price for o in it.offerings if o.capacity_type == "on-demand" and o.available)
    ranked = sorted(range(len(fc)), key=lambda t: (od(fc[t]), fc[t].name))
    assert set(ts) <= set(ranked[:100])
    assert ts == ranked[:60]


def test_gosort_restatement_sorts(fx):
    rng = np.random.Generator(np.random.PCG64(7))
    for n in (1, 5, 12, 13, 49, 50, 51, 200, 1000):
        keys = rng.integers(0, 6, size=n)
        perm = np.arange(n, dtype=np.int32)
        out = pyoracle.go_sort_slice_ints(keys, perm)
        assert sorted(out.tolist()) == list(range(n))
        assert (np.diff(keys[out]) >= 0).all()
        # deterministic
        assert (pyoracle.go_sort_slice_ints(keys, perm) == out).all()


def test_scale_digest_fixture_shape():
    """tests/golden/scale_digests.json (oracle digests for the 200k-pod GPU parity test) is complete and well-formed."""
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "scale_digests.json")) as f:
        fx_ = json.load(f)
    want = {"n_pods", "n_nodeclaims", "pod_result", "pod_order", "nodeclaim_nodepool", "nodeclaim_n_pods",
            "nodeclaim_slice_pos", "nodeclaim_n_options", "nodeclaim_types", "requirements"}
    for name, rec in fx_.items():
        assert set(rec) == want, name
        assert rec["n_pods"] >= (10_000 if name.startswith("node_dense") else 50_000) and rec["n_nodeclaims"] > 0
        for k in want - {"n_pods", "n_nodeclaims"}:
            assert len(rec[k]) == 64 and int(rec[k], 16) >= 0


def test_result_digest_deterministic(golden):
    """The digest the 200k fixture relies on is a pure function of the Solve output (two oracle runs agree)."""
    import parity
    prob = synth.config2(n_pods=800, catalog=golden)
    a = parity.result_digest(parity.run_oracle(prob))
    b = parity.result_digest(parity.run_oracle(prob))
    assert a == b and a["n_nodeclaims"] > 0
