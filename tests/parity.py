"""Helpers: run a problem on the device and on the CPU oracle and compare outputs exactly."""
import numpy as np

import pyoracle
from kpsim import model


def run_device(ctx, prob, catalog_view=None):
    cv = catalog_view or model.CatalogView(prob.catalog)
    ctx.upload_catalog(cv)
    iv = model.SolveInputView(prob)
    cap_nc = max(16, prob.pods.n + 1)
    m = prob.max_instance_types if prob.max_instance_types > 0 else len(prob.catalog)
    out = model.OutputBuffers(prob.pods.n, cap_nc, cap_nc * m)
    ctx.solve(iv, out)
    r = out.results()
    reqs = [model.parse_requirements_blob(ctx.nodeclaim_requirements(i)) for i in range(r.n_nodeclaims)]
    return r, reqs


def run_oracle(prob, catalog_view=None):
    o = pyoracle.solve(prob, catalog_view)
    r = o.results
    reqs = [model.parse_requirements_blob(o.requirements(i)) for i in range(r.n_nodeclaims)]
    return r, reqs


def assert_same(dev, orc, check_reqs=True):
    rd, qd = dev
    ro, qo = orc
    assert rd.n_nodeclaims == ro.n_nodeclaims, (rd.n_nodeclaims, ro.n_nodeclaims)
    np.testing.assert_array_equal(rd.pod_result, ro.pod_result)
    np.testing.assert_array_equal(rd.pod_order, ro.pod_order)
    np.testing.assert_array_equal(rd.nodeclaim_nodepool, ro.nodeclaim_nodepool)
    np.testing.assert_array_equal(rd.nodeclaim_n_pods, ro.nodeclaim_n_pods)
    np.testing.assert_array_equal(rd.nodeclaim_slice_pos, ro.nodeclaim_slice_pos)
    np.testing.assert_array_equal(rd.nodeclaim_n_options, ro.nodeclaim_n_options)
    for i in range(rd.n_nodeclaims):
        assert rd.nodeclaim_types[i] == ro.nodeclaim_types[i], i
    if check_reqs:
        for i in range(rd.n_nodeclaims):
            assert qd[i] == qo[i], (i, qd[i], qo[i])


def result_digest(res):
    """sha256 per output field of a Solve result ((Results, requirements) as returned by run_device / run_oracle), so
    a full-size oracle run can be committed as a small fixture (tests/golden/gen_scale_digest.py)."""
    import hashlib
    r, q = res
    h = lambda b: hashlib.sha256(b).hexdigest()  # noqa: E731
    return {
        "n_nodeclaims": int(r.n_nodeclaims),
        "pod_result": h(np.ascontiguousarray(r.pod_result, np.int64).tobytes()),
        "pod_order": h(np.ascontiguousarray(r.pod_order, np.int64).tobytes()),
        "nodeclaim_nodepool": h(np.ascontiguousarray(r.nodeclaim_nodepool, np.int64).tobytes()),
        "nodeclaim_n_pods": h(np.ascontiguousarray(r.nodeclaim_n_pods, np.int64).tobytes()),
        "nodeclaim_slice_pos": h(np.ascontiguousarray(r.nodeclaim_slice_pos, np.int64).tobytes()),
        "nodeclaim_n_options": h(np.ascontiguousarray(r.nodeclaim_n_options, np.int64).tobytes()),
        "nodeclaim_types": h(repr([list(map(int, r.nodeclaim_types[i])) for i in range(r.n_nodeclaims)]).encode()),
        "requirements": h(repr(q).encode()),
    }
