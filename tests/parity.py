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
