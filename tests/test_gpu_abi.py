"""GPU: C-ABI state machine and input edge cases through libkpsim.so (call-order errors, optional fields, several
contexts in one process)."""
import ctypes as C

import numpy as np
import pytest

import parity
from kpsim import abi, model, native, synth

pytestmark = pytest.mark.gpu


def test_failed_catalog_upload_invalidates_prepared_solve(golden):
    """A catalog upload (even one that fails validation) drops every prepared solve: execute and fetch then report
    KP_E_STATE instead of launching kernels over tables of the previous catalog."""
    ctx = native.Context(0)
    try:
        prob = synth.subsample(synth.config2(catalog=golden), 300)
        cv = model.CatalogView(prob.catalog)
        ctx.upload_catalog(cv)
        iv = model.SolveInputView(prob)
        ctx.prepare(iv)
        ctx.execute()
        bad = model.CatalogView(prob.catalog[:10])
        bad.view.offering_type[0] = 10 ** 6  # offering_type out of range → KP_E_INVALID
        with pytest.raises(native.KpError) as e:
            ctx.upload_catalog(bad)
        assert e.value.status == abi.KP_E_INVALID
        with pytest.raises(native.KpError) as e:
            ctx.execute()
        assert e.value.status == abi.KP_E_STATE
        out = model.OutputBuffers(prob.pods.n, prob.pods.n + 16, (prob.pods.n + 16) * 60)
        with pytest.raises(native.KpError) as e:
            ctx.fetch(out)
        assert e.value.status == abi.KP_E_STATE
        # a good upload + prepare recovers
        ctx.upload_catalog(cv)
        ctx.prepare(iv)
        ctx.execute()
        ctx.fetch(out)
    finally:
        ctx.close()


def test_solve_without_uids_matches_oracle(golden):
    """kp_pods_view.uids is optional: NULL means empty UIDs (ties keep input order on both sides)."""
    ctx = native.Context(0)
    try:
        prob = synth.subsample(synth.config2(catalog=golden), 400)
        prob.pods.creation_ns[:] = prob.pods.creation_ns[0]
        cv = model.CatalogView(prob.catalog)
        ctx.upload_catalog(cv)
        iv = model.SolveInputView(prob)
        iv.view.pods.uids = C.cast(None, abi.c_char_pp)
        out = model.OutputBuffers(prob.pods.n, prob.pods.n + 16, (prob.pods.n + 16) * 60)
        ctx.solve(iv, out)
        got = out.results()
        import pyoracle
        ob = model.OutputBuffers(prob.pods.n, prob.pods.n + 16, (prob.pods.n + 16) * 60)
        h = C.c_void_p()
        assert pyoracle.lib().orc_solve(C.byref(cv.view), C.byref(iv.view), C.byref(ob.view), C.byref(h)) == 0
        want = ob.results()
        pyoracle.lib().orc_result_free(h)
        np.testing.assert_array_equal(got.pod_result, want.pod_result)
        np.testing.assert_array_equal(got.pod_order, want.pod_order)
        assert got.nodeclaim_types == want.nodeclaim_types
    finally:
        ctx.close()


def test_two_contexts_one_process(golden):
    """Two contexts in one process (one per caller thread in a controller) give identical results for the same input."""
    a, b = native.Context(0), native.Context(0)
    try:
        prob = synth.subsample(synth.config2(catalog=golden), 500)
        ra = parity.run_device(a, prob)
        rb = parity.run_device(b, prob)
        parity.assert_same(ra, rb)
    finally:
        a.close()
        b.close()
