"""CPU: the C-ABI library builds, loads and exports every symbol include/kpsim.h declares (no compute calls)."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "karpenter-provider-aws_amd", "lib", "libkpsim.so")


def declared_symbols():
    with open(os.path.join(ROOT, "include", "kpsim.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:kp_status|const char\*|int32_t)\s+(kp_[a-z_]+)\(", text, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "karpenter-provider-aws_amd")])
    return C.CDLL(LIB)


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ("kp_ctx_create", "kp_catalog_upload", "kp_solve", "kp_solve_execute", "kp_result_nodeclaim_requirements"):
        assert s in syms


def test_library_exports_all_declared_symbols(lib):
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert missing == []


def test_version_string(lib):
    lib.kp_version.restype = C.c_char_p
    assert b"gfx950" in lib.kp_version()


def test_kpsim_native_exports_match_header():
    from kpsim import native
    assert sorted(native.EXPORTS) == declared_symbols()


def test_oracle_library_loads():
    import pyoracle
    L = pyoracle.lib()
    for s in ("orc_solve", "orc_instance_type_resources", "orc_go_sort_slice_ints", "orc_result_free"):
        assert hasattr(L, s)


def test_views_marshal(golden):
    """Catalog and solve-input views build from the model without touching a device."""
    from kpsim import model, synth
    cv = model.CatalogView(golden[:50])
    assert cv.view.n_types == 50 and cv.n_offerings == 50 * 6
    prob = synth.config1(n_pods=10, catalog=golden[:50])
    iv = model.SolveInputView(prob)
    assert iv.view.pods.n_pods == 10 and iv.view.n_nodepools == 1
