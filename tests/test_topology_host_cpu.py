"""CPU: which topology inputs the C-ABI host layer accepts (row N1: one device group per TopologyGroup.Hash() identity,
with the first owner's node filter and minDomains), decided by kp_solve_prepare / kp_consolidate_prepare built over
the CPU stub of the HIP runtime (tests/cpu_stub, build/libkpsim_stub.so) and run in a child process
(tests/stub_topology_checks.py).  The device's results for the accepted inputs are the -m gpu tests
(test_gpu_topology.py, test_gpu_consolidation.py); here: the first-owner KATs and the shared-identity fuzz families are
accepted, and an identity whose owners' selections differ while its first owner differs between probes is refused."""
import json
import os
import shutil
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
STUB = os.path.join(HERE, "cpu_stub")


@pytest.fixture(scope="module")
def checks():
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    subprocess.check_call(["make", "-s", "-C", STUB, "build/libkpsim_stub.so"], stdout=subprocess.DEVNULL)
    env = dict(os.environ, KPSIM_LIB=os.path.join(STUB, "build", "libkpsim_stub.so"))
    r = subprocess.run([sys.executable, os.path.join(HERE, "stub_topology_checks.py"), "8"], capture_output=True,
                       text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_first_owner_kats_accepted(checks):
    for k in ("filter_True", "filter_False", "min_domains_True", "min_domains_False"):
        assert checks[k] == "ok", (k, checks[k])


def test_shared_identity_fuzz_accepted(checks):
    for k, v in checks.items():
        if k.startswith("fuzz_") or k.startswith("cons_fuzz_"):
            assert v == "ok", (k, v)
    assert checks["cons_pending_True"] == "ok" and checks["cons_pending_False"] == "ok"


def test_relaxed_only_identity_accepted(checks):
    """one variant group per filter, born by the first relaxation (topo_build's variant groups)"""
    assert checks["relaxed_only_True"] == "ok" and checks["relaxed_only_False"] == "ok"


def test_probe_dependent_selection_refused(checks):
    """an identity whose owners select different pods and whose first owner differs between probes"""
    v = checks["cons_selection"]
    assert v.startswith("KP_E_UNSUPPORTED") and "different selections" in v


def test_reserved_offering_refusal_reasons(checks):
    """ResvTab limits name their cause: a type with more than 64 reservations, or more than 1,024 reserved offerings."""
    assert checks["resv_per_type_70"].startswith("KP_E_UNSUPPORTED") and "m5.large has more than 64" in checks["resv_per_type_70"]
    assert checks["resv_over_max"].startswith("KP_E_UNSUPPORTED") and "KP_MAX_RO" in checks["resv_over_max"]


def test_reservation_id_selection_beyond_64(checks):
    """pod and NodePool requirements on capacity-reservation-id over 200 reservations are accepted (per-type values
    through ResvTab rows); minValues on that key is refused (distinct counts use 64-bit masks)"""
    assert checks["resv_id_selection"] == "ok"
    assert checks["resv_id_min_values"].startswith("KP_E_UNSUPPORTED") and "minValues" in checks["resv_id_min_values"]
