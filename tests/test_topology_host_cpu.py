"""CPU: which topology inputs the C-ABI host layer accepts (row N1: one device group per TopologyGroup.Hash() identity,
with the first owner's node filter and minDomains), decided by kp_solve_prepare / kp_consolidate_prepare built over
the CPU stub of the HIP runtime (tests/cpu_stub, build/libkpsim_stub.so) and run in a child process
(tests/stub_topology_checks.py).  The device's results for the accepted inputs are the -m gpu tests
(test_gpu_topology.py, test_gpu_consolidation.py); here: the first-owner KATs and the shared-identity fuzz families are
accepted, and the two shapes whose first owner the device cannot fix at prepare are refused."""
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
    assert checks["cons_pending_True"] == "ok"


def test_relaxed_only_identity_refused(checks):
    assert checks["relaxed_only"].startswith("KP_E_UNSUPPORTED") and "only relaxed pods create" in checks["relaxed_only"]


def test_probe_dependent_owner_refused(checks):
    v = checks["cons_pending_False"]
    assert v.startswith("KP_E_UNSUPPORTED") and "differs between consolidation probes" in v
