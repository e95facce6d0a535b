"""ORACLE — test infrastructure only.  ctypes binding of oracle/build/liboracle.so.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = C.CDLL(LIB)
        from kpsim import abi
        _lib.orc_solve.argtypes = [C.POINTER(abi.kp_catalog_view), C.POINTER(abi.kp_solve_input),
                                   C.POINTER(abi.kp_solve_output), C.POINTER(C.c_void_p)]
        _lib.orc_solve.restype = C.c_int32
        _lib.orc_solve_opts.argtypes = [C.POINTER(abi.kp_catalog_view), C.POINTER(abi.kp_solve_input),
                                        C.POINTER(abi.kp_device_opts), C.POINTER(abi.kp_solve_output),
                                        C.POINTER(C.c_void_p)]
        _lib.orc_solve_opts.restype = C.c_int32
        _lib.orc_result_nodeclaim_requirements.argtypes = [C.c_void_p, C.c_int32, C.c_char_p, C.c_int64,
                                                           C.POINTER(C.c_int64)]
        _lib.orc_result_nodeclaim_requirements.restype = C.c_int32
        _lib.orc_result_free.argtypes = [C.c_void_p]
        _lib.orc_instance_type_resources.argtypes = [C.POINTER(OrcEc2Info), C.POINTER(OrcTypeOpts)] + \
            [C.POINTER(C.c_int64)] * 4
        _lib.orc_consolidate_probe_count.argtypes = [C.POINTER(abi.kp_consolidate_input)]
        _lib.orc_consolidate_probe_count.restype = C.c_int32
        _lib.orc_consolidate.argtypes = [C.POINTER(abi.kp_catalog_view), C.POINTER(abi.kp_consolidate_input),
                                         C.POINTER(abi.kp_probe_result), C.c_int32, C.c_int32]
        _lib.orc_consolidate.restype = C.c_int32
        _lib.orc_consolidate_command.argtypes = [C.POINTER(abi.kp_catalog_view), C.POINTER(abi.kp_consolidate_input),
                                                 C.c_int32, C.POINTER(abi.kp_consolidation_command), C.c_int32]
        _lib.orc_consolidate_command.restype = C.c_int32
        _lib.orc_consolidate_opts.argtypes = [C.POINTER(abi.kp_catalog_view), C.POINTER(abi.kp_consolidate_input),
                                              C.POINTER(abi.kp_device_opts), C.POINTER(abi.kp_probe_result), C.c_int32,
                                              C.c_int32]
        _lib.orc_consolidate_opts.restype = C.c_int32
        _lib.orc_consolidate_command_opts.argtypes = [C.POINTER(abi.kp_catalog_view), C.POINTER(abi.kp_consolidate_input),
                                                      C.POINTER(abi.kp_device_opts), C.c_int32,
                                                      C.POINTER(abi.kp_consolidation_command), C.c_int32]
        _lib.orc_consolidate_command_opts.restype = C.c_int32
        _lib.orc_consolidate_replacement_opts.argtypes = [C.POINTER(abi.kp_catalog_view),
                                                          C.POINTER(abi.kp_consolidate_input),
                                                          C.POINTER(abi.kp_device_opts), C.c_int32, C.c_int32,
                                                          C.POINTER(abi.kp_consolidation_command)]
        _lib.orc_consolidate_replacement_opts.restype = C.c_int32
        _lib.orc_launch_select.argtypes = [C.POINTER(abi.kp_catalog_view), C.c_int32, C.POINTER(abi.kp_launch_request),
                                           C.c_int32, C.POINTER(abi.kp_launch_result), C.POINTER(C.c_int32), C.c_int32,
                                           C.POINTER(C.c_int32), C.c_int32]
        _lib.orc_launch_select.restype = C.c_int32
        _lib.orc_go_sort_slice_ints.argtypes = [C.POINTER(C.c_int64), C.POINTER(C.c_int32), C.c_int32]
    return _lib


class OrcEc2Info(C.Structure):
    _fields_ = [("vcpus", C.c_int32), ("memory_mib", C.c_int64), ("arm64", C.c_int32), ("amd64", C.c_int32),
                ("default_card_max_enis", C.c_int32), ("ipv4_per_eni", C.c_int32), ("instance_storage_gb", C.c_int64),
                ("nvidia_gpus", C.c_int32), ("amd_gpus", C.c_int32), ("habana_gpus", C.c_int32),
                ("neuron_devices", C.c_int32), ("neuron_cores", C.c_int32), ("efa", C.c_int32),
                ("has_limits", C.c_int32), ("limits_trunking", C.c_int32), ("limits_branch", C.c_int32),
                ("limits_ipv4_per_eni", C.c_int32)]


class OrcTypeOpts(C.Structure):
    _fields_ = [("vm_memory_overhead_pct", C.c_double), ("reserved_enis", C.c_int32), ("ami_family", C.c_int32),
                ("max_pods", C.c_int32), ("pods_per_core", C.c_int32), ("raid0", C.c_int32)]


AMI = {"AL2023": 0, "AL2": 1, "Bottlerocket": 2, "Windows2022": 3, "Windows2019": 3, "Custom": 4}


def instance_type_resources(info, opts, vpclimits):
    """(capacity, kube_reserved, eviction, allocatable) as int64[12] milli, ORC_R_* axis order == kpsim RESOURCES."""
    L = lib()
    cards = info.get("cards") or []
    gpus = info.get("gpus") or []
    nd = info.get("neuron_devices") or []
    lim = vpclimits.get(info["name"])
    e = OrcEc2Info(
        vcpus=int(info["vcpus"]), memory_mib=int(info["memory_mib"]),
        arm64=1 if info["architectures"] and info["architectures"][0] == "arm64" else 0,
        amd64=1 if "x86_64" in info["architectures"] else 0,
        default_card_max_enis=int(cards[info.get("default_card", 0)] if cards else info.get("max_enis", 0)),
        ipv4_per_eni=int(info["ipv4_per_eni"]),
        instance_storage_gb=-1 if info.get("instance_storage_gb") is None else int(info["instance_storage_gb"]),
        nvidia_gpus=sum(g["count"] for g in gpus if g["manufacturer"] == "NVIDIA"),
        amd_gpus=sum(g["count"] for g in gpus if g["manufacturer"] == "AMD"),
        habana_gpus=sum(g["count"] for g in gpus if g["manufacturer"] == "Habana"),
        neuron_devices=sum(d["count"] for d in nd), neuron_cores=(nd[0]["count"] * nd[0]["cores"]) if nd else 0,
        efa=int(info.get("efa_max") or 0), has_limits=1 if lim else 0,
        limits_trunking=1 if lim and lim["trunking"] else 0, limits_branch=lim["branch_interface"] if lim else 0,
        limits_ipv4_per_eni=lim["ipv4_per_interface"] if lim else 0)
    o = OrcTypeOpts(vm_memory_overhead_pct=opts.vm_memory_overhead_pct, reserved_enis=opts.reserved_enis,
                    ami_family=AMI[opts.ami_family], max_pods=-1 if opts.max_pods is None else opts.max_pods,
                    pods_per_core=0 if opts.pods_per_core is None else opts.pods_per_core, raid0=1 if opts.raid0 else 0)
    outs = [np.zeros(12, np.int64) for _ in range(4)]
    L.orc_instance_type_resources(C.byref(e), C.byref(o), *[a.ctypes.data_as(C.POINTER(C.c_int64)) for a in outs])
    return tuple(outs)


def go_sort_slice_ints(keys_by_id, perm):
    keys = np.ascontiguousarray(keys_by_id, np.int64)
    p = np.ascontiguousarray(perm, np.int32).copy()
    lib().orc_go_sort_slice_ints(keys.ctypes.data_as(C.POINTER(C.c_int64)), p.ctypes.data_as(C.POINTER(C.c_int32)),
                                 len(p))
    return p


class OracleResult:
    def __init__(self, results, handle):
        self.results = results
        self._h = handle

    def requirements(self, nc):
        L = lib()
        need = C.c_int64(0)
        buf = C.create_string_buffer(1 << 16)
        st = L.orc_result_nodeclaim_requirements(self._h, nc, buf, len(buf), C.byref(need))
        if st == 2:
            buf = C.create_string_buffer(need.value)
            st = L.orc_result_nodeclaim_requirements(self._h, nc, buf, len(buf), C.byref(need))
        assert st == 0, st
        return buf.value.decode()

    def __del__(self):
        if self._h:
            lib().orc_result_free(self._h)
            self._h = None


def solve(problem, catalog_view=None, preference_policy=0, reserved_capacity=1):
    """Run the CPU oracle on a kpsim.model.Problem (solver parameters as kp_device_opts).  Returns OracleResult."""
    from kpsim import abi, model
    L = lib()
    opts = abi.kp_device_opts(preference_policy=preference_policy, reserved_capacity=reserved_capacity)
    cv = catalog_view or model.CatalogView(problem.catalog)
    iv = model.SolveInputView(problem)
    cap_nc = max(16, problem.pods.n + 1)
    ob = model.OutputBuffers(problem.pods.n, cap_nc, cap_nc * max(1, problem.max_instance_types or len(problem.catalog)))
    h = C.c_void_p()
    st = L.orc_solve_opts(C.byref(cv.view), C.byref(iv.view), C.byref(opts), C.byref(ob.view), C.byref(h))
    if st != 0:
        raise RuntimeError("orc_solve failed: %d" % st)
    return OracleResult(ob.results(), h)


def consolidate(cp, mode, probe_begin=0, probe_end=0, spot_to_spot=False, max_candidates=100, n_threads=1,
                catalog_view=None, preference_policy=0):
    """CPU oracle consolidation probes for a kpsim.model.ConsolidationProblem -> numpy array of abi.PROBE_DTYPE."""
    from kpsim import abi, model
    L = lib()
    opts = abi.kp_device_opts(preference_policy=preference_policy)
    cv = catalog_view or model.CatalogView(cp.cluster.catalog)
    iv = model.ConsolidateInputView(cp, mode, probe_begin, probe_end, spot_to_spot, max_candidates)
    n = L.orc_consolidate_probe_count(C.byref(iv.view))
    b0 = max(0, probe_begin)
    b1 = probe_end if 0 < probe_end < n else n
    out = np.zeros(max(1, b1 - b0), abi.PROBE_DTYPE)
    st = L.orc_consolidate_opts(C.byref(cv.view), C.byref(iv.view), C.byref(opts),
                                out.ctypes.data_as(C.POINTER(abi.kp_probe_result)), len(out), n_threads)
    if st != 0:
        raise RuntimeError("orc_consolidate failed: %d" % st)
    return out[:max(0, b1 - b0)]


def consolidate_command(cp, mode, spot_to_spot=False, max_candidates=100, n_threads=1, catalog_view=None,
                        preference_policy=0):
    """CPU oracle consolidation command (orc_consolidate_command) -> kpsim.consolidation.Command."""
    from kpsim import abi, consolidation, model
    L = lib()
    opts = abi.kp_device_opts(preference_policy=preference_policy)
    cv = catalog_view or model.CatalogView(cp.cluster.catalog)
    iv = model.ConsolidateInputView(cp, mode, 0, 0, spot_to_spot, max_candidates)
    st, cmd = consolidation.command_call(
        lambda cc: L.orc_consolidate_command_opts(C.byref(cv.view), C.byref(iv.view), C.byref(opts), mode, C.byref(cc),
                                                  n_threads))
    if st != 0:
        raise RuntimeError("orc_consolidate_command failed: %d" % st)
    return cmd


def consolidate_replacement(cp, mode, probe, spot_to_spot=False, max_candidates=100, preference_policy=0):
    """CPU oracle command of one given probe (orc_consolidate_replacement_opts) -> kpsim.consolidation.Command."""
    from kpsim import abi, consolidation, model
    L = lib()
    opts = abi.kp_device_opts(preference_policy=preference_policy)
    cv = model.CatalogView(cp.cluster.catalog)
    iv = model.ConsolidateInputView(cp, mode, 0, 0, spot_to_spot, max_candidates)
    st, cmd = consolidation.command_call(
        lambda cc: L.orc_consolidate_replacement_opts(C.byref(cv.view), C.byref(iv.view), C.byref(opts), mode, probe,
                                                      C.byref(cc)))
    if st != 0:
        raise RuntimeError("orc_consolidate_replacement failed: %d" % st)
    return cmd


def last_consolidate_seconds():
    """Probe-phase wall time of the last consolidate() call (the oracle's input parsing excluded)."""
    L = lib()
    L.orc_consolidate_last_probe_seconds.restype = C.c_double
    return float(L.orc_consolidate_last_probe_seconds())


def launch_select(catalog_view, batch, M=60):
    """orc_launch_select over a kpsim.model.LaunchBatchView → (status, model.LaunchResults)."""
    from kpsim import model
    L = lib()
    return model.launch_call(lambda *a: L.orc_launch_select(C.byref(catalog_view.view), *a), catalog_view, batch, M)
