"""Loader for libkpsim.so (the gfx950 library).  Fails loudly if it is missing: there is no CPU fallback."""
import ctypes as C
import os

from . import abi

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "..", "lib", "libkpsim.so")

EXPORTS = [
    "kp_ctx_create", "kp_ctx_destroy", "kp_last_error", "kp_version", "kp_catalog_upload", "kp_catalog_patch_avail",
    "kp_catalog_patch_price", "kp_solve", "kp_solve_prepare", "kp_solve_execute", "kp_solve_fetch",
    "kp_result_nodeclaim_requirements", "kp_last_kernel_times", "kp_consolidate_probe_count", "kp_consolidate",
    "kp_consolidate_stats", "kp_consolidate_prepare", "kp_consolidate_execute", "kp_launch_select", "kp_launch_stats",
    "kp_nodeclaim_labels", "kp_catalog_build", "kp_catalog_get_view", "kp_catalog_overhead", "kp_catalog_resource_name",
    "kp_catalog_free", "kp_consolidate_command", "kp_consolidate_replacement",
]

_lib = None


class KpError(RuntimeError):
    def __init__(self, status, msg=""):
        super().__init__("%s: %s" % (abi.STATUS_NAMES.get(status, status), msg))
        self.status = status


def load():
    global _lib
    if _lib is not None:
        return _lib
    path = os.path.normpath(os.environ.get("KPSIM_LIB", LIB_PATH))  # A/B diagnostics override
    if not os.path.exists(path):
        raise ImportError("libkpsim.so not built at %s (run __graft_entry__.build() or make -C karpenter-provider-aws_amd)"
                          % path)
    L = C.CDLL(path)
    L.kp_ctx_create.argtypes = [C.POINTER(abi.kp_device_opts), C.POINTER(C.c_void_p)]
    L.kp_ctx_destroy.argtypes = [C.c_void_p]
    L.kp_last_error.argtypes = [C.c_void_p]
    L.kp_last_error.restype = C.c_char_p
    L.kp_version.restype = C.c_char_p
    L.kp_catalog_upload.argtypes = [C.c_void_p, C.POINTER(abi.kp_catalog_view), C.c_uint64]
    L.kp_catalog_patch_avail.argtypes = [C.c_void_p, C.POINTER(C.c_uint8), C.c_int32, C.c_uint64]
    L.kp_catalog_patch_price.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_double), C.c_int32, C.c_uint64]
    L.kp_solve.argtypes = [C.c_void_p, C.POINTER(abi.kp_solve_input), C.POINTER(abi.kp_solve_output)]
    L.kp_solve_prepare.argtypes = [C.c_void_p, C.POINTER(abi.kp_solve_input)]
    L.kp_solve_execute.argtypes = [C.c_void_p]
    L.kp_solve_fetch.argtypes = [C.c_void_p, C.POINTER(abi.kp_solve_output)]
    L.kp_result_nodeclaim_requirements.argtypes = [C.c_void_p, C.c_int32, C.c_char_p, C.c_int64, C.POINTER(C.c_int64)]
    L.kp_last_kernel_times.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.c_int32]
    L.kp_consolidate_probe_count.argtypes = [C.POINTER(abi.kp_consolidate_input)]
    L.kp_consolidate.argtypes = [C.c_void_p, C.POINTER(abi.kp_consolidate_input), C.POINTER(abi.kp_probe_result),
                                 C.c_int32]
    L.kp_consolidate_prepare.argtypes = [C.c_void_p, C.POINTER(abi.kp_consolidate_input)]
    L.kp_consolidate_execute.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.POINTER(abi.kp_probe_result),
                                         C.c_int32]
    L.kp_consolidate_stats.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int64), C.c_int32]
    L.kp_consolidate_command.argtypes = [C.c_void_p, C.c_int32, C.POINTER(abi.kp_consolidation_command)]
    if hasattr(L, "kp_consolidate_replacement"):  # (absent from pre-round-5 libraries, A/B only)
        L.kp_consolidate_replacement.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(abi.kp_consolidation_command)]
    L.kp_launch_select.argtypes = [C.c_void_p, C.c_int32, C.POINTER(abi.kp_launch_request), C.c_int32,
                                   C.POINTER(abi.kp_launch_result), C.POINTER(C.c_int32), C.c_int32,
                                   C.POINTER(C.c_int32), C.c_int32]
    L.kp_launch_stats.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.c_int32]
    L.kp_nodeclaim_labels.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_char_p, C.c_char_p, C.c_int32, C.c_char_p,
                                      C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    for f in EXPORTS:
        if os.environ.get("KPSIM_LIB") and not hasattr(L, f):
            continue  # A/B diagnostics: an older library without a later entry point (its callers are not used)
        if f not in ("kp_last_error", "kp_version", "kp_catalog_resource_name"):
            getattr(L, f).restype = C.c_int32
    _lib = L
    return L


class Context:
    """One kp_ctx (device stream + buffers).  Not thread-safe; use one per thread."""

    def __init__(self, device=0, preference_policy=abi.KP_PREFERENCE_RESPECT, devices=None, reserved_capacity=1):
        L = load()
        self.L = L
        h = C.c_void_p()
        opts = abi.kp_device_opts(device=device, preference_policy=preference_policy, reserved_capacity=reserved_capacity)
        if devices:
            import numpy as np
            self._devs = np.ascontiguousarray(devices, np.int32)
            opts.n_devices = len(self._devs)
            opts.devices = self._devs.ctypes.data_as(C.POINTER(C.c_int32))
        st = L.kp_ctx_create(C.byref(opts), C.byref(h))
        if st != 0:
            raise KpError(st, "kp_ctx_create(device=%d) — a gfx950 device is required" % device)
        self.h = h
        self._catalog = None
        # bumped by every call that replaces the ctx's catalog or prepared pass (kp_catalog_*, kp_solve*,
        # kp_consolidate[_prepare]): lets a caller tell whether the pass it prepared is still the ctx's
        self.pass_gen = 0

    def check(self, st, what):
        if st != 0:
            raise KpError(st, "%s: %s" % (what, self.L.kp_last_error(self.h).decode()))

    def upload_catalog(self, catalog_view, epoch=1):
        self.pass_gen += 1
        self.check(self.L.kp_catalog_upload(self.h, C.byref(catalog_view.view), epoch), "kp_catalog_upload")
        self._catalog = catalog_view

    def patch_avail(self, available, epoch):
        self.pass_gen += 1
        import numpy as np
        a = np.ascontiguousarray(available, np.uint8)
        self.check(self.L.kp_catalog_patch_avail(self.h, a.ctypes.data_as(C.POINTER(C.c_uint8)), len(a), epoch),
                   "kp_catalog_patch_avail")

    def patch_price(self, idx, price, epoch):
        self.pass_gen += 1
        import numpy as np
        i = np.ascontiguousarray(idx, np.int32)
        p = np.ascontiguousarray(price, np.float64)
        self.check(self.L.kp_catalog_patch_price(self.h, i.ctypes.data_as(C.POINTER(C.c_int32)),
                                                 p.ctypes.data_as(C.POINTER(C.c_double)), len(i), epoch),
                   "kp_catalog_patch_price")

    def launch_select(self, batch, M=60):
        """kp_launch_select over a model.LaunchBatchView → model.LaunchResults (instance.go:132-137 per request)."""
        from kpsim import model
        st, res = model.launch_call(lambda *a: self.L.kp_launch_select(self.h, *a), self._catalog, batch, M)
        self.check(st, "kp_launch_select")
        return res

    def nodeclaim_labels(self, type_index, offering, zone_id=None, nodepool=None, efa_enabled=False):
        """kp_nodeclaim_labels (instanceToNodeClaim, cloudprovider.go:381-444) → (labels dict, capacity[R],
        allocatable[R]) for an instance of catalog row type_index launched through offering row `offering`."""
        import numpy as np
        from kpsim import model
        need = C.c_int64(0)
        buf = C.create_string_buffer(1 << 14)
        cap = np.zeros(model.R, np.int64)
        alloc = np.zeros(model.R, np.int64)
        self.check(self.L.kp_nodeclaim_labels(self.h, type_index, offering, zone_id.encode() if zone_id else None,
                                              nodepool.encode() if nodepool else None, 1 if efa_enabled else 0, buf,
                                              len(buf), C.byref(need), cap.ctypes.data_as(C.POINTER(C.c_int64)),
                                              alloc.ctypes.data_as(C.POINTER(C.c_int64))), "kp_nodeclaim_labels")
        labels = dict(line.split("\t", 1) for line in buf.value.decode().splitlines() if line)
        return labels, cap, alloc

    def launch_stats(self, n=2):
        """[kernel ms, whole call ms] (n=6 adds the host phases: encode, merge + upload, download waits, expand;
        n=7 the number of sub-batches the call was pipelined over)."""
        ms = (C.c_double * n)()
        self.check(self.L.kp_launch_stats(self.h, ms, n), "kp_launch_stats")
        return list(ms)

    def prepare(self, input_view):
        self.pass_gen += 1
        self.check(self.L.kp_solve_prepare(self.h, C.byref(input_view.view)), "kp_solve_prepare")

    def execute(self):
        self.check(self.L.kp_solve_execute(self.h), "kp_solve_execute")

    def fetch(self, out_buffers):
        self.check(self.L.kp_solve_fetch(self.h, C.byref(out_buffers.view)), "kp_solve_fetch")

    def solve(self, input_view, out_buffers):
        self.pass_gen += 1
        self.check(self.L.kp_solve(self.h, C.byref(input_view.view), C.byref(out_buffers.view)), "kp_solve")

    def nodeclaim_requirements(self, nc):
        need = C.c_int64(0)
        buf = C.create_string_buffer(1 << 16)
        st = self.L.kp_result_nodeclaim_requirements(self.h, nc, buf, len(buf), C.byref(need))
        if st == abi.KP_E_BUFFER:
            buf = C.create_string_buffer(need.value)
            st = self.L.kp_result_nodeclaim_requirements(self.h, nc, buf, len(buf), C.byref(need))
        self.check(st, "kp_result_nodeclaim_requirements")
        return buf.value.decode()

    def kernel_times_ms(self):
        """[queue sort, class masks, template filter, FFD, finalize] of the last execute (HIP events)."""
        a = (C.c_double * 5)()
        self.check(self.L.kp_last_kernel_times(self.h, a, 5), "kp_last_kernel_times")
        return list(a)

    def ffd_cycles(self):
        """FFD-kernel counters of the last fetched solve (kpsim.h kp_last_kernel_times [5..19]): s_memtime cycles
        (with KPSIM_PROFILE=1) of the fast loop, sort, slow-path rounds, templates, -, full sort, six evaluation
        stages; then quick accepts, slow-path pods, witness misses, quick-path cycles (pop, scan, check, commit)."""
        a = (C.c_double * 42)()
        self.check(self.L.kp_last_kernel_times(self.h, a, 42), "kp_last_kernel_times")
        return list(a)[5:]

    def consolidate(self, cons_view):
        """kp_consolidate over the view's probe range -> numpy array of abi.PROBE_DTYPE (one row per probe)."""
        self.pass_gen += 1
        import numpy as np
        v = cons_view.view
        n = self.L.kp_consolidate_probe_count(C.byref(v))
        b0 = max(0, v.probe_begin)
        b1 = v.probe_end if 0 < v.probe_end < n else n
        out = np.zeros(max(1, b1 - b0), abi.PROBE_DTYPE)
        self.check(self.L.kp_consolidate(self.h, C.byref(v), out.ctypes.data_as(C.POINTER(abi.kp_probe_result)),
                                         len(out)), "kp_consolidate")
        return out[:max(0, b1 - b0)]

    def consolidate_prepare(self, cons_view):
        self.pass_gen += 1
        self.check(self.L.kp_consolidate_prepare(self.h, C.byref(cons_view.view)), "kp_consolidate_prepare")

    def consolidate_execute(self, mode, n_probes, begin=0, end=0):
        """Probes [begin, end) of `mode` over the prepared pass; n_probes = the mode's probe count."""
        import numpy as np
        b1 = end if 0 < end < n_probes else n_probes
        out = np.zeros(max(1, b1 - begin), abi.PROBE_DTYPE)
        self.check(self.L.kp_consolidate_execute(self.h, mode, begin, end,
                                                 out.ctypes.data_as(C.POINTER(abi.kp_probe_result)), len(out)),
                   "kp_consolidate_execute")
        return out[:max(0, b1 - begin)]

    def consolidate_command(self, mode):
        """kp_consolidate_command over the prepared pass -> kpsim.consolidation.Command (with the replacement)."""
        from kpsim import consolidation
        st, cmd = consolidation.command_call(lambda cc: self.L.kp_consolidate_command(self.h, mode, C.byref(cc)))
        self.check(st, "kp_consolidate_command")
        return cmd

    def consolidate_replacement(self, mode, probe):
        """kp_consolidate_replacement: the command of one probe of the prepared pass (its row and, for a REPLACE, the
        replacement NodeClaim) -> kpsim.consolidation.Command."""
        from kpsim import consolidation
        st, cmd = consolidation.command_call(
            lambda cc: self.L.kp_consolidate_replacement(self.h, mode, probe, C.byref(cc)))
        self.check(st, "kp_consolidate_replacement")
        return cmd

    def consolidate_stats(self):
        """(ms[prep, probe kernel, call], counters[20]) of the last kp_consolidate (kpsim.h kp_consolidate_stats)."""
        ms = (C.c_double * 3)()
        ct = (C.c_int64 * 20)()
        self.check(self.L.kp_consolidate_stats(self.h, ms, ct, 20), "kp_consolidate_stats")
        return list(ms), list(ct)

    def close(self):
        if getattr(self, "h", None):
            self.L.kp_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
