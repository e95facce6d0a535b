#!/usr/bin/env python3
"""Benchmark: pods scheduled/sec for Solve on BASELINE.json configs[1] (50k heterogeneous pods × the 918-type
EC2 catalog × 3 AZ × {spot, on-demand}) on the gfx950 library.

    python bench.py [--gpus N] [--steps K] [--warmup W]

One step = one kp_solve_execute (queue sort, class×type masks, template filter, the FFD Solve kernel and
Truncate(60)) with every input already resident in HBM.  Provisioning Solve is a serial chain, so N GPUs run
N independent replicas ("replicas only"); value = pods of all ranks ÷ max-over-ranks time.
Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "karpenter-provider-aws_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

T_START = time.perf_counter()
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
# ctx.ffd_cycles(): FFD kernel counters (the cyc_* stage cycles only under KPSIM_PROFILE=1)
FFD_COUNTERS = ["cyc_fast_loop", "cyc_sort", "cyc_slow_eval", "cyc_templates", "-", "cyc_sort_full", "ev_req", "ev_mask",
                "ev_off", "ev_types", "ev_min", "ev_calls", "quick_accepts", "slow_pods", "witness_misses", "cyc_q_pop",
                "cyc_q_scan", "cyc_q_check", "cyc_q_commit", "n_noinv", "n_winmove", "n_ldssort", "n_pivot", "n_winload",
                "n_flush", "n_shape", "n_lds_append", "n_lds_nowin", "n_lds_outside", "n_batches", "topo_quick",
                "cyc_topo_setup", "cyc_topo_scan", "rej_requirements", "rej_topology", "rej_types", "rej_min_values"]


def log(msg):
    """Progress to stderr (a long silent run looks hung to the GPU harness)."""
    print("[bench %.0fs] %s" % (time.perf_counter() - T_START, msg), file=sys.stderr, flush=True)


def oracle_solve_seconds(orc):
    """The oracle's own Solve-loop + FinalizeScheduling/Truncate time (it reports its phases in kp_solve_stats)."""
    st = orc.results.stats
    return (st["ns_device_solve"] + st["ns_device_finalize"]) / 1e9


def algorithmic_bytes(stats, n_nodeclaims, T, R=12, K_bytes=64):
    """B_solve = Σ_steps [N_t × S_nc + S_pod] + P_new × T × S_type,
    S_nc = ceil(T/8) + 8R + 64, S_pod = 8R + 64, S_type = 8R + 2·32 + 16·6."""
    s_nc = (T + 7) // 8 + 8 * R + K_bytes
    s_pod = 8 * R + K_bytes
    s_type = 8 * R + 64 + 96
    return stats["nodeclaim_candidates_scanned"] * s_nc + stats["pods_popped"] * s_pod + n_nodeclaims * T * s_type


def consolidation_bytes(cst, A, R=12):
    """Algorithmic bytes of the probe kernel: every existing-node slot examined reads its headroom on
    the A active axes and one compatibility bit; every pod popped reads its requests, class and shape (S_pod); every
    NodeClaim / template evaluation reads one NodeClaim row (S_nc = ceil(T/8) + 8R + 64, T = 918); the queue
    bitmap scan reads and clears 8 B per word; a chunk the headroom summary rules out costs its summary row and one
    compatibility word (8A + 8 B) instead of its 64 node slots."""
    s_nc = (918 + 7) // 8 + 8 * R + 64
    s_pod = 8 * R + 64
    return (cst[1] * (8 * A + 1 / 8) + cst[0] * s_pod + (cst[2] + cst[3]) * s_nc + cst[5] * 16 + cst[15] * (8 * A + 8))


def consolidation_leg(a, cat, local, rank, world, dist, barrier, headroom=None):
    """BASELINE configs[3]: single-node consolidation over every candidate of a 5k-node / ~100k-pod cluster plus the
    multi-node prefix probes (first 100 by disruption cost).  headroom=None: nodes at 40-60% utilisation (the probes'
    pods all fit the other nodes: DELETE decisions, existing-node first-fit only); headroom=0.02: every node's free
    cpu / memory capped at 2% of allocatable, so the probes scan the whole cluster, run NodeClaim.Add and the templates
    and mostly decide REPLACE (the "config4-replace" leg: the NodeClaim path timed at scale).  With N GPUs the library shards the probes itself: rank 0
    opens one multi-device ctx over devices 0..N-1 (kp_device_opts.devices), which evaluates one
    contiguous probe shard per device on its own host thread and gathers the results in-process; the other ranks only
    join the barriers.  The decision (kpsim.consolidation.compute_command) replays over the gathered vector."""
    from kpsim import abi, consolidation, model, native, synth
    cp = synth.config4(n_nodes=a.nodes, catalog=cat, headroom=headroom)
    n_s = model.consolidation_probe_count(len(cp.candidates), abi.KP_CONSOLIDATE_SINGLE)
    n_m = model.consolidation_probe_count(len(cp.candidates), abi.KP_CONSOLIDATE_MULTI)
    ctx = None
    if rank == 0:
        ctx = native.Context(local) if world == 1 else native.Context(devices=list(range(world)))
        ctx.upload_catalog(model.CatalogView(cat))
        ctx.consolidate_prepare(model.ConsolidateInputView(cp, abi.KP_CONSOLIDATE_SINGLE))

    def step():
        # one pass over both probe lists (KP_CONSOLIDATE_BOTH: one launch per device, the longest multi-node prefixes
        # first, the single-node probes on the remaining compute units); the library shards it over its devices itself
        # (no torch.distributed collective).  The decisions replay MultiNodeConsolidation's binary search and
        # SingleNodeConsolidation's first-valid scan over the two slices.
        res = ctx.consolidate_execute(abi.KP_CONSOLIDATE_BOTH, n_m + n_s)
        st = ctx.consolidate_stats()
        part = {abi.KP_CONSOLIDATE_MULTI: res[:n_m], abi.KP_CONSOLIDATE_SINGLE: res[n_m:]}
        fn = lambda c, mode, b0, b1: part[mode]  # noqa: E731 (whole ranges: distributed=False)
        cs = consolidation.compute_command(cp, abi.KP_CONSOLIDATE_SINGLE, fn, distributed=False)
        cm = consolidation.compute_command(cp, abi.KP_CONSOLIDATE_MULTI, fn, distributed=False)
        return cs, cm, st, res

    if rank == 0:
        for _ in range(max(1, a.warmup)):
            step()
    barrier()
    t0 = time.perf_counter()
    kms, kcs = [], []
    cs = cm = None
    if rank == 0:
        for _ in range(a.steps):
            cs, cm, st, res = step()
            kms.append([st[0][0], st[0][1]])
            kcs.append(np.array(st[1]))
    elapsed = time.perf_counter() - t0
    barrier()
    if dist is not None:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    if rank != 0:
        return None
    km = np.array(kms).mean(axis=0)
    cst = np.array(kcs).mean(axis=0)
    A = int(np.any(cp.cluster.pods.requests != 0, axis=0).sum())  # active axes (no daemon overhead in config4)
    B = consolidation_bytes(cst, A)
    kern_s = km[1] / 1e3
    achieved = B / kern_s / 1e9 if kern_s > 0 else 0.0
    out = {
        # the controller-visible figure: one disruption pass (both probe lists, the decision replay) — the reference
        # visits ~8 probes per command sequentially; candidates/s counts every probe the pass evaluates
        "metric": "consolidation pass latency",
        "value": elapsed / a.steps * 1e3,
        "unit": "ms",
        "higher_is_better": False,
        "candidates_per_s": (n_s + n_m) * a.steps / elapsed,
        "n_gpus": world,
        "ms_per_step": elapsed / a.steps * 1e3,
        "scaling": "strong",
        "config": {"workload": "config4%s: %d existing nodes, %d bound pods (config2 classes), single-node probes over "
                               "all %d candidates + %d multi-node prefix probes" % (
                                   "" if headroom is None else "-replace (node headroom %g)" % headroom,
                                   len(cp.cluster.existing), cp.cluster.pods.n, n_s, n_m),
                   "parallelism": "probe shards x%d (one multi-device ctx, in-library gather)" % world},
        "decisions": {"single": [cs.decision, cs.candidates[:1]], "multi": [cm.decision, len(cm.candidates)]},
        "probe_decisions": {"none": int((res["decision"] == abi.KP_DECISION_NONE).sum()),
                            "delete": int((res["decision"] == abi.KP_DECISION_DELETE).sum()),
                            "replace": int((res["decision"] == abi.KP_DECISION_REPLACE).sum())},
        "kernel_ms_rank0": {"prep": km[0], "probes": km[1]},
        "counters_per_step": dict(zip(["pods_popped", "existing_slots", "nodeclaim_evals", "template_evals", "probes",
                                       "bitmap_words", "placed_existing", "new_nodeclaims", "chunk_loads", "chunk_hits",
                                       "cyc_build", "cyc_scan", "cyc_nodeclaim", "cyc_decide", "cyc_total", "chunk_skips",
                                       "relaxed"],
                                      [int(x) for x in cst])),
        "roofline": {"bound": "hbm", "kernel": "consolidate_kernel", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "algorithmic_bytes": int(B),
                     "kernel_ms": float(km[1]),
                     "traffic_per_launch": pmc_traffic("consolidate" if headroom is None else "consolidate_replace")},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        import pyoracle
        nthr = min(16, os.cpu_count() or 1)
        r1 = pyoracle.consolidate(cp, abi.KP_CONSOLIDATE_SINGLE, n_threads=nthr)
        cpu_s = pyoracle.last_consolidate_seconds()
        r2 = pyoracle.consolidate(cp, abi.KP_CONSOLIDATE_MULTI, n_threads=nthr)
        cpu_s += pyoracle.last_consolidate_seconds()
        out["cpu_baseline"] = {"value": cpu_s * 1e3, "unit": "ms", "candidates_per_s": (n_s + n_m) / cpu_s,
                               "cores": nthr, "cpu_model": cpu_model(), "kind": "port",
                               "sample": "oracle orc_consolidate (std::thread x %d) over the full pass: %.3f s of "
                                         "probes, timed inside the oracle (input parsing excluded)" % (nthr, cpu_s)}
        d1 = ctx.consolidate_execute(abi.KP_CONSOLIDATE_SINGLE, n_s)
        d2 = ctx.consolidate_execute(abi.KP_CONSOLIDATE_MULTI, n_m)
        same = all((d1[f] == r1[f]).all() and (d2[f] == r2[f]).all() for f in
                   ("decision", "valid", "n_new_nodeclaims", "n_replacement_types", "candidate_price", "replacement_price"))
        out["parity_vs_cpu_baseline"] = bool(same)
    ctx.close()
    return out


def launch_bytes(T, R=12, K=32, O=6):
    """SURVEY §8d S_type = 8R + 2K + 16·O per instance type; one launch request sweeps every type of the catalog."""
    return T * (8 * R + 2 * K + 16 * O)


def pmc_traffic(short):
    """HBM bytes per launch of a kernel from the committed PMC pass (tools/pmc_summary.py), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_%s.json" % short)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get("hbm_bytes_per_launch")


def launch_leg(a, golden, local, rank, world, dist, barrier):
    """BASELINE configs[4] launch side: CloudProvider.Create's instance-type selection (filter.go chain, Truncate(60),
    getCapacityType, override offerings) for a batch of NodeClaims over the catalog with 60 reserved types (40 ODCR
    default + 20 capacity-block, 10% expiring).  200k pods at ~20 pods/node → a 10k-NodeClaim batch.  Requests are
    independent, so ranks take contiguous slices of one fixed batch (strong scaling, no data-path collective)."""
    from kpsim import abi, model, native, synth
    import launch_cases as LC
    cat = synth.config5_catalog(golden)
    reqs_all = synth.launch_requests(cat, n=a.launch_batch)
    from kpsim.consolidation import shard_range
    b0, b1 = shard_range(a.launch_batch, rank, world)  # the slice kpsim.launch.select_sharded gives this rank
    batch = model.LaunchBatchView(reqs_all[b0:b1])
    ctx = native.Context(local)
    cv = model.CatalogView(cat)
    ctx.upload_catalog(cv)
    for _ in range(max(1, a.warmup)):
        res = ctx.launch_select(batch, 60)
    barrier()
    kms, cms = [], []
    t0 = time.perf_counter()
    phases, busy = [], []
    for _ in range(a.steps):
        res = ctx.launch_select(batch, 60)
        st8 = ctx.launch_stats(8)
        kms.append(st8[0])
        cms.append(st8[1])
        phases.append(st8[2:6])
        nsub = int(st8[6])
        busy.append(st8[7])
    elapsed = time.perf_counter() - t0
    barrier()
    kern = float(np.mean(kms))
    if dist is not None:
        import torch
        tt = torch.tensor([elapsed, kern], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, kern = float(tt[0].item()), float(tt[1].item())
    T = len(cat)
    B = launch_bytes(T) * batch.n
    achieved = B / (kern / 1e3) / 1e9 if kern > 0 else 0.0
    st = res.rows["status"]
    out = {
        "metric": "launch selections/sec (filter chain + Truncate(60) per NodeClaim)",
        "value": a.launch_batch / (kern / 1e3) if kern > 0 else 0.0,
        "unit": "nodeclaims/s",
        "n_gpus": world,
        "steps": a.steps,
        "kernel_ms": kern,  # Σ launch_kernel durations of the call's sub-batches (≥ the device busy time below)
        "device_busy_ms": float(np.mean(busy)),
        "call_ms": float(np.mean(cms)),
        # the call pipelines nsub sub-batches: host encoding / expansion of one overlaps the kernel of another, so the
        # phases below are host-side sums (wait_download = time the host waited for a sub-batch's kernel + download)
        "sub_batches": nsub,
        "call_phases_ms": dict(zip(["encode", "merge_upload", "wait_download", "expand"],
                                   [float(x) for x in np.mean(phases, axis=0)])),
        "call_rate_pcie_inclusive": a.launch_batch * a.steps / elapsed,
        "scaling": "strong",
        "config": {"workload": "config5 launch batch: %d NodeClaims x %d types (%d reserved offerings)" % (
            a.launch_batch, T, sum(o.capacity_type == "reserved" for it in cat for o in it.offerings)),
            "parallelism": "batch slices x%d" % world},
        "outcomes": {"ok": int((st == abi.KP_OK).sum()), "ice": int((st == abi.KP_E_INSUFFICIENT_CAPACITY).sum()),
                     "reserved": int((res.rows["capacity_type"] == abi.KP_CT_RESERVED).sum())},
        # per launch: algorithmic bytes B / nsub over the mean launch duration kern / nsub (the same ratio)
        "roofline": {"bound": "hbm", "kernel": "launch_kernel", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "algorithmic_bytes": int(B),
                     "launches_per_step": nsub, "algorithmic_bytes_per_launch": int(B / nsub), "traffic": pmc_traffic("launch"),
                     # the algorithmic bytes are catalog rows served from LDS / L2: measured HBM traffic per launch
                     # over the launch time is the kernel's real HBM rate (it is bound by its block barriers)
                     "measured_traffic_frac": (pmc_traffic("launch") / (kern / nsub / 1e3) / 1e9 / HBM_PEAK_GBS
                                               if pmc_traffic("launch") and kern > 0 else None)},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        import pyoracle
        n = min(batch.n, 1000)
        sb = model.LaunchBatchView(reqs_all[:n])
        t = time.perf_counter()
        pyoracle.launch_select(cv, model.LaunchBatchView([]), 60)
        parse_s = time.perf_counter() - t  # catalog parse of the oracle call
        t = time.perf_counter()
        stc, orc = pyoracle.launch_select(cv, sb, 60)
        cpu_s = max(1e-9, time.perf_counter() - t - parse_s)
        out["cpu_baseline"] = {"value": n / cpu_s, "unit": "nodeclaims/s", "cores": 1, "cpu_model": cpu_model(), "kind": "port",
                               "sample": "oracle orc_launch_select, 1 thread, first %d requests of the batch: %.2f s "
                                         "(catalog parsing, %.2f s, excluded)" % (n, cpu_s, parse_s)}
        dev = ctx.launch_select(sb, 60)
        try:
            assert stc == abi.KP_OK
            LC.assert_same(dev, orc)
            out["parity_vs_cpu_baseline"] = True
        except AssertionError:
            out["parity_vs_cpu_baseline"] = False
    ctx.close()
    return out


ROOFLINE_NOTE = ("the Solve is one serial chain run by ONE workgroup (8 waves on 1 of 256 CUs; every placement changes "
                 "the state the next pod is checked against), so algorithmic bytes / kernel time is not an HBM-bandwidth "
                 "figure: the kernel is latency-bound (waves waiting on dependent LDS / L2 round trips) — "
                 "stage_cycles_per_pod breaks its time down")


def cpu_model():
    """The GPU box host's CPU model (lscpu "Model name", from /proc/cpuinfo), stated with every cpu_baseline."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.lower().startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def stage_cycles_per_pod(ctx, iv, out, n_pods):
    """One more kp_solve with KPSIM_PROFILE=1 (s_memtime stamps, after the timed region): the FFD kernel's shader-clock
    cycles per pod by stage (wave 0's fast loop and slice sort, the block's slow-path evaluations and templates, the
    topology prefilter setup / first-survivor scan), and the pods each path placed."""
    prev = os.environ.get("KPSIM_PROFILE")
    os.environ["KPSIM_PROFILE"] = "1"
    try:
        ctx.solve(iv, out)
        cyc = dict(zip(FFD_COUNTERS, ctx.ffd_cycles()))
    finally:  # a caller's own KPSIM_PROFILE (tools/profile_round.sh's stage run) stays for the later legs
        if prev is None:
            del os.environ["KPSIM_PROFILE"]
        else:
            os.environ["KPSIM_PROFILE"] = prev
    ctx.prepare(iv)
    out = {k: cyc[k] / n_pods for k in ("cyc_fast_loop", "cyc_sort", "cyc_slow_eval", "cyc_templates", "cyc_topo_setup",
                                        "cyc_topo_scan") if cyc.get(k)}
    out.update({k: int(cyc[k]) for k in ("quick_accepts", "topo_quick", "slow_pods", "ev_calls") if k in cyc})
    return out


def ffd_kernel_name(prob):
    """The Solve kernel instantiation a problem launches (kp_launch_ffd): topology groups → ffd_topo_kernel, reserved
    offerings → ffd_resv_kernel, both → ffd_resv_topo_kernel (preference relaxation adds _pref)."""
    topo = any(pc.topology for pc in prob.classes)
    resv = any(o.capacity_type == "reserved" for it in prob.catalog for o in it.offerings)
    pref = any(pc.preferred_terms or len(pc.required_terms) > 1 or
               any(t.when_unsatisfiable == "ScheduleAnyway" or t.weight for t in pc.topology) for pc in prob.classes)
    return "ffd_" + ("pref_" if pref else "") + ("resv_" if resv else "") + ("topo_" if topo else "") + "kernel"


def solve_leg(a, cat, prob, metric, workload, cpu_sample, local, rank, world, dist, barrier):
    """A further Solve workload, same step as the headline leg: one kp_solve_execute with HBM-resident inputs; replicas
    across ranks (weak scaling, no collective); CPU baseline on a seeded subsample, with device parity on it."""
    from kpsim import model, native, synth
    ctx = native.Context(local)
    ctx.upload_catalog(model.CatalogView(cat))
    iv = model.SolveInputView(prob)
    cap_nc = max(16, prob.pods.n + 1)
    out = model.OutputBuffers(prob.pods.n, cap_nc, cap_nc * 60)
    t = time.perf_counter()
    ctx.solve(iv, out)
    e2e_ms = (time.perf_counter() - t) * 1e3
    log("%s: first solve %.1f ms" % (workload.split(":")[0], e2e_ms))
    res = out.results()
    ctx.prepare(iv)
    for _ in range(a.warmup):
        ctx.execute()
    barrier()
    kts = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ctx.execute()
        kts.append(ctx.kernel_times_ms())
    elapsed = time.perf_counter() - t0
    barrier()
    if dist is not None:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    kt = np.array(kts).mean(axis=0)
    P, T = prob.pods.n, len(cat)
    B = algorithmic_bytes(res.stats, res.n_nodeclaims, T)
    achieved = B / (kt[3] / 1e3) / 1e9
    line = {
        "metric": metric,
        "value": P * a.steps * world / elapsed,
        "unit": "pods/s",
        "n_gpus": world,
        "ms_per_step": elapsed / a.steps * 1e3,
        "scaling": "weak",
        "config": {"workload": workload, "parallelism": "replicas" if world > 1 else "single"},
        "kernel_ms": {"queue_sort": float(kt[0]), "class_mask": float(kt[1]), "template_init": float(kt[2]),
                      "ffd": float(kt[3]), "finalize": float(kt[4])},
        "end_to_end_ms": e2e_ms,
        "nodeclaims": res.n_nodeclaims,
        "unschedulable": int((res.pod_result == -1).sum()),
        "roofline": {"bound": "hbm", "kernel": ffd_kernel_name(prob), "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "algorithmic_bytes": int(B), "kernel_ms": float(kt[3]),
                     "traffic": pmc_traffic({"ffd_topo_kernel": "ffd_topo", "ffd_resv_kernel": "ffd_resv"}.get(
                         ffd_kernel_name(prob), "ffd"))},
        "solve_stats": {k: v for k, v in res.stats.items() if not k.startswith("ns_")},
        "ffd_counters": dict(zip(FFD_COUNTERS, ctx.ffd_cycles())),
        "cpu_baseline": None,
    }
    line["roofline"]["note"] = ROOFLINE_NOTE
    line["stage_cycles_per_pod"] = stage_cycles_per_pod(ctx, iv, out, P)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        import parity
        import pyoracle
        full = cpu_sample <= 0 or cpu_sample >= P
        sample = prob if full else synth.subsample(prob, cpu_sample)
        log("cpu baseline: oracle on %d pods" % sample.pods.n)
        orc = pyoracle.solve(sample)
        cpu_s = oracle_solve_seconds(orc)
        what = "the full %d-pod workload" % sample.pods.n if full else "a seeded %d-pod subsample" % sample.pods.n
        line["cpu_baseline"] = {"value": sample.pods.n / cpu_s, "unit": "pods/s", "cores": 1, "cpu_model": cpu_model(),
                                "kind": "port",
                                "sample": "oracle (1 thread) on %s: %.2f s of Solve + Truncate "
                                          "(input parsing excluded)" % (what, cpu_s)}
        dev = parity.run_device(ctx, sample)
        if not full:
            # the device on the same sample, so the CPU baseline is compared like for like (the leg's value is the
            # full workload's)
            line["gpu_on_cpu_sample"] = {"pods": sample.pods.n, "ffd_ms": float(ctx.kernel_times_ms()[3]),
                                         "pods_per_s": sample.pods.n / (ctx.kernel_times_ms()[3] / 1e3)}
        try:
            parity.assert_same(dev, (orc.results, [model.parse_requirements_blob(orc.requirements(i))
                                                   for i in range(orc.results.n_nodeclaims)]))
            line["parity_vs_cpu_baseline"] = True
        except AssertionError:
            line["parity_vs_cpu_baseline"] = False
    ctx.close()
    return line


def topology_leg(a, cat, local, rank, world, dist, barrier):
    """BASELINE configs[2]: 50k pods with zonal + hostname topology spread and hostname anti-affinity over five weighted
    NodePools with cpu limits (synth.config3)."""
    from kpsim import synth
    prob = synth.config3(n_pods=a.pods, catalog=cat)
    n_topo = int(sum(1 for c in prob.pods.class_id if prob.classes[int(c)].topology))
    return solve_leg(a, cat, prob, "pods scheduled/sec (Solve, config3: topology spread + anti-affinity, 5 weighted NodePools)",
                     "config3: %d pods (%d with topology terms), 250 classes x %d types, 5 NodePools"
                     % (prob.pods.n, n_topo, len(cat)), a.topo_cpu_sample, local, rank, world, dist, barrier)


def reserved_leg(a, cat, local, rank, world, dist, barrier):
    """BASELINE configs[4] as a Solve: config-2 pods over the catalog with 60 reserved offerings (40 ODCR, 20 capacity
    blocks), ODCR-first NodePools; the ReservationManager runs in strict mode (synth.config5)."""
    from kpsim import synth
    cat5 = synth.config5_catalog(cat)
    prob = synth.config5(n_pods=a.resv_pods, catalog=cat5)
    return solve_leg(a, cat5, prob, "pods scheduled/sec (Solve, config5: reserved offerings, ODCR-first NodePools)",
                     "config5: %d pods, 250 classes x %d types (60 reserved offerings), 3 NodePools"
                     % (prob.pods.n, len(cat5)), a.resv_cpu_sample, local, rank, world, dist, barrier)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pods", type=int, default=50_000)
    ap.add_argument("--cpu-sample", type=int, default=0, help="pods in the CPU-baseline sample (0 = the full workload)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-consolidation", action="store_true")
    ap.add_argument("--no-consolidation-replace", action="store_true")
    ap.add_argument("--no-config4", action="store_true", help="skip the config-4 consolidation pass (keep the replace leg)")
    ap.add_argument("--nodes", type=int, default=5000, help="config4 cluster size (consolidation leg)")
    ap.add_argument("--launch-batch", type=int, default=10_000, help="config5 launch batch (NodeClaims)")
    ap.add_argument("--no-launch", action="store_true")
    ap.add_argument("--no-topology", action="store_true")
    ap.add_argument("--topo-cpu-sample", type=int, default=50_000,
                    help="pods in config3's CPU-baseline sample (default: the full workload, ~46 s of oracle time)")
    ap.add_argument("--no-reserved", action="store_true")
    ap.add_argument("--resv-pods", type=int, default=200_000, help="config5 Solve pods")
    ap.add_argument("--resv-cpu-sample", type=int, default=40_000,
                    help="pods in config5's CPU-baseline sample (the full 200k takes the oracle ~9 min: its reservation "
                         "bookkeeping grows with NodeClaims x pods; DESIGN.md §6)")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")

    from kpsim import catalog, model, native, synth

    fx = catalog.load_fixtures()
    cat = catalog.golden_catalog(fx=fx)
    prob = synth.config2(n_pods=a.pods, catalog=cat)
    ctx = native.Context(local)
    cv = model.CatalogView(cat)
    ctx.upload_catalog(cv)
    iv = model.SolveInputView(prob)
    cap_nc = max(16, prob.pods.n + 1)
    out = model.OutputBuffers(prob.pods.n, cap_nc, cap_nc * 60)

    # end-to-end (PCIe-inclusive) call once, for the record
    t = time.perf_counter()
    ctx.solve(iv, out)
    e2e_ms = (time.perf_counter() - t) * 1e3
    res = out.results()
    cyc = ctx.ffd_cycles()
    # the same kp_solve call again (warm: device buffers, kernel modules and the hipcub workspace exist), with its
    # phases from kp_solve_stats: host prepare (intern + encode + upload), device execute, fetch + decode
    e2e_warm = []
    for _ in range(3):
        t = time.perf_counter()
        ctx.solve(iv, out)
        e2e_warm.append((time.perf_counter() - t) * 1e3)
    st = out.results().stats
    solve_call = {"ms": float(np.median(e2e_warm)), "host_prep_ms": st["ns_host_prep"] / 1e6,
                  "device_execute_ms": st["ns_device_solve"] / 1e6, "fetch_ms": st["ns_device_finalize"] / 1e6}
    ctx.prepare(iv)  # inputs resident in HBM from here on

    for _ in range(a.warmup):
        ctx.execute()

    def barrier():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    barrier()
    ffd_ms = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ctx.execute()  # synchronous on the library's stream
        ffd_ms.append(ctx.kernel_times_ms())
    elapsed = time.perf_counter() - t0
    barrier()
    if dist is not None:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    kt = np.array(ffd_ms).mean(axis=0)
    stages = stage_cycles_per_pod(ctx, iv, out, prob.pods.n) if rank == 0 else None
    P = prob.pods.n
    value = P * a.steps * world / elapsed
    T = len(cat)
    B = algorithmic_bytes(res.stats, res.n_nodeclaims, T)
    ffd_s = kt[3] / 1e3
    achieved = B / ffd_s / 1e9
    traffic = pmc_traffic("ffd")

    log("config2 solve leg done: %.1f ms/step" % (elapsed / a.steps * 1e3))
    cons = None if (a.no_consolidation or a.no_config4) else consolidation_leg(a, cat, local, rank, world, dist, barrier)
    log("consolidation leg done")
    cons_r = None if (a.no_consolidation or a.no_consolidation_replace) else consolidation_leg(
        a, cat, local, rank, world, dist, barrier, headroom=0.02)
    log("consolidation replace leg done")
    launch = None if a.no_launch else launch_leg(a, cat, local, rank, world, dist, barrier)
    log("launch leg done")
    topo = None if a.no_topology else topology_leg(a, cat, local, rank, world, dist, barrier)
    log("topology leg done")
    resv = None if a.no_reserved else reserved_leg(a, cat, local, rank, world, dist, barrier)
    log("reserved leg done")

    cpu = None
    parity_ok = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        import parity
        import pyoracle
        full = a.cpu_sample <= 0 or a.cpu_sample >= prob.pods.n
        sample = prob if full else synth.subsample(prob, a.cpu_sample)
        log("cpu baseline: oracle on %d pods" % sample.pods.n)
        orc = pyoracle.solve(sample)
        cpu_s = oracle_solve_seconds(orc)
        what = ("the full %d-pod config2 workload" % sample.pods.n if full else
                "a seeded %d-pod subsample of the config2 workload (same catalog, NodePools, classes)" % sample.pods.n)
        cpu = {"value": sample.pods.n / cpu_s, "unit": "pods/s", "cores": 1, "cpu_model": cpu_model(), "kind": "port",
               "sample": "oracle (C++ restatement of Solve, 1 thread) on %s: %.2f s of Solve + Truncate "
                         "(input parsing excluded)" % (what, cpu_s)}
        dev = parity.run_device(ctx, sample)
        try:
            parity.assert_same(dev, (orc.results, [model.parse_requirements_blob(orc.requirements(i))
                                                    for i in range(orc.results.n_nodeclaims)]))
            parity_ok = True
        except AssertionError:
            parity_ok = False

    if rank == 0:
        line = {
            "metric": "pods scheduled/sec (Solve, 50k pods × EC2 catalog)",
            "value": value,
            "unit": "pods/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (seeded config2 over the reference's golden 918-type catalog)",
            "config": {"workload": "config2: %d heterogeneous pods (250 classes) x %d types x 3 AZ x {spot,on-demand},"
                                   " 2 NodePools" % (P, T), "pods": P, "types": T,
                       "parallelism": "replicas" if world > 1 else "single"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "ffd_kernel", "kernel_ms": float(kt[3]), "algorithmic_bytes": int(B),
                         "note": ROOFLINE_NOTE},
            "stage_cycles_per_pod": stages,
            "cpu_baseline": cpu,
            "parity_vs_cpu_baseline": parity_ok,  # device result bit-identical to the oracle's on the same input
            "kernel_ms": {"queue_sort": float(kt[0]), "class_mask": float(kt[1]), "template_init": float(kt[2]),
                          "ffd": float(kt[3]), "finalize": float(kt[4])},
            "end_to_end_ms": e2e_ms,
            "solve_call_warm": solve_call,
            "ffd_counters": dict(zip(FFD_COUNTERS, cyc)),
            "nodeclaims": res.n_nodeclaims,
            "unschedulable": int((res.pod_result == -1).sum()),
            "solve_stats": {k: v for k, v in res.stats.items() if not k.startswith("ns_")},
            "consolidation": cons,
            "consolidation_replace": cons_r,
            "launch": launch,
            "topology": topo,
            "reserved": resv,
        }
        print(json.dumps(line))
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
