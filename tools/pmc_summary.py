"""Summarise a tools/profile_round.sh run into profiles/: the kernel-trace stats CSV (copied as-is) and
profiles/pmc_<kernel>.json with the HBM bytes per launch of ffd_kernel, consolidate_kernel and launch_kernel (MI355X_MICROARCH.md: FETCH_SIZE is doubled on
gfx950 for wide streaming reads; WRITE_SIZE taken as is).  Usage: python tools/pmc_summary.py <outdir> <tag>"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def find(d, pattern):
    hits = sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))
    if not hits:
        raise SystemExit("no %s under %s" % (pattern, d))
    return hits[0]


def counter_per_launch(d, name, kernel="ffd_kernel"):
    vals = {}
    with open(find(d, "*counter_collection.csv")) as f:
        for row in csv.DictReader(f):
            if kernel in row.get("Kernel_Name", "") and row.get("Counter_Name") == name:
                key = row.get("Dispatch_Id") or row.get("Correlation_Id")
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    if not vals:
        raise SystemExit("no %s rows for %s" % (name, kernel))
    return sum(vals.values()) / len(vals), len(vals)


def main():
    out, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = find(os.path.join(out, "trace"), "*kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, "%s_kernel_stats.csv" % tag))
    recs = []
    # per kernel: profiles/pmc_<short>.json (bench.py reads hbm_bytes_per_launch as roofline.traffic)
    for kernel, short in (("ffd_kernel", "ffd"), ("ffd_topo_kernel", "ffd_topo"), ("consolidate_kernel", "consolidate"),
                          ("launch_kernel", "launch")):
        fetch_kb, nf = counter_per_launch(os.path.join(out, "fetch"), "FETCH_SIZE", kernel)
        write_kb, nw = counter_per_launch(os.path.join(out, "write"), "WRITE_SIZE", kernel)
        # rocprofv3 FETCH_SIZE / WRITE_SIZE are in KiB
        fetch_b, write_b = fetch_kb * 1024.0, write_kb * 1024.0
        rec = {
            "kernel": kernel,
            "round": tag,
            "command": "python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --no-reserved --no-consolidation-replace "
                       "(config2 and config3 50k-pod Solves; config4; config5 launch)",
            "fetch_size_bytes_raw": fetch_b,
            "write_size_bytes": write_b,
            "hbm_bytes_per_launch": 2.0 * fetch_b + write_b,
            "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); WRITE_SIZE as reported",
            "launches": {"fetch_pass": nf, "write_pass": nw},
        }
        for name in ("pmc_%s.json" % short, "%s_pmc_%s.json" % (tag, short)):
            with open(os.path.join(prof, name), "w") as f:
                json.dump(rec, f, indent=1)
        recs.append(rec)
    # the Solve kernels' SQ issue / wait counters (per launch) and their KPSIM_PROFILE stage cycles
    for kernel, short in (("ffd_kernel", "ffd"), ("ffd_topo_kernel", "ffd_topo")):
        sq = {}
        for pas in ("sq1", "sq2"):
            d = os.path.join(out, pas)
            if not os.path.isdir(d):
                continue
            names = set()
            with open(find(d, "*counter_collection.csv")) as f:
                for row in csv.DictReader(f):
                    if kernel in row.get("Kernel_Name", ""):
                        names.add(row["Counter_Name"])
            for nm in sorted(names):
                v, _ = counter_per_launch(d, nm, kernel)
                sq[nm] = v
        stages = {}
        sj = os.path.join(out, "stages.json")
        if os.path.exists(sj):
            with open(sj) as f:
                b = json.load(f)
            leg = b if short == "ffd" else (b.get("topology") or {})
            stages = {"kernel_ms": (leg.get("kernel_ms") or {}).get("ffd"), "ffd_counters": leg.get("ffd_counters"),
                      "solve_stats": leg.get("solve_stats")}
        if sq or stages:
            rec = {"kernel": kernel, "round": tag, "sq_counters_per_launch": sq,
                   "note": "SQ_* summed over the kernel's workgroup (one workgroup, 8 waves); cycles in shader clocks; "
                           "stage cycles from KPSIM_PROFILE=1 s_memtime stamps (wave 0's fast loop, the block's slow "
                           "path, templates) in a separate run",
                   "kpsim_profile": stages}
            with open(os.path.join(prof, "%s_pmc_%s_sq.json" % (tag, short)), "w") as f:
                json.dump(rec, f, indent=1)
    with open(stats) as f:
        print(f.read())
    for rec in recs:
        print(json.dumps(rec))


if __name__ == "__main__":
    main()
