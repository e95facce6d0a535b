"""Summarise a tools/profile_round.sh run into profiles/: the kernel-trace stats CSV (copied as-is) and
profiles/pmc_<kernel>.json with the HBM bytes per launch of the Solve kernels (config 2 / 3 / 5), consolidate_kernel
(config 4 and the config4-replace leg, whose FULL variant is consolidate_full_kernel) and launch_kernel (MI355X_MICROARCH.md: FETCH_SIZE is doubled on
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


WAVES = {"ffd_kernel": 8, "ffd_topo_kernel": 4, "ffd_resv_kernel": 8}  # kp_layout.h KP_NWAVES / KP_NWAVES_TOPO
MAIN_CMD = ("python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --no-consolidation-replace (config 2, config 4, "
            "config 5 launch, config 3, config 5 200k Solve)")
REPL_CMD = ("python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --no-config4 --no-launch --no-topology --no-reserved "
            "(config 2 and the config4-replace consolidation leg)")


def hbm_record(out, sub, kernel, tag, command):
    fetch_kb, nf = counter_per_launch(os.path.join(out, "fetch" + sub), "FETCH_SIZE", kernel)
    write_kb, nw = counter_per_launch(os.path.join(out, "write" + sub), "WRITE_SIZE", kernel)
    fetch_b, write_b = fetch_kb * 1024.0, write_kb * 1024.0  # rocprofv3 FETCH_SIZE / WRITE_SIZE are in KiB
    return {
        "kernel": kernel,
        "round": tag,
        "command": command,
        "fetch_size_bytes_raw": fetch_b,
        "write_size_bytes": write_b,
        "hbm_bytes_per_launch": 2.0 * fetch_b + write_b,
        "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); WRITE_SIZE as reported",
        "launches": {"fetch_pass": nf, "write_pass": nw},
    }


def main():
    out, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = find(os.path.join(out, "trace"), "*kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, "%s_kernel_stats.csv" % tag))
    if os.path.isdir(os.path.join(out, "trace_replace")):
        shutil.copy(find(os.path.join(out, "trace_replace"), "*kernel_stats.csv"),
                    os.path.join(prof, "%s_kernel_stats_replace.csv" % tag))
    recs = []
    # per kernel: profiles/pmc_<short>.json (bench.py reads hbm_bytes_per_launch as roofline.traffic)
    for kernel, short, sub, cmd in (("ffd_kernel", "ffd", "", MAIN_CMD), ("ffd_topo_kernel", "ffd_topo", "", MAIN_CMD),
                                    ("ffd_resv_kernel", "ffd_resv", "", MAIN_CMD),
                                    ("consolidate_kernel", "consolidate", "", MAIN_CMD),
                                    ("launch_kernel", "launch", "", MAIN_CMD),
                                    ("consolidate_kernel", "consolidate_replace", "_replace", REPL_CMD),
                                    ("consolidate_full_kernel", "consolidate_full_replace", "_replace", REPL_CMD)):
        if not os.path.isdir(os.path.join(out, "fetch" + sub)):
            continue
        rec = hbm_record(out, sub, kernel, tag, cmd)
        for name in ("pmc_%s.json" % short, "%s_pmc_%s.json" % (tag, short)):
            with open(os.path.join(prof, name), "w") as f:
                json.dump(rec, f, indent=1)
        recs.append(rec)
    # the Solve kernels' SQ issue / wait counters (per launch) and their KPSIM_PROFILE stage cycles
    legs = {"ffd_kernel": None, "ffd_topo_kernel": "topology", "ffd_resv_kernel": "reserved"}
    for kernel, short in (("ffd_kernel", "ffd"), ("ffd_topo_kernel", "ffd_topo"), ("ffd_resv_kernel", "ffd_resv")):
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
        if sq.get("SQ_WAVE_CYCLES"):
            sq["wait_any_over_wave_cycles"] = sq.get("SQ_WAIT_ANY", 0.0) / sq["SQ_WAVE_CYCLES"]
        stages = {}
        sj = os.path.join(out, "stages.json")
        if os.path.exists(sj):
            with open(sj) as f:
                b = json.loads(f.read().strip().splitlines()[-1])
            leg = b if legs[kernel] is None else (b.get(legs[kernel]) or {})
            stages = {"kernel_ms": (leg.get("kernel_ms") or {}).get("ffd"),
                      "stage_cycles_per_pod": leg.get("stage_cycles_per_pod"),
                      "ffd_counters": leg.get("ffd_counters"), "solve_stats": leg.get("solve_stats")}
        if sq or stages:
            rec = {"kernel": kernel, "round": tag, "sq_counters_per_launch": sq,
                   "note": "SQ_* summed over the kernel's one workgroup (%d waves); cycles in shader clocks; stage "
                           "cycles from KPSIM_PROFILE=1 s_memtime stamps in a separate run (ffd_counters: that run's "
                           "whole-solve totals; stage_cycles_per_pod: per pod)" % WAVES[kernel],
                   "kpsim_profile": stages}
            with open(os.path.join(prof, "%s_pmc_%s_sq.json" % (tag, short)), "w") as f:
                json.dump(rec, f, indent=1)
    with open(stats) as f:
        print(f.read())
    for rec in recs:
        print(json.dumps(rec))


if __name__ == "__main__":
    main()
