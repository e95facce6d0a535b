#!/bin/bash
# GPU box: rocprofv3 counter passes over the config-2 / config-3 Solve legs (ffd_kernel, ffd_topo_kernel): SQ issue /
# wait breakdown, then FETCH_SIZE and WRITE_SIZE passes (gfx950: one TCC counter group per pass).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-r04}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$ROOT/bench.py --no-cpu-baseline --no-consolidation --no-launch --no-reserved --steps 1 --warmup 0"
timeout -s KILL 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM -T -d "$OUT/sq1" -o run --output-format csv -- python3 $BENCH > "$OUT/sq1.json" 2> "$OUT/sq1.err" || { tail -5 "$OUT/sq1.err"; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -T -d "$OUT/sq2" -o run --output-format csv -- python3 $BENCH > "$OUT/sq2.json" 2> "$OUT/sq2.err" || { tail -5 "$OUT/sq2.err"; exit 1; }
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/fetch" -o run --output-format csv -- python3 $BENCH > "$OUT/fetch.json" 2>/dev/null || exit 1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/write" -o run --output-format csv -- python3 $BENCH > "$OUT/write.json" 2>/dev/null || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for f in sorted(glob.glob(out + "/*/*counter_collection.csv")):
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "ffd" not in k: continue
        acc[(k, r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, c), v in sorted(acc.items()): print(f.split("/")[-3], k[:30], c, "%.4g" % v)
PY
