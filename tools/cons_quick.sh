#!/bin/bash
# GPU-box check of a consolidation-kernel change: consolidation parity suite, then the two consolidation legs (config4
# and config4-replace, 10 steps, with the oracle's parity check), then a profiled run (stage cycles + counters).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_consolidation.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tc.log 2>&1 || { tail -30 gpurun_out/tc.log; exit 1; }
tail -2 gpurun_out/tc.log
timeout -k 10 300 python bench.py --no-launch --no-topology --no-reserved --steps 10 --warmup 3 > gpurun_out/bcq.json 2> gpurun_out/bcq.err || { tail -5 gpurun_out/bcq.err; exit 1; }
KPSIM_PROFILE=1 timeout -k 10 300 python bench.py --no-launch --no-topology --no-reserved --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/bcp.json 2> gpurun_out/bcp.err || { tail -5 gpurun_out/bcp.err; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/bcq.json", "gpurun_out/bcp.json"):
    d = json.load(open(f))
    for leg in ("consolidation", "consolidation_replace"):
        c = d[leg]
        print(f, leg, "cands/s %.0f ms %.3f" % (c["candidates_per_s"], c["ms_per_step"]), c["kernel_ms_rank0"], "parity",
              c.get("parity_vs_cpu_baseline"), c.get("probe_decisions"))
        print("   ", {k: v for k, v in c["counters_per_step"].items() if v})
PY
grep "\[kpsim\]" gpurun_out/bcp.err | tail -8
