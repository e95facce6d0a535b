#!/bin/bash
# GPU-box check for the consolidation path: parity tests, then a profiled bench (counters + stage cycles).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_consolidation.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tc.log 2>&1
rc=$?
tail -3 gpurun_out/tc.log
[ $rc -ne 0 ] && { grep -E "Error|error|assert" gpurun_out/tc.log | head -20; exit $rc; }
KPSIM_PROFILE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/bp.json 2> gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/b.json 2> gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
python3 - <<'PY'
import json
for f in ["gpurun_out/bp.json", "gpurun_out/b.json"]:
    c = json.load(open(f))["consolidation"]
    print(f, "cands/s %.0f ms/step %.3f" % (c["candidates_per_s"], c["ms_per_step"]), c["kernel_ms_rank0"])
    print("  ", {k: v for k, v in c["counters_per_step"].items() if v}, c.get("counters_multi"))
PY
