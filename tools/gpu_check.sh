#!/bin/bash
# GPU-box check used during development: gpu parity tests, bench, profiled bench; summary to stdout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?
tail -3 gpurun_out/t.log
[ $rc -ne 0 ] && { grep -E "Error|error|assert" gpurun_out/t.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err || exit $?
KPSIM_PROFILE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/bp.json 2> gpurun_out/bp.err || exit $?
python3 - <<'PY'
import json
for f in ["gpurun_out/b.json", "gpurun_out/bp.json"]:
    d = json.load(open(f))
    print(f, "ms/step %.2f ffd %.2f" % (d["ms_per_step"], d["kernel_ms"]["ffd"]),
          {k: v for k, v in d["ffd_counters"].items() if v})
PY
