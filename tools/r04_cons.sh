#!/bin/bash
# round 4: consolidation parity (incl. preferences / BestEffort / hostname affinity in probes) + preferences suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_consolidation.py tests/test_gpu_preferences.py -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/r04c.log 2>&1
rc=$?
tail -25 gpurun_out/r04c.log
exit $rc
