#!/bin/bash
# round 4 GPU check: the Solve / topology / preference / consolidation / reserved parity suites (PYTEST_K filter), then
# the config-2 and config-3 Solve legs (5 steps) and the topology quick-accept diagnostics.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/rc.log 2>&1 || { tail -30 gpurun_out/rc.log; exit 1; }
tail -2 gpurun_out/rc.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-consolidation --no-launch --no-reserved --steps 5 --warmup 1 > gpurun_out/bfq.json 2> gpurun_out/bfq.err || { tail -5 gpurun_out/bfq.err; exit 1; }
python3 -c "
import json; b=json.load(open('gpurun_out/bfq.json')); t=b.get('topology') or {}
print('pods/s %.0f ms %.3f ffd %.3f' % (b['value'], b['ms_per_step'], b['kernel_ms']['ffd']), 'topo ffd', (t.get('kernel_ms') or {}).get('ffd'))"
KPSIM_PROFILE=1 timeout -k 10 200 python bench.py --no-consolidation --no-launch --no-reserved --no-cpu-baseline --steps 1 --warmup 0 2>&1 >/dev/null | grep "topology pods past" || true
