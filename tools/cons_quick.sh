#!/bin/bash
# GPU-box check of a consolidation-kernel change: consolidation parity suite, then the consolidation leg (5 steps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_consolidation.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tc.log 2>&1 || { tail -30 gpurun_out/tc.log; exit 1; }
tail -2 gpurun_out/tc.log
timeout -k 10 300 python bench.py --no-launch --no-topology --no-reserved --steps 10 --warmup 3 > gpurun_out/bcq.json 2> gpurun_out/bcq.err || { tail -5 gpurun_out/bcq.err; exit 1; }
python3 -c "
import json; c=json.load(open('gpurun_out/bcq.json'))['consolidation']; print('cands/s %.0f ms %.3f' % (c['value'], c['ms_per_step']), c['kernel_ms_rank0'], 'parity', c.get('parity_vs_cpu_baseline'))"
