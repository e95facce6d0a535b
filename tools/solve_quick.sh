#!/bin/bash
# GPU box: Solve legs only (config2 headline, config3 topology, config5 reserved), no CPU baseline, then the GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-consolidation --no-launch --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/sq.json 2> gpurun_out/sq.err || { tail -3 gpurun_out/sq.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/sq.json'))
print('config2 ffd %.2f ms, step %.2f, warm call %s' % (d['kernel_ms']['ffd'], d['ms_per_step'], d['solve_call_warm']), {k: d['ffd_counters'][k] for k in ('quick_accepts', 'slow_pods')})
for l in ('topology', 'reserved'): print(l, 'ffd %.1f ms' % d[l]['kernel_ms']['ffd'], {k: d[l]['ffd_counters'][k] for k in ('quick_accepts', 'slow_pods')})"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1; tail -2 gpurun_out/t.log
