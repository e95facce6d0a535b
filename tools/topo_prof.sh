#!/bin/bash
# GPU box: profiled config-3 (topology) Solve: stage cycles and the evaluation-failure counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
KPSIM_PROFILE=1 timeout -k 10 200 python bench.py --no-consolidation --no-launch --no-reserved --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/tp.json 2> gpurun_out/tp.err || { tail -3 gpurun_out/tp.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/tp.json'))
for leg in (d, d['topology']):
    print(leg['kernel_ms']['ffd'], {k: v for k, v in leg['ffd_counters'].items() if v}, leg['solve_stats'])"
