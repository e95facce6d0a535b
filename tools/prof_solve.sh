#!/bin/bash
# GPU box: config-2 Solve leg under KPSIM_PROFILE=1 (stage cycles, slow-path reasons), then unprofiled timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
KPSIM_PROFILE=1 timeout -k 10 200 python bench.py --no-consolidation --no-launch --no-reserved --no-topology --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/ps.json 2> gpurun_out/ps.err || { tail -3 gpurun_out/ps.err; exit 1; }
grep "slow-path pods\|topology pods past" gpurun_out/ps.err || true
timeout -k 10 200 python bench.py --no-consolidation --no-launch --no-reserved --no-topology --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/pq.json 2> gpurun_out/pq.err || { tail -3 gpurun_out/pq.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ps.json')); q=json.load(open('gpurun_out/pq.json'))
print('unprofiled ffd', q['kernel_ms']['ffd'], 'profiled', d['kernel_ms']['ffd'])
print({k: v for k, v in d['ffd_counters'].items() if v}, d['solve_stats'])"
