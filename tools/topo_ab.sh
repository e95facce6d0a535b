#!/bin/bash
# GPU box: config-3 (topology) Solve profiled with and without the team evaluation (KPSIM_NO_TEAM)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in team noteam; do
  env_=""; [ $v = noteam ] && export KPSIM_NO_TEAM=1
  KPSIM_PROFILE=1 timeout -k 10 200 python bench.py --no-consolidation --no-launch --no-reserved --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/tp_$v.json 2> gpurun_out/tp_$v.err || { tail -3 gpurun_out/tp_$v.err; exit 1; }
  timeout -k 10 200 python bench.py --no-consolidation --no-launch --no-reserved --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/tq_$v.json 2> gpurun_out/tq_$v.err || { tail -3 gpurun_out/tq_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/tp_$v.json'))['topology']; q=json.load(open('gpurun_out/tq_$v.json'))['topology']
print('$v', 'unprofiled ffd', q['kernel_ms']['ffd'], 'profiled', d['kernel_ms']['ffd'])
print({k: v for k, v in d['ffd_counters'].items() if v}, d['solve_stats'])"
done
