#!/bin/bash
# GPU box: topology parity suite, then the config-3 leg timed (3 steps) and profiled (stage + loop-segment cycles).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_topology.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tt.log 2>&1 || { tail -30 gpurun_out/tt.log; exit 1; }
tail -2 gpurun_out/tt.log
timeout -k 10 300 python bench.py --no-consolidation --no-launch --no-reserved --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/tq.json 2> gpurun_out/tq.err || { tail -3 gpurun_out/tq.err; exit 1; }
KPSIM_PROFILE=1 timeout -k 10 200 python bench.py --no-consolidation --no-launch --no-reserved --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/tp.json 2> gpurun_out/tp.err || { tail -3 gpurun_out/tp.err; exit 1; }
python3 -c "
import json
q=json.load(open('gpurun_out/tq.json'))
print('timed: config2 ffd %.2f ms, config3 ffd %.2f ms' % (q['kernel_ms']['ffd'], q['topology']['kernel_ms']['ffd']))
d=json.load(open('gpurun_out/tp.json'))['topology']
print('profiled config3', d['kernel_ms']['ffd'], {k: v for k, v in d['ffd_counters'].items() if v})"
grep "solve loop segments\|topology pods past\|slow-path pods" gpurun_out/tp.err
