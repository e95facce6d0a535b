#!/bin/bash
# GPU box: config-3 Solve with and without the topology scan's rejection memo (KPSIM_NO_TOPO_MEMO), interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in memo nomemo; do
    ( [ $v = nomemo ] && export KPSIM_NO_TOPO_MEMO=1; timeout -k 10 200 python bench.py --no-cpu-baseline --no-consolidation --no-launch --no-reserved --steps 2 --warmup 1 > gpurun_out/tm_$v.json 2> gpurun_out/tm_$v.err ) || { tail -3 gpurun_out/tm_$v.err; exit 1; }
    python3 -c "
import json; b=json.load(open('gpurun_out/tm_$v.json'))
print('$r $v config2 ffd %.2f config3 ffd %.1f' % (b['kernel_ms']['ffd'], b['topology']['kernel_ms']['ffd']), b['topology']['solve_stats'])"
  done
done
