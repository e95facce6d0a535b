#!/bin/bash
# GPU box: config-2 Solve leg with each library under tools/ab/ (KPSIM_LIB override), two rounds, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for lib in tools/ab/*.so; do
    n=$(basename $lib .so)
    KPSIM_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-consolidation --no-launch --no-reserved --no-topology --steps 5 --warmup 1 > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { tail -5 gpurun_out/ab_$n.err; exit 1; }
    python3 -c "
import json; b=json.load(open('gpurun_out/ab_$n.json'))
print('$r $n ms %.3f ffd %.3f' % (b['ms_per_step'], b['kernel_ms']['ffd']), b['kernel_ms'])"
  done
done
