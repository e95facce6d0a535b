#!/bin/bash
# GPU box: config-2 and config-3 Solve legs with each library under tools/ab/ (KPSIM_LIB override), two rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for lib in tools/ab/*.so; do
    n=$(basename $lib .so)
    KPSIM_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-consolidation --no-launch --no-reserved --steps 2 --warmup 1 > gpurun_out/abt_$n.json 2> gpurun_out/abt_$n.err || { tail -5 gpurun_out/abt_$n.err; exit 1; }
    python3 -c "
import json; b=json.load(open('gpurun_out/abt_$n.json'))
print('$r $n config2 ffd %.2f config3 ffd %.1f' % (b['kernel_ms']['ffd'], b['topology']['kernel_ms']['ffd']))"
  done
done
