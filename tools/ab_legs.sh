#!/bin/bash
# GPU box: the Solve legs (config 2, config 3 topology, config 5 reserved) with each library under tools/ab/ and the
# working tree's (KPSIM_LIB override), ROUNDS rounds interleaved; prints the FFD kernel ms of each leg.
# Usage: tools/ab_legs.sh [rounds] [legs: c2,c3,c5]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${1:-2}
LEGS=${2:-c2,c3,c5}
libs="karpenter-provider-aws_amd/lib/libkpsim.so $(ls tools/ab/*.so 2>/dev/null)"
for r in $(seq 1 $ROUNDS); do
  for lib in $libs; do
    n=$(basename $(dirname $(dirname $lib)))_$(basename $lib .so)
    args="--no-cpu-baseline --no-consolidation --no-launch --steps 3 --warmup 1"
    [[ $LEGS == *c3* ]] || args="$args --no-topology"
    [[ $LEGS == *c5* ]] || args="$args --no-reserved"
    KPSIM_LIB=$PWD/$lib timeout -k 10 300 python bench.py $args > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { tail -5 gpurun_out/ab_$n.err; exit 1; }
    python3 -c "
import json; b=json.loads(open('gpurun_out/ab_$n.json').read().strip().splitlines()[-1])
t=(b.get('topology') or {}).get('kernel_ms',{}).get('ffd'); v=(b.get('reserved') or {}).get('kernel_ms',{}).get('ffd')
print('$r %-34s c2 ffd %.2f ms' % ('$n', b['kernel_ms']['ffd']), (' c3 ffd %.1f' % t) if t else '', (' c5 ffd %.1f' % v) if v else '', flush=True)"
  done
done
