#!/bin/bash
# GPU box: the consolidation legs (config 4 and config4-replace) with each library under tools/ab/ and the working
# tree's (KPSIM_LIB override), ROUNDS rounds interleaved; prints pass ms and probe kernel ms of both legs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${1:-2}
libs="karpenter-provider-aws_amd/lib/libkpsim.so $(ls tools/ab/*.so 2>/dev/null)"
for r in $(seq 1 $ROUNDS); do
  for lib in $libs; do
    n=$(basename $(dirname $(dirname $lib)))_$(basename $lib .so)
    KPSIM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-launch --no-topology --no-reserved --steps 10 --warmup 2 > gpurun_out/abc_$n.json 2> gpurun_out/abc_$n.err || { tail -5 gpurun_out/abc_$n.err; exit 1; }
    python3 -c "
import json; b=json.loads(open('gpurun_out/abc_$n.json').read().strip().splitlines()[-1])
c=b['consolidation']; x=b['consolidation_replace']
print('$r %-34s config4 pass %.3f ms probes %.3f | replace pass %.3f ms probes %.3f' % ('$n', c['value'], c['kernel_ms_rank0']['probes'], x['value'], x['kernel_ms_rank0']['probes']), flush=True)"
  done
done
