#!/bin/bash
# A/B timing of libkpsim builds on the GPU box: the in-tree library plus any lib/libkpsim_<name>.so variants
# (built here with different flags / -D settings), Solve leg only.  Usage: bash tools/ab_variants.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in karpenter-provider-aws_amd/lib/libkpsim*.so; do
  n=$(basename "$L" .so)
  KPSIM_LIB=$PWD/$L timeout -k 10 200 python bench.py --no-consolidation --no-launch --no-topology --no-cpu-baseline --steps 5 > gpurun_out/ab_$n.json || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$n.json')); print('$n', d['ms_per_step'], d['kernel_ms']['ffd'])"
done
