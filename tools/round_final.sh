#!/bin/bash
# GPU box, end of a round: the GPU suite, the full bench (CPU baselines included) and the rocprofv3 profile round.
# Usage: bash tools/round_final.sh <round-tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r03}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -5 gpurun_out/bench_full.err; exit 1; }
bash tools/profile_round.sh "$TAG"
