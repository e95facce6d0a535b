#!/bin/bash
# Round profile on the GPU box: kernel-trace stats of the bench command, then one PMC pass per TCC counter
# (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950).  Usage: tools/profile_round.sh <round-tag>
set -euo pipefail
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1"
# kernel-trace stats over every leg; the PMC passes run the config2 Solve, consolidation and launch legs only, so the
# per-launch traffic of ffd_kernel is config2's (the topology / reservation legs launch other instantiations)
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d "$OUT/trace" -o run --output-format csv -- python3 $BENCH --no-consolidation-replace > "$OUT/trace.json"
BENCH="$BENCH --no-topology --no-reserved --no-consolidation-replace"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/fetch" -o run --output-format csv -- python3 $BENCH > "$OUT/fetch.json"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/write" -o run --output-format csv -- python3 $BENCH > "$OUT/write.json"
python3 "$ROOT/tools/pmc_summary.py" "$OUT" "$TAG"
