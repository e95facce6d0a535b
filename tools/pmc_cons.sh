#!/bin/bash
# GPU box: FETCH_SIZE / WRITE_SIZE passes over the config-4 consolidation leg only (consolidate_kernel traffic)
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmc_cons_${1:-r04}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 --no-topology --no-reserved --no-launch --no-consolidation-replace"
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/fetch" -o run --output-format csv -- python3 $B > "$OUT/fetch.json"
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/write" -o run --output-format csv -- python3 $B > "$OUT/write.json"
