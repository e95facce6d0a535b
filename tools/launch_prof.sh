#!/bin/bash
# rocprofv3 kernel trace of the launch leg with 1 and 2 sub-batches: per-launch launch_kernel durations vs the events.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for k in 1 2; do
KPSIM_LAUNCH_SUB=$k timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_l$k" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-consolidation --no-topology --no-reserved --steps 10 --warmup 2 > "$R/gpurun_out/blp$k.json" 2> "$R/gpurun_out/blp$k.err" || exit 1
python3 -c "
import json; l=json.load(open('$R/gpurun_out/blp$k.json'))['launch']; print('sub $k', 'kernel %.3f call %.3f' % (l['kernel_ms'], l['call_ms']))"
f=$(find "$R/gpurun_out/prof_l$k" -name "*kernel_stats.csv" | head -1); grep -i "launch_kernel" "$f"
done
