#!/bin/bash
# rocprofv3 host-trap PC sampling of one config2 Solve (ffd_kernel hot instructions); samples under gpurun_out/pcs.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval ${PCS_INTERVAL:-10} -d "$R/gpurun_out/pcs" -o run --output-format csv -- python3 "$R/tools/prof_solve.py" config2 50000 > "$R/gpurun_out/pcs.log" 2>&1 || { tail -20 "$R/gpurun_out/pcs.log"; exit 1; }
ls -la "$R/gpurun_out/pcs"
find "$R/gpurun_out/pcs" -name "*.csv" -exec sh -c 'echo "== $1"; head -3 "$1"; wc -l "$1"' _ {} \;
