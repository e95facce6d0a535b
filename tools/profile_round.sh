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
# kernel-trace stats over every leg but the replace leg; each Solve leg launches its own instantiation (ffd_kernel:
# config 2, ffd_topo_kernel: config 3, ffd_resv_kernel: config 5), so per-kernel rows are per-leg rows
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d "$OUT/trace" -o run --output-format csv -- python3 $BENCH --no-consolidation-replace > "$OUT/trace.json"
# the HBM passes include the config-3 leg (ffd_topo_kernel); the SQ issue / wait passes cover the two Solve legs
SOLVE="$BENCH --no-consolidation --no-launch --no-reserved"
BENCH="$BENCH --no-reserved --no-consolidation-replace"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/fetch" -o run --output-format csv -- python3 $BENCH > "$OUT/fetch.json"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/write" -o run --output-format csv -- python3 $BENCH > "$OUT/write.json"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM -T -d "$OUT/sq1" -o run --output-format csv -- python3 $SOLVE > "$OUT/sq1.json"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -T -d "$OUT/sq2" -o run --output-format csv -- python3 $SOLVE > "$OUT/sq2.json"
# KPSIM_PROFILE stage cycles of the same Solve legs (s_memtime stamps; a separate, unprofiled-by-rocprof run)
KPSIM_PROFILE=1 timeout -k 10 300 python3 $SOLVE --steps 1 --warmup 0 > "$OUT/stages.json" 2> "$OUT/stages.err"
python3 "$ROOT/tools/pmc_summary.py" "$OUT" "$TAG"
