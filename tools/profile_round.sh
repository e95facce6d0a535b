#!/bin/bash
# Round profile on the GPU box: kernel-trace stats of the bench legs, one PMC pass per TCC counter (FETCH_SIZE and
# WRITE_SIZE do not fit one pass on gfx950), SQ issue / wait passes and KPSIM_PROFILE stage cycles of the three Solve
# legs.  Every dominant kernel is covered: ffd_kernel (config 2), ffd_topo_kernel (config 3), ffd_resv_kernel
# (config 5), consolidate_kernel (config 4; and the config4-replace leg in its own runs, whose FULL variant is
# consolidate_full_kernel), launch_kernel.  Usage: tools/profile_round.sh <round-tag>
set -euo pipefail
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1"
MAIN="$BENCH --no-consolidation-replace"                          # config 2, 4, launch, 3, 5
REPL="$BENCH --no-config4 --no-launch --no-topology --no-reserved"  # config 2 + the config4-replace leg
SOLVE="$BENCH --no-consolidation --no-launch"                     # config 2, 3, 5
pass() {  # name, timeout, rocprofv3 args..., -- command
    local name=$1 lim=$2; shift 2
    echo "[profile_round] $name" >&2
    timeout -k 10 "$lim" rocprofv3 "$@" > "$OUT/$name.json"
}
pass trace 300 --kernel-trace --stats -T -d "$OUT/trace" -o run --output-format csv -- python3 $MAIN
pass trace_replace 300 --kernel-trace --stats -T -d "$OUT/trace_replace" -o run --output-format csv -- python3 $REPL
pass fetch 400 --pmc FETCH_SIZE -T -d "$OUT/fetch" -o run --output-format csv -- python3 $MAIN
pass write 400 --pmc WRITE_SIZE -T -d "$OUT/write" -o run --output-format csv -- python3 $MAIN
pass fetch_replace 300 --pmc FETCH_SIZE -T -d "$OUT/fetch_replace" -o run --output-format csv -- python3 $REPL
pass write_replace 300 --pmc WRITE_SIZE -T -d "$OUT/write_replace" -o run --output-format csv -- python3 $REPL
pass sq1 400 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM -T -d "$OUT/sq1" -o run --output-format csv -- python3 $SOLVE
pass sq2 400 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -T -d "$OUT/sq2" -o run --output-format csv -- python3 $SOLVE
# KPSIM_PROFILE stage cycles of the same Solve legs (s_memtime stamps; a separate run rocprof does not profile)
echo "[profile_round] stages" >&2
KPSIM_PROFILE=1 timeout -k 10 300 python3 $SOLVE --steps 1 --warmup 0 > "$OUT/stages.json" 2> "$OUT/stages.err"
python3 "$ROOT/tools/pmc_summary.py" "$OUT" "$TAG"
