#!/bin/bash
# rocprofv3 evidence for the bench workload (run on the GPU box from the repo root):
#   1. kernel trace + stats (per-kernel average durations)
#   2. separate --pmc passes: FETCH_SIZE, WRITE_SIZE, SQ wave/instruction counters
# then tools/pmc_summary.py folds them into profiles/<tag>_pmc.json (+ latest_pmc.json) and copies the
# kernel stats CSV to profiles/<tag>_kernel_stats.csv.  Usage: bash tools/profile.sh <tag>
set -o pipefail
TAG=${1:-latest}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --profile-only"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/stats" -o run -- $B > "$OUT/stats.log" 2>&1 || { echo "stats pass failed"; tail -20 "$OUT/stats.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d "$OUT/fetch" -o run -- $B > "$OUT/fetch.log" 2>&1 || { echo "fetch pass failed"; tail -20 "$OUT/fetch.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d "$OUT/write" -o run -- $B > "$OUT/write.log" 2>&1 || { echo "write pass failed"; tail -20 "$OUT/write.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -f csv -d "$OUT/sq" -o run -- $B > "$OUT/sq.log" 2>&1 || { echo "sq pass failed"; tail -20 "$OUT/sq.log"; exit 1; }
python3 tools/pmc_summary.py "$OUT" "$TAG"
