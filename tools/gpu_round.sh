#!/bin/bash
# GPU box: the -m gpu suite (forced-parity dumps + per-check log) then the default bench line.  Stops after anything
# other than a normal pytest pass / fail (a fault, abort or time limit).
set -u
tag=${1:-r3}
mkdir -p gpurun_out/dumps_$tag
export H12_FORCED_DUMP=gpurun_out/dumps_$tag H12_FORCED_LOG=gpurun_out/${tag}_forced.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -rf > gpurun_out/${tag}_gputest.txt 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
rc2=$?
echo "bench rc=$rc2"
tail -c 3000 gpurun_out/${tag}_bench.json
exit $rc2
