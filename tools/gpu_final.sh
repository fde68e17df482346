#!/bin/bash
# GPU box, end of a round: the -m gpu suite, smoke(), the default bench line, and the rocprofv3 stats + PMC passes
# of the same kernel source (profiles/latest_pmc.json for bench.py's roofline.traffic).  Usage: bash tools/gpu_final.sh <tag>
set -o pipefail
tag=${1:-final}
o=gpurun_out
mkdir -p $o
H12_FORCED_LOG=$o/${tag}_forced.log timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -rf > $o/${tag}_gputest.txt 2>&1
rc=$?
tail -2 $o/${tag}_gputest.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/${tag}_smoke.txt 2>&1 || { echo "smoke failed"; tail -5 $o/${tag}_smoke.txt; exit 1; }
tail -1 $o/${tag}_smoke.txt
bash tools/profile.sh $tag > $o/${tag}_profile.log 2>&1 || { echo "profile failed"; tail -5 $o/${tag}_profile.log; exit 1; }
echo "profile ok"
timeout -k 10 300 python -u bench.py > $o/${tag}_bench.json 2> $o/${tag}_bench.err || { echo "bench failed"; exit 1; }
tail -c 600 $o/${tag}_bench.json
exit $rc
