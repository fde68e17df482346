mkdir -p gpurun_out
timeout -k 5 60 ./tools/probe/tailbench 2 > gpurun_out/r4g_bigcode.txt 2>&1 || echo "tailbench failed"
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 5 100 rocprofv3 -L > /tmp/counters.txt 2>&1 || echo "list failed"
grep -o "SQC_[A-Z_0-9]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_LEVEL[A-Z_]*\|TCC_[A-Z_0-9]*" /tmp/counters.txt | sort -u > $R/gpurun_out/r4g_counters.txt
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r4g_train_prof -o train -- python3 bench.py --mode train --iterations 3 --no-cpu-baseline > gpurun_out/r4g_train.log 2>&1 || echo "train prof failed"
find /tmp/r4g_train_prof -name "*stats*" -exec cp {} gpurun_out/ \;
ls -la gpurun_out | head -30
echo done
