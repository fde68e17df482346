# instruction-cache counters of the bench workload + the PPO learner's kernel breakdown (GPU box, repo root)
set -o pipefail
mkdir -p gpurun_out
R=$PWD
export TMPDIR=/tmp
B="python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --profile-only"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ SQC_TC_STALL SQ_IFETCH SQ_WAVES --kernel-trace -f csv -d /tmp/icache -o run -- $B > gpurun_out/r4h_icache.log 2>&1 || { echo "icache pass failed"; tail -5 gpurun_out/r4h_icache.log; }
find /tmp/icache -name "*counter_collection*" -exec cp {} gpurun_out/r4h_icache_counters.csv \;
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_IFETCH_LEVEL SQ_WAVES --kernel-trace -f csv -d /tmp/sqw -o run -- $B > gpurun_out/r4h_sqw.log 2>&1 || { echo "sq pass failed"; tail -5 gpurun_out/r4h_sqw.log; }
find /tmp/sqw -name "*counter_collection*" -exec cp {} gpurun_out/r4h_sqw_counters.csv \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/train -o train -- python3 bench.py --mode train --iterations 3 --no-cpu-baseline > gpurun_out/r4h_train.log 2>&1 || echo "train prof failed"
find /tmp/train -name "*kernel_stats*" -exec cp {} gpurun_out/r4h_train_kernel_stats.csv \;
ls -la gpurun_out
echo done
