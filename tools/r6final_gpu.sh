set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6final_smoke.txt 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r6final_smoke.txt; exit 1; }
echo smoke ok
bash tools/profile.sh r6final || exit 1
timeout -k 10 300 python3 -u bench.py > gpurun_out/r6final_bench.json 2> gpurun_out/r6final_bench.err || { echo "bench failed"; tail -20 gpurun_out/r6final_bench.err; exit 1; }
tail -1 gpurun_out/r6final_bench.json | cut -c1-400
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r6final_bench20.json 2> gpurun_out/r6final_bench20.err || { echo "bench20 failed"; exit 1; }
bash tools/task_lines.sh r6final || exit 1
cat gpurun_out/r6final_task_lines.txt
