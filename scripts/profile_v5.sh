set -e
bash scripts/profile_step.sh gpurun_out/prof5 --steps 20 --warmup 15 > gpurun_out/prof5.log 2>&1
f=$(find gpurun_out/prof5 -name "*kernel_trace.csv" | head -1)
python scripts/timeline.py $f 5 > gpurun_out/timeline5.txt
f2=$(find gpurun_out/prof5 -name "*kernel_stats.csv" | head -1)
cp $f2 gpurun_out/kstats5.csv
head -3 gpurun_out/prof5.log | tail -1; cat gpurun_out/timeline5.txt
