export PYTHONPATH=$PWD
timeout -k 10 300 python benchmarks/selfplay_dp_benchmark.py --playouts 1600 --moves 2 > gpurun_out/selfplay_1600.log 2>&1; tail -1 gpurun_out/selfplay_1600.log
ALPHAGO_AMD_PRECISION=fp8 timeout -k 10 300 python benchmarks/selfplay_dp_benchmark.py --playouts 1600 --moves 2 > gpurun_out/selfplay_1600_fp8.log 2>&1; tail -1 gpurun_out/selfplay_1600_fp8.log
timeout -k 10 300 python benchmarks/value_training_benchmark.py > gpurun_out/value_bench.log 2>&1; tail -1 gpurun_out/value_bench.log
