export PYTHONPATH=$PWD
timeout -k 10 250 python benchmarks/search_benchmark.py 64 800 32 > gpurun_out/search64.log 2>&1; tail -2 gpurun_out/search64.log
timeout -k 10 250 python benchmarks/search_benchmark.py 256 800 32 > gpurun_out/search256.log 2>&1; tail -2 gpurun_out/search256.log
ALPHAGO_AMD_PRECISION=fp8 timeout -k 10 250 python benchmarks/search_benchmark.py 256 800 32 > gpurun_out/search256f8.log 2>&1; tail -2 gpurun_out/search256f8.log
