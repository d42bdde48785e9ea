mkdir -p gpurun_out/r2f
timeout -k 10 300 python -u -m pytest tests/test_determinism_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2f/det.log 2>&1; echo rc=$? >> gpurun_out/r2f/det.log
timeout -k 10 300 python benchmarks/graph_step_benchmark.py --batches 16,64,256 > gpurun_out/r2f/graph_serial.jsonl 2>&1
ALPHAGO_AMD_GRAPH_OVERLAP=1 timeout -k 10 300 python benchmarks/graph_step_benchmark.py --batches 16,256 > gpurun_out/r2f/graph_overlap.jsonl 2>&1
