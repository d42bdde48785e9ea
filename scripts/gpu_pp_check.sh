export PYTHONPATH=.
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -v --timeout 120 --timeout-method thread -k "${TESTK:-tile or ring or bitmask}" --deselect dummy > gpurun_out/t_pp.log 2>&1 
echo "pytest rc=$?"
tail -5 gpurun_out/t_pp.log
timeout -k 10 200 python -u scripts/lab/kbench_fwd_variants.py --tiles ${TILES:-384,11,384,11} > gpurun_out/kv2.log 2>&1
cat gpurun_out/kv2.log | grep -v amdgpu.ids
