#!/bin/bash
# Round-6 batch 4: small-batch SL -- eager vs graph step at B = 16, the reduce stream, the merged
# split-K reduce (one launch per backward) vs one reduce per layer, and the headline's split count.
O=gpurun_out/r6/b4
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
B="--steps 200 --warmup 50 --data random --pool 8192 --min-warmup-s 2"
step merged_test 300 python -u -m pytest tests/test_hip_trainer.py -x -v --timeout 120 --timeout-method thread -k merged_reduce
step b16_eager 120 python bench.py --batch 16 $B
step b16_graph 120 python bench.py --batch 16 --graph $B
step b16_rs 120 python bench.py --batch 16 --reduce-stream 1 $B
for rep in 1 2; do
  for b in 16 32 64 128; do
    for m in 0 1; do
      step mr${b}_m${m}_r$rep 120 python bench.py --batch $b --merged-reduce $m $B
    done
  done
done
step b16_graph_m1 120 python bench.py --batch 16 --graph --merged-reduce 1 $B
prof prof16_m1 180 20 --batch 16 --merged-reduce 1 --steps 40 --warmup 20 --data random --pool 8192
for rep in 1 2; do
  for w in 0 256; do
    step head_w${w}_r$rep 150 python bench.py --wgrad-wgs $w --steps 30 --warmup 10
  done
  step head_m1_r$rep 150 python bench.py --merged-reduce 1 --steps 30 --warmup 10
done
python3 - $O <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.log"))):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); c = d["config"]
            print(os.path.basename(f), c["per_gpu_batch"], c["graph"], c.get("merged_reduce"), d["value"],
                  d["ms_per_step"], d["host_ms_per_step"])
PY
