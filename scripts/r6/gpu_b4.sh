#!/bin/bash
# Round-6 batch 4: small-batch SL with the split-free wgrad: same-box A/B of
# --wgrad-direct 0/1, eager vs graph step at B = 16, the batch sweep, and a B = 16 kernel timeline.
O=gpurun_out/r6/b4
mkdir -p $O
export PYTHONUNBUFFERED=1
source scripts/r6/lib.sh
B="--steps 200 --warmup 50 --data random --pool 8192 --min-warmup-s 2"
for rep in 1; do
  for d in 0 1; do
    step b16_d${d}_r$rep 120 python bench.py --batch 16 --wgrad-direct $d $B
    step b16g_d${d}_r$rep 120 python bench.py --batch 16 --wgrad-direct $d --graph $B
  done
  step b16_rs_r$rep 120 python bench.py --batch 16 --reduce-stream 1 $B
done
for b in 1 4 8 32; do
  for d in 0 1; do
    step b${b}_d$d 120 python bench.py --batch $b --wgrad-direct $d $B
  done
done
prof prof4_direct 180 20 --batch 4 --wgrad-direct 1 --steps 40 --warmup 20 --data random --pool 8192
prof prof4_splitk 180 20 --batch 4 --wgrad-direct 0 --steps 40 --warmup 20 --data random --pool 8192
python3 - $O <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "b*.log"))):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); c = d["config"]
            print(os.path.basename(f), c["per_gpu_batch"], c["graph"], c.get("wgrad_direct"), d["value"],
                  d["ms_per_step"], d["host_ms_per_step"])
PY
# headline: fewer wgrad splits (smaller split-K slab, fewer resident waves), same box, alternating
for rep in 1 2; do
  for w in 0 256; do
    step head_w${w}_r$rep 150 python bench.py --wgrad-wgs $w --steps 30 --warmup 10
  done
done
grep -h '"value"' $O/head_*.log | cut -c1-120
