#!/bin/bash
# Round 4 batches R + S in one call: forward latency at small batches, fused sampling tests and RL /
# value-generate throughput, then the full GPU suite.
bash scripts/r4/batch_r.sh && bash scripts/r4/batch_s.sh
