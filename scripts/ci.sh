#!/bin/bash
# CI entry point (reference: .travis.yml flake8 + unittest discover).
# CPU: build native code, byte-compile everything, run the non-GPU tests.
# GPU (optional, on an MI355X box): CI_GPU=1 scripts/ci.sh also runs -m gpu and smoke().
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD
python -c "import __graft_entry__ as g; g.build()"
python -m compileall -q alphago_amd tests benchmarks bench.py __graft_entry__.py
if python -c "import flake8" 2>/dev/null; then python -m flake8 --max-line-length 120 alphago_amd; fi
python -m pytest tests -q -m "not gpu"   # includes the ASan/UBSan/TSan engine self-tests
if [ "${CI_GPU:-0}" = "1" ]; then
  timeout -k 10 900 python -m pytest tests -q -m gpu
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
