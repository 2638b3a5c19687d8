#!/bin/bash
# Eager host path (GPU box): tools/eager_probe.py, the eager bench line, the GPU suite.  Usage: bash tools/gpu_eager.sh [TAG]
set -u
O=gpurun_out/${1:-eager}; mkdir -p $O
timeout -k 10 200 python tools/eager_probe.py > $O/probe.json 2>&1 || exit 1
tail -1 $O/probe.json
timeout -k 10 200 python bench.py --eager --no-cpu-baseline > $O/bench_eager.log 2>&1 || exit 1
grep -h '"value"' $O/bench_eager.log | cut -c1-200
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_gpu.log; exit $rc
