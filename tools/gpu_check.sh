#!/bin/bash
# Quick GPU check of the current tree (GPU box): the GPU suite, two default benches, the driver's
# 20 / 5 line, every BASELINE config, and the K1 phase timeline (tools/stamps.py, diagnostic build
# in tools/_abl).  Any failure other than a test failure ends the script.
# Usage: bash tools/gpu_check.sh TAG
set -u
TAG=${1:-check}
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
for r in 1 2; do timeout -k 10 200 python bench.py > $O/bench_$r.log 2>&1 || exit 1; done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 || exit 1
timeout -k 10 900 bash tools/configs.sh $TAG > $O/configs.log 2>&1 || exit 1
[ -f tools/_abl/libd2d_stamps.so ] && { timeout -k 10 300 python tools/stamps.py run --scenario corridor > $O/stamps.json 2>&1 || exit 1; }
exit 0
