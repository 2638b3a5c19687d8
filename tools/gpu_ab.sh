#!/bin/bash
# A/B of tools/_abl/libd2d_var_<tag>.so builds plus the GPU suite on the current tree (GPU box).
# Usage: bash tools/gpu_ab.sh OUTTAG TAG... [-- extra]   (env: NOTEST=1 skips pytest, TRAFFIC=1 adds
# the FETCH / WRITE / lane-utilisation passes of the current tree)
set -u
O=gpurun_out/$1; shift
TAGS="$*"
mkdir -p $O
export TMPDIR=/tmp
[ -x tools/ubench_lat ] && { timeout -k 10 60 ./tools/ubench_lat > $O/lat.json 2>&1 || exit 1; cat $O/lat.json; }
if [ "${NOTEST:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
fi
timeout -k 10 600 python tools/variants.py run $TAGS --envs 65536 --scenario corridor --rounds 3 > $O/ab_corridor.log 2>&1 || exit 1
timeout -k 10 600 python tools/variants.py run $TAGS --envs 65536 --scenario S_corridor --rounds 2 > $O/ab_S_corridor.log 2>&1 || exit 1
timeout -k 10 400 python tools/variants.py run $TAGS --envs 4096 --scenario corridor_free --rounds 3 > $O/ab_small.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 || exit 1
timeout -k 10 200 python bench.py > $O/bench.log 2>&1 || exit 1
timeout -k 10 300 python tools/stamps.py run --scenario corridor > $O/stamps.json 2>&1 || exit 1
if [ "${TRAFFIC:-0}" = 1 ]; then bash tools/gpu_traffic.sh $(basename $O) > $O/traffic.log 2>&1 || exit 1; fi
exit 0
