#!/bin/bash
# K5 variants on the fresh curriculum (GPU box): GPU fresh tests on the product build, then per variant
# (tools/_abl/libd2d_var_<tag>.so) the fresh step time (tools/fresh_probe.py, two interleaved rounds)
# and K5 stamps of the given stamp builds.  Usage: bash tools/gpu_k5ab.sh TAG "VARIANTS" "STAMP_BUILDS"
set -u
O=gpurun_out/$1; V=$2; SB=${3:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fresh.py tests/test_ppo.py tests/test_curriculum.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest_fresh.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_fresh.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do for v in $V; do
  timeout -k 10 300 python3 tools/fresh_probe.py 65536 300 tools/_abl/libd2d_var_$v.so > $O/probe_${v}_$r.log 2>&1 || exit 1
  echo "$v: $(tail -1 $O/probe_${v}_$r.log)"
done; done
for b in $SB; do timeout -k 10 300 python tools/gen_stamps.py tools/_abl/libd2d_var_$b.so > $O/gen_stamps_$b.json 2>&1 || exit 1; done
exit 0
