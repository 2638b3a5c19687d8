#!/bin/bash
# One GPU-box session: parity tests, smoke, a short bench, and a rocprofv3 kernel trace.
# Every GPU step has its own time limit; a crash / fault / timeout ends the script (no retries).
# Usage (from the repo root, on the box): bash tools/gpu_check.sh [tag]
set -u
TAG=${1:-r01}
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

run() {  # run <name> <timeout-s> <cmd...>; allow exit 0/1 (test failures), stop on anything else
  local name=$1 lim=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}

run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py
run bench_k20 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
