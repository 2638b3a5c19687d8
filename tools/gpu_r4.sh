#!/bin/bash
# Round-4 GPU session: parity tests, smoke, benches (driver's 20/5 and steady state), then the
# rocprofv3 passes (kernel trace; PMC bytes, SQ, VALU mix) of tools/profile.sh.
# Every GPU step has its own time limit; a crash / fault / timeout ends the script (no retries).
# Usage: bash tools/gpu_r4.sh TAG   (SKIP_TESTS=1: benches + profile only; SKIP_PROF=1: no profile)
set -u
TAG=${1:-r04}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <name> <timeout-s> <cmd...>: allow 0/1 (test failures), stop on anything else
  local name=$1 lim=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 6 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
if [ "${SKIP_TESTS:-0}" = 0 ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
run bench_k20 300 python bench.py --steps 20 --warmup 5
run bench 400 python bench.py --no-cpu-baseline
if [ "${CONFIGS:-0}" = 1 ]; then
  run cfg_free4096 300 python bench.py --scenario corridor_free --envs 4096 --no-cpu-baseline
  run cfg_large 300 python bench.py --scenario large --no-cpu-baseline
  run cfg_S_corridor 300 python bench.py --scenario S_corridor --no-cpu-baseline
  run cfg_mixed 300 python bench.py --scenario mixed --no-cpu-baseline
fi
if [ "${SKIP_PROF:-0}" = 0 ]; then
  run profile 1100 bash tools/profile.sh "$TAG"
fi
