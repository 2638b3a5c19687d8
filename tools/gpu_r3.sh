#!/bin/bash
# Round-3 GPU session: parity tests, smoke, benches (driver's 20/5 and steady state), kernel trace.
# Every GPU step has its own time limit; a crash / fault / timeout ends the script (no retries).
set -u
TAG=${1:-r03}
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
SKIP_TESTS=${SKIP_TESTS:-0}
ONLY_PROF=${ONLY_PROF:-0}
if [ "$SKIP_TESTS" = 0 ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
run bench_k20 300 python bench.py --steps 20 --warmup 5
run bench 400 python bench.py --no-cpu-baseline
run bench_free4096 300 python bench.py --scenario corridor_free --envs 4096 --no-cpu-baseline
cd /tmp
run kt_k20 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/kt_k20" -o kt -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline
if [ "${PLACE:-0}" = 1 ]; then
  cd "$R"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -o /tmp/ubench_place tools/ubench_place.hip && \
  run place 120 /tmp/ubench_place
fi
