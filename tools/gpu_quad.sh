#!/bin/bash
# Quad-workgroup K1: parity subset, then A/B benches (D2D_QUAD=0 vs auto) on corridor / mixed / S_corridor / large.
set -u
R=$(pwd); OUT=$R/gpurun_out/${1:-quad}; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "=== $name"; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
  echo "rc=$rc"; grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|[0-9]* passed.*\|[0-9]* failed.*' "$OUT/$name.log" | tr '\n' ' '; echo
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP $name rc=$rc"; tail -20 "$OUT/$name.log"; exit $rc; fi; }
run tests 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "quad or grid_bitwise or config5 or full_size"
for scn in corridor mixed S_corridor large; do
  run b_${scn}_q0 300 env D2D_QUAD=0 python bench.py --scenario $scn --steps 1000 --warmup 300 --no-cpu-baseline
  run b_${scn}_q 300 python bench.py --scenario $scn --steps 1000 --warmup 300 --no-cpu-baseline
done
run k20_q0 300 env D2D_QUAD=0 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
run k20_q 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
