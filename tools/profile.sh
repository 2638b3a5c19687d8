#!/bin/bash
# rocprofv3 passes on the bench workload (GPU box).  Kernel trace + stats in one pass; PMC counters
# in their own passes (never combined with sys/runtime traces).  Usage: bash tools/profile.sh TAG
set -u
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --no-cpu-baseline"
KR="--kernel-include-regex d2d_step_kernel"

step() {  # step <name> <timeout> <cmd...>: stop on any failure
  local name=$1 lim=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 5 "$OUT/$name.log"
  echo "=== $name rc=$rc"
  [ $rc -eq 0 ] || { echo "STOP"; exit $rc; }
}

step kt 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/kt" -o kt -- $B --steps 300 --warmup 30
step pmc_sq 600 rocprofv3 $KR -T --output-format csv -d "$OUT/pmc_sq" -o sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY -- $B --steps 20 --warmup 5
step pmc_fetch 600 rocprofv3 $KR -T --output-format csv -d "$OUT/pmc_fetch" -o fetch --pmc FETCH_SIZE -- $B --steps 20 --warmup 5
step pmc_write 600 rocprofv3 $KR -T --output-format csv -d "$OUT/pmc_write" -o write --pmc WRITE_SIZE -- $B --steps 20 --warmup 5
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
step pmc_clk 600 rocprofv3 $KR -T --output-format csv -d "$OUT/pmc_clk" -o clk --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -- $B --steps 20 --warmup 5
step pmc_sq2 600 rocprofv3 $KR -T --output-format csv -d "$OUT/pmc_sq2" -o sq2 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 -- $B --steps 20 --warmup 5
