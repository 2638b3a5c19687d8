#!/bin/bash
# rocprofv3 passes on the bench workload (GPU box).  Kernel trace + stats in their own passes; PMC
# counters in separate passes (never combined with sys/runtime traces), on the eager step loop.
# Usage: bash tools/profile.sh TAG     -> gpurun_out/prof_TAG/...
set -u
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --no-cpu-baseline"
KR="--kernel-include-regex d2d_(step|fill)_kernel"

step() {  # step <name> <timeout> <cmd...>: stop on any failure
  local name=$1 lim=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 3 "$OUT/$name.log"
  echo "=== $name rc=$rc"
  [ $rc -eq 0 ] || { echo "STOP"; exit $rc; }
}

# the bench's own defaults (2 000 graph-replayed steps after 300 warmup steps)
step kt 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/kt" -o kt -- $B
step kt_graph 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/kt_graph" -o kt -- $B --graph
step pmc_fetch 600 rocprofv3 $KR -T --output-format csv -d "$OUT/pmc_fetch" -o fetch --pmc FETCH_SIZE -- $B --eager --steps 40 --warmup 300
step pmc_write 600 rocprofv3 $KR -T --output-format csv -d "$OUT/pmc_write" -o write --pmc WRITE_SIZE -- $B --eager --steps 40 --warmup 300
step pmc_sq 600 rocprofv3 $KR -T --output-format csv -d "$OUT/pmc_sq" -o sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY -- $B --eager --steps 40 --warmup 300
# the VALU instruction mix (fp64 FMA / ADD / MUL / TRANS vs 32-bit int / conversions) and the fp64 flop
# counters: the fp64 co-roofline of the bench line (tools/valu.py --mix)
step pmc_mix 600 rocprofv3 $KR -T --output-format csv -d "$OUT/pmc_mix" -o mix --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT -- $B --eager --steps 40 --warmup 300
step pmc_mix2 600 rocprofv3 $KR -T --output-format csv -d "$OUT/pmc_mix2" -o mix2 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_WAVES -- $B --eager --steps 40 --warmup 300
# VALU lane utilisation (thread-cycles over 64 x VALU-issue cycles): the fp64 flops over active lanes
step pmc_util 600 rocprofv3 $KR -T --output-format csv -d "$OUT/pmc_util" -o util --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES -- $B --eager --steps 40 --warmup 300
step pmc_clk 600 rocprofv3 $KR -T --output-format csv -d "$OUT/pmc_clk" -o clk --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -- $B --eager --steps 40 --warmup 300
python3 "$R/tools/traffic.py" "$OUT" --out "$OUT/traffic.json"
python3 "$R/tools/valu.py" "$OUT"/pmc_sq/sq_counter_collection.csv --mix "$OUT"/pmc_mix/mix_counter_collection.csv "$OUT"/pmc_mix2/mix2_counter_collection.csv --util "$OUT"/pmc_util/util_counter_collection.csv --out "$OUT/valu.json"
