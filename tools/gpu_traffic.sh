#!/bin/bash
# HBM traffic of the current tree's step kernel (GPU box): FETCH_SIZE and WRITE_SIZE in their own
# rocprofv3 passes on the eager bench loop, then tools/traffic.py.  Usage: bash tools/gpu_traffic.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$1
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --no-cpu-baseline"
KR="--kernel-include-regex d2d_(step|fill)_kernel"
timeout -k 10 600 rocprofv3 $KR -T --output-format csv -d "$OUT/pmc_fetch" -o fetch --pmc FETCH_SIZE -- $B --eager --steps 40 --warmup 300 > "$OUT/pmc_fetch.log" 2>&1 || exit 1
timeout -k 10 600 rocprofv3 $KR -T --output-format csv -d "$OUT/pmc_write" -o write --pmc WRITE_SIZE -- $B --eager --steps 40 --warmup 300 > "$OUT/pmc_write.log" 2>&1 || exit 1
timeout -k 10 600 rocprofv3 $KR -T --output-format csv -d "$OUT/pmc_util" -o util --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES -- $B --eager --steps 40 --warmup 300 > "$OUT/pmc_util.log" 2>&1 || exit 1
python3 "$R/tools/traffic.py" "$OUT" --out "$OUT/traffic.json"
