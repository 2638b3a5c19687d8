#!/bin/bash
# Fresh-curriculum probes (GPU box): wall time per step and the rocprofv3 kernel split for each
# library given (tools/variants.py builds).  Usage: bash tools/gpu_fresh.sh TAG LIB...
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/fresh_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for L in "$@"; do
  b=$(basename "$L" .so)
  timeout -k 10 300 python3 "$R/tools/fresh_probe.py" 65536 300 "$R/$L" > "$OUT/$b.log" 2>&1 || { echo "STOP $b"; exit 1; }
  tail -1 "$OUT/$b.log"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/kt_$b" -o kt -- \
     python3 "$R/tools/fresh_probe.py" 65536 200 "$R/$L" > "$OUT/kt_$b.log" 2>&1) || { echo "STOP kt $b"; exit 1; }
  f=$(find "$OUT/kt_$b" -name '*kernel_stats.csv' | head -1); cut -d, -f1-7 "$f" | head -6
done
