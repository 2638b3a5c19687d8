#!/bin/bash
# Spread of the driver-shaped bench line (20 timed steps after 5 warm-up steps) on one box:
# N plain runs, then N runs under a kernel trace whose per-launch K1 durations show whether a slow
# run is uniformly slow or carries a few slow launches (tools/k20_probe.py reads the CSVs).
# Usage (GPU box): bash tools/k20_probe.sh TAG [N]   -> gpurun_out/k20_TAG/
set -u
TAG=${1:-r06}
N=${2:-4}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/k20_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for i in $(seq 1 "$N"); do
  timeout -k 10 120 python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/plain_$i.log" 2>&1 \
    || { echo "STOP plain_$i"; exit 1; }
  tail -n 1 "$OUT/plain_$i.log" | cut -c1-120
done
for i in $(seq 1 "$N"); do
  timeout -k 10 180 rocprofv3 --kernel-trace -T --output-format csv -d "$OUT/kt_$i" -o kt -- \
    python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/kt_$i.log" 2>&1 \
    || { echo "STOP kt_$i"; exit 1; }
  tail -n 1 "$OUT/kt_$i.log" | cut -c1-120
done
python3 "$R/tools/k20_probe.py" "$OUT" | tee "$OUT/summary.txt"
