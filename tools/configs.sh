#!/bin/bash
# bench.py on every single-GPU BASELINE.json config (GPU box); one JSON line per config into
# gpurun_out/configs_TAG.jsonl.  Each run has its own time limit; any failure ends the script.
# Usage: bash tools/configs.sh TAG
set -u
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/configs_$TAG.jsonl
: > "$OUT"
run() {  # run <label> <bench args...>
  local label=$1; shift
  echo "=== $label ($(date +%T))"
  timeout -k 10 300 python3 "$R/bench.py" --no-cpu-baseline "$@" > "$R/gpurun_out/cfg_$label.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { echo "STOP $label rc=$rc"; tail -n 5 "$R/gpurun_out/cfg_$label.log"; exit $rc; }
  grep '^{' "$R/gpurun_out/cfg_$label.log" | sed "s/^{/{\"label\": \"$label\", /" >> "$OUT"
  tail -n 1 "$OUT" | cut -c1-160
}
run cfg1_free_4096 --scenario corridor_free --envs 4096
run cfg2_corridor_65536 --scenario corridor
run cfg3_large_65536 --scenario large
run cfg3_S_corridor_65536 --scenario S_corridor
run cfg4_mixed_65536 --scenario mixed
run cfg2_free_65536 --scenario corridor_free
run cfg2_corridor_65536_graph --scenario corridor --graph
run cfg2_corridor_65536_info --scenario corridor --info
run fresh_curriculum_65536 --scenario curriculum
