#!/bin/bash
# GPU session (bash tools/gpu_session.sh TAG): parity suite, smoke, benches (driver's 20/5, steady
# state, every BASELINE config + the fresh curriculum), rocprofv3 kernel trace + PMC passes of the
# headline, the fresh curriculum's kernel split, PPO on corridor and on the fresh curriculum.
# Every GPU step has its own time limit; a crash / fault / timeout ends the script (no retries).
set -u
TAG=${1:-r05}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
SKIP=" ${SKIP:-} "  # names of steps to skip, e.g. SKIP="profile ppo_corridor"
run() {  # run <name> <timeout-s> <cmd...>: allow 0/1 (test failures), stop on anything else
  local name=$1 lim=$2; shift 2
  case "$SKIP" in *" $name "*) echo "=== $name skipped"; return 0;; esac
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 3 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_k20 300 python bench.py --steps 20 --warmup 5
run bench 400 python bench.py
run configs 900 bash tools/configs.sh "$TAG"
run profile 1100 bash tools/profile.sh "$TAG"
run fresh 600 bash tools/gpu_fresh.sh "$TAG" drone-2d-custom-gym-env-for-reinforcement-learning_amd/_lib/libdrone2d_hip.so
run ppo_corridor 600 python tools/train_ppo.py --updates 60
case "$SKIP" in *" ppo_corridor "*) ;; *) cp gpurun_out/ppo.jsonl "$OUT/ppo_corridor_60.jsonl";; esac
run ppo_fresh 600 python tools/train_ppo.py --curriculum --pool 0 --updates 100
case "$SKIP" in *" ppo_fresh "*) ;; *) cp gpurun_out/ppo.jsonl "$OUT/ppo_fresh_100.jsonl";; esac
