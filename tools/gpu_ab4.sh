#!/bin/bash
# Interleaved A/B of variant builds on four 65 536-env configs (GPU box).  Usage: bash tools/gpu_ab4.sh TAG A B
set -u
O=gpurun_out/$1; shift; mkdir -p $O
for sc in corridor S_corridor large mixed; do
  timeout -k 10 400 python tools/variants.py run "$@" --envs 65536 --scenario $sc --rounds 2 > $O/ab_$sc.log 2>&1 || exit 1
  grep -h ms_per_step_min $O/ab_$sc.log
done
exit 0
