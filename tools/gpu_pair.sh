#!/bin/bash
# Two-group K1 placement A/B (GPU box): the product build (four-role workgroups) against the pair
# kernel (D2D_K1_PAIR=1) in two placement patterns, interleaved processes.
set -u
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
for sc in corridor corridor_free; do for r in 1 2; do
  timeout -k 10 300 python tools/variants.py run base --envs 65536 --scenario $sc --rounds 1 > $O/base_${sc}_$r.log 2>&1 || exit 1
  D2D_K1_PAIR=1 timeout -k 10 300 python tools/variants.py run pairold pairnew --envs 65536 --scenario $sc --rounds 1 > $O/pair_${sc}_$r.log 2>&1 || exit 1
  grep -h ms_per_step_min $O/base_${sc}_$r.log $O/pair_${sc}_$r.log | head -5
done; done
exit 0
