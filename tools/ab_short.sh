#!/bin/bash
# Diagnostic (GPU box): the bench line with captured graphs vs eager launches, alternating on one
# box.  Usage: bash tools/ab_short.sh STEPS WARMUP ROUNDS OUTTAG
S=${1:-20}; W=${2:-5}; N=${3:-5}; O=gpurun_out/${4:-ab_short}
mkdir -p $O
for r in $(seq 1 $N); do
  for m in graph eager; do
    if [ $m = eager ]; then X=; else X=--graph; fi
    timeout -k 10 200 python bench.py --steps $S --warmup $W --no-cpu-baseline $X > $O/b_${m}_$r.log 2>&1 || exit 1
  done
done
for f in $O/b_*.log; do tail -1 $f | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$f', round(d['value']/1e9,3), round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), d['gpu_clock']['before_timed']['pp_dpm_sclk_mhz'], d['gpu_clock']['after_timed']['pp_dpm_sclk_mhz'])"; done
