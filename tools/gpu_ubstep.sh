#!/bin/bash
set -u
O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 120 python tools/ubench_step.py run "$@" --waves 64 > $O/ubstep_64.json 2>&1 || exit 1
timeout -k 10 120 python tools/ubench_step.py run "$@" --waves 4096 > $O/ubstep_4096.json 2>&1 || exit 1
tail -1 $O/ubstep_64.json; tail -1 $O/ubstep_4096.json
