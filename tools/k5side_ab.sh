#!/bin/bash
# Fresh curriculum: K5 on a side stream beside the next K1 (tools/patches/k5_side.patch variants,
# built by tools/variants.py) against the serial product order, alternating; then a kernel trace of
# each side variant.  Usage (GPU box): bash tools/k5side_ab.sh VARIANT...   -> gpurun_out/k5side/
set -u
mkdir -p gpurun_out/k5side
export TMPDIR=/tmp
for i in 1 2; do
  for v in base "$@"; do
    timeout -k 10 150 python tools/fresh_probe.py 65536 400 tools/_abl/libd2d_var_$v.so 2>&1 | grep -E "fresh|priority" || exit 1
  done
done
for v in "$@"; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/k5side/kt_$v -o kt -- \
    python3 tools/fresh_probe.py 65536 400 tools/_abl/libd2d_var_$v.so > gpurun_out/k5side/kt_$v.log 2>&1 || exit 1
  grep fresh gpurun_out/k5side/kt_$v.log
done
