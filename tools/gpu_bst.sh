#!/bin/bash
# Brent-step phase stamps (tools/bstamps.py) and K1 phase stamps (tools/stamps.py) at small and full batch.
set -u
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/bstamps.py run --scenario corridor_free --envs 4096 > $O/bst_small.json 2>&1 || exit 1
timeout -k 10 300 python tools/bstamps.py run --scenario corridor --envs 65536 > $O/bst_corridor.json 2>&1 || exit 1
timeout -k 10 300 python tools/stamps.py run --scenario corridor_free --envs 4096 > $O/stamps_small.json 2>&1 || exit 1
exit 0
