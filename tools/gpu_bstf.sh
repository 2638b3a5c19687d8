#!/bin/bash
set -u
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python tools/bstamps.py run --scenario curriculum --envs 65536 > $O/bst_fresh.json 2>&1 || exit 1
tail -c 1500 $O/bst_fresh.json
