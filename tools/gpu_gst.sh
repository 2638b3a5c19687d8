#!/bin/bash
# K5 (fresh-curriculum generator) phase stamps of a D2D_GEN_STAMPS build (GPU box).
set -u
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python tools/gen_stamps.py tools/_abl/libd2d_var_gst.so > $O/gen_stamps.json 2>&1 || exit 1
tail -c 2500 $O/gen_stamps.json
