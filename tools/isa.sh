#!/bin/bash
# Device assembly of the product library + per-kernel resource summary (CPU container).
# Usage: bash tools/isa.sh [out.s] [extra hipcc flags...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-/tmp/d2d_isa.s}; shift || true
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -Wall -Werror \
  -Wno-unused-command-line-argument -I"$R/include" --cuda-device-only -S -o "$OUT" "$@" \
  "$R/drone-2d-custom-gym-env-for-reinforcement-learning_amd/csrc/d2d_hip.hip"
python3 - "$OUT" <<'PY'
import re, sys
t = open(sys.argv[1]).read()
for m in re.finditer(r"\.name:\s+(\S+)\n(.*?)(?=\n\s+- \.|\Z)", t, re.S):
    pass
for name in re.findall(r"^(_ZN4d2dk\w+):", t, re.M):
    blk = t[t.index(name + ":"):]
    g = lambda k: (re.search(r"; " + k + r":\s*(\d+)", blk) or [None, "?"])[1]
    print(f"{name[:60]:60s} vgpr {g('NumVgprs')} agpr {g('NumAgprs')} spill {g('ScratchSize')} lds {g('LDSByteSize') } occ {g('Occupancy')}")
PY
