#!/bin/bash
# A/B GPU session (GPU box): driver-style first 20/5 line, GPU suite, A/B of tools/_abl variant
# builds, default bench, rocprofv3 kernel-trace summary.  Each GPU step under its own timeout; a
# crash / abort / timeout ends the script (test failures, rc 1, do not).
# Usage: bash tools/gpu_ab.sh OUTTAG [VARIANT_TAG...]   env: NOTEST=1, NOPROF=1, AB_SCN="corridor S_corridor"
set -u
O=gpurun_out/$1; shift
TAGS="$*"
mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
fail() { echo "STOP at $1 (rc $2)"; exit $2; }
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_k20_first.log 2>&1 || fail bench_k20_first $?
tail -1 $O/bench_k20_first.log
if [ "${NOTEST:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -le 1 ] || fail pytest $rc
fi
if [ -n "$TAGS" ]; then
  for scn in ${AB_SCN:-corridor S_corridor}; do
    timeout -k 10 600 python tools/variants.py run $TAGS --envs 65536 --scenario $scn --rounds 3 > $O/ab_$scn.log 2>&1 || fail ab_$scn $?
    python - $O/ab_$scn.log <<'PY'
import json, sys
t = open(sys.argv[1]).read(); d = json.loads(t[t.index("{"):])
print(d["scenario"], {k: round(v["ms_per_step_min"] * 1e3, 2) for k, v in d["variants"].items()})
PY
  done
fi
timeout -k 10 200 python bench.py > $O/bench.log 2>&1 || fail bench $?
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 || fail bench_k20 $?
if [ "${NOPROF:-0}" != 1 ]; then
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/$O/kt -o kt -- python3 $R/bench.py --no-cpu-baseline > $R/$O/kt.log 2>&1) || fail rocprof $?
  find $O/kt -name '*kernel_stats.csv' -exec head -5 {} \;
fi
exit 0
