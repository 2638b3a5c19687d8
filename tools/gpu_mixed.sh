#!/bin/bash
# Mixed-batch placement session: parity of the balanced layout, the mixed bench, the per-CU trace.
set -u
R=$(pwd); O=$R/gpurun_out/${1:-mixed}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "balanced or mixed or grouped or layout" > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --scenario mixed --no-cpu-baseline > $O/bench_mixed.log 2>&1 || exit $?
tail -1 $O/bench_mixed.log | cut -c1-400
timeout -k 10 200 python3 tools/cu_map.py --scenario mixed --out $O/mixed.npz || exit $?
