#!/bin/bash
# Round-5 A/B session (GPU box): the two-group K1 (D2D_K1_PAIR=1) and the exact-trig build against
# the default library -- parity first (the pair kernel under the GPU parity suite, the exact build's
# closed-loop identity test), then interleaved benches.  Any failure other than a test failure ends
# the script.   Usage: bash tools/gpu_pair_ab.sh [TAG]
set -u
TAG=${1:-r05c}
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
D2D_K1_PAIR=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_closed_loop.py -x -q --timeout 200 --timeout-method thread > $O/pytest_pair.log 2>&1; rc=$?; echo "pytest_pair rc=$rc"; tail -2 $O/pytest_pair.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_harness.py -x -q -k "exact_trig or hip_matches" --timeout 200 --timeout-method thread > $O/pytest_exact.log 2>&1; rc=$?; echo "pytest_exact rc=$rc"; tail -2 $O/pytest_exact.log; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
 for s in corridor large S_corridor corridor_free; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --scenario $s > $O/base_${s}_$r.log 2>&1 || exit 1
  D2D_K1_PAIR=1 timeout -k 10 120 python bench.py --no-cpu-baseline --scenario $s > $O/pair_${s}_$r.log 2>&1 || exit 1
 done
 timeout -k 10 120 python bench.py --no-cpu-baseline --exact-trig > $O/exact_corridor_$r.log 2>&1 || exit 1
done
D2D_K1_PAIR=1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/pair_k20.log 2>&1 || exit 1
cd /tmp && D2D_K1_PAIR=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_pair -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/kt_pair.log 2>&1
