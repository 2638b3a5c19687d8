#!/bin/bash
# The fresh curriculum after a K5 change (GPU box): its GPU tests, the curriculum bench, K5 stamps and a
# kernel trace of the fresh step loop.  Usage: bash tools/gpu_fresh_k5.sh TAG
set -u
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fresh.py tests/test_ppo.py tests/test_curriculum.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/pytest_fresh.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_fresh.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --scenario curriculum > $O/bench_curriculum.log 2>&1 || exit 1
timeout -k 10 300 python tools/gen_stamps.py tools/_abl/libd2d_var_gst.so > $O/gen_stamps.json 2>&1 || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_fresh -o kt -- python3 $GRAFT_REPO_ROOT/tools/fresh_probe.py 65536 200 $GRAFT_REPO_ROOT/drone-2d-custom-gym-env-for-reinforcement-learning_amd/_lib/libdrone2d_hip.so > $GRAFT_REPO_ROOT/$O/kt_fresh.log 2>&1) || exit 1
grep -h '"value"' $O/bench_curriculum.log | cut -c1-200
