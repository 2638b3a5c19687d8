set -u
O=gpurun_out/r05g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fresh.py tests/test_ppo.py -x -q --timeout 200 --timeout-method thread -k "fresh or rollout" > $O/pytest_fresh.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_fresh.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline --scenario curriculum > $O/bench_curriculum.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/fresh_probe.py 65536 300 drone-2d-custom-gym-env-for-reinforcement-learning_amd/_lib/libdrone2d_hip.so > $O/fresh_probe.log 2>&1 || exit 1
tail -1 $O/fresh_probe.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_fresh -o kt -- python3 $GRAFT_REPO_ROOT/tools/fresh_probe.py 65536 200 $GRAFT_REPO_ROOT/drone-2d-custom-gym-env-for-reinforcement-learning_amd/_lib/libdrone2d_hip.so > $GRAFT_REPO_ROOT/$O/kt_fresh.log 2>&1) || exit 1
for cw in 100 300 1000; do for r in 1 2; do timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --clock-warmup-ms $cw > $O/k20_cw${cw}_$r.log 2>&1 || exit 1; done; done
