#!/bin/bash
# Fresh-curriculum check on the GPU box: the fresh / pool / curriculum GPU tests, step-time probes of
# the product library against tools/_abl/ variants, 8 PPO updates and the bench line on the fresh
# curriculum.  Usage: bash tools/gpu_check_fresh.sh TAG [variant.so ...]
set -u
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fresh.py tests/test_gpu_pool.py tests/test_curriculum.py -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
grep -q " passed" $O/pytest.log && ! grep -q "failed\| error" $O/pytest.log || { echo STOP tests; exit 1; }
bash tools/gpu_fresh.sh $TAG drone-2d-custom-gym-env-for-reinforcement-learning_amd/_lib/libdrone2d_hip.so "$@" || exit 1
timeout -k 10 250 python -u tools/train_ppo.py --curriculum --pool 0 --updates 8 > $O/ppo_fresh.jsonl 2> $O/ppo_fresh.err || { echo STOP ppo; exit 1; }
tail -2 $O/ppo_fresh.jsonl | cut -c1-300
timeout -k 10 300 python bench.py --scenario curriculum --no-cpu-baseline > $O/bench_curriculum.log 2>&1 || { echo STOP bench; exit 1; }
grep '^{' $O/bench_curriculum.log | cut -c1-200
