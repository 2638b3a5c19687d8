#!/bin/bash
# Fresh-curriculum check on the GPU box: the fresh / pool / curriculum GPU tests, step-time probes of
# the product library against tools/_abl/ variants, and 8 PPO updates on the fresh curriculum.
# Usage: bash tools/gpu_check_fresh.sh TAG [variant.so ...]
set -u
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fresh.py tests/test_gpu_pool.py tests/test_curriculum.py -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
grep -q " passed" $O/pytest.log && ! grep -q "failed\|error" $O/pytest.log || { echo STOP tests; exit 1; }
bash tools/gpu_fresh.sh $TAG drone-2d-custom-gym-env-for-reinforcement-learning_amd/_lib/libdrone2d_hip.so "$@" || exit 1
timeout -k 10 250 python -u tools/train_ppo.py --curriculum --pool 0 --updates 8 > $O/ppo_fresh.jsonl 2> $O/ppo_fresh.err || { echo STOP ppo; exit 1; }
tail -2 $O/ppo_fresh.jsonl | cut -c1-300
# the Brent-step stamps of the small batch (configs[1]) and the headline batch (diagnostic build)
timeout -k 10 200 python -u tools/bstamps.py run --scenario corridor_free --envs 4096 --out $O/bstamps_corridor_free_4096.json > $O/bstamps_4096.log 2>&1 || { echo STOP bst; exit 1; }
timeout -k 10 200 python -u tools/bstamps.py run --scenario corridor --envs 65536 --out $O/bstamps_corridor_65536.json > $O/bstamps_65536.log 2>&1 || { echo STOP bst2; exit 1; }
tail -1 $O/bstamps_4096.log; tail -1 $O/bstamps_65536.log
# knot-scan address-space A/B (D2D_KS_OFF)
timeout -k 10 300 python -u tools/variants.py run base ks --envs 65536 --rounds 3 > $O/var_ks_65536.log 2>&1 || { echo STOP var; exit 1; }
timeout -k 10 200 python -u tools/variants.py run base ks --envs 4096 --scenario corridor_free --rounds 3 > $O/var_ks_4096.log 2>&1 || { echo STOP var2; exit 1; }
grep -A3 '"base"\|"ks"' $O/var_ks_65536.log | grep min; grep -A3 '"base"\|"ks"' $O/var_ks_4096.log | grep min
bash tools/gpu_fresh.sh ${TAG}ks tools/_abl/libd2d_var_ks.so || exit 1
