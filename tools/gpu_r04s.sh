# round 4: K1 queue code out of the LDS kernels -- A/B vs the round-3 build, fresh tests, PPO on the fresh curriculum
set -u
O=gpurun_out/r04s; mkdir -p $O
bash tools/gpu_ab_envs.sh r04s 65536 'corridor mixed' fmold cur || exit 1
bash tools/gpu_ab_envs.sh r04s 4096 'corridor_free' fmold cur || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_fresh.py tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 400 python tools/train_ppo.py --curriculum --pool 0 --updates 100 > $O/ppo_fresh_100.jsonl 2> $O/ppo_fresh.err || { echo STOP ppo; tail -3 $O/ppo_fresh.err; exit 1; }
tail -2 $O/ppo_fresh_100.jsonl | cut -c1-400
