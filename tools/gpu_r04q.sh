# round 4: dual-layout library -- GPU suite, layout A/B against the round-3 field-major build, fresh probe
set -u
O=gpurun_out/r04q; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log; grep FAILED $O/pytest_gpu.log | head -5
bash tools/gpu_ab_envs.sh r04q 65536 'mixed corridor large' fmold cur || exit 1
bash tools/gpu_ab_envs.sh r04q 4096 'corridor_free' fmold cur || exit 1
bash tools/gpu_fresh.sh r04q drone-2d-custom-gym-env-for-reinforcement-learning_amd/_lib/libdrone2d_hip.so
