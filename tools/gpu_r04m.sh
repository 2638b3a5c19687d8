# round 4: GPU suite on the tree, the fresh-curriculum bench line and kernel split (GPU box)
set -u
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log
grep FAILED $O/pytest_gpu.log | head -5
timeout -k 10 300 python bench.py --scenario curriculum > $O/bench_curriculum.log 2>&1 || { echo STOP bench; exit 1; }
tail -1 $O/bench_curriculum.log | cut -c1-400
bash tools/gpu_fresh.sh r04m drone-2d-custom-gym-env-for-reinforcement-learning_amd/_lib/libdrone2d_hip.so
