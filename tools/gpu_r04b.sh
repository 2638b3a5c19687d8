set -u
bash tools/gpu_r4.sh r04b_prune
rc=$?; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash tools/role_mix.sh base nocont r0 r1 r2 r3 > gpurun_out/role_mix.txt 2>&1
