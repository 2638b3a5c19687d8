set -e
mkdir -p gpurun_out/ub
timeout -k 10 120 ./tools/ubench_sweep > gpurun_out/ub/sweep.txt 2>&1
cat gpurun_out/ub/sweep.txt
timeout -k 10 300 python tools/variants.py run t0 t1 --rounds 4 > gpurun_out/ub/v_tail.log 2>&1
timeout -k 10 300 python tools/variants.py run t0 t1 --rounds 3 --scenario S_corridor > gpurun_out/ub/v_tail_S.log 2>&1
grep -h '"scenario"\|ms_per_step_min' gpurun_out/ub/v_tail*.log
