set -e
O=gpurun_out/rm2
mkdir -p $O
timeout -k 10 400 python tools/variants.py run rm0 rm1 --rounds 6 --scenario mixed > $O/v_mixed.log 2>&1
timeout -k 10 300 python tools/variants.py run rm0 rm1 --rounds 4 --scenario corridor > $O/v_corridor.log 2>&1
grep -h '"scenario"\|ms_per_step_min\|ms_per_step_all' $O/v_*.log
