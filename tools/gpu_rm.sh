set -e
O=gpurun_out/rm
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for sc in corridor large S_corridor mixed; do
  timeout -k 10 300 python tools/variants.py run rm0 rm1 --rounds 3 --scenario $sc > $O/v_$sc.log 2>&1
done
timeout -k 10 300 python tools/variants.py run rm0 rm1 --rounds 3 --envs 4096 --scenario corridor_free > $O/v_free4096.log 2>&1
timeout -k 10 300 python tools/fresh_probe.py 65536 300 tools/_abl/libd2d_var_rm0.so > $O/fresh_rm0.log 2>&1
timeout -k 10 300 python tools/fresh_probe.py 65536 300 tools/_abl/libd2d_var_rm1.so > $O/fresh_rm1.log 2>&1
grep -h '"scenario"\|"envs"\|ms_per_step_min' $O/v_*.log
grep -h "fresh" $O/fresh_*.log
timeout -k 10 120 ./tools/ubench_sweep > $O/sweep.txt 2>&1
cat $O/sweep.txt
timeout -k 10 300 python tools/variants.py run t0 t1 --rounds 3 > $O/v_tail.log 2>&1
grep -h 'ms_per_step_min' $O/v_tail.log
