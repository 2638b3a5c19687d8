set -u
for v in gst gst1w gstnt; do
  timeout -k 10 200 python tools/gen_stamps.py tools/_abl/libd2d_var_$v.so > gpurun_out/gen_stamps_r04k_$v.json 2>gpurun_out/gen_stamps_r04k_$v.err || { echo "STOP $v"; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/gen_stamps_r04k_$v.json')); s=d['steps'][1]; print('$v', {k: s[k] for k in s if k not in ('span_first_start_to_last_end','start_spread')})"
done
bash tools/gpu_fresh.sh r04k tools/_abl/libd2d_var_base.so tools/_abl/libd2d_var_one.so tools/_abl/libd2d_var_abl1.so
