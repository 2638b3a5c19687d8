# round 4: fresh-curriculum checks (GPU box): generator parity tests, K5 stamps, K1 record prefetch A/B
set -u
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fresh.py tests/test_curriculum.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_fresh.log 2>&1
tail -2 $O/pytest_fresh.log
timeout -k 10 200 python tools/gen_stamps.py tools/_abl/libd2d_var_gst.so > $O/gen_stamps.json 2>$O/gen_stamps.err || { echo STOP stamps; exit 1; }
python -c "
import json; d=json.load(open('$O/gen_stamps.json')); s=d['steps'][1]; print({k: s[k] for k in s if k not in ('span_first_start_to_last_end','start_spread')})"
bash tools/gpu_fresh.sh r04n tools/_abl/libd2d_var_base.so tools/_abl/libd2d_var_rpf.so
