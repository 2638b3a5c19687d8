# round 4: K1 phase stamps in the driver's early window (warmup 5) against the steady state (300)
set -u
O=gpurun_out/r04y; mkdir -p $O
timeout -k 10 200 python tools/stamps.py run --warm 5 --small 0 > $O/stamps_w5.log 2>&1 || { echo STOP w5; tail -3 $O/stamps_w5.log; exit 1; }
cp gpurun_out/stamps.json $O/stamps_w5.json
timeout -k 10 200 python tools/stamps.py run --warm 300 --small 0 > $O/stamps_w300.log 2>&1 || { echo STOP w300; exit 1; }
cp gpurun_out/stamps.json $O/stamps_w300.json
python3 - <<'PY'
import json
for w in ("w5", "w300"):
    d = json.load(open(f"gpurun_out/r04y/stamps_{w}.json"))[0]
    print(w, "span", d["kernel_span_cycles"], {k: {kk: vv[0] for kk, vv in d[k].items()} for k in ("wave0", "wave1", "wave2", "wave3")})
PY
