set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
for s in perpendicular parallel S_parallel corridor S_corridor large impossible mixed; do
  timeout -k 10 120 python3 "$R/bench.py" --no-cpu-baseline --scenario $s > "$R/gpurun_out/scn_$s.log" 2>&1 || { echo STOP $s; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['value']/1e9,3), round(d['roofline']['kernel_ms']*1e3,1))" "$R/gpurun_out/scn_$s.log" $s
done
