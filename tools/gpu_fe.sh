set -u
O=gpurun_out/fe1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 bash tools/ubench_traffic.sh r05c > $O/ubench_traffic.log 2>&1 || exit 1
NOTEST=1 bash tools/gpu_ab.sh fe1 base fe
