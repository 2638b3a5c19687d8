set -u
R=$(pwd); O=$R/gpurun_out/${1:-ppo4}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ppo.py tests/test_abi.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -5 $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/train_ppo.py --updates 60 > $O/train60.log 2>&1 || exit $?
tail -2 $O/train60.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $R/tools/train_ppo.py --updates 8 > $O/kt.log 2>&1 || exit $?
