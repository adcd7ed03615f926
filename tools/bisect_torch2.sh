cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/bis2
timeout -k 10 200 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_decode_async.py -x -q --timeout 60 --timeout-method thread -p no:cacheprovider > gpurun_out/bis2/prio1.log 2>&1; echo "prio1 rc=$?" >> gpurun_out/bis2/summary.txt
CLONOS_GATHER_PRIO=0 timeout -k 10 200 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_decode_async.py -x -q --timeout 60 --timeout-method thread -p no:cacheprovider > gpurun_out/bis2/prio0.log 2>&1; echo "prio0 rc=$?" >> gpurun_out/bis2/summary.txt
echo done
