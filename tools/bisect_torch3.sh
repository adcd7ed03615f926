cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/bis3
timeout -k 10 200 python -u -m pytest tests/test_gpu_decode.py tools/probe_torch_test.py -x -q -s --timeout 60 --timeout-method thread -p no:cacheprovider > gpurun_out/bis3/a.log 2>&1; echo "a rc=$?"
echo done
