cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/bis
for k in random_all_tags many_spans config2_large config3_mixed order_zero long_records decode_errors logs_in_hbm segment_sizes; do
  timeout -k 10 100 python -u -m pytest tests/test_gpu_decode.py tools/probe_torch_test.py -k "$k or probe" -x -q -s --timeout 60 --timeout-method thread -p no:cacheprovider > gpurun_out/bis/$k.log 2>&1
  echo "$k rc=$?" >> gpurun_out/bis/summary.txt
done
echo done
