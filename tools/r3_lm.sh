# Decode A/B on one MI355X (run under gpurun): the long-record check (tools/dbg_lm.py), the
# decode GPU tests, then tools/ab.sh over two engine builds made with tools/ab_build.sh
# (config-2 bench and the 128-log config-3 subset).
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/lm
timeout -k 10 200 python3 tools/dbg_lm.py > gpurun_out/lm/dbg.txt 2>&1 || { tail -30 gpurun_out/lm/dbg.txt; exit 1; }
cat gpurun_out/lm/dbg.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_decode.py tests/test_gpu_golden.py tests/test_gpu_decode_async.py tests/test_gpu_replay.py > gpurun_out/lm/tests.log 2>&1 || { tail -30 gpurun_out/lm/tests.log; exit 1; }
tail -3 gpurun_out/lm/tests.log
NO_C3= bash tools/ab.sh 3 wbit wbit2 > gpurun_out/lm/ab.txt 2>&1; cat gpurun_out/lm/ab.txt | tail -4
