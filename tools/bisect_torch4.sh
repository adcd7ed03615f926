cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/bis4
timeout -k 10 200 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_decode_async.py -x -q --timeout 60 --timeout-method thread -p no:cacheprovider > gpurun_out/bis4/a.log 2>&1; echo "a rc=$?"
python3 -c "
import clonos_amd, os
maps=open('/proc/self/maps').read()
print(sorted(set(l.split()[-1] for l in maps.splitlines() if 'amdhip64' in l)))" > gpurun_out/bis4/maps.txt 2>&1
echo done
