"""GPU, world_size 2 (gloo transport, both ranks on cuda:0): sharing-depth replication
over real engines -- device slice into the send blob, all-gather, device-input batched
processUpstreamDelta into the replicas -- reproduces every wanted log byte for byte."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_replication_engines_world2():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(HERE, "gpu_dist_worker.py")], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "replicas verified:" in r.stdout
