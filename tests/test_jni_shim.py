"""CPU: the JNI shim (jni/clonos_jni.c) type-checks against include/clonos_engine.h, and
every native the Java side declares (ClonosEngine.java) has a C implementation with the
JNI-mangled name.  No JDK here: the check compiles with tests/jni_stub/jni.h (the JNI
types and the JNIEnv functions the shim uses)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "jni", "java", "org", "apache", "flink", "runtime", "causal", "engine", "ClonosEngine.java")
SHIM = os.path.join(ROOT, "jni", "clonos_jni.c")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_shim_type_checks():
    subprocess.run(["gcc", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                    "-I", os.path.join(ROOT, "tests", "jni_stub"), "-I", os.path.join(ROOT, "include"), SHIM],
                   check=True)


def test_every_native_is_implemented():
    natives = set(re.findall(r"static native \w+(?:\[\])? (n\w+)\(", open(JAVA).read()))
    impl = set(re.findall(r"FN\((n[A-Z]\w*)\)", open(SHIM).read()))
    assert len(natives) >= 19
    assert natives == impl, (natives - impl, impl - natives)


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_replay_prepare_marshalling(tmp_path):
    """nReplayPrepare through a fake JNIEnv (tests/jni_replay_host.c): the real
    clg_response_put accumulates the buffers, a recorder stands in for clg_replay_prepare and
    checks the vertex, the subpartition table and the response entries the shim builds, and
    the shim packs res / subRes exactly as EngineReplayPreparation.java reads them, on success
    and on an engine error.  No GPU: the engine call itself is the recorder."""
    lib_dir = os.path.join(ROOT, "clonos_amd")
    if not os.path.exists(os.path.join(lib_dir, "libclonos_engine.so")):
        pytest.skip("libclonos_engine.so not built")
    exe = str(tmp_path / "jni_replay_host")
    subprocess.run(["gcc", "-O1", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter", "-Wno-unused-function",
                    "-I", os.path.join(ROOT, "tests", "jni_stub"), "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "jni_replay_host.c"), "-L", lib_dir, "-lclonos_engine",
                    "-Wl,-rpath," + lib_dir, "-Wl,--allow-shlib-undefined", "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip() == "OK", r.stdout + r.stderr
