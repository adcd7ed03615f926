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
