"""The JNI shim (jni/pbx_jni.c) unit-tested on the CPU.  There is no JDK in this image, so it
is compiled against a minimal test-only JNI environment (tests/jni_mock/jni.h: the calls the
shim makes) and a scripted fake of the libpbx entry points (tests/jni_mock/fake_pbx.c), and
driven by tests/jni_mock/jni_test.c: getTile's status slot and result release (no garbage
owner on a call-level failure, NOT_RESIDENT reported, responses past 2^31-1 bytes refused),
writeRows' piecewise whole-row copies, createPlane's 409, registerPlane's all-or-nothing,
registerZarr's offset checks against both Java arrays."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_jni_shim_logic(tmp_path):
    m = os.path.join(ROOT, "tests", "jni_mock")
    exe = str(tmp_path / "jni_test")
    subprocess.check_call(["gcc", "-std=c11", "-O1", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                           "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                           "-I", m, "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "jni", "pbx_jni.c"), os.path.join(m, "fake_pbx.c"),
                           os.path.join(m, "jni_test.c"), "-o", exe])
    # (the mock VM never frees its arrays: leak reports would be the harness's own)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 0, out.stderr + out.stdout
    assert "jni shim ok" in out.stdout
