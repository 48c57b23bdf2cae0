"""C++ runtime self-test under AddressSanitizer + UndefinedBehaviorSanitizer
(host code only).  Builds tests/native/runtime_selftest.cpp with
every runtime source except the Python bindings and runs it on logical CPU
devices."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "cekirdekler_amd", "csrc")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_runtime_selftest_asan_ubsan(tmp_path):
    sys.path.insert(0, ROOT)
    from cekirdekler_amd.build_native import SOURCES

    srcs = [os.path.join(CSRC, s) for s in SOURCES if s != "bindings.cpp"]
    exe = str(tmp_path / "runtime_selftest")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           "-D__HIP_PLATFORM_AMD__=1", f"-I{CSRC}", f"-I{ROCM}/include",
           os.path.join(ROOT, "tests", "native", "runtime_selftest.cpp"), *srcs,
           f"-L{ROCM}/lib", f"-Wl,-rpath,{ROCM}/lib", "-lamdhip64", "-lhiprtc", "-lrccl",
           "-lrocprofiler-sdk-roctx", "-ldl", "-lpthread", "-lrt", "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1", HIP_VISIBLE_DEVICES="", CEK_CACHE_DIR=str(tmp_path / "cache"))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-6000:]
    assert "runtime self-test passed" in r.stdout
