"""Host-side native runtime under AddressSanitizer + UBSan.

Compiles tests/cpp/test_runtime.cpp with the torch-free C++ cores
(csrc/runtime_core.cpp, csrc/lmdb_core.cpp) using ``-fsanitize=address,undefined``
and runs it: bucket planning, in-order bucket release, LMDB write/read round
trip including overflow pages.  CPU only.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_host_runtime_asan(tmp_path):
    exe = tmp_path / "test_runtime"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", f"-I{ROOT}/csrc", f"{ROOT}/tests/cpp/test_runtime.cpp",
           f"{ROOT}/csrc/runtime_core.cpp", f"{ROOT}/csrc/lmdb_core.cpp", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ)
    env.pop("LD_PRELOAD", None)  # ASan must be the first DSO; run the binary without preloads
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0"
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout
