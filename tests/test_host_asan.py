"""AddressSanitizer + UBSan build and run of the native host planning code
(psrsigsim_amd/csrc/pss_host.cpp), SURVEY.md §5: the host side is compiled
with g++ -fsanitize=address,undefined next to a driver (tests/asan/host_asan.cpp)
that calls every pss_host_* entry point at edge sizes on exactly sized heap
buffers; the child process fails on any sanitizer report.  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_planning_under_asan(tmp_path):
    exe = str(tmp_path / "host_asan")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-pthread", "-I" + os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "asan", "host_asan.cpp"),
           os.path.join(ROOT, "psrsigsim_amd", "csrc", "pss_host.cpp"), "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    # verify_asan_link_order=0: the environment may preload its own library
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host_asan: ok" in r.stdout
