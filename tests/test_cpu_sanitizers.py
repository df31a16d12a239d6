"""Sanitizer builds of the product's threaded host-core CPU path (csrc/cpu_ops.cpp, row A16; SURVEY §5 'race detection';
VERDICT r5 item 7): cpu_ops.cpp and tests/cpu_ops_sanitize_driver.cpp compiled with AddressSanitizer + UBSan (every
report fatal) and, separately, with ThreadSanitizer, then run: both entry points over ragged / tiny / empty /
threading-sized inputs at 1..64 worker threads and from four concurrent host callers, each result checked against a
scalar restatement in the driver.  Host code only (no GPU), so it runs in the CPU suite."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "bitsandbytes-sycl_amd", "csrc", "cpu_ops.cpp")
DRIVER = os.path.join(ROOT, "tests", "cpu_ops_sanitize_driver.cpp")


@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_cpu_ops_under_sanitizer(tmp_path, san):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = tmp_path / "drv"
    flags = ["-O1", "-g", "-std=c++17", "-ffp-contract=off", "-pthread", f"-fsanitize={san}",
             "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-Wall", "-Wextra", "-Werror"]
    r = subprocess.run([gxx, *flags, SRC, DRIVER, "-o", str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert r.stdout.startswith("OK"), r.stdout
