"""The native PS service under ThreadSanitizer and AddressSanitizer+UBSan: a
multi-threaded stress client (csrc/tests/ps_stress.cc) exercising every op family concurrently;
the invariants (exact locked adds, exact global-step count, every token dequeued) and a clean
sanitizer report are both required."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CXX = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.mark.skipif(not os.path.exists(CXX) and not shutil.which("clang++"), reason="no clang++")
@pytest.mark.parametrize("kind", ["thread", "address"])
def test_ps_service_sanitized_stress(kind):
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "build_sanitizers.sh"), kind], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    exe = os.path.join(ROOT, "build", "san", "ps_stress_%s" % ("tsan" if kind == "thread" else "asan"))
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, "6", "80"], capture_output=True, text=True, timeout=600, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "-> OK" in out and "WARNING: ThreadSanitizer" not in out and "ERROR: AddressSanitizer" not in out
