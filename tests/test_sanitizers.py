"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer: the wire
codec (fuzzed truncations / bit flips / streaming probe), SSTable reader and
the batcher under concurrent offers, streamed rows and lanes
(tests/native/sanitize_main.cpp).  GPU sanitizers are not available on this
pool; the HIP side is covered by the numerics tests."""
import os
import shutil
import subprocess

import pytest

from rust_tensorflow_serving2_amd import _build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "rust_tensorflow_serving2_amd", "csrc")


SRCS = ("wire.cpp", "sstable.cpp", "batcher.cpp", "http2_server.cpp", "router.cpp", "request_log.cpp", "ingest.cpp")


def _build_driver(tmp_path, name, flags, cxx=None):
    cxx = cxx or os.environ.get("CXX", "g++")
    if shutil.which(cxx) is None:
        pytest.skip("no C++ compiler")
    exe = str(tmp_path / name)
    srcs = [os.path.join(ROOT, "tests", "native", "sanitize_main.cpp")] + [os.path.join(CSRC, f) for f in SRCS]
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-msse4.2", "-pthread"] + flags + \
        [f"-I{CSRC}", "-o", exe] + srcs + [_build._nghttp2_lib(), "-ldl", "-lrt"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    return exe


@pytest.mark.timeout(600)
def test_native_host_code_under_asan_ubsan(tmp_path):
    exe = _build_driver(tmp_path, "sanitize_asan", ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"])
    # verify_asan_link_order=0: other preloaded libraries may precede the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout + r.stderr)[-6000:]


@pytest.mark.timeout(900)
def test_native_host_code_under_tsan(tmp_path):
    """The same driver under ThreadSanitizer: batcher offers / streamed rows /
    lanes / close and the router threads must be free of data races.

    Built with LLVM's clang++ + compiler-rt TSan (ROCm ships it): GCC 11's
    libtsan has no interceptor for pthread_cond_clockwait, which libstdc++
    uses for condition_variable::wait_until, so it misreports every timed
    wait as a double lock."""
    clang = "/opt/rocm/lib/llvm/bin/clang++"
    if not os.path.exists(clang):
        pytest.skip("no LLVM clang++ with a compiler-rt TSan runtime")
    exe = _build_driver(tmp_path, "sanitize_tsan", ["-fsanitize=thread"], cxx=clang)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1:report_signal_unsafe=0")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    if r.returncode != 0 and "FATAL: ThreadSanitizer: unexpected memory mapping" in r.stderr:
        pytest.skip("TSan cannot run under this kernel's address-space layout")
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout + r.stderr)[-8000:]
