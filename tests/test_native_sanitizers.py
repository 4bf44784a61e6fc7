"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only; GPU sanitizers are
not available on this pool).  The scheduler (dpwa_amd/csrc/sched.cpp) is pure host C++: it is
compiled here with g++ together with tests/native/sched_stress.cpp, which drives every entry
point with random call sequences and malformed arguments and checks conn.py:178-317's
invariants after each call."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]


def _build(tmp_path, sources, out):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path / out)
    cmd = [gxx, "-std=c++17", "-O1", "-g", *SAN, "-I", os.path.join(ROOT, "include"),
           *[os.path.join(ROOT, s) for s in sources], "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0 and ("asan" in r.stderr or "ubsan" in r.stderr):
        pytest.skip("sanitizer runtime not installed: " + r.stderr[-200:])
    assert r.returncode == 0, r.stderr
    return exe


def test_scheduler_under_asan_ubsan(tmp_path):
    exe = _build(tmp_path, ["dpwa_amd/csrc/sched.cpp", "tests/native/sched_stress.cpp"], "sched_stress")
    # verify_asan_link_order=0: the environment may preload a library of its own ahead of ASan's
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, "300"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sched stress ok" in r.stdout


def test_gossip_board_under_asan_ubsan(tmp_path):
    """board.cpp's host protocol (publish_wait / advertise / acquire / release, host forms) with
    4 ranks as threads of one process, 2000 free-running rounds each: no torn or rewritten
    snapshot is ever read, versions never go backwards, no wait times out
    (tests/native/board_stress.cpp).  Built with ROCm's clang against the HIP runtime, which
    the host paths link but never call."""
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cxx = os.path.join(rocm, "lib", "llvm", "bin", "clang++")
    if not os.path.exists(cxx):
        pytest.skip("no ROCm clang++")
    exe = str(tmp_path / "board_stress")
    cmd = [cxx, "-std=c++17", "-O1", "-g", *SAN, "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(rocm, "include"),
           "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "dpwa_amd/csrc/board.cpp"),
           os.path.join(ROOT, "tests/native/board_stress.cpp"), "-L", os.path.join(rocm, "lib"), "-lamdhip64",
           "-Wl,-rpath," + os.path.join(rocm, "lib"), "-lpthread", "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, "4", "2000"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "board stress ok" in r.stdout


def _tsan_build(tmp_path):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "node_tsan")
    srcs = ["dpwa_amd/csrc/node.cpp", "dpwa_amd/csrc/sched.cpp", "dpwa_amd/csrc/trace.cpp",
            "tests/native/fake_learner.cpp", "tests/native/node_tsan.cpp"]
    cmd = [gxx, "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-fno-omit-frame-pointer", "-I",
           os.path.join(ROOT, "include"), *[os.path.join(ROOT, s) for s in srcs], "-o", exe, "-ldl", "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0 and "tsan" in r.stderr:
        pytest.skip("TSan runtime not installed: " + r.stderr[-200:])
    assert r.returncode == 0, r.stderr
    return exe


def test_node_and_scheduler_under_tsan(tmp_path):
    """SURVEY §5 race detection: node.cpp + sched.cpp under ThreadSanitizer (the counterpart of the
    reference's races at conn.py:106, 240, 259, 313).  Four threads each drive their own group of
    four lock-step nodes over the host-only learner (tests/native/node_tsan.cpp: stalls, rescue
    lanes, faults, flow control, the Bernoulli gate) for 2,000 rounds, with the roctx trace hooks
    switched on -- the ABI's promise that calls are reentrant per handle.  TSan must stay silent;
    the control (two threads bumping one plain int) shows the build is instrumented."""
    exe = _tsan_build(tmp_path)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1", DPWA_ROCTX="1")
    r = subprocess.run([exe, "racy"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0 and "data race" in r.stderr, (r.returncode, r.stderr[-2000:])
    r = subprocess.run([exe, "4", "4", "2000"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "node tsan ok" in r.stdout and "8000 rounds" in r.stdout
