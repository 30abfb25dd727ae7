"""Sanitizer builds of the native host code (ASan/UBSan and TSan in CI).

The FramePool (csrc/runtime/frame_pool.cpp) is compiled together with a multi-threaded stress
harness (tests/native/frame_pool_stress.cpp) once with ``-fsanitize=address,undefined`` and once
with ``-fsanitize=thread`` — host code only, CPU storage — and run; any report fails the test.
GPU sanitizers are not available on the MI355X pool, so device code is covered by the
numerics tests instead."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
SRC = ROOT / "tests" / "native" / "frame_pool_stress.cpp"


def _torch_flags():
    import torch
    t = Path(torch.__file__).resolve().parent
    inc = [f"-I{t / 'include'}", f"-I{t / 'include' / 'torch' / 'csrc' / 'api' / 'include'}"]
    libs = [f"-L{t / 'lib'}", f"-Wl,-rpath,{t / 'lib'}", "-ltorch", "-ltorch_cpu", "-lc10"]
    return inc, libs, str(t / "lib")


@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_frame_pool_under_sanitizers(tmp_path, san):
    # ROCm's clang: its TSan runtime intercepts pthread_cond_clockwait (GCC 11's libtsan does
    # not, and then reports std::condition_variable::wait_for as a double lock)
    clang = Path("/opt/rocm/lib/llvm/bin/clang++")
    cxx = str(clang) if clang.exists() else "g++"
    inc, libs, libdir = _torch_flags()
    exe = tmp_path / f"frame_pool_{san.split(',')[0]}"
    cmd = [cxx, "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer",
           "-D_GLIBCXX_USE_CXX11_ABI=1", *inc, str(SRC), "-o", str(exe), *libs, "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        pytest.fail(f"sanitizer build failed:\n{r.stderr[-3000:]}")
    env = dict(os.environ, LD_LIBRARY_PATH=libdir, OMP_NUM_THREADS="1",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1:report_signal_unsafe=0")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out
    assert "WARNING: ThreadSanitizer" not in out, out[-4000:]
    assert "bad=0" in out


def test_sexpr_codec_under_asan_ubsan(tmp_path):
    """the native S-expression codec parses every inbound MQTT payload, so
    it runs here built with ``-fsanitize=address,undefined`` (the CPython extension, loaded
    into an uninstrumented interpreter with the ASan runtime preloaded and PYTHONMALLOC=malloc
    so Python objects are ASan allocations too) over a seeded random corpus, deep nesting past
    the 512 limit, huge / malformed canonical lengths and long tokens, each result compared
    with the pure-Python codec (tests/native/sexpr_asan_driver.py)."""
    import sysconfig
    src = ROOT / "aiko_services_amd" / "csrc" / "host" / "sexpr.c"
    so = tmp_path / "_sexpr.so"
    cc = "gcc"
    cmd = [cc, "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           "-fno-sanitize-recover=undefined", "-shared", "-fPIC", "-I", sysconfig.get_paths()["include"],
           str(src), "-o", str(so)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        pytest.fail(f"sanitizer build failed:\n{r.stderr[-3000:]}")
    asan = subprocess.run([cc, "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    env = dict(os.environ, LD_PRELOAD=asan, PYTHONMALLOC="malloc",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, str(ROOT / "tests" / "native" / "sexpr_asan_driver.py"), str(so), str(ROOT)],
                       capture_output=True, text=True, timeout=600, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert "SEXPR_ASAN_OK" in out, out[-2000:]
