"""Host sanitizers (SURVEY §5 "Race detection / sanitizers": host ASan/UBSan
on the C-ABI glue). Two CPU programs, no GPU needed:

* tests/sanitize/capi_checks.cpp against libhrec's sources compiled with
  -fsanitize=address,undefined on the HOST side only (each -fsanitize= right
  after -Xarch_host; device code is built as usual and never launched): every
  C-ABI entry point rejects bad arguments with HREC_E_INVALID + a message
  before touching the device, the workspace-size queries are UB-free over a
  sweep of shapes, hrec_last_error is thread-local;
* tests/sanitize/oracle_checks.c with oracle/als_oracle.c (the C restatement
  used as the checker and the CPU baseline) under ASan (leak check on) +
  UBSan.

Objects are cached in tests/_san_build/ (git-ignored) by a hash of the
sources and flags, so only the first run pays the ~1-2 min compile.
"""
import hashlib
import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "hybrid-als-twotower-recommender_amd", "csrc")
SAN = os.path.join(ROOT, "tests", "sanitize")
OUT = os.path.join(ROOT, "tests", "_san_build")
HIPCC = "/opt/rocm/bin/hipcc"
CLANG = "/opt/rocm/lib/llvm/bin/clang++"
HOST_SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined"]
FLAGS = ["--offload-arch=gfx950", "-O1", "-g", "-std=c++17", "-fPIC", *HOST_SAN]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


def _digest(paths, extra):
    h = hashlib.sha256(" ".join(extra).encode())
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(os.path.basename(p).encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def _run(cmd, env=None):
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, f"{' '.join(cmd[:3])} ... failed ({r.returncode}):\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    return r


@pytest.mark.skipif(not (os.path.exists(HIPCC) and os.path.exists(CLANG)), reason="ROCm toolchain not present")
def test_capi_argument_checks_under_asan_ubsan():
    srcs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))
    deps = srcs + [os.path.join(CSRC, "common.h"), os.path.join(ROOT, "include", "hrec.h"),
                   os.path.join(SAN, "capi_checks.cpp")]
    tag = _digest(deps, FLAGS)
    bdir = os.path.join(OUT, "capi_" + tag)
    exe = os.path.join(bdir, "capi_checks")
    if not os.path.exists(exe):
        if os.path.isdir(OUT):  # drop builds of older sources
            for d in os.listdir(OUT):
                shutil.rmtree(os.path.join(OUT, d), ignore_errors=True)
        os.makedirs(bdir, exist_ok=True)

        def obj(src):
            o = os.path.join(bdir, os.path.basename(src) + ".o")
            _run([HIPCC, *FLAGS, "-c", src, "-o", o])
            return o

        with ThreadPoolExecutor(max(1, min(8, os.cpu_count() or 1))) as ex:
            objs = list(ex.map(obj, srcs))
        drv = os.path.join(bdir, "drv.o")
        _run([CLANG, "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-c",
              os.path.join(SAN, "capi_checks.cpp"), "-o", drv])
        _run([HIPCC, "--offload-arch=gfx950", "-fsanitize=address,undefined", "-fno-gpu-sanitize", drv, *objs,
              "-lpthread", "-o", exe + ".tmp"])
        os.replace(exe + ".tmp", exe)
    r = _run([exe], env=ENV)
    assert "capi_checks OK" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-2000:]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not present")
def test_oracle_c_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "oracle_checks")
    _run(["gcc", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-ffp-contract=off",
          os.path.join(SAN, "oracle_checks.c"), os.path.join(ROOT, "oracle", "als_oracle.c"), "-o", exe, "-lm"])
    r = _run([exe], env=dict(ENV, ASAN_OPTIONS="detect_leaks=1"))
    assert "oracle_checks OK" in r.stdout
    assert "runtime error" not in r.stderr, r.stderr[-2000:]
