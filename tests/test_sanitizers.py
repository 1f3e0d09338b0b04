"""CPU: the host code of the engine under sanitizers.  GPU sanitizers are not
available on this pool, so each target is the host-only part of libmbls or a test harness
around it, built with ROCm's clang (its TSan intercepts the condition-variable waits of
libstdc++ 11, which GCC 11's TSan misreports as double locks):

* host staging + batch split (csrc/mbls_host.hpp: par_for packing from several callers at once,
  plan_shards) under ASan+UBSan and under TSan -- tests/sanitize/host_sanitize.cpp;
* the batching queue (csrc/mbls_queue.cpp, two workers, 48 callers) over a host fake of the
  layer-1 batch calls, under TSan and under ASan+UBSan -- tests/sanitize/queue_sanitize.cpp;
* both NIF shims (nif/bls_nif.c, nif/bls_device_nif.c) over the fake BEAM and a host fake of
  libmbls, with the real queue and status strings, under ASan+UBSan (LeakSanitizer on) --
  every success / error / raise / badarg path, and 12 concurrent callers through the queue;
* the device arithmetic compiled for the host (tests/hostsim) with UBSan in trap mode
  (`-Xarch_host -fsanitize=undefined`), running tests/test_hostsim_arith.py against it.
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "lambda_ethereum_consensus_amd", "csrc")
NIF = os.path.join(ROOT, "lambda_ethereum_consensus_amd", "nif")
SAN = os.path.join(ROOT, "tests", "sanitize")
STUB = os.path.join(ROOT, "tests", "nif_stub")
INC = os.path.join(ROOT, "include")
LLVM = "/opt/rocm/lib/llvm/bin"
ASAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"]
TSAN = ["-fsanitize=thread"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", TSAN_OPTIONS="halt_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _cc(name):
    path = os.path.join(LLVM, name)
    if not os.path.exists(path):
        pytest.skip(f"{path} not available")
    return path


def _run(cmd, timeout=300):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=ENV)
    assert r.returncode == 0, (" ".join(cmd[:3]), r.stdout[-2000:], r.stderr[-6000:])
    return r.stdout


def _cxx(out, srcs, san, tmp):
    exe = str(tmp / out)
    _run([_cc("clang++"), "-std=c++17", "-O1", "-g", *san, "-I", CSRC, "-I", INC, *srcs, "-o", exe, "-lpthread"])
    return exe


@pytest.mark.parametrize("san", ["asan_ubsan", "tsan"])
def test_host_staging_and_partition(san, tmp_path):
    exe = _cxx("host_" + san, [os.path.join(SAN, "host_sanitize.cpp")], ASAN if san == "asan_ubsan" else TSAN, tmp_path)
    assert "host staging OK" in _run([exe])


@pytest.mark.parametrize("san", ["asan_ubsan", "tsan"])
def test_batching_queue(san, tmp_path):
    exe = _cxx("queue_" + san, [os.path.join(SAN, "queue_sanitize.cpp"), os.path.join(CSRC, "mbls_queue.cpp")],
               ASAN if san == "asan_ubsan" else TSAN, tmp_path)
    out = _run([exe])
    assert "queue OK" in out and "bad=0" in out


def test_nif_shims(tmp_path):
    cc = _cc("clang")
    objs = []
    for src, init in (("bls_nif.c", "bls_nif_init"), ("bls_device_nif.c", "dev_nif_init")):
        o = str(tmp_path / (src + ".o"))
        _run([cc, "-std=gnu11", "-O1", "-g", *ASAN, "-Wall", "-Werror", "-I", STUB, "-I", INC, f"-Dnif_init={init}",
              "-c", os.path.join(NIF, src), "-o", o])
        objs.append(o)
    for src in (os.path.join(SAN, "nif_sanitize.c"), os.path.join(STUB, "fake_beam.c")):
        o = str(tmp_path / (os.path.basename(src) + ".o"))
        _run([cc, "-std=gnu11", "-O1", "-g", *ASAN, "-Wall", "-Werror", "-I", STUB, "-I", INC, "-c", src, "-o", o])
        objs.append(o)
    exe = str(tmp_path / "nif_asan")
    _run([_cc("clang++"), "-std=c++17", "-O1", "-g", *ASAN, "-I", INC, *objs, os.path.join(CSRC, "mbls_queue.cpp"),
          os.path.join(CSRC, "mbls_status.cpp"), "-o", exe, "-lpthread"])
    assert "nif OK" in _run([exe])


def test_device_arithmetic_under_ubsan():
    """The radix-2^28 Fp/Fp2/Fp12, curve, hash-to-G2 and pairing code of csrc/*.hpp, built for
    the host with UBSan traps (any undefined behaviour -> SIGILL), through the bit-exact
    oracle comparisons of test_hostsim_arith.py."""
    if not shutil.which("hipcc"):
        pytest.skip("hipcc not available")
    from tests.conftest import build_hostsim

    so = build_hostsim(so=os.path.join(ROOT, "tests", "hostsim", "libhostsim_ubsan.so"),
                       extra=("-Xarch_host", "-fsanitize=undefined", "-Xarch_host", "-fsanitize-trap=undefined"))
    env = dict(os.environ, MBLS_HOSTSIM_SO=so)
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_hostsim_arith.py")], capture_output=True, text=True,
                       timeout=900, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
