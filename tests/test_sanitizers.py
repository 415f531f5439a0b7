"""Host sanitizer builds: the product's host setup code (raptor_amd/csrc/host_*.cpp)
and the CPU oracle, each driven through its setup / kernel / reader paths under
-fsanitize=address,undefined.  CPU only; any ASan report or UBSan runtime error fails."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sanitize")


@pytest.fixture(scope="module")
def built(tmp_path_factory):
    if shutil.which("g++") is None or shutil.which("gcc") is None:
        pytest.skip("no host compiler")
    out = str(tmp_path_factory.mktemp("san"))
    subprocess.run(["make", "-s", "-j2", "-C", HERE, f"OUT={out}"], check=True, timeout=600)
    return out


@pytest.mark.parametrize("driver", ["host_driver", "oracle_driver"])
def test_sanitized_run(built, tmp_path, driver):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", OMP_NUM_THREADS="4")
    p = subprocess.run([os.path.join(built, driver), str(tmp_path)], env=env, capture_output=True,
                       text=True, timeout=600)
    log = p.stdout + p.stderr
    assert p.returncode == 0, log[-4000:]
    assert "ERROR: AddressSanitizer" not in log and "runtime error" not in log, log[-4000:]
    assert "driver ok" in p.stdout
