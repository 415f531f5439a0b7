"""The bit-exact GPU suite on the runtime the bench binds.

The driver's `pytest -m gpu` process imports torch first, so the library there runs on torch's
bundled HIP 7.0 / RCCL 2.26; bench.py is torch-free and binds ROCm 7.2's HIP and RCCL, the ones
libraptor_amd.so was built against.  test_bit_exact_suite_torch_free re-runs the
single-process parity files -- kernels, V-cycles, full-size 256^3 cases, loopback ranks, device
formats, file I/O -- in a child pytest with AMG_TEST_NATIVE=1 (tests/util.py: Context.native,
DeviceVector copies, no torch import), and test_native_process_binds_rocm, run inside that
child, checks the child never imported torch and bound HIP >= 7.2 / RCCL >= 2.27.7.  The
child's output is streamed line by line, so a long phase never looks silent."""
import json
import os
import subprocess
import sys
import time

import pytest

from tests.util import native_mode

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = ["tests/test_gpu_native_runtime.py", "tests/test_gpu_parity.py", "tests/test_gpu_kernel_paths.py",
         "tests/test_gpu_multirank.py", "tests/test_gpu_formats.py", "tests/test_gpu_io.py"]


def test_native_process_binds_rocm(ctx):
    if not native_mode():
        pytest.skip("runs inside the torch-free child of test_bit_exact_suite_torch_free")
    import raptor_amd as ra

    assert "torch" not in sys.modules
    v = ra.runtime_versions()
    assert v["hip_runtime"] >= 70200000 and v["rccl"] >= 22707, v
    with open(os.environ["AMG_TEST_NATIVE_REPORT"], "w") as f:
        json.dump(v, f)


def test_bit_exact_suite_torch_free(capfd, tmp_path):
    if native_mode():
        pytest.skip("this is the child")
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    report = tmp_path / "runtime.json"
    env = dict(os.environ, AMG_TEST_NATIVE="1", AMG_TEST_NATIVE_REPORT=str(report), PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-u", "-m", "pytest", "-x", "-q", "-m", "gpu", "-p", "no:cacheprovider",
           "--timeout", "600", "--timeout-method", "thread", "-rs", *FILES]
    t0 = time.perf_counter()
    proc = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    tail = []
    try:
        for raw in proc.stdout:
            line = raw.decode(errors="replace").rstrip("\n")
            tail = (tail + [line])[-60:]
            with capfd.disabled():
                print(f"[native {time.perf_counter() - t0:6.1f}s] {line}", flush=True)
        rc = proc.wait(timeout=60)
    finally:
        if proc.poll() is None:
            proc.kill()
            proc.wait()
    text = "\n".join(tail)
    assert rc == 0, f"torch-free suite failed (rc {rc}):\n{text}"
    assert " passed" in text, text
    v = json.loads(report.read_text())  # written by test_native_process_binds_rocm in the child
    assert v["hip_runtime"] >= 70200000, v
