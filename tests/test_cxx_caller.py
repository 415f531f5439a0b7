"""The boundary as BASELINE.json:5 words it -- "C++ host code calls HIP through a thin
extern-"C" layer": tests/cxx/cxx_driver.cpp is a compiled C++ program over the header-only
facade include/raptor_amd.hpp (RAII Context / ParCSRMatrix / ParMultilevel, C-ABI error codes
as raptor_amd::Error).  No Python or torch runs in its process, so the library binds the ROCm HIP
runtime and RCCL it was built against (tests/test_gpu_rccl.py runs under torch's bundled
copies).  Its solve history must equal the oracle's (tests/golden/cxx_7pt24_hist.txt, made by
tests/golden/gen_cxx_golden.py) within 1e-10 relative."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cxx", "build", "cxx_driver")
GOLD = os.path.join(ROOT, "tests", "golden", "cxx_7pt24_hist.txt")


def test_cxx_driver_built_and_linked():
    """build() compiles the C++ caller against include/raptor_amd.hpp and links it to the
    in-tree libraptor_amd.so (no GPU needed to check the link)."""
    assert os.path.exists(EXE), "run __graft_entry__.build() (make -C tests/cxx)"
    out = subprocess.run(["ldd", EXE], capture_output=True, text=True, check=True).stdout
    lib = [l for l in out.splitlines() if "libraptor_amd.so" in l]
    assert lib and os.path.realpath(lib[0].split("=>")[1].split()[0]) == \
        os.path.realpath(os.path.join(ROOT, "raptor_amd", "libraptor_amd.so"))
    assert "libtorch" not in out and "python" not in out


def test_golden_history_is_the_oracles(oracle):
    import numpy as np

    O = oracle
    A = O.gen_7pt(24, 24, 24)
    H = O.Hierarchy(A, **O.DEFAULTS["pmis"])
    b = A.spmv(O.vec_uniform(A.shape[0], 42))
    _, hist = H.solve(np.zeros(A.shape[0]), b, max_iter=10)
    gold = np.loadtxt(GOLD)
    assert np.array_equal(hist, gold)


def _run(args, timeout=180, env_extra=None):
    env = dict(os.environ)
    env.update(NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1", OMP_NUM_THREADS="2",
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.update(env_extra or {})
    p = subprocess.run([EXE] + args, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert p.returncode == 0, f"{args}: exit {p.returncode}\n{p.stdout[-3000:]}\n{p.stderr[-3000:]}"
    return p.stdout


@pytest.mark.gpu
def test_cxx_solve_matches_golden():
    out = _run(["solve", GOLD])
    assert len(out.strip().splitlines()) == 11


@pytest.mark.gpu
def test_cxx_errors_surface_as_exceptions():
    assert "0 failures" in _run(["errors"])


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_cxx_rccl_ranks_match_golden(nranks, graph):
    """N forked ranks, RCCL halo exchange (socket transport on one GPU), torch-free.  graph:
    every rank captures whole V-cycles (halo send/recv groups, the coarse allgather and the
    fused residual-norm allgather inside the graph) and replays them; the driver fails if a
    rank fell back to eager cycles, and the history must still be the oracle's."""
    _run(["ranks", str(nranks)] + (["graph"] if graph else []) + [GOLD], timeout=240)


@pytest.mark.gpu
def test_cxx_rccl_graph_cycles_equal_eager():
    """Captured V-cycles replayed back to back (one synchronisation) equal the same cycles
    run eagerly by a second solver, bit for bit, on both ranks."""
    out = _run(["ranks", "2", "graph", GOLD], env_extra={"AMG_CXX_GRAPH_MULT": "4"})
    assert "replay == eager on every rank" in out
