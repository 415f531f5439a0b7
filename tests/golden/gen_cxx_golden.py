"""tests/golden/cxx_7pt24_hist.txt: the oracle's ParMultilevel::solve history that the compiled
C++ caller (tests/cxx/cxx_driver.cpp) must reproduce -- 7-pt Poisson 24^3, PMIS + classical
interpolation, Jacobi(2/3) 1+1 V-cycles, b = A x* with x* = splitmix64 U(-1,1) seed 42, x0 = 0,
10 iterations.  The oracle builds its own hierarchy (the product's equals it, integer setup
bit-exact).  Run: python tests/golden/gen_cxx_golden.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import oracle as O  # noqa: E402


def main():
    A = O.gen_7pt(24, 24, 24)
    n = A.shape[0]
    H = O.Hierarchy(A, **O.DEFAULTS["pmis"])
    b = A.spmv(O.vec_uniform(n, 42))
    _, hist = H.solve(np.zeros(n), b, max_iter=10)
    with open(os.path.join(HERE, "cxx_7pt24_hist.txt"), "w") as f:
        f.write("# ||b - A x_k||, k = 0..10: oracle, 7-pt 24^3, PMIS + Jacobi (gen_cxx_golden.py)\n")
        for v in hist:
            f.write(f"{v:.17g}\n")
    print(H.num_levels, hist[-1] / hist[0])


if __name__ == "__main__":
    main()
