/* oracle_driver.c -- AddressSanitizer / UBSan run of the CPU oracle (test infrastructure,
 * oracle/amg_oracle.c + io_oracle.c): hierarchies for the three model problems, level
 * kernels, cycles, solve, PCG, RCM and the permutation. */
#include <stdio.h>
#include <stdlib.h>

#include "../../oracle/amg_oracle.h"

static int run_opt(orc_csr* A, int coarsen, int smoother, double theta, int interp, double drop_tol);
static int run(orc_csr* A, int coarsen, int smoother, double theta) {
    return run_opt(A, coarsen, smoother, theta, ORC_INTERP_CLASSICAL, 0.0);
}
static int run_opt(orc_csr* A, int coarsen, int smoother, double theta, int interp, double drop_tol) {
    orc_options o = {coarsen, smoother, theta, 2.0 / 3.0, 1, 1, 25, 64, 64, 0x5EED};
    o.interp = interp;  /* r6 options: extended+i (P_max 4) and the coarse drop tolerance */
    o.p_max = 4;
    o.drop_tol = drop_tol;
    int64_t n = orc_csr_rows(A);
    double* b = malloc(sizeof(double) * n);
    double* x = calloc(n, sizeof(double));
    double* y = malloc(sizeof(double) * n);
    double hist[6];
    orc_vec_uniform(n, 0, 42, b);
    orc_hier* H = orc_hier_setup(A, &o);
    int lv = orc_hier_levels(H);
    orc_hier_cycle(H, x, b);
    orc_hybrid_gs(A, x, b, y, 64);
    orc_hybrid_gs_backward(A, x, b, y, 17);
    orc_jacobi(A, x, b, y, 2.0 / 3.0);
    orc_residual(A, x, b, y);
    orc_hier_solve(H, x, b, 5, 0.0, hist);
    orc_hier_pcg(H, x, b, 5, 0.0, hist);
    orc_hier_free(H);
    free(b);
    free(x);
    free(y);
    return lv;
}

int main(void) {
    int lv = 0;
    orc_csr* A = orc_gen_7pt(14, 13, 12);
    lv += run(A, ORC_COARSEN_PMIS, ORC_SMOOTH_JACOBI, 0.25);
    lv += run_opt(A, ORC_COARSEN_PMIS, ORC_SMOOTH_JACOBI, 0.25, ORC_INTERP_EXT_I, 0.05);
    lv += run_opt(A, ORC_COARSEN_SA, ORC_SMOOTH_HYBRID_GS, 0.08, ORC_INTERP_CLASSICAL, 0.02);
    orc_csr_free(A);
    A = orc_gen_5pt(40, 33);
    lv += run(A, ORC_COARSEN_RS, ORC_SMOOTH_JACOBI, 0.25);
    orc_csr_free(A);
    A = orc_gen_27pt(11, 10, 9, 1.0, 1.0, 1e-3);
    lv += run(A, ORC_COARSEN_SA, ORC_SMOOTH_HYBRID_GS, 0.08);
    orc_csr_free(A);
    A = orc_gen_graph_laplacian(60, 50, 3);
    int64_t n = orc_csr_rows(A);
    int64_t* p = malloc(sizeof(int64_t) * n);
    orc_rcm(A, p);
    orc_csr* B = orc_permute(A, p);
    lv += run(B, ORC_COARSEN_SA, ORC_SMOOTH_HYBRID_GS, 0.08);
    orc_csr_free(B);
    orc_csr_free(A);
    free(p);
    printf("oracle sanitizer driver ok: %d levels\n", lv);
    return 0;
}
