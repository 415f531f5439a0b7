/*
 * amg_oracle.h -- CPU oracle for the AMG V-cycle hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline.  The product path
 * (raptor_amd/, include/raptor_amd.h) never links or calls it.
 *
 * PARITY UNPINNED against Siddarthareddy1/raptor: /root/reference holds three RAPTOR
 * flowchart files and no AMG, SpMV, coarsening or halo code, so no
 * reference file:line or golden vector exists for any function here.  Every function
 * cites the spec line it restates (BASELINE.json:5 north_star) and
 * is cross-checked against scipy.sparse fixtures committed under tests/golden/
 * (tests/golden/gen_golden.py).  The algorithm definitions (tie-breaks, summation
 * orders) are fixed in DESIGN.md section 3 and are shared bit-for-bit with the product.
 *
 * Conventions: serial, fp64 values, int64 indices, CSR with columns sorted ascending,
 * diagonal stored.  Compiled with -ffp-contract=off so every product and sum is rounded
 * exactly as written (the GPU kernels are compiled the same way).
 */
#ifndef AMG_ORACLE_H
#define AMG_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_csr {
    int64_t n_rows, n_cols;
    int64_t* rp;   /* n_rows + 1 */
    int64_t* col;  /* nnz */
    double* val;   /* nnz */
} orc_csr;

/* ---- CSR objects --------------------------------------------------------------- */
orc_csr* orc_csr_new(int64_t n_rows, int64_t n_cols, const int64_t* rp, const int64_t* col,
                     const double* val);
void orc_csr_free(orc_csr* A);
int64_t orc_csr_nnz(const orc_csr* A);
int64_t orc_csr_rows(const orc_csr* A);
int64_t orc_csr_cols(const orc_csr* A);
void orc_csr_export(const orc_csr* A, int64_t* rp, int64_t* col, double* val);

/* ---- model problems (BASELINE.json:7-9) --------------------------- */
orc_csr* orc_gen_5pt(int64_t nx, int64_t ny);
orc_csr* orc_gen_7pt(int64_t nx, int64_t ny, int64_t nz);
orc_csr* orc_gen_27pt(int64_t nx, int64_t ny, int64_t nz, double ex, double ey, double ez);
/* x*_i = uniform(-1,1) from splitmix64(seed, global index i) */
void orc_vec_uniform(int64_t n, int64_t first_gid, uint64_t seed, double* out);

/* ---- level kernels ------------------------------------ */
void orc_spmv(const orc_csr* A, const double* x, double* y);
void orc_spmv_add(const orc_csr* A, const double* x, double* y);
void orc_residual(const orc_csr* A, const double* x, const double* b, double* r);
void orc_jacobi(const orc_csr* A, const double* x, const double* b, double* xout, double omega);
void orc_hybrid_gs(const orc_csr* A, const double* x, const double* b, double* xout,
                   int64_t block);
/* backward sweep: rows of each block in descending order, new values for in-block j > i */
void orc_hybrid_gs_backward(const orc_csr* A, const double* x, const double* b, double* xout,
                            int64_t block);
/* blocks clipped to rank segments starting at cuts[0..ncuts) (cuts[0] = 0) */
void orc_hybrid_gs_cut(const orc_csr* A, const double* x, const double* b, double* xout,
                       int64_t block, int32_t backward, int32_t ncuts, const int64_t* cuts);
double orc_norm2(int64_t n, const double* v);

/* ---- setup building blocks ---------------------------- */
orc_csr* orc_transpose(const orc_csr* A);
orc_csr* orc_spgemm(const orc_csr* A, const orc_csr* B);
orc_csr* orc_strength_classical(const orc_csr* A, double theta);
orc_csr* orc_strength_symmetric(const orc_csr* A, double theta);
void orc_rs_split(const orc_csr* S, int32_t* cf);   /* cf: 1 = C, 0 = F */
void orc_pmis_split(const orc_csr* S, uint64_t seed, int32_t* cf);
orc_csr* orc_interp_classical(const orc_csr* A, const orc_csr* S, const int32_t* cf);
/* extended+i (distance two) with P_max truncation (p_max = 0: none); DESIGN.md 3 (r6) */
orc_csr* orc_interp_ext_i(const orc_csr* A, const orc_csr* S, const int32_t* cf, int64_t p_max);
int64_t orc_mis2_aggregate(const orc_csr* S, uint64_t seed, int32_t* agg);
/* SA smoothing (r6): filtered operator, max-norm power-iteration rho, smoothed P */
#define ORC_SA_RHO_ITERS 10
orc_csr* orc_sa_filter(const orc_csr* A, double theta);
double orc_sa_rho(const orc_csr* F, const double* d, uint64_t seed);
orc_csr* orc_sa_prolongator(const orc_csr* A, const int32_t* agg, int64_t n_agg, double theta,
                            uint64_t seed);
/* coarse-operator drop tolerance: small off-diagonals lumped onto the diagonal (r6) */
orc_csr* orc_sparsify(const orc_csr* A, double tau);
/* SA strength threshold of the next level: theta * 0.75 */
double orc_sa_theta_next(double theta);
void orc_dense_inverse(int64_t n, const orc_csr* A, double* inv); /* row-major n*n */

/* unstructured inputs (io_oracle.c, row f2; specs in DESIGN.md 8) */
orc_csr* orc_gen_graph_laplacian(int64_t nx, int64_t ny, uint64_t seed);
void orc_rcm(const orc_csr* A, int64_t* new_to_old);
orc_csr* orc_permute(const orc_csr* A, const int64_t* new_to_old);  /* P A P^T */

/* ---- hierarchy (ParMultilevel analogue) --------------------- */
enum { ORC_COARSEN_RS = 0, ORC_COARSEN_PMIS = 1, ORC_COARSEN_SA = 2 };
enum { ORC_SMOOTH_JACOBI = 0, ORC_SMOOTH_HYBRID_GS = 1 };
enum { ORC_INTERP_CLASSICAL = 0, ORC_INTERP_EXT_I = 1 };

typedef struct orc_options {
    int32_t coarsen;
    int32_t smoother;
    double strong_threshold;
    double jacobi_omega;
    int32_t pre_sweeps, post_sweeps;
    int32_t max_levels;
    int64_t max_coarse;
    int64_t gs_block;
    uint64_t seed;
    int32_t interp;  /* RS / PMIS: ORC_INTERP_CLASSICAL or ORC_INTERP_EXT_I */
    int64_t p_max;   /* ext+i truncation: entries kept per row (0: all) */
    double drop_tol; /* coarse-operator drop tolerance (0: Galerkin) */
} orc_options;

typedef struct orc_hier orc_hier;
orc_hier* orc_hier_setup(const orc_csr* A, const orc_options* opt);
/* hierarchy from given level operators (A[0..nlev), P/R[0..nlev-1)); copies them and
 * computes the coarsest inverse.  Lets the CPU baseline run on the product's hierarchy. */
orc_hier* orc_hier_from_levels(int32_t nlev, const orc_csr* const* A, const orc_csr* const* P,
                               const orc_csr* const* R, const orc_options* opt);
/* rank partition of level `level` (start rows); hybrid GS blocks are clipped to it */
void orc_hier_set_cuts(orc_hier* H, int32_t level, int32_t ncuts, const int64_t* cuts);
void orc_hier_free(orc_hier* H);
int32_t orc_hier_levels(const orc_hier* H);
/* which: 0 = A_l, 1 = P_l, 2 = R_l (borrowed pointer, do not free) */
const orc_csr* orc_hier_matrix(const orc_hier* H, int32_t level, int32_t which);
/* integer splitting of level l: C/F marker (RS/PMIS) or aggregate id (SA) */
void orc_hier_split(const orc_hier* H, int32_t level, int32_t* out);
void orc_hier_cycle(orc_hier* H, double* x, const double* b);
int32_t orc_num_threads(void); /* OpenMP threads the level kernels use */
void orc_set_num_threads(int32_t n); /* OpenMP team size of later parallel regions (n > 0) */
int32_t orc_hier_solve(orc_hier* H, double* x, const double* b, int32_t max_iter, double tol,
                       double* hist);
/* CG preconditioned by one V-cycle (z = 0; cycle(z, r)) per iteration (row f3). */
int32_t orc_hier_pcg(orc_hier* H, double* x, const double* b, int32_t max_iter, double tol,
                     double* hist);

#ifdef __cplusplus
}
#endif
#endif
