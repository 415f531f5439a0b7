/*
 * raptor_amd.h -- C-ABI drop-in boundary for the MI355X AMG V-cycle hot path.
 *
 * Spec: BASELINE.json:5 (north_star) asks for an AMG V-cycle that "keeps the
 * ParMultilevel/ParCSRMatrix API surface so it drops in as the level solver: C++ host code
 * calls HIP through a thin extern-"C" layer".  The mounted reference (Siddarthareddy1/raptor)
 * holds no such interface -- it is three RAPTOR flowchart files, SURVEY.md section 0 -- so
 * there is no reference file:line to replace; each entry point below cites the SURVEY.md
 * section 8 row and the RAPtor-style method it stands for.  Names follow SURVEY.md 8(b).
 *
 * Rules of the boundary:
 *   - plain C types only; host arrays are borrowed for the duration of a call;
 *   - vectors passed to compute calls are DEVICE pointers of the rank-local length,
 *     fp64, owned by the caller; all work is enqueued on the context's HIP stream;
 *   - every call returns AMG_OK (0) or an error code; amg_last_error() gives the message
 *     for the calling thread.  No exception crosses the boundary.
 *   - one context per GPU per process (rank); a context is not re-entrant.
 */
#ifndef RAPTOR_AMD_H
#define RAPTOR_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AMG_OK 0
#define AMG_ERR_INVALID 1   /* bad argument / state                          */
#define AMG_ERR_HIP 2       /* HIP runtime error                              */
#define AMG_ERR_RCCL 3      /* RCCL error                                      */
#define AMG_ERR_COMM 4      /* host exchange callback failed                  */
#define AMG_ERR_INTERNAL 5  /* invariant violated (bug)                        */
#define AMG_ERR_NOMEM 6     /* host or device allocation failed                */

typedef struct amg_context_s* amg_context;
typedef struct amg_matrix_s* amg_matrix;
typedef struct amg_solver_s* amg_solver;

/* Host-side all-to-all-v of bytes among the ranks of the context.  Used only during
 * setup (halo plans, ghost rows, coarse numbering).  send_bytes[r] bytes starting at
 * sendbuf + sum(send_bytes[0..r)) go to rank r; recv_bytes[r] bytes arrive from rank r,
 * packed the same way.  Must return 0 on success.  The data path never calls it: the
 * solve-time halo exchange is RCCL over xGMI. */
typedef int (*amg_alltoallv_fn)(void* user, const void* sendbuf, const int64_t* send_bytes,
                                void* recvbuf, const int64_t* recv_bytes);

/* ---- error / version ----------------------------------------------------------- */
const char* amg_last_error(void);
int amg_version(void); /* 100 * major + minor */
/* Versions of the runtimes this process actually bound (the loader may have mapped copies
 * other than the ones the library was built against, e.g. a framework's bundled HIP / RCCL):
 * hipRuntimeGetVersion() and ncclGetVersion() (e.g. 22706 = RCCL 2.27.6).               */
int amg_runtime_versions(int32_t* hip_runtime, int32_t* rccl);

/* ---- context (one per GPU / rank) ----------------------------------------------- */
/* hip_stream: a hipStream_t owned by the caller (NULL: the context creates one).      */
int amg_context_create(int device, void* hip_stream, amg_context* out);
/* Multi-GPU: rank/nranks of a row partition, the 128-byte RCCL unique id produced by
 * rank 0's amg_rccl_unique_id(), and the host exchange used during setup.              */
int amg_context_set_comm(amg_context ctx, int rank, int nranks, const void* rccl_unique_id,
                         amg_alltoallv_fn exchange, void* user);
int amg_rccl_unique_id(void* out128);
/* In-process virtual ranks: `nranks` contexts of ONE process (one thread each, any devices)
 * join the world named `world`; halo exchange and allgathers become device-to-device copies
 * ordered by events and host barriers, the setup exchange an in-process all-to-all-v.  For
 * running and testing the multi-rank path on a single GPU (RCCL refuses two ranks per GPU).
 * Every collective call must be made by all ranks, from their own threads. */
int amg_context_set_loopback(amg_context ctx, int rank, int nranks, const char* world);
int amg_context_stream(amg_context ctx, void** hip_stream);
int amg_context_synchronize(amg_context ctx);
int amg_context_destroy(amg_context ctx);

/* ---- ParCSRMatrix ------------------------------------------ */
/* Rank-local rows [first_row, first_row + n_local) of an n_global x n_global matrix;
 * row_ptr[n_local+1], col_global[nnz] (global column ids; sorted per row on entry or
 * sorted by the call), val[nnz].  Collective over the ranks of the context.
 * Memory: on one rank a square matrix also keeps its uploaded CSR on the device (int32
 * row_ptr / col + fp64 val, 4 (n+1) + 12 nnz bytes: ~5 GB for a 256^3 27-point operator) as
 * the level-0 image of a later amg_solver_setup, which takes it over; the first computation
 * on the matrix (amg_par_csr_mult, _residual, ...) frees it instead (a setup after that
 * uploads the operator again).                                                             */
int amg_par_csr_create(amg_context ctx, int64_t n_global, int64_t first_row, int64_t n_local,
                       const int64_t* row_ptr, const int64_t* col_global, const double* val,
                       amg_matrix* out);

#define AMG_STENCIL_5PT 0    /* 2D Poisson, nz must be 1            (BASELINE.json:7)  */
#define AMG_STENCIL_7PT 1    /* 3D Poisson                           (BASELINE.json:8)  */
#define AMG_STENCIL_27PT 2   /* 3D Q1 anisotropic diffusion eps[3]   (BASELINE.json:9)  */
/* Generates this rank's z-slab (2D: y-slab) of the model problem directly on the host of
 * the rank and uploads it: par_stencil_grid analogue.  Collective.                       */
int amg_par_stencil_create(amg_context ctx, int kind, int64_t nx, int64_t ny, int64_t nz,
                           const double* eps3, amg_matrix* out);
/* The same problem numbered box by box: the grid is cut into bx x by x bz boxes (box
 * (ix, iy, iz) covers x in [nx ix / bx, nx (ix + 1) / bx), ...; boxes numbered x fastest),
 * each box's points get consecutive global ids (lexicographic inside the box), and rank r
 * holds boxes [nb r / P, nb (r + 1) / P) -- e.g. 512^3 over 8 GPUs as 2 x 2 x 2 cubes of 256^3
 * instead of z-slabs of 512 x 512 x 64.  The matrix is P A P^T of the natural-order stencil;
 * boxes (1, 1, P) (2D: (1, P, 1)) give exactly amg_par_stencil_create's rows.  Collective. */
int amg_par_stencil_create_boxes(amg_context ctx, int kind, int64_t nx, int64_t ny, int64_t nz,
                                 int64_t bx, int64_t by, int64_t bz, const double* eps3,
                                 amg_matrix* out);

/* ---- unstructured inputs ------------------------------------ */
/* All of these use the even row partition: rank r holds rows [n r / P, n (r+1) / P).
 * Seeded, randomly numbered graph Laplacian on an nx x ny lattice with long-range edges
 * (the offline substitute for SuiteSparse G3_circuit, BASELINE.json:11).  Collective.   */
int amg_par_graph_laplacian_create(amg_context ctx, int64_t nx, int64_t ny, uint64_t seed,
                                   amg_matrix* out);
/* readParMatrix analogue: Matrix Market (coordinate real/integer/pattern, general/
 * symmetric/skew-symmetric; duplicates summed in file order) or binary CSR ("RAMGCSR1"
 * header, then int64 n_rows, n_cols, nnz, int64 row_ptr[n+1], int64 col[nnz], double
 * val[nnz]), detected from the first bytes.  Every rank reads only what it keeps of a
 * binary file.  Collective.                                                              */
int amg_par_csr_read(amg_context ctx, const char* path, amg_matrix* out);
/* Binary CSR writer; every rank writes its rows at their global offsets.  Collective.  */
int amg_par_csr_write(amg_matrix A, const char* path);
#define AMG_REORDER_RCM 1
/* B = P A P^T for a bandwidth-reducing symmetric permutation (reverse Cuthill-McKee on
 * the pattern of A + A^T).  new_to_old_local[n_local of B] receives the old global id of
 * each new local row (x_new[i] = x_old[new_to_old_local[i]]).  Gathers the whole graph
 * on every rank.  Collective.                                                            */
int amg_par_csr_reorder(amg_matrix A, int method, amg_matrix* out, int64_t* new_to_old_local);

typedef struct amg_matrix_info {
    int64_t n_global_rows, n_global_cols;
    int64_t first_row, n_local_rows;
    int64_t first_col, n_local_cols;
    int64_t nnz_local;
    int64_t n_halo;        /* off-process columns received per mult                     */
    int64_t n_send;        /* entries sent per mult                                      */
    int32_t n_neighbors;   /* ranks exchanged with                                       */
    int32_t n_blocks;      /* CSR-stream row blocks                                      */
    int32_t n_vi_blocks;   /* row blocks stored value-indexed (<= 256 distinct values)   */
    int64_t spmv_bytes;    /* HBM bytes one mult() moves in the stored format: headers,  *
                            * index/value streams, row_ptr, x (once), y                  */
    int32_t n_templates;   /* row templates built (0: none; <= 255)                      */
    int64_t template_rows; /* rows mult() runs through the row-template kernel           */
    int32_t format;        /* AMG_FORMAT_* in effect                                     */
    int32_t kernel_variant;/* level-kernel variant bits in effect           */
    int64_t csr_bytes;     /* SURVEY.md 8(d) plain-CSR SpMV bytes: 12 nnz + 4 (n+1) +     *
                            * 8 (local + halo columns) + 8 n                              */
    int32_t tpl_window;    /* template x window, doubles per workgroup (0: none)         */
    int32_t tpl_lanes;     /* window doubles loaded per lane (4, 8, 12, 16; 0: none)      */
    int32_t tpl_march_shift; /* z-marching shift in 512-row blocks (0: no march)          */
    int64_t mult_add_bytes;  /* stored-format bytes of mult_add / residual / jacobi        */
    int64_t residual_bytes;
    int64_t jacobi_bytes;
    int64_t gs_bytes;        /* sliced-ELL bytes of one hybrid GS sweep (0: not built)     */
    int32_t tpl_master;      /* uniform-stencil rows: entries of the master template every *
                              * template is a subsequence of (7, 27; 0: per-template      *
                              * tables)                                    */
    int32_t tile_line_bytes; /* x-tile line width of the block kernels: 64 or 32 (0: no x  *
                              * tile)                                      */
    int32_t gs_split;        /* 1: hybrid GS sweeps run split -- a CSR-block pass over the  *
                              * old-value couplings + the in-chunk chain walk (4.2c)     */
    int32_t gs_chain_maxw;   /* split sweeps: most in-chunk couplings of one row, forward |  *
                              * backward << 16 (the chain walk's widest LDS-queue bucket) */
    int32_t deferred;        /* 1: a level operator whose device formats are not built yet (the  *
                              * V-cycle runs a cycle-order copy): shape fields     *
                              * are valid, format fields 0 until the first compute call builds it */
} amg_matrix_info;
int amg_par_csr_info(amg_matrix A, amg_matrix_info* info);

/* Storage format the level kernels of A use (rows a2-a4).  AUTO (default): row templates
 * where rows share a shape, CSR blocks with x tiles and value indexing elsewhere
 * (DESIGN.md 4.0-4.1).  BLOCKS: CSR blocks on every row.  CSR: plain CSR -- int32 row_ptr,
 * int32 col, fp64 val, exactly the arrays SURVEY.md 8(d) prices (the roofline leg; DESIGN.md
 * 4.5); selecting it uploads those arrays once.  Results are bit-identical in every format. */
#define AMG_FORMAT_AUTO 0
#define AMG_FORMAT_CSR 1
#define AMG_FORMAT_BLOCKS 2
int amg_par_csr_set_format(amg_matrix A, int32_t format);
/* Diagnostic: a 64-bit FNV-1a digest over the device format arrays of A (block-aligned col /
 * val streams, block list and headers, x-tile ids and indices, value tables and indices,
 * diagonal slots, row ends), so two builds of one operator can be compared byte for byte
 * (the GPU-built formats against the host builders, AMG_DEVICE_FORMATS=0). */
int amg_par_csr_format_digest(amg_matrix A, uint64_t* digest);
/* Host copy of the local rows (global column ids). */
int amg_par_csr_export(amg_matrix A, int64_t* row_ptr, int64_t* col_global, double* val);

/* ParCSRMatrix::mult and the level kernels (rows a2-a5).  Device pointers, local length.
 * Each call performs the RCCL halo exchange of x it needs, overlapped with the interior
 * rows.                                                                                  */
int amg_par_csr_mult(amg_matrix A, const double* x, double* y);            /* y = A x       */
int amg_par_csr_mult_add(amg_matrix A, const double* x, double* y);        /* y = y + A x   */
int amg_par_csr_residual(amg_matrix A, const double* x, const double* b, double* r);
int amg_par_csr_jacobi(amg_matrix A, const double* x, const double* b, double* x_out,
                       double omega);
int amg_par_csr_hybrid_gs(amg_matrix A, const double* x, const double* b, double* x_out,
                          int64_t block);
/* the backward sweep (rows of each block in descending order; the V-cycle's post-smoother) */
int amg_par_csr_hybrid_gs_backward(amg_matrix A, const double* x, const double* b, double* x_out,
                                   int64_t block);
/* C = A * B (ParCSRMatrix * ParCSRMatrix, row a10): the Galerkin SpGEMM kernel (one
 * wavefront per output row, LDS hash, canonical accumulation order => bit-identical to the
 * oracle).  A's column partition must equal B's row partition.  Collective.              */
int amg_par_csr_matmat(amg_matrix A, amg_matrix B, amg_matrix* C);
/* ||b - A x||_2 over all ranks (deterministic reduction order). */
int amg_par_csr_residual_norm(amg_matrix A, const double* x, const double* b, double* out);
int amg_par_csr_destroy(amg_matrix A);

/* ---- ParMultilevel (rows a6-a10) -------------------------------------------------- */
#define AMG_COARSEN_RS 0     /* Ruge-Stueben first pass (serial only)                    */
#define AMG_COARSEN_PMIS 1   /* PMIS, partition independent                              */
#define AMG_COARSEN_SA 2     /* smoothed aggregation over MIS(2) aggregates              */
#define AMG_SMOOTH_JACOBI 0
#define AMG_SMOOTH_HYBRID_GS 1
#define AMG_INTERP_CLASSICAL 0  /* RS / PMIS: distance-one classical (modified) interpolation  */
#define AMG_INTERP_EXT_I 1      /* RS / PMIS: distance-two extended+i with P_max truncation    *
                                 * (one rank)                                    */

typedef struct amg_options {
    int32_t coarsen;
    int32_t smoother;
    double strong_threshold;  /* 0.25 classical, 0.08 SA (x 0.75 per level)               */
    double jacobi_omega;      /* 2/3                                                     */
    int32_t pre_sweeps, post_sweeps;
    int32_t max_levels;
    int64_t max_coarse;       /* stop when the global size is <= this; dense solve there */
    int64_t gs_block;         /* hybrid GS block (global row multiples)                 */
    uint64_t seed;            /* PMIS / MIS(2) hash seed                                 */
    int32_t setup_device;     /* 1 (default): setup on the GPU -- strength, PMIS / MIS(2),
                                 P, R = P^T (one rank; several ranks: host) and the
                                 Galerkin SpGEMM R(AP); 2: Galerkin SpGEMM only; 0: host.
                                 Results are identical in every mode.                     */
    int64_t replicate_below;  /* multi-rank: levels with <= this many global rows are held
                                 whole by every rank and cycled without communication (one
                                 allgather of b per cycle); 0 = never.  Default 262144.     */
    int32_t interp;           /* RS / PMIS: AMG_INTERP_CLASSICAL (default) or AMG_INTERP_EXT_I */
    int32_t p_max;            /* AMG_INTERP_EXT_I: interpolation entries kept per row (the
                                 largest |w|, rescaled to the row sum); 0 = all.  Default 4  */
    double drop_tol;          /* coarse-operator drop tolerance (non-Galerkin): off-diagonals of
                                 A_{l+1} = R A_l P with |a_ij| < drop_tol sqrt(|a_ii a_jj|) are
                                 added to the diagonal (row order; row sums kept).  0 = the
                                 Galerkin operator (default).  DESIGN.md 3                  */
} amg_options;

#define AMG_PRESET_PMIS_JACOBI 0  /* config 2/4: 7-pt Poisson, Jacobi V-cycle            */
#define AMG_PRESET_RS_JACOBI 1    /* config 1: 2D 5-pt, Ruge-Stueben                      */
#define AMG_PRESET_SA_HYBRID_GS 2 /* config 3/5: smoothed aggregation + hybrid GS         */
int amg_options_default(int preset, amg_options* opt);

int amg_solver_setup(amg_matrix A, const amg_options* opt, amg_solver* out);
int amg_solver_num_levels(amg_solver S, int32_t* out);

typedef struct amg_level_info {
    int64_t n_global, nnz_global;          /* A_l                                        */
    int64_t n_local, nnz_local;
    int64_t p_nnz_local, r_nnz_local;      /* P_l, R_l (0 on the coarsest level)         */
    int64_t bytes_per_cycle_local;         /* plain-CSR bytes of the level's
                                              share of one V-cycle                         */
    int64_t stored_bytes_per_cycle_local;  /* the same, in the stored formats the kernels
                                              stream (templates, CSR-VI blocks, sliced ELL) */
} amg_level_info;
int amg_solver_level_info(amg_solver S, int32_t level, amg_level_info* info);
/* which: 0 = A_l, 1 = P_l, 2 = R_l; 3, 4, 5 = the same operators as the V-cycle runs them
   (a Jacobi level of a grid-built hierarchy runs its points in a private brick order on one
   rank, DESIGN.md 4.1 r5: these operators then apply to vectors in that order; elsewhere they
   are 0, 1, 2).  Borrowed handle, valid while S lives. */
int amg_solver_level_matrix(amg_solver S, int32_t level, int32_t which, amg_matrix* out);
/* Integer setup result of level l for the local rows: C/F marker (1 = C, 0 = F) for
 * RS/PMIS, global aggregate id for SA.  Bit-exact against the oracle. */
int amg_solver_level_split(amg_solver S, int32_t level, int32_t* out_local);
/* One V-cycle x <- cycle(x, b) (ParMultilevel::cycle). */
int amg_solver_cycle(amg_solver S, double* x, const double* b);
/* ParMultilevel::solve: r0 = ||b-Ax||; up to max_iter cycles until ||r||/r0 < tol.
 * hist (host, max_iter+1 doubles) receives the residual history; *iters the count.
 * Norms stay on the device until the end: no host sync inside the loop. */
int amg_solver_solve(amg_solver S, double* x, const double* b, int32_t max_iter, double tol,
                     double* hist, int32_t* iters);
/* Conjugate gradients preconditioned by one V-cycle per iteration (row f3: the natural
 * caller of the cycle).  Same contract as amg_solver_solve; hist receives ||r_k||. */
int amg_solver_pcg(amg_solver S, double* x, const double* b, int32_t max_iter, double tol,
                   double* hist, int32_t* iters);
/* Capture each V-cycle in a hipGraph and replay it (1 = on).  Default: on for 1 rank; off
 * for loopback ranks (they meet at host barriers); for RCCL ranks on where the process runs
 * the runtime whole-cycle capture was validated on (HIP >= 7.2 with RCCL >= 2.27.7: the
 * send/recv groups and allgathers are captured with the kernels, each replay waited for
 * before the next enqueue).  On older runtimes (torch's bundled HIP 7.0 / RCCL 2.26.6)
 * enable = 1 with several ranks returns AMG_ERR_INVALID naming the versions;
 * AMG_RCCL_GRAPH=1 / 0 in the environment overrides the version check. */
int amg_solver_set_graph(amg_solver S, int32_t enable);
/* 1 while cycles replay a hipGraph (0 after set_graph(0), or if the runtime refused to
 * instantiate a multi-rank graph and the solver fell back to eager launches). */
int amg_solver_get_graph(amg_solver S, int32_t* enabled);
/* In-graph time of every operation of one V-cycle (one rank; measurement, no reference
 * counterpart): the cycle is captured into one graph with an event-record node after every
 * operation (smoothing sweep, residual, restriction, coarse solve, interpolation) and replayed
 * `reps` times; us[k] is the median event-to-event time of operation k in microseconds,
 * labels + k * label_bytes its NUL-terminated name "L<level> <op>".  *in_graph: 2 = that
 * graph; 1 = a runtime that does not time event nodes: one graph per operation, replayed back
 * to back with timing events between them (each time then includes a graph launch); 0 = eager
 * cycles (graphs off).  *n_ops receives the operation count (only the first n_max are
 * written).  x is updated by the reps cycles like amg_solver_cycle. */
int amg_solver_cycle_timeline(amg_solver S, double* x, const double* b, int32_t reps, int32_t n_max,
                              double* us, char* labels, int32_t label_bytes, int32_t* n_ops,
                              int32_t* in_graph);
int amg_solver_destroy(amg_solver S);

/* ---- host-only hierarchy (no GPU needed) ------------------------------------------ */
/* The setup half of ParMultilevel (rows a8-a10) run on the CPU of each rank: exactly the
 * code amg_solver_setup() runs before uploading.  Exposed for inspection and for CPU
 * parity tests (multi-rank through `exchange`; NULL allowed when nranks == 1).           */
typedef struct amg_host_hierarchy_s* amg_host_hierarchy;
int amg_host_hierarchy_build(int rank, int nranks, amg_alltoallv_fn exchange, void* user,
                             int64_t n_global, int64_t first_row, int64_t n_local,
                             const int64_t* row_ptr, const int64_t* col_global,
                             const double* val, const amg_options* opt,
                             amg_host_hierarchy* out);
int amg_host_hierarchy_num_levels(amg_host_hierarchy H, int32_t* out);
/* which: 0 = A_l, 1 = P_l, 2 = R_l.  sizes[5] = {n_global_rows, n_global_cols, first_row,
 * n_local_rows, nnz_local}. */
int amg_host_hierarchy_level_size(amg_host_hierarchy H, int32_t level, int32_t which,
                                  int64_t* sizes5);
int amg_host_hierarchy_level_export(amg_host_hierarchy H, int32_t level, int32_t which,
                                    int64_t* row_ptr, int64_t* col_global, double* val);
int amg_host_hierarchy_level_split(amg_host_hierarchy H, int32_t level, int32_t* out_local);
/* row-major n_c x n_c inverse of the coarsest operator (identical on every rank) */
int amg_host_hierarchy_coarse_inverse(amg_host_hierarchy H, double* out);
int amg_host_hierarchy_destroy(amg_host_hierarchy H);

/* Host-only halves of the unstructured-input calls above (no GPU needed): the exact code
 * the amg_par_* versions run before uploading.  sizes5 as for the hierarchy levels.      */
typedef struct amg_host_csr_s* amg_host_csr;
int amg_host_csr_graph_laplacian(int rank, int nranks, int64_t nx, int64_t ny, uint64_t seed,
                                 amg_host_csr* out);
int amg_host_csr_stencil(int rank, int nranks, int kind, int64_t nx, int64_t ny, int64_t nz,
                         int64_t bx, int64_t by, int64_t bz, const double* eps3, amg_host_csr* out);
int amg_host_csr_read(int rank, int nranks, const char* path, amg_host_csr* out);
int amg_host_csr_write(int rank, int nranks, amg_alltoallv_fn exchange, void* user,
                       amg_host_csr A, const char* path);
int amg_host_csr_reorder(int rank, int nranks, amg_alltoallv_fn exchange, void* user,
                         amg_host_csr A, int method, amg_host_csr* out, int64_t* new_to_old_local);
int amg_host_csr_size(amg_host_csr A, int64_t* sizes5);
int amg_host_csr_export(amg_host_csr A, int64_t* row_ptr, int64_t* col_global, double* val);
int amg_host_csr_destroy(amg_host_csr A);

/* ---- vectors ---------------------------------------------------------------------- */
/* out[i] = uniform(-1,1) from splitmix64(seed, first_gid + i) on the device. */
int amg_vector_uniform(amg_context ctx, int64_t n, int64_t first_gid, uint64_t seed,
                       double* out);
/* dst = src on the context stream (16-byte nontemporal copy kernel; 16-byte aligned device
 * pointers).  bench.py times it as the box's STREAM-copy ceiling. */
int amg_vector_copy(amg_context ctx, int64_t n, const double* src, double* dst);
/* One read pass over src (16-byte loads, as amg_vector_copy without the stores), per-wave
 * partial sums into partials[n_partials] (n_partials >= 4 * ceil(n / 2048)).  bench.py times
 * it as the box's read-bandwidth ceiling: most level kernels read far more than they write. */
int amg_vector_read(amg_context ctx, int64_t n, const double* src, double* partials, int64_t n_partials);

/* ---- device memory and timing (torch-free callers) --------------------------------- */
/* What a caller without a framework needs around the compute calls: device buffers, copies,
 * and events on the context stream (bench.py and the RCCL workers use these so that the
 * process binds the HIP runtime and RCCL the library was built against).  */
int amg_device_malloc(amg_context ctx, int64_t bytes, void** out);
/* waits for the context stream, then frees */
int amg_device_free(amg_context ctx, void* p);
/* bytes from src to dst, host or device on either side (unified addressing), ordered after
 * the work already on the context stream; returns when the copy has landed.             */
int amg_memcpy(amg_context ctx, void* dst, const void* src, int64_t bytes);
/* device memset, enqueued on the context stream */
int amg_memset_async(amg_context ctx, void* p, int value, int64_t bytes);
typedef struct amg_event_s* amg_event;
int amg_event_create(amg_context ctx, amg_event* out);
int amg_event_record(amg_event e);                                   /* on the context stream */
int amg_event_elapsed_ms(amg_event start, amg_event end, float* ms); /* waits for `end`       */
int amg_event_destroy(amg_event e);

#ifdef __cplusplus
}
#endif
#endif
