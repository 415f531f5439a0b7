/*
 * amg_oracle.c -- serial CPU restatement of the AMG V-cycle hot path.  TEST INFRASTRUCTURE.
 *
 * Used only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
 * checker.  PARITY UNPINNED against Siddarthareddy1/raptor (the reference has no AMG code,
 * SURVEY.md section 0); pinned instead to scipy.sparse fixtures in tests/golden/.
 * Each function cites the spec row it restates: BASELINE.json:5 (north_star) and the
 * SURVEY.md section 8(a) row ids a1..a11.  Algorithm definitions (tie-breaks, summation
 * order) are the ones in DESIGN.md section 3; the product implements the same definitions
 * independently in raptor_amd/csrc/.
 *
 * Deliberately simple: one loop nest per definition, int64 indices, no threads except
 * optional OpenMP on row-independent level kernels (bit-identical for any thread count).
 */
#include "amg_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define XMALLOC(T, n) ((T*)xmalloc(sizeof(T) * (size_t)((n) > 0 ? (n) : 1)))
static void* xmalloc(size_t b) {
    void* p = malloc(b);
    if (!p) {
        fprintf(stderr, "amg_oracle: out of memory (%zu bytes)\n", b);
        abort();
    }
    return p;
}

/* ------------------------------------------------------------------------------ */
/* CSR objects                                                                     */
/* ------------------------------------------------------------------------------ */
static orc_csr* csr_alloc(int64_t n_rows, int64_t n_cols, int64_t nnz) {
    orc_csr* A = XMALLOC(orc_csr, 1);
    A->n_rows = n_rows;
    A->n_cols = n_cols;
    A->rp = XMALLOC(int64_t, n_rows + 1);
    A->col = XMALLOC(int64_t, nnz);
    A->val = XMALLOC(double, nnz);
    return A;
}

orc_csr* orc_csr_new(int64_t n_rows, int64_t n_cols, const int64_t* rp, const int64_t* col,
                     const double* val) {
    int64_t nnz = rp[n_rows];
    orc_csr* A = csr_alloc(n_rows, n_cols, nnz);
    memcpy(A->rp, rp, sizeof(int64_t) * (size_t)(n_rows + 1));
    memcpy(A->col, col, sizeof(int64_t) * (size_t)nnz);
    memcpy(A->val, val, sizeof(double) * (size_t)nnz);
    return A;
}

void orc_csr_free(orc_csr* A) {
    if (!A) return;
    free(A->rp);
    free(A->col);
    free(A->val);
    free(A);
}

int64_t orc_csr_nnz(const orc_csr* A) { return A->rp[A->n_rows]; }
int64_t orc_csr_rows(const orc_csr* A) { return A->n_rows; }
int64_t orc_csr_cols(const orc_csr* A) { return A->n_cols; }

void orc_csr_export(const orc_csr* A, int64_t* rp, int64_t* col, double* val) {
    int64_t nnz = A->rp[A->n_rows];
    memcpy(rp, A->rp, sizeof(int64_t) * (size_t)(A->n_rows + 1));
    memcpy(col, A->col, sizeof(int64_t) * (size_t)nnz);
    memcpy(val, A->val, sizeof(double) * (size_t)nnz);
}

static double diag_of(const orc_csr* A, int64_t i) {
    for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k)
        if (A->col[k] == i) return A->val[k];
    return 0.0;
}

/* ------------------------------------------------------------------------------ */
/* Model problems (SURVEY.md 8d "Synthetic inputs"; BASELINE.json:7-9)             */
/* Dirichlet, interior nodes only, row id = i + nx*(j + ny*k), columns ascending.  */
/* ------------------------------------------------------------------------------ */
orc_csr* orc_gen_5pt(int64_t nx, int64_t ny) {
    int64_t n = nx * ny;
    orc_csr* A = csr_alloc(n, n, 5 * n);
    int64_t nnz = 0;
    A->rp[0] = 0;
    for (int64_t j = 0; j < ny; ++j)
        for (int64_t i = 0; i < nx; ++i) {
            int64_t r = i + nx * j;
            if (j > 0) { A->col[nnz] = r - nx; A->val[nnz++] = -1.0; }
            if (i > 0) { A->col[nnz] = r - 1; A->val[nnz++] = -1.0; }
            A->col[nnz] = r; A->val[nnz++] = 4.0;
            if (i < nx - 1) { A->col[nnz] = r + 1; A->val[nnz++] = -1.0; }
            if (j < ny - 1) { A->col[nnz] = r + nx; A->val[nnz++] = -1.0; }
            A->rp[r + 1] = nnz;
        }
    return A;
}

orc_csr* orc_gen_7pt(int64_t nx, int64_t ny, int64_t nz) {
    int64_t n = nx * ny * nz, pl = nx * ny;
    orc_csr* A = csr_alloc(n, n, 7 * n);
    int64_t nnz = 0;
    A->rp[0] = 0;
    for (int64_t k = 0; k < nz; ++k)
        for (int64_t j = 0; j < ny; ++j)
            for (int64_t i = 0; i < nx; ++i) {
                int64_t r = i + nx * (j + ny * k);
                if (k > 0) { A->col[nnz] = r - pl; A->val[nnz++] = -1.0; }
                if (j > 0) { A->col[nnz] = r - nx; A->val[nnz++] = -1.0; }
                if (i > 0) { A->col[nnz] = r - 1; A->val[nnz++] = -1.0; }
                A->col[nnz] = r; A->val[nnz++] = 6.0;
                if (i < nx - 1) { A->col[nnz] = r + 1; A->val[nnz++] = -1.0; }
                if (j < ny - 1) { A->col[nnz] = r + nx; A->val[nnz++] = -1.0; }
                if (k < nz - 1) { A->col[nnz] = r + pl; A->val[nnz++] = -1.0; }
                A->rp[r + 1] = nnz;
            }
    return A;
}

/* Trilinear (Q1) FE stiffness of -div(diag(ex,ey,ez) grad u), scaled by 36:
 * s(dx,dy,dz) = ex*K[dx]*m[dy]*m[dz] + ey*m[dx]*K[dy]*m[dz] + ez*m[dx]*m[dy]*K[dz]
 * with K = {-1, 2, -1}, m = {1, 4, 1}; evaluated left to right in fp64. */
static double stencil27(int dx, int dy, int dz, double ex, double ey, double ez) {
    static const double K[3] = {-1.0, 2.0, -1.0};
    static const double m[3] = {1.0, 4.0, 1.0};
    double t1 = ex * K[dx + 1] * m[dy + 1] * m[dz + 1];
    double t2 = ey * m[dx + 1] * K[dy + 1] * m[dz + 1];
    double t3 = ez * m[dx + 1] * m[dy + 1] * K[dz + 1];
    return t1 + t2 + t3;
}

orc_csr* orc_gen_27pt(int64_t nx, int64_t ny, int64_t nz, double ex, double ey, double ez) {
    int64_t n = nx * ny * nz;
    orc_csr* A = csr_alloc(n, n, 27 * n);
    int64_t nnz = 0;
    A->rp[0] = 0;
    for (int64_t k = 0; k < nz; ++k)
        for (int64_t j = 0; j < ny; ++j)
            for (int64_t i = 0; i < nx; ++i) {
                int64_t r = i + nx * (j + ny * k);
                for (int dz = -1; dz <= 1; ++dz)
                    for (int dy = -1; dy <= 1; ++dy)
                        for (int dx = -1; dx <= 1; ++dx) {
                            int64_t ii = i + dx, jj = j + dy, kk = k + dz;
                            if (ii < 0 || ii >= nx || jj < 0 || jj >= ny || kk < 0 || kk >= nz)
                                continue;
                            A->col[nnz] = ii + nx * (jj + ny * kk);
                            A->val[nnz++] = stencil27(dx, dy, dz, ex, ey, ez);
                        }
                A->rp[r + 1] = nnz;
            }
    return A;
}

static uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void orc_vec_uniform(int64_t n, int64_t first_gid, uint64_t seed, double* out) {
    for (int64_t i = 0; i < n; ++i) {
        uint64_t u = mix64(seed * 0xD1B54A32D192ED03ull + (uint64_t)(first_gid + i));
        out[i] = (double)(u >> 11) * 0x1.0p-52 - 1.0;
    }
}

static uint32_t hash32(int64_t gid, uint64_t seed) {
    return (uint32_t)(mix64((uint64_t)gid ^ (seed * 0x9E3779B97F4A7C15ull)) >> 32);
}

/* ------------------------------------------------------------------------------ */
/* Level kernels: SpMV / residual / Jacobi / hybrid GS (rows a2-a5).               */
/* Every row sum is s = 0; s += a_ij * x_j in CSR order (no FMA).                  */
/* ------------------------------------------------------------------------------ */
static inline double row_dot(const orc_csr* A, int64_t i, const double* x) {
    double s = 0.0;
    for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) s += A->val[k] * x[A->col[k]];
    return s;
}

void orc_spmv(const orc_csr* A, const double* x, double* y) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < A->n_rows; ++i) y[i] = row_dot(A, i, x);
}

void orc_spmv_add(const orc_csr* A, const double* x, double* y) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < A->n_rows; ++i) y[i] = y[i] + row_dot(A, i, x);
}

void orc_residual(const orc_csr* A, const double* x, const double* b, double* r) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < A->n_rows; ++i) r[i] = b[i] - row_dot(A, i, x);
}

/* x_out_i = x_i + omega * (dinv_i * (b_i - (A x)_i)),  dinv_i = 1.0 / a_ii */
void orc_jacobi(const orc_csr* A, const double* x, const double* b, double* xout, double omega) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < A->n_rows; ++i) {
        double dinv = 1.0 / diag_of(A, i);
        xout[i] = x[i] + omega * (dinv * (b[i] - row_dot(A, i, x)));
    }
}

/* Hybrid Gauss-Seidel (row a5): blocks [B*q, B*q+B); inside a block forward GS, across
 * blocks Jacobi.  acc = b_i; acc -= a_ij*x_j over "old" entries (j != i, j outside
 * [block_start, i)) in CSR order; then acc -= a_ij*xnew_j over in-block lower entries in
 * CSR order; xnew_i = acc * dinv_i. */
/* one GS block [s, e) of the l1 hybrid Gauss-Seidel: Gauss-Seidel inside the
 * block, Jacobi for couplings outside it, and the diagonal augmented by the l1 norm of the
 * outside couplings, d_i = a_ii + sum_{j outside} |a_ij| (summed in CSR order), applied in
 * correction form x_i' = x_i + r_i / d_i, which makes the sweep convergent for any SPD A.  Forward: rows s..e-1, new values for in-block j < i;
 * backward: rows e-1..s, new values for in-block j > i.  Old-value couplings are subtracted
 * first in CSR order, then new-value couplings in sweep order (ascending j forward,
 * descending j backward). */
static void gs_block_rows(const orc_csr* A, const double* x, const double* b, double* xout,
                          int64_t s, int64_t e, int backward) {
    for (int64_t t = 0; t < e - s; ++t) {
        int64_t i = backward ? e - 1 - t : s + t;
        int64_t lo = backward ? i + 1 : s, hi = backward ? e : i; /* new-value range [lo, hi) */
        double acc = b[i], l1 = 0.0;
        for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) {
            int64_t j = A->col[k];
            if (j < s || j >= e) l1 += fabs(A->val[k]);
        }
        double dinv = 1.0 / (diag_of(A, i) + l1);
        for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) {
            int64_t j = A->col[k];
            if (j >= lo && j < hi) continue;
            acc -= A->val[k] * x[j]; /* includes the diagonal, old x_i */
        }
        if (!backward) {
            for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) {
                int64_t j = A->col[k];
                if (j >= lo && j < hi) acc -= A->val[k] * xout[j];
            }
        } else {
            for (int64_t k = A->rp[i + 1] - 1; k >= A->rp[i]; --k) {
                int64_t j = A->col[k];
                if (j >= lo && j < hi) acc -= A->val[k] * xout[j];
            }
        }
        xout[i] = x[i] + acc * dinv; /* correction form: the fixed point solves A x = b */
    }
}

/* Blocks = global multiples of `block` clipped to the rank segments [cuts[t], cuts[t+1])
 * (cuts[0] = 0, the last segment ends at n): GS never reaches across a rank boundary,
 * exactly like the product's per-rank blocks. */
void orc_hybrid_gs_cut(const orc_csr* A, const double* x, const double* b, double* xout,
                       int64_t block, int32_t backward, int32_t ncuts, const int64_t* cuts) {
    int64_t n = A->n_rows;
    for (int32_t t = 0; t < ncuts; ++t) {
        int64_t lo = cuts[t], hi = t + 1 < ncuts ? cuts[t + 1] : n;
        if (hi <= lo) continue;
        int64_t q0 = lo / block, q1 = (hi - 1) / block;
#pragma omp parallel for schedule(static)
        for (int64_t q = q0; q <= q1; ++q) {
            int64_t s = q * block > lo ? q * block : lo;
            int64_t e = (q + 1) * block < hi ? (q + 1) * block : hi;
            gs_block_rows(A, x, b, xout, s, e, backward);
        }
    }
}

void orc_hybrid_gs(const orc_csr* A, const double* x, const double* b, double* xout,
                   int64_t block) {
    const int64_t zero = 0;
    orc_hybrid_gs_cut(A, x, b, xout, block, 0, 1, &zero);
}

void orc_hybrid_gs_backward(const orc_csr* A, const double* x, const double* b, double* xout,
                            int64_t block) {
    const int64_t zero = 0;
    orc_hybrid_gs_cut(A, x, b, xout, block, 1, 1, &zero);
}

double orc_norm2(int64_t n, const double* v) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) s += v[i] * v[i];
    return sqrt(s);
}

/* ------------------------------------------------------------------------------ */
/* Transpose and SpGEMM (row a10).                                                  */
/* ------------------------------------------------------------------------------ */
orc_csr* orc_transpose(const orc_csr* A) {
    int64_t nnz = orc_csr_nnz(A);
    orc_csr* T = csr_alloc(A->n_cols, A->n_rows, nnz);
    memset(T->rp, 0, sizeof(int64_t) * (size_t)(A->n_cols + 1));
    for (int64_t k = 0; k < nnz; ++k) T->rp[A->col[k] + 1]++;
    for (int64_t c = 0; c < A->n_cols; ++c) T->rp[c + 1] += T->rp[c];
    int64_t* pos = XMALLOC(int64_t, A->n_cols);
    memcpy(pos, T->rp, sizeof(int64_t) * (size_t)A->n_cols);
    for (int64_t i = 0; i < A->n_rows; ++i) /* ascending i => rows of T sorted */
        for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) {
            int64_t p = pos[A->col[k]]++;
            T->col[p] = i;
            T->val[p] = A->val[k];
        }
    free(pos);
    return T;
}

static int cmp_i64(const void* a, const void* b) {
    int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    return (x > y) - (x < y);
}

/* C = A*B.  Row i: acc_j = 0.0, then for k in A row i (CSR order), for j in B row k (CSR
 * order): acc_j += a_ik * b_kj.  Pattern = structural union (zeros kept), cols sorted. */
orc_csr* orc_spgemm(const orc_csr* A, const orc_csr* B) {
    int64_t n = A->n_rows, m = B->n_cols;
    int64_t* mark = XMALLOC(int64_t, m);
    double* acc = XMALLOC(double, m);
    for (int64_t j = 0; j < m; ++j) mark[j] = -1;
    int64_t cap = orc_csr_nnz(A) + orc_csr_nnz(B) + 16, nnz = 0;
    int64_t* rp = XMALLOC(int64_t, n + 1);
    int64_t* col = XMALLOC(int64_t, cap);
    double* val = XMALLOC(double, cap);
    int64_t* list = XMALLOC(int64_t, m);
    rp[0] = 0;
    for (int64_t i = 0; i < n; ++i) {
        int64_t len = 0;
        for (int64_t ka = A->rp[i]; ka < A->rp[i + 1]; ++ka) {
            int64_t k = A->col[ka];
            double a = A->val[ka];
            for (int64_t kb = B->rp[k]; kb < B->rp[k + 1]; ++kb) {
                int64_t j = B->col[kb];
                if (mark[j] != i) {
                    mark[j] = i;
                    acc[j] = 0.0;
                    list[len++] = j;
                }
                acc[j] += a * B->val[kb];
            }
        }
        qsort(list, (size_t)len, sizeof(int64_t), cmp_i64);
        if (nnz + len > cap) {
            while (nnz + len > cap) cap *= 2;
            col = (int64_t*)realloc(col, sizeof(int64_t) * (size_t)cap);
            val = (double*)realloc(val, sizeof(double) * (size_t)cap);
            if (!col || !val) abort();
        }
        for (int64_t t = 0; t < len; ++t) {
            col[nnz] = list[t];
            val[nnz++] = acc[list[t]];
        }
        rp[i + 1] = nnz;
    }
    free(mark);
    free(acc);
    free(list);
    orc_csr* C = XMALLOC(orc_csr, 1);
    C->n_rows = n;
    C->n_cols = m;
    C->rp = rp;
    C->col = col;
    C->val = val;
    return C;
}

/* ------------------------------------------------------------------------------ */
/* Strength of connection (rows a8, a9).                                            */
/* ------------------------------------------------------------------------------ */
/* classical: m_i = max_{j != i} (-a_ij); if m_i <= 0 no strong; else j strong iff
 * -a_ij >= theta * m_i.  S keeps a_ij as its value, never the diagonal. */
orc_csr* orc_strength_classical(const orc_csr* A, double theta) {
    int64_t n = A->n_rows, nnz = 0;
    orc_csr* S = csr_alloc(n, A->n_cols, orc_csr_nnz(A));
    S->rp[0] = 0;
    for (int64_t i = 0; i < n; ++i) {
        double mx = 0.0;
        int any = 0;
        for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) {
            if (A->col[k] == i) continue;
            double v = -A->val[k];
            if (!any || v > mx) mx = v;
            any = 1;
        }
        if (any && mx > 0.0) {
            double thr = theta * mx;
            for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) {
                if (A->col[k] == i) continue;
                if (-A->val[k] >= thr) {
                    S->col[nnz] = A->col[k];
                    S->val[nnz++] = A->val[k];
                }
            }
        }
        S->rp[i + 1] = nnz;
    }
    return S;
}

/* symmetric, signed (SA, r6): j != i strong iff -a_ij >= theta * sqrt(|a_ii * a_jj|).
 * Positive couplings are never strong: the 27-pt Q1 operator's +16 z couplings (eps_z = 1e-3)
 * made |a_ij| aggregates span the weakly coupled direction. */
static int sa_strong(double aij, double di, double dj, double theta) {
    return -aij >= theta * sqrt(fabs(di * dj));
}

orc_csr* orc_strength_symmetric(const orc_csr* A, double theta) {
    int64_t n = A->n_rows, nnz = 0;
    double* d = XMALLOC(double, n);
    for (int64_t i = 0; i < n; ++i) d[i] = diag_of(A, i);
    orc_csr* S = csr_alloc(n, A->n_cols, orc_csr_nnz(A));
    S->rp[0] = 0;
    for (int64_t i = 0; i < n; ++i) {
        for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) {
            int64_t j = A->col[k];
            if (j == i) continue;
            if (sa_strong(A->val[k], d[i], d[j], theta)) {
                S->col[nnz] = j;
                S->val[nnz++] = A->val[k];
            }
        }
        S->rp[i + 1] = nnz;
    }
    free(d);
    return S;
}

/* ------------------------------------------------------------------------------ */
/* Ruge-Stueben first pass (row a8).  lambda_i = |S^T_i|; repeatedly take the       */
/* undecided point with the largest lambda (ties: smallest index) as C; its         */
/* undecided dependents become F (and raise lambda of the points they depend on);  */
/* undecided points it depends on lose one lambda.  Isolated points are F.          */
/* ------------------------------------------------------------------------------ */
enum { ST_U = -1, ST_F = 0, ST_C = 1 };

typedef struct { int64_t lam, idx; } hent;
static int hbetter(hent a, hent b) { return a.lam > b.lam || (a.lam == b.lam && a.idx < b.idx); }
typedef struct { hent* a; int64_t n, cap; } heap;
static void hpush(heap* h, int64_t lam, int64_t idx) {
    if (h->n == h->cap) {
        h->cap = h->cap ? h->cap * 2 : 1024;
        h->a = (hent*)realloc(h->a, sizeof(hent) * (size_t)h->cap);
        if (!h->a) abort();
    }
    int64_t c = h->n++;
    hent e = {lam, idx};
    while (c > 0) {
        int64_t p = (c - 1) / 2;
        if (!hbetter(e, h->a[p])) break;
        h->a[c] = h->a[p];
        c = p;
    }
    h->a[c] = e;
}
static hent hpop(heap* h) {
    hent top = h->a[0], last = h->a[--h->n];
    int64_t c = 0;
    for (;;) {
        int64_t l = 2 * c + 1, r = l + 1, b = c;
        hent be = last;
        if (l < h->n && hbetter(h->a[l], be)) { b = l; be = h->a[l]; }
        if (r < h->n && hbetter(h->a[r], be)) { b = r; be = h->a[r]; }
        if (b == c) break;
        h->a[c] = h->a[b];
        c = b;
    }
    if (h->n > 0) h->a[c] = last;
    return top;
}

void orc_rs_split(const orc_csr* S, int32_t* cf) {
    int64_t n = S->n_rows;
    orc_csr* ST = orc_transpose(S);
    int64_t* lam = XMALLOC(int64_t, n);
    heap h = {0, 0, 0};
    for (int64_t i = 0; i < n; ++i) {
        int64_t ns = S->rp[i + 1] - S->rp[i], nt = ST->rp[i + 1] - ST->rp[i];
        cf[i] = (ns == 0 && nt == 0) ? ST_F : ST_U;
        lam[i] = nt;
        if (cf[i] == ST_U) hpush(&h, lam[i], i);
    }
    while (h.n > 0) {
        hent e = hpop(&h);
        int64_t i = e.idx;
        if (cf[i] != ST_U || e.lam != lam[i]) continue;
        cf[i] = ST_C;
        for (int64_t t = ST->rp[i]; t < ST->rp[i + 1]; ++t) {
            int64_t j = ST->col[t];
            if (cf[j] != ST_U) continue;
            cf[j] = ST_F;
            for (int64_t u = S->rp[j]; u < S->rp[j + 1]; ++u) {
                int64_t k = S->col[u];
                if (cf[k] == ST_U) {
                    lam[k]++;
                    hpush(&h, lam[k], k);
                }
            }
        }
        for (int64_t t = S->rp[i]; t < S->rp[i + 1]; ++t) {
            int64_t j = S->col[t];
            if (cf[j] == ST_U) {
                lam[j]--;
                hpush(&h, lam[j], j);
            }
        }
    }
    free(h.a);
    free(lam);
    orc_csr_free(ST);
}

/* ------------------------------------------------------------------------------ */
/* PMIS (row a8; partition-independent).  key_i = (|S^T_i| << 32) | hash32(i), ties  */
/* by larger index.  Points with |S^T_i| = 0 start F.  Each round (synchronous):    */
/* undecided i becomes C iff key_i beats every undecided j in S_i u S^T_i; then     */
/* undecided i with a C point in S_i becomes F.                                     */
/* ------------------------------------------------------------------------------ */
static int key_gt(uint64_t ka, int64_t ia, uint64_t kb, int64_t ib) {
    return ka > kb || (ka == kb && ia > ib);
}

void orc_pmis_split(const orc_csr* S, uint64_t seed, int32_t* cf) {
    int64_t n = S->n_rows;
    orc_csr* ST = orc_transpose(S);
    uint64_t* key = XMALLOC(uint64_t, n);
    int32_t* newc = XMALLOC(int32_t, n);
    int64_t nu = 0;
    for (int64_t i = 0; i < n; ++i) {
        uint64_t cnt = (uint64_t)(ST->rp[i + 1] - ST->rp[i]);
        key[i] = (cnt << 32) | (uint64_t)hash32(i, seed);
        cf[i] = cnt == 0 ? ST_F : ST_U;
        nu += cf[i] == ST_U;
    }
    while (nu > 0) {
        for (int64_t i = 0; i < n; ++i) {
            newc[i] = 0;
            if (cf[i] != ST_U) continue;
            int best = 1;
            for (int64_t t = S->rp[i]; t < S->rp[i + 1] && best; ++t) {
                int64_t j = S->col[t];
                if (cf[j] == ST_U && key_gt(key[j], j, key[i], i)) best = 0;
            }
            for (int64_t t = ST->rp[i]; t < ST->rp[i + 1] && best; ++t) {
                int64_t j = ST->col[t];
                if (cf[j] == ST_U && key_gt(key[j], j, key[i], i)) best = 0;
            }
            newc[i] = best;
        }
        for (int64_t i = 0; i < n; ++i)
            if (newc[i]) cf[i] = ST_C;
        nu = 0;
        for (int64_t i = 0; i < n; ++i) {
            if (cf[i] != ST_U) continue;
            for (int64_t t = S->rp[i]; t < S->rp[i + 1]; ++t)
                if (cf[S->col[t]] == ST_C) {
                    cf[i] = ST_F;
                    break;
                }
            nu += cf[i] == ST_U;
        }
    }
    free(key);
    free(newc);
    orc_csr_free(ST);
}

/* ------------------------------------------------------------------------------ */
/* Classical (modified) interpolation, distance 1 (row a8).                          */
/* F row i: C_i = strong C neighbours; d = a_ii + sum of weak a_ij (CSR order); for  */
/* each strong F neighbour k (CSR order): s_k = sum of a_km over m in C_i whose sign */
/* is opposite to a_kk (row k order); s_k == 0 -> d += a_ik, else num_m +=           */
/* (a_ik * a_km) / s_k over the same m (row k order); num_j starts at a_ij.          */
/* w_ij = -num_j / d.  C row: 1 at its coarse index.                                 */
/* ------------------------------------------------------------------------------ */
orc_csr* orc_interp_classical(const orc_csr* A, const orc_csr* S, const int32_t* cf) {
    int64_t n = A->n_rows;
    int64_t* cmap = XMALLOC(int64_t, n);
    int64_t nc = 0;
    for (int64_t i = 0; i < n; ++i) cmap[i] = cf[i] == ST_C ? nc++ : -1;
    int64_t* strong = XMALLOC(int64_t, n); /* strong[j] == i  <=> j in S_i   */
    int64_t* cpos = XMALLOC(int64_t, n);   /* cpos[j] = slot of j in C_i or -1 */
    double* num = XMALLOC(double, n);
    for (int64_t j = 0; j < n; ++j) strong[j] = -1, cpos[j] = -1;
    int64_t cap = orc_csr_nnz(A) + n, nnz = 0;
    orc_csr* P = csr_alloc(n, nc, cap);
    int64_t* clist = XMALLOC(int64_t, n);
    P->rp[0] = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (cf[i] == ST_C) {
            P->col[nnz] = cmap[i];
            P->val[nnz++] = 1.0;
            P->rp[i + 1] = nnz;
            continue;
        }
        for (int64_t t = S->rp[i]; t < S->rp[i + 1]; ++t) strong[S->col[t]] = i;
        int64_t nci = 0;
        double d = 0.0;
        for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) {
            int64_t j = A->col[k];
            if (j == i) { d = A->val[k]; break; }
        }
        for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) {
            int64_t j = A->col[k];
            if (j == i) continue;
            if (strong[j] == i && cf[j] == ST_C) {
                cpos[j] = nci;
                clist[nci++] = j;
                num[j] = A->val[k];
            } else if (strong[j] != i) {
                d += A->val[k];
            }
        }
        if (nci > 0) {
            for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) {
                int64_t kk = A->col[k];
                if (kk == i || strong[kk] != i || cf[kk] == ST_C) continue;
                /* only couplings of sign opposite to a_kk distribute (no cancellation) */
                int pos = diag_of(A, kk) > 0.0;
                double s = 0.0;
                for (int64_t u = A->rp[kk]; u < A->rp[kk + 1]; ++u)
                    if (cpos[A->col[u]] >= 0 && (pos ? A->val[u] < 0.0 : A->val[u] > 0.0))
                        s += A->val[u];
                if (s == 0.0) {
                    d += A->val[k];
                } else {
                    for (int64_t u = A->rp[kk]; u < A->rp[kk + 1]; ++u)
                        if (cpos[A->col[u]] >= 0 && (pos ? A->val[u] < 0.0 : A->val[u] > 0.0))
                            num[A->col[u]] += (A->val[k] * A->val[u]) / s;
                }
            }
        }
        /* clist is in ascending column order (CSR order of row i) == ascending cmap */
        for (int64_t t = 0; t < nci; ++t) {
            int64_t j = clist[t];
            P->col[nnz] = cmap[j];
            P->val[nnz++] = -num[j] / d;
            cpos[j] = -1;
        }
        P->rp[i + 1] = nnz;
    }
    free(cmap);
    free(strong);
    free(cpos);
    free(num);
    free(clist);
    return P;
}

/* Extended+i interpolation (row a8 option, r6; De Sterck, Falgout, Nolting, Yang 2008),
 * distance two.  F row i: the interpolatory set Chat_i = strong C neighbours (S_i order),
 * then the strong C neighbours of each strong F neighbour k (S_i order, S_k order), each once;
 * num_j = 0.0 for j in Chat_i; d = a_ii; in row i's CSR order, a_ij goes to num_j for j in
 * Chat_i, to d for a weak j (j not in S_i); then for each strong F neighbour k in row i's
 * order, with abar_kl = a_kl of sign opposite to a_kk (else 0): s_k = sum of abar_kl over l
 * in Chat_i u {i} (row k order, from 0.0); s_k = 0 adds a_ik to d, else (row k order)
 * num_l += (a_ik abar_kl) / s_k for l in Chat_i and d += (a_ik abar_ki) / s_k for l = i;
 * w_ij = -num_j / d, columns ascending.  P_max truncation (p_max > 0, a row of more entries):
 * tot = sum of the row's w (column order), the p_max largest |w| kept (ties: smaller column),
 * kept = their sum (column order), each kept w *= (tot / kept) unless kept = 0. */
static int ext_abar(double akl, int pos) { return pos ? akl < 0.0 : akl > 0.0; }

orc_csr* orc_interp_ext_i(const orc_csr* A, const orc_csr* S, const int32_t* cf, int64_t p_max) {
    int64_t n = A->n_rows;
    int64_t* cmap = XMALLOC(int64_t, n);
    int64_t nc = 0;
    for (int64_t i = 0; i < n; ++i) cmap[i] = cf[i] == ST_C ? nc++ : -1;
    int64_t* strong = XMALLOC(int64_t, n); /* strong[j] == i <=> j in S_i     */
    int64_t* inC = XMALLOC(int64_t, n);    /* inC[j] == i    <=> j in Chat_i  */
    double* num = XMALLOC(double, n);
    int64_t* list = XMALLOC(int64_t, n);
    double* w = XMALLOC(double, n);
    char* keep = XMALLOC(char, n);
    for (int64_t j = 0; j < n; ++j) strong[j] = -1, inC[j] = -1;
    int64_t cap = 64, nnz = 0;
    int64_t* pc = XMALLOC(int64_t, cap);
    double* pv = XMALLOC(double, cap);
    int64_t* rp = XMALLOC(int64_t, n + 1);
    rp[0] = 0;
    for (int64_t i = 0; i < n; ++i) {
        int64_t m = 0;
        if (cf[i] == ST_C) {
            list[0] = i;
            w[0] = 1.0;
            keep[0] = 1;
            m = 1;
        } else {
            for (int64_t t = S->rp[i]; t < S->rp[i + 1]; ++t) strong[S->col[t]] = i;
            for (int64_t t = S->rp[i]; t < S->rp[i + 1]; ++t) {
                int64_t j = S->col[t];
                if (cf[j] == ST_C && inC[j] != i) inC[j] = i, list[m++] = j, num[j] = 0.0;
            }
            for (int64_t t = S->rp[i]; t < S->rp[i + 1]; ++t) {
                int64_t k = S->col[t];
                if (cf[k] == ST_C) continue;
                for (int64_t u = S->rp[k]; u < S->rp[k + 1]; ++u) {
                    int64_t j = S->col[u];
                    if (cf[j] == ST_C && inC[j] != i) inC[j] = i, list[m++] = j, num[j] = 0.0;
                }
            }
            double d = diag_of(A, i);
            for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) {
                int64_t j = A->col[k];
                if (j == i) continue;
                if (inC[j] == i) num[j] += A->val[k];
                else if (strong[j] != i) d += A->val[k];
            }
            for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) {
                int64_t kk = A->col[k];
                if (kk == i || strong[kk] != i || cf[kk] == ST_C) continue;
                int pos = diag_of(A, kk) > 0.0;
                double sk = 0.0;
                for (int64_t u = A->rp[kk]; u < A->rp[kk + 1]; ++u) {
                    int64_t l = A->col[u];
                    if (ext_abar(A->val[u], pos) && (inC[l] == i || l == i)) sk += A->val[u];
                }
                if (sk == 0.0) {
                    d += A->val[k];
                    continue;
                }
                for (int64_t u = A->rp[kk]; u < A->rp[kk + 1]; ++u) {
                    int64_t l = A->col[u];
                    if (!ext_abar(A->val[u], pos)) continue;
                    if (inC[l] == i) num[l] += (A->val[k] * A->val[u]) / sk;
                    else if (l == i) d += (A->val[k] * A->val[u]) / sk;
                }
            }
            qsort(list, (size_t)m, sizeof(int64_t), cmp_i64);
            for (int64_t t = 0; t < m; ++t) w[t] = -num[list[t]] / d, keep[t] = 1;
            if (p_max > 0 && m > p_max) {
                double tot = 0.0, kept = 0.0;
                for (int64_t t = 0; t < m; ++t) tot += w[t], keep[t] = 0;
                for (int64_t r = 0; r < p_max; ++r) {
                    int64_t best = -1;
                    for (int64_t t = 0; t < m; ++t)
                        if (!keep[t] && (best < 0 || fabs(w[t]) > fabs(w[best]))) best = t;
                    keep[best] = 1;
                }
                for (int64_t t = 0; t < m; ++t)
                    if (keep[t]) kept += w[t];
                if (kept != 0.0) {
                    double f = tot / kept;
                    for (int64_t t = 0; t < m; ++t)
                        if (keep[t]) w[t] = w[t] * f;
                }
            }
        }
        if (nnz + m > cap) {
            while (nnz + m > cap) cap *= 2;
            pc = (int64_t*)realloc(pc, sizeof(int64_t) * (size_t)cap);
            pv = (double*)realloc(pv, sizeof(double) * (size_t)cap);
            if (!pc || !pv) abort();
        }
        for (int64_t t = 0; t < m; ++t)
            if (keep[t]) pc[nnz] = cmap[list[t]], pv[nnz++] = w[t];
        rp[i + 1] = nnz;
    }
    free(cmap);
    free(strong);
    free(inC);
    free(num);
    free(list);
    free(w);
    free(keep);
    orc_csr* P = XMALLOC(orc_csr, 1);
    P->n_rows = n;
    P->n_cols = nc;
    P->rp = rp;
    P->col = pc;
    P->val = pv;
    return P;
}

/* ------------------------------------------------------------------------------ */
/* MIS(2) aggregation (row a9; partition-independent).  Tuples (state, hash32, id)   */
/* with state OUT < UNDECIDED < IN; two synchronous max-propagation hops over the  */
/* closed strength neighbourhood; undecided i becomes IN if the 2-hop max is its own */
/* tuple, OUT if the 2-hop max is IN.  Roots = IN, numbered in ascending index.     */
/* Pass 1: a node next to a root joins it.  Pass 2: any other node joins the pass-1 */
/* neighbour with the largest |s_ij| (ties: smallest aggregate id).                 */
/* ------------------------------------------------------------------------------ */
typedef struct { int32_t st; uint32_t h; int64_t id; } tup;
static int tup_gt(tup a, tup b) {
    if (a.st != b.st) return a.st > b.st;
    if (a.h != b.h) return a.h > b.h;
    return a.id > b.id;
}

int64_t orc_mis2_aggregate(const orc_csr* S, uint64_t seed, int32_t* agg) {
    int64_t n = S->n_rows;
    enum { M_OUT = 0, M_U = 1, M_IN = 2 };
    int32_t* st = XMALLOC(int32_t, n);
    tup* t0 = XMALLOC(tup, n);
    tup* t1 = XMALLOC(tup, n);
    for (int64_t i = 0; i < n; ++i) st[i] = M_U;
    int64_t nu = n;
    while (nu > 0) {
        for (int64_t i = 0; i < n; ++i) {
            t0[i].st = st[i];
            t0[i].h = hash32(i, seed);
            t0[i].id = i;
        }
        for (int hop = 0; hop < 2; ++hop) {
            for (int64_t i = 0; i < n; ++i) {
                tup m = t0[i];
                for (int64_t t = S->rp[i]; t < S->rp[i + 1]; ++t)
                    if (tup_gt(t0[S->col[t]], m)) m = t0[S->col[t]];
                t1[i] = m;
            }
            tup* sw = t0; t0 = t1; t1 = sw;
        }
        nu = 0;
        for (int64_t i = 0; i < n; ++i) {
            if (st[i] != M_U) continue;
            if (t0[i].id == i) st[i] = M_IN;
            else if (t0[i].st == M_IN) st[i] = M_OUT;
            nu += st[i] == M_U;
        }
    }
    int64_t na = 0;
    int32_t* a1 = XMALLOC(int32_t, n);
    for (int64_t i = 0; i < n; ++i) agg[i] = st[i] == M_IN ? (int32_t)na++ : -1;
    for (int64_t i = 0; i < n; ++i) {
        a1[i] = agg[i];
        if (agg[i] >= 0) continue;
        for (int64_t t = S->rp[i]; t < S->rp[i + 1]; ++t)
            if (st[S->col[t]] == M_IN) { a1[i] = agg[S->col[t]]; break; }
    }
    for (int64_t i = 0; i < n; ++i) {
        agg[i] = a1[i];
        if (a1[i] >= 0) continue;
        double best = -1.0;
        int32_t ba = -1;
        for (int64_t t = S->rp[i]; t < S->rp[i + 1]; ++t) {
            int64_t j = S->col[t];
            if (a1[j] < 0) continue;
            double w = fabs(S->val[t]);
            if (w > best || (w == best && a1[j] < ba)) { best = w; ba = a1[j]; }
        }
        agg[i] = ba;
        if (ba < 0) { fprintf(stderr, "amg_oracle: unaggregated node %lld\n", (long long)i); abort(); }
    }
    free(a1);
    free(st);
    free(t0);
    free(t1);
    return na;
}

double orc_sa_theta_next(double theta) { return theta * 0.75; }

/* Coarse-operator drop tolerance (r6 option, non-Galerkin): off-diagonal a_ij of A_c with
 * |a_ij| < tau * sqrt(|a_ii a_jj|) (a_ii, a_jj the stored diagonals) are removed and added to
 * the diagonal, in row order from a_ii; kept entries stay in row order.  Row sums are kept.
 * A row without a stored diagonal is left as it is. */
orc_csr* orc_sparsify(const orc_csr* A, double tau) {
    int64_t n = A->n_rows, nnz = 0;
    double* d = XMALLOC(double, n);
    char* has = XMALLOC(char, n);
    for (int64_t i = 0; i < n; ++i) {
        has[i] = 0;
        d[i] = 0.0;
        for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k)
            if (A->col[k] == i) { d[i] = A->val[k]; has[i] = 1; break; }
    }
    orc_csr* B = csr_alloc(n, A->n_cols, orc_csr_nnz(A));
    B->rp[0] = 0;
    for (int64_t i = 0; i < n; ++i) {
        double f = d[i];
        if (has[i])
            for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) {
                int64_t j = A->col[k];
                if (j != i && fabs(A->val[k]) < tau * sqrt(fabs(d[i] * d[j]))) f += A->val[k];
            }
        for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) {
            int64_t j = A->col[k];
            if (!has[i]) {
                B->col[nnz] = j;
                B->val[nnz++] = A->val[k];
            } else if (j == i) {
                B->col[nnz] = j;
                B->val[nnz++] = f;
            } else if (!(fabs(A->val[k]) < tau * sqrt(fabs(d[i] * d[j])))) {
                B->col[nnz] = j;
                B->val[nnz++] = A->val[k];
            }
        }
        B->rp[i + 1] = nnz;
    }
    free(d);
    free(has);
    return B;
}

/* Filtered operator of SA smoothing (row a9, r6): the diagonal and the strong off-diagonals
 * (sa_strong, the strength test above) in CSR order; the diagonal value becomes
 * f_i = a_ii + the weak off-diagonal a_ij, added in row order.  Row sums are kept. */
orc_csr* orc_sa_filter(const orc_csr* A, double theta) {
    int64_t n = A->n_rows, nnz = 0;
    double* d = XMALLOC(double, n);
    for (int64_t i = 0; i < n; ++i) d[i] = diag_of(A, i);
    orc_csr* F = csr_alloc(n, A->n_cols, orc_csr_nnz(A));
    F->rp[0] = 0;
    for (int64_t i = 0; i < n; ++i) {
        double f = d[i];
        for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) {
            int64_t j = A->col[k];
            if (j != i && !sa_strong(A->val[k], d[i], d[j], theta)) f += A->val[k];
        }
        for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) {
            int64_t j = A->col[k];
            if (j == i) {
                F->col[nnz] = j;
                F->val[nnz++] = f;
            } else if (sa_strong(A->val[k], d[i], d[j], theta)) {
                F->col[nnz] = j;
                F->val[nnz++] = A->val[k];
            }
        }
        F->rp[i + 1] = nnz;
    }
    free(d);
    return F;
}

/* rho(D^-1 A_F), D = diag(A) (row a9, r6): ORC_SA_RHO_ITERS power steps normalised in the max
 * norm, which is exact in any order (so the same on every partition): x = u / max|u| with
 * u = vec_uniform(seed); per step y_i = (A_F x)_i / a_ii (row_dot order), lam = max|y_i|,
 * stop if lam = 0, else x = y / lam.  Returns the last lam. */
double orc_sa_rho(const orc_csr* F, const double* d, uint64_t seed) {
    int64_t n = F->n_rows;
    double* x = XMALLOC(double, n);
    double* y = XMALLOC(double, n);
    orc_vec_uniform(n, 0, seed, x);
    double m = 0.0;
    for (int64_t i = 0; i < n; ++i) m = fabs(x[i]) > m ? fabs(x[i]) : m;
    if (m > 0.0)
        for (int64_t i = 0; i < n; ++i) x[i] = x[i] / m;
    double lam = 0.0;
    for (int it = 0; it < ORC_SA_RHO_ITERS; ++it) {
        lam = 0.0;
        for (int64_t i = 0; i < n; ++i) {
            y[i] = row_dot(F, i, x) / d[i];
            lam = fabs(y[i]) > lam ? fabs(y[i]) : lam;
        }
        if (lam == 0.0) break;
        for (int64_t i = 0; i < n; ++i) x[i] = y[i] / lam;
    }
    free(x);
    free(y);
    return lam;
}

/* Smoothed prolongator (row a9; r6 definition): T_i,agg(i) = 1/sqrt(|agg|); A_F =
 * orc_sa_filter(A, theta); rho = orc_sa_rho(A_F, diag A, seed); omega = (4/3)/rho (0 if
 * rho = 0); P_ij = T_ij - (omega * (1/a_ii)) * (A_F T)_ij over the union pattern (A_F T by
 * orc_spgemm: each entry summed from 0.0 over A_F's row in order). */
orc_csr* orc_sa_prolongator(const orc_csr* A, const int32_t* agg, int64_t n_agg, double theta,
                            uint64_t seed) {
    int64_t n = A->n_rows;
    int64_t* size = XMALLOC(int64_t, n_agg);
    for (int64_t a = 0; a < n_agg; ++a) size[a] = 0;
    for (int64_t i = 0; i < n; ++i) size[agg[i]]++;
    orc_csr* T = csr_alloc(n, n_agg, n);
    T->rp[0] = 0;
    for (int64_t i = 0; i < n; ++i) {
        T->col[i] = agg[i];
        T->val[i] = 1.0 / sqrt((double)size[agg[i]]);
        T->rp[i + 1] = i + 1;
    }
    double* d = XMALLOC(double, n);
    for (int64_t i = 0; i < n; ++i) d[i] = diag_of(A, i);
    orc_csr* F = orc_sa_filter(A, theta);
    double rho = orc_sa_rho(F, d, seed);
    double omega = rho > 0.0 ? (4.0 / 3.0) / rho : 0.0;
    orc_csr* AT = orc_spgemm(F, T);
    orc_csr* P = csr_alloc(n, n_agg, orc_csr_nnz(AT) + n);
    int64_t nnz = 0;
    P->rp[0] = 0;
    for (int64_t i = 0; i < n; ++i) {
        double c = omega * (1.0 / d[i]);
        int64_t ka = AT->rp[i], ea = AT->rp[i + 1], kt = T->rp[i], et = T->rp[i + 1];
        while (ka < ea || kt < et) {
            int64_t ja = ka < ea ? AT->col[ka] : INT64_MAX, jt = kt < et ? T->col[kt] : INT64_MAX;
            int64_t j = ja < jt ? ja : jt;
            double tv = 0.0, av = 0.0;
            if (jt == j) tv = T->val[kt++];
            if (ja == j) av = AT->val[ka++];
            P->col[nnz] = j;
            P->val[nnz++] = tv - c * av;
        }
        P->rp[i + 1] = nnz;
    }
    orc_csr_free(AT);
    orc_csr_free(F);
    orc_csr_free(T);
    free(d);
    free(size);
    return P;
}

/* Gauss-Jordan inverse with partial pivoting (first max), row-major. */
void orc_dense_inverse(int64_t n, const orc_csr* A, double* inv) {
    double* M = XMALLOC(double, n * n);
    memset(M, 0, sizeof(double) * (size_t)(n * n));
    memset(inv, 0, sizeof(double) * (size_t)(n * n));
    for (int64_t i = 0; i < n; ++i) {
        for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) M[i * n + A->col[k]] = A->val[k];
        inv[i * n + i] = 1.0;
    }
    for (int64_t c = 0; c < n; ++c) {
        int64_t p = c;
        for (int64_t r = c + 1; r < n; ++r)
            if (fabs(M[r * n + c]) > fabs(M[p * n + c])) p = r;
        if (p != c)
            for (int64_t j = 0; j < n; ++j) {
                double t = M[c * n + j]; M[c * n + j] = M[p * n + j]; M[p * n + j] = t;
                t = inv[c * n + j]; inv[c * n + j] = inv[p * n + j]; inv[p * n + j] = t;
            }
        double ip = 1.0 / M[c * n + c];
        for (int64_t j = 0; j < n; ++j) {
            M[c * n + j] *= ip;
            inv[c * n + j] *= ip;
        }
#pragma omp parallel for schedule(static)
        for (int64_t r = 0; r < n; ++r) {
            if (r == c) continue;
            double f = M[r * n + c];
            if (f == 0.0) continue;
            for (int64_t j = 0; j < n; ++j) {
                M[r * n + j] -= f * M[c * n + j];
                inv[r * n + j] -= f * inv[c * n + j];
            }
        }
    }
    free(M);
}

/* ------------------------------------------------------------------------------ */
/* Hierarchy + V-cycle (row a7).                                                     */
/* ------------------------------------------------------------------------------ */
#define ORC_MAX_LEVELS 40
struct orc_hier {
    orc_options opt;
    int32_t nlev;
    orc_csr* A[ORC_MAX_LEVELS];
    orc_csr* P[ORC_MAX_LEVELS];
    orc_csr* R[ORC_MAX_LEVELS];
    int32_t* split[ORC_MAX_LEVELS];
    double* x[ORC_MAX_LEVELS];
    double* b[ORC_MAX_LEVELS];
    double* r[ORC_MAX_LEVELS];
    double* t[ORC_MAX_LEVELS];
    double* inv; /* coarsest level dense inverse, row-major */
    int32_t ncuts[ORC_MAX_LEVELS]; /* 0: one segment (serial) */
    int64_t* cuts[ORC_MAX_LEVELS];
};

void orc_hier_set_cuts(orc_hier* H, int32_t level, int32_t ncuts, const int64_t* cuts) {
    if (level < 0 || level >= H->nlev) return;
    free(H->cuts[level]);
    H->cuts[level] = (int64_t*)malloc(sizeof(int64_t) * (size_t)(ncuts > 0 ? ncuts : 1));
    memcpy(H->cuts[level], cuts, sizeof(int64_t) * (size_t)ncuts);
    H->ncuts[level] = ncuts;
}

orc_hier* orc_hier_setup(const orc_csr* A0, const orc_options* opt) {
    orc_hier* H = (orc_hier*)calloc(1, sizeof(orc_hier));
    H->opt = *opt;
    H->A[0] = orc_csr_new(A0->n_rows, A0->n_cols, A0->rp, A0->col, A0->val);
    int32_t l = 0;
    int32_t maxl = opt->max_levels < ORC_MAX_LEVELS ? opt->max_levels : ORC_MAX_LEVELS;
    double theta = opt->strong_threshold;
    for (; l + 1 < maxl && H->A[l]->n_rows > opt->max_coarse; theta = orc_sa_theta_next(theta)) {
        orc_csr* A = H->A[l];
        int64_t n = A->n_rows;
        int32_t* split = XMALLOC(int32_t, n);
        orc_csr* P;
        if (opt->coarsen == ORC_COARSEN_SA) {
            /* theta_l = theta_{l-1} * 3/4 (r6; rounded per level) */
            orc_csr* S = orc_strength_symmetric(A, theta);
            int64_t na = orc_mis2_aggregate(S, opt->seed + (uint64_t)l, split);
            P = orc_sa_prolongator(A, split, na, theta, opt->seed + (uint64_t)l);
            orc_csr_free(S);
        } else {
            orc_csr* S = orc_strength_classical(A, opt->strong_threshold);
            if (opt->coarsen == ORC_COARSEN_RS) orc_rs_split(S, split);
            else orc_pmis_split(S, opt->seed + (uint64_t)l, split);
            P = opt->interp == ORC_INTERP_EXT_I ? orc_interp_ext_i(A, S, split, opt->p_max)
                                                : orc_interp_classical(A, S, split);
            orc_csr_free(S);
        }
        /* coarsening stalled: no coarse points, no reduction, or < 20% reduction on a level
         * small enough (<= 8192 rows) to become the dense-solved coarsest */
        if (P->n_cols == 0 || P->n_cols >= n || (n <= 8192 && 5 * P->n_cols > 4 * n)) {
            orc_csr_free(P);
            free(split);
            break;
        }
        orc_csr* R = orc_transpose(P);
        orc_csr* AP = orc_spgemm(A, P);
        H->A[l + 1] = orc_spgemm(R, AP);
        orc_csr_free(AP);
        if (opt->drop_tol > 0.0) {
            orc_csr* B = orc_sparsify(H->A[l + 1], opt->drop_tol);
            orc_csr_free(H->A[l + 1]);
            H->A[l + 1] = B;
        }
        H->P[l] = P;
        H->R[l] = R;
        H->split[l] = split;
        ++l;
    }
    H->nlev = l + 1;
    for (int32_t k = 0; k < H->nlev; ++k) {
        int64_t n = H->A[k]->n_rows;
        H->x[k] = XMALLOC(double, n);
        H->b[k] = XMALLOC(double, n);
        H->r[k] = XMALLOC(double, n);
        H->t[k] = XMALLOC(double, n);
    }
    int64_t nc = H->A[H->nlev - 1]->n_rows;
    H->inv = XMALLOC(double, nc * nc);
    orc_dense_inverse(nc, H->A[H->nlev - 1], H->inv);
    return H;
}

static orc_csr* csr_copy(const orc_csr* M) {
    return orc_csr_new(M->n_rows, M->n_cols, M->rp, M->col, M->val);
}

orc_hier* orc_hier_from_levels(int32_t nlev, const orc_csr* const* A, const orc_csr* const* P,
                               const orc_csr* const* R, const orc_options* opt) {
    if (nlev < 1 || nlev > ORC_MAX_LEVELS) return NULL;
    orc_hier* H = (orc_hier*)calloc(1, sizeof(orc_hier));
    H->opt = *opt;
    H->nlev = nlev;
    for (int32_t k = 0; k < nlev; ++k) {
        int64_t n = A[k]->n_rows;
        H->A[k] = csr_copy(A[k]);
        if (k + 1 < nlev) {
            H->P[k] = csr_copy(P[k]);
            H->R[k] = csr_copy(R[k]);
        }
        H->x[k] = XMALLOC(double, n);
        H->b[k] = XMALLOC(double, n);
        H->r[k] = XMALLOC(double, n);
        H->t[k] = XMALLOC(double, n);
    }
    int64_t nc = H->A[nlev - 1]->n_rows;
    H->inv = XMALLOC(double, nc * nc);
    orc_dense_inverse(nc, H->A[nlev - 1], H->inv);
    return H;
}

void orc_hier_free(orc_hier* H) {
    if (!H) return;
    for (int32_t k = 0; k < H->nlev; ++k) {
        orc_csr_free(H->A[k]);
        orc_csr_free(H->P[k]);
        orc_csr_free(H->R[k]);
        free(H->split[k]);
        free(H->x[k]);
        free(H->b[k]);
        free(H->r[k]);
        free(H->t[k]);
        free(H->cuts[k]);
    }
    free(H->inv);
    free(H);
}

int32_t orc_hier_levels(const orc_hier* H) { return H->nlev; }

const orc_csr* orc_hier_matrix(const orc_hier* H, int32_t level, int32_t which) {
    if (level < 0 || level >= H->nlev) return NULL;
    return which == 0 ? H->A[level] : which == 1 ? H->P[level] : H->R[level];
}

void orc_hier_split(const orc_hier* H, int32_t level, int32_t* out) {
    memcpy(out, H->split[level], sizeof(int32_t) * (size_t)H->A[level]->n_rows);
}

/* post = 1: post-smoothing.  Hybrid GS sweeps forward before the coarse correction and
 * backward after it, so the V-cycle is a symmetric operator (usable inside CG). */
static void smooth(orc_hier* H, int32_t l, double* x, const double* b, double* tmp, int post) {
    const orc_csr* A = H->A[l];
    const int64_t zero = 0;
    if (H->opt.smoother == ORC_SMOOTH_HYBRID_GS)
        orc_hybrid_gs_cut(A, x, b, tmp, H->opt.gs_block, post, H->ncuts[l] > 0 ? H->ncuts[l] : 1,
                          H->ncuts[l] > 0 ? H->cuts[l] : &zero);
    else orc_jacobi(A, x, b, tmp, H->opt.jacobi_omega);
    memcpy(x, tmp, sizeof(double) * (size_t)A->n_rows);
}

/* Coarsest level: x_i = sum_j inv_ij b_j as 64 interleaved partial sums --
 * p_l = sum over j = l, l + 64, l + 128, ... in ascending order, each from 0.0 -- combined by
 * the butterfly p_l <- p_l + p_{l xor m} for m = 32, 16, ..., 1 (every l at once); x_i = p_0.
 * The GPU runs one wavefront per row, lane l = p_l, the butterfly as shuffles. */
static double coarse_row(const double* inv_row, const double* b, int64_t n) {
    double p[64], q[64];
    for (int l = 0; l < 64; ++l) {
        double s = 0.0;
        for (int64_t j = l; j < n; j += 64) s += inv_row[j] * b[j];
        p[l] = s;
    }
    for (int m = 32; m >= 1; m >>= 1) {
        for (int l = 0; l < 64; ++l) q[l] = p[l] + p[l ^ m];
        memcpy(p, q, sizeof(p));
    }
    return p[0];
}

/* cycle(l): nu1 smooths; r = b - A x; b_{l+1} = R r; x_{l+1} = 0; cycle(l+1);
 * x = x + P x_{l+1}; nu2 smooths.  Coarsest: x = inv b (coarse_row). */
static void cycle_rec(orc_hier* H, int32_t l, double* x, const double* b) {
    const orc_csr* A = H->A[l];
    int64_t n = A->n_rows;
    if (l == H->nlev - 1) {
        for (int64_t i = 0; i < n; ++i) x[i] = coarse_row(H->inv + i * n, b, n);
        return;
    }
    for (int32_t s = 0; s < H->opt.pre_sweeps; ++s) smooth(H, l, x, b, H->t[l], 0);
    orc_residual(A, x, b, H->r[l]);
    orc_spmv(H->R[l], H->r[l], H->b[l + 1]);
    int64_t nc = H->A[l + 1]->n_rows;
    memset(H->x[l + 1], 0, sizeof(double) * (size_t)nc);
    cycle_rec(H, l + 1, H->x[l + 1], H->b[l + 1]);
    orc_spmv_add(H->P[l], H->x[l + 1], x);
    for (int32_t s = 0; s < H->opt.post_sweeps; ++s) smooth(H, l, x, b, H->t[l], 1);
}

void orc_hier_cycle(orc_hier* H, double* x, const double* b) { cycle_rec(H, 0, x, b); }

int32_t orc_hier_solve(orc_hier* H, double* x, const double* b, int32_t max_iter, double tol,
                       double* hist) {
    const orc_csr* A = H->A[0];
    int64_t n = A->n_rows;
    orc_residual(A, x, b, H->r[0]);
    double r0 = orc_norm2(n, H->r[0]);
    hist[0] = r0;
    int32_t it = 0;
    while (it < max_iter) {
        orc_hier_cycle(H, x, b);
        orc_residual(A, x, b, H->r[0]);
        double rn = orc_norm2(n, H->r[0]);
        hist[++it] = rn;
        if (r0 > 0.0 && rn / r0 < tol) break;
    }
    return it;
}

static double dotp(int64_t n, const double* a, const double* b) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) s += a[i] * b[i];
    return s;
}

/* PCG (row f3): r = b - Ax; z = M r; p = z; loop { q = Ap; alpha = (r,z)/(p,q);
 * x += alpha p; r -= alpha q; record ||r||; z = M r; beta = (r,z_new)/(r,z); p = z + beta p } */
int32_t orc_hier_pcg(orc_hier* H, double* x, const double* b, int32_t max_iter, double tol,
                     double* hist) {
    const orc_csr* A = H->A[0];
    int64_t n = A->n_rows;
    double* r = XMALLOC(double, n);
    double* z = XMALLOC(double, n);
    double* p = XMALLOC(double, n);
    double* q = XMALLOC(double, n);
    orc_residual(A, x, b, r);
    double r0 = sqrt(dotp(n, r, r));
    hist[0] = r0;
    memset(z, 0, sizeof(double) * (size_t)n);
    orc_hier_cycle(H, z, r);
    memcpy(p, z, sizeof(double) * (size_t)n);
    double rz = dotp(n, r, z);
    int32_t it = 0;
    while (it < max_iter) {
        orc_spmv(A, p, q);
        double alpha = rz / dotp(n, p, q);
        for (int64_t i = 0; i < n; ++i) {
            x[i] = x[i] + alpha * p[i];
            r[i] = r[i] - alpha * q[i];
        }
        double rn = sqrt(dotp(n, r, r));
        hist[++it] = rn;
        if (tol > 0.0 && r0 > 0.0 && rn / r0 < tol) break;
        if (it == max_iter) break;
        memset(z, 0, sizeof(double) * (size_t)n);
        orc_hier_cycle(H, z, r);
        double rzn = dotp(n, r, z);
        double beta = rzn / rz;
        for (int64_t i = 0; i < n; ++i) p[i] = z[i] + beta * p[i];
        rz = rzn;
    }
    free(r);
    free(z);
    free(p);
    free(q);
    return it;
}

#ifdef _OPENMP
#include <omp.h>
#endif
int32_t orc_num_threads(void) {
#ifdef _OPENMP
    return (int32_t)omp_get_max_threads();
#else
    return 1;
#endif
}

void orc_set_num_threads(int32_t n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads((int)n);
#else
    (void)n;
#endif
}
