// setup_device.hip -- AMG setup on the GPU: strength of connection,
// PMIS splitting, classical interpolation, MIS(2) aggregation, the smoothed-aggregation
// prolongator and the transpose R = P^T, for one rank.  Every integer decision and every
// floating-point sum follows host_setup.cpp / oracle/amg_oracle.c exactly, so
// the hierarchy is bit-identical to the host path's; the Galerkin products stay on the
// device SpGEMM (spgemm.hip).  Several ranks keep the host path (host_setup.cpp), whose
// rounds exchange halo states between ranks.
//
// Layout: one upload of A per level -- int32 row_ptr, int32 columns (single rank: global =
// local ids), fp64 values; the strength graph S stays on the device; per-row kernels are one
// thread per row (rows are short and independent); rounds (PMIS, MIS(2)) are synchronous:
// each round reads the previous round's states only.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <climits>
#include <cmath>

#include "device.hpp"

namespace amg {

namespace {

enum { ST_U = -1, ST_F = 0, ST_C = 1 };
enum { M_OUT = 0, M_U = 1, M_IN = 2 };
constexpr int kT = 256;

inline unsigned grid1(long long n) { return (unsigned)std::max<long long>(1, (n + kT - 1) / kT); }

__device__ __forceinline__ unsigned long long dmix(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// host_comm.cpp hash32()
__device__ __forceinline__ unsigned dhash32(long long gid, unsigned long long seed) {
    return (unsigned)(dmix((unsigned long long)gid ^ (seed * 0x9E3779B97F4A7C15ull)) >> 32);
}

// binary search of c in the ascending cols[lo, hi)
__device__ __forceinline__ int dfind(const int* cols, int lo, int hi, int c) {
    while (lo < hi) {
        const int m = (lo + hi) >> 1;
        const int v = cols[m];
        if (v == c) return m;
        if (v < c) lo = m + 1;
        else hi = m;
    }
    return -1;
}

struct DCsr {
    const int* rp;
    const int* col;
    const double* val;
    int n;
};

// ---- strength ------------------------------------------------------------------------
// classical: m_i = max_{j != i} (-a_ij) (first entry sets it); none if m_i <= 0;
// strong iff -a_ij >= theta m_i.  Pass 0 counts, pass 1 fills (row order kept).
template <bool FILL>
__global__ void strength_classical_kernel(DCsr A, double theta, int* cnt, const int* srp, int* scol,
                                          double* sval) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= A.n) return;
    double mx = 0.0;
    bool any = false;
    for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) {
        if (A.col[k] == i) continue;
        const double v = -A.val[k];
        if (!any || v > mx) mx = v;
        any = true;
    }
    const bool has = any && mx > 0.0;
    const double thr = theta * mx;
    int q = FILL ? srp[i] : 0, c = 0;
    for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) {
        if (!(has && A.col[k] != i && -A.val[k] >= thr)) continue;
        if (FILL) {
            scol[q] = A.col[k];
            sval[q++] = A.val[k];
        }
        ++c;
    }
    if (!FILL) cnt[i] = c;
}

// a_ii: the first diagonal entry of the row (0 if none), like diagonal()
__global__ void diagonal_kernel(DCsr A, double* d) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= A.n) return;
    double v = 0.0;
    for (int k = A.rp[i]; k < A.rp[i + 1]; ++k)
        if (A.col[k] == i) {
            v = A.val[k];
            break;
        }
    d[i] = v;
}

// symmetric: |a_ij| >= theta sqrt(|a_ii a_jj|), j != i
template <bool FILL>
__global__ void strength_symmetric_kernel(DCsr A, const double* d, double theta, int* cnt, const int* srp,
                                          int* scol, double* sval) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= A.n) return;
    int q = FILL ? srp[i] : 0, c = 0;
    for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) {
        const int j = A.col[k];
        if (j == i) continue;
        if (!(fabs(A.val[k]) >= theta * sqrt(fabs(d[i] * d[j])))) continue;
        if (FILL) {
            scol[q] = j;
            sval[q++] = A.val[k];
        }
        ++c;
    }
    if (!FILL) cnt[i] = c;
}

// ---- PMIS ------------------------------------------------------------------------------
__global__ void col_count_kernel(DCsr S, int* tcnt) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= S.n) return;
    for (int k = S.rp[i]; k < S.rp[i + 1]; ++k) atomicAdd(&tcnt[S.col[k]], 1);
}

// S^T adjacency (row j of S^T = the rows i with j in S_i; order within a row arbitrary --
// PMIS only takes maxima over the set)
__global__ void transpose_fill_kernel(DCsr S, int* cursor, int* tcol) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= S.n) return;
    for (int k = S.rp[i]; k < S.rp[i + 1]; ++k) tcol[atomicAdd(&cursor[S.col[k]], 1)] = i;
}

__global__ void pmis_init_kernel(int n, const int* tcnt, unsigned long long seed,
                                 unsigned long long* key, int* cf) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    key[i] = ((unsigned long long)tcnt[i] << 32) | (unsigned long long)dhash32(i, seed);
    cf[i] = tcnt[i] == 0 ? ST_F : ST_U;
}

// undecided i -> C iff its (key, id) beats every undecided j in S_i u S^T_i
__global__ void pmis_select_kernel(DCsr S, const int* trp, const int* tcol,
                                   const unsigned long long* key, const int* cf, unsigned char* newc) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= S.n) return;
    newc[i] = 0;
    if (cf[i] != ST_U) return;
    const unsigned long long ki = key[i];
    bool best = true;
    for (int k = S.rp[i]; k < S.rp[i + 1] && best; ++k) {
        const int j = S.col[k];
        if (cf[j] != ST_U) continue;
        const unsigned long long kj = key[j];
        if (kj > ki || (kj == ki && j > i)) best = false;
    }
    for (int t = trp[i]; t < trp[i + 1] && best; ++t) {
        const int j = tcol[t];
        if (cf[j] != ST_U) continue;
        const unsigned long long kj = key[j];
        if (kj > ki || (kj == ki && j > i)) best = false;
    }
    newc[i] = best;
}

__global__ void pmis_apply_kernel(int n, const unsigned char* newc, int* cf) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i < n && newc[i]) cf[i] = ST_C;
}

// undecided i with a C point in S_i -> F; count the undecided that remain
__global__ void pmis_fpass_kernel(DCsr S, int* cf, unsigned long long* nu) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= S.n || cf[i] != ST_U) return;
    for (int k = S.rp[i]; k < S.rp[i + 1]; ++k)
        if (cf[S.col[k]] == ST_C) {
            cf[i] = ST_F;
            return;
        }
    atomicAdd(nu, 1ull);
}

// ---- classical interpolation ------------------------------------------------------------
// is j a strong neighbour of i (S rows ascending)
__device__ __forceinline__ bool strong(const DCsr& S, int i, int j) {
    return dfind(S.col, S.rp[i], S.rp[i + 1], j) >= 0;
}

// F row i: d = a_ii + weak couplings + couplings to strong F neighbours whose s_k is 0;
// w_ij = -num_j / d for j in C_i (strong C neighbours), num_j = a_ij + sum over strong F
// neighbours k (A-row order) of (a_ik a_kj) / s_k, s_k = sum of row k's couplings to C_i of
// sign opposite to a_kk.  Same loops and order as host_setup.cpp interp_classical().
template <bool FILL>
__global__ void interp_kernel(DCsr A, DCsr S, const int* cf, const int* cmap, int* cnt, const int* prp,
                              int* pcol, double* pval) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= A.n) return;
    if (cf[i] == ST_C) {
        if (FILL) {
            pcol[prp[i]] = cmap[i];
            pval[prp[i]] = 1.0;
        } else {
            cnt[i] = 1;
        }
        return;
    }
    auto in_ci = [&](int m) { return m != i && cf[m] == ST_C && strong(S, i, m); };
    double d = 0.0;
    for (int k = A.rp[i]; k < A.rp[i + 1]; ++k)
        if (A.col[k] == i) {
            d = A.val[k];
            break;
        }
    int nci = 0;
    for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) {
        const int j = A.col[k];
        if (j == i) continue;
        const bool st = strong(S, i, j);
        if (st && cf[j] == ST_C) ++nci;
        else if (!st) d += A.val[k];
    }
    if (!FILL) {
        cnt[i] = nci;
        return;
    }
    if (nci == 0) return;
    // s_k == 0 neighbours add a_ik to d, in A-row order (second pass of the host loop)
    for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) {
        const int kk = A.col[k];
        if (kk == i || cf[kk] == ST_C || !strong(S, i, kk)) continue;
        double akk = 0.0;
        for (int u = A.rp[kk]; u < A.rp[kk + 1]; ++u)
            if (A.col[u] == kk) {
                akk = A.val[u];
                break;
            }
        const bool pos = akk > 0.0;
        double s = 0.0;
        for (int u = A.rp[kk]; u < A.rp[kk + 1]; ++u) {
            const double v = A.val[u];
            if ((pos ? v < 0.0 : v > 0.0) && in_ci(A.col[u])) s += v;
        }
        if (s == 0.0) d += A.val[k];
    }
    // num_j accumulates in this row's own P slots (pval), k outer: s_k is formed once per
    // strong F neighbour instead of once per (j, k) pair, and every num_j still receives its
    // terms in A-row order of k -- the host loop's order, so the weights are bit-identical
    const int q0 = prp[i];
    int q = q0;
    for (int kj = A.rp[i]; kj < A.rp[i + 1]; ++kj) {
        const int j = A.col[kj];
        if (j == i || cf[j] != ST_C || !strong(S, i, j)) continue;
        pcol[q] = cmap[j];
        pval[q++] = A.val[kj];
    }
    for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) {
        const int kk = A.col[k];
        if (kk == i || cf[kk] == ST_C || !strong(S, i, kk)) continue;
        double akk = 0.0;
        for (int u = A.rp[kk]; u < A.rp[kk + 1]; ++u)
            if (A.col[u] == kk) {
                akk = A.val[u];
                break;
            }
        const bool pos = akk > 0.0;
        double s = 0.0;
        for (int u = A.rp[kk]; u < A.rp[kk + 1]; ++u) {
            const double v = A.val[u];
            if ((pos ? v < 0.0 : v > 0.0) && in_ci(A.col[u])) s += v;
        }
        if (s == 0.0) continue;
        q = q0;
        for (int kj = A.rp[i]; kj < A.rp[i + 1]; ++kj) {
            const int j = A.col[kj];
            if (j == i || cf[j] != ST_C || !strong(S, i, j)) continue;
            const int uj = dfind(A.col, A.rp[kk], A.rp[kk + 1], j);
            if (uj >= 0 && (pos ? A.val[uj] < 0.0 : A.val[uj] > 0.0)) pval[q] += (A.val[k] * A.val[uj]) / s;
            ++q;
        }
    }
    for (q = q0; q < q0 + nci; ++q) pval[q] = -pval[q] / d;
}

// ---- MIS(2) aggregation -----------------------------------------------------------------
__global__ void mis2_tuple_kernel(int n, const int* st, const unsigned* hs, unsigned long long* h,
                                  unsigned long long* l) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    h[i] = ((unsigned long long)(unsigned)st[i] << 32) | hs[i];
    l[i] = (unsigned long long)i;
}

__global__ void mis2_hop_kernel(DCsr S, const unsigned long long* h0, const unsigned long long* l0,
                                unsigned long long* h1, unsigned long long* l1) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= S.n) return;
    unsigned long long mh = h0[i], ml = l0[i];
    for (int k = S.rp[i]; k < S.rp[i + 1]; ++k) {
        const int j = S.col[k];
        const unsigned long long xh = h0[j], xl = l0[j];
        if (xh > mh || (xh == mh && xl > ml)) mh = xh, ml = xl;
    }
    h1[i] = mh;
    l1[i] = ml;
}

__global__ void mis2_update_kernel(int n, const unsigned long long* h, const unsigned long long* l,
                                   int* st, unsigned long long* nu) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= n || st[i] != M_U) return;
    if (l[i] == (unsigned long long)i) st[i] = M_IN;
    else if ((h[i] >> 32) == M_IN) st[i] = M_OUT;
    if (st[i] == M_U) atomicAdd(nu, 1ull);
}

__global__ void flag_eq_kernel(int n, const int* st, int value, int* flag) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i < n) flag[i] = st[i] == value;
}

// pass 1: a root keeps its id; others join the first root neighbour in S-row order
__global__ void mis2_pass1_kernel(DCsr S, const int* st, const int* rootid, int* a1) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= S.n) return;
    if (st[i] == M_IN) {
        a1[i] = rootid[i];
        return;
    }
    int a = -1;
    for (int k = S.rp[i]; k < S.rp[i + 1]; ++k) {
        const int j = S.col[k];
        if (st[j] == M_IN) {
            a = rootid[j];
            break;
        }
    }
    a1[i] = a;
}

// pass 2: the rest join the pass-1 neighbour with max |s_ij| (ties: smaller aggregate id)
__global__ void mis2_pass2_kernel(DCsr S, const int* a1, int* agg, unsigned long long* orphans) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= S.n) return;
    if (a1[i] >= 0) {
        agg[i] = a1[i];
        return;
    }
    double best = -1.0;
    int ba = -1;
    for (int k = S.rp[i]; k < S.rp[i + 1]; ++k) {
        const int aj = a1[S.col[k]];
        if (aj < 0) continue;
        const double w = fabs(S.val[k]);
        if (w > best || (w == best && aj < ba)) best = w, ba = aj;
    }
    agg[i] = ba;
    if (ba < 0) atomicAdd(orphans, 1ull);
}

__global__ void agg_size_kernel(int n, const int* agg, int* size) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i < n) atomicAdd(&size[agg[i]], 1);
}

// rho_i = sum_k |a_ik| / |a_ii| (row order), and T_i = 1 / sqrt(|agg(i)|)
__global__ void sa_rows_kernel(DCsr A, const double* d, const int* agg, const int* size, double* rho,
                               double* tval) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= A.n) return;
    double s = 0.0;
    for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) s += fabs(A.val[k]);
    rho[i] = s / fabs(d[i]);
    tval[i] = 1.0 / sqrt((double)size[agg[i]]);
}

// ---- transpose: R = P^T, rows of R sorted by fine index (stable radix sort on columns) ---
__global__ void iota_kernel(int n, int* v) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i < n) v[i] = i;
}

__global__ void expand_rows_kernel(const int* rp, int n, int* rowof) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    for (int k = rp[i]; k < rp[i + 1]; ++k) rowof[k] = i;
}

__global__ void gather_transpose_kernel(int nnz, const int* perm, const int* rowof, const double* val,
                                        long long* rcol, double* rval) {
    const int t = blockIdx.x * kT + threadIdx.x;
    if (t >= nnz) return;
    const int k = perm[t];
    rcol[t] = rowof[k];
    rval[t] = val[k];
}

__global__ void count_cols_kernel(int nnz, const int* col, int* cnt) {
    const int t = blockIdx.x * kT + threadIdx.x;
    if (t < nnz) atomicAdd(&cnt[col[t]], 1);
}

// ---- helpers ---------------------------------------------------------------------------
// exclusive scan of n ints into out[0..n] (out[n] = total)
int64_t exclusive_scan(hipStream_t s, const int* in, int* out, int n, DevBuf<char>& tmp) {
    size_t bytes = 0;
    HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, n + 1, s));
    if (tmp.n < bytes) tmp.alloc(bytes);
    HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp.p, bytes, in, out, n + 1, s));
    int total = 0;
    HIP_CHECK(hipMemcpyAsync(&total, out + n, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    return total;
}

// the level operator on the device (single rank: global column ids are local)
struct DevLevel {
    DevBuf<int> rp, col;
    DevBuf<double> val;
    int n = 0;
    DCsr view() const { return DCsr{rp.p, col.p, val.p, n}; }
};

void upload_level(const HostCSR& A, DevLevel& D) {
    const int64_t n = A.nrows(), nnz = A.nnz();
    AMG_CHECK(n < INT_MAX && nnz < INT_MAX, "device setup: level exceeds int32 indexing");
    std::vector<int> rp(n + 1), col((size_t)std::max<int64_t>(nnz, 1));
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i <= n; ++i) rp[i] = (int)A.rp[i];
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < nnz; ++k) col[k] = (int)A.col[k];
    D.n = (int)n;
    D.rp.upload(rp.data(), rp.size());
    D.col.upload(col.data(), col.size());
    if (nnz) D.val.upload(A.val.data(), (size_t)nnz);
    else D.val.alloc(1);
}

struct DevS {  // strength graph
    DevBuf<int> rp, col;
    DevBuf<double> val;
    int n = 0;
    DCsr view() const { return DCsr{rp.p, col.p, val.p, n}; }
};

template <class CountK, class FillK>
void build_strength(hipStream_t s, int n, DevS& S, DevBuf<char>& tmp, CountK count, FillK fill) {
    DevBuf<int> cnt;
    cnt.alloc((size_t)n + 1);
    HIP_CHECK(hipMemsetAsync(cnt.p, 0, sizeof(int) * cnt.n, s));
    count(cnt.p);
    S.rp.alloc((size_t)n + 1);
    const int64_t nnz = exclusive_scan(s, cnt.p, S.rp.p, n, tmp);
    S.col.alloc((size_t)std::max<int64_t>(nnz, 1));
    S.val.alloc((size_t)std::max<int64_t>(nnz, 1));
    S.n = n;
    fill(S.rp.p, S.col.p, S.val.p);
    HIP_CHECK(hipGetLastError());
}

std::vector<int32_t> download_ints(hipStream_t s, const int* p, int64_t n) {
    std::vector<int32_t> h((size_t)n);
    if (n) HIP_CHECK(hipMemcpyAsync(h.data(), p, sizeof(int) * n, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    return h;
}

}  // namespace

// One level of the setup on the device (single rank): P and the integer split (C/F marker
// for RS-family coarsening, aggregate id for SA).  Returns false when the device path does
// not apply (several ranks, RS coarsening -- the serial Ruge-Stueben pass stays on the host).
bool level_setup_device(Context& ctx, const HostComm& comm, const HostCSR& A, const amg_options& opt,
                        int level, HostCSR& P, std::vector<int32_t>& split) {
    if (comm.nranks != 1 || opt.coarsen == AMG_COARSEN_RS) return false;
    hipStream_t s = ctx.stream;
    const int n = (int)A.nrows();
    if (n == 0) return false;
    PhaseTimer tm(comm);
    DevLevel D;
    upload_level(A, D);
    DevBuf<char> tmp;
    DevS S;
    const DCsr Av = D.view();
    if (opt.coarsen == AMG_COARSEN_PMIS) {
        const double theta = opt.strong_threshold;
        build_strength(
            s, n, S, tmp,
            [&](int* cnt) {
                hipLaunchKernelGGL(strength_classical_kernel<false>, dim3(grid1(n)), dim3(kT), 0, s, Av, theta, cnt,
                                   nullptr, nullptr, nullptr);
            },
            [&](const int* srp, int* scol, double* sval) {
                hipLaunchKernelGGL(strength_classical_kernel<true>, dim3(grid1(n)), dim3(kT), 0, s, Av, theta,
                                   nullptr, srp, scol, sval);
            });
        tm.lap("  device strength");
        const DCsr Sv = S.view();
        // |S^T_i| and the S^T adjacency
        DevBuf<int> tcnt, trp, tcol, cursor;
        tcnt.alloc((size_t)n + 1);
        HIP_CHECK(hipMemsetAsync(tcnt.p, 0, sizeof(int) * tcnt.n, s));
        hipLaunchKernelGGL(col_count_kernel, dim3(grid1(n)), dim3(kT), 0, s, Sv, tcnt.p);
        trp.alloc((size_t)n + 1);
        const int64_t snnz = exclusive_scan(s, tcnt.p, trp.p, n, tmp);
        tcol.alloc((size_t)std::max<int64_t>(snnz, 1));
        cursor.alloc((size_t)n + 1);
        HIP_CHECK(hipMemcpyAsync(cursor.p, trp.p, sizeof(int) * (n + 1), hipMemcpyDeviceToDevice, s));
        hipLaunchKernelGGL(transpose_fill_kernel, dim3(grid1(n)), dim3(kT), 0, s, Sv, cursor.p, tcol.p);
        DevBuf<unsigned long long> key, nu;
        DevBuf<int> cf;
        DevBuf<unsigned char> newc;
        key.alloc(n);
        cf.alloc(n);
        newc.alloc(n);
        nu.alloc(1);
        hipLaunchKernelGGL(pmis_init_kernel, dim3(grid1(n)), dim3(kT), 0, s, n, tcnt.p,
                           (unsigned long long)(opt.seed + (uint64_t)level), key.p, cf.p);
        HIP_CHECK(hipGetLastError());
        for (int round = 0;; ++round) {
            AMG_CHECK(round <= n, "PMIS did not terminate");
            hipLaunchKernelGGL(pmis_select_kernel, dim3(grid1(n)), dim3(kT), 0, s, Sv, trp.p, tcol.p, key.p, cf.p,
                               newc.p);
            hipLaunchKernelGGL(pmis_apply_kernel, dim3(grid1(n)), dim3(kT), 0, s, n, newc.p, cf.p);
            HIP_CHECK(hipMemsetAsync(nu.p, 0, sizeof(unsigned long long), s));
            hipLaunchKernelGGL(pmis_fpass_kernel, dim3(grid1(n)), dim3(kT), 0, s, Sv, cf.p, nu.p);
            HIP_CHECK(hipGetLastError());
            unsigned long long left = 0;
            HIP_CHECK(hipMemcpyAsync(&left, nu.p, sizeof(left), hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
            if (left == 0) break;
        }
        tm.lap("  device PMIS");
        // coarse numbering: C points in row order
        DevBuf<int> cflag, cmap;
        cflag.alloc((size_t)n + 1);
        cmap.alloc((size_t)n + 1);
        HIP_CHECK(hipMemsetAsync(cflag.p, 0, sizeof(int) * cflag.n, s));
        hipLaunchKernelGGL(flag_eq_kernel, dim3(grid1(n)), dim3(kT), 0, s, n, cf.p, (int)ST_C, cflag.p);
        const int64_t nc = exclusive_scan(s, cflag.p, cmap.p, n, tmp);
        split = download_ints(s, cf.p, n);
        // P: count, scan, fill
        DevBuf<int> pcnt, prp, pcol;
        DevBuf<double> pval;
        pcnt.alloc((size_t)n + 1);
        HIP_CHECK(hipMemsetAsync(pcnt.p, 0, sizeof(int) * pcnt.n, s));
        hipLaunchKernelGGL(interp_kernel<false>, dim3(grid1(n)), dim3(kT), 0, s, Av, Sv, cf.p, cmap.p, pcnt.p,
                           nullptr, nullptr, nullptr);
        prp.alloc((size_t)n + 1);
        const int64_t pnnz = exclusive_scan(s, pcnt.p, prp.p, n, tmp);
        pcol.alloc((size_t)std::max<int64_t>(pnnz, 1));
        pval.alloc((size_t)std::max<int64_t>(pnnz, 1));
        hipLaunchKernelGGL(interp_kernel<true>, dim3(grid1(n)), dim3(kT), 0, s, Av, Sv, cf.p, cmap.p, nullptr,
                           prp.p, pcol.p, pval.p);
        HIP_CHECK(hipGetLastError());
        std::vector<int> hrp = download_ints(s, prp.p, (int64_t)n + 1), hcol = download_ints(s, pcol.p, pnnz);
        P = HostCSR();
        P.n_global_rows = A.n_global_rows;
        P.n_global_cols = nc;
        P.row_starts = A.row_starts;
        P.col_starts = {0, nc};
        P.rp.assign(hrp.begin(), hrp.end());
        P.col.assign(hcol.begin(), hcol.end());
        P.val.resize((size_t)pnnz);
        if (pnnz) HIP_CHECK(hipMemcpyAsync(P.val.data(), pval.p, sizeof(double) * pnnz, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        tm.lap("  device interpolation");
        return true;
    }
    // smoothed aggregation
    AMG_CHECK(opt.coarsen == AMG_COARSEN_SA, "unknown coarsening");
    const double theta = std::ldexp(opt.strong_threshold, -level);
    DevBuf<double> d;
    d.alloc(n);
    hipLaunchKernelGGL(diagonal_kernel, dim3(grid1(n)), dim3(kT), 0, s, Av, d.p);
    build_strength(
        s, n, S, tmp,
        [&](int* cnt) {
            hipLaunchKernelGGL(strength_symmetric_kernel<false>, dim3(grid1(n)), dim3(kT), 0, s, Av, d.p, theta,
                               cnt, nullptr, nullptr, nullptr);
        },
        [&](const int* srp, int* scol, double* sval) {
            hipLaunchKernelGGL(strength_symmetric_kernel<true>, dim3(grid1(n)), dim3(kT), 0, s, Av, d.p, theta,
                               nullptr, srp, scol, sval);
        });
    tm.lap("  device strength");
    const DCsr Sv = S.view();
    std::vector<unsigned> hs(n);
    for (int i = 0; i < n; ++i) hs[i] = hash32(i, opt.seed + (uint64_t)level);
    DevBuf<unsigned> dhs;
    dhs.upload(hs.data(), hs.size());
    DevBuf<int> st;
    DevBuf<unsigned long long> h0, l0, h1, l1, nu;
    st.alloc(n);
    h0.alloc(n), l0.alloc(n), h1.alloc(n), l1.alloc(n), nu.alloc(1);
    {
        std::vector<int> init(n, M_U);
        st.upload(init.data(), init.size());
    }
    for (int round = 0;; ++round) {
        AMG_CHECK(round <= n, "MIS(2) did not terminate");
        hipLaunchKernelGGL(mis2_tuple_kernel, dim3(grid1(n)), dim3(kT), 0, s, n, st.p, dhs.p, h0.p, l0.p);
        for (int hop = 0; hop < 2; ++hop) {
            hipLaunchKernelGGL(mis2_hop_kernel, dim3(grid1(n)), dim3(kT), 0, s, Sv, h0.p, l0.p, h1.p, l1.p);
            std::swap(h0.p, h1.p);
            std::swap(l0.p, l1.p);
        }
        HIP_CHECK(hipMemsetAsync(nu.p, 0, sizeof(unsigned long long), s));
        hipLaunchKernelGGL(mis2_update_kernel, dim3(grid1(n)), dim3(kT), 0, s, n, h0.p, l0.p, st.p, nu.p);
        HIP_CHECK(hipGetLastError());
        unsigned long long left = 0;
        HIP_CHECK(hipMemcpyAsync(&left, nu.p, sizeof(left), hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        if (left == 0) break;
    }
    DevBuf<int> flag, rootid, a1, agg, size;
    flag.alloc((size_t)n + 1);
    rootid.alloc((size_t)n + 1);
    HIP_CHECK(hipMemsetAsync(flag.p, 0, sizeof(int) * flag.n, s));
    hipLaunchKernelGGL(flag_eq_kernel, dim3(grid1(n)), dim3(kT), 0, s, n, st.p, (int)M_IN, flag.p);
    const int64_t na = exclusive_scan(s, flag.p, rootid.p, n, tmp);
    a1.alloc(n);
    agg.alloc(n);
    hipLaunchKernelGGL(mis2_pass1_kernel, dim3(grid1(n)), dim3(kT), 0, s, Sv, st.p, rootid.p, a1.p);
    HIP_CHECK(hipMemsetAsync(nu.p, 0, sizeof(unsigned long long), s));
    hipLaunchKernelGGL(mis2_pass2_kernel, dim3(grid1(n)), dim3(kT), 0, s, Sv, a1.p, agg.p, nu.p);
    HIP_CHECK(hipGetLastError());
    unsigned long long orphans = 0;
    HIP_CHECK(hipMemcpyAsync(&orphans, nu.p, sizeof(orphans), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (orphans) throw Error(AMG_ERR_INTERNAL, "MIS(2): unaggregated node");
    tm.lap("  device aggregation");
    // tentative prolongator T (1 / sqrt(|aggregate|)), rho = max_i sum_k |a_ik| / |a_ii|
    size.alloc((size_t)std::max<int64_t>(na, 1));
    HIP_CHECK(hipMemsetAsync(size.p, 0, sizeof(int) * size.n, s));
    hipLaunchKernelGGL(agg_size_kernel, dim3(grid1(n)), dim3(kT), 0, s, n, agg.p, size.p);
    DevBuf<double> rho, tv;
    rho.alloc(n);
    tv.alloc(n);
    hipLaunchKernelGGL(sa_rows_kernel, dim3(grid1(n)), dim3(kT), 0, s, Av, d.p, agg.p, size.p, rho.p, tv.p);
    HIP_CHECK(hipGetLastError());
    split = download_ints(s, agg.p, n);
    std::vector<double> hrho(n), htv(n), hd(n);
    HIP_CHECK(hipMemcpyAsync(hrho.data(), rho.p, sizeof(double) * n, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(htv.data(), tv.p, sizeof(double) * n, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(hd.data(), d.p, sizeof(double) * n, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    double r = 0.0;
    for (int i = 0; i < n; ++i)
        if (hrho[i] > r) r = hrho[i];
    const double omega = (4.0 / 3.0) / r;
    HostCSR T;
    T.n_global_rows = A.n_global_rows;
    T.n_global_cols = na;
    T.row_starts = A.row_starts;
    T.col_starts = {0, na};
    T.rp.resize((size_t)n + 1);
    T.col.resize(n);
    T.val = htv;
    for (int i = 0; i <= n; ++i) T.rp[i] = i;
    for (int i = 0; i < n; ++i) T.col[i] = split[i];
    tm.lap("  device tentative prolongator");
    HostCSR AT = spgemm_device(ctx, comm, A, T);
    tm.lap("  device A*T");
    // P = T - (omega / a_ii) A T, rows merged by column (same as sa_prolongator)
    P = HostCSR();
    P.n_global_rows = A.n_global_rows;
    P.n_global_cols = na;
    P.row_starts = A.row_starts;
    P.col_starts = {0, na};
    P.rp.assign((size_t)n + 1, 0);
    std::vector<int64_t> len(n);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        int64_t c = AT.rp[i + 1] - AT.rp[i];
        const int64_t jt = T.col[i];
        if (!std::binary_search(AT.col.begin() + AT.rp[i], AT.col.begin() + AT.rp[i + 1], jt)) ++c;
        len[i] = c;
    }
    for (int i = 0; i < n; ++i) P.rp[i + 1] = P.rp[i] + len[i];
    P.col.resize(P.rp[n]);
    P.val.resize(P.rp[n]);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        const double c = omega * (1.0 / hd[i]);
        int64_t ka = AT.rp[i], ea = AT.rp[i + 1], kt = T.rp[i], et = T.rp[i + 1], q = P.rp[i];
        while (ka < ea || kt < et) {
            const int64_t ja = ka < ea ? AT.col[ka] : INT64_MAX, jt = kt < et ? T.col[kt] : INT64_MAX;
            const int64_t j = ja < jt ? ja : jt;
            double tvv = 0.0, av = 0.0;
            if (jt == j) tvv = T.val[kt++];
            if (ja == j) av = AT.val[ka++];
            P.col[q] = j;
            P.val[q++] = tvv - c * av;
        }
    }
    tm.lap("  device smoothed prolongator");
    return true;
}

// R = P^T on the device for one rank: stable radix sort of the entries by column keeps each
// R row in ascending fine-row order, like transpose().
bool transpose_device(Context& ctx, const HostComm& comm, const HostCSR& P, HostCSR& R) {
    if (comm.nranks != 1) return false;
    hipStream_t s = ctx.stream;
    const int64_t n = P.nrows(), nnz = P.nnz(), nc = P.n_global_cols;
    if (nnz == 0 || n >= INT_MAX || nnz >= INT_MAX || nc >= INT_MAX) return false;
    std::vector<int> rp(n + 1), col(nnz);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i <= n; ++i) rp[i] = (int)P.rp[i];
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < nnz; ++k) col[k] = (int)P.col[k];
    DevBuf<int> drp, dcol, keys_out, idx_in, idx_out, rowof, cnt, rrp;
    DevBuf<double> dval;
    DevBuf<long long> rcol;
    DevBuf<double> rval;
    DevBuf<char> tmp;
    drp.upload(rp.data(), rp.size());
    dcol.upload(col.data(), col.size());
    dval.upload(P.val.data(), P.val.size());
    keys_out.alloc(nnz);
    idx_in.alloc(nnz);
    idx_out.alloc(nnz);
    rowof.alloc(nnz);
    hipLaunchKernelGGL(iota_kernel, dim3(grid1(nnz)), dim3(kT), 0, s, (int)nnz, idx_in.p);
    hipLaunchKernelGGL(expand_rows_kernel, dim3(grid1(n)), dim3(kT), 0, s, drp.p, (int)n, rowof.p);
    int bits = 1;
    while (bits < 31 && (1ll << bits) < nc) ++bits;
    size_t bytes = 0;
    HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, dcol.p, keys_out.p, idx_in.p, idx_out.p,
                                                 (int)nnz, 0, bits, s));
    tmp.alloc(bytes);
    HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp.p, bytes, dcol.p, keys_out.p, idx_in.p, idx_out.p,
                                                 (int)nnz, 0, bits, s));
    rcol.alloc(nnz);
    rval.alloc(nnz);
    hipLaunchKernelGGL(gather_transpose_kernel, dim3(grid1(nnz)), dim3(kT), 0, s, (int)nnz, idx_out.p,
                       rowof.p, dval.p, rcol.p, rval.p);
    cnt.alloc((size_t)nc + 1);
    HIP_CHECK(hipMemsetAsync(cnt.p, 0, sizeof(int) * cnt.n, s));
    hipLaunchKernelGGL(count_cols_kernel, dim3(grid1(nnz)), dim3(kT), 0, s, (int)nnz, dcol.p, cnt.p);
    rrp.alloc((size_t)nc + 1);
    exclusive_scan(s, cnt.p, rrp.p, (int)nc, tmp);
    HIP_CHECK(hipGetLastError());
    R = HostCSR();
    R.n_global_rows = nc;
    R.n_global_cols = P.n_global_rows;
    R.row_starts = P.col_starts;
    R.col_starts = P.row_starts;
    std::vector<int> hrp = download_ints(s, rrp.p, nc + 1);
    R.rp.assign(hrp.begin(), hrp.end());
    R.col.resize(nnz);
    R.val.resize(nnz);
    std::vector<long long> tc(nnz);
    HIP_CHECK(hipMemcpyAsync(tc.data(), rcol.p, sizeof(long long) * nnz, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(R.val.data(), rval.p, sizeof(double) * nnz, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    std::copy(tc.begin(), tc.end(), R.col.begin());
    return true;
}

}  // namespace amg
