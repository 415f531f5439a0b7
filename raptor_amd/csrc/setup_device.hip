// setup_device.hip -- AMG setup on the GPU: strength of connection,
// PMIS splitting, classical interpolation, MIS(2) aggregation and the smoothed-aggregation
// prolongator on any number of ranks, the transpose R = P^T on one rank.  Every integer
// decision and every floating-point sum follows host_setup.cpp / oracle/amg_oracle.c exactly
// (DESIGN.md 3), so the hierarchy is bit-identical to the host path's at every rank count;
// the Galerkin products stay on the device SpGEMM (spgemm.hip).
//
// Layout: one upload of this rank's rows of A per level -- int32 row_ptr, int32 GLOBAL column
// ids, fp64 values; the strength graph S stays on the device; per-row kernels are one thread
// per row (rows are short and independent); rounds (PMIS, MIS(2)) are synchronous: each round
// reads the previous round's states only, other ranks' states through a halo (Dist) that is
// forwarded between rounds (device pack, host setup exchange, upload).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>

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

// rows of this rank: local row i is global row lo + i; columns are GLOBAL ids (int32: the
// global size is checked < 2^31), ascending per row -- the host image's order, so every
// loop below visits entries exactly as host_setup.cpp does
struct DCsr {
    const int* rp;
    const int* col;
    const double* val;
    int n;
    int lo;
};

// where the state of global point g lives: local rows [lo, lo + n) or the sorted halo ids
// gid[0, nh) (several ranks: states forwarded from their owners each round)
struct Dist {
    int lo, n;
    const int* gid;
    int nh;
    // >= 0: local index; < 0: halo index -(t + 1); INT_MIN: neither
    __device__ __forceinline__ int loc(int g) const {
        if (g >= lo && g < lo + n) return g - lo;
        int a = 0, b = nh;
        while (a < b) {
            const int m = (a + b) >> 1;
            const int v = gid[m];
            if (v == g) return -m - 1;
            if (v < g) a = m + 1;
            else b = m;
        }
        return INT_MIN;
    }
    template <class T>
    __device__ __forceinline__ T get(const T* local, const T* halo, int g) const {
        const int l = loc(g);
        return l >= 0 ? local[l] : halo[-l - 1];
    }
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
    const int gi = A.lo + i;
    for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) {
        if (A.col[k] == gi) continue;
        const double v = -A.val[k];
        if (!any || v > mx) mx = v;
        any = true;
    }
    const bool has = any && mx > 0.0;
    const double thr = theta * mx;
    int q = FILL ? srp[i] : 0, c = 0;
    for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) {
        if (!(has && A.col[k] != gi && -A.val[k] >= thr)) continue;
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
        if (A.col[k] == A.lo + i) {
            v = A.val[k];
            break;
        }
    d[i] = v;
}

// SA strength, signed (r6; host_setup.cpp sa_strong): -a_ij >= theta sqrt(|a_ii a_jj|), j != i
// (a_jj of another rank's column through D: the forwarded diagonal hd)
__device__ __forceinline__ bool dsa_strong(double aij, double di, double dj, double theta) {
    return -aij >= theta * sqrt(fabs(di * dj));
}

template <bool FILL>
__global__ void strength_symmetric_kernel(DCsr A, Dist D, const double* d, const double* hd, double theta,
                                          int* cnt, const int* srp, int* scol, double* sval) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= A.n) return;
    int q = FILL ? srp[i] : 0, c = 0;
    for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) {
        const int j = A.col[k];
        if (j == A.lo + i) continue;
        if (!dsa_strong(A.val[k], d[i], D.get(d, hd, j), theta)) continue;
        if (FILL) {
            scol[q] = j;
            sval[q++] = A.val[k];
        }
        ++c;
    }
    if (!FILL) cnt[i] = c;
}

// ---- PMIS ------------------------------------------------------------------------------
// |S^T_i| over this rank's rows: local columns only (off-rank dependents arrive as pairs)
__global__ void col_count_kernel(DCsr S, int* tcnt) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= S.n) return;
    for (int k = S.rp[i]; k < S.rp[i + 1]; ++k) {
        const int c = S.col[k] - S.lo;
        if (c >= 0 && c < S.n) atomicAdd(&tcnt[c], 1);
    }
}

// S^T adjacency of the local-local part (row j of S^T = the global ids of local rows i with
// j in S_i; order within a row arbitrary -- PMIS only takes maxima over the set)
__global__ void transpose_fill_kernel(DCsr S, int* cursor, int* tcol) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= S.n) return;
    for (int k = S.rp[i]; k < S.rp[i + 1]; ++k) {
        const int c = S.col[k] - S.lo;
        if (c >= 0 && c < S.n) tcol[atomicAdd(&cursor[c], 1)] = S.lo + i;
    }
}

// entries of S whose column lives on another rank: (column, dependent row) pairs, row order
template <bool FILL>
__global__ void offrank_kernel(DCsr S, int* cnt, const int* orp, int* pc, int* pj) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= S.n) return;
    int q = FILL ? orp[i] : 0, c = 0;
    for (int k = S.rp[i]; k < S.rp[i + 1]; ++k) {
        const int g = S.col[k];
        if (g >= S.lo && g < S.lo + S.n) continue;
        if (FILL) {
            pc[q] = g;
            pj[q++] = S.lo + i;
        }
        ++c;
    }
    if (!FILL) cnt[i] = c;
}

// key = |S^T_i| << 32 | hash32(global id): tcnt = local dependents, ecnt = off-rank ones
__global__ void pmis_init_kernel(int n, int lo, const int* tcnt, const int* erp, unsigned long long seed,
                                 unsigned long long* key, int* cf) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    const int c = tcnt[i] + (erp ? erp[i + 1] - erp[i] : 0);
    key[i] = ((unsigned long long)c << 32) | (unsigned long long)dhash32(lo + i, seed);
    cf[i] = c == 0 ? ST_F : ST_U;
}

// undecided i -> C iff its (key, global id) beats every undecided j in S_i u S^T_i (local
// dependents tcol, off-rank dependents ecol); halo states / keys through D
__global__ void pmis_select_kernel(DCsr S, Dist D, const int* trp, const int* tcol, const int* erp,
                                   const int* ecol, const unsigned long long* key,
                                   const unsigned long long* hkey, const int* cf, const int* hcf,
                                   unsigned char* newc) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= S.n) return;
    newc[i] = 0;
    if (cf[i] != ST_U) return;
    const unsigned long long ki = key[i];
    const int gi = S.lo + i;
    bool best = true;
    auto beats = [&](int g) {  // false when undecided neighbour g outranks i
        const int l = D.loc(g);
        const int sj = l >= 0 ? cf[l] : hcf[-l - 1];
        if (sj != ST_U) return true;
        const unsigned long long kj = l >= 0 ? key[l] : hkey[-l - 1];
        return !(kj > ki || (kj == ki && g > gi));
    };
    for (int k = S.rp[i]; k < S.rp[i + 1] && best; ++k) best = beats(S.col[k]);
    for (int t = trp[i]; t < trp[i + 1] && best; ++t) best = beats(tcol[t]);
    if (erp)
        for (int t = erp[i]; t < erp[i + 1] && best; ++t) best = beats(ecol[t]);
    newc[i] = best;
}

__global__ void pmis_apply_kernel(int n, const unsigned char* newc, int* cf) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i < n && newc[i]) cf[i] = ST_C;
}

// undecided i with a C point in S_i -> F; count the undecided that remain
__global__ void pmis_fpass_kernel(DCsr S, Dist D, int* cf, const int* hcf, unsigned long long* nu) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= S.n || cf[i] != ST_U) return;
    for (int k = S.rp[i]; k < S.rp[i + 1]; ++k)
        if (D.get(cf, hcf, S.col[k]) == ST_C) {
            cf[i] = ST_F;
            return;
        }
    atomicAdd(nu, 1ull);
}

// halo forwarding: packed[t] = local[send_idx[t]]
template <class T>
__global__ void pack_kernel_t(int n, const int* idx, const T* local, T* packed) {
    const int t = blockIdx.x * kT + threadIdx.x;
    if (t < n) packed[t] = local[idx[t]];
}

// ---- classical interpolation ------------------------------------------------------------
// is global j a strong neighbour of local row i (S rows ascending)
__device__ __forceinline__ bool strong(const DCsr& S, int i, int j) {
    return dfind(S.col, S.rp[i], S.rp[i + 1], j) >= 0;
}

// rows of A reachable from this rank: local rows, and the ghost rows of the halo points
// (D's halo = A's off-rank columns; ghost row t of halo point D.gid[t], global column ids)
struct ARows {
    DCsr A;
    Dist D;
    const int* grp;
    const int* gcol;
    const double* gval;
    __device__ __forceinline__ void row(int g, int& b, int& e, const int*& c, const double*& v) const {
        const int l = D.loc(g);
        if (l >= 0) {
            b = A.rp[l], e = A.rp[l + 1], c = A.col, v = A.val;
        } else {
            const int t = -l - 1;
            b = grp[t], e = grp[t + 1], c = gcol, v = gval;
        }
    }
};

// F row i: d = a_ii + weak couplings + couplings to strong F neighbours whose s_k is 0;
// w_ij = -num_j / d for j in C_i (strong C neighbours), num_j = a_ij + sum over strong F
// neighbours k (A-row order) of (a_ik a_kj) / s_k, s_k = sum of row k's couplings to C_i of
// sign opposite to a_kk.  Same loops and order as host_setup.cpp interp_classical().
// cf / cmap of halo points through R.D (hcf, hcmap); P columns are global coarse ids.
template <bool FILL>
__device__ void interp_row_serial(const ARows& R, const DCsr& S, const int* cf, const int* hcf, const int* cmap,
                                  const int* hcmap, int* cnt, const int* prp, int* pcol, double* pval, int i) {
    const DCsr& A = R.A;
    if (cf[i] == ST_C) {
        if (FILL) {
            pcol[prp[i]] = cmap[i];
            pval[prp[i]] = 1.0;
        } else {
            cnt[i] = 1;
        }
        return;
    }
    const int gi = A.lo + i;
    // strong first: a strong neighbour is a column of row i, so its state is local or halo
    auto is_c = [&](int g) { return R.D.get(cf, hcf, g) == ST_C; };
    auto in_ci = [&](int m) { return m != gi && strong(S, i, m) && is_c(m); };
    double d = 0.0;
    for (int k = A.rp[i]; k < A.rp[i + 1]; ++k)
        if (A.col[k] == gi) {
            d = A.val[k];
            break;
        }
    int nci = 0;
    for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) {
        const int j = A.col[k];
        if (j == gi) continue;
        const bool st = strong(S, i, j);
        if (st && is_c(j)) ++nci;
        else if (!st) d += A.val[k];
    }
    if (!FILL) {
        cnt[i] = nci;
        return;
    }
    if (nci == 0) return;
    // s_k of strong F neighbour kk over its row (local or ghost)
    auto s_of = [&](int kk, bool& pos) {
        int b, e;
        const int* rc;
        const double* rv;
        R.row(kk, b, e, rc, rv);
        double akk = 0.0;
        for (int u = b; u < e; ++u)
            if (rc[u] == kk) {
                akk = rv[u];
                break;
            }
        pos = akk > 0.0;
        double s = 0.0;
        for (int u = b; u < e; ++u) {
            const double v = rv[u];
            if ((pos ? v < 0.0 : v > 0.0) && in_ci(rc[u])) s += v;
        }
        return s;
    };
    // s_k == 0 neighbours add a_ik to d, in A-row order (second pass of the host loop)
    for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) {
        const int kk = A.col[k];
        if (kk == gi || !strong(S, i, kk) || is_c(kk)) continue;
        bool pos;
        if (s_of(kk, pos) == 0.0) d += A.val[k];
    }
    // num_j accumulates in this row's own P slots (pval), k outer: s_k is formed once per
    // strong F neighbour instead of once per (j, k) pair, and every num_j still receives its
    // terms in A-row order of k -- the host loop's order, so the weights are bit-identical
    const int q0 = prp[i];
    int q = q0;
    for (int kj = A.rp[i]; kj < A.rp[i + 1]; ++kj) {
        const int j = A.col[kj];
        if (j == gi || !strong(S, i, j) || !is_c(j)) continue;
        pcol[q] = R.D.get(cmap, hcmap, j);
        pval[q++] = A.val[kj];
    }
    for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) {
        const int kk = A.col[k];
        if (kk == gi || !strong(S, i, kk) || is_c(kk)) continue;
        bool pos;
        const double s = s_of(kk, pos);
        if (s == 0.0) continue;
        int b, e;
        const int* rc;
        const double* rv;
        R.row(kk, b, e, rc, rv);
        q = q0;
        for (int kj = A.rp[i]; kj < A.rp[i + 1]; ++kj) {
            const int j = A.col[kj];
            if (j == gi || !strong(S, i, j) || !is_c(j)) continue;
            const int uj = dfind(rc, b, e, j);
            if (uj >= 0 && (pos ? rv[uj] < 0.0 : rv[uj] > 0.0)) pval[q] += (A.val[k] * rv[uj]) / s;
            ++q;
        }
    }
    for (q = q0; q < q0 + nci; ++q) pval[q] = -pval[q] / d;
}

template <bool FILL>
__global__ void interp_kernel(ARows R, DCsr S, const int* cf, const int* hcf, const int* cmap,
                              const int* hcmap, int* cnt, const int* prp, int* pcol, double* pval) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i < R.A.n) interp_row_serial<FILL>(R, S, cf, hcf, cmap, hcmap, cnt, prp, pcol, pval, i);
}

// Wave-per-row form of interp_kernel for operators with long rows (the Galerkin levels: a
// thread per row walked 50-100-entry rows and their neighbours' rows serially, 13-52 ms per
// launch on grids of 3-4,249 workgroups).  The same sums in the same order:
//  * lanes classify the row's entries (strong / C / diagonal) into LDS and form s_k of the
//    strong F neighbours, one neighbour per lane (s_k's own loop is serial, as in s_of);
//  * lane 0 forms d in the host's two passes (weak couplings in row order, then the strong F
//    neighbours with s_k == 0 in row order);
//  * lane q forms num_j of the q-th strong C neighbour: a_ij, then + (a_ik a_kj) / s_k over the
//    strong F neighbours k in row order -- one accumulator per lane, the host's k order.
// Rows longer than kIwMax entries run interp_kernel's loops on lane 0.
constexpr int kIwWaves = 4, kIwMax = 512;
enum { IW_STRONG = 1, IW_C = 2, IW_DIAG = 4, IW_POS = 8 };

template <bool FILL>
__device__ void interp_row_serial(const ARows& R, const DCsr& S, const int* cf, const int* hcf, const int* cmap,
                                  const int* hcmap, int* cnt, const int* prp, int* pcol, double* pval, int i);

template <bool FILL>
__global__ __launch_bounds__(64 * kIwWaves) void interp_wave_kernel(ARows R, DCsr S, const int* cf, const int* hcf,
                                                                    const int* cmap, const int* hcmap, int* cnt,
                                                                    const int* prp, int* pcol, double* pval) {
    __shared__ unsigned char fl_s[kIwWaves][kIwMax];
    __shared__ double sv_s[kIwWaves][kIwMax];
    const DCsr& A = R.A;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = blockIdx.x * kIwWaves + w;
    if (i >= A.n) return;  // wave-uniform
    unsigned char* fl = fl_s[w];
    double* sv = sv_s[w];
    const int b0 = A.rp[i], e0 = A.rp[i + 1], len = e0 - b0;
    if (cf[i] == ST_C || len > kIwMax) {
        if (lane == 0) interp_row_serial<FILL>(R, S, cf, hcf, cmap, hcmap, cnt, prp, pcol, pval, i);
        return;
    }
    const int gi = A.lo + i;
    auto is_c = [&](int g) { return R.D.get(cf, hcf, g) == ST_C; };
    auto in_ci = [&](int m) { return m != gi && strong(S, i, m) && is_c(m); };
    // entry classes; nci = strong C neighbours
    int nci = 0;
    for (int k0 = 0; k0 < len; k0 += 64) {
        const int k = k0 + lane;
        unsigned char f = 0;
        if (k < len) {
            const int j = A.col[b0 + k];
            if (j == gi) {
                f = IW_DIAG;
            } else if (strong(S, i, j)) {
                f = IW_STRONG | (is_c(j) ? IW_C : 0);
            }
            fl[k] = f;
        }
        nci += __popcll(__ballot(f == (IW_STRONG | IW_C)));
    }
    if (!FILL) {
        if (lane == 0) cnt[i] = nci;
        return;
    }
    if (nci == 0) return;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    // s_k of the strong F neighbours (interp_kernel's s_of), one per lane
    for (int k0 = 0; k0 < len; k0 += 64) {
        const int k = k0 + lane;
        if (k < len && fl[k] == IW_STRONG) {
            const int kk = A.col[b0 + k];
            int b, e;
            const int* rc;
            const double* rv;
            R.row(kk, b, e, rc, rv);
            double akk = 0.0;
            for (int u = b; u < e; ++u)
                if (rc[u] == kk) {
                    akk = rv[u];
                    break;
                }
            const bool pos = akk > 0.0;
            double sk = 0.0;
            for (int u = b; u < e; ++u) {
                const double v = rv[u];
                if ((pos ? v < 0.0 : v > 0.0) && in_ci(rc[u])) sk += v;
            }
            sv[k] = sk;
            if (pos) fl[k] = IW_STRONG | IW_POS;
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // d: a_ii (first diagonal entry), + weak couplings in row order, + strong F with s_k == 0
    double d = 0.0;
    if (lane == 0) {
        for (int k = 0; k < len; ++k)
            if (fl[k] & IW_DIAG) {
                d = A.val[b0 + k];
                break;
            }
        for (int k = 0; k < len; ++k)
            if (fl[k] == 0) d += A.val[b0 + k];
        for (int k = 0; k < len; ++k)
            if ((fl[k] & (IW_STRONG | IW_C)) == IW_STRONG && sv[k] == 0.0) d += A.val[b0 + k];
    }
    d = __shfl(d, 0, 64);
    // num_j, lane = strong C neighbour (q order = row order)
    const int q0 = prp[i];
    int qbase = 0;
    for (int k0 = 0; k0 < len; k0 += 64) {
        const int kj = k0 + lane;
        const bool isc = kj < len && fl[kj] == (IW_STRONG | IW_C);
        const unsigned long long m = __ballot(isc);
        if (isc) {
            const int q = qbase + __popcll(m & ((1ull << lane) - 1ull));
            const int j = A.col[b0 + kj];
            double num = A.val[b0 + kj];
            for (int k = 0; k < len; ++k) {
                const unsigned char f = fl[k];
                if ((f & (IW_STRONG | IW_C)) != IW_STRONG) continue;
                const double sk = sv[k];
                if (sk == 0.0) continue;
                const int kk = A.col[b0 + k];
                int b, e;
                const int* rc;
                const double* rv;
                R.row(kk, b, e, rc, rv);
                const int uj = dfind(rc, b, e, j);
                const bool pos = (f & IW_POS) != 0;
                if (uj >= 0 && (pos ? rv[uj] < 0.0 : rv[uj] > 0.0)) num += (A.val[b0 + k] * rv[uj]) / sk;
            }
            pcol[q0 + q] = R.D.get(cmap, hcmap, j);
            pval[q0 + q] = -num / d;
        }
        qbase += __popcll(m);
    }
}

// ---- MIS(2) aggregation -----------------------------------------------------------------
// tuple (state, hash, global id) of every local point, packed hi = state << 32 | hash, lo = id
__global__ void mis2_tuple_kernel(int n, int lo, const int* st, const unsigned* hs, unsigned long long* h,
                                  unsigned long long* l) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    h[i] = ((unsigned long long)(unsigned)st[i] << 32) | hs[i];
    l[i] = (unsigned long long)(lo + i);
}

// one hop of the lexicographic max over S_i (halo tuples through D: hh / hl)
__global__ void mis2_hop_kernel(DCsr S, Dist D, const unsigned long long* h0, const unsigned long long* l0,
                                const unsigned long long* hh, const unsigned long long* hl,
                                unsigned long long* h1, unsigned long long* l1) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= S.n) return;
    unsigned long long mh = h0[i], ml = l0[i];
    for (int k = S.rp[i]; k < S.rp[i + 1]; ++k) {
        const int l = D.loc(S.col[k]);
        const unsigned long long xh = l >= 0 ? h0[l] : hh[-l - 1], xl = l >= 0 ? l0[l] : hl[-l - 1];
        if (xh > mh || (xh == mh && xl > ml)) mh = xh, ml = xl;
    }
    h1[i] = mh;
    l1[i] = ml;
}

__global__ void mis2_update_kernel(int n, int lo, const unsigned long long* h, const unsigned long long* l,
                                   int* st, unsigned long long* nu) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= n || st[i] != M_U) return;
    if (l[i] == (unsigned long long)(lo + i)) st[i] = M_IN;
    else if ((h[i] >> 32) == M_IN) st[i] = M_OUT;
    if (st[i] == M_U) atomicAdd(nu, 1ull);
}

// pass 1: a root keeps its aggregate id (aggr: the global id of a root, -1 otherwise); the
// others join the first root neighbour in S-row order
__global__ void mis2_pass1_kernel(DCsr S, Dist D, const int* aggr, const int* haggr, int* a1) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= S.n) return;
    int a = aggr[i];
    if (a < 0)
        for (int k = S.rp[i]; k < S.rp[i + 1]; ++k) {
            const int aj = D.get(aggr, haggr, S.col[k]);
            if (aj >= 0) {
                a = aj;
                break;
            }
        }
    a1[i] = a;
}

// pass 2: the rest join the pass-1 neighbour with max |s_ij| (ties: smaller aggregate id)
__global__ void mis2_pass2_kernel(DCsr S, Dist D, const int* a1, const int* ha1, int* agg,
                                  unsigned long long* orphans) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= S.n) return;
    if (a1[i] >= 0) {
        agg[i] = a1[i];
        return;
    }
    double best = -1.0;
    int ba = -1;
    for (int k = S.rp[i]; k < S.rp[i + 1]; ++k) {
        const int aj = D.get(a1, ha1, S.col[k]);
        if (aj < 0) continue;
        const double w = fabs(S.val[k]);
        if (w > best || (w == best && aj < ba)) best = w, ba = aj;
    }
    agg[i] = ba;
    if (ba < 0) atomicAdd(orphans, 1ull);
}

// ---- SA smoothing (r6; host_setup.cpp sa_filter / sa_rho / sa_prolongator) ------------------
// the filtered operator: the diagonal and the strong off-diagonals in row order; the diagonal
// value f_i = a_ii + the weak off-diagonals (row order).  Pass 0 counts, pass 1 fills.
template <bool FILL>
__global__ void sa_filter_kernel(DCsr A, Dist D, const double* d, const double* hd, double theta, int* cnt,
                                 const int* frp, int* fcol, double* fval) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= A.n) return;
    const int gi = A.lo + i;
    if (!FILL) {
        int c = 0;
        for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) {
            const int j = A.col[k];
            c += j == gi || dsa_strong(A.val[k], d[i], D.get(d, hd, j), theta);
        }
        cnt[i] = c;
        return;
    }
    double f = d[i];
    for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) {
        const int j = A.col[k];
        if (j != gi && !dsa_strong(A.val[k], d[i], D.get(d, hd, j), theta)) f += A.val[k];
    }
    int q = frp[i];
    for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) {
        const int j = A.col[k];
        if (j == gi) {
            fcol[q] = j;
            fval[q++] = f;
        } else if (dsa_strong(A.val[k], d[i], D.get(d, hd, j), theta)) {
            fcol[q] = j;
            fval[q++] = A.val[k];
        }
    }
}

// the largest |v_i|: non-negative doubles order like their bit patterns, so an integer
// atomicMax is exact in any order
__device__ __forceinline__ void dmax_abs(unsigned long long* m, double v) {
    atomicMax(m, (unsigned long long)__double_as_longlong(fabs(v)));
}

__global__ void max_abs_kernel(int n, const double* __restrict__ x, unsigned long long* m) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i < n) dmax_abs(m, x[i]);
}

__global__ void div_scalar_kernel(int n, const double* __restrict__ y, double lam, double* __restrict__ x) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i < n) x[i] = y[i] / lam;
}

// one power step: y_i = (A_F x)_i / a_ii (row order from 0.0), max |y_i|
__global__ void sa_power_kernel(DCsr F, Dist D, const double* __restrict__ x, const double* __restrict__ hx,
                                const double* __restrict__ d, double* __restrict__ y, unsigned long long* m) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= F.n) return;
    double s = 0.0;
    for (int k = F.rp[i]; k < F.rp[i + 1]; ++k) s += F.val[k] * D.get(x, hx, F.col[k]);
    const double v = s / d[i];
    y[i] = v;
    dmax_abs(m, v);
}

// P = T - (omega / a_ii) (A_F T): row i's products (agg_k, f_ik t_k) in A_F's row order,
// insertion-sorted by aggregate (stable: row order kept inside an aggregate) into the row's
// slice of the scratch; pass 0 sorts and counts the distinct aggregates with T's (agg_i);
// pass 1 sums each aggregate's products from 0.0 in that order and merges T's entry
template <bool FILL>
__global__ void sa_smooth_kernel(DCsr F, Dist D, const int* __restrict__ agg, const int* __restrict__ hagg,
                                 const double* __restrict__ t, const double* __restrict__ ht,
                                 const double* __restrict__ d, double omega, int* __restrict__ skey,
                                 double* __restrict__ sval, long long* __restrict__ cnt,
                                 const long long* __restrict__ prp, long long* __restrict__ pcol,
                                 double* __restrict__ pval) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= F.n) return;
    const int b = F.rp[i], e = F.rp[i + 1], ai = agg[i];
    if (!FILL) {
        for (int k = b; k < e; ++k) {
            const int g = F.col[k];
            const int key = D.get(agg, hagg, g);
            const double v = F.val[k] * D.get(t, ht, g);
            int p = k;
            while (p > b && skey[p - 1] > key) {
                skey[p] = skey[p - 1];
                sval[p] = sval[p - 1];
                --p;
            }
            skey[p] = key;
            sval[p] = v;
        }
        long long c = 0;
        bool tin = false;
        for (int k = b; k < e; ++k) {
            if (k == b || skey[k] != skey[k - 1]) ++c;
            tin = tin || skey[k] == ai;
        }
        cnt[i] = c + (tin ? 0 : 1);
        return;
    }
    const double c = omega * (1.0 / d[i]);
    long long q = prp[i];
    bool tleft = true;
    int k = b;
    while (k < e || tleft) {
        const long long ja = k < e ? (long long)skey[k] : LLONG_MAX, jj = tleft ? (long long)ai : LLONG_MAX;
        const long long j = ja < jj ? ja : jj;
        double tvv = 0.0, av = 0.0;
        if (jj == j) {
            tvv = t[i];
            tleft = false;
        }
        if (ja == j)
            for (; k < e && skey[k] == j; ++k) av += sval[k];
        pcol[q] = j;
        pval[q++] = tvv - c * av;
    }
}

// MIS(2) roots: flags for the exclusive scan that numbers them, then each root's aggregate id
__global__ void root_flag_kernel(int n, const int* st, int* flag) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i < n) flag[i] = st[i] == M_IN;
}

__global__ void root_id_kernel(int n, const int* st, const int* pos, int base, int* aggr) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i < n) aggr[i] = st[i] == M_IN ? base + pos[i] : -1;
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

// N ranks: the transpose's exchange record (the host transpose's layout: R row j, R column i
// = global fine row, value)
struct TRec {
    long long j, i;
    double v;
};

// send side: entries in (column, fine row) order -- the radix sort by column is stable over
// the row-major entry order -- as records; the owner of column j receives a contiguous range
__global__ void transpose_records_kernel(int nnz, const int* __restrict__ keys, const int* __restrict__ perm,
                                        const int* __restrict__ rowof, const double* __restrict__ val,
                                        long long i0, TRec* __restrict__ out) {
    const int t = blockIdx.x * kT + threadIdx.x;
    if (t >= nnz) return;
    const int k = perm[t];
    out[t] = TRec{keys[t], i0 + rowof[k], val[k]};
}

// receive side: the local row of every record (j - lo), the key of a stable sort that keeps
// rank order, then ascending i, inside each row
__global__ void record_rows_kernel(int m, const TRec* __restrict__ in, long long lo, int* __restrict__ key) {
    const int t = blockIdx.x * kT + threadIdx.x;
    if (t < m) key[t] = (int)(in[t].j - lo);
}

__global__ void gather_records_kernel(int m, const int* __restrict__ perm, const TRec* __restrict__ in,
                                      long long* __restrict__ rcol, double* __restrict__ rval) {
    const int t = blockIdx.x * kT + threadIdx.x;
    if (t >= m) return;
    const TRec e = in[perm[t]];
    rcol[t] = e.i;
    rval[t] = e.v;
}

// first sorted position with key >= bound[o], per owner boundary o
__global__ void owner_bounds_kernel(int m, const int* __restrict__ keys, int nb, const long long* __restrict__ bound,
                                    long long* __restrict__ out) {
    const int o = blockIdx.x * kT + threadIdx.x;
    if (o >= nb) return;
    int lo = 0, hi = m;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((long long)keys[mid] < bound[o]) lo = mid + 1;
        else hi = mid;
    }
    out[o] = lo;
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

int64_t exclusive_scan64(hipStream_t s, const long long* in, long long* out, int n, DevBuf<char>& tmp) {
    size_t bytes = 0;
    HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, n + 1, s));
    if (tmp.n < bytes) tmp.alloc(bytes);
    HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp.p, bytes, in, out, n + 1, s));
    long long total = 0;
    HIP_CHECK(hipMemcpyAsync(&total, out + n, sizeof(long long), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    return total;
}

// index-width conversions of the setup's device images (grid-stride: up to 2^31 entries)
__global__ void narrow_kernel(long long n, const long long* __restrict__ in, int* __restrict__ out) {
    for (long long t = (long long)blockIdx.x * kT + threadIdx.x; t < n; t += (long long)gridDim.x * kT)
        out[t] = (int)in[t];
}

__global__ void widen_kernel(long long n, const int* __restrict__ in, long long* __restrict__ out) {
    for (long long t = (long long)blockIdx.x * kT + threadIdx.x; t < n; t += (long long)gridDim.x * kT)
        out[t] = in[t];
}

inline unsigned grid_cap(long long n) { return std::min<unsigned>(grid1(n), 1u << 16); }

// P = T - (omega / a_ii) A T on the device, rows merged by column exactly as the host merge in
// level_setup_device (sa_prolongator): T has one entry per row (aggregate agg_i, value t_i)
template <bool FILL>
__global__ void sa_smooth_kernel(int n, const long long* __restrict__ atrp, const long long* __restrict__ atcol,
                                 const double* __restrict__ atval, const long long* __restrict__ agg,
                                 const double* __restrict__ tval, const double* __restrict__ d, double omega,
                                 long long* __restrict__ cnt, const long long* __restrict__ prp,
                                 long long* __restrict__ pcol, double* __restrict__ pval) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    const long long b = atrp[i], e = atrp[i + 1], jt = agg[i];
    if (!FILL) {
        long long lo = b, hi = e;
        while (lo < hi) {
            const long long m = (lo + hi) >> 1;
            if (atcol[m] < jt) lo = m + 1;
            else hi = m;
        }
        cnt[i] = (e - b) + ((lo < e && atcol[lo] == jt) ? 0 : 1);
        return;
    }
    const double c = omega * (1.0 / d[i]);
    long long ka = b, q = prp[i];
    bool tleft = true;
    while (ka < e || tleft) {
        const long long ja = ka < e ? atcol[ka] : LLONG_MAX, jj = tleft ? jt : LLONG_MAX;
        const long long j = ja < jj ? ja : jj;
        double tvv = 0.0, av = 0.0;
        if (jj == j) {
            tvv = tval[i];
            tleft = false;
        }
        if (ja == j) av = atval[ka++];
        pcol[q] = j;
        pval[q++] = tvv - c * av;
    }
}

}  // namespace

void DevCsr::ensure_rp32(hipStream_t s) {
    if (rp32.p) return;
    AMG_CHECK(rp64.p && nnz < INT_MAX, "device image: row pointers exceed int32 indexing");
    rp32.alloc((size_t)n + 1);
    hipLaunchKernelGGL(narrow_kernel, dim3(grid_cap(n + 1)), dim3(kT), 0, s, (long long)n + 1, rp64.p, rp32.p);
    HIP_CHECK(hipGetLastError());
}

void DevCsr::ensure_rp64(hipStream_t s) {
    if (rp64.p) return;
    AMG_CHECK(rp32.p, "device image without row pointers");
    rp64.alloc((size_t)n + 1);
    hipLaunchKernelGGL(widen_kernel, dim3(grid_cap(n + 1)), dim3(kT), 0, s, (long long)n + 1, rp32.p, rp64.p);
    HIP_CHECK(hipGetLastError());
}

void DevCsr::ensure_col32(hipStream_t s) {
    if (col32.p) return;
    AMG_CHECK(col64.p && ncols < INT_MAX, "device image: columns exceed int32 indexing");
    col32.alloc((size_t)std::max<int64_t>(nnz, 1));
    if (nnz)
        hipLaunchKernelGGL(narrow_kernel, dim3(grid_cap(nnz)), dim3(kT), 0, s, (long long)nnz, col64.p, col32.p);
    HIP_CHECK(hipGetLastError());
}

void DevCsr::ensure_col64(hipStream_t s) {
    if (col64.p) return;
    AMG_CHECK(col32.p, "device image without columns");
    col64.alloc((size_t)std::max<int64_t>(nnz, 1));
    if (nnz)
        hipLaunchKernelGGL(widen_kernel, dim3(grid_cap(nnz)), dim3(kT), 0, s, (long long)nnz, col32.p, col64.p);
    HIP_CHECK(hipGetLastError());
}

DevCsr* SetupImages::find(const HostCSR& M) {
    for (auto& kv : e)
        if (kv.first == M.rp.data() && kv.second->n == M.nrows() && kv.second->nnz == M.nnz()) return kv.second.get();
    return nullptr;
}

DevCsr& SetupImages::get(const HostCSR& M) {
    if (DevCsr* d = find(M)) return *d;
    static_assert(sizeof(long long) == sizeof(int64_t), "int64 columns");
    std::unique_ptr<DevCsr> d(new DevCsr());
    d->rp64.upload(reinterpret_cast<const long long*>(M.rp.data()), M.rp.size());
    if (M.nnz()) {
        d->col64.upload(reinterpret_cast<const long long*>(M.col.data()), (size_t)M.nnz());
        d->val.upload(M.val.data(), (size_t)M.nnz());
    } else {
        d->col64.alloc(1);
        d->val.alloc(1);
    }
    DevCsr& r = *d;
    put(M, std::move(d));
    return r;
}

void SetupImages::put(const HostCSR& M, std::unique_ptr<DevCsr> d) {
    d->n = M.nrows();
    d->nnz = M.nnz();
    d->ncols = M.n_global_cols;
    for (auto& kv : e)
        if (kv.first == M.rp.data()) {
            kv.second = std::move(d);
            return;
        }
    e.emplace_back(M.rp.data(), std::move(d));
}

void SetupImages::keep_only(const HostCSR& M) {
    std::vector<std::pair<const int64_t*, std::unique_ptr<DevCsr>>> keep;
    for (auto& kv : e)
        if (kv.first == M.rp.data()) keep.push_back(std::move(kv));
    e.swap(keep);
}

namespace {

// coarse drop tolerance on the device (one rank: global column = local row).  d_i = the row's
// stored diagonal (first match, 0.0 without one: then nothing of the row is dropped)
__global__ void sp_diag_kernel(long long n, const long long* __restrict__ rp, const long long* __restrict__ col,
                               const double* __restrict__ val, double* __restrict__ d) {
    for (long long i = (long long)blockIdx.x * kT + threadIdx.x; i < n; i += (long long)gridDim.x * kT) {
        double v = 0.0;
        for (long long k = rp[i]; k < rp[i + 1]; ++k)
            if (col[k] == i) {
                v = val[k];
                break;
            }
        d[i] = v;
    }
}

__device__ __forceinline__ bool sp_dropped(long long i, long long j, double v, const double* d, double tau) {
    return j != i && fabs(v) < tau * sqrt(fabs(d[i] * d[j]));
}

// FILL = false: kept entries per row; true: the kept entries in row order, the diagonal's value
// a_ii + the dropped entries of the row (row order) -- host sparsify's loop
template <bool FILL>
__global__ void sp_rows_kernel(long long n, const long long* __restrict__ rp, const long long* __restrict__ col,
                               const double* __restrict__ val, const double* __restrict__ d, double tau,
                               int* __restrict__ cnt, const int* __restrict__ orp, long long* __restrict__ ocol,
                               double* __restrict__ oval) {
    for (long long i = (long long)blockIdx.x * kT + threadIdx.x; i < n; i += (long long)gridDim.x * kT) {
        if (!FILL) {
            int c = 0;
            for (long long k = rp[i]; k < rp[i + 1]; ++k) c += sp_dropped(i, col[k], val[k], d, tau) ? 0 : 1;
            cnt[i] = c;
            continue;
        }
        double f = d[i];
        for (long long k = rp[i]; k < rp[i + 1]; ++k)
            if (sp_dropped(i, col[k], val[k], d, tau)) f += val[k];
        long long o = orp[i];
        for (long long k = rp[i]; k < rp[i + 1]; ++k) {
            const long long j = col[k];
            if (sp_dropped(i, j, val[k], d, tau)) continue;
            ocol[o] = j;
            oval[o] = j == i ? f : val[k];
            ++o;
        }
    }
}

std::vector<int32_t> download_ints(hipStream_t s, const int* p, int64_t n);

}  // namespace

HostCSR sparsify_device(Context& ctx, const HostComm& comm, const HostCSR& A, double tau, SetupImages* imgs) {
    DevCsr* D = imgs && comm.nranks == 1 ? imgs->find(A) : nullptr;
    if (!D || A.nrows() >= INT_MAX || A.nnz() >= INT_MAX) return sparsify(comm, A, tau);  // int32 scan
    hipStream_t s = ctx.stream;
    D->ensure_rp64(s);
    D->ensure_col64(s);
    const int64_t n = A.nrows();
    DevBuf<double> d;
    DevBuf<int> cnt, orp;
    DevBuf<char> tmp;
    d.alloc((size_t)std::max<int64_t>(n, 1));
    cnt.alloc((size_t)n + 1);
    orp.alloc((size_t)n + 1);
    HIP_CHECK(hipMemsetAsync(cnt.p, 0, sizeof(int) * cnt.n, s));
    if (n) {
        hipLaunchKernelGGL(sp_diag_kernel, dim3(grid_cap(n)), dim3(kT), 0, s, (long long)n, D->rp64.p, D->col64.p,
                           D->val.p, d.p);
        hipLaunchKernelGGL(sp_rows_kernel<false>, dim3(grid_cap(n)), dim3(kT), 0, s, (long long)n, D->rp64.p,
                           D->col64.p, D->val.p, d.p, tau, cnt.p, nullptr, nullptr, nullptr);
        HIP_CHECK(hipGetLastError());
    }
    const int64_t nnz = exclusive_scan(s, cnt.p, orp.p, (int)n, tmp);
    std::unique_ptr<DevCsr> B(new DevCsr());
    B->rp32 = std::move(orp);
    B->col64.alloc((size_t)std::max<int64_t>(nnz, 1));
    B->val.alloc((size_t)std::max<int64_t>(nnz, 1));
    if (n)
        hipLaunchKernelGGL(sp_rows_kernel<true>, dim3(grid_cap(n)), dim3(kT), 0, s, (long long)n, D->rp64.p, D->col64.p,
                           D->val.p, d.p, tau, nullptr, B->rp32.p, B->col64.p, B->val.p);
    HIP_CHECK(hipGetLastError());
    HostCSR out;
    out.n_global_rows = A.n_global_rows;
    out.n_global_cols = A.n_global_cols;
    out.row_starts = A.row_starts;
    out.col_starts = A.col_starts;
    std::vector<int> hrp = download_ints(s, B->rp32.p, n + 1);
    out.rp.assign(hrp.begin(), hrp.end());
    out.col.resize((size_t)nnz);
    out.val.resize((size_t)nnz);
    static_assert(sizeof(long long) == sizeof(int64_t), "int64 columns");
    copy_to_host(out.col.data(), B->col64.p, sizeof(long long) * nnz, s);
    copy_to_host(out.val.data(), B->val.p, sizeof(double) * nnz, nullptr);
    imgs->put(out, std::move(B));
    return out;
}

namespace {

// the level operator on the device: this rank's rows, global column ids (int32)
struct DevLevel {
    DevBuf<int> rp, col;
    DevBuf<double> val;
    int n = 0, lo = 0;
    DCsr view() const { return DCsr{rp.p, col.p, val.p, n, lo}; }
};

void upload_level(const HostComm& comm, const HostCSR& A, DevLevel& D) {
    const int64_t n = A.nrows(), nnz = A.nnz();
    AMG_CHECK(n < INT_MAX && nnz < INT_MAX && A.n_global_cols < INT_MAX,
              "device setup: level exceeds int32 indexing");
    std::vector<int> rp(n + 1), col((size_t)std::max<int64_t>(nnz, 1));
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i <= n; ++i) rp[i] = (int)A.rp[i];
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < nnz; ++k) col[k] = (int)A.col[k];
    D.n = (int)n;
    D.lo = (int)A.row_starts[comm.rank];
    D.rp.upload(rp.data(), rp.size());
    D.col.upload(col.data(), col.size());
    if (nnz) D.val.upload(A.val.data(), (size_t)nnz);
    else D.val.alloc(1);
}

struct DevS {  // strength graph / SA's filtered operator (this rank's rows, global column ids)
    DevBuf<int> rp, col;
    DevBuf<double> val;
    int n = 0, lo = 0;
    int64_t nnz = 0;
    DCsr view() const { return DCsr{rp.p, col.p, val.p, n, lo}; }
};

template <class CountK, class FillK>
void build_strength(hipStream_t s, int n, int lo, DevS& S, DevBuf<char>& tmp, CountK count, FillK fill) {
    DevBuf<int> cnt;
    cnt.alloc((size_t)n + 1);
    HIP_CHECK(hipMemsetAsync(cnt.p, 0, sizeof(int) * cnt.n, s));
    count(cnt.p);
    S.rp.alloc((size_t)n + 1);
    const int64_t nnz = exclusive_scan(s, cnt.p, S.rp.p, n, tmp);
    S.nnz = nnz;
    S.col.alloc((size_t)std::max<int64_t>(nnz, 1));
    S.val.alloc((size_t)std::max<int64_t>(nnz, 1));
    S.n = n;
    S.lo = lo;
    fill(S.rp.p, S.col.p, S.val.p);
    HIP_CHECK(hipGetLastError());
}

std::vector<int32_t> download_ints(hipStream_t s, const int* p, int64_t n) {
    std::vector<int32_t> h((size_t)n);
    copy_to_host(h.data(), p, sizeof(int) * n, s);
    return h;
}

// A halo on the device: the sorted global ids (Dist lookups), the local send indices, and
// forward(): pack on the device, the setup exchange on the host, the halo values uploaded
struct DevHalo {
    const HaloPlan* plan = nullptr;
    DevBuf<int> gid, sidx;
    void build(const HaloPlan& p) {
        plan = &p;
        std::vector<int> g(p.halo_gid.begin(), p.halo_gid.end()), si(p.send_idx.begin(), p.send_idx.end());
        gid.upload(g.data(), g.size());
        sidx.upload(si.data(), si.size());
    }
    Dist dist(int lo, int n) const { return Dist{lo, n, gid.p, (int)plan->n_halo()}; }
    template <class T>
    void forward(hipStream_t s, const HostComm& comm, const T* local, DevBuf<T>& halo) const {
        const HaloPlan& p = *plan;
        const int ns = (int)p.send_idx.size();
        DevBuf<T> packed;
        packed.alloc((size_t)std::max(ns, 1));
        if (ns) hipLaunchKernelGGL(pack_kernel_t<T>, dim3(grid1(ns)), dim3(kT), 0, s, ns, sidx.p, local, packed.p);
        std::vector<T> sbuf((size_t)ns), rbuf((size_t)p.n_halo());
        if (ns) HIP_CHECK(hipMemcpyAsync(sbuf.data(), packed.p, sizeof(T) * ns, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        std::vector<int64_t> sb(comm.nranks, 0), rb(comm.nranks, 0);
        for (size_t q = 0; q < p.send_procs.size(); ++q)
            sb[p.send_procs[q]] = (p.send_ptr[q + 1] - p.send_ptr[q]) * (int64_t)sizeof(T);
        for (size_t q = 0; q < p.recv_procs.size(); ++q)
            rb[p.recv_procs[q]] = (p.recv_ptr[q + 1] - p.recv_ptr[q]) * (int64_t)sizeof(T);
        comm.alltoallv(sbuf.data(), sb, rbuf.data(), rb);
        if (halo.n < rbuf.size() || halo.n == 0) halo.alloc(std::max<size_t>(rbuf.size(), 1));
        if (!rbuf.empty())
            HIP_CHECK(hipMemcpyAsync(halo.p, rbuf.data(), sizeof(T) * rbuf.size(), hipMemcpyHostToDevice, s));
        HIP_CHECK(hipStreamSynchronize(s));
    }
};

}  // namespace

// One level of the setup on the device: P and the integer split (C/F marker for RS-family
// coarsening, aggregate id for SA), on any number of ranks.  Each rank works on its rows
// with global column ids; the states of other ranks' points arrive through halo forwards
// (pack on the device, the setup exchange on the host) -- exactly the synchronous rounds of
// host_setup.cpp pmis_split / interp_classical / mis2_aggregate / sa_prolongator, so the
// hierarchy is bit-identical to the host path's at every rank count.  Returns false for
// Ruge-Stueben (the serial first pass stays on the host).
bool level_setup_device(Context& ctx, const HostComm& comm, const HostCSR& A, const amg_options& opt,
                        int level, HostCSR& P, std::vector<int32_t>& split, SetupImages* imgs) {
    // Ruge-Stueben (serial first pass) and extended+i (one rank, host): the host path
    if (opt.coarsen == AMG_COARSEN_RS) return false;
    if (opt.coarsen == AMG_COARSEN_PMIS && opt.interp == AMG_INTERP_EXT_I) return false;
    hipStream_t s = ctx.stream;
    const int n = (int)A.nrows();
    if (comm.nranks == 1 && n == 0) return false;
    PhaseTimer tm(comm);
    // A on the device: the setup's image (one rank: uploaded once, or left there by the
    // previous level's Galerkin product), else uploaded for this level
    DevLevel D;
    DevCsr* DA = imgs ? &imgs->get(A) : nullptr;
    if (DA) {
        AMG_CHECK(n < INT_MAX && A.n_global_cols < INT_MAX, "device setup: level exceeds int32 indexing");
        DA->ensure_rp32(s);
        DA->ensure_col32(s);
    } else {
        upload_level(comm, A, D);
    }
    const int lo = (int)A.row_starts[comm.rank];
    DevBuf<char> tmp;
    DevS S;
    const DCsr Av = DA ? DCsr{DA->rp32.p, DA->col32.p, DA->val.p, n, lo} : D.view();
    if (opt.coarsen == AMG_COARSEN_PMIS) {
        const double theta = opt.strong_threshold;
        build_strength(
            s, n, lo, S, tmp,
            [&](int* cnt) {
                if (n)
                    hipLaunchKernelGGL(strength_classical_kernel<false>, dim3(grid1(n)), dim3(kT), 0, s, Av, theta,
                                       cnt, nullptr, nullptr, nullptr);
            },
            [&](const int* srp, int* scol, double* sval) {
                if (n)
                    hipLaunchKernelGGL(strength_classical_kernel<true>, dim3(grid1(n)), dim3(kT), 0, s, Av, theta,
                                       nullptr, srp, scol, sval);
            });
        tm.lap("  device strength");
        const DCsr Sv = S.view();
        // |S^T_i| and the S^T adjacency of the local-local part
        DevBuf<int> tcnt, trp, tcol, cursor;
        tcnt.alloc((size_t)n + 1);
        HIP_CHECK(hipMemsetAsync(tcnt.p, 0, sizeof(int) * tcnt.n, s));
        if (n) hipLaunchKernelGGL(col_count_kernel, dim3(grid1(n)), dim3(kT), 0, s, Sv, tcnt.p);
        trp.alloc((size_t)n + 1);
        const int64_t tnnz = exclusive_scan(s, tcnt.p, trp.p, n, tmp);
        tcol.alloc((size_t)std::max<int64_t>(tnnz, 1));
        cursor.alloc((size_t)n + 1);
        HIP_CHECK(hipMemcpyAsync(cursor.p, trp.p, sizeof(int) * (n + 1), hipMemcpyDeviceToDevice, s));
        if (n) hipLaunchKernelGGL(transpose_fill_kernel, dim3(grid1(n)), dim3(kT), 0, s, Sv, cursor.p, tcol.p);
        // several ranks: off-rank dependents (pairs (i, j), j on another rank depends on local
        // i) and the halo of the neighbourhoods S_i u S^T_i, as pmis_split builds them
        HaloPlan hplan;
        DevHalo H;
        DevBuf<int> erp, ecol;
        if (comm.nranks > 1) {
            DevBuf<int> ocnt, orp, opc, opj;
            ocnt.alloc((size_t)n + 1);
            HIP_CHECK(hipMemsetAsync(ocnt.p, 0, sizeof(int) * ocnt.n, s));
            if (n)
                hipLaunchKernelGGL(offrank_kernel<false>, dim3(grid1(n)), dim3(kT), 0, s, Sv, ocnt.p, nullptr,
                                   nullptr, nullptr);
            orp.alloc((size_t)n + 1);
            const int64_t no = exclusive_scan(s, ocnt.p, orp.p, n, tmp);
            opc.alloc((size_t)std::max<int64_t>(no, 1));
            opj.alloc((size_t)std::max<int64_t>(no, 1));
            if (n)
                hipLaunchKernelGGL(offrank_kernel<true>, dim3(grid1(n)), dim3(kT), 0, s, Sv, nullptr, orp.p, opc.p,
                                   opj.p);
            const std::vector<int32_t> pc = download_ints(s, opc.p, no), pj = download_ints(s, opj.p, no);
            std::vector<std::vector<int64_t>> sendp(comm.nranks);
            std::vector<int64_t> need;
            for (int64_t t = 0; t < no; ++t) {
                const int o = owner_of(A.col_starts, pc[t]);
                sendp[o].push_back(pc[t]);
                sendp[o].push_back(pj[t]);
                need.push_back(pc[t]);
            }
            const auto gotp = comm.exchange(sendp);
            std::vector<int> ec((size_t)n + 1, 0);
            for (int r = 0; r < comm.nranks; ++r)
                for (size_t t = 0; t < gotp[r].size(); t += 2) ++ec[gotp[r][t] - lo + 1];
            for (int i = 0; i < n; ++i) ec[i + 1] += ec[i];
            std::vector<int> el((size_t)std::max(ec[n], 1)), pos(ec.begin(), ec.end() - 1);
            for (int r = 0; r < comm.nranks; ++r)
                for (size_t t = 0; t < gotp[r].size(); t += 2) {
                    el[pos[gotp[r][t] - lo]++] = (int)gotp[r][t + 1];
                    need.push_back(gotp[r][t + 1]);
                }
            erp.upload(ec.data(), ec.size());
            ecol.upload(el.data(), el.size());
            hplan = build_halo_plan(comm, A.col_starts, std::move(need));
        }
        H.build(hplan);
        const Dist Dn = H.dist(lo, n);
        DevBuf<unsigned long long> key, hkey, nu;
        DevBuf<int> cf, hcf;
        DevBuf<unsigned char> newc;
        key.alloc((size_t)std::max(n, 1));
        cf.alloc((size_t)std::max(n, 1));
        newc.alloc((size_t)std::max(n, 1));
        nu.alloc(1);
        hkey.alloc(1);
        hcf.alloc(1);
        if (n)
            hipLaunchKernelGGL(pmis_init_kernel, dim3(grid1(n)), dim3(kT), 0, s, n, lo, tcnt.p,
                               comm.nranks > 1 ? erp.p : nullptr, (unsigned long long)(opt.seed + (uint64_t)level),
                               key.p, cf.p);
        HIP_CHECK(hipGetLastError());
        const bool dist = comm.nranks > 1;
        if (dist) H.forward(s, comm, key.p, hkey);
        for (int round = 0;; ++round) {
            AMG_CHECK(round <= A.n_global_rows, "PMIS did not terminate");
            if (dist) H.forward(s, comm, cf.p, hcf);
            if (n) {
                hipLaunchKernelGGL(pmis_select_kernel, dim3(grid1(n)), dim3(kT), 0, s, Sv, Dn, trp.p, tcol.p,
                                   dist ? erp.p : nullptr, dist ? ecol.p : nullptr, key.p, hkey.p, cf.p, hcf.p,
                                   newc.p);
                hipLaunchKernelGGL(pmis_apply_kernel, dim3(grid1(n)), dim3(kT), 0, s, n, newc.p, cf.p);
            }
            if (dist) H.forward(s, comm, cf.p, hcf);
            HIP_CHECK(hipMemsetAsync(nu.p, 0, sizeof(unsigned long long), s));
            if (n) hipLaunchKernelGGL(pmis_fpass_kernel, dim3(grid1(n)), dim3(kT), 0, s, Sv, Dn, cf.p, hcf.p, nu.p);
            HIP_CHECK(hipGetLastError());
            unsigned long long left = 0;
            HIP_CHECK(hipMemcpyAsync(&left, nu.p, sizeof(left), hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
            const int64_t all = dist ? comm.allreduce_sum((int64_t)left) : (int64_t)left;
            if (all == 0) break;
        }
        tm.lap("  device PMIS");
        // coarse numbering: C points in row order, ranks in order
        split = download_ints(s, cf.p, n);
        int64_t ncl = 0;
        for (int32_t v : split) ncl += v == ST_C;
        std::vector<int64_t> cstarts(comm.nranks + 1, 0);
        {
            const std::vector<int64_t> counts = comm.allgather(ncl);
            for (int r = 0; r < comm.nranks; ++r) cstarts[r + 1] = cstarts[r] + counts[r];
        }
        AMG_CHECK(cstarts[comm.nranks] < INT_MAX, "device setup: coarse level exceeds int32 indexing");
        std::vector<int> hcmap((size_t)std::max(n, 1), -1);
        for (int i = 0, c = (int)cstarts[comm.rank]; i < n; ++i)
            if (split[i] == ST_C) hcmap[i] = c++;
        DevBuf<int> cmap;
        cmap.upload(hcmap.data(), hcmap.size());
        // A's halo: states and coarse ids of the off-rank columns, and their ghost rows
        HaloPlan aplan;
        GhostRows G;
        if (dist) {
            aplan = halo_plan_for_cols(comm, A);
            G = fetch_rows(comm, aplan, A);
        }
        DevHalo AH;
        AH.build(aplan);
        DevBuf<int> acf, acmap, grp, gcol;
        DevBuf<double> gval;
        acf.alloc(1);
        acmap.alloc(1);
        if (dist) {
            std::vector<int32_t> hcfa(aplan.n_halo());
            std::vector<int64_t> cm64(hcmap.begin(), hcmap.begin() + n), hcm64(aplan.n_halo());
            aplan.forward(comm, split.data(), hcfa.data());
            aplan.forward(comm, cm64.data(), hcm64.data());
            std::vector<int> hcma(hcm64.begin(), hcm64.end());
            acf.upload(hcfa.data(), hcfa.size());
            acmap.upload(hcma.data(), hcma.size());
            AMG_CHECK(G.rp.back() < INT_MAX, "device setup: ghost rows exceed int32 indexing");
            std::vector<int> gr(G.rp.begin(), G.rp.end()), gc(G.col.begin(), G.col.end());
            grp.upload(gr.data(), gr.size());
            gcol.upload(gc.data(), std::max<size_t>(gc.size(), 1));
            gval.upload(G.val.data(), std::max<size_t>(G.val.size(), 1));
        } else {
            grp.alloc(1);
            gcol.alloc(1);
            gval.alloc(1);
        }
        const ARows Ar{Av, AH.dist(lo, n), grp.p, gcol.p, gval.p};
        tm.lap("  device coarse ids + ghost rows");
        // P: count, scan, fill
        DevBuf<int> pcnt, prp, pcol;
        DevBuf<double> pval;
        pcnt.alloc((size_t)n + 1);
        HIP_CHECK(hipMemsetAsync(pcnt.p, 0, sizeof(int) * pcnt.n, s));
        // long rows (the Galerkin levels): a wave per row (interp_wave_kernel); AMG_INTERP_WAVE_NPR
        // sets the average row length from which it is taken (default 12; 0: always)
        const char* wenv = std::getenv("AMG_INTERP_WAVE_NPR");
        const int wave_npr = wenv && *wenv ? std::atoi(wenv) : 12;
        const bool wave = n > 0 && A.nnz() >= (int64_t)wave_npr * n;
        const dim3 wgrid((unsigned)((n + kIwWaves - 1) / kIwWaves)), wblk(64 * kIwWaves);
        if (n && wave)
            hipLaunchKernelGGL(interp_wave_kernel<false>, wgrid, wblk, 0, s, Ar, Sv, cf.p, acf.p, cmap.p, acmap.p,
                               pcnt.p, nullptr, nullptr, nullptr);
        else if (n)
            hipLaunchKernelGGL(interp_kernel<false>, dim3(grid1(n)), dim3(kT), 0, s, Ar, Sv, cf.p, acf.p, cmap.p,
                               acmap.p, pcnt.p, nullptr, nullptr, nullptr);
        prp.alloc((size_t)n + 1);
        const int64_t pnnz = exclusive_scan(s, pcnt.p, prp.p, n, tmp);
        pcol.alloc((size_t)std::max<int64_t>(pnnz, 1));
        pval.alloc((size_t)std::max<int64_t>(pnnz, 1));
        if (n && wave)
            hipLaunchKernelGGL(interp_wave_kernel<true>, wgrid, wblk, 0, s, Ar, Sv, cf.p, acf.p, cmap.p, acmap.p,
                               nullptr, prp.p, pcol.p, pval.p);
        else if (n)
            hipLaunchKernelGGL(interp_kernel<true>, dim3(grid1(n)), dim3(kT), 0, s, Ar, Sv, cf.p, acf.p, cmap.p,
                               acmap.p, nullptr, prp.p, pcol.p, pval.p);
        HIP_CHECK(hipGetLastError());
        std::vector<int> hrp = download_ints(s, prp.p, (int64_t)n + 1), hcol = download_ints(s, pcol.p, pnnz);
        P = HostCSR();
        P.n_global_rows = A.n_global_rows;
        P.n_global_cols = cstarts[comm.nranks];
        P.row_starts = A.row_starts;
        P.col_starts = cstarts;
        P.rp.assign(hrp.begin(), hrp.end());
        P.col.assign(hcol.begin(), hcol.end());
        P.val.resize((size_t)pnnz);
        copy_to_host(P.val.data(), pval.p, sizeof(double) * pnnz, s);
        if (imgs) {  // P where it was computed, for the transpose and the Galerkin product
            std::unique_ptr<DevCsr> d(new DevCsr());
            d->rp32 = std::move(prp);
            d->col32 = std::move(pcol);
            d->val = std::move(pval);
            imgs->put(P, std::move(d));
        }
        tm.lap("  device interpolation");
        return true;
    }
    // smoothed aggregation (host_setup.cpp strength_symmetric, mis2_aggregate, sa_prolongator)
    AMG_CHECK(opt.coarsen == AMG_COARSEN_SA, "unknown coarsening");
    const bool dist = comm.nranks > 1;
    const double theta = sa_theta(opt.strong_threshold, level);
    // A's halo: a_jj of other ranks' columns, then the MIS(2) tuples and aggregate ids of the
    // strong neighbours (S is a subset of A's pattern)
    HaloPlan aplan;
    if (dist) aplan = halo_plan_for_cols(comm, A);
    DevHalo AH;
    AH.build(aplan);
    const Dist Da = AH.dist(lo, n);
    DevBuf<double> d, hd;
    d.alloc((size_t)std::max(n, 1));
    hd.alloc(1);
    if (n) hipLaunchKernelGGL(diagonal_kernel, dim3(grid1(n)), dim3(kT), 0, s, Av, d.p);
    if (dist) AH.forward(s, comm, d.p, hd);
    build_strength(
        s, n, lo, S, tmp,
        [&](int* cnt) {
            if (n)
                hipLaunchKernelGGL(strength_symmetric_kernel<false>, dim3(grid1(n)), dim3(kT), 0, s, Av, Da, d.p,
                                   hd.p, theta, cnt, nullptr, nullptr, nullptr);
        },
        [&](const int* srp, int* scol, double* sval) {
            if (n)
                hipLaunchKernelGGL(strength_symmetric_kernel<true>, dim3(grid1(n)), dim3(kT), 0, s, Av, Da, d.p,
                                   hd.p, theta, nullptr, srp, scol, sval);
        });
    tm.lap("  device strength");
    const DCsr Sv = S.view();
    std::vector<unsigned> hs((size_t)std::max(n, 1));
    for (int i = 0; i < n; ++i) hs[i] = hash32(lo + i, opt.seed + (uint64_t)level);
    DevBuf<unsigned> dhs;
    dhs.upload(hs.data(), hs.size());
    DevBuf<int> st;
    DevBuf<unsigned long long> h0, l0, h1, l1, hh, hl, nu;
    const size_t nn = (size_t)std::max(n, 1);
    st.alloc(nn);
    h0.alloc(nn), l0.alloc(nn), h1.alloc(nn), l1.alloc(nn), nu.alloc(1), hh.alloc(1), hl.alloc(1);
    {
        std::vector<int> init(nn, M_U);
        st.upload(init.data(), init.size());
    }
    for (int round = 0;; ++round) {
        AMG_CHECK(round <= A.n_global_rows, "MIS(2) did not terminate");
        if (n) hipLaunchKernelGGL(mis2_tuple_kernel, dim3(grid1(n)), dim3(kT), 0, s, n, lo, st.p, dhs.p, h0.p, l0.p);
        for (int hop = 0; hop < 2; ++hop) {
            if (dist) {
                AH.forward(s, comm, h0.p, hh);
                AH.forward(s, comm, l0.p, hl);
            }
            if (n)
                hipLaunchKernelGGL(mis2_hop_kernel, dim3(grid1(n)), dim3(kT), 0, s, Sv, Da, h0.p, l0.p, hh.p, hl.p,
                                   h1.p, l1.p);
            std::swap(h0.p, h1.p);
            std::swap(l0.p, l1.p);
        }
        HIP_CHECK(hipMemsetAsync(nu.p, 0, sizeof(unsigned long long), s));
        if (n) hipLaunchKernelGGL(mis2_update_kernel, dim3(grid1(n)), dim3(kT), 0, s, n, lo, h0.p, l0.p, st.p, nu.p);
        HIP_CHECK(hipGetLastError());
        unsigned long long left = 0;
        HIP_CHECK(hipMemcpyAsync(&left, nu.p, sizeof(left), hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        if ((dist ? comm.allreduce_sum((int64_t)left) : (int64_t)left) == 0) break;
    }
    // roots numbered in global row order (ranks in order); aggr = a root's aggregate id, -1
    // (r5: an exclusive scan of the root flags on the device, not a host pass over the states)
    DevBuf<int> rflag, rpos;
    rflag.alloc(nn + 1);
    rpos.alloc(nn + 1);
    HIP_CHECK(hipMemsetAsync(rflag.p, 0, sizeof(int) * rflag.n, s));
    if (n) hipLaunchKernelGGL(root_flag_kernel, dim3(grid1(n)), dim3(kT), 0, s, n, st.p, rflag.p);
    const int64_t nroot = exclusive_scan(s, rflag.p, rpos.p, n, tmp);
    std::vector<int64_t> astarts(comm.nranks + 1, 0);
    {
        const std::vector<int64_t> counts = comm.allgather(nroot);
        for (int r = 0; r < comm.nranks; ++r) astarts[r + 1] = astarts[r] + counts[r];
    }
    const int64_t na = astarts[comm.nranks];
    AMG_CHECK(na < INT_MAX, "device setup: coarse level exceeds int32 indexing");
    DevBuf<int> aggr, haggr_d, a1, ha1, agg;
    aggr.alloc(nn);
    if (n)
        hipLaunchKernelGGL(root_id_kernel, dim3(grid1(n)), dim3(kT), 0, s, n, st.p, rpos.p,
                           (int)astarts[comm.rank], aggr.p);
    haggr_d.alloc(1);
    ha1.alloc(1);
    a1.alloc(nn);
    agg.alloc(nn);
    if (dist) AH.forward(s, comm, aggr.p, haggr_d);
    if (n) hipLaunchKernelGGL(mis2_pass1_kernel, dim3(grid1(n)), dim3(kT), 0, s, Sv, Da, aggr.p, haggr_d.p, a1.p);
    if (dist) AH.forward(s, comm, a1.p, ha1);
    HIP_CHECK(hipMemsetAsync(nu.p, 0, sizeof(unsigned long long), s));
    if (n)
        hipLaunchKernelGGL(mis2_pass2_kernel, dim3(grid1(n)), dim3(kT), 0, s, Sv, Da, a1.p, ha1.p, agg.p, nu.p);
    HIP_CHECK(hipGetLastError());
    unsigned long long orphans = 0;
    HIP_CHECK(hipMemcpyAsync(&orphans, nu.p, sizeof(orphans), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (orphans) throw Error(AMG_ERR_INTERNAL, "MIS(2): unaggregated node");
    split = download_ints(s, agg.p, n);
    tm.lap("  device aggregation");
    // aggregate sizes (owners count their members, members elsewhere report in), T = 1 /
    // sqrt(|aggregate|)
    const int64_t alo = astarts[comm.rank], ahi = astarts[comm.rank + 1];
    std::vector<int64_t> size((size_t)(ahi - alo), 0);
    std::vector<std::vector<int64_t>> sendc(comm.nranks);
    std::vector<int64_t> needa;
    if (!dist) {  // every aggregate is this rank's: counted in parallel (integer counts)
#pragma omp parallel for schedule(static)
        for (int i = 0; i < n; ++i) {
#pragma omp atomic
            size[split[i] - alo]++;
        }
    } else {
        for (int i = 0; i < n; ++i) {
            const int64_t a = split[i];
            if (a >= alo && a < ahi) {
                size[a - alo]++;
            } else {
                sendc[owner_of(astarts, a)].push_back(a);
                needa.push_back(a);
            }
        }
    }
    if (dist) {
        const auto got = comm.exchange(sendc);
        for (int r = 0; r < comm.nranks; ++r)
            for (int64_t a : got[r]) size[a - alo]++;
    }
    HaloPlan splan;
    std::vector<int64_t> hsize;
    if (dist) {
        splan = build_halo_plan(comm, astarts, std::move(needa));
        hsize.resize(splan.n_halo());
        splan.forward(comm, size.data(), hsize.data());
    }
    std::vector<double> tv((size_t)std::max(n, 1));
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        const int64_t a = split[i];
        const int64_t sz = (a >= alo && a < ahi) ? size[a - alo] : hsize[splan.find(a)];
        tv[i] = 1.0 / std::sqrt((double)sz);
    }
    DevBuf<double> dt, hdt;
    dt.upload(tv.data(), tv.size());
    hdt.alloc(1);
    if (dist) AH.forward(s, comm, dt.p, hdt);  // t of the halo columns (A_F T)
    tm.lap("  device tentative prolongator");
    // the filtered operator A_F (r6): the diagonal + the strong couplings, weak ones lumped
    DevS F;
    build_strength(
        s, n, lo, F, tmp,
        [&](int* cnt) {
            if (n)
                hipLaunchKernelGGL(sa_filter_kernel<false>, dim3(grid1(n)), dim3(kT), 0, s, Av, Da, d.p, hd.p, theta,
                                   cnt, nullptr, nullptr, nullptr);
        },
        [&](const int* frp, int* fcol, double* fval) {
            if (n)
                hipLaunchKernelGGL(sa_filter_kernel<true>, dim3(grid1(n)), dim3(kT), 0, s, Av, Da, d.p, hd.p, theta,
                                   nullptr, frp, fcol, fval);
        });
    const DCsr Fv = F.view();
    // rho(D^-1 A_F): power steps in the max norm (exact maxima, the same on every partition)
    double rho = 0.0;
    {
        DevBuf<double> x, y, hx;
        DevBuf<unsigned long long> mx;
        x.alloc((size_t)std::max(n, 1));
        y.alloc((size_t)std::max(n, 1));
        hx.alloc(1);
        mx.alloc(1);
        auto global_max = [&]() {
            unsigned long long bits = 0;
            HIP_CHECK(hipMemcpyAsync(&bits, mx.p, sizeof(bits), hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
            double m;
            std::memcpy(&m, &bits, sizeof(m));
            return dist ? comm.allreduce_max(m) : m;
        };
        launch_uniform(s, n, lo, opt.seed + (uint64_t)level, x.p);
        HIP_CHECK(hipMemsetAsync(mx.p, 0, sizeof(unsigned long long), s));
        if (n) hipLaunchKernelGGL(max_abs_kernel, dim3(grid1(n)), dim3(kT), 0, s, n, x.p, mx.p);
        const double m0 = global_max();
        if (m0 > 0.0 && n) hipLaunchKernelGGL(div_scalar_kernel, dim3(grid1(n)), dim3(kT), 0, s, n, x.p, m0, x.p);
        for (int it = 0; it < kSaRhoIters; ++it) {
            if (dist) AH.forward(s, comm, x.p, hx);
            HIP_CHECK(hipMemsetAsync(mx.p, 0, sizeof(unsigned long long), s));
            if (n) hipLaunchKernelGGL(sa_power_kernel, dim3(grid1(n)), dim3(kT), 0, s, Fv, Da, x.p, hx.p, d.p, y.p, mx.p);
            HIP_CHECK(hipGetLastError());
            rho = global_max();
            if (rho == 0.0) break;
            if (n) hipLaunchKernelGGL(div_scalar_kernel, dim3(grid1(n)), dim3(kT), 0, s, n, y.p, rho, x.p);
        }
    }
    const double omega = rho > 0.0 ? (4.0 / 3.0) / rho : 0.0;
    tm.lap("  device filtered operator + rho");
    // P = T - (omega / a_ii) A_F T on the device, on any number of ranks; one rank keeps it as
    // the setup's image of P (transpose, Galerkin product)
    static_assert(sizeof(long long) == sizeof(int64_t), "int64 columns");
    DevBuf<int> hagg, skey;
    DevBuf<double> sval;
    hagg.alloc(1);
    if (dist) AH.forward(s, comm, agg.p, hagg);
    const int64_t fnnz = F.nnz;
    skey.alloc((size_t)std::max<int64_t>(fnnz, 1));
    sval.alloc((size_t)std::max<int64_t>(fnnz, 1));
    DevBuf<long long> pcnt, prp, pcol;
    DevBuf<double> pval;
    pcnt.alloc((size_t)n + 1);
    HIP_CHECK(hipMemsetAsync(pcnt.p, 0, sizeof(long long) * pcnt.n, s));
    if (n)
        hipLaunchKernelGGL(sa_smooth_kernel<false>, dim3(grid1(n)), dim3(kT), 0, s, Fv, Da, agg.p, hagg.p, dt.p,
                           hdt.p, d.p, omega, skey.p, sval.p, pcnt.p, nullptr, nullptr, nullptr);
    prp.alloc((size_t)n + 1);
    const int64_t pnnz = exclusive_scan64(s, pcnt.p, prp.p, n, tmp);
    pcol.alloc((size_t)std::max<int64_t>(pnnz, 1));
    pval.alloc((size_t)std::max<int64_t>(pnnz, 1));
    if (n)
        hipLaunchKernelGGL(sa_smooth_kernel<true>, dim3(grid1(n)), dim3(kT), 0, s, Fv, Da, agg.p, hagg.p, dt.p,
                           hdt.p, d.p, omega, skey.p, sval.p, nullptr, prp.p, pcol.p, pval.p);
    HIP_CHECK(hipGetLastError());
    P = HostCSR();
    P.n_global_rows = A.n_global_rows;
    P.n_global_cols = na;
    P.row_starts = A.row_starts;
    P.col_starts = astarts;
    P.rp.resize((size_t)n + 1);
    P.col.resize((size_t)pnnz);
    P.val.resize((size_t)pnnz);
    copy_to_host(P.rp.data(), prp.p, sizeof(long long) * (n + 1), s);
    copy_to_host(P.col.data(), pcol.p, sizeof(long long) * pnnz, nullptr);
    copy_to_host(P.val.data(), pval.p, sizeof(double) * pnnz, nullptr);
    if (imgs && !dist) {  // (N ranks: the transpose and SpGEMM build their own images of P)
        std::unique_ptr<DevCsr> dp(new DevCsr());
        dp->rp64 = std::move(prp);
        dp->col64 = std::move(pcol);
        dp->val = std::move(pval);
        imgs->put(P, std::move(dp));
    }
    tm.lap("  device smoothed prolongator");
    return true;
}

namespace {

void sort_pairs_stable(hipStream_t s, const int* keys_in, int* keys_out, const int* vals_in, int* vals_out, int m,
                       int64_t key_range, DevBuf<char>& tmp) {
    int bits = 1;
    while (bits < 31 && (1ll << bits) < key_range) ++bits;
    size_t bytes = 0;
    HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, keys_in, keys_out, vals_in, vals_out, m, 0, bits, s));
    if (tmp.n < bytes) tmp.alloc(bytes);
    HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp.p, bytes, keys_in, keys_out, vals_in, vals_out, m, 0, bits, s));
}

// R = P^T on N ranks (host_comm.cpp transpose(), the same records and exchange): each rank
// sorts its entries by global column on the device (stable: fine rows stay ascending), ships
// each owner its contiguous record range (one all-to-all-v), and the owner sorts what it
// received by local row, stably -- rank order, then ascending fine row, as the host
// transpose places them.  Bit-identical to it.
bool transpose_device_dist(Context& ctx, const HostComm& comm, const HostCSR& P, HostCSR& R, SetupImages* imgs) {
    hipStream_t s = ctx.stream;
    const int64_t n = P.nrows(), nnz = P.nnz(), nc = P.n_global_cols;
    const int64_t lo = P.col_starts[comm.rank], m_rows = P.col_starts[comm.rank + 1] - lo;
    // every rank takes the same path (the exchange is collective)
    int64_t ok = n < INT_MAX && nnz < INT_MAX && nc < INT_MAX;
    for (int64_t v : comm.allgather(ok)) ok = ok && v;
    if (!ok) return false;
    static_assert(sizeof(TRec) == 24, "record layout");
    DevBuf<char> tmp;
    const int nr = comm.nranks, me = comm.rank;
    // records sorted by column: owner o's range [off[o], off[o + 1]); this rank's own range
    // stays on the device, only the others' travel through the host exchange
    std::vector<long long> off((size_t)nr + 1, 0);
    DevBuf<TRec> recs;
    std::vector<TRec> sbuf;
    if (nnz) {
        SetupImages local;
        DevCsr& dP = (imgs ? *imgs : local).get(P);
        dP.ensure_rp32(s);
        dP.ensure_col32(s);
        DevBuf<int> keys_out, idx_in, idx_out, rowof;
        DevBuf<long long> dbound, doff;
        keys_out.alloc(nnz);
        idx_in.alloc(nnz);
        idx_out.alloc(nnz);
        rowof.alloc(nnz);
        recs.alloc(nnz);
        hipLaunchKernelGGL(iota_kernel, dim3(grid1(nnz)), dim3(kT), 0, s, (int)nnz, idx_in.p);
        if (n) hipLaunchKernelGGL(expand_rows_kernel, dim3(grid1(n)), dim3(kT), 0, s, dP.rp32.p, (int)n, rowof.p);
        sort_pairs_stable(s, dP.col32.p, keys_out.p, idx_in.p, idx_out.p, (int)nnz, nc, tmp);
        hipLaunchKernelGGL(transpose_records_kernel, dim3(grid1(nnz)), dim3(kT), 0, s, (int)nnz, keys_out.p, idx_out.p,
                           rowof.p, dP.val.p, (long long)P.row_starts[me], recs.p);
        std::vector<long long> bound(P.col_starts.begin() + 1, P.col_starts.end());
        dbound.upload(bound.data(), bound.size());
        doff.alloc((size_t)nr);
        hipLaunchKernelGGL(owner_bounds_kernel, dim3(grid1(nr)), dim3(kT), 0, s, (int)nnz, keys_out.p, nr, dbound.p,
                           doff.p);
        HIP_CHECK(hipGetLastError());
        copy_to_host(off.data() + 1, doff.p, sizeof(long long) * nr, s);
        off[nr] = nnz;
        const int64_t nsend = nnz - (off[me + 1] - off[me]);
        sbuf.resize((size_t)nsend);
        copy_to_host(sbuf.data(), recs.p, sizeof(TRec) * off[me], nullptr);
        copy_to_host(sbuf.data() + off[me], recs.p + off[me + 1], sizeof(TRec) * (nnz - off[me + 1]), nullptr);
    }
    std::vector<int64_t> cnt(nr, 0), sb(nr), rb(nr);
    for (int o = 0; o < nr; ++o) cnt[o] = off[o + 1] - off[o];
    const std::vector<int64_t> rcnt = comm.alltoall_counts(cnt);
    int64_t rtot = 0, rfor = 0, before = 0;
    for (int o = 0; o < nr; ++o) {
        sb[o] = o == me ? 0 : cnt[o] * (int64_t)sizeof(TRec);
        rb[o] = o == me ? 0 : rcnt[o] * (int64_t)sizeof(TRec);
        rtot += rcnt[o];
        if (o != me) rfor += rcnt[o];
        if (o < me) before += rcnt[o];
    }
    std::vector<TRec> rbuf((size_t)rfor);
    comm.alltoallv(sbuf.data(), sb, rbuf.data(), rb);
    std::vector<TRec>().swap(sbuf);
    AMG_CHECK(rtot < INT_MAX && m_rows < INT_MAX, "device transpose: rows exceed int32 indexing");
    R = HostCSR();
    R.n_global_rows = nc;
    R.n_global_cols = P.n_global_rows;
    R.row_starts = P.col_starts;
    R.col_starts = P.row_starts;
    R.rp.assign((size_t)m_rows + 1, 0);
    R.col.resize((size_t)rtot);
    R.val.resize((size_t)rtot);
    if (rtot) {
        // received records in rank order: [ranks < me | own range (device to device) | ranks > me]
        DevBuf<TRec> drec;
        DevBuf<int> key, key_out, idx_in, idx_out, cntd, rrp;
        DevBuf<long long> rcol;
        DevBuf<double> rval;
        const int64_t own = rtot - rfor;
        drec.alloc((size_t)rtot);
        if (before) copy_to_device(drec.p, rbuf.data(), sizeof(TRec) * before);
        if (own)
            HIP_CHECK(hipMemcpyAsync(drec.p + before, recs.p + off[me], sizeof(TRec) * own, hipMemcpyDeviceToDevice, s));
        if (rfor > before)
            copy_to_device(drec.p + before + own, rbuf.data() + before, sizeof(TRec) * (rfor - before));
        std::vector<TRec>().swap(rbuf);
        HIP_CHECK(hipStreamSynchronize(s));
        recs.reset();
        key.alloc(rtot);
        key_out.alloc(rtot);
        idx_in.alloc(rtot);
        idx_out.alloc(rtot);
        hipLaunchKernelGGL(record_rows_kernel, dim3(grid1(rtot)), dim3(kT), 0, s, (int)rtot, drec.p, (long long)lo, key.p);
        hipLaunchKernelGGL(iota_kernel, dim3(grid1(rtot)), dim3(kT), 0, s, (int)rtot, idx_in.p);
        sort_pairs_stable(s, key.p, key_out.p, idx_in.p, idx_out.p, (int)rtot, m_rows, tmp);
        rcol.alloc(rtot);
        rval.alloc(rtot);
        hipLaunchKernelGGL(gather_records_kernel, dim3(grid1(rtot)), dim3(kT), 0, s, (int)rtot, idx_out.p, drec.p,
                           rcol.p, rval.p);
        cntd.alloc((size_t)m_rows + 1);
        HIP_CHECK(hipMemsetAsync(cntd.p, 0, sizeof(int) * cntd.n, s));
        hipLaunchKernelGGL(count_cols_kernel, dim3(grid1(rtot)), dim3(kT), 0, s, (int)rtot, key.p, cntd.p);
        rrp.alloc((size_t)m_rows + 1);
        exclusive_scan(s, cntd.p, rrp.p, (int)m_rows, tmp);
        HIP_CHECK(hipGetLastError());
        const std::vector<int> hrp = download_ints(s, rrp.p, m_rows + 1);
        R.rp.assign(hrp.begin(), hrp.end());
        copy_to_host(R.col.data(), rcol.p, sizeof(long long) * rtot, s);
        copy_to_host(R.val.data(), rval.p, sizeof(double) * rtot, nullptr);
        if (imgs) {  // R where it was computed, for the Galerkin product
            std::unique_ptr<DevCsr> d(new DevCsr());
            d->rp32 = std::move(rrp);
            d->col64 = std::move(rcol);
            d->val = std::move(rval);
            imgs->put(R, std::move(d));
        }
    }
    return true;
}

}  // namespace

// R = P^T on the device for one rank: stable radix sort of the entries by column keeps each
// R row in ascending fine-row order, like transpose().
bool transpose_device(Context& ctx, const HostComm& comm, const HostCSR& P, HostCSR& R, SetupImages* imgs) {
    if (comm.nranks != 1) return transpose_device_dist(ctx, comm, P, R, imgs);
    hipStream_t s = ctx.stream;
    const int64_t n = P.nrows(), nnz = P.nnz(), nc = P.n_global_cols;
    if (nnz == 0 || n >= INT_MAX || nnz >= INT_MAX || nc >= INT_MAX) return false;
    DevBuf<int> drp_up, dcol_up, keys_out, idx_in, idx_out, rowof, cnt, rrp;
    DevBuf<double> dval_up;
    DevBuf<long long> rcol;
    DevBuf<double> rval;
    DevBuf<char> tmp;
    const int *drp_p, *dcol_p;
    const double* dval_p;
    if (imgs) {  // P's image (left on the device by the level setup)
        DevCsr& dP = imgs->get(P);
        dP.ensure_rp32(s);
        dP.ensure_col32(s);
        drp_p = dP.rp32.p, dcol_p = dP.col32.p, dval_p = dP.val.p;
    } else {
        std::vector<int> rp(n + 1), col(nnz);
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i <= n; ++i) rp[i] = (int)P.rp[i];
#pragma omp parallel for schedule(static)
        for (int64_t k = 0; k < nnz; ++k) col[k] = (int)P.col[k];
        drp_up.upload(rp.data(), rp.size());
        dcol_up.upload(col.data(), col.size());
        dval_up.upload(P.val.data(), P.val.size());
        drp_p = drp_up.p, dcol_p = dcol_up.p, dval_p = dval_up.p;
    }
    keys_out.alloc(nnz);
    idx_in.alloc(nnz);
    idx_out.alloc(nnz);
    rowof.alloc(nnz);
    hipLaunchKernelGGL(iota_kernel, dim3(grid1(nnz)), dim3(kT), 0, s, (int)nnz, idx_in.p);
    hipLaunchKernelGGL(expand_rows_kernel, dim3(grid1(n)), dim3(kT), 0, s, drp_p, (int)n, rowof.p);
    int bits = 1;
    while (bits < 31 && (1ll << bits) < nc) ++bits;
    size_t bytes = 0;
    HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, dcol_p, keys_out.p, idx_in.p, idx_out.p,
                                                 (int)nnz, 0, bits, s));
    tmp.alloc(bytes);
    HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp.p, bytes, dcol_p, keys_out.p, idx_in.p, idx_out.p,
                                                 (int)nnz, 0, bits, s));
    rcol.alloc(nnz);
    rval.alloc(nnz);
    hipLaunchKernelGGL(gather_transpose_kernel, dim3(grid1(nnz)), dim3(kT), 0, s, (int)nnz, idx_out.p,
                       rowof.p, dval_p, rcol.p, rval.p);
    cnt.alloc((size_t)nc + 1);
    HIP_CHECK(hipMemsetAsync(cnt.p, 0, sizeof(int) * cnt.n, s));
    hipLaunchKernelGGL(count_cols_kernel, dim3(grid1(nnz)), dim3(kT), 0, s, (int)nnz, dcol_p, cnt.p);
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
    static_assert(sizeof(long long) == sizeof(int64_t), "int64 columns");
    copy_to_host(R.col.data(), rcol.p, sizeof(long long) * nnz, s);
    copy_to_host(R.val.data(), rval.p, sizeof(double) * nnz, nullptr);
    if (imgs) {  // R where it was computed, for the Galerkin product
        std::unique_ptr<DevCsr> d(new DevCsr());
        d->rp32 = std::move(rrp);
        d->col64 = std::move(rcol);
        d->val = std::move(rval);
        imgs->put(R, std::move(d));
    }
    return true;
}

}  // namespace amg
