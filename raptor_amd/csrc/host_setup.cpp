// host_setup.cpp -- AMG setup on the host: strength, Ruge-Stueben / PMIS splitting,
// classical interpolation, MIS(2) aggregation, smoothed prolongator, coarse inverse.
// SURVEY.md 8a rows a8, a9 (integer results bit-exact against the oracle at any rank
// count; DESIGN.md section 3 fixes every tie-break and summation order).
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <queue>

#include "host.hpp"

namespace amg {

enum { ST_U = -1, ST_F = 0, ST_C = 1 };

std::vector<double> diagonal(const HostComm& comm, const HostCSR& A) {
    int64_t n = A.nrows(), lo = A.row_starts[comm.rank];
    std::vector<double> d(n, 0.0);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i)
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k)
            if (A.col[k] == lo + i) {
                d[i] = A.val[k];
                break;
            }
    return d;
}

static HostCSR same_shape(const HostCSR& A) {
    HostCSR S;
    S.n_global_rows = A.n_global_rows;
    S.n_global_cols = A.n_global_cols;
    S.row_starts = A.row_starts;
    S.col_starts = A.col_starts;
    return S;
}

// filter rows of A by a per-entry predicate, keeping order
template <class F>
static HostCSR filter_rows(const HostCSR& A, F keep) {
    HostCSR S = same_shape(A);
    int64_t n = A.nrows();
    std::vector<uint8_t> flag(A.nnz());
    std::vector<int64_t> len(n);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        int64_t c = 0;
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) c += (flag[k] = keep(i, k) ? 1 : 0);
        len[i] = c;
    }
    S.rp.assign(n + 1, 0);
    for (int64_t i = 0; i < n; ++i) S.rp[i + 1] = S.rp[i] + len[i];
    S.col.resize(S.rp[n]);
    S.val.resize(S.rp[n]);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        int64_t q = S.rp[i];
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k)
            if (flag[k]) S.col[q] = A.col[k], S.val[q++] = A.val[k];
    }
    return S;
}

// classical: m_i = max_{j != i} (-a_ij); none if m_i <= 0; strong iff -a_ij >= theta*m_i
HostCSR strength_classical(const HostComm& comm, const HostCSR& A, double theta) {
    int64_t n = A.nrows(), lo = A.row_starts[comm.rank];
    std::vector<double> thr(n);
    std::vector<uint8_t> has(n);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        double mx = 0.0;
        bool any = false;
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
            if (A.col[k] == lo + i) continue;
            double v = -A.val[k];
            if (!any || v > mx) mx = v;
            any = true;
        }
        has[i] = any && mx > 0.0;
        thr[i] = theta * mx;
    }
    return filter_rows(A, [&](int64_t i, int64_t k) {
        return has[i] && A.col[k] != lo + i && -A.val[k] >= thr[i];
    });
}

// SA, signed (r6): -a_ij >= theta * sqrt(|a_ii * a_jj|), j != i (sa_strong)
HostCSR strength_symmetric(const HostComm& comm, const HostCSR& A, double theta) {
    int64_t lo = A.row_starts[comm.rank], hi = A.row_starts[comm.rank + 1];
    std::vector<double> d = diagonal(comm, A);
    HaloPlan plan = halo_plan_for_cols(comm, A);
    std::vector<double> hd(plan.n_halo());
    plan.forward(comm, d.data(), hd.data());
    return filter_rows(A, [&](int64_t i, int64_t k) {
        int64_t j = A.col[k];
        if (j == lo + i) return false;
        double dj = (j >= lo && j < hi) ? d[j - lo] : hd[plan.find(j)];
        return sa_strong(A.val[k], d[i], dj, theta);
    });
}

// SA's filtered operator (r6; oracle orc_sa_filter): the diagonal and the strong off-diagonals
// in row order; the diagonal value becomes a_ii + the weak off-diagonals (row order)
HostCSR sa_filter(const HostComm& comm, const HostCSR& A, double theta) {
    int64_t lo = A.row_starts[comm.rank], hi = A.row_starts[comm.rank + 1];
    std::vector<double> d = diagonal(comm, A);
    HaloPlan plan = halo_plan_for_cols(comm, A);
    std::vector<double> hd(plan.n_halo());
    plan.forward(comm, d.data(), hd.data());
    auto strong = [&](int64_t i, int64_t k) {
        int64_t j = A.col[k];
        double dj = (j >= lo && j < hi) ? d[j - lo] : hd[plan.find(j)];
        return sa_strong(A.val[k], d[i], dj, theta);
    };
    HostCSR F = filter_rows(A, [&](int64_t i, int64_t k) { return A.col[k] == lo + i || strong(i, k); });
    const int64_t n = A.nrows();
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        double f = d[i];
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k)
            if (A.col[k] != lo + i && !strong(i, k)) f += A.val[k];
        for (int64_t k = F.rp[i]; k < F.rp[i + 1]; ++k)
            if (F.col[k] == lo + i) F.val[k] = f;
    }
    return F;
}

// coarse-operator drop tolerance (r6 option; oracle orc_sparsify): the same loop as sa_filter
// with |a_ij| < tau sqrt(|a_ii a_jj|) for "dropped".  A row without a stored diagonal has
// d_i = 0, so nothing of it is dropped (the oracle leaves such rows as they are).
HostCSR sparsify(const HostComm& comm, const HostCSR& A, double tau) {
    int64_t lo = A.row_starts[comm.rank], hi = A.row_starts[comm.rank + 1];
    std::vector<double> d = diagonal(comm, A);
    HaloPlan plan = halo_plan_for_cols(comm, A);
    std::vector<double> hd(plan.n_halo());
    plan.forward(comm, d.data(), hd.data());
    auto dropped = [&](int64_t i, int64_t k) {
        int64_t j = A.col[k];
        if (j == lo + i) return false;
        double dj = (j >= lo && j < hi) ? d[j - lo] : hd[plan.find(j)];
        return std::fabs(A.val[k]) < tau * std::sqrt(std::fabs(d[i] * dj));
    };
    HostCSR B = filter_rows(A, [&](int64_t i, int64_t k) { return !dropped(i, k); });
    const int64_t n = A.nrows();
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        double f = d[i];
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k)
            if (dropped(i, k)) f += A.val[k];
        for (int64_t k = B.rp[i]; k < B.rp[i + 1]; ++k)
            if (B.col[k] == lo + i) B.val[k] = f;
    }
    return B;
}

// local transpose pattern of the local-local part of S (row i -> local j with i in S_j)
static void local_transpose(const HostCSR& S, int64_t lo, int64_t hi, std::vector<int64_t>& tp,
                            std::vector<int64_t>& tc) {
    int64_t n = S.nrows();
    tp.assign(n + 1, 0);
    for (int64_t k = 0; k < S.nnz(); ++k)
        if (S.col[k] >= lo && S.col[k] < hi) tp[S.col[k] - lo + 1]++;
    for (int64_t i = 0; i < n; ++i) tp[i + 1] += tp[i];
    tc.resize(tp[n]);
    std::vector<int64_t> pos(tp.begin(), tp.end() - 1);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t k = S.rp[j]; k < S.rp[j + 1]; ++k)
            if (S.col[k] >= lo && S.col[k] < hi) tc[pos[S.col[k] - lo]++] = lo + j;
}

// --------------------------------------------------------------------------------
// Ruge-Stueben first pass (serial definition; needs the whole matrix on one rank).
// --------------------------------------------------------------------------------
std::vector<int32_t> rs_split(const HostComm& comm, const HostCSR& S) {
    AMG_CHECK(comm.nranks == 1, "Ruge-Stueben splitting is serial: use PMIS for multi-rank");
    int64_t n = S.nrows();
    std::vector<int64_t> tp, tc;
    local_transpose(S, 0, n, tp, tc);
    std::vector<int32_t> cf(n);
    std::vector<int64_t> lam(n);
    // max-heap on (lam, -idx): larger lambda first, then smaller index
    using E = std::pair<int64_t, int64_t>;
    auto worse = [](const E& a, const E& b) {
        return a.first < b.first || (a.first == b.first && a.second > b.second);
    };
    std::priority_queue<E, std::vector<E>, decltype(worse)> pq(worse);
    for (int64_t i = 0; i < n; ++i) {
        int64_t ns = S.rp[i + 1] - S.rp[i], nt = tp[i + 1] - tp[i];
        cf[i] = (ns == 0 && nt == 0) ? ST_F : ST_U;
        lam[i] = nt;
        if (cf[i] == ST_U) pq.push({lam[i], i});
    }
    while (!pq.empty()) {
        E e = pq.top();
        pq.pop();
        int64_t i = e.second;
        if (cf[i] != ST_U || e.first != lam[i]) continue;
        cf[i] = ST_C;
        for (int64_t t = tp[i]; t < tp[i + 1]; ++t) {
            int64_t j = tc[t];
            if (cf[j] != ST_U) continue;
            cf[j] = ST_F;
            for (int64_t u = S.rp[j]; u < S.rp[j + 1]; ++u) {
                int64_t k = S.col[u];
                if (cf[k] == ST_U) pq.push({++lam[k], k});
            }
        }
        for (int64_t t = S.rp[i]; t < S.rp[i + 1]; ++t) {
            int64_t j = S.col[t];
            if (cf[j] == ST_U) pq.push({--lam[j], j});
        }
    }
    return cf;
}

// --------------------------------------------------------------------------------
// PMIS (distributed, synchronous; identical to the serial definition at any rank count)
// --------------------------------------------------------------------------------
std::vector<int32_t> pmis_split(const HostComm& comm, const HostCSR& S, uint64_t seed) {
    int64_t n = S.nrows(), lo = S.row_starts[comm.rank], hi = S.row_starts[comm.rank + 1];
    // |S^T_i| and the off-process points depending on i
    std::vector<int64_t> tp, tc;
    local_transpose(S, lo, hi, tp, tc);
    std::vector<std::vector<int64_t>> sendp(comm.nranks);  // pairs (i, j): j depends on i
    for (int64_t j = 0; j < n; ++j)
        for (int64_t k = S.rp[j]; k < S.rp[j + 1]; ++k) {
            int64_t i = S.col[k];
            if (i < lo || i >= hi) {
                int o = owner_of(S.col_starts, i);
                sendp[o].push_back(i);
                sendp[o].push_back(lo + j);
            }
        }
    auto gotp = comm.exchange(sendp);
    std::vector<int64_t> cnt(n);
    for (int64_t i = 0; i < n; ++i) cnt[i] = tp[i + 1] - tp[i];
    std::vector<std::vector<int64_t>> ext(n);
    for (int r = 0; r < comm.nranks; ++r)
        for (size_t t = 0; t < gotp[r].size(); t += 2) {
            cnt[gotp[r][t] - lo]++;
            ext[gotp[r][t] - lo].push_back(gotp[r][t + 1]);
        }
    // neighbourhood G_i = S_i u S^T_i (global ids)
    std::vector<int64_t> gp(n + 1, 0), gc;
    for (int64_t i = 0; i < n; ++i) {
        for (int64_t k = S.rp[i]; k < S.rp[i + 1]; ++k) gc.push_back(S.col[k]);
        for (int64_t t = tp[i]; t < tp[i + 1]; ++t) gc.push_back(tc[t]);
        for (int64_t g : ext[i]) gc.push_back(g);
        gp[i + 1] = (int64_t)gc.size();
    }
    std::vector<int64_t> need;
    for (int64_t g : gc)
        if (g < lo || g >= hi) need.push_back(g);
    HaloPlan plan = build_halo_plan(comm, S.col_starts, std::move(need));
    std::vector<int64_t> gloc(gc.size());  // >= 0 local, < 0 halo -(t+1)
    for (size_t t = 0; t < gc.size(); ++t)
        gloc[t] = (gc[t] >= lo && gc[t] < hi) ? gc[t] - lo : -(plan.find(gc[t]) + 1);
    // S column locators (subset of G's halo)
    std::vector<int64_t> sloc(S.nnz());
    for (int64_t k = 0; k < S.nnz(); ++k)
        sloc[k] = (S.col[k] >= lo && S.col[k] < hi) ? S.col[k] - lo : -(plan.find(S.col[k]) + 1);

    std::vector<uint64_t> key(n), hkey(plan.n_halo());
    std::vector<int32_t> cf(n), hcf(plan.n_halo());
    int64_t nu = 0;
    for (int64_t i = 0; i < n; ++i) {
        key[i] = ((uint64_t)cnt[i] << 32) | (uint64_t)hash32(lo + i, seed);
        cf[i] = cnt[i] == 0 ? ST_F : ST_U;
        nu += cf[i] == ST_U;
    }
    plan.forward(comm, key.data(), hkey.data());
    std::vector<int64_t> hgid = plan.halo_gid;
    nu = comm.allreduce_sum(nu);
    std::vector<uint8_t> newc(n);
    while (nu > 0) {
        plan.forward(comm, cf.data(), hcf.data());
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < n; ++i) {
            newc[i] = 0;
            if (cf[i] != ST_U) continue;
            bool best = true;
            for (int64_t t = gp[i]; t < gp[i + 1] && best; ++t) {
                int64_t l = gloc[t];
                int32_t sj = l >= 0 ? cf[l] : hcf[-l - 1];
                if (sj != ST_U) continue;
                uint64_t kj = l >= 0 ? key[l] : hkey[-l - 1];
                int64_t gj = gc[t];
                if (kj > key[i] || (kj == key[i] && gj > lo + i)) best = false;
            }
            newc[i] = best;
        }
        for (int64_t i = 0; i < n; ++i)
            if (newc[i]) cf[i] = ST_C;
        plan.forward(comm, cf.data(), hcf.data());
        int64_t lu = 0;
#pragma omp parallel for schedule(static) reduction(+ : lu)
        for (int64_t i = 0; i < n; ++i) {
            if (cf[i] != ST_U) continue;
            for (int64_t k = S.rp[i]; k < S.rp[i + 1]; ++k) {
                int64_t l = sloc[k];
                if ((l >= 0 ? cf[l] : hcf[-l - 1]) == ST_C) {
                    cf[i] = ST_F;
                    break;
                }
            }
            lu += cf[i] == ST_U;
        }
        nu = comm.allreduce_sum(lu);
    }
    return cf;
}

// --------------------------------------------------------------------------------
// Classical (modified) interpolation, distance 1.  See the oracle for the formula.
// --------------------------------------------------------------------------------
// Extended+i interpolation (r6 option; oracle orc_interp_ext_i): distance two,
// P_max truncation.  One rank (the distance-two sets need the rows of strong F neighbours and
// their strong C neighbours' states, which a multi-rank setup would fetch two halos deep).
HostCSR interp_ext_i(const HostComm& comm, const HostCSR& A, const HostCSR& S, const std::vector<int32_t>& cf,
                     int p_max) {
    AMG_CHECK(comm.nranks == 1, "extended+i interpolation is implemented for one rank");
    const int64_t n = A.nrows();
    std::vector<int64_t> cmap(n);
    int64_t nc = 0;
    for (int64_t i = 0; i < n; ++i) cmap[i] = cf[i] == ST_C ? nc++ : -1;
    const std::vector<double> diag = diagonal(comm, A);
    std::vector<std::vector<int64_t>> pcol(n);
    std::vector<std::vector<double>> pval(n);
#pragma omp parallel
    {
        std::vector<int64_t> strong(n, -1), inC(n, -1), list;
        std::vector<double> num(n), w;
        std::vector<char> keep;
#pragma omp for schedule(dynamic, 1024)
        for (int64_t i = 0; i < n; ++i) {
            if (cf[i] == ST_C) {
                pcol[i].push_back(cmap[i]);
                pval[i].push_back(1.0);
                continue;
            }
            list.clear();
            for (int64_t t = S.rp[i]; t < S.rp[i + 1]; ++t) strong[S.col[t]] = i;
            for (int64_t t = S.rp[i]; t < S.rp[i + 1]; ++t) {
                const int64_t j = S.col[t];
                if (cf[j] == ST_C && inC[j] != i) inC[j] = i, list.push_back(j), num[j] = 0.0;
            }
            for (int64_t t = S.rp[i]; t < S.rp[i + 1]; ++t) {
                const int64_t k = S.col[t];
                if (cf[k] == ST_C) continue;
                for (int64_t u = S.rp[k]; u < S.rp[k + 1]; ++u) {
                    const int64_t j = S.col[u];
                    if (cf[j] == ST_C && inC[j] != i) inC[j] = i, list.push_back(j), num[j] = 0.0;
                }
            }
            double d = diag[i];
            for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
                const int64_t j = A.col[k];
                if (j == i) continue;
                if (inC[j] == i) num[j] += A.val[k];
                else if (strong[j] != i) d += A.val[k];
            }
            for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
                const int64_t kk = A.col[k];
                if (kk == i || strong[kk] != i || cf[kk] == ST_C) continue;
                const bool pos = diag[kk] > 0.0;
                auto abar = [pos](double v) { return pos ? v < 0.0 : v > 0.0; };
                double sk = 0.0;
                for (int64_t u = A.rp[kk]; u < A.rp[kk + 1]; ++u) {
                    const int64_t l = A.col[u];
                    if (abar(A.val[u]) && (inC[l] == i || l == i)) sk += A.val[u];
                }
                if (sk == 0.0) {
                    d += A.val[k];
                    continue;
                }
                for (int64_t u = A.rp[kk]; u < A.rp[kk + 1]; ++u) {
                    const int64_t l = A.col[u];
                    if (!abar(A.val[u])) continue;
                    if (inC[l] == i) num[l] += (A.val[k] * A.val[u]) / sk;
                    else if (l == i) d += (A.val[k] * A.val[u]) / sk;
                }
            }
            std::sort(list.begin(), list.end());
            const int64_t m = (int64_t)list.size();
            w.resize(m);
            keep.assign(m, 1);
            for (int64_t t = 0; t < m; ++t) w[t] = -num[list[t]] / d;
            if (p_max > 0 && m > p_max) {
                double tot = 0.0, kept = 0.0;
                for (int64_t t = 0; t < m; ++t) tot += w[t], keep[t] = 0;
                for (int r = 0; r < p_max; ++r) {
                    int64_t best = -1;
                    for (int64_t t = 0; t < m; ++t)
                        if (!keep[t] && (best < 0 || std::fabs(w[t]) > std::fabs(w[best]))) best = t;
                    keep[best] = 1;
                }
                for (int64_t t = 0; t < m; ++t)
                    if (keep[t]) kept += w[t];
                if (kept != 0.0) {
                    const double f = tot / kept;
                    for (int64_t t = 0; t < m; ++t)
                        if (keep[t]) w[t] = w[t] * f;
                }
            }
            for (int64_t t = 0; t < m; ++t)
                if (keep[t]) pcol[i].push_back(cmap[list[t]]), pval[i].push_back(w[t]);
        }
    }
    HostCSR P;
    P.n_global_rows = n;
    P.n_global_cols = nc;
    P.row_starts = A.row_starts;
    P.col_starts = {0, nc};
    P.rp.assign(n + 1, 0);
    for (int64_t i = 0; i < n; ++i) P.rp[i + 1] = P.rp[i] + (int64_t)pcol[i].size();
    P.col.resize(P.rp[n]);
    P.val.resize(P.rp[n]);
    for (int64_t i = 0; i < n; ++i) {
        std::copy(pcol[i].begin(), pcol[i].end(), P.col.begin() + P.rp[i]);
        std::copy(pval[i].begin(), pval[i].end(), P.val.begin() + P.rp[i]);
    }
    return P;
}

HostCSR interp_classical(const HostComm& comm, const HostCSR& A, const HostCSR& S,
                         const std::vector<int32_t>& cf) {
    int64_t n = A.nrows(), lo = A.row_starts[comm.rank], hi = A.row_starts[comm.rank + 1];
    int64_t ncl = 0;
    for (int32_t v : cf) ncl += v == ST_C;
    std::vector<int64_t> counts = comm.allgather(ncl);
    std::vector<int64_t> cstarts(comm.nranks + 1, 0);
    for (int r = 0; r < comm.nranks; ++r) cstarts[r + 1] = cstarts[r] + counts[r];
    std::vector<int64_t> cmap(n, -1);
    for (int64_t i = 0, c = cstarts[comm.rank]; i < n; ++i)
        if (cf[i] == ST_C) cmap[i] = c++;
    HaloPlan plan = halo_plan_for_cols(comm, A);
    std::vector<int32_t> hcf(plan.n_halo());
    std::vector<int64_t> hcmap(plan.n_halo());
    plan.forward(comm, cf.data(), hcf.data());
    plan.forward(comm, cmap.data(), hcmap.data());
    GhostRows G = fetch_rows(comm, plan, A);

    HostCSR P;
    P.n_global_rows = A.n_global_rows;
    P.n_global_cols = cstarts[comm.nranks];
    P.row_starts = A.row_starts;
    P.col_starts = cstarts;
    int nt = omp_get_max_threads();
    std::vector<std::vector<int64_t>> tcol(nt), tlen(nt);
    std::vector<std::vector<double>> tval(nt);
#pragma omp parallel num_threads(nt)
    {
        int t = omp_get_thread_num(), T = omp_get_num_threads();
        int64_t r0 = n * t / T, r1 = n * (t + 1) / T;
        std::vector<int64_t> ci;  // C_i global ids (ascending)
        std::vector<double> num;
        auto state = [&](int64_t g, int64_t* cm) -> int32_t {
            if (g >= lo && g < hi) {
                if (cm) *cm = cmap[g - lo];
                return cf[g - lo];
            }
            int64_t h = plan.find(g);
            if (cm) *cm = hcmap[h];
            return hcf[h];
        };
        for (int64_t i = r0; i < r1; ++i) {
            int64_t gi = lo + i;
            if (cf[i] == ST_C) {
                tcol[t].push_back(cmap[i]);
                tval[t].push_back(1.0);
                tlen[t].push_back(1);
                continue;
            }
            const int64_t* sb = S.col.data() + S.rp[i];
            const int64_t* se = S.col.data() + S.rp[i + 1];
            auto is_strong = [&](int64_t g) { return std::binary_search(sb, se, g); };
            double d = 0.0;
            for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k)
                if (A.col[k] == gi) {
                    d = A.val[k];
                    break;
                }
            ci.clear();
            num.clear();
            for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
                int64_t j = A.col[k];
                if (j == gi) continue;
                bool st = is_strong(j);
                if (st && state(j, nullptr) == ST_C) {
                    ci.push_back(j);
                    num.push_back(A.val[k]);
                } else if (!st) {
                    d += A.val[k];
                }
            }
            if (!ci.empty()) {
                for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
                    int64_t kk = A.col[k];
                    if (kk == gi || !is_strong(kk) || state(kk, nullptr) == ST_C) continue;
                    const int64_t* rc;
                    const double* rv;
                    int64_t rl;
                    if (kk >= lo && kk < hi) {
                        int64_t r = kk - lo;
                        rc = &A.col[A.rp[r]], rv = &A.val[A.rp[r]], rl = A.rp[r + 1] - A.rp[r];
                    } else {
                        int64_t h = plan.find(kk);
                        rc = &G.col[G.rp[h]], rv = &G.val[G.rp[h]], rl = G.rp[h + 1] - G.rp[h];
                    }
                    // only couplings of sign opposite to a_kk distribute (no cancellation)
                    double akk = 0.0;
                    for (int64_t u = 0; u < rl; ++u)
                        if (rc[u] == kk) {
                            akk = rv[u];
                            break;
                        }
                    const bool pos = akk > 0.0;
                    auto opp = [pos](double v) { return pos ? v < 0.0 : v > 0.0; };
                    double s = 0.0;
                    for (int64_t u = 0; u < rl; ++u)
                        if (opp(rv[u]) && std::binary_search(ci.begin(), ci.end(), rc[u])) s += rv[u];
                    if (s == 0.0) {
                        d += A.val[k];
                    } else {
                        for (int64_t u = 0; u < rl; ++u) {
                            if (!opp(rv[u])) continue;
                            auto it = std::lower_bound(ci.begin(), ci.end(), rc[u]);
                            if (it != ci.end() && *it == rc[u])
                                num[it - ci.begin()] += (A.val[k] * rv[u]) / s;
                        }
                    }
                }
            }
            for (size_t q = 0; q < ci.size(); ++q) {
                int64_t cm;
                state(ci[q], &cm);
                tcol[t].push_back(cm);
                tval[t].push_back(-num[q] / d);
            }
            tlen[t].push_back((int64_t)ci.size());
        }
    }
    P.rp.assign(n + 1, 0);
    int64_t r = 0;
    for (int t = 0; t < nt; ++t)
        for (int64_t l : tlen[t]) P.rp[r + 1] = P.rp[r] + l, ++r;
    for (int t = 0; t < nt; ++t) {
        P.col.insert(P.col.end(), tcol[t].begin(), tcol[t].end());
        P.val.insert(P.val.end(), tval[t].begin(), tval[t].end());
    }
    return P;
}

// --------------------------------------------------------------------------------
// MIS(2) aggregation (distributed, synchronous).  Tuple (state, hash, id) packed as
// hi = state << 32 | hash, lo = id; lexicographic max.
// --------------------------------------------------------------------------------
std::vector<int64_t> mis2_aggregate(const HostComm& comm, const HostCSR& S, uint64_t seed,
                                    int64_t* n_agg_global, std::vector<int64_t>* agg_starts) {
    enum { M_OUT = 0, M_U = 1, M_IN = 2 };
    int64_t n = S.nrows(), lo = S.row_starts[comm.rank], hi = S.row_starts[comm.rank + 1];
    HaloPlan plan = halo_plan_for_cols(comm, S);
    int64_t nh = plan.n_halo();
    std::vector<int64_t> sloc(S.nnz());
    for (int64_t k = 0; k < S.nnz(); ++k)
        sloc[k] = (S.col[k] >= lo && S.col[k] < hi) ? S.col[k] - lo : -(plan.find(S.col[k]) + 1);
    std::vector<int32_t> st(n, M_U);
    std::vector<uint64_t> h0(n), l0(n), h1(n), l1(n), hh(nh), hl(nh);
    std::vector<uint32_t> hs(n);
    for (int64_t i = 0; i < n; ++i) hs[i] = hash32(lo + i, seed);
    int64_t nu = comm.allreduce_sum(n);
    while (nu > 0) {
        for (int64_t i = 0; i < n; ++i) {
            h0[i] = ((uint64_t)(uint32_t)st[i] << 32) | hs[i];
            l0[i] = (uint64_t)(lo + i);
        }
        for (int hop = 0; hop < 2; ++hop) {
            plan.forward(comm, h0.data(), hh.data());
            plan.forward(comm, l0.data(), hl.data());
#pragma omp parallel for schedule(static)
            for (int64_t i = 0; i < n; ++i) {
                uint64_t mh = h0[i], ml = l0[i];
                for (int64_t k = S.rp[i]; k < S.rp[i + 1]; ++k) {
                    int64_t l = sloc[k];
                    uint64_t xh = l >= 0 ? h0[l] : hh[-l - 1], xl = l >= 0 ? l0[l] : hl[-l - 1];
                    if (xh > mh || (xh == mh && xl > ml)) mh = xh, ml = xl;
                }
                h1[i] = mh;
                l1[i] = ml;
            }
            h0.swap(h1);
            l0.swap(l1);
        }
        int64_t lu = 0;
        for (int64_t i = 0; i < n; ++i) {
            if (st[i] != M_U) continue;
            if (l0[i] == (uint64_t)(lo + i)) st[i] = M_IN;
            else if ((h0[i] >> 32) == M_IN) st[i] = M_OUT;
            lu += st[i] == M_U;
        }
        nu = comm.allreduce_sum(lu);
    }
    int64_t nroot = 0;
    for (int32_t s : st) nroot += s == M_IN;
    std::vector<int64_t> counts = comm.allgather(nroot);
    agg_starts->assign(comm.nranks + 1, 0);
    for (int r = 0; r < comm.nranks; ++r) (*agg_starts)[r + 1] = (*agg_starts)[r] + counts[r];
    *n_agg_global = (*agg_starts)[comm.nranks];
    std::vector<int64_t> agg(n, -1), hagg(nh), a1(n);
    for (int64_t i = 0, c = (*agg_starts)[comm.rank]; i < n; ++i)
        if (st[i] == M_IN) agg[i] = c++;
    plan.forward(comm, agg.data(), hagg.data());  // -1 for non-roots
    for (int64_t i = 0; i < n; ++i) {
        a1[i] = agg[i];
        if (agg[i] >= 0) continue;
        for (int64_t k = S.rp[i]; k < S.rp[i + 1]; ++k) {
            int64_t l = sloc[k];
            int64_t aj = l >= 0 ? agg[l] : hagg[-l - 1];
            if (aj >= 0) {  // neighbour is a root (only roots carry an id here)
                a1[i] = aj;
                break;
            }
        }
    }
    std::vector<int64_t> ha1(nh);
    plan.forward(comm, a1.data(), ha1.data());
    for (int64_t i = 0; i < n; ++i) {
        agg[i] = a1[i];
        if (a1[i] >= 0) continue;
        double best = -1.0;
        int64_t ba = -1;
        for (int64_t k = S.rp[i]; k < S.rp[i + 1]; ++k) {
            int64_t l = sloc[k];
            int64_t aj = l >= 0 ? a1[l] : ha1[-l - 1];
            if (aj < 0) continue;
            double w = std::fabs(S.val[k]);
            if (w > best || (w == best && aj < ba)) best = w, ba = aj;
        }
        if (ba < 0) throw Error(AMG_ERR_INTERNAL, "MIS(2): unaggregated node");
        agg[i] = ba;
    }
    return agg;
}

HostCSR sa_prolongator(const HostComm& comm, const HostCSR& A, const std::vector<int64_t>& agg,
                       int64_t n_agg, const std::vector<int64_t>& agg_starts, double theta, uint64_t seed) {
    int64_t n = A.nrows(), alo = agg_starts[comm.rank], ahi = agg_starts[comm.rank + 1];
    int64_t lo = A.row_starts[comm.rank], hi = A.row_starts[comm.rank + 1];
    // aggregate sizes: owners sum member counts
    std::vector<int64_t> size(ahi - alo, 0);
    std::vector<std::vector<int64_t>> sendc(comm.nranks);
    for (int64_t i = 0; i < n; ++i) {
        if (agg[i] >= alo && agg[i] < ahi) size[agg[i] - alo]++;
        else sendc[owner_of(agg_starts, agg[i])].push_back(agg[i]);
    }
    auto got = comm.exchange(sendc);
    for (int r = 0; r < comm.nranks; ++r)
        for (int64_t a : got[r]) size[a - alo]++;
    std::vector<int64_t> need;
    for (int64_t a : agg)
        if (a < alo || a >= ahi) need.push_back(a);
    HaloPlan splan = build_halo_plan(comm, agg_starts, std::move(need));
    std::vector<int64_t> hsize(splan.n_halo());
    splan.forward(comm, size.data(), hsize.data());
    HostCSR T;
    T.n_global_rows = A.n_global_rows;
    T.n_global_cols = n_agg;
    T.row_starts = A.row_starts;
    T.col_starts = agg_starts;
    T.rp.resize(n + 1);
    T.col.resize(n);
    T.val.resize(n);
    T.rp[0] = 0;
    for (int64_t i = 0; i < n; ++i) {
        int64_t a = agg[i];
        int64_t sz = (a >= alo && a < ahi) ? size[a - alo] : hsize[splan.find(a)];
        T.col[i] = a;
        T.val[i] = 1.0 / std::sqrt((double)sz);
        T.rp[i + 1] = i + 1;
    }
    std::vector<double> d = diagonal(comm, A);
    HostCSR F = sa_filter(comm, A, theta);
    // rho(D^-1 A_F): power steps in the max norm from x = u / max|u| (u = the seeded uniform
    // vector of the global ids); maxima are exact in any order, so every partition agrees
    HaloPlan fplan = halo_plan_for_cols(comm, F);
    std::vector<int64_t> where(F.nnz());  // >= 0 local index, < 0: -(halo index + 1)
    for (int64_t k = 0; k < F.nnz(); ++k) {
        int64_t j = F.col[k];
        where[k] = (j >= lo && j < hi) ? j - lo : -(fplan.find(j) + 1);
    }
    std::vector<double> x(n), y(n), hx(fplan.n_halo());
    for (int64_t i = 0; i < n; ++i) {
        uint64_t u = mix64(seed * 0xD1B54A32D192ED03ull + (uint64_t)(lo + i));
        x[i] = (double)(u >> 11) * 0x1.0p-52 - 1.0;
    }
    double m = 0.0;
    for (int64_t i = 0; i < n; ++i) m = std::max(m, std::fabs(x[i]));
    m = comm.allreduce_max(m);
    if (m > 0.0)
        for (int64_t i = 0; i < n; ++i) x[i] = x[i] / m;
    double rho = 0.0;
    for (int it = 0; it < kSaRhoIters; ++it) {
        fplan.forward(comm, x.data(), hx.data());
        double lam = 0.0;
#pragma omp parallel for schedule(static) reduction(max : lam)
        for (int64_t i = 0; i < n; ++i) {
            double s = 0.0;
            for (int64_t k = F.rp[i]; k < F.rp[i + 1]; ++k)
                s += F.val[k] * (where[k] >= 0 ? x[where[k]] : hx[-where[k] - 1]);
            y[i] = s / d[i];
            lam = std::max(lam, std::fabs(y[i]));
        }
        rho = comm.allreduce_max(lam);
        if (rho == 0.0) break;
        for (int64_t i = 0; i < n; ++i) x[i] = y[i] / rho;
    }
    double omega = rho > 0.0 ? (4.0 / 3.0) / rho : 0.0;
    HostCSR AT = spgemm(comm, F, T);
    HostCSR P;
    P.n_global_rows = A.n_global_rows;
    P.n_global_cols = n_agg;
    P.row_starts = A.row_starts;
    P.col_starts = agg_starts;
    P.rp.assign(n + 1, 0);
    P.col.reserve(AT.nnz() + n);
    P.val.reserve(AT.nnz() + n);
    for (int64_t i = 0; i < n; ++i) {
        double c = omega * (1.0 / d[i]);
        int64_t ka = AT.rp[i], ea = AT.rp[i + 1], kt = T.rp[i], et = T.rp[i + 1];
        while (ka < ea || kt < et) {
            int64_t ja = ka < ea ? AT.col[ka] : INT64_MAX, jt = kt < et ? T.col[kt] : INT64_MAX;
            int64_t j = ja < jt ? ja : jt;
            double tv = 0.0, av = 0.0;
            if (jt == j) tv = T.val[kt++];
            if (ja == j) av = AT.val[ka++];
            P.col.push_back(j);
            P.val.push_back(tv - c * av);
        }
        P.rp[i + 1] = (int64_t)P.col.size();
    }
    return P;
}

// Gather the whole coarsest matrix on every rank; Gauss-Jordan with partial pivoting
// (first maximum), same loop order as the oracle => bit-identical inverse.
std::vector<double> dense_inverse_gathered(const HostComm& comm, const HostCSR& A) {
    int64_t n = A.n_global_rows, lo = A.row_starts[comm.rank];
    std::vector<std::vector<int64_t>> si(comm.nranks);
    std::vector<std::vector<double>> sv(comm.nranks);
    for (int r = 0; r < comm.nranks; ++r)
        for (int64_t i = 0; i < A.nrows(); ++i)
            for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
                si[r].push_back((lo + i) * n + A.col[k]);
                sv[r].push_back(A.val[k]);
            }
    auto gi = comm.exchange(si);
    auto gv = comm.exchange(sv);
    std::vector<double> M(n * n, 0.0), inv(n * n, 0.0);
    for (int r = 0; r < comm.nranks; ++r)
        for (size_t t = 0; t < gi[r].size(); ++t) M[gi[r][t]] = gv[r][t];
    for (int64_t i = 0; i < n; ++i) inv[i * n + i] = 1.0;
    for (int64_t c = 0; c < n; ++c) {
        int64_t p = c;
        for (int64_t r = c + 1; r < n; ++r)
            if (std::fabs(M[r * n + c]) > std::fabs(M[p * n + c])) p = r;
        if (p != c)
            for (int64_t j = 0; j < n; ++j) {
                std::swap(M[c * n + j], M[p * n + j]);
                std::swap(inv[c * n + j], inv[p * n + j]);
            }
        double ip = 1.0 / M[c * n + c];
        for (int64_t j = 0; j < n; ++j) {
            M[c * n + j] *= ip;
            inv[c * n + j] *= ip;
        }
        // rows are independent within a pivot step: parallel, same arithmetic per element
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
    return inv;
}

void build_hierarchy(const HostComm& comm, const HostCSR& A0, const amg_options& opt,
                     HostHierarchy& H, const SpgemmFn& galerkin, const LevelSetupFn& level_fn,
                     const TransposeFn& transpose_fn, const LevelDoneFn& level_done,
                     const RapFn& rap_fn) {
    AMG_CHECK(opt.max_levels >= 1, "max_levels must be >= 1");
    AMG_CHECK(opt.drop_tol >= 0.0 && std::isfinite(opt.drop_tol), "drop_tol must be finite and >= 0");
    auto mm = [&](const HostCSR& X, const HostCSR& Y) {
        return galerkin ? galerkin(X, Y) : spgemm(comm, X, Y);
    };
    H.levels.clear();
    H.A0 = &A0;
    H.levels.emplace_back();
    PhaseTimer tm(comm);
    for (int l = 0;; ++l) {
        const HostCSR& A = H.A(l);
        const std::string L = "L" + std::to_string(l) + " ";
        const int64_t n = A.n_global_rows;
        if (l + 1 >= opt.max_levels || n <= opt.max_coarse) break;
        const std::string rname = "setup level " + std::to_string(l);
        RoctxRange range(rname.c_str());
        HostCSR P;
        std::vector<int32_t> split(A.nrows());
        if (level_fn && level_fn(l, A, P, split)) {
            tm.lap(L + "device strength + split / aggregates + P");
        } else if (opt.coarsen == AMG_COARSEN_SA) {
            const double theta = sa_theta(opt.strong_threshold, l);
            HostCSR S = strength_symmetric(comm, A, theta);
            tm.lap(L + "strength");
            int64_t na = 0;
            std::vector<int64_t> astarts;
            std::vector<int64_t> agg = mis2_aggregate(comm, S, opt.seed + (uint64_t)l, &na, &astarts);
            for (size_t i = 0; i < agg.size(); ++i) split[i] = (int32_t)agg[i];
            tm.lap(L + "aggregate");
            P = sa_prolongator(comm, A, agg, na, astarts, theta, opt.seed + (uint64_t)l);
            tm.lap(L + "prolongator");
        } else if (opt.coarsen == AMG_COARSEN_RS || opt.coarsen == AMG_COARSEN_PMIS) {
            HostCSR S = strength_classical(comm, A, opt.strong_threshold);
            tm.lap(L + "strength");
            split = opt.coarsen == AMG_COARSEN_RS ? rs_split(comm, S)
                                                  : pmis_split(comm, S, opt.seed + (uint64_t)l);
            tm.lap(L + "split");
            P = opt.interp == AMG_INTERP_EXT_I ? interp_ext_i(comm, A, S, split, opt.p_max)
                                               : interp_classical(comm, A, S, split);
            tm.lap(L + "interpolation");
        } else {
            throw Error(AMG_ERR_INVALID, "unknown coarsening");
        }
        const int64_t nc = P.n_global_cols;
        // coarsening stalled (same rule as the oracle): no coarse points, no reduction, or
        // less than 20% reduction on a level small enough to be the dense-solved coarsest
        if (nc == 0 || nc >= n || (n <= 8192 && 5 * nc > 4 * n)) break;
        HostCSR R;
        if (!(transpose_fn && transpose_fn(P, R))) R = transpose(comm, P);
        tm.lap(L + "transpose");
        HostCSR Ac;
        if (rap_fn) {
            Ac = rap_fn(R, A, P);  // the drop tolerance applied (RapFn)
            tm.lap(L + "R*(AP)");
        } else {
            HostCSR AP = mm(A, P);
            tm.lap(L + "A*P");
            Ac = mm(R, AP);
            tm.lap(L + "R*(AP)");
            if (opt.drop_tol > 0.0) {
                Ac = sparsify(comm, Ac, opt.drop_tol);
                tm.lap(L + "drop tolerance");
            }
        }
        H.levels[l].split = std::move(split);
        H.levels[l].P = std::move(P);
        H.levels[l].R = std::move(R);
        H.levels.emplace_back();
        H.levels[l + 1].A = std::move(Ac);
        if (level_done) level_done(l);
    }
    const HostCSR& Ac = H.A(H.levels.size() - 1);
    AMG_CHECK(Ac.n_global_rows <= 20000,
              "coarsest level too large for the dense solve (raise max_levels / max_coarse?)");
    H.coarse_inv = dense_inverse_gathered(comm, Ac);
    tm.lap("coarse dense inverse n=" + std::to_string(Ac.n_global_rows));
}

}  // namespace amg
