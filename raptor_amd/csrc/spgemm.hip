// spgemm.hip -- Galerkin-product SpGEMM C = A * B on gfx950.
//
// Canonical order (identical to oracle/amg_oracle.c orc_spgemm): for each
// output row, acc_j = 0.0; for k over A's row in CSR order, for j over B's row k:
// acc_j += a_ik * b_kj.  One wavefront owns one output row: the k loop is sequential
// (wave-uniform) and the 64 lanes split B's row k, whose columns are distinct -- so each
// accumulator receives exactly one update per k step and the summation order per column
// is the oracle's.  Accumulators live in an open-addressing table in LDS (64-bit CAS on
// the key, plain RMW on the value by the lane that owns the key).  Rows are binned by
// the upper bound sum_k |B_k| into table sizes 256 .. 8192; the rare larger rows are
// computed on the host with the same order.  Two passes: symbolic (count), numeric (fill
// sorted by column: rank = number of smaller keys).
#include <omp.h>

#include <algorithm>
#include <numeric>

#include "device.hpp"

namespace amg {

namespace {

constexpr int kWave = 64;

__device__ __forceinline__ unsigned hslot(long long j, unsigned mask) {
    unsigned long long z = (unsigned long long)j * 0x9E3779B97F4A7C15ull;
    return (unsigned)(z >> 40) & mask;
}

// one 64-lane workgroup per row of `rows`; T table entries (power of two).  A row whose
// distinct columns do not fit (a probe sequence longer than the table) is abandoned: the
// symbolic pass marks it with count -1 and the host computes it.
template <int T, bool NUMERIC>
__global__ __launch_bounds__(kWave) void spgemm_rows_kernel(
    const int* __restrict__ rows, int nrows, const long long* __restrict__ arp,
    const int* __restrict__ acol, const double* __restrict__ aval,
    const long long* __restrict__ brp, const long long* __restrict__ bcol,
    const double* __restrict__ bval, long long* __restrict__ counts,
    const long long* __restrict__ crp, long long* __restrict__ ccol, double* __restrict__ cval) {
    __shared__ long long keys[T];
    __shared__ double vals[NUMERIC ? T : 1];
    __shared__ int nocc, ovf;
    const int lane = threadIdx.x;
    const int w = blockIdx.x;
    if (w >= nrows) return;
    const int i = rows[w];
    for (int t = lane; t < T; t += kWave) {
        keys[t] = -1;
        if (NUMERIC) vals[t] = 0.0;
    }
    if (lane == 0) ovf = 0;
    __syncthreads();
    const unsigned mask = T - 1;
    for (long long ka = arp[i]; ka < arp[i + 1]; ++ka) {
        const int k = acol[ka];
        const double a = aval[ka];
        for (long long q = brp[k] + lane; q < brp[k + 1]; q += kWave) {
            const long long j = bcol[q];
            unsigned h = hslot(j, mask);
            int probes = 0;
            for (;;) {
                const long long prev = atomicCAS((unsigned long long*)&keys[h], (unsigned long long)-1LL,
                                                 (unsigned long long)j);
                if (prev == -1 || prev == j) break;
                h = (h + 1) & mask;
                if (++probes >= T) break;  // table full
            }
            if (probes >= T) {
                ovf = 1;
                break;
            }
            if (NUMERIC) vals[h] += a * bval[q];
        }
        __syncthreads();  // next k step sees every update of this one
        if (ovf) break;   // workgroup-uniform after the barrier
    }
    if (!NUMERIC) {
        if (lane == 0) nocc = 0;
        __syncthreads();
        int c = 0;
        for (int t = lane; t < T; t += kWave) c += keys[t] != -1;
        atomicAdd(&nocc, c);
        __syncthreads();
        if (lane == 0) counts[i] = ovf ? -1 : nocc;
        return;
    }
    // compact the occupied slots in place (targets never pass the chunk being read), pad to
    // a power of two with +inf keys and sort by column (bitonic network in LDS)
    int m = 0;
    for (int b = 0; b < T; b += kWave) {
        const long long j = keys[b + lane];
        const double v = vals[b + lane];
        const bool occ = j != -1;
        const unsigned long long bal = __ballot(occ);
        __syncthreads();
        if (occ) {
            const int pos = m + __popcll(bal & ((1ull << lane) - 1ull));
            keys[pos] = j;
            vals[pos] = v;
        }
        m += __popcll(bal);
        __syncthreads();
    }
    int P = 1;
    while (P < m) P <<= 1;
    for (int t = m + lane; t < P; t += kWave) keys[t] = 0x7fffffffffffffffLL;
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1)
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
            for (int t = lane; t < P; t += kWave) {
                const int u = t ^ jj;
                if (u > t) {
                    const long long kt = keys[t], ku = keys[u];
                    if (((t & k) == 0) == (kt > ku)) {
                        keys[t] = ku;
                        keys[u] = kt;
                        const double vt = vals[t];
                        vals[t] = vals[u];
                        vals[u] = vt;
                    }
                }
            }
            __syncthreads();
        }
    const long long base = crp[i];
    for (int e = lane; e < m; e += kWave) {
        ccol[base + e] = keys[e];
        cval[base + e] = vals[e];
    }
}

template <int T, bool NUMERIC>
void launch_bin(hipStream_t s, const std::vector<int>& rows, DevBuf<int>& drows, const long long* arp,
                const int* acol, const double* aval, const long long* brp, const long long* bcol,
                const double* bval, long long* counts, const long long* crp, long long* ccol,
                double* cval) {
    if (rows.empty()) return;
    drows.upload(rows.data(), rows.size());
    hipLaunchKernelGGL((spgemm_rows_kernel<T, NUMERIC>), dim3((unsigned)rows.size()), dim3(kWave), 0, s,
                       drows.p, (int)rows.size(), arp, acol, aval, brp, bcol, bval, counts, crp, ccol,
                       cval);
    HIP_CHECK(hipGetLastError());
}

}  // namespace

HostCSR spgemm_device(Context& ctx, const HostComm& comm, const HostCSR& A, const HostCSR& B) {
    AMG_CHECK(A.col_starts == B.row_starts, "spgemm: A columns and B rows partitioned differently");
    PhaseTimer tm(comm);
    HaloPlan plan = halo_plan_for_cols(comm, A);
    GhostRows G = fetch_rows(comm, plan, B);
    const int64_t n = A.nrows(), nbl = B.nrows(), lo = B.row_starts[comm.rank],
                  hi = B.row_starts[comm.rank + 1];
    // B rows = [local rows | ghost rows]; A columns renumbered into that row space
    std::vector<long long> brp(nbl + plan.n_halo() + 1);
    for (int64_t r = 0; r <= nbl; ++r) brp[r] = B.rp[r];
    for (int64_t t = 0; t < plan.n_halo(); ++t) brp[nbl + t + 1] = B.rp[nbl] + G.rp[t + 1];
    std::vector<int> acol(A.nnz());
    std::vector<int64_t> ub(n, 0);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        int64_t u = 0;
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
            const int64_t c = A.col[k];
            const int64_t r = (c >= lo && c < hi) ? c - lo : nbl + plan.find(c);
            acol[k] = (int)r;
            u += brp[r + 1] - brp[r];
        }
        ub[i] = u;
    }
    const int64_t bnnz = brp.back();
    // the B image [local rows | ghost rows] is assembled on the device (two uploads each),
    // not in a host copy of B; the host fallback reads B or G through bcol_at / bval_at
    static_assert(sizeof(long long) == sizeof(int64_t), "int64 columns");
    const int64_t bl = B.nnz();
    auto bcol_at = [&](long long q) -> int64_t { return q < bl ? B.col[q] : G.col[q - bl]; };
    auto bval_at = [&](long long q) -> double { return q < bl ? B.val[q] : G.val[q - bl]; };
    // bins by table size (load factor <= 1/2 on the upper bound); rows beyond the largest
    // table try it anyway (their distinct columns are usually far fewer than the bound) and
    // fall back to the host only when it overflows
    static constexpr int kBins[] = {256, 1024, 4096, 8192};
    std::vector<int> bins[4];
    for (int64_t i = 0; i < n; ++i) {
        int b = 0;
        while (b < 3 && 2 * ub[i] > kBins[b]) ++b;
        bins[b].push_back((int)i);
    }
    tm.lap("    spgemm: column map, B image, bins");
    hipStream_t s = ctx.stream;
    DevBuf<long long> d_arp, d_brp, d_bcol, d_counts, d_crp, d_ccol;
    DevBuf<int> d_acol, d_rows[4];
    DevBuf<double> d_aval, d_bval, d_cval;
    d_arp.upload(reinterpret_cast<const long long*>(A.rp.data()), A.rp.size());
    d_acol.upload(acol.data(), acol.size());
    d_aval.upload(A.val.data(), A.val.size());
    d_brp.upload(brp.data(), brp.size());
    d_bcol.alloc((size_t)bnnz);
    d_bval.alloc((size_t)bnnz);
    if (bl) {
        HIP_CHECK(hipMemcpy(d_bcol.p, B.col.data(), sizeof(long long) * bl, hipMemcpyHostToDevice));
        HIP_CHECK(hipMemcpy(d_bval.p, B.val.data(), sizeof(double) * bl, hipMemcpyHostToDevice));
    }
    if (bnnz > bl) {
        HIP_CHECK(hipMemcpy(d_bcol.p + bl, G.col.data(), sizeof(long long) * (bnnz - bl), hipMemcpyHostToDevice));
        HIP_CHECK(hipMemcpy(d_bval.p + bl, G.val.data(), sizeof(double) * (bnnz - bl), hipMemcpyHostToDevice));
    }
    d_counts.alloc((size_t)std::max<int64_t>(n, 1));
    HIP_CHECK(hipMemsetAsync(d_counts.p, 0, sizeof(long long) * d_counts.n, s));
    tm.lap("    spgemm: uploads");
#define AMG_BIN(T, NUM, b)                                                                          \
    launch_bin<T, NUM>(s, bins[b], d_rows[b], d_arp.p, d_acol.p, d_aval.p, d_brp.p, d_bcol.p,      \
                       d_bval.p, d_counts.p, d_crp.p, d_ccol.p, d_cval.p)
    AMG_BIN(256, false, 0);
    AMG_BIN(1024, false, 1);
    AMG_BIN(4096, false, 2);
    AMG_BIN(8192, false, 3);
    std::vector<long long> counts((size_t)n);
    if (n) HIP_CHECK(hipMemcpyAsync(counts.data(), d_counts.p, sizeof(long long) * n, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    tm.lap("    spgemm: symbolic");
    // rows that overflowed the largest table: host, same canonical order, a dense
    // accumulator per thread (acc_j in k order, then the touched columns sorted)
    std::vector<int64_t> host_rows;
    {
        std::vector<int> keep;
        for (int i : bins[3])
            if (counts[i] < 0) host_rows.push_back(i);
            else keep.push_back(i);
        bins[3].swap(keep);
    }
    std::vector<std::vector<std::pair<int64_t, double>>> hostout(host_rows.size());
    if (!host_rows.empty()) {
        const int64_t ncol = B.n_global_cols;
        // dense accumulators: at most ~2 GB of them across threads
        const int nth = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)host_rows.size(), (int64_t)omp_get_max_threads(),
                                                                     (int64_t)2000000000 / (9 * std::max<int64_t>(ncol, 1))}));
        (void)nth;
#pragma omp parallel num_threads(nth)
        {
            std::vector<double> acc((size_t)ncol, 0.0);
            std::vector<char> seen((size_t)ncol, 0);
            std::vector<int64_t> touched;
#pragma omp for schedule(dynamic, 1)
            for (size_t t = 0; t < host_rows.size(); ++t) {
                const int64_t i = host_rows[t];
                touched.clear();
                for (int64_t ka = A.rp[i]; ka < A.rp[i + 1]; ++ka) {
                    const int64_t r = acol[ka];
                    for (long long q = brp[r]; q < brp[r + 1]; ++q) {
                        const int64_t j = bcol_at(q);
                        if (!seen[j]) seen[j] = 1, touched.push_back(j);
                        acc[j] += A.val[ka] * bval_at(q);
                    }
                }
                std::sort(touched.begin(), touched.end());
                auto& out = hostout[t];
                out.reserve(touched.size());
                for (int64_t j : touched) {
                    out.push_back({j, acc[j]});
                    acc[j] = 0.0;
                    seen[j] = 0;
                }
                counts[i] = (long long)out.size();
            }
        }
    }
    tm.lap("    spgemm: host rows (" + std::to_string(host_rows.size()) + ")");
    HostCSR C;
    C.n_global_rows = A.n_global_rows;
    C.n_global_cols = B.n_global_cols;
    C.row_starts = A.row_starts;
    C.col_starts = B.col_starts;
    C.rp.assign(n + 1, 0);
    for (int64_t i = 0; i < n; ++i) C.rp[i + 1] = C.rp[i] + counts[i];
    const int64_t cnnz = C.rp[n];
    d_crp.upload(reinterpret_cast<const long long*>(C.rp.data()), C.rp.size());
    d_ccol.alloc((size_t)std::max<int64_t>(cnnz, 1));
    d_cval.alloc((size_t)std::max<int64_t>(cnnz, 1));
    AMG_BIN(256, true, 0);
    AMG_BIN(1024, true, 1);
    AMG_BIN(4096, true, 2);
    AMG_BIN(8192, true, 3);
#undef AMG_BIN
    C.col.resize(cnnz);
    C.val.resize(cnnz);
    if (cnnz) {
        HIP_CHECK(hipMemcpyAsync(C.col.data(), d_ccol.p, sizeof(long long) * cnnz, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipMemcpyAsync(C.val.data(), d_cval.p, sizeof(double) * cnnz, hipMemcpyDeviceToHost, s));
    }
    HIP_CHECK(hipStreamSynchronize(s));
    tm.lap("    spgemm: numeric + download");
    for (size_t t = 0; t < host_rows.size(); ++t) {
        int64_t p = C.rp[host_rows[t]];
        for (auto& e : hostout[t]) C.col[p] = e.first, C.val[p++] = e.second;
    }
    return C;
}

}  // namespace amg
