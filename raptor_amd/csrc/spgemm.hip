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
#include <array>
#include <functional>
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
    // a launch covers at most 2^24 rows: HIP counts a grid in threads (uint32 per dimension),
    // and one 64-lane workgroup per row of a 512^3 level (134M rows) would exceed it
    constexpr size_t kMaxRows = size_t(1) << 24;
    for (size_t off = 0; off < rows.size(); off += kMaxRows) {
        const size_t cnt = std::min(kMaxRows, rows.size() - off);
        hipLaunchKernelGGL((spgemm_rows_kernel<T, NUMERIC>), dim3((unsigned)cnt), dim3(kWave), 0, s,
                           drows.p + off, (int)cnt, arp, acol, aval, brp, bcol, bval, counts, crp, ccol, cval);
        HIP_CHECK(hipGetLastError());
    }
}

}  // namespace

namespace {

// rows of a device CSR gathered into 16-byte (column, value) records: wave w copies row
// rows[w] to out[off[w]...] (ghost rows of A P for the ranks that asked for them)
struct PackRec {
    long long c;
    double v;
};

__global__ __launch_bounds__(kWave) void pack_rows_kernel(int nrows, const long long* __restrict__ rows,
                                                          const long long* __restrict__ off,
                                                          const long long* __restrict__ rp,
                                                          const long long* __restrict__ col,
                                                          const double* __restrict__ val, PackRec* __restrict__ out) {
    const int w = blockIdx.x;
    if (w >= nrows) return;
    const long long r = rows[w], b = rp[r], e = rp[r + 1], o = off[w];
    for (long long k = b + threadIdx.x; k < e; k += kWave) out[o + (k - b)] = PackRec{col[k], val[k]};
}

// received records into the B image's column / value arrays
__global__ void unpack_recs_kernel(long long n, const PackRec* __restrict__ in, long long* __restrict__ col,
                                   double* __restrict__ val) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    if (t < n) {
        col[t] = in[t].c;
        val[t] = in[t].v;
    }
}

// C = A * B with B's row image on the device: brp (host and device copies), bcol, bval.
// acol: A's columns as rows of that image; ub: per row the bound sum_k |B_k|.  C stays on
// the device (crp also on the host); rows that overflow the largest LDS table are computed on
// the host (bhost() supplies B's host arrays for them) and uploaded into place.
struct BImage {
    const long long* brp_host;  // nb + 1 entries
    const long long *d_brp, *d_bcol;
    const double* d_bval;
    int64_t ncol;  // global column count (host fallback accumulators)
    // host arrays of the image for the rare fallback rows: col / val of image entry q
    std::function<void(std::function<int64_t(long long)>&, std::function<double(long long)>&)> bhost;
};

// the left operand: device arrays (row pointers, B-image row of each entry, values) and what
// the host fallback rows read (the host rows and values, and each entry's B-image row)
struct AOperand {
    const HostCSR* host;
    std::function<int64_t(int64_t)> acol_at;  // B-image row of entry k (null: host->col[k])
    const long long* d_rp;
    const int* d_col;
    const double* d_val;
};

struct AUpload {
    DevBuf<long long> rp;
    DevBuf<int> col;
    DevBuf<double> val;
};

AOperand upload_a(PhaseTimer& tm, const HostCSR& A, const std::vector<int>& acol, AUpload& u) {
    u.rp.upload(reinterpret_cast<const long long*>(A.rp.data()), A.rp.size());
    u.col.upload(acol.data(), acol.size());
    u.val.upload(A.val.data(), A.val.size());
    tm.lap("    spgemm: uploads of A");
    const int* ac = acol.data();
    return AOperand{&A, [ac](int64_t k) -> int64_t { return ac[k]; }, u.rp.p, u.col.p, u.val.p};
}

void spgemm_core(Context& ctx, PhaseTimer& tm, const AOperand& Aop, const std::vector<int64_t>& ub,
                 const BImage& B, DevCSR64& C) {
    const HostCSR& A = *Aop.host;
    const int64_t n = A.nrows();
    // bins by table size (load factor <= 1/2 on the upper bound); rows beyond the largest
    // table try it anyway (their distinct columns are usually far fewer than the bound) and
    // fall back to the host only when it overflows.  Chunks bin in parallel and concatenate
    // in chunk order: each bin lists its rows ascending, as a serial pass would.
    static constexpr int kBins[] = {256, 1024, 4096, 8192};
    // rows binned in parallel chunks, concatenated in chunk order (each bin lists its rows
    // ascending, as a serial pass would)
    auto bin_rows = [n](std::vector<int>(&bins)[4], const std::function<int(int64_t)>& bin_of) {
        const int nch = (int)std::max<int64_t>(1, std::min<int64_t>(256, n / 65536));
        std::vector<std::array<std::vector<int>, 4>> part((size_t)nch);
#pragma omp parallel for schedule(dynamic, 1)
        for (int c = 0; c < nch; ++c) {
            const int64_t r0 = n * c / nch, r1 = n * (c + 1) / nch;
            for (int64_t i = r0; i < r1; ++i) {
                const int b = bin_of(i);
                if (b >= 0) part[(size_t)c][b].push_back((int)i);
            }
        }
        for (int b = 0; b < 4; ++b) {
            size_t tot = 0;
            for (auto& pc : part) tot += pc[b].size();
            bins[b].clear();
            bins[b].reserve(tot);
            for (auto& pc : part) bins[b].insert(bins[b].end(), pc[b].begin(), pc[b].end());
        }
    };
    // symbolic: rows whose bound fits 256 slots there, every other row first in the 1024-slot
    // table (r5: a row's distinct columns are usually far fewer than its bound -- sa27's
    // R0 (A0 P0) rows bound ~7,000, hold a few hundred -- and a 128 KiB table of 8192 slots runs
    // one workgroup per CU), the rows that overflow it again in 8192 slots
    std::vector<int> bins[4];
    bin_rows(bins, [&](int64_t i) { return 2 * ub[i] > kBins[0] ? 1 : 0; });
    tm.lap("    spgemm: bins");
    hipStream_t s = ctx.stream;
    DevBuf<long long> d_counts;
    DevBuf<int> d_rows[4];
    d_counts.alloc((size_t)std::max<int64_t>(n, 1));
    HIP_CHECK(hipMemsetAsync(d_counts.p, 0, sizeof(long long) * d_counts.n, s));
#define AMG_BIN(T, NUM, b)                                                                          \
    launch_bin<T, NUM>(s, bins[b], d_rows[b], Aop.d_rp, Aop.d_col, Aop.d_val, B.d_brp, B.d_bcol,   \
                       B.d_bval, d_counts.p, C.d_rp.p, C.d_col.p, C.d_val.p)
    AMG_BIN(256, false, 0);
    AMG_BIN(1024, false, 1);
    std::vector<long long> counts((size_t)n);
    if (n) HIP_CHECK(hipMemcpyAsync(counts.data(), d_counts.p, sizeof(long long) * n, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    {
        std::vector<int> retry;
        for (int i : bins[1])
            if (counts[i] < 0) retry.push_back(i);
        if (!retry.empty()) {
            bins[3].swap(retry);
            AMG_BIN(8192, false, 3);
            HIP_CHECK(hipMemcpyAsync(counts.data(), d_counts.p, sizeof(long long) * n, hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
        }
    }
    tm.lap("    spgemm: symbolic");
    // rows that overflowed the largest table: host, same canonical order, a dense
    // accumulator per thread (acc_j in k order, then the touched columns sorted)
    std::vector<int64_t> host_rows;
    for (int64_t i = 0; i < n; ++i)
        if (counts[i] < 0) host_rows.push_back(i);
    // numeric: the table each row's exact count fits at load <= 1/2 (the 8192-slot table
    // above that: the symbolic pass found the row fits it)
    bin_rows(bins, [&](int64_t i) {
        const long long c = counts[i];
        if (c < 0) return -1;
        int b = 0;
        while (b < 3 && 2 * c > kBins[b]) ++b;
        return b;
    });
    std::vector<std::vector<std::pair<int64_t, double>>> hostout(host_rows.size());
    if (!host_rows.empty()) {
        std::function<int64_t(long long)> bcol_at;
        std::function<double(long long)> bval_at;
        B.bhost(bcol_at, bval_at);
        const int64_t ncol = B.ncol;
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
                    const int64_t r = Aop.acol_at ? Aop.acol_at(ka) : A.col[ka];
                    for (long long q = B.brp_host[r]; q < B.brp_host[r + 1]; ++q) {
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
    C.rp.assign(n + 1, 0);
    for (int64_t i = 0; i < n; ++i) C.rp[i + 1] = C.rp[i] + counts[i];
    const int64_t cnnz = C.rp[n];
    C.d_rp.upload(C.rp.data(), C.rp.size());
    C.d_col.alloc((size_t)std::max<int64_t>(cnnz, 1));
    C.d_val.alloc((size_t)std::max<int64_t>(cnnz, 1));
    AMG_BIN(256, true, 0);
    AMG_BIN(1024, true, 1);
    AMG_BIN(4096, true, 2);
    AMG_BIN(8192, true, 3);
#undef AMG_BIN
    for (size_t t = 0; t < host_rows.size(); ++t) {
        const auto& out = hostout[t];
        std::vector<long long> hc(out.size());
        std::vector<double> hv(out.size());
        for (size_t e = 0; e < out.size(); ++e) hc[e] = out[e].first, hv[e] = out[e].second;
        const long long at = C.rp[host_rows[t]];
        if (!out.empty()) {
            HIP_CHECK(hipMemcpyAsync(C.d_col.p + at, hc.data(), sizeof(long long) * hc.size(), hipMemcpyHostToDevice, s));
            HIP_CHECK(hipMemcpyAsync(C.d_val.p + at, hv.data(), sizeof(double) * hv.size(), hipMemcpyHostToDevice, s));
            HIP_CHECK(hipStreamSynchronize(s));
        }
    }
    HIP_CHECK(hipStreamSynchronize(s));
    tm.lap("    spgemm: numeric");
}

HostCSR download(Context& ctx, PhaseTimer& tm, const HostCSR& A, const HostCSR& B, DevCSR64& C) {
    HostCSR out;
    out.n_global_rows = A.n_global_rows;
    out.n_global_cols = B.n_global_cols;
    out.row_starts = A.row_starts;
    out.col_starts = B.col_starts;
    out.rp.assign(C.rp.begin(), C.rp.end());
    const int64_t cnnz = C.nnz();
    out.col.resize(cnnz);
    out.val.resize(cnnz);
    copy_to_host(out.col.data(), C.d_col.p, sizeof(long long) * cnnz, ctx.stream);
    copy_to_host(out.val.data(), C.d_val.p, sizeof(double) * cnnz, nullptr);
    tm.lap("    spgemm: download");
    return out;
}

// B-image row bounds sum_k |B_{acol_k}| per row of A, on the device (the SpGEMM bins)
__global__ void row_bound_kernel(long long n, const long long* __restrict__ arp, const int* __restrict__ acol,
                                 const long long* __restrict__ brp, long long* __restrict__ ub) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    long long u = 0;
    for (long long k = arp[i]; k < arp[i + 1]; ++k) {
        const int c = acol[k];
        u += brp[c + 1] - brp[c];
    }
    ub[i] = u;
}

// N ranks: the B-image row of every entry of A (global column c): c - lo for B's local rows,
// n_local + (position of c among the sorted halo ids) for its ghost rows
__global__ void bimage_rows_kernel(long long nnz, const int* __restrict__ col, long long lo, long long hi,
                                   long long n_local, const long long* __restrict__ halo, int nh, int* __restrict__ out) {
    for (long long k = (long long)blockIdx.x * 256 + threadIdx.x; k < nnz; k += (long long)gridDim.x * 256) {
        const long long c = col[k];
        if (c >= lo && c < hi) {
            out[k] = (int)(c - lo);
        } else {
            int a = 0, b = nh;
            while (a < b) {
                const int m = (a + b) >> 1;
                if (halo[m] < c) a = m + 1;
                else b = m;
            }
            out[k] = (int)(n_local + a);
        }
    }
}

// A's B-image rows and per-row bounds on the device (N ranks); returns the bounds on the host
std::vector<int64_t> device_column_map(hipStream_t s, DevCsr& A, const HaloPlan& plan, int64_t lo, int64_t hi,
                                       int64_t n_local, const long long* d_brp, DevBuf<int>& acol) {
    A.ensure_rp64(s);
    A.ensure_col32(s);
    DevBuf<long long> dh;
    std::vector<long long> hg(plan.halo_gid.begin(), plan.halo_gid.end());
    dh.upload(hg.data(), std::max<size_t>(hg.size(), 1));
    acol.alloc((size_t)std::max<int64_t>(A.nnz, 1));
    if (A.nnz)
        hipLaunchKernelGGL(bimage_rows_kernel, dim3((unsigned)std::min<int64_t>((A.nnz + 255) / 256, 1 << 16)), dim3(256),
                           0, s, (long long)A.nnz, A.col32.p, (long long)lo, (long long)hi, (long long)n_local, dh.p,
                           (int)plan.n_halo(), acol.p);
    std::vector<int64_t> ub((size_t)A.n);
    if (A.n) {
        DevBuf<long long> d_ub;
        d_ub.alloc((size_t)A.n);
        hipLaunchKernelGGL(row_bound_kernel, dim3((unsigned)((A.n + 255) / 256)), dim3(256), 0, s, (long long)A.n,
                           A.rp64.p, acol.p, d_brp, d_ub.p);
        HIP_CHECK(hipGetLastError());
        copy_to_host(ub.data(), d_ub.p, sizeof(long long) * A.n, s);
    }
    HIP_CHECK(hipStreamSynchronize(s));  // dh is freed on return
    return ub;
}

}  // namespace

void spgemm_images(Context& ctx, PhaseTimer& tm, const HostCSR& Ah, DevCsr& A, const long long* brp_host,
                   const HostCSR* Bh, DevCsr& B, int64_t bncol, DevCSR64& C) {
    hipStream_t s = ctx.stream;
    A.ensure_rp64(s);
    A.ensure_col32(s);
    B.ensure_rp64(s);
    B.ensure_col64(s);
    const int64_t n = A.n;
    AMG_CHECK(n == Ah.nrows() && A.nnz == Ah.nnz(), "spgemm: device image does not match its host matrix");
    std::vector<int64_t> ub((size_t)n);
    if (n) {
        DevBuf<long long> d_ub;
        d_ub.alloc((size_t)n);
        hipLaunchKernelGGL(row_bound_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (long long)n,
                           A.rp64.p, A.col32.p, B.rp64.p, d_ub.p);
        HIP_CHECK(hipGetLastError());
        copy_to_host(ub.data(), d_ub.p, sizeof(long long) * n, s);
    }
    tm.lap("    spgemm: row bounds (device)");
    // host copies of the B image only if some row overflows the LDS tables
    std::vector<long long> hc;
    std::vector<double> hv;
    BImage img{brp_host, B.rp64.p, B.col64.p, B.val.p, bncol,
               [&](std::function<int64_t(long long)>& ca, std::function<double(long long)>& va) {
                   if (Bh) {
                       ca = [Bh](long long q) -> int64_t { return Bh->col[q]; };
                       va = [Bh](long long q) -> double { return Bh->val[q]; };
                       return;
                   }
                   hc.resize((size_t)B.nnz);
                   hv.resize((size_t)B.nnz);
                   copy_to_host(hc.data(), B.col64.p, sizeof(long long) * B.nnz, s);
                   copy_to_host(hv.data(), B.val.p, sizeof(double) * B.nnz, nullptr);
                   ca = [&](long long q) -> int64_t { return hc[q]; };
                   va = [&](long long q) -> double { return hv[q]; };
               }};
    spgemm_core(ctx, tm, AOperand{&Ah, nullptr, A.rp64.p, A.col32.p, A.val.p}, ub, img, C);
}

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
    tm.lap("    spgemm: column map, B image");
    // the B image [local rows | ghost rows] is assembled on the device (two uploads each),
    // not in a host copy of B; the host fallback reads B or G in place
    static_assert(sizeof(long long) == sizeof(int64_t), "int64 columns");
    const int64_t bl = B.nnz();
    DevBuf<long long> d_brp, d_bcol;
    DevBuf<double> d_bval;
    d_brp.upload(brp.data(), brp.size());
    d_bcol.alloc((size_t)std::max<int64_t>(bnnz, 1));
    d_bval.alloc((size_t)std::max<int64_t>(bnnz, 1));
    copy_to_device(d_bcol.p, B.col.data(), sizeof(long long) * bl);
    copy_to_device(d_bval.p, B.val.data(), sizeof(double) * bl);
    copy_to_device(d_bcol.p + bl, G.col.data(), sizeof(long long) * (bnnz - bl));
    copy_to_device(d_bval.p + bl, G.val.data(), sizeof(double) * (bnnz - bl));
    tm.lap("    spgemm: upload of B");
    BImage img{brp.data(), d_brp.p, d_bcol.p, d_bval.p, B.n_global_cols,
               [&](std::function<int64_t(long long)>& ca, std::function<double(long long)>& va) {
                   ca = [&](long long q) -> int64_t { return q < bl ? B.col[q] : G.col[q - bl]; };
                   va = [&](long long q) -> double { return q < bl ? B.val[q] : G.val[q - bl]; };
               }};
    DevCSR64 C;
    AUpload au;
    spgemm_core(ctx, tm, upload_a(tm, A, acol, au), ub, img, C);
    return download(ctx, tm, A, B, C);
}

namespace {

// Several ranks: A P stays on the device between the two products.  The
// rows of A P that other ranks' R columns reference are gathered on the device
// (pack_rows_kernel), and only those travel: download, one host all-to-all-v, upload behind
// this rank's own rows, which are copied device to device into the B image of R (A P).  Same
// products and order as the two spgemm_device calls it replaces: bit-identical.
HostCSR galerkin_device_dist(Context& ctx, const HostComm& comm, const HostCSR& R, const HostCSR& A,
                             const HostCSR& P, SetupImages* imgs) {
    AMG_CHECK(A.col_starts == P.row_starts && R.col_starts == A.row_starts, "galerkin: partitions differ");
    PhaseTimer tm(comm);
    hipStream_t s = ctx.stream;
    static_assert(sizeof(long long) == sizeof(int64_t), "int64 columns");
    // A, P and R from the setup's device images (r5; uploaded here without them); their
    // columns mapped to B-image rows on the device
    SetupImages local;
    SetupImages& im = imgs ? *imgs : local;
    // ---- A P: B image = [P's rows | ghost rows of P] (spgemm_device's first product)
    DevCSR64 AP;
    {
        HaloPlan plan = halo_plan_for_cols(comm, A);
        GhostRows G = fetch_rows(comm, plan, P);
        const int64_t nbl = P.nrows(), lo = P.row_starts[comm.rank], hi = P.row_starts[comm.rank + 1];
        std::vector<long long> brp(nbl + plan.n_halo() + 1);
        for (int64_t r = 0; r <= nbl; ++r) brp[r] = P.rp[r];
        for (int64_t t = 0; t < plan.n_halo(); ++t) brp[nbl + t + 1] = P.rp[nbl] + G.rp[t + 1];
        const int64_t bl = P.nnz(), bnnz = brp.back();
        DevBuf<long long> d_brp, d_bcol;
        DevBuf<double> d_bval;
        d_brp.upload(brp.data(), brp.size());
        d_bcol.alloc((size_t)std::max<int64_t>(bnnz, 1));
        d_bval.alloc((size_t)std::max<int64_t>(bnnz, 1));
        DevCsr& dP = im.get(P);
        dP.ensure_col64(s);
        if (bl) {
            HIP_CHECK(hipMemcpyAsync(d_bcol.p, dP.col64.p, sizeof(long long) * bl, hipMemcpyDeviceToDevice, s));
            HIP_CHECK(hipMemcpyAsync(d_bval.p, dP.val.p, sizeof(double) * bl, hipMemcpyDeviceToDevice, s));
        }
        HIP_CHECK(hipStreamSynchronize(s));
        copy_to_device(d_bcol.p + bl, G.col.data(), sizeof(long long) * (bnnz - bl));
        copy_to_device(d_bval.p + bl, G.val.data(), sizeof(double) * (bnnz - bl));
        DevCsr& dA = im.get(A);
        DevBuf<int> acol;
        const std::vector<int64_t> ub = device_column_map(s, dA, plan, lo, hi, nbl, d_brp.p, acol);
        tm.lap("    galerkin: A P column map (device), P image");
        BImage img{brp.data(), d_brp.p, d_bcol.p, d_bval.p, P.n_global_cols,
                   [&](std::function<int64_t(long long)>& ca, std::function<double(long long)>& va) {
                       ca = [&](long long q) -> int64_t { return q < bl ? P.col[q] : G.col[q - bl]; };
                       va = [&](long long q) -> double { return q < bl ? P.val[q] : G.val[q - bl]; };
                   }};
        const AOperand aop{&A,
                           [&](int64_t k) -> int64_t {
                               const int64_t c = A.col[k];
                               return (c >= lo && c < hi) ? c - lo : nbl + plan.find(c);
                           },
                           dA.rp64.p, acol.p, dA.val.p};
        spgemm_core(ctx, tm, aop, ub, img, AP);
    }
    // ---- ghost rows of A P for R's off-rank columns, gathered on the device
    const int64_t nl = A.nrows(), lo = A.row_starts[comm.rank], hi = A.row_starts[comm.rank + 1];
    HaloPlan rplan = halo_plan_for_cols(comm, R);
    std::vector<int64_t> len(nl), hlen(rplan.n_halo());
    for (int64_t i = 0; i < nl; ++i) len[i] = AP.rp[i + 1] - AP.rp[i];
    rplan.forward(comm, len.data(), hlen.data());
    std::vector<long long> grp(rplan.n_halo() + 1, 0);
    for (int64_t t = 0; t < rplan.n_halo(); ++t) grp[t + 1] = grp[t] + hlen[t];
    const int64_t nsend = (int64_t)rplan.send_idx.size();
    std::vector<long long> soff(nsend + 1, 0);
    for (int64_t t = 0; t < nsend; ++t) soff[t + 1] = soff[t] + len[rplan.send_idx[t]];
    std::vector<PackRec> sbuf((size_t)soff[nsend]), rbuf((size_t)grp.back());
    if (nsend > 0 && soff[nsend] > 0) {
        DevBuf<long long> d_rows, d_off;
        DevBuf<PackRec> d_out;
        std::vector<long long> rows(rplan.send_idx.begin(), rplan.send_idx.end());
        d_rows.upload(rows.data(), rows.size());
        d_off.upload(soff.data(), soff.size());
        d_out.alloc((size_t)soff[nsend]);
        for (int64_t w0 = 0; w0 < nsend; w0 += (int64_t)1 << 24) {
            const int cnt = (int)std::min<int64_t>((int64_t)1 << 24, nsend - w0);
            hipLaunchKernelGGL(pack_rows_kernel, dim3(cnt), dim3(kWave), 0, s, cnt, d_rows.p + w0, d_off.p + w0,
                               AP.d_rp.p, AP.d_col.p, AP.d_val.p, d_out.p);
        }
        HIP_CHECK(hipGetLastError());
        copy_to_host(sbuf.data(), d_out.p, sizeof(PackRec) * sbuf.size(), s);
    }
    std::vector<int64_t> sb(comm.nranks, 0), rb(comm.nranks, 0);
    for (size_t p = 0; p < rplan.send_procs.size(); ++p)
        sb[rplan.send_procs[p]] = (soff[rplan.send_ptr[p + 1]] - soff[rplan.send_ptr[p]]) * (int64_t)sizeof(PackRec);
    for (size_t p = 0; p < rplan.recv_procs.size(); ++p)
        rb[rplan.recv_procs[p]] = (grp[rplan.recv_ptr[p + 1]] - grp[rplan.recv_ptr[p]]) * (int64_t)sizeof(PackRec);
    comm.alltoallv(sbuf.data(), sb, rbuf.data(), rb);
    std::vector<PackRec>().swap(sbuf);
    tm.lap("    galerkin: ghost rows of A P (device gather, exchange)");
    // ---- R (A P): B image = [A P's rows (device to device) | ghost rows]
    const int64_t apl = AP.nnz(), gnnz = grp.back(), bnnz = apl + gnnz;
    std::vector<long long> brp(nl + rplan.n_halo() + 1);
    for (int64_t r = 0; r <= nl; ++r) brp[r] = AP.rp[r];
    for (int64_t t = 0; t < rplan.n_halo(); ++t) brp[nl + t + 1] = apl + grp[t + 1];
    DevBuf<long long> d_brp, d_bcol;
    DevBuf<double> d_bval;
    d_brp.upload(brp.data(), brp.size());
    d_bcol.alloc((size_t)std::max<int64_t>(bnnz, 1));
    d_bval.alloc((size_t)std::max<int64_t>(bnnz, 1));
    if (apl) {
        HIP_CHECK(hipMemcpyAsync(d_bcol.p, AP.d_col.p, sizeof(long long) * apl, hipMemcpyDeviceToDevice, s));
        HIP_CHECK(hipMemcpyAsync(d_bval.p, AP.d_val.p, sizeof(double) * apl, hipMemcpyDeviceToDevice, s));
    }
    if (gnnz) {
        DevBuf<PackRec> d_in;
        d_in.upload(rbuf.data(), rbuf.size());
        hipLaunchKernelGGL(unpack_recs_kernel, dim3((unsigned)((gnnz + 255) / 256)), dim3(256), 0, s, (long long)gnnz,
                           d_in.p, d_bcol.p + apl, d_bval.p + apl);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipStreamSynchronize(s));  // d_in is freed at the end of this scope
    }
    DevCsr& dR = im.get(R);
    DevBuf<int> rcol;
    const std::vector<int64_t> rub = device_column_map(s, dR, rplan, lo, hi, nl, d_brp.p, rcol);
    AP.d_col.reset();
    AP.d_val.reset();
    tm.lap("    galerkin: R column map, A P image");
    // host copies of the image only if some row of R (A P) overflows the LDS tables
    std::vector<long long> hc;
    std::vector<double> hv;
    BImage img{brp.data(), d_brp.p, d_bcol.p, d_bval.p, P.n_global_cols,
               [&](std::function<int64_t(long long)>& ca, std::function<double(long long)>& va) {
                   hc.resize(bnnz);
                   hv.resize(bnnz);
                   copy_to_host(hc.data(), d_bcol.p, sizeof(long long) * bnnz, s);
                   copy_to_host(hv.data(), d_bval.p, sizeof(double) * bnnz, nullptr);
                   ca = [&](long long q) -> int64_t { return hc[q]; };
                   va = [&](long long q) -> double { return hv[q]; };
               }};
    DevCSR64 RAP;
    const AOperand rop{&R,
                       [&](int64_t k) -> int64_t {
                           const int64_t c = R.col[k];
                           return (c >= lo && c < hi) ? c - lo : nl + rplan.find(c);
                       },
                       dR.rp64.p, rcol.p, dR.val.p};
    spgemm_core(ctx, tm, rop, rub, img, RAP);
    HostCSR out = download(ctx, tm, R, P, RAP);
    if (imgs) {  // the next level's operator (its strength / splitting and products)
        std::unique_ptr<DevCsr> d(new DevCsr());
        d->rp64 = std::move(RAP.d_rp);
        d->col64 = std::move(RAP.d_col);
        d->val = std::move(RAP.d_val);
        imgs->put(out, std::move(d));
    }
    return out;
}

}  // namespace

// R (A P) with A P kept on the device between the two products (one rank: no ghost rows, so
// A P's rows are the B image of the second product as they stand; several ranks:
// galerkin_device_dist, the ghost rows of A P gathered on the device).
HostCSR galerkin_device(Context& ctx, const HostComm& comm, const HostCSR& R, const HostCSR& A,
                        const HostCSR& P, SetupImages* imgs) {
    if (comm.nranks > 1) return galerkin_device_dist(ctx, comm, R, A, P, imgs);
    AMG_CHECK(A.col_starts == P.row_starts && R.col_starts == A.row_starts, "galerkin: partitions differ");
    PhaseTimer tm(comm);
    // one rank: A's (global = local) columns are P's rows, R's are A P's rows; all three
    // operands are read from their device images (uploaded here unless the setup holds them)
    SetupImages local;
    SetupImages& im = imgs ? *imgs : local;
    DevCsr& dA = im.get(A);
    DevCsr& dP = im.get(P);
    DevCsr& dR = im.get(R);
    tm.lap("    galerkin: device images of A, P, R");
    DevCSR64 AP;
    spgemm_images(ctx, tm, A, dA, reinterpret_cast<const long long*>(P.rp.data()), &P, dP, P.n_global_cols, AP);
    DevCsr dAP;  // A P as the B image of the second product, where it was computed
    dAP.n = A.nrows();
    dAP.nnz = AP.nnz();
    dAP.ncols = P.n_global_cols;
    dAP.rp64 = std::move(AP.d_rp);
    dAP.col64 = std::move(AP.d_col);
    dAP.val = std::move(AP.d_val);
    DevCSR64 RAP;
    spgemm_images(ctx, tm, R, dR, AP.rp.data(), nullptr, dAP, P.n_global_cols, RAP);
    dAP = DevCsr();
    HostCSR out = download(ctx, tm, R, P, RAP);
    if (imgs) {  // the next level's operator, for its strength / aggregation and products
        std::unique_ptr<DevCsr> d(new DevCsr());
        d->rp64 = std::move(RAP.d_rp);
        d->col64 = std::move(RAP.d_col);
        d->val = std::move(RAP.d_val);
        imgs->put(out, std::move(d));
    }
    return out;
}

}  // namespace amg
