// formats.hip -- the per-nonzero parts of the CSR-stream formats built on the GPU
// (DESIGN.md 4.3): block-aligned col / val streams, fixed-stride x-tile line ids, per-entry
// tile indices (lane-major), the value index (per-block sorted tables of distinct value bit
// patterns, 1-byte indices, diagonal table slots) and per-row ends.  The host keeps what is
// sequential -- the greedy row-block cut (x tiles) and the 32-byte block headers -- and hands
// the cut over as block / tile arrays.  Every output is byte-identical to the host builders
// in par_matrix.hip, which AMG_DEVICE_FORMATS=0 selects (tests/test_gpu_formats.py compares
// the two).
#include "device.hpp"

namespace amg {

namespace {

constexpr int kT = 256;
static_assert(kT == kTPB && kTileLines % kT == 0 && kTileLinesMax % kT == 0, "one thread per lane");

__device__ __forceinline__ size_t lane_pos_d(int j, int nu) {
    return (size_t)((j & (2 * kTPB - 1)) >> 1) * (size_t)nu + 2 * (size_t)(j / (2 * kTPB)) + (size_t)(j & 1);
}

__device__ __forceinline__ int gather_slots_d(int nz) { return nz > 4 * kTPB ? 8 : nz > 2 * kTPB ? 4 : 2; }

__device__ __forceinline__ unsigned long long bits_of(double v) { return (unsigned long long)__double_as_longlong(v); }

// block q's entries to its even offset koff[q] (16-byte aligned value pairs)
__global__ __launch_bounds__(kT) void copy_blocks_kernel(const int2* __restrict__ blocks, const int* __restrict__ rp,
                                                         const int* __restrict__ col, const double* __restrict__ val,
                                                         const long long* __restrict__ koff, int* __restrict__ cb,
                                                         double* __restrict__ vb) {
    const int q = blockIdx.x;
    const int2 b = blocks[q];
    const int kb = rp[b.x], nz = rp[b.y] - kb;
    const long long o = koff[q];
    for (int j = threadIdx.x; j < nz; j += kT) {
        cb[o + j] = col[kb + j];
        vb[o + j] = val[kb + j];
    }
}

// x-tile line ids at a fixed stride, padded with the block's last line (0 for untiled blocks)
__global__ __launch_bounds__(kT) void tile_fixed_kernel(const int* __restrict__ tile_ptr,
                                                        const int* __restrict__ tile_lines, int tl,
                                                        int* __restrict__ fx) {
    const int q = blockIdx.x;
    const int t0 = tile_ptr[q], nt = tile_ptr[q + 1] - t0;
    for (int j = threadIdx.x; j < tl; j += kT)
        fx[(size_t)q * tl + j] = (nt > 0 && nt <= tl) ? tile_lines[t0 + min(j, nt - 1)] : 0;
}

// per entry: slot of its x line in the block's sorted tile * lw + element in the line,
// lane-major (lane_pos); blocks over kCAP entries or without a tile keep zeros
__global__ __launch_bounds__(kT) void tile_index_kernel(const int2* __restrict__ blocks, const int* __restrict__ rp,
                                                        const int* __restrict__ col, const int* __restrict__ tile_ptr,
                                                        const int* __restrict__ tile_lines, int ncl, int lw,
                                                        uint16_t* __restrict__ perm) {
    const int q = blockIdx.x;
    const int2 b = blocks[q];
    const int kb = rp[b.x], nz = rp[b.y] - kb;
    const int t0 = tile_ptr[q], nt = tile_ptr[q + 1] - t0;
    if (nz > kCAP || nt <= 0 || nt > kCAP / lw) return;
    const int sh = lw == 8 ? 3 : 2;
    const int hl0 = (int)(((long long)ncl + lw - 1) / lw);
    for (int j = threadIdx.x; j < nz; j += kT) {
        const int c = col[kb + j];
        const int L = c < ncl ? c >> sh : hl0 + ((c - ncl) >> sh);
        const int e = c < ncl ? (c & (lw - 1)) : ((c - ncl) & (lw - 1));
        int lo = 0, hi = nt;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (tile_lines[t0 + mid] < L) lo = mid + 1;
            else hi = mid;
        }
        perm[(size_t)q * kCAP + lane_pos_d(j, kCAP / kTPB)] = (uint16_t)(lo * lw + e);
    }
}

// the block's value bit patterns sorted ascending in keys[0, nz); returns the padded size
__device__ int load_sorted(unsigned long long* keys, const double* __restrict__ val, int kb, int nz) {
    int P = 1;
    while (P < nz) P <<= 1;
    for (int t = threadIdx.x; t < P; t += kT) keys[t] = t < nz ? bits_of(val[kb + t]) : ~0ull;
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1)
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
            for (int t = threadIdx.x; t < P; t += kT) {
                const int u = t ^ jj;
                if (u > t) {
                    const unsigned long long a = keys[t], c = keys[u];
                    if (((t & k) == 0) == (a > c)) {
                        keys[t] = c;
                        keys[u] = a;
                    }
                }
            }
            __syncthreads();
        }
    return P;
}

// distinct values per block with 1..kCAP entries: the table size if <= 256, else 0
__global__ __launch_bounds__(kT) void vi_count_kernel(const int2* __restrict__ blocks, const int* __restrict__ rp,
                                                      const double* __restrict__ val, int* __restrict__ tsz) {
    __shared__ unsigned long long keys[kCAP];
    __shared__ int cnt;
    const int q = blockIdx.x;
    const int2 b = blocks[q];
    const int kb = rp[b.x], nz = rp[b.y] - kb;
    if (nz == 0 || nz > kCAP) {
        if (threadIdx.x == 0) tsz[q] = 0;
        return;
    }
    if (threadIdx.x == 0) cnt = 0;
    load_sorted(keys, val, kb, nz);
    int c = 0;
    for (int t = threadIdx.x; t < nz; t += kT) c += t == 0 || keys[t] != keys[t - 1];
    atomicAdd(&cnt, c);
    __syncthreads();
    if (threadIdx.x == 0) tsz[q] = cnt <= 256 ? cnt : 0;
}

struct ViArgs {
    const int2* blocks;
    const int* rp;
    const int* col;
    const double* val;
    const int* tptr;         // per block: table offset, -1 = value stream
    const long long* vofs;   // per block: offset in the index stream
    double* tab;
    uint8_t* idx;
    uint8_t* dvi;            // square: per row, table slot of a_ii
    uint8_t* dvi_ok;         // square: per block, every row has a nonzero diagonal
    int tiled, square;
};

// the table (sorted distinct bit patterns), each entry's index, and the diagonal slots
__global__ __launch_bounds__(kT) void vi_fill_kernel(ViArgs a) {
    __shared__ unsigned long long keys[kCAP];
    __shared__ unsigned long long utab[256];
    __shared__ int tsum[kT];
    __shared__ int ok;
    const int q = blockIdx.x;
    if (a.tptr[q] < 0) return;
    const int2 b = a.blocks[q];
    const int kb = a.rp[b.x], nz = a.rp[b.y] - kb;
    load_sorted(keys, a.val, kb, nz);
    // compact: thread t owns the run [t * per, (t + 1) * per) of the sorted keys
    const int per = (nz + kT - 1) / kT, t0 = threadIdx.x * per, t1 = min(t0 + per, nz);
    int c = 0;
    for (int t = t0; t < t1; ++t) c += t == 0 || keys[t] != keys[t - 1];
    tsum[threadIdx.x] = c;
    if (threadIdx.x == 0) ok = 1;
    __syncthreads();
    if (threadIdx.x == 0)
        for (int t = 1; t < kT; ++t) tsum[t] += tsum[t - 1];
    __syncthreads();
    int u = threadIdx.x == 0 ? 0 : tsum[threadIdx.x - 1];
    for (int t = t0; t < t1; ++t)
        if (t == 0 || keys[t] != keys[t - 1]) utab[u++] = keys[t];
    __syncthreads();
    const int nu = tsum[kT - 1];
    for (int t = threadIdx.x; t < nu; t += kT) a.tab[a.tptr[q] + t] = __longlong_as_double((long long)utab[t]);
    auto slot = [&](unsigned long long key) {
        int lo = 0, hi = nu;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (utab[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    const long long base = a.vofs[q];
    const int gs = gather_slots_d(nz);
    for (int j = threadIdx.x; j < nz; j += kT) {
        const size_t pos = a.tiled ? lane_pos_d(j, kCAP / kTPB) : (size_t)(j % kTPB) * gs + (size_t)(j / kTPB);
        a.idx[base + pos] = (uint8_t)slot(bits_of(a.val[kb + j]));
    }
    if (!a.square) return;
    for (int r = b.x + threadIdx.x; r < b.y; r += kT) {
        int k = a.rp[r];
        const int e = a.rp[r + 1];
        while (k < e && a.col[k] != r) ++k;  // local column r is the diagonal (square: rows = columns)
        if (k == e || a.val[k] == 0.0) {
            ok = 0;
            continue;
        }
        a.dvi[r] = (uint8_t)slot(bits_of(a.val[k]));
    }
    __syncthreads();
    if (threadIdx.x == 0) a.dvi_ok[q] = (uint8_t)ok;
}

// per row: end of its nonzeros relative to its block's first (blocks of <= kCAP entries)
__global__ __launch_bounds__(kT) void row_end_kernel(const int2* __restrict__ blocks, const int* __restrict__ rp,
                                                     uint16_t* __restrict__ re) {
    const int q = blockIdx.x;
    const int2 b = blocks[q];
    if (rp[b.y] - rp[b.x] > kCAP) return;
    for (int r = b.x + threadIdx.x; r < b.y; r += kT) re[r] = (uint16_t)(rp[r + 1] - rp[b.x]);
}

int host_gather_slots(int nz) { return nz > 4 * kTPB ? 8 : nz > 2 * kTPB ? 4 : 2; }

}  // namespace

// AMG_DEVICE_FORMATS=0: the host builders (A/B and the format-identity test; read at every
// build, so one process can build an operator both ways)
bool device_formats() {
    const char* e = std::getenv("AMG_DEVICE_FORMATS");
    return !(e && *e && std::atoi(e) == 0);
}

void build_formats_device(DevMatrix& M, const std::vector<int>& hrp, const hvec<int>& hcol, const hvec<double>& hval,
                          const std::vector<int2>& blocks, const std::vector<int>& tile_ptr,
                          const std::vector<int>& tile_lines, const std::vector<int64_t>& koff, FormatHeaderInfo& out) {
    const int nbk = (int)blocks.size();
    const int64_t nnz = (int64_t)hcol.size() - kPad;  // hcol carries kPad trailing zeros
    AMG_CHECK(nnz == hrp.back(), "format build: column array size");
    // a stream of the build's own: the worker thread's builds run beside the setup thread's
    // kernels on the context stream
    hipStream_t s = nullptr;
    HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    struct StreamGuard {
        hipStream_t s;
        ~StreamGuard() { (void)hipStreamDestroy(s); }
    } sg{s};
    // the CSR in local numbering (rp is M.rp, uploaded by the caller)
    DevBuf<int> dcol, dtp, dtl;
    DevBuf<double> dval;
    DevBuf<long long> dkoff;
    dcol.upload(hcol.data(), (size_t)std::max<int64_t>(nnz, 1));
    dval.upload(hval.data(), (size_t)std::max<int64_t>(nnz, 1));
    dtp.upload(tile_ptr.data(), tile_ptr.size());
    dtl.upload(tile_lines.data(), std::max<size_t>(tile_lines.size(), 1));
    static_assert(sizeof(long long) == sizeof(int64_t), "int64 offsets");
    dkoff.upload(reinterpret_cast<const long long*>(koff.data()), koff.size());
    const size_t nstream = (size_t)(koff[nbk] + kPad);
    M.col.alloc(nstream);
    M.val.alloc(nstream);
    HIP_CHECK(hipMemsetAsync(M.col.p, 0, nstream * sizeof(int), s));
    HIP_CHECK(hipMemsetAsync(M.val.p, 0, nstream * sizeof(double), s));
    if (nbk)
        hipLaunchKernelGGL(copy_blocks_kernel, dim3(nbk), dim3(kT), 0, s, M.blocks.p, M.rp.p, dcol.p, dval.p, dkoff.p,
                           M.col.p, M.val.p);
    HIP_CHECK(hipGetLastError());
    if (M.tiled) {
        M.tile_fixed.alloc((size_t)std::max(nbk, 1) * (kCAP / M.line_w));
        M.lcol.alloc((size_t)std::max(nbk, 1) * kCAP);
        HIP_CHECK(hipMemsetAsync(M.tile_fixed.p, 0, M.tile_fixed.n * sizeof(int), s));
        HIP_CHECK(hipMemsetAsync(M.lcol.p, 0, M.lcol.n * sizeof(uint16_t), s));
        if (nbk) {
            hipLaunchKernelGGL(tile_fixed_kernel, dim3(nbk), dim3(kT), 0, s, dtp.p, dtl.p, kCAP / M.line_w,
                               M.tile_fixed.p);
            hipLaunchKernelGGL(tile_index_kernel, dim3(nbk), dim3(kT), 0, s, M.blocks.p, M.rp.p, dcol.p, dtp.p, dtl.p,
                               (int)M.n_cols_local, M.line_w, M.lcol.p);
        }
        HIP_CHECK(hipGetLastError());
    } else {
        M.tile_fixed.reset();
        M.lcol.reset();
    }
    // value index: table sizes, offsets on the host, then tables / indices / diagonal slots
    out.vt_off.assign((size_t)nbk, -1);
    out.vt_len.assign((size_t)nbk, 0);
    out.dvi_ok.assign((size_t)nbk, 0);
    out.vofs.clear();
    std::vector<int> tsz((size_t)std::max(nbk, 1), 0);
    {
        DevBuf<int> dtsz;
        dtsz.alloc((size_t)std::max(nbk, 1));
        if (nbk) hipLaunchKernelGGL(vi_count_kernel, dim3(nbk), dim3(kT), 0, s, M.blocks.p, M.rp.p, dval.p, dtsz.p);
        HIP_CHECK(hipGetLastError());
        copy_to_host(tsz.data(), dtsz.p, sizeof(int) * (size_t)nbk, s);
    }
    int64_t total = 0, vin = 0;
    int nvi = 0;
    for (int q = 0; q < nbk; ++q)
        if (tsz[q] > 0) {
            out.vt_off[q] = (int)total;
            out.vt_len[q] = tsz[q];
            total += tsz[q];
            vin += hrp[blocks[q].y] - hrp[blocks[q].x];
            ++nvi;
        }
    M.n_vi_blocks = nvi;
    M.vi_nnz = vin;
    if (nvi == 0) {
        M.vtab.reset();
        M.vidx.reset();
        M.dvi.reset();
    } else {
        AMG_CHECK(total < INT_MAX, "value tables too large");
        out.vofs.assign((size_t)nbk + 1, 0);
        for (int q = 0; q < nbk; ++q) {
            const int nz = hrp[blocks[q].y] - hrp[blocks[q].x];
            out.vofs[q + 1] = out.vofs[q] + (M.tiled ? kCAP : tsz[q] == 0 ? 0 : host_gather_slots(nz) * kTPB);
        }
        AMG_CHECK(out.vofs[nbk] < INT_MAX, "value index stream too large");
        DevBuf<int> dtptr;
        DevBuf<long long> dvofs;
        DevBuf<uint8_t> dok;
        dtptr.upload(out.vt_off.data(), (size_t)nbk);
        dvofs.upload(reinterpret_cast<const long long*>(out.vofs.data()), out.vofs.size());
        dok.alloc((size_t)nbk);
        M.vtab.alloc((size_t)total);
        M.vidx.alloc((size_t)out.vofs[nbk] + 16);
        HIP_CHECK(hipMemsetAsync(M.vidx.p, 0, M.vidx.n, s));
        HIP_CHECK(hipMemsetAsync(dok.p, 0, dok.n, s));
        if (M.square) {
            M.dvi.alloc((size_t)M.n_rows + 1);
            HIP_CHECK(hipMemsetAsync(M.dvi.p, 0, M.dvi.n, s));
        } else {
            M.dvi.reset();
        }
        ViArgs va{M.blocks.p, M.rp.p, dcol.p, dval.p, dtptr.p, dvofs.p, M.vtab.p, M.vidx.p,
                  M.square ? M.dvi.p : nullptr, dok.p, M.tiled ? 1 : 0, M.square ? 1 : 0};
        hipLaunchKernelGGL(vi_fill_kernel, dim3(nbk), dim3(kT), 0, s, va);
        HIP_CHECK(hipGetLastError());
        std::vector<uint8_t> okh((size_t)nbk);
        copy_to_host(okh.data(), dok.p, (size_t)nbk, s);
        for (int q = 0; q < nbk; ++q) out.dvi_ok[q] = (char)okh[q];
    }
    M.rend.alloc((size_t)M.n_rows + 1);
    HIP_CHECK(hipMemsetAsync(M.rend.p, 0, M.rend.n * sizeof(uint16_t), s));
    if (nbk) hipLaunchKernelGGL(row_end_kernel, dim3(nbk), dim3(kT), 0, s, M.blocks.p, M.rp.p, M.rend.p);
    HIP_CHECK(hipGetLastError());
    // one rank, square, no halo: the local columns are the global ones -- the uploaded CSR is
    // the solver setup's level-0 image (DevMatrix::setup_csr)
    if (M.keep_setup_csr && M.square && !M.replicated && M.ctx->host.nranks == 1 && M.first_col == 0 &&
        M.plan.n_halo() == 0) {
        std::unique_ptr<DevCsr> d(new DevCsr());
        d->rp32.alloc((size_t)M.n_rows + 1);
        HIP_CHECK(hipMemcpyAsync(d->rp32.p, M.rp.p, sizeof(int) * (M.n_rows + 1), hipMemcpyDeviceToDevice, s));
        d->col32 = std::move(dcol);
        d->val = std::move(dval);
        M.setup_csr = std::move(d);
    }
    HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace amg
