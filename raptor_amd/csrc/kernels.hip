// kernels.hip -- hand-written gfx950 kernels for the AMG level operations.
// SURVEY.md 8a rows a2-a6; DESIGN.md section 4 (layout, rooflines).
//
// CSR-stream SpMV family (HBM-bound, AI ~0.13 flop/B; no MFMA):
//   one 256-thread workgroup per row block of <= kCAP nonzeros and <= 256 rows;
//   phase 1: the workgroup streams the block's col/val ranges with consecutive lanes on
//            consecutive nonzeros (fully coalesced, nontemporal: each byte is read once),
//            gathers x (L2 / Infinity-Cache resident) and stages products in LDS;
//   phase 2: one lane per row sums its products sequentially in CSR order and applies the
//            fused epilogue (SpMV, y += Ax, residual, Jacobi).
// Products are rounded and summed exactly as the oracle does (-ffp-contract=off), so the
// kernels are bit-identical to oracle/amg_oracle.c.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "device.hpp"

namespace amg {

namespace {

struct CsrArgs {
    const int2* blocks;
    const int* rp;
    const int* col;
    const double* val;
    const double* x;   // local part of x
    const double* xh;  // halo part of x
    int ncl;           // number of local columns
    const double* b;
    const double* dinv;
    double* y;
    double omega;
    double* partial;
    const int* tile_ptr;     // x tiles (par_matrix.hip build_row_blocks)
    const int* tile_lines;
    const uint16_t* lcol;
    int hl0;                 // first halo line id = ceil(ncl / 8)
    int nhalo;
    const int* vt_ptr;       // value-indexed blocks: table offset, -1 = value stream
    const double* vtab;
    const uint8_t* vidx;     // lane-major 1-byte indices (8 per lane per block)
};

__device__ __forceinline__ double xload(const CsrArgs& a, int c) {
    const double* p = c < a.ncl ? a.x + c : a.xh + (c - a.ncl);
    return *p;
}

// fused epilogue; *res receives b - s for the residual and Jacobi modes (for the norm)
template <int MODE>
__device__ __forceinline__ double epilogue(const CsrArgs& a, int r, double s, double* res) {
    if (MODE == KM_SPMV) return s;
    if (MODE == KM_SPMV_ADD) return a.y[r] + s;
    const double t = a.b[r] - s;
    *res = t;
    if (MODE == KM_RESID) return t;
    // Jacobi: x + omega * (dinv * (b - s))
    return a.x[r] + a.omega * (a.dinv[r] * t);
}

// XCD-aware bijection: consecutive row blocks land on the same XCD (blocks b and b+8 share
// one under round-robin dispatch), so a row block's x neighbours (+-nx*ny rows) are in the
// same L2.  Placement only changes speed, never results (MI355X_MICROARCH.md).
__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int q = nb >> 3, rem = nb & 7, x = b & 7;
    return x * q + min(x, rem) + (b >> 3);
}

// Blocks hold <= kTPB rows, so lane t owns at most row r0 + t.  Its row bounds and
// epilogue operands are loaded at entry, in flight together with the phase-1 stream, so
// the epilogue costs no extra memory round trip after the barrier.
//
// TILE: instead of gathering x from global memory per nonzero, the workgroup first loads its
// x tile (the block's distinct 64-byte lines, coalesced: 8 lanes per line) into LDS while the
// val / 16-bit tile-index streams are in flight; products then read x from LDS.  Same
// products, same order: bit-identical to the gather path and the oracle.
//
// VI (value-indexed CSR): a block whose nonzeros take at most 256 distinct values (by bit
// pattern) streams a 1-byte index per nonzero (lane-major, one 8-byte load per lane) and
// reads the values from its small table (L1/L2-resident) instead of streaming 8 bytes per
// nonzero.  The table holds the exact fp64 bits, so products are unchanged.
template <int MODE, bool NORM, bool XCD, bool TILE, bool VI>
__global__ __launch_bounds__(kTPB) void csr_stream_kernel(CsrArgs a, int first_block) {
    // one 16 KiB stage: first the x tile, then (after the products are in registers) the
    // products -- the same LDS footprint as the gather path, so the same occupancy
    static_assert(kTileLines * 8 <= kCAP, "x tile must fit the product stage");
    __shared__ double prod[kCAP];
    double* const xt = prod;
    __shared__ double red[kTPB / 64];
    const int bid = first_block + (XCD ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x);
    const int2 br = a.blocks[bid];
    const int r0 = br.x, r1 = br.y;
    const int tid = threadIdx.x;
    const int r = r0 + tid;
    const bool own = r < r1;
    const int k0 = a.rp[r0];
    const int nnz = a.rp[r1] - k0;
    int e0 = 0, e1 = 0;
    double pb = 0.0, pd = 0.0, px = 0.0;
    if (own) {
        e0 = a.rp[r] - k0;
        e1 = a.rp[r + 1] - k0;
        if (MODE == KM_SPMV_ADD) px = a.y[r];
        if (MODE == KM_RESID || MODE == KM_JACOBI) pb = a.b[r];
        if (MODE == KM_JACOBI) {
            pd = a.dinv[r];
            px = a.x[r];
        }
    }
    double sq = 0.0;
    const int t0 = TILE ? a.tile_ptr[bid] : 0;
    const int ntl = TILE ? a.tile_ptr[bid + 1] - t0 : 0;
    if (nnz <= kCAP && (!TILE || ntl <= kTileLines)) {
        constexpr int U = kCAP / kTPB;  // 8 nonzeros per lane
        double v[U];
        const int vt = VI ? a.vt_ptr[bid] : -1;  // block-uniform
        auto load_vals = [&]() {
            if (VI && vt >= 0) {
                typedef unsigned int v2u __attribute__((ext_vector_type(2)));
                const v2u q = __builtin_nontemporal_load(
                    (const v2u*)(a.vidx + (size_t)bid * kCAP + (size_t)tid * U));
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const unsigned w = u < 4 ? q.x : q.y;
                    const int k = tid + u * kTPB;
                    if (k < nnz) v[u] = a.vtab[vt + ((w >> (8 * (u & 3))) & 0xffu)];
                }
            } else {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int k = tid + u * kTPB;
                    if (k < nnz) v[u] = __builtin_nontemporal_load(a.val + k0 + k);
                }
            }
        };
        if (TILE) {
            static_assert(U == 8, "lane-major tile indices assume 8 entries per lane");
            typedef unsigned int v4u __attribute__((ext_vector_type(4)));
            const v4u q = __builtin_nontemporal_load(
                (const v4u*)(a.lcol + (size_t)bid * kCAP + (size_t)tid * U));
            const unsigned li[U] = {q.x & 0xffffu, q.x >> 16, q.y & 0xffffu, q.y >> 16,
                                    q.z & 0xffffu, q.z >> 16, q.w & 0xffffu, q.w >> 16};
            load_vals();
            // x tile: element e of line L is column 8L + e (local) or halo entry 8(L - hl0) + e
            // fixed 8 slots per lane, fully unrolled: all line ids, then all x loads in flight
            constexpr int TU = kTileLines * 8 / kTPB;
            const int nt = ntl * 8;
            int Ls[TU];
#pragma unroll
            for (int j = 0; j < TU; ++j) {
                const int idx = tid + j * kTPB;
                Ls[j] = idx < nt ? a.tile_lines[t0 + (idx >> 3)] : 0;
            }
            double xs[TU];
#pragma unroll
            for (int j = 0; j < TU; ++j) {
                const int idx = tid + j * kTPB, e = idx & 7, L = Ls[j];
                const double* p = nullptr;
                if (idx < nt) {
                    if (L < a.hl0) {
                        const int c = L * 8 + e;
                        if (c < a.ncl) p = a.x + c;
                    } else {
                        const int h = (L - a.hl0) * 8 + e;
                        if (h < a.nhalo) p = a.xh + h;
                    }
                }
                xs[j] = p ? *p : 0.0;
            }
#pragma unroll
            for (int j = 0; j < TU; ++j) {
                const int idx = tid + j * kTPB;
                if (idx < nt) xt[idx] = xs[j];
            }
            __syncthreads();
            double pr[U];
#pragma unroll
            for (int u = 0; u < U; ++u) pr[u] = v[u] * xt[li[u]];
            __syncthreads();  // every lane has read the tile; reuse it for the products
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int k = tid + u * kTPB;
                if (k < nnz) prod[k] = pr[u];
            }
        } else {
            int c[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int k = tid + u * kTPB;
                if (k < nnz) c[u] = __builtin_nontemporal_load(a.col + k0 + k);
            }
            load_vals();
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int k = tid + u * kTPB;
                if (k < nnz) prod[k] = v[u] * xload(a, c[u]);
            }
        }
        __syncthreads();
        if (own) {
            double s = 0.0;
            for (int k = e0; k < e1; ++k) s += prod[k];
            double out;
            if (MODE == KM_SPMV) {
                out = s;
            } else if (MODE == KM_SPMV_ADD) {
                out = px + s;
            } else {
                const double t = pb - s;
                if (NORM) sq = t * t;
                out = MODE == KM_RESID ? t : px + a.omega * (pd * t);
            }
            a.y[r] = out;
        }
    } else {
        // one row longer than the LDS stage: chunked, summed by lane 0 in CSR order
        double s = 0.0;
        for (int base = 0; base < nnz; base += kCAP) {
            const int cnt = min(kCAP, nnz - base);
            for (int k = tid; k < cnt; k += kTPB)
                prod[k] = a.val[k0 + base + k] * xload(a, a.col[k0 + base + k]);
            __syncthreads();
            if (tid == 0)
                for (int k = 0; k < cnt; ++k) s += prod[k];
            __syncthreads();
        }
        if (tid == 0) {
            double res = 0.0;
            a.y[r0] = epilogue<MODE>(a, r0, s, &res);
            if (NORM) sq = res * res;
        }
    }
    if (NORM) {
        // fixed-shape reduction: wave butterfly then 4 wave sums in order
        for (int off = 32; off > 0; off >>= 1) sq += __shfl_down(sq, off, 64);
        if ((tid & 63) == 0) red[tid >> 6] = sq;
        __syncthreads();
        if (tid == 0) a.partial[bid] = (red[0] + red[1]) + (red[2] + red[3]);
    }
}

// l1 hybrid Gauss-Seidel (row a5; definition DESIGN.md 3).  One wavefront per slab of <= 64
// rows (whole GS chunks), lane = row.
//  phase 1: the lane walks its row in the slab's sliced-ELL layout (entry k of all lanes is
//           one coalesced 512-byte load) and subtracts every old-value coupling, diagonal
//           included, in CSR order; the new-value ("chain") couplings -- in-chunk j < i
//           forward, j > i backward -- are contiguous in the sorted row and are skipped.
//  phase 2: the in-chunk triangular solve, column-oriented: at step t the row finishing now
//           (lane t forward, lane n-1-t backward) has its final value; it is broadcast with
//           v_readlane and every lane whose next chain column is that row subtracts
//           a_ij * x_j.  Each lane keeps its next four chain entries in registers and
//           refills from the (cache-hot) sliced-ELL arrays, so chain couplings are consumed
//           in sweep order (ascending j forward, descending j backward) exactly like the
//           oracle, with no LDS and no barrier.
//  x_i' = x_i + acc * dinv_l1.
struct GsArgs {
    const int4* slabs;
    const int* col;      // sliced-ELL, -1 = padding
    const double* val;
    const double* x;
    const double* xh;    // halo values (columns >= ncl)
    int ncl;
    const double* b;
    const double* dinv;  // l1 diagonal inverse
    double* y;
    long long first_row;
    long long B;
    int n;               // local rows (chunks are clipped to the rank)
    int nslab;
    double* partial;     // NORM: per-slab sum of (b - A x_old)^2
};

__device__ __forceinline__ double bcast_lane(double v, int lane) {
    const long long bits = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)bits, lane);
    const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// WIDE (dense coarse operators, average slab width >= kGsWide): one wave per workgroup, the
// slab's chain entries go to LDS as a 64 x 64 column-major block plus a per-lane bit mask in
// phase 1, so the triangular solve never reloads them; phase 1 keeps 16 loads in flight.
// Narrow: 4 waves per workgroup (no LDS), 8 loads in flight, register ring of chain entries.
template <bool BACK, bool WIDE, bool NORM>
__global__ __launch_bounds__(WIDE ? 64 : 256) void hybrid_gs_kernel(GsArgs a) {
    constexpr int U = WIDE ? 16 : 8;
    // wave index made provably uniform: slab fields land in SGPRs, the step loop is scalar
    const int wave = __builtin_amdgcn_readfirstlane(
        (int)(WIDE ? blockIdx.x : blockIdx.x * 4 + (threadIdx.x >> 6)));
    if (wave >= a.nslab) return;
    const int lane = threadIdx.x & 63;
    const int4 sl = a.slabs[wave];
    const int r = sl.x + lane;
    const bool live = lane < sl.y;
    int lo = 0, hi = 0;  // chain (new-value) column range [lo, hi)
    double acc = 0.0, xi = 0.0, dinv = 0.0;
    if (live) {
        const long long g = a.first_row + r;
        long long cs = (g / a.B) * a.B - a.first_row, ce = cs + a.B;
        cs = cs < 0 ? 0 : cs;
        ce = ce > a.n ? a.n : ce;
        lo = BACK ? r + 1 : (int)cs;
        hi = BACK ? (int)ce : r;
        acc = a.b[r];
        xi = a.x[r];
        dinv = a.dinv[r];
    }
    const size_t base = (size_t)sl.z * 64 + lane;
    const int* colp = a.col + base;
    const double* valp = a.val + base;
    __shared__ double chainL[WIDE ? 64 * 64 : 1];
    double s_old = 0.0;           // NORM: sum_j a_ij x_j (old x), for ||b - A x||
    unsigned long long mask = 0;  // WIDE: bit t = coupling to slab row t
    int kf = -1, kl = -1;         // narrow: first / last chain entry of the row
    // software pipeline: block k0 + U's (col, val) stream in while block k0 gathers x
    int cn[U];
    double vn[U];
    auto fetch = [&](int k0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in = k0 + u < sl.w;  // uniform
            cn[u] = in ? __builtin_nontemporal_load(colp + (size_t)(k0 + u) * 64) : -1;
            vn[u] = in ? __builtin_nontemporal_load(valp + (size_t)(k0 + u) * 64) : 0.0;
        }
    };
    fetch(0);
    for (int k0 = 0; k0 < sl.w; k0 += U) {
        int c[U];
        double v[U], xv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) c[u] = cn[u], v[u] = vn[u];
        if (k0 + U < sl.w) fetch(k0 + U);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool old = c[u] >= 0 && (NORM || !(c[u] >= lo && c[u] < hi));
            xv[u] = old ? (c[u] < a.ncl ? a.x[c[u]] : a.xh[c[u] - a.ncl]) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (c[u] < 0) continue;  // padding (also every entry of a dead lane)
            if (NORM) s_old += v[u] * xv[u];  // A x_old in CSR order: the residual's bits
            if (c[u] >= lo && c[u] < hi) {
                if (WIDE) {
                    const int t = c[u] - sl.x;
                    chainL[t * 64 + lane] = v[u];
                    mask |= 1ull << t;
                } else {
                    kf = kf < 0 ? k0 + u : kf;
                    kl = k0 + u;
                }
                continue;
            }
            acc -= v[u] * xv[u];
        }
    }
    if (WIDE) {
        for (int t = 0; t < sl.y; ++t) {
            const int j = BACK ? sl.y - 1 - t : t;  // lane whose row is final now
            const double lv = chainL[j * 64 + lane];
            const double xj = bcast_lane(xi + acc * dinv, j);
            if ((mask >> j) & 1ull) acc -= lv * xj;
        }
    } else {
        // register ring of the next four chain entries, in consumption order
        int c0 = -1, c1 = -1, c2 = -1, c3 = -1;
        double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
        int kn = BACK ? kl : kf;  // next entry to load
        int left = kf < 0 ? 0 : kl - kf + 1;
        auto load = [&](int& cc, double& vv) {
            if (left > 0) {
                cc = colp[(size_t)kn * 64];
                vv = valp[(size_t)kn * 64];
                kn += BACK ? -1 : 1;
                --left;
            } else {
                cc = -1;
            }
        };
        load(c0, v0);
        load(c1, v1);
        load(c2, v2);
        load(c3, v3);
        for (int t = 0; t < sl.y; ++t) {
            const int j = BACK ? sl.y - 1 - t : t;
            const double xj = bcast_lane(xi + acc * dinv, j);
            if (c0 == sl.x + j) {
                acc -= v0 * xj;
                c0 = c1, v0 = v1;
                c1 = c2, v1 = v2;
                c2 = c3, v2 = v3;
                load(c3, v3);
            }
        }
    }
    if (live) a.y[r] = xi + acc * dinv;
    if (NORM) {  // ||b - A x_old||^2 partial of this slab; butterfly order is fixed
        const double rr = live ? a.b[r] - s_old : 0.0;
        double q = rr * rr;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) q += __shfl_xor(q, m);
        if (lane == 0) a.partial[wave] = q;
    }
}

__global__ void jacobi_zero_kernel(long long n, const double* b, const double* dinv, double* y,
                                   double omega) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long stride = (long long)gridDim.x * blockDim.x;
    for (; i < n; i += stride) y[i] = omega * (dinv[i] * b[i]);
}

__global__ void pack_kernel(long long n, const int* idx, const double* x, double* out) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = x[idx[i]];
}

__global__ void zero_kernel(long long n, double* y) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long stride = (long long)gridDim.x * blockDim.x;
    for (; i < n; i += stride) y[i] = 0.0;
}

// deterministic two-stage sum of n partials: block g sums [g*4096, (g+1)*4096) with 16
// fixed loads per lane, a fixed shuffle tree and 4 wave sums in order
constexpr int kRedSpan = kTPB * 16;
__global__ __launch_bounds__(kTPB) void sum_partials_kernel(int n, const double* p, double* out) {
    __shared__ double red[kTPB / 64];
    const int base = blockIdx.x * kRedSpan + threadIdx.x;
    double v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int i = base + j * kTPB;
        v[j] = i < n ? p[i] : 0.0;
    }
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += v[j];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// sum of per-rank sums in rank order (identical on every rank), sqrt, append to hist
__global__ void finish_norm_kernel(int n, const double* in, double* hist, int* counter) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        double s = 0.0;
        for (int i = 0; i < n; ++i) s += in[i];
        hist[*counter] = sqrt(s);
        *counter += 1;
    }
}

// coarsest level: x_i = sum_j inv_ij * b_j, sequential j per lane (bit-identical to the
// oracle); invT is stored column-major for coalesced lanes
__global__ void dense_gemv_kernel(long long nl, long long n, const double* invT,
                                  const double* bfull, double* x) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nl) return;
    double s = 0.0;
    for (long long j = 0; j < n; ++j) s += invT[j * nl + i] * bfull[j];
    x[i] = s;
}

__device__ __forceinline__ unsigned long long dmix64(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void uniform_kernel(long long n, long long first, unsigned long long seed, double* out) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long stride = (long long)gridDim.x * blockDim.x;
    for (; i < n; i += stride) {
        unsigned long long u = dmix64(seed * 0xD1B54A32D192ED03ull + (unsigned long long)(first + i));
        out[i] = (double)(u >> 11) * 0x1.0p-52 - 1.0;
    }
}

inline int grid_for(long long n, int tpb = kTPB) {
    long long g = (n + tpb - 1) / tpb;
    if (g > 256 * 16) g = 256 * 16;
    return (int)(g < 1 ? 1 : g);
}

// ---- PCG vector kernels (row f3) ---------------------------------------------------
// dot partials: block g covers [g*kDotSpan, (g+1)*kDotSpan) with 8 fixed loads per lane,
// fixed shuffle tree, 4 wave sums in order => deterministic for a given n
constexpr int kDotSpan = kTPB * 8;
__global__ __launch_bounds__(kTPB) void dot_partials_kernel(long long n, const double* a,
                                                            const double* b, double* partial) {
    __shared__ double red[kTPB / 64];
    const long long base = (long long)blockIdx.x * kDotSpan + threadIdx.x;
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const long long i = base + (long long)j * kTPB;
        if (i < n) s += a[i] * b[i];
    }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// out = sum_{i<n} in[i] (rank order), optional sqrt
__global__ void finish_sum_kernel(int n, const double* in, double* out, int take_sqrt) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        double s = 0.0;
        for (int i = 0; i < n; ++i) s += in[i];
        *out = take_sqrt ? sqrt(s) : s;
    }
}

// x += (rz/pq) p ; r -= (rz/pq) q
__global__ void pcg_xr_kernel(long long n, const double* rz, const double* pq, const double* p,
                              const double* q, double* x, double* r) {
    const double alpha = *rz / *pq;
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (; i < n; i += stride) {
        x[i] = x[i] + alpha * p[i];
        r[i] = r[i] - alpha * q[i];
    }
}

// p = z + (rz_new/rz_old) p
__global__ void pcg_p_kernel(long long n, const double* rz_new, const double* rz_old,
                             const double* z, double* p) {
    const double beta = *rz_new / *rz_old;
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (; i < n; i += stride) p[i] = z[i] + beta * p[i];
}

__global__ void append_kernel(const double* v, double* hist, int* counter) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        hist[*counter] = *v;
        *counter += 1;
    }
}

}  // namespace

int dot_partial_count(int64_t n) { return (int)std::max<int64_t>(1, (n + kDotSpan - 1) / kDotSpan); }

void launch_dot_partials(hipStream_t s, int64_t n, const double* a, const double* b, double* partial) {
    const int g = dot_partial_count(n);
    hipLaunchKernelGGL(dot_partials_kernel, dim3(g), dim3(kTPB), 0, s, (long long)n, a, b, partial);
    HIP_CHECK(hipGetLastError());
}

void launch_finish_sum(hipStream_t s, int n, const double* in, double* out, bool take_sqrt) {
    hipLaunchKernelGGL(finish_sum_kernel, dim3(1), dim3(64), 0, s, n, in, out, take_sqrt ? 1 : 0);
    HIP_CHECK(hipGetLastError());
}

void launch_pcg_xr(hipStream_t s, int64_t n, const double* rz, const double* pq, const double* p,
                   const double* q, double* x, double* r) {
    if (n <= 0) return;
    hipLaunchKernelGGL(pcg_xr_kernel, dim3(grid_for(n)), dim3(kTPB), 0, s, (long long)n, rz, pq, p, q, x, r);
    HIP_CHECK(hipGetLastError());
}

void launch_pcg_p(hipStream_t s, int64_t n, const double* rz_new, const double* rz_old,
                  const double* z, double* p) {
    if (n <= 0) return;
    hipLaunchKernelGGL(pcg_p_kernel, dim3(grid_for(n)), dim3(kTPB), 0, s, (long long)n, rz_new, rz_old, z, p);
    HIP_CHECK(hipGetLastError());
}

void launch_append(hipStream_t s, const double* v, double* hist, int* counter) {
    hipLaunchKernelGGL(append_kernel, dim3(1), dim3(64), 0, s, v, hist, counter);
    HIP_CHECK(hipGetLastError());
}

// CSR-stream variant: bit 0 = 16-byte vector loads, bit 1 = XCD-aware block order.
// AMG_KERNEL_VARIANT overrides the default (A/B timing; results are identical).
int kernel_variant() {
    const char* e = getenv("AMG_KERNEL_VARIANT");
    return e ? (atoi(e) & 3) : kDefaultVariant;
}

void launch_csr_stream(hipStream_t s, int mode, bool norm, const DevMatrix& A, int first_block,
                       int n_blocks, const double* x, const double* b, double* y, double omega,
                       double* partial) {
    if (n_blocks <= 0) return;
    CsrArgs a{A.blocks.p, A.rp.p, A.col.p, A.val.p, x, A.halo.p, (int)A.n_cols_local,
              b, A.dinv.p, y, omega, partial, A.tile_ptr.p, A.tile_lines.p, A.lcol.p,
              (int)((A.n_cols_local + 7) / 8), (int)A.n_halo(), A.vt_ptr.p, A.vtab.p, A.vidx.p};
    dim3 g(n_blocks), t(kTPB);
    // variant bits: 2 = XCD-ordered blocks, 4 = gather path (no x tile).  Default: x tile;
    // XCD order for rectangular operators (P, R: +5..17% measured), plain order for square
    // ones (neutral).  (A 16-byte vector-load variant measured 15-20% slower on every level,
    // profiles/r1b_spmv_variants.txt, and was removed.)
    // bit 8 = value-indexed blocks (default on when any block qualifies).  The environment
    // override (experiments, scripts/spmv_variants.py) gives all bits explicitly.
    const char* ev = getenv("AMG_KERNEL_VARIANT");
    int var = ev ? atoi(ev) : (A.default_variant | (A.n_vi_blocks > 0 ? 8 : 0));
    if (A.n_vi_blocks == 0) var &= ~8;
#define AMG_L1(M, N, X, T, V) hipLaunchKernelGGL((csr_stream_kernel<M, N, X, T, V>), g, t, 0, s, a, first_block)
#define AMG_L2(M, N, V)                                               \
    do {                                                              \
        const bool xo = var & 2, tl = !(var & 4);                     \
        if (xo && tl) AMG_L1(M, N, true, true, V);                    \
        else if (xo) AMG_L1(M, N, true, false, V);                    \
        else if (tl) AMG_L1(M, N, false, true, V);                    \
        else AMG_L1(M, N, false, false, V);                           \
    } while (0)
#define AMG_L(M, N)                                                   \
    do {                                                              \
        if (var & 8) AMG_L2(M, N, true);                              \
        else AMG_L2(M, N, false);                                     \
    } while (0)
    switch (mode) {
        case KM_SPMV: AMG_L(KM_SPMV, false); break;
        case KM_SPMV_ADD: AMG_L(KM_SPMV_ADD, false); break;
        case KM_RESID:
            if (norm) AMG_L(KM_RESID, true);
            else AMG_L(KM_RESID, false);
            break;
        case KM_JACOBI:
            if (norm) AMG_L(KM_JACOBI, true);
            else AMG_L(KM_JACOBI, false);
            break;
        default: throw Error(AMG_ERR_INTERNAL, "bad kernel mode");
    }
#undef AMG_L
#undef AMG_L2
#undef AMG_L1
    HIP_CHECK(hipGetLastError());
}

void launch_hybrid_gs(hipStream_t s, const DevMatrix& A, const double* x, const double* b,
                      double* y, bool backward, double* partial) {
    if (A.n_gs_slabs <= 0) return;
    AMG_ASSERT(!(backward && partial));
    GsArgs a{A.gs_slabs.p, A.gs_col.p, A.gs_val.p, x, A.halo.p, (int)A.n_cols_local, b,
             A.gs_dinv.p, y, (long long)A.first_row, (long long)A.gs_block, (int)A.n_rows,
             A.n_gs_slabs, partial};
    static const int forced = [] {
        const char* e = std::getenv("AMG_GS_VARIANT");  // 0 narrow, 1 wide (experiments)
        return e ? std::atoi(e) : -1;
    }();
    const bool wide = forced >= 0 ? forced == 1 : A.gs_wide;
    const dim3 grid(wide ? A.n_gs_slabs : (A.n_gs_slabs + 3) / 4), block(wide ? 64 : 256);
#define AMG_GS(BK, WD, NM) hipLaunchKernelGGL((hybrid_gs_kernel<BK, WD, NM>), grid, block, 0, s, a)
    if (wide) {
        if (backward) AMG_GS(true, true, false);
        else if (partial) AMG_GS(false, true, true);
        else AMG_GS(false, true, false);
    } else {
        if (backward) AMG_GS(true, false, false);
        else if (partial) AMG_GS(false, false, true);
        else AMG_GS(false, false, false);
    }
#undef AMG_GS
    HIP_CHECK(hipGetLastError());
}

void launch_jacobi_zero(hipStream_t s, int64_t n, const double* b, const double* dinv, double* y,
                        double omega) {
    if (n <= 0) return;
    hipLaunchKernelGGL(jacobi_zero_kernel, dim3(grid_for(n)), dim3(kTPB), 0, s, (long long)n, b,
                       dinv, y, omega);
    HIP_CHECK(hipGetLastError());
}

void launch_pack(hipStream_t s, int64_t n, const int* idx, const double* x, double* out) {
    if (n <= 0) return;
    hipLaunchKernelGGL(pack_kernel, dim3((unsigned)((n + kTPB - 1) / kTPB)), dim3(kTPB), 0, s,
                       (long long)n, idx, x, out);
    HIP_CHECK(hipGetLastError());
}

void launch_zero(hipStream_t s, int64_t n, double* y) {
    if (n <= 0) return;
    hipLaunchKernelGGL(zero_kernel, dim3(grid_for(n)), dim3(kTPB), 0, s, (long long)n, y);
    HIP_CHECK(hipGetLastError());
}

void launch_reduce_partials(hipStream_t s, int n, const double* partial, double* tmp, double* out) {
    if (n <= kRedSpan) {
        hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(kTPB), 0, s, n, partial, out);
    } else {
        const int g = (n + kRedSpan - 1) / kRedSpan;
        hipLaunchKernelGGL(sum_partials_kernel, dim3(g), dim3(kTPB), 0, s, n, partial, tmp);
        launch_reduce_partials(s, g, tmp, tmp + g, out);
    }
    HIP_CHECK(hipGetLastError());
}

void launch_finish_norm(hipStream_t s, int n, const double* in, double* hist, int* counter) {
    hipLaunchKernelGGL(finish_norm_kernel, dim3(1), dim3(64), 0, s, n, in, hist, counter);
    HIP_CHECK(hipGetLastError());
}

void launch_dense_gemv(hipStream_t s, int64_t n_local, int64_t n, const double* invT,
                       const double* bfull, double* x) {
    if (n_local <= 0) return;
    hipLaunchKernelGGL(dense_gemv_kernel, dim3((unsigned)((n_local + 63) / 64)), dim3(64), 0, s,
                       (long long)n_local, (long long)n, invT, bfull, x);
    HIP_CHECK(hipGetLastError());
}

void launch_uniform(hipStream_t s, int64_t n, int64_t first_gid, uint64_t seed, double* out) {
    if (n <= 0) return;
    hipLaunchKernelGGL(uniform_kernel, dim3(grid_for(n)), dim3(kTPB), 0, s, (long long)n,
                       (long long)first_gid, (unsigned long long)seed, out);
    HIP_CHECK(hipGetLastError());
}

}  // namespace amg
