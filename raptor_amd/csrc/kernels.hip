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

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "device.hpp"

namespace amg {

// Phase trace of the x-tile block kernel (diagnostic build only: make EXTRA=-DAMG_CSR_PHASES=1;
// scripts/csr_phase_trace.py).  Thread 0 of each block waits for its own outstanding loads at
// fixed points and stamps s_memtime there: [0] entry, [1] batch 1 in (header, line ids, tile /
// VI indices), [2] batch 2 in (x tile, value table, row operands), [3] x tile in LDS (first
// barrier passed), [4] products in LDS (second barrier), [5] row sums stored; [6] / [7]
// s_memrealtime (100 MHz) at entry and exit.  The waits serialise thread 0's loads a little.
#ifndef AMG_CSR_PHASES
#define AMG_CSR_PHASES 0
#endif
#if AMG_CSR_PHASES
__device__ unsigned long long* g_csr_phase;
#define AMG_PHASE(k)                                                   \
    do {                                                               \
        if (threadIdx.x == 0) {                                        \
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); \
            csr_ph[k] = __builtin_amdgcn_s_memtime();                  \
        }                                                              \
    } while (0)
#else
#define AMG_PHASE(k) \
    do {             \
    } while (0)
#endif

namespace {

// Sum over the 64 lanes of a wave, the same value in every lane: DPP row_shr steps 1, 2, 4, 8
// build each 16-lane row's prefix sum (VALU; lanes before the row start read 0), then the four
// row totals are added in order (readlane).  The norm partials used a shuffle tree instead:
// 6 ds_bpermute round trips at the end of every block (27-pt residual + norm 195 vs 168 us).
// Fixed order: deterministic, and the same in every kernel family.
template <int S>
__device__ __forceinline__ double row_shr_f64(double v) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)u, 0x110 + S, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), 0x110 + S, 0xf, 0xf, true);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double lane_f64(double v, int l) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ double wave_sum(double v) {
    v += row_shr_f64<1>(v);
    v += row_shr_f64<2>(v);
    v += row_shr_f64<4>(v);
    v += row_shr_f64<8>(v);
    return (lane_f64(v, 15) + lane_f64(v, 31)) + (lane_f64(v, 47) + lane_f64(v, 63));
}

struct CsrArgs {
    const int4* hdr;         // 2 x int4 per block (par_matrix.hip): {r0, r1, k0, nnz},
                             // {diag slot, tile lines, value-table offset (-1), table size}
    const int* tile_ids;     // kCAP / LW x-tile line ids per block (padded with the last)
    const uint16_t* lcol;    // lane-major 16-bit tile indices (kCAP per block)
    const uint8_t* vidx;     // lane-major 1-byte value indices (kCAP per block)
    const double* vtab;      // value tables
    const uint16_t* rend;    // per row: end of its nonzeros relative to the block's first
    const uint8_t* dvi;      // per row of a VI square operator: table index of a_ii
    const int* rp;
    const int* col;
    const double* val;
    const double* x;   // local part of x
    const double* xh;  // halo part of x
    int ncl;           // number of local columns
    int nhalo;
    int hl0;           // first halo line id = ceil(ncl / LW)
    int wide_x;        // ncl >= 2 and nhalo != 1: 16-byte x-tile loads are in bounds
    int vi_packed;     // rectangular operator: VI indices packed NU per lane at header field 0
    const double* b;
    const double* dinv;
    double* y;
    double omega;
    double* partial;
    int part_off;      // partial slot of block bid's wave w: part_off + bid * kNormParts + w
    double* y2;        // SPMV only, non-null: y2[r] = omega * (dinv[r] * y[r]) as well (the next
                       // level's first Jacobi sweep from x = 0, fused into the restriction)
    const uint16_t* col16;  // gather operators: 16-bit column codes (C16 kernels), with
    const int4* gband;      // the block's 4 band bases: col = base[code >> 14] + (code & 0x3fff)
    int nblk;               // blocks of this launch
};

// the fused second output of a restriction (CsrArgs::y2): jacobi_zero_kernel's expression;
// d = dinv[r], loaded with the row operands (a load after the sum cost a memory round trip
// per block)
template <int MODE>
__device__ __forceinline__ void store_y2(const CsrArgs& a, int r, double out, double d) {
    if (MODE == KM_SPMV && a.y2) a.y2[r] = a.omega * (d * out);
}

__device__ __forceinline__ double xload(const CsrArgs& a, int c) {
    const double* p = c < a.ncl ? a.x + c : a.xh + (c - a.ncl);
    return *p;
}

// fused epilogue; *res receives b - s for the residual and Jacobi modes (for the norm)
template <int MODE>
__device__ __forceinline__ double epilogue(const CsrArgs& a, int r, double s, double* res) {
    if (MODE == KM_SPMV) return s;
    if (MODE == KM_GSACC) return s;  // block_long: s already starts at b (an empty row: b)
    if (MODE == KM_SPMV_ADD) return a.y[r] + s;
    const double t = a.b[r] - s;
    *res = t;
    if (MODE == KM_RESID) return t;
    // Jacobi: x + omega * (dinv * (b - s))
    return a.x[r] + a.omega * (a.dinv[r] * t);
}

// s += stage[k] for k in [lo, hi), in order.  Eight LDS reads are issued before their eight
// dependent adds, so a long row waits on LDS once per eight entries instead of once per
// entry (the adds stay sequential: the oracle's summation order).
#ifndef AMG_ROWSUM_AHEAD  // build-time A/B knob: LDS reads issued ahead of a long row's adds
#define AMG_ROWSUM_AHEAD 16
#endif
__device__ __forceinline__ double lds_row_sum(const double* stage, int lo, int hi, double s) {
    int k = lo;
    if constexpr (AMG_ROWSUM_AHEAD >= 16) {
        // long rows (restrictions of SA hierarchies: 100-700 entries): one LDS round trip per
        // 16 entries
        for (; k + 16 <= hi; k += 16) {
            double v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) v[u] = stage[k + u];
#pragma unroll
            for (int u = 0; u < 16; ++u) s += v[u];
        }
    }
    for (; k + 8 <= hi; k += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = stage[k + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; k < hi; ++k) s += stage[k];
    return s;
}

// XCD-aware bijection: consecutive row blocks land on the same XCD (blocks b and b+8 share
// one under round-robin dispatch), so a row block's x neighbours (+-nx*ny rows) are in the
// same L2.  Placement only changes speed, never results (MI355X_MICROARCH.md).
__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int q = nb >> 3, rem = nb & 7, x = b & 7;
    return x * q + min(x, rem) + (b >> 3);
}

typedef unsigned int v2u_t __attribute__((ext_vector_type(2)));
typedef unsigned int v4u_t __attribute__((ext_vector_type(4)));
typedef double v2d_t __attribute__((ext_vector_type(2)));
typedef int v2i_t __attribute__((ext_vector_type(2)));


// Entries [q, q+1] of a vector of n >= 2 doubles: a 16-byte load at min(q, n - 2); when q is
// the last entry its value is the second half.  Entries past n are garbage (never used).
__device__ __forceinline__ v2d_t load_pair(const double* base, int q, int n) {
    const int st = min(q, n - 2);
    const v2d_t v = *(const v2d_t*)(base + st);
    return v2d_t{q == st ? v.x : v.y, v.y};
}

// One workgroup per row block (<= kCAP nonzeros, <= kTPB rows).  Bit-identical to the oracle:
// products a_ij * x_j are formed in registers, staged in LDS, and lane r sums its row's
// products in CSR order before the fused epilogue.
//
// The kernel is built for memory-level parallelism.  Every load is unconditional and issued
// in dependency batches with no divergent branch between them (out-of-range lanes re-read
// the block's last entry -- the same address, merged by the TA -- and results are masked only
// at the LDS / y stores); an earlier form guarded each load with its own bounds test, the
// compiler wrapped each in a branch and drained vmcnt at every join, and the kernel was
// latency-bound (profiles/r1h_variants.txt: 278 -> 184 us on the 256^3 level-0 SpMV).
//   batch 1 (block id only): header (scalar), one x-tile line id per lane (fixed stride),
//            16-bit tile indices, VI indices
//   batch 2: x tile (16-byte loads, 4 per lane; line ids via ds_bpermute), values or VI
//            table, row bounds and epilogue operands  [gather: columns, then x]
// PMC (SQ_WAIT_INST_ANY ~42% of wave cycles) showed the VMEM issue queue, not HBM, as the
// limit, so the per-wave vector-memory instruction count is kept low (10 for SpMV).
//
// TILE: the block's distinct 64-byte lines of x go to LDS; products read x from LDS through a
// 16-bit index per nonzero.  Jacobi reads x[r] from the tile too when the block's own lines
// are consecutive in it (header diag slot).  VIB: the block's nonzeros take <= 256 distinct
// values; a 1-byte index per nonzero selects from the table staged in LDS.  NU: lane slots
// in use (8 = full; the gather path of sparse rectangular blocks uses fewer).
// Batch 1 of an x-tile block (depends on the block id only): issued with the header, before
// the loads that depend on it.
// the x-tile line ids lane `lane` of wave `wv` loads (tile_line_ids) and where lane `lane`
// finds the line of its 16-byte slot pair j (tile_line_src): 64-byte lines, 4 lanes per line,
// line 16 wv + (lane >> 2) + 64 j; 32-byte lines, 2 lanes per line, line 32 wv + (lane >> 1) +
// 128 j (each lane holds two ids: j = 0, 1 and j = 2, 3).  Either way slot pair j of lane t is
// stage[2 t + 512 j].
template <int LW>
__device__ __forceinline__ int tile_id_index(int wv, int lane, int k) {
    return LW == 8 ? 16 * wv + (lane & 15) + 64 * (lane >> 4) : 32 * wv + (lane & 31) + 128 * (lane >> 5) + 256 * k;
}

struct CsrPre {
    int4 h0, h1;
    int tid_line, tid_line2;
    v4u_t lq;
    v2u_t vq;
};

template <bool VI, int LW = 8>
__device__ __forceinline__ void csr_pre_tile(const CsrArgs& a, int bid, CsrPre& p) {
    constexpr int TL = kCAP / LW;  // line ids per block
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    p.h0 = a.hdr[2 * bid];
    p.h1 = a.hdr[2 * bid + 1];
    p.tid_line = a.tile_ids[(size_t)bid * TL + tile_id_index<LW>(wv, lane, 0)];
    p.tid_line2 = LW == 4 ? a.tile_ids[(size_t)bid * TL + tile_id_index<LW>(wv, lane, 1)] : 0;
    p.lq = __builtin_nontemporal_load((const v4u_t*)(a.lcol + (size_t)bid * kCAP + (size_t)tid * (kCAP / kTPB)));
    p.vq = v2u_t{0u, 0u};
    // square operators with value-indexed blocks hold kCAP index bytes for every block
    if (VI) p.vq = __builtin_nontemporal_load((const v2u_t*)(a.vidx + (size_t)bid * kCAP + (size_t)tid * (kCAP / kTPB)));
}

// PRE: 0 = load batch 1 here; 1 / 2 = batch 1 was issued with the header into *pre (2: with
// VI indices)
// RPB: rows per lane (gather blocks of rectangular operators hold up to kTPB * kGatherRPB
// rows; a short-row P block of 256 rows filled a quarter of its 2048-entry stage)
template <int MODE, bool NORM, bool TILE, bool VIB, int NU, int PRE = 0, int RPB = 1, bool C16 = false,
          int LW = 8>
__device__ __forceinline__ double block_main(const CsrArgs& a, int bid, double* stage, double* tabl,
                                             int* rends, CsrPre* pre = nullptr,
                                             unsigned long long* csr_ph = nullptr) {
    constexpr int U = kCAP / kTPB;  // 8 lane slots
    static_assert(NU >= 2 && NU % 2 == 0 && NU <= U && (TILE ? NU == U : true), "slot pairs");
    static_assert(RPB == 1 || (!NORM && (MODE == KM_SPMV || MODE == KM_SPMV_ADD)),
                  "several rows per lane: SpMV / y += Ax only");
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    static_assert(!PRE || TILE, "prefetched batch 1: x-tile path only");
    static_assert(!C16 || !TILE, "column codes: gather path only");
    int tid_line = 0, tid_line2 = 0;
    v4u_t lq = {0u, 0u, 0u, 0u};
    v2u_t vq = {0u, 0u};
    int4 h0, h1, gb = {0, 0, 0, 0};
    if constexpr (PRE > 0) {
        tid_line = pre->tid_line;
        tid_line2 = pre->tid_line2;
        lq = pre->lq;
        vq = pre->vq;
        h0 = pre->h0;
        h1 = pre->h1;
    } else {
    if (TILE) {
        // the lines wave w's 16-byte tile slots need (tile_id_index)
        tid_line = a.tile_ids[(size_t)bid * (kCAP / LW) + tile_id_index<LW>(wv, lane, 0)];
        if (LW == 4) tid_line2 = a.tile_ids[(size_t)bid * (kCAP / LW) + tile_id_index<LW>(wv, lane, 1)];
    }
    if (TILE) lq = __builtin_nontemporal_load((const v4u_t*)(a.lcol + (size_t)bid * kCAP + (size_t)tid * U));
    h0 = a.hdr[2 * bid];
    h1 = a.hdr[2 * bid + 1];
    if (C16) gb = a.gband[bid];  // with the header: no extra round
    if (VIB) {
        if (!a.vi_packed) {
            vq = __builtin_nontemporal_load((const v2u_t*)(a.vidx + (size_t)bid * kCAP + (size_t)tid * U));
        } else {  // gather blocks: NU bytes per lane at the block's offset
            const uint8_t* p = a.vidx + (size_t)(unsigned)h1.x + (size_t)tid * NU;
            if (NU == 8) vq = __builtin_nontemporal_load((const v2u_t*)p);
            else if (NU == 4) vq.x = __builtin_nontemporal_load((const unsigned*)p);
            else vq.x = __builtin_nontemporal_load((const unsigned short*)p);
        }
    }
    }
    const int r0 = h0.x, r1 = h0.y, k0 = h0.z, nnz = h0.w;
    const int r = r0 + tid;
    const bool own = r < r1;
    // rows r0 + tid + kTPB j, j >= 1 (RPB > 1): ends and y operands, loaded with batch 2
    int e1m[RPB > 1 ? RPB : 1];
    double pxm[RPB > 1 ? RPB : 1];
    if constexpr (RPB > 1) {
#pragma unroll
        for (int j = 1; j < RPB; ++j) {
            const int rj = r0 + tid + kTPB * j, rjj = rj < r1 ? rj : r0;
            e1m[j] = a.rend[rjj];
            rends[tid + kTPB * j] = e1m[j];
            pxm[j] = MODE == KM_SPMV_ADD ? a.y[rjj] : MODE == KM_SPMV && a.y2 ? a.dinv[rjj] : 0.0;
        }
    }
    // Entry-to-lane map.  TILE: lane t holds entries 512 p + 2 t + {0, 1} (p < 4) of the
    // block-aligned val stream (k0 even): 16-byte value loads (profiles/r1o_libab.txt: A2
    // SpMV / Jacobi -8% / -9%).  Gather: lane t holds entries t + 256 u, so one wave-
    // instruction's x gathers cover consecutive nonzeros (pairs measured 5-7% slower on P/R).
    // Lanes past the block re-read its last entry / pair.
    int c[U];
    if (!TILE && !C16) {
#pragma unroll
        for (int u = 0; u < NU; ++u)
            c[u] = __builtin_nontemporal_load(a.col + k0 + min(tid + u * kTPB, nnz - 1));
    } else if (C16) {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const unsigned code = __builtin_nontemporal_load(a.col16 + k0 + min(tid + u * kTPB, nnz - 1));
            const unsigned t = code >> 14;
            const int base = t == 0 ? gb.x : t == 1 ? gb.y : t == 2 ? gb.z : gb.w;
            c[u] = base + (int)(code & 0x3fffu);
        }
    }
    double v[U], tv = 0.0;
    if (VIB) {
        tv = a.vtab[h1.z + min(tid, h1.w - 1)];
    } else if (TILE) {
        const int plast = (nnz - 1) & ~1;
#pragma unroll
        for (int p = 0; p < U / 2; ++p) {
            const v2d_t vv = __builtin_nontemporal_load((const v2d_t*)(a.val + k0 + min(2 * tid + 2 * kTPB * p, plast)));
            v[2 * p] = vv.x;
            v[2 * p + 1] = vv.y;
        }
    } else {
#pragma unroll
        for (int u = 0; u < NU; ++u)
            v[u] = __builtin_nontemporal_load(a.val + k0 + min(tid + u * kTPB, nnz - 1));
    }
    // row operands (lanes past the block re-read row r0); row start = previous lane's end,
    // exchanged through LDS behind the first barrier
    const int rr = own ? r : r0;
    const int e1 = a.rend[rr];
    rends[tid] = e1;
    const bool px_tile = TILE && MODE == KM_JACOBI && h1.x >= 0;       // block-uniform
    const bool pd_tab = VIB && MODE == KM_JACOBI && (h1.y & kHdrDvi) != 0;  // block-uniform
    double pb = 0.0, pd = 0.0, px = 0.0;
    int dv = 0;
    if (MODE == KM_SPMV_ADD) px = a.y[rr];
    if (MODE == KM_SPMV && a.y2) pd = a.dinv[rr];  // store_y2
    if (MODE == KM_RESID || MODE == KM_JACOBI || MODE == KM_GSACC) pb = a.b[rr];
    if (MODE == KM_JACOBI) {
        if (pd_tab) dv = a.dvi[rr];
        else pd = a.dinv[rr];
        if (!px_tile) px = a.x[rr];
    }
    // the scheduling barrier keeps every earlier load issued before the first x load waits
    // for its line / column id
    __builtin_amdgcn_sched_barrier(0);
    double xs[U];
    if (TILE) {
        // slot pair j of lane l: elements e, e + 1 of its line (tile_id_index), e = 2 (l & 3)
        // (64-byte lines) or 2 (l & 1) (32-byte lines); element e of line L is column
        // LW L + e (local) or halo entry LW (L - hl0) + e
        const int e = LW == 8 ? 2 * (lane & 3) : 2 * (lane & 1);
        auto line_of_pair = [&](int j) {
            return LW == 8 ? __shfl(tid_line, (lane >> 2) + 16 * j, 64)
                           : __shfl(j < 2 ? tid_line : tid_line2, (lane >> 1) + 32 * (j & 1), 64);
        };
        if (a.wide_x) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int L = line_of_pair(j);
                const v2d_t p2 = L < a.hl0 ? load_pair(a.x, L * LW + e, a.ncl)
                                           : load_pair(a.xh, (L - a.hl0) * LW + e, a.nhalo);
                xs[2 * j] = p2.x;
                xs[2 * j + 1] = p2.y;
            }
        } else {  // a vector of one entry: 8-byte loads (degenerate coarse partitions)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int L = line_of_pair(j);
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const double* p = L < a.hl0 ? a.x + min(L * LW + e + h, a.ncl - 1)
                                                : a.xh + min((L - a.hl0) * LW + e + h, a.nhalo - 1);
                    xs[2 * j + h] = *p;
                }
            }
        }
        if constexpr (PRE > 0) AMG_PHASE(2);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            *(v2d_t*)(stage + 2 * tid + 512 * j) = v2d_t{xs[2 * j], xs[2 * j + 1]};
    } else {
#pragma unroll
        for (int u = 0; u < NU; ++u) xs[u] = xload(a, c[u]);
    }
    if (VIB) tabl[tid] = tv;
    if (TILE || VIB) __syncthreads();
    if constexpr (PRE > 0) AMG_PHASE(3);
    constexpr int LS = LW == 8 ? 3 : 2;
    if (px_tile) px = stage[(h1.x + (rr >> LS) - (r0 >> LS)) * LW + (rr & (LW - 1))];
    // 1 / a_ii from the table: the same correctly rounded division the host does for dinv
    if (pd_tab) pd = 1.0 / tabl[dv];
    if (VIB) {
        const unsigned w[2] = {vq.x, vq.y};
#pragma unroll
        for (int u = 0; u < NU; ++u) v[u] = tabl[(w[u >> 2] >> (8 * (u & 3))) & 0xffu];
    }
    double pr[U];
    if (TILE) {
        const unsigned li[U] = {lq.x & 0xffffu, lq.x >> 16, lq.y & 0xffffu, lq.y >> 16,
                                lq.z & 0xffffu, lq.z >> 16, lq.w & 0xffffu, lq.w >> 16};
#pragma unroll
        for (int u = 0; u < U; ++u) pr[u] = v[u] * stage[li[u]];
        __syncthreads();  // every lane has read the tile; reuse it for the products
    } else {
#pragma unroll
        for (int u = 0; u < NU; ++u) pr[u] = v[u] * xs[u];
    }
    if (MODE == KM_GSACC) {  // acc -= p is acc + (-p) bit for bit (negation is exact)
#pragma unroll
        for (int u = 0; u < U; ++u) pr[u] = -pr[u];
    }
    if (TILE) {
#pragma unroll
        for (int p = 0; p < U / 2; ++p) *(v2d_t*)(stage + 2 * tid + 2 * kTPB * p) = v2d_t{pr[2 * p], pr[2 * p + 1]};
    } else {
#pragma unroll
        for (int u = 0; u < NU; ++u) stage[tid + u * kTPB] = pr[u];
    }
    __syncthreads();
    if constexpr (PRE > 0) AMG_PHASE(4);
    if constexpr (RPB > 1) {
#pragma unroll
        for (int j = 1; j < RPB; ++j) {
            const int k = tid + kTPB * j, rj = r0 + k;
            if (rj < r1) {
                const double sj = lds_row_sum(stage, rends[k - 1], e1m[j], 0.0);
                a.y[rj] = MODE == KM_SPMV ? sj : pxm[j] + sj;
                store_y2<MODE>(a, rj, sj, pxm[j]);
            }
        }
    }
    const int e0 = tid ? rends[tid - 1] : 0;
    double s = MODE == KM_GSACC ? pb : 0.0;  // GSACC: acc = b, then acc -= a_ij x_j in order
    s = lds_row_sum(stage, e0, e1, s);
    double out, sq = 0.0;
    if (MODE == KM_SPMV || MODE == KM_GSACC) {
        out = s;
    } else if (MODE == KM_SPMV_ADD) {
        out = px + s;
    } else {
        const double t = pb - s;
        if (NORM) sq = own ? t * t : 0.0;
        out = MODE == KM_RESID ? t : px + a.omega * (pd * t);
    }
    if (own) {
        a.y[r] = out;
        store_y2<MODE>(a, r, out, pd);
    }
    if constexpr (PRE > 0) AMG_PHASE(5);
    return sq;
}

template <int MODE, bool NORM, bool TILE, bool VIB, int GRPB = 1, bool C16 = false, int LW = 8>
__device__ __forceinline__ double block_dispatch(const CsrArgs& a, int bid, int nnz, double* stage,
                                                 double* tabl, int* rends) {
    constexpr int RP = (MODE == KM_SPMV || MODE == KM_SPMV_ADD) && !NORM ? GRPB : 1;
    if constexpr (TILE) {
        // a tiled short-row P holds up to kTPB * GRPB rows per block: every row is summed
        // (AMG_CSR_PRE_TILE=0 builds reach this branch)
        return block_main<MODE, NORM, TILE, VIB, 8, 0, RP, false, LW>(a, bid, stage, tabl, rends);
    } else {
        if (nnz > 4 * kTPB) return block_main<MODE, NORM, TILE, VIB, 8, 0, RP, C16>(a, bid, stage, tabl, rends);
        if (nnz > 2 * kTPB) return block_main<MODE, NORM, TILE, VIB, 4, 0, RP, C16>(a, bid, stage, tabl, rends);
        return block_main<MODE, NORM, TILE, VIB, 2, 0, RP, C16>(a, bid, stage, tabl, rends);
    }
}

// empty block, or one row longer than the LDS stage / a tile: chunked, lane 0 sums
template <int MODE, bool NORM>
__device__ __forceinline__ double block_long(const CsrArgs& a, int4 h0, double* stage) {
    const int tid = threadIdx.x;
    const int r0 = h0.x, r1 = h0.y, k0 = h0.z, nnz = h0.w;
    double s = MODE == KM_GSACC && nnz > 0 ? a.b[r0] : 0.0, sq = 0.0;
    for (int base = 0; base < nnz; base += kCAP) {
        const int cnt = min(kCAP, nnz - base);
        for (int k = tid; k < cnt; k += kTPB) {
            const double p = a.val[k0 + base + k] * xload(a, a.col[k0 + base + k]);
            stage[k] = MODE == KM_GSACC ? -p : p;
        }
        __syncthreads();
        if (tid == 0)
            s = lds_row_sum(stage, 0, cnt, s);
        __syncthreads();
    }
    for (int r = r0 + tid; r < r1; r += kTPB) {
        if (r == r0 || nnz == 0) {  // nnz == 0: every row of the block is empty
            double res = 0.0;
            const double o = MODE == KM_GSACC && nnz == 0 ? a.b[r] : epilogue<MODE>(a, r, s, &res);
            a.y[r] = o;
            if (MODE == KM_SPMV && a.y2) store_y2<MODE>(a, r, o, a.dinv[r]);
            if (NORM) sq += res * res;
        }
    }
    return sq;
}

// fixed-shape wave reduction, one partial per wave (kNormParts per block): no block barrier
// at the end of the kernel; the partials are summed in fixed order
template <bool NORM>
__device__ __forceinline__ void block_partial(const CsrArgs& a, int bid, double sq) {
    if (NORM) {
        sq = wave_sum(sq);
        if ((threadIdx.x & 63) == 0) a.partial[a.part_off + bid * kNormParts + (threadIdx.x >> 6)] = sq;
    }
}

// GRPB: rows per lane of gather blocks (1, or kGatherRPB for short-row rectangular operators
// whose blocks hold up to kTPB * kGatherRPB rows; DevMatrix::gather_rpb)
// C16: gather path with 16-bit column codes (DevMatrix::col16)
// LW: doubles per x-tile line (8: 256 lines of 64 B, 4: 512 lines of 32 B; DevMatrix::line_w)
template <int MODE, bool NORM, bool XCD, bool TILE, bool VI, int GRPB = 1, bool C16 = false, int LW = 8>
__global__ __launch_bounds__(kTPB, GRPB > 1 ? 7 : 8) void csr_block_kernel(CsrArgs a, int first_block) {
    static_assert(kCAP / kTPB == 8 && (LW == 8 || LW == 4) && kTPB == 256,
                  "lane-major layouts assume 8 entries per lane, 4 waves");
    __shared__ __attribute__((aligned(16))) double stage[kCAP];  // x tile, then products
    __shared__ double tabl[VI ? 256 : 1];
    __shared__ int rends[kTPB * GRPB];
    const int bid = first_block + (XCD ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x);
    if constexpr (TILE && AMG_CSR_PRE_TILE) {
        // square operators: batch 1 (tile line ids, tile / VI indices: fixed offsets from the
        // block id) issued together with the header instead of after it -- one dependent
        // round of loads less per block
        constexpr int PV = VI ? 2 : 1;
        unsigned long long* csr_ph = nullptr;
#if AMG_CSR_PHASES
        __shared__ unsigned long long ph_lds[8];
        csr_ph = ph_lds;
        if (threadIdx.x == 0) csr_ph[6] = __builtin_amdgcn_s_memrealtime();
        AMG_PHASE(0);
#endif
        CsrPre f;
        csr_pre_tile<VI, LW>(a, bid, f);
#if AMG_CSR_PHASES
        if (threadIdx.x == 0) asm volatile("" ::"v"(f.tid_line), "v"(f.lq.x), "v"(f.vq.x), "s"(f.h0.x), "s"(f.h1.x));
        AMG_PHASE(1);
#endif
        const int4 h0 = f.h0, h1 = f.h1;
        double sq;
        if (h0.w <= kCAP && (h1.y & 0xffff) <= kCAP / LW && h0.w > 0) {
            if (VI && h1.z >= 0) sq = block_main<MODE, NORM, true, true, 8, PV, GRPB, false, LW>(a, bid, stage, tabl, rends, &f, csr_ph);
            else sq = block_main<MODE, NORM, true, false, 8, PV, GRPB, false, LW>(a, bid, stage, tabl, rends, &f, csr_ph);
        } else {
            sq = block_long<MODE, NORM>(a, h0, stage);
        }
        block_partial<NORM>(a, bid, sq);
#if AMG_CSR_PHASES
        if (threadIdx.x == 0 && g_csr_phase) {
            csr_ph[7] = __builtin_amdgcn_s_memrealtime();
            for (int k = 0; k < 8; ++k) g_csr_phase[(size_t)(bid - first_block) * 8 + k] = csr_ph[k];
        }
#endif
        return;
    }
    const int4 h0 = a.hdr[2 * bid], h1 = a.hdr[2 * bid + 1];
    const int nnz = h0.w;
    double sq;
    if (nnz <= kCAP && (!TILE || (h1.y & 0xffff) <= kCAP / LW) && nnz > 0) {
        if (VI && h1.z >= 0) sq = block_dispatch<MODE, NORM, TILE, true, GRPB, C16, LW>(a, bid, nnz, stage, tabl, rends);
        else sq = block_dispatch<MODE, NORM, TILE, false, GRPB, C16, LW>(a, bid, nnz, stage, tabl, rends);
    } else {
        sq = block_long<MODE, NORM>(a, h0, stage);
    }
    block_partial<NORM>(a, bid, sq);
}

// Plain CSR (AMG_FORMAT_CSR): exactly the arrays SURVEY.md 8(d) prices --
// int32 row_ptr, int32 col, fp64 val -- and nothing else (no headers, tiles, value indexing
// or templates).  It is the roofline leg scored on 8(d)'s algorithmic bytes, and the path for
// callers that hand over a matrix to be used as stored.  One 256-lane workgroup per 256
// consecutive rows (XCD-remapped, so neighbouring row blocks share an L2).  The workgroup
// streams its nonzero range [rp[r0], rp[r1]) in chunks of kCAP entries: lane t takes entries
// base + 2t + 512p (p < 4) as a 16-byte value pair and an 8-byte column pair, both
// nontemporal (each byte is read once), gathers x (L2-resident), and stages the products in
// LDS; lane r then sums its row's products over the chunk in CSR order.  Rows never straddle
// a workgroup, so every row sum runs from 0.0 in the oracle's order: bit-identical.
struct PlainArgs {
    const int* rp;
    const int* col;     // local | halo numbering, 2 padding entries
    const double* val;  // 2 padding entries
    const double* x;
    const double* xh;
    int ncl, n;
    const double* b;
    const double* dinv;
    double* y;
    double omega;
    double* partial;
};

__device__ __forceinline__ double plain_x(const PlainArgs& a, int c) {
    return c < a.ncl ? a.x[c] : a.xh[c - a.ncl];
}

template <int MODE, bool NORM>
__global__ __launch_bounds__(kTPB, 8) void csr_plain_kernel(PlainArgs a) {
    __shared__ __attribute__((aligned(16))) double stage[kCAP];
    const int tid = threadIdx.x;
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int r0 = bid * kTPB, r1 = min(a.n, r0 + kTPB), r = r0 + tid;
    const bool own = r < r1;
    const int rr = own ? r : r1 - 1;
    const int k0 = a.rp[r0], k1 = a.rp[r1];  // workgroup-uniform (scalar loads)
    const int rs = a.rp[rr], re = a.rp[rr + 1];
    double pb = 0.0, pd = 0.0, px = 0.0;
    if (MODE == KM_SPMV_ADD) px = a.y[rr];
    if (MODE == KM_RESID || MODE == KM_JACOBI) pb = a.b[rr];
    if (MODE == KM_JACOBI) {
        pd = a.dinv[rr];
        px = a.x[rr];
    }
    const int plast = max(k1 - 1, 0) & ~1;  // last pair holding a real entry (padding after)
    double s = 0.0;
    for (int base = k0 & ~1; base < k1; base += kCAP) {
        v2d_t vv[4];
        v2i_t cc[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int q = min(base + 2 * tid + 2 * kTPB * p, plast);
            vv[p] = __builtin_nontemporal_load((const v2d_t*)(a.val + q));
            cc[p] = __builtin_nontemporal_load((const v2i_t*)(a.col + q));
        }
#pragma unroll
        for (int p = 0; p < 4; ++p)
            *(v2d_t*)(stage + 2 * tid + 2 * kTPB * p) =
                v2d_t{vv[p].x * plain_x(a, cc[p].x), vv[p].y * plain_x(a, cc[p].y)};
        __syncthreads();
        const int lo = max(rs, base) - base, hi = min(re, base + kCAP) - base;
        s = lds_row_sum(stage, lo, hi, s);
        __syncthreads();  // the next chunk overwrites the stage
    }
    double out, sq = 0.0;
    if (MODE == KM_SPMV) {
        out = s;
    } else if (MODE == KM_SPMV_ADD) {
        out = px + s;
    } else {
        const double t = pb - s;
        if (NORM) sq = own ? t * t : 0.0;
        out = MODE == KM_RESID ? t : px + a.omega * (pd * t);
    }
    if (own) a.y[r] = out;
    if (NORM) {
        sq = wave_sum(sq);
        if ((tid & 63) == 0) a.partial[bid * kNormParts + (tid >> 6)] = sq;
    }
}


// STREAM-copy ceiling (bench.py): one pass, 4 x 16-byte pairs per lane (1 KiB-strided, so a
// wave instruction moves 1 KiB), plain loads and stores.  Same-box probe (profiles/
// r2c_copy_probe.txt): 5.6 TB/s, against 4.1-5.3 TB/s for grid-stride forms and 5.2 TB/s for
// hipMemcpyAsync.
__global__ __launch_bounds__(kTPB) void copy_kernel(long long npair, const v2d_t* __restrict__ src,
                                                     v2d_t* __restrict__ dst) {
    const long long i = (long long)blockIdx.x * 4 * kTPB + threadIdx.x;
    if (i + 3 * kTPB < npair) {
        v2d_t v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = src[i + u * kTPB];
#pragma unroll
        for (int u = 0; u < 4; ++u) dst[i + u * kTPB] = v[u];
    } else {
        for (long long k = i; k < npair; k += kTPB) dst[k] = src[k];
    }
}

// READ ceiling (bench.py): the copy kernel's access pattern with the stores dropped -- one pass
// of 16-byte loads, 4 pairs per lane, one partial sum per workgroup (so the loads are live).
// Most level kernels read 5-20x what they write, so the read rate, not the copy rate, is the
// ceiling they approach.
__global__ __launch_bounds__(kTPB) void read_kernel(long long npair, const v2d_t* __restrict__ src,
                                                     double* __restrict__ part) {
    const long long i = (long long)blockIdx.x * 4 * kTPB + threadIdx.x;
    double s = 0.0;
    if (i + 3 * kTPB < npair) {
        v2d_t v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(src + i + u * kTPB);
#pragma unroll
        for (int u = 0; u < 4; ++u) s += v[u].x + v[u].y;
    } else {
        for (long long k = i; k < npair; k += kTPB) s += src[k].x + src[k].y;
    }
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) part[(long long)blockIdx.x * 4 + (threadIdx.x >> 6)] = s;
}

// Row-template kernel.  A templated row is (column - row) offsets, values and
// 1/a_ii shared with every row of the same shape -- for a constant-coefficient stencil a few
// dozen templates cover the operator -- so the kernel streams 1 byte per row (its template
// id) plus the vectors, instead of per-nonzero indices and values.  Lane = row, kTplRPL rows
// per lane (rows r0 + lane + kTPB j of the workgroup's kTplRows).  Each row's sum runs in CSR
// order from 0.0 -- the oracle's order, so the results are bit-identical.
//
// x window (NPL > 0): the template offsets, merged into a few bands [lo, hi], tell which x
// every workgroup reads: x[r0 + lo, r0 + kTplRows + hi] per band.  The workgroup loads the
// bands into LDS once (NPL 8-byte loads per lane, all issued before the first is used; 512
// contiguous bytes per wave-instruction) and every product reads x from LDS through the
// entry's window slot (tpl_ldo).  Without the window (operators whose bands do not fit) each
// product loads x from global memory, 8 entries per batch.  Measured on the 7-pt 256^3
// operator: window 5x fewer vector-memory instructions than the global loads, which were
// latency-bound at ~1/4 of the HBM rate (profiles/r1t_*).
struct TplArgs {
    const uint8_t* id;   // per row (kTplNone: not templated here)
    const int* hdr;      // per template: start | len << 16 | diag entry << 24
    const int* off;      // per entry: window slot (NPL > 0) or column - row
    const double* val;   // per entry
    const double* pd;    // per template: 1/a_ii (Jacobi)
    int ntpl, nent, n;
    int nband, win;            // x-window bands, window size (doubles, even)
    int wend;                  // window end relative to r0 (last band's end)
    int blo[kTplBands];        // band b covers x[r0 + blo[b] + i], i < bbase[b+1] - bbase[b]
    int bbase[kTplBands + 1];  // first window slot of band b
    // per chunk u of kTPB * S window slots (S = 2: slot pairs, S = 1: single slots): slot
    // i = S tid + kTPB S u holds x[r0 + i + (S tid >= thr ? dhi : dlo)] -- bands are at least
    // kTplRows slots long, so at most one band starts inside a chunk (tpl_chunk_tables)
    int wdlo[2][kTplChunks], wdhi[2][kTplChunks], wthr[2][kTplChunks];
    const double* x;
    const double* b;
    double* y;
    double omega;
    double* partial;
    const int* wsrc;  // march (variant bit 128): per window slot, the slot of the block one
                      // stride back that holds the same x (-1: load it)
    // uniform stencil (MNE > 0 kernels, variant bit 512): hdr = per-template entry masks, nent
    // = 0; the master's window slots and values (read from kernel arguments: scalar loads),
    // its diagonal entry and 1/a_ii
    int mdiag;
    double mpd;
    int mslot[kTplMasterMax];
    double mval[kTplMasterMax];
};

// dynamic LDS: window | values | 1/a_ii (Jacobi only) | entry slots or offsets | headers.
// (Leaving out the 2 KiB of 1/a_ii outside Jacobi measured neutral on the 7-pt SpMV,
// profiles/r1t_lds_ab.txt; kept because it costs nothing.)
// (A 1/a_ii table of ntpl instead of 256 entries -- 8 instead of 7 Jacobi workgroups per CU
// -- made the 7-pt Jacobi slower, 102 -> 120 us, profiles/r1u_pdtrim_ab.txt.)
// host: the per-chunk band tables of TplArgs (wdlo / wdhi / wthr) from blo / bbase / nband
inline void tpl_chunk_tables(TplArgs& a) {
    for (int S = 1; S <= 2; ++S)
        for (int u = 0; u < kTplChunks; ++u) {
            const int c0 = kTPB * S * u, c1 = c0 + kTPB * S;
            int q = 0;
            while (q + 1 < a.nband && a.bbase[q + 1] <= c0) ++q;
            const int dlo = a.nband ? a.blo[q] - a.bbase[q] : 0;
            int thr = 1 << 30, dhi = dlo;
            if (q + 1 < a.nband && a.bbase[q + 1] < c1) {
                thr = a.bbase[q + 1] - c0;
                dhi = a.blo[q + 1] - a.bbase[q + 1];
                AMG_ASSERT(q + 2 >= a.nband || a.bbase[q + 2] >= c1);  // one band start per chunk
            }
            a.wdlo[S - 1][u] = dlo;
            a.wdhi[S - 1][u] = dhi;
            a.wthr[S - 1][u] = thr;
        }
}

inline size_t tpl_lds_bytes(int win, int nent, bool jacobi) {
    return 8 * ((size_t)win + (size_t)nent + (jacobi ? kTplMax + 1 : 0)) + 4 * ((size_t)nent + kTplMax + 1);
}

struct TplLds {
    double* win;
    double* val;
    double* pd;
    int* off;
    int* hdr;
};

template <int MODE>
__device__ __forceinline__ TplLds tpl_lds_layout(const TplArgs& a) {
    extern __shared__ __attribute__((aligned(16))) double tpl_lds[];
    TplLds L;
    L.win = tpl_lds;
    L.val = L.win + a.win;
    L.pd = L.val + a.nent;
    L.off = (int*)(L.pd + (MODE == KM_JACOBI ? kTplMax + 1 : 0));
    L.hdr = L.off + a.nent;
    return L;
}

// x through a buffer descriptor: 32-bit offsets, out-of-range loads return 0 (window slots
// before row 0 / past row n - 1 are never read)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tpl_xrs(const TplArgs& a) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, (int)((unsigned)a.n * 8u), 0x00020000);
}

// template table into LDS (L2-resident; the caller's barrier publishes it)
template <int MODE, int MNE = 0>
__device__ __forceinline__ void tpl_stage_table(const TplArgs& a, const TplLds& L) {
    const int tid = threadIdx.x;
    for (int k = tid; k < a.nent; k += kTPB) {
        L.off[k] = a.off[k];
        L.val[k] = a.val[k];
    }
    if (tid < a.ntpl) {
        L.hdr[tid] = a.hdr[tid];  // MNE > 0: the template's entry mask
        if (MODE == KM_JACOBI && MNE == 0) L.pd[tid] = a.pd[tid];
    }
    // length 0, no diagonal / no master entry
    if (tid == kTplNone) L.hdr[kTplNone] = MNE > 0 ? 0 : (int)(255u << 24);
}

// x offsets (relative to the block's first row) of the lane's window slots i_u = S (tid +
// kTPB u), S = 2 for slot pairs: one compare and select per slot against the chunk's
// workgroup-uniform band start (an unrolled select over all kTplBands bands cost more VALU
// than the 27-pt rows themselves, profiles/r2w_tpl_sq_instr.txt)
template <int S, int NS>
__device__ __forceinline__ void tpl_slot_offsets(const TplArgs& a, int (&go)[NS]) {
    static_assert(NS <= kTplChunks, "window chunks");
    const int t = S * (int)threadIdx.x;
#pragma unroll
    for (int u = 0; u < NS; ++u)
        go[u] = t + kTPB * S * u + (t >= a.wthr[S - 1][u] ? a.wdhi[S - 1][u] : a.wdlo[S - 1][u]);
}

// the row operands and x window of the rows block starting at r0, into registers
// lane tid's row j of a block: local index tpl_lrow<ROT>(tid, j).  ROT (uniform-stencil kernels)
// rotates the lanes by one row, so on a 256-wide grid the two x-boundary rows of a y line (local
// 0 and 255) land in the same wave (lanes 255 and 254) and the other three waves hold interior
// rows only -- waves with a boundary row take the masked path (tpl_rows_master)
template <bool ROT>
__device__ __forceinline__ int tpl_lrow(int tid, int j) {
    return kTPB * j + (ROT ? ((tid + 1) & (kTPB - 1)) : tid);
}

template <int MODE, int NPL, bool ROT = false>
struct TplFetch {
    static constexpr int R = kTplRPL, NP = NPL > 0 ? NPL : 1;
    int id[R], rr[R];
    double pb[R], py[R], wv[NP];
    bool pairs;

    __device__ __forceinline__ void issue(const TplArgs& a, __amdgpu_buffer_rsrc_t xrs, int r0) {
        issue_ids(a, r0);
        issue_operands(a);
        issue_window(a, xrs, r0);
    }

    __device__ __forceinline__ void issue_ids(const TplArgs& a, int r0) {
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const int r = r0 + tpl_lrow<ROT>((int)threadIdx.x, j);
            rr[j] = min(r, a.n - 1);
            const int t = a.id[rr[j]];
            id[j] = r < a.n ? t : kTplNone;
        }
    }

    // b / y: needed only by the epilogue
    __device__ __forceinline__ void issue_operands(const TplArgs& a) {
#pragma unroll
        for (int j = 0; j < R; ++j) {
            pb[j] = 0.0;
            py[j] = 0.0;
            if (MODE == KM_RESID || MODE == KM_JACOBI) pb[j] = a.b[rr[j]];
            if (MODE == KM_SPMV_ADD) py[j] = a.y[rr[j]];
        }
    }

    __device__ __forceinline__ void issue_window(const TplArgs& a, __amdgpu_buffer_rsrc_t xrs, int r0) {
        const int tid = threadIdx.x;
        // Blocks whose window lies inside x (all but the first and last few) load slot pairs
        // with 16-byte loads (bands start at even offsets and hold an even number of slots);
        // the others load single slots, out-of-range ones returning 0.
        pairs = r0 + a.blo[0] >= 0 && r0 + a.wend <= a.n;  // workgroup-uniform
        if (NPL > 0 && pairs) {
            int go[NP / 2 > 0 ? NP / 2 : 1];
            tpl_slot_offsets<2>(a, go);
#pragma unroll
            for (int u = 0; u < NP / 2; ++u) {
                const int vo = 2 * (tid + kTPB * u) < a.win ? (r0 + go[u]) * 8 : -16;
                const v2d_t p2 = __builtin_bit_cast(v2d_t, __builtin_amdgcn_raw_buffer_load_b128(xrs, vo, 0, 0));
                wv[2 * u] = p2.x;
                wv[2 * u + 1] = p2.y;
            }
        } else if (NPL > 0) {
            int go[NP];
            tpl_slot_offsets<1>(a, go);
#pragma unroll
            for (int u = 0; u < NP; ++u) {
                const int vo = tid + kTPB * u < a.win ? (r0 + go[u]) * 8 : -8;  // negative: returns 0
                wv[u] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xrs, vo, 0, 0));
            }
        }
    }

    __device__ __forceinline__ void commit(const TplArgs& a, const TplLds& L) const {
        const int tid = threadIdx.x;
        if (NPL > 0 && pairs) {
#pragma unroll
            for (int u = 0; u < NP / 2; ++u) {
                const int i = 2 * (tid + kTPB * u);
                if (i < a.win) *(v2d_t*)(L.win + i) = v2d_t{wv[2 * u], wv[2 * u + 1]};
            }
        } else if (NPL > 0) {
#pragma unroll
            for (int u = 0; u < NP; ++u) {
                const int i = tid + kTPB * u;
                if (i < a.win) L.win[i] = wv[u];
            }
        }
    }
};

// the rows of one block: sums in CSR order, fused epilogue, y stores; returns the lane's
// (b - Ax)^2 sum for the norm
template <int MODE, bool NORM, int NPL>
__device__ __forceinline__ double tpl_rows(const TplArgs& a, const TplLds& L, __amdgpu_buffer_rsrc_t xrs,
                                           int r0, const int* id, const int* rr, const double* pb,
                                           const double* py) {
    constexpr int R = kTplRPL, C = 8;  // C: global-path loads per batch
    const int tid = threadIdx.x;
    int st[R], ln[R], dk[R], Lm = 0;
    double s[R], xr[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
        const unsigned h = (unsigned)L.hdr[id[j]];
        st[j] = (int)(h & 0xffffu);
        ln[j] = (int)((h >> 16) & 0xffu);
        dk[j] = (int)(h >> 24);
        Lm = max(Lm, ln[j]);
        s[j] = 0.0;
        xr[j] = 0.0;
        // Jacobi needs x[r]; a template without a diagonal entry reads it here (rare)
        if (MODE == KM_JACOBI && dk[j] == 255 && id[j] != kTplNone) xr[j] = a.x[rr[j]];
    }
    if constexpr (NPL > 0 && AMG_TPL_BATCH > 0) {
        // window, batched: both rows of the lane advance together, B entries per batch; the
        // slot reads of a batch are all issued before the window reads that depend on them,
        // so a batch waits on LDS twice instead of once per entry (A/B build knob)
        constexpr int B = AMG_TPL_BATCH > 0 ? AMG_TPL_BATCH : 1;
        const int elast = a.nent - 1;
        for (int k0 = 0; k0 < Lm; k0 += B) {
            int o[B][R];
            double xv[B][R];
#pragma unroll
            for (int u = 0; u < B; ++u)
#pragma unroll
                for (int j = 0; j < R; ++j) o[u][j] = L.off[min(st[j] + k0 + u, elast)];
#pragma unroll
            for (int u = 0; u < B; ++u)
#pragma unroll
                for (int j = 0; j < R; ++j) xv[u][j] = L.win[o[u][j] + kTPB * j + tid];
#pragma unroll
            for (int u = 0; u < B; ++u)
#pragma unroll
                for (int j = 0; j < R; ++j) {
                    const int k = k0 + u;
                    const double p = L.val[min(st[j] + k, elast)] * xv[u][j];
                    s[j] = k < ln[j] ? s[j] + p : s[j];
                    if (MODE == KM_JACOBI) xr[j] = k == dk[j] ? xv[u][j] : xr[j];
                }
        }
    } else if constexpr (NPL > 0) {
        // window: 4 entries per step -- runs start at multiples of 4 entries (padded,
        // build_templates), so one ds_read_b128 of slots and two of values serve 4 entries:
        // 5 LDS cycles per entry instead of 8 with per-entry reads (the template kernels are
        // LDS-bound on the 27-pt operator, profiles/r2w_tpl_sq_*.txt); entries past the row's
        // length are masked, the sum keeps CSR order
        // (the lane's two rows advancing together measured slower: 27-pt SpMV 159 vs 147 us,
        // profiles/r2w_wide_forms.txt)
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const int base = kTPB * j + tid;
            for (int k = 0; k < ln[j]; k += 4) {
                const int e = st[j] + k;
                const int4 o = *(const int4*)(L.off + e);
                const v2d_t v0 = *(const v2d_t*)(L.val + e), v1 = *(const v2d_t*)(L.val + e + 2);
                const double x0 = L.win[o.x + base], x1 = L.win[o.y + base];
                const double x2 = L.win[o.z + base], x3 = L.win[o.w + base];
                s[j] = s[j] + v0.x * x0;
                s[j] = k + 1 < ln[j] ? s[j] + v0.y * x1 : s[j];
                s[j] = k + 2 < ln[j] ? s[j] + v1.x * x2 : s[j];
                s[j] = k + 3 < ln[j] ? s[j] + v1.y * x3 : s[j];
            }
        }
        // Jacobi: x_r from the window at the diagonal entry (fewer registers than a select
        // per entry)
#pragma unroll
        for (int j = 0; j < R; ++j)
            if (MODE == KM_JACOBI && dk[j] != 255) xr[j] = L.win[L.off[st[j] + dk[j]] + kTPB * j + tid];
    } else {
        // global x: both rows of the lane advance together, C entries per batch, every load
        // of a batch issued before its first product
        const int elast = a.nent - 1;
        for (int k0 = 0; k0 < Lm; k0 += C) {
            double xv[C][R];
#pragma unroll
            for (int u = 0; u < C; ++u)
#pragma unroll
                for (int j = 0; j < R; ++j) {
                    const int k = k0 + u;
                    const int o = k < ln[j] ? L.off[min(st[j] + k, elast)] : 0;
                    xv[u][j] = __builtin_bit_cast(
                        double, __builtin_amdgcn_raw_buffer_load_b64(xrs, (rr[j] + o) * 8, 0, 0));
                }
            __builtin_amdgcn_sched_barrier(0);  // values read after the loads (register budget)
#pragma unroll
            for (int u = 0; u < C; ++u)
#pragma unroll
                for (int j = 0; j < R; ++j) {
                    const int k = k0 + u;
                    const double p = L.val[min(st[j] + k, elast)] * xv[u][j];
                    s[j] = k < ln[j] ? s[j] + p : s[j];
                    if (MODE == KM_JACOBI) xr[j] = k == dk[j] ? xv[u][j] : xr[j];
                }
        }
    }
    double sq = 0.0;
#pragma unroll
    for (int j = 0; j < R; ++j) {
        const bool own = id[j] != kTplNone;
        double out;
        if (MODE == KM_SPMV) {
            out = s[j];
        } else if (MODE == KM_SPMV_ADD) {
            out = py[j] + s[j];
        } else {
            const double t = pb[j] - s[j];
            if (NORM) sq += own ? t * t : 0.0;
            out = MODE == KM_RESID ? t : xr[j] + a.omega * (L.pd[MODE == KM_JACOBI ? id[j] : 0] * t);
        }
        if (own) a.y[r0 + kTPB * j + tid] = out;
    }
    return sq;
}

// Uniform-stencil rows (variant bit 512): every template is the master
// template with entries removed (DevMatrix::tpl_mne), so a row is an entry mask.  The master's
// values and window slots are kernel arguments (scalar registers, wave-uniform), and a lane
// reads only x from the window: per entry one LDS read, one address add, one multiply and one
// add, where tpl_rows reads slots and values from LDS tables and selects per entry (~10 VALU
// per entry: the 27-pt kernels were VALU-issue bound, profiles/r2w_tpl_sq_instr.txt).  In a
// wave whose rows are all the master the adds are unconditional; otherwise a lane adds only
// the entries its row has.  Each row's products and their order are its own CSR row's:
// results are bit-identical to tpl_rows (and the oracle).
// The lane's window base for each of its rows.  With AMG_TPL_SPLIT_READS the row stride (kTPB
// doubles) is hidden from the compiler, so the rows' reads of one entry stay two ds_read_b64
// (2 LDS cycles each) instead of being merged into one ds_read2st64_b64 (8 cycles for the same
// 1 KiB: MI355X_MICROARCH.md, LDS table); costs one address add per entry
template <int R>
__device__ __forceinline__ void tpl_row_bases(const TplLds& L, const double* (&wr)[R]) {
    int rs = kTPB;
#if AMG_TPL_SPLIT_READS
    asm volatile("" : "+v"(rs));
#endif
    const double* w0 = L.win + tpl_lrow<true>((int)threadIdx.x, 0);
#pragma unroll
    for (int j = 0; j < R; ++j) wr[j] = w0 + j * rs;
}

// The master's products of a lane's R rows, s[j] += v_e x_e in CSR order (masked entries add
// +0.0: s + (+0.0) == s bit for bit, s starts at +0.0 and a round-to-nearest sum is never -0.0
// unless both terms are).  (Issuing the window reads of 9 entries before their products, a
// round-4 build knob, ran slower: profiles/r4_ring_ab.txt.)
template <int MNE, int R, class Slot, class Val>
__device__ __forceinline__ void tpl_master_sums(const double* const (&wr)[R], const unsigned (&m)[R], bool full,
                                                Slot slot, Val val, double (&s)[R]) {
    constexpr int EB = 1;
    if (full) {
#pragma unroll
        for (int e0 = 0; e0 < MNE; e0 += EB) {
            double xv[EB][R];
#pragma unroll
            for (int u = 0; u < EB; ++u)
#pragma unroll
                for (int j = 0; j < R; ++j) xv[u][j] = e0 + u < MNE ? wr[j][slot(e0 + u)] : 0.0;
#pragma unroll
            for (int u = 0; u < EB; ++u)
#pragma unroll
                for (int j = 0; j < R; ++j)
                    if (e0 + u < MNE) s[j] = s[j] + val(e0 + u) * xv[u][j];
        }
    } else {
#pragma unroll
        for (int e0 = 0; e0 < MNE; e0 += EB) {
            double xv[EB][R];
#pragma unroll
            for (int u = 0; u < EB; ++u)
#pragma unroll
                for (int j = 0; j < R; ++j) xv[u][j] = e0 + u < MNE ? wr[j][slot(e0 + u)] : 0.0;
#pragma unroll
            for (int u = 0; u < EB; ++u) {
                const int e = e0 + u;
                if (e >= MNE) continue;
                const double v = val(e);
#if AMG_TPL_MASK_BRANCH
                double p[R];
#pragma unroll
                for (int j = 0; j < R; ++j) {
                    p[j] = v * xv[u][j];
                    asm volatile("" : "+v"(p[j]));
                }
#pragma unroll
                for (int j = 0; j < R; ++j)
                    if ((m[j] >> e) & 1u) {
                        asm volatile("" : "+v"(s[j]));
                        s[j] = s[j] + p[j];
                    }
#else
#pragma unroll
                for (int j = 0; j < R; ++j) {
                    // the addend, not the add, is selected (a branch per entry serialised the reads)
                    const double p = v * xv[u][j];
                    s[j] = s[j] + (((m[j] >> e) & 1u) ? p : 0.0);
                }
#endif
            }
        }
    }
}

// tpl_master_sums for the hybrid-GS old-value pass: acc[j] -= v_e x_e over the master's
// entries except the chain coupling EC of a row whose chain neighbour is in its chunk, sold[j]
// (NORM) += every product of the row (its A x for the residual norm); the same batched reads
template <int MNE, int EC, bool NORM, int R, class Slot, class Val>
__device__ __forceinline__ void tpl_master_gs_sums(const double* const (&wr)[R], const unsigned (&m)[R], bool full,
                                                   const bool (&chain)[R], Slot slot, Val val, double (&acc)[R],
                                                   double (&sold)[R]) {
    constexpr int EB = 1;
#pragma unroll
    for (int e0 = 0; e0 < MNE; e0 += EB) {
        double xv[EB][R];
#pragma unroll
        for (int u = 0; u < EB; ++u)
#pragma unroll
            for (int j = 0; j < R; ++j) xv[u][j] = e0 + u < MNE ? wr[j][slot(e0 + u)] : 0.0;
#pragma unroll
        for (int u = 0; u < EB; ++u) {
            const int e = e0 + u;
            if (e >= MNE) continue;
            const double v = val(e);
#pragma unroll
            for (int j = 0; j < R; ++j) {
                const double p = v * xv[u][j];
                if (full) {
                    if (NORM) sold[j] = sold[j] + p;
                    if (e == EC) acc[j] = acc[j] - (chain[j] ? 0.0 : p);
                    else acc[j] = acc[j] - p;
                } else {
                    // selected addends (tpl_rows_master): acc - (+0.0) == acc for every acc
                    const bool in = (m[j] >> e) & 1u;
                    if (NORM) sold[j] = sold[j] + (in ? p : 0.0);
                    acc[j] = acc[j] - (in && !(e == EC && chain[j]) ? p : 0.0);
                }
            }
        }
    }
}

template <int MODE, bool NORM, int MNE>
__device__ __forceinline__ double tpl_rows_master(const TplArgs& a, const TplLds& L, int r0, const int* id,
                                                  const double* pb, const double* py) {
    static_assert(MNE > 0 && MNE <= kTplMasterMax && MNE < 32, "master entry masks are 32-bit");
    constexpr int R = kTplRPL;
    constexpr unsigned kFull = (1u << MNE) - 1u;
    const int tid = threadIdx.x;
    unsigned m[R];
    bool full = true;
#pragma unroll
    for (int j = 0; j < R; ++j) {
        m[j] = (unsigned)L.hdr[id[j]];
        full = full && m[j] == kFull;
    }
    const double* wr[R];
    tpl_row_bases<R>(L, wr);
    double s[R];
#pragma unroll
    for (int j = 0; j < R; ++j) s[j] = 0.0;
    tpl_master_sums<MNE, R>(wr, m, __all(full), [&](int e) { return a.mslot[e]; }, [&](int e) { return a.mval[e]; }, s);
    double sq = 0.0;
#pragma unroll
    for (int j = 0; j < R; ++j) {
        const bool own = id[j] != kTplNone;
        double out;
        if (MODE == KM_SPMV) {
            out = s[j];
        } else if (MODE == KM_SPMV_ADD) {
            out = py[j] + s[j];
        } else {
            const double t = pb[j] - s[j];
            if (NORM) sq += own ? t * t : 0.0;
            // Jacobi: x_r from the window at the master's diagonal slot (every template has it)
            out = MODE == KM_RESID ? t : wr[j][a.mslot[a.mdiag]] + a.omega * (a.mpd * t);
        }
        if (own) a.y[r0 + tpl_lrow<true>(tid, j)] = out;
    }
    return sq;
}

template <int MODE, bool NORM, int NPL, int MNE>
__device__ __forceinline__ double tpl_rows_any(const TplArgs& a, const TplLds& L, __amdgpu_buffer_rsrc_t xrs,
                                               int r0, const int* id, const int* rr, const double* pb,
                                               const double* py) {
    if constexpr (MNE > 0) {
        static_assert(NPL > 0, "uniform-stencil rows read the x window");
        return tpl_rows_master<MODE, NORM, MNE>(a, L, r0, id, pb, py);
    } else {
        return tpl_rows<MODE, NORM, NPL>(a, L, xrs, r0, id, rr, pb, py);
    }
}

template <bool NORM>
__device__ __forceinline__ void tpl_partial(const TplArgs& a, int blk, double sq) {
    if (NORM) {
        sq = wave_sum(sq);
        if ((threadIdx.x & 63) == 0) a.partial[blk * kNormParts + (threadIdx.x >> 6)] = sq;
    }
}


// waves per SIMD the persistent and marching forms are compiled for: windows of more than
// 8 slots per lane (27-pt: 3084 doubles, ~34 KiB of LDS with the table) fit 4 workgroups per
// CU, i.e. 4 waves per SIMD, so those forms may use 128 VGPRs (at 6 they spilled their
// register-prefetched window to scratch)
constexpr int tpl_waves(int npl) { return npl > 8 ? 4 : 6; }
// the 7-pt marching form at 7 waves (72 VGPRs): its Jacobi + norm variant took 74 at 6 waves
// (a wave per SIMD fewer than the plain Jacobi: 101 vs 83 us per launch)
#ifndef AMG_MARCH_NORM_WAVES  // build-time A/B knob: waves per SIMD of the 7-pt Jacobi + norm form
#define AMG_MARCH_NORM_WAVES 7
#endif
constexpr int tpl_march_waves(int npl, bool norm) { return npl == 8 ? (norm ? AMG_MARCH_NORM_WAVES : 7) : tpl_waves(npl); }

// one workgroup per block of kTplRows rows
template <int MODE, bool NORM, int NPL, int MNE = 0>
__global__ __launch_bounds__(kTPB, 6) void tpl_kernel(TplArgs a) {
    const TplLds L = tpl_lds_layout<MODE>(a);
    const __amdgpu_buffer_rsrc_t xrs = tpl_xrs(a);
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int r0 = blk * kTplRows;
    TplFetch<MODE, NPL, (MNE > 0)> f;
    f.issue(a, xrs, r0);  // row operands and window first: independent of the table
    tpl_stage_table<MODE, MNE>(a, L);
    f.commit(a, L);
    __syncthreads();
    tpl_partial<NORM>(a, blk, tpl_rows_any<MODE, NORM, NPL, MNE>(a, L, xrs, r0, f.id, f.rr, f.pb, f.py));
}

// Persistent form of the window path: a grid of resident workgroups (a multiple of 8), XCD
// x = blockIdx % 8 owning a contiguous 1/8 of the blocks, its workgroups sweeping them side by
// side (iteration i: blocks start_x + i * per + lw), so an XCD's L2 holds the planes its
// workgroups share.  The table is staged once; the next block's row operands and window are
// fetched into registers while the current block is computed from LDS (double buffering
// through registers), so the load latency overlaps the arithmetic.
template <int MODE, bool NORM, int NPL, int MNE = 0>
__global__ __launch_bounds__(kTPB, tpl_waves(NPL)) void tpl_persist_kernel(TplArgs a, int nblk) {
    static_assert(NPL > 0, "window path only");
    const TplLds L = tpl_lds_layout<MODE>(a);
    const __amdgpu_buffer_rsrc_t xrs = tpl_xrs(a);
    const int x = blockIdx.x & 7, lw = blockIdx.x >> 3, per = gridDim.x >> 3;
    const int q = nblk >> 3, rem = nblk & 7;
    const int b0 = x * q + min(x, rem), b1 = b0 + q + (x < rem ? 1 : 0);
    int blk = b0 + lw;
    if (blk >= b1) return;  // workgroup-uniform: no barrier is skipped by part of a group
    // f: the next block's ids and window (registers); c: the current block's row operands
    TplFetch<MODE, NPL, (MNE > 0)> f, c;
    f.issue_ids(a, blk * kTplRows);
    f.issue_window(a, xrs, blk * kTplRows);
    tpl_stage_table<MODE, MNE>(a, L);
    for (;;) {
        f.commit(a, L);
#pragma unroll
        for (int j = 0; j < kTplRPL; ++j) c.id[j] = f.id[j], c.rr[j] = f.rr[j];
        c.issue_operands(a);  // b / y: needed only at the end of the rows below
        __syncthreads();      // window (and, first time, table) visible
        const int nxt = blk + per;
        if (nxt < b1) {  // in flight during the rows below
            f.issue_ids(a, nxt * kTplRows);
            f.issue_window(a, xrs, nxt * kTplRows);
        }
        tpl_partial<NORM>(a, blk, tpl_rows_any<MODE, NORM, NPL, MNE>(a, L, xrs, blk * kTplRows, c.id, c.rr, c.pb, c.py));
        if (nxt >= b1) break;
        __syncthreads();  // every wave is done reading the window before it is overwritten
        blk = nxt;
    }
}

// z-marching form of the window path (variant bit 128).  Workgroup chains
// walk blocks c, c + S, c + 2S, ... (S blocks = the shift D the host found, e.g. one plane of
// the 7-pt operator), so the -plane band and the middle of the centre band of a block are
// the previous block's centre and +plane bands: those slots are copied inside LDS (wsrc) and
// only the rest is loaded -- 1024 instead of 2048 doubles per 7-pt block.  The next block's
// loaded slots and row ids are prefetched into registers during the current block.
template <int MODE, bool NORM, int NPL, int MNE = 0>
__global__ __launch_bounds__(kTPB, tpl_march_waves(NPL, NORM)) void tpl_march_kernel(TplArgs a, int nblk, int S, int nchunk) {
    static_assert(NPL > 0 && NPL % 2 == 0, "window path, slot pairs");
    constexpr int NP = NPL / 2;  // slot pairs per lane (16-byte loads and LDS copies)
    const TplLds L = tpl_lds_layout<MODE>(a);
    const __amdgpu_buffer_rsrc_t xrs = tpl_xrs(a);
    const int tid = threadIdx.x;
    // pair u of this lane: slots i, i + 1 with i = 2 (tid + kTPB u); bands have even starts
    // and lengths and the shift is even, so both slots of a pair share their source
    int gof[NP], src[NP];
    tpl_slot_offsets<2>(a, gof);
#pragma unroll
    for (int u = 0; u < NP; ++u) {
        const int i = 2 * (tid + kTPB * u);
        src[u] = i < a.win ? a.wsrc[i] : -2;  // -2: pair past the window
    }
    tpl_stage_table<MODE, MNE>(a, L);
    const int K = (nblk + S - 1) / S;           // blocks per column
    const int per = (K + nchunk - 1) / nchunk;  // blocks per chain
    // chains ordered (chunk, column); XCD x = blockIdx % 8 takes a contiguous 1/8 of them, so
    // the workgroups of one XCD walk neighbouring columns of the same planes side by side
    const int C = S * nchunk, x = blockIdx.x & 7, lw = blockIdx.x >> 3, nw = gridDim.x >> 3;
    const int c0 = x * (C >> 3) + min(x, C & 7), c1 = c0 + (C >> 3) + (x < (C & 7) ? 1 : 0);
    TplFetch<MODE, NPL, (MNE > 0)> f, c;
    v2d_t gv[NP];
    for (int ch = c0 + lw; ch < c1; ch += nw) {
        const int col = ch % S, t0 = (ch / S) * per, t1 = min(K, t0 + per);
        if (t0 >= t1 || col + S * t0 >= nblk) continue;  // workgroup-uniform
        // first block of the chain: every pair from x (out-of-range pairs load 0)
        f.issue_ids(a, (col + S * t0) * kTplRows);
#pragma unroll
        for (int u = 0; u < NP; ++u)
            gv[u] = __builtin_bit_cast(v2d_t, __builtin_amdgcn_raw_buffer_load_b128(
                xrs, src[u] != -2 ? ((col + S * t0) * kTplRows + gof[u]) * 8 : -16, 0, 0));
        for (int t = t0; t < t1; ++t) {
            const int blk = col + S * t;
            if (blk >= nblk) break;  // uniform
            const int r0 = blk * kTplRows;
            const bool first = t == t0;
            v2d_t wv[NP];
#pragma unroll
            for (int u = 0; u < NP; ++u) wv[u] = (!first && src[u] >= 0) ? *(const v2d_t*)(L.win + src[u]) : gv[u];
#pragma unroll
            for (int j = 0; j < kTplRPL; ++j) c.id[j] = f.id[j], c.rr[j] = f.rr[j];
            c.issue_operands(a);
            __syncthreads();  // every wave is done with the previous window (rows and copies)
#pragma unroll
            for (int u = 0; u < NP; ++u)
                if (src[u] != -2) *(v2d_t*)(L.win + 2 * (tid + kTPB * u)) = wv[u];
            __syncthreads();
            const int nb = blk + S;
            if (t + 1 < t1 && nb < nblk) {  // in flight during the rows below
                f.issue_ids(a, nb * kTplRows);
#pragma unroll
                for (int u = 0; u < NP; ++u)
                    gv[u] = src[u] == -1 ? __builtin_bit_cast(v2d_t, __builtin_amdgcn_raw_buffer_load_b128(
                                               xrs, (nb * kTplRows + gof[u]) * 8, 0, 0))
                                         : v2d_t{0.0, 0.0};
            }
            tpl_partial<NORM>(a, blk, tpl_rows_any<MODE, NORM, NPL, MNE>(a, L, xrs, r0, c.id, c.rr, c.pb, c.py));
        }
        __syncthreads();  // the next chain's first window overwrites this one
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
    const uint8_t* vid;  // DICT: 1-byte value indices (4 entries of a lane per dword)
    const double* vtab;  // DICT: the value table
    int ndict;
    int slab0;           // first slab of this launch (waves index slabs slab0 + wave)
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
// DICT: the operator's values come from a <= 256-entry table staged in LDS, through 1-byte
// indices loaded four entries per dword (5 B per ELL cell instead of 12).
template <bool BACK, bool WIDE, bool NORM, bool DICT>
__global__ __launch_bounds__(WIDE ? 64 : 256) void hybrid_gs_kernel(GsArgs a) {
    constexpr int U = WIDE ? 16 : 8;
    static_assert(U % 4 == 0, "dictionary dwords hold 4 entries");
    __shared__ double dtab[DICT ? 256 : 1];
    if (DICT) {
        for (int i = threadIdx.x; i < a.ndict; i += blockDim.x) dtab[i] = a.vtab[i];
        __syncthreads();
    }
    // wave index made provably uniform: slab fields land in SGPRs, the step loop is scalar.
    // XCD-aware (r6): consecutive slabs -- rows that share x lines -- on one XCD's L2
    // (xcd_remap); slabs of one sweep are independent, so results do not change.  G3
    // substitute level 0: 60.0 -> 59.1 us per sweep, 2,370 -> 2,393 V-cycles/s (profiles/r6/r6g3_*)
    const int blk = xcd_remap((int)blockIdx.x, (int)gridDim.x);
    const int wave = __builtin_amdgcn_readfirstlane(
        (int)(WIDE ? blk : blk * 4 + (threadIdx.x >> 6))) + a.slab0;
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
    const uint8_t* vidp = a.vid + (size_t)sl.z * 64 + 4 * (size_t)lane;  // DICT
    auto vbyte = [&](int k) { return (int)vidp[(size_t)(k & ~3) * 64 + (k & 3)]; };
    __shared__ double chainL[WIDE ? 64 * 64 : 1];
    double s_old = 0.0;           // NORM: sum_j a_ij x_j (old x), for ||b - A x||
    unsigned long long mask = 0;  // WIDE: bit t = coupling to slab row t
    int kf = -1, kl = -1;         // narrow: first / last chain entry of the row
    // software pipeline: block k0 + U's (col, val) stream in while block k0 gathers x
    int cn[U];
    double vn[U];
    unsigned wn[U / 4];  // DICT: the next step's value-index dwords (looked up when consumed)
    auto fetch = [&](int k0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in = k0 + u < sl.w;  // uniform
            cn[u] = in ? __builtin_nontemporal_load(colp + (size_t)(k0 + u) * 64) : -1;
            if (!DICT) vn[u] = in ? __builtin_nontemporal_load(valp + (size_t)(k0 + u) * 64) : 0.0;
        }
        if (DICT) {
#pragma unroll
            for (int q = 0; q < U / 4; ++q)
                wn[q] = k0 + 4 * q < sl.w
                            ? __builtin_nontemporal_load((const unsigned*)(vidp + (size_t)(k0 + 4 * q) * 64))
                            : 0u;
        }
    };
    fetch(0);
    for (int k0 = 0; k0 < sl.w; k0 += U) {
        int c[U];
        double v[U], xv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) c[u] = cn[u];
        if (DICT) {
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = dtab[(wn[u >> 2] >> (8 * (u & 3))) & 0xffu];
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = vn[u];
        }
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
                vv = DICT ? dtab[vbyte(kn)] : valp[(size_t)kn * 64];
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
    if (NORM) {  // ||b - A x_old||^2 partial of this slab (wave_sum: fixed order)
        const double rr = live ? a.b[r] - s_old : 0.0;
        double q = rr * rr;
        q = wave_sum(q);
        if (lane == 0) a.partial[wave] = q;
    }
}

// l1 hybrid Gauss-Seidel on row templates, for operators whose in-chunk
// couplings are the +-1 neighbours only (a stencil with its x line along the chunk).  Rows
// whose (template, l1 diagonal) pair is shared -- boundary class x position of the row in its
// GS chunk -- stream a 1-byte GS-template id.  Two kernels per sweep:
//  tpl_gs_acc_kernel  (lane = row, 512-row blocks, the template x window in LDS):
//      acc_i = b_i - sum of the old-value couplings in CSR order (diagonal included; the
//      chain coupling -- offset -1 forward / +1 backward when that neighbour is in the
//      row's chunk -- skipped), stored to `racc`; NORM: (b - A x_old)^2 partials
//  tpl_gs_chain_kernel (lane = chunk, 256 chunks per workgroup):
//      the chunk's rows in sweep order, 8 rows of (acc, x, id) per batch in registers with
//      the next batch in flight: acc -= a_i,i-+1 x'_prev; x'_i = x_i + acc * dinv_l1.
// The oracle's order exactly (one chain coupling, subtracted after the old ones).  The chain
// is a sequential recurrence per chunk; lane = chunk runs 64 chunks per wave instruction.  A
// single-kernel form (same recurrence walked by 8 lanes of a 512-row block, or broadcast with
// v_readlane by every row's lane) took 880-920 / 727 us per 27-pt 256^3 sweep.
struct TplGsArgs {
    TplArgs t;           // id = GS-template id per row; hdr = base template header per GS
                         // template; off = window slots; val; y = racc (acc kernel)
    const int* ke;       // per GS template: the chain entry's index in the row (-1: none)
    const int* blocks;   // the 512-row blocks on the template path
    int nblk;
    long long first_row;
    int B;
    int part_off;        // NORM: partial of block list entry q, wave w at part_off + 4 q + w
};

// MNE > 0 (variant bit 512): uniform stencil, L.hdr holds each GS template's master-entry
// mask (tpl_rows_master); the chain coupling is master entry EC (offset -1 forward, +1
// backward: 2 / 4 of the 7-pt master, 12 / 14 of the 27-pt one -- launch_tpl_gs checks)
template <bool BACK, bool NORM, int NPL, int MNE = 0>
__global__ __launch_bounds__(kTPB, 6) void tpl_gs_acc_kernel(TplGsArgs g) {
    static_assert(NPL > 0, "window path only");
    constexpr int R = kTplRPL;
    const TplArgs& a = g.t;
    const TplLds L = tpl_lds_layout<KM_RESID>(a);
    int* loffr = L.hdr + kTplMax + 1;  // per GS template: index (in the row) of its chain entry
    const int tid = threadIdx.x, lane = tid & 63;
    const __amdgpu_buffer_rsrc_t xrs = tpl_xrs(a);
    const int q = xcd_remap(blockIdx.x, gridDim.x);
    const int r0 = (g.blocks ? g.blocks[q] : q) * kTplRows;  // null list: every block (no dependent load)
    TplFetch<KM_RESID, NPL, (MNE > 0)> f;  // ids, b, window
    f.issue(a, xrs, r0);
    tpl_stage_table<KM_RESID, MNE>(a, L);
    if (MNE == 0 && tid < a.ntpl) loffr[tid] = g.ke[tid];
    f.commit(a, L);
    __syncthreads();
    double sq = 0.0;
    // the chain neighbour is in the row's chunk (chunks = global multiples of B; the rank
    // start is a multiple of 64 and B | 64, so pos = i mod B and only the rank end clips)
    bool chain[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
        const int i = r0 + tpl_lrow<(MNE > 0)>(tid, j), pos = i & (g.B - 1);
        chain[j] = BACK ? (pos != g.B - 1 && i + 1 < a.n) : pos != 0;
    }
    if constexpr (MNE > 0) {
        static_assert(MNE == 7 || MNE == 27, "chain entry of the instantiated masters");
        constexpr int EC = MNE == 27 ? (BACK ? 14 : 12) : (BACK ? 4 : 2);
        constexpr unsigned kFull = (1u << MNE) - 1u;
        unsigned m[R];
        bool full = true;
        double acc[R], sold[R];
#pragma unroll
        for (int j = 0; j < R; ++j) {
            m[j] = (unsigned)L.hdr[f.id[j]];
            full = full && m[j] == kFull;
            acc[j] = f.pb[j];
            sold[j] = 0.0;
        }
        const double* wr[R];
        tpl_row_bases<R>(L, wr);
        if (__all(full))
            tpl_master_gs_sums<MNE, EC, NORM, R>(wr, m, true, chain, [&](int e) { return a.mslot[e]; },
                                                 [&](int e) { return a.mval[e]; }, acc, sold);
        else
            tpl_master_gs_sums<MNE, EC, NORM, R>(wr, m, false, chain, [&](int e) { return a.mslot[e]; },
                                                 [&](int e) { return a.mval[e]; }, acc, sold);
#pragma unroll
        for (int j = 0; j < R; ++j)
            if (f.id[j] != kTplNone) {
                a.y[r0 + tpl_lrow<true>(tid, j)] = acc[j];
                if (NORM) {
                    const double rr = f.pb[j] - sold[j];
                    sq += rr * rr;
                }
            }
    } else {
#pragma unroll
    for (int j = 0; j < R; ++j) {
        const int lr = kTPB * j + tid, i = r0 + lr;
        const unsigned h = (unsigned)L.hdr[f.id[j]];
        const int st = (int)(h & 0xffffu), ln = (int)((h >> 16) & 0xffu);
        // template entry of the chain coupling (loffr holds the ntpl GS templates only)
        const int ke = chain[j] && f.id[j] != kTplNone ? loffr[f.id[j]] : -1;
        double acc = f.pb[j], sold = 0.0;
        for (int k = 0; k < ln; k += 4) {  // 4 entries per step, as in tpl_rows
            const int e = st + k;
            const int4 o = *(const int4*)(L.off + e);
            const v2d_t v0 = *(const v2d_t*)(L.val + e), v1 = *(const v2d_t*)(L.val + e + 2);
            const double p[4] = {v0.x * L.win[o.x + lr], v0.y * L.win[o.y + lr], v1.x * L.win[o.z + lr],
                                 v1.y * L.win[o.w + lr]};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const bool in = k + u < ln;
                if (NORM) sold = in ? sold + p[u] : sold;
                acc = in && k + u != ke ? acc - p[u] : acc;
            }
        }
        if (f.id[j] != kTplNone) {
            a.y[i] = acc;
            if (NORM) {
                const double rr = f.pb[j] - sold;
                sq += rr * rr;
            }
        }
    }
    }
    if (NORM) {
        sq = wave_sum(sq);
        if (lane == 0) a.partial[g.part_off + 4 * q + (tid >> 6)] = sq;
    }
}

struct TplGsChainArgs {
    const double* racc;
    const double* x;
    const uint8_t* id;
    const double* dl;    // per GS template: 1 / (a_ii + l1)
    const double* cv;    // per GS template: coefficient of the chain neighbour (-1 fwd, +1 bwd)
    const int* cf;       // per GS template: bit 0 has the -1 entry, bit 1 the +1 entry
    int ntpl;
    const int* blocks;
    int nblk;
    int B;
    int n;
    long long first_row;
    double* y;
};

// One wave per 64 chunks.  Batch k = rows 8k .. 8k+7 of every chunk: the wave loads the
// batch's 64-byte lines cooperatively (16 bytes per lane, 4 lanes per line, each line read
// once) into LDS while the previous batch is walked, then lane c walks chunk c's 8 rows from
// LDS.  (Lane c loading its own chunk's lines took 161 us per 27-pt 256^3 sweep: 64 distinct
// lines per wave instruction, each fetched again by the next quarter-line load.)
template <bool BACK>
__global__ __launch_bounds__(64) void tpl_gs_chain_kernel(TplGsChainArgs a) {
    // 16 rows per batch: a chunk's batch is one whole 128-byte line of acc, x and y (8 rows =
    // half lines left the other half to be fetched again a batch later: FETCH_SIZE 1.84x the
    // algorithmic reads, WRITE_SIZE 1.25x, profiles/r4mn_gs_pmc.txt)
    constexpr int U = 16;
    // per-GS-template tables sized by the launch (ntpl entries; 27-pt: 27): a wave-sized
    // workgroup with 5 KiB of fixed 256-entry tables fit 11 per CU, 3.7 TB/s on the 27-pt sweep
    extern __shared__ __attribute__((aligned(16))) double chain_lds[];
    double* sdl = chain_lds;
    double* scv = sdl + a.ntpl;
    int* scf = (int*)(scv + a.ntpl);
    // stage of one batch, row-major by batch row u with a padded stride (kSt = 65): lane c's
    // walk reads u * kSt + c (consecutive lanes, no bank conflict); chunk-major [c][u] had a
    // 64-byte lane stride and a 16-way conflict on every read of the walk
    constexpr int kSt = 65;
    __shared__ __attribute__((aligned(16))) double sacc[kSt * U], sx[kSt * U];
    __shared__ __attribute__((aligned(16))) unsigned sid[64 * (U / 4)];
    const int lane = threadIdx.x;
    constexpr int kBit = BACK ? 2 : 1;
    for (int k = lane; k < a.ntpl; k += 64) {
        sdl[k] = a.dl[k];
        scv[k] = a.cv[k];
        scf[k] = a.cf[k] & kBit;
    }
    const int cpb = kTplRows / a.B;  // chunks per block
    const long long nq = (long long)a.nblk * cpb;
    const long long q0 = (long long)blockIdx.x * 64;
    auto cstart = [&](long long qc) {
        return (a.blocks ? a.blocks[qc / cpb] : (int)(qc / cpb)) * kTplRows + (int)(qc % cpb) * a.B;
    };
    // my chunk
    const long long qc = q0 + lane;
    const bool live = qc < nq;
    const int c0 = live ? cstart(qc) : 0;
    const int c1 = live ? min(c0 + a.B, a.n) : 0;
    // fast path: B % U == 0 and every chunk of the wave whole (wave-uniform)
    const bool whole = a.B % U == 0 && q0 + 64 <= nq && __all(c1 - c0 == a.B);
    __syncthreads();
    double prev = 0.0;
    if (whole) {
        // load assignment u (8 per array): line of chunk 8 u + lane / 8, 16-byte piece lane % 8
        constexpr int NL = U / 2;  // 16-byte pieces per lane per array
        int ls[NL];
#pragma unroll
        for (int u = 0; u < NL; ++u) ls[u] = cstart(q0 + (64 / NL) * u + lane / NL) + 2 * (lane % NL);
        const int nb = a.B / U;
        v2d_t ra[NL], rx[NL];
        v4u_t ri;  // the lane's chunk's U one-byte template ids of the batch
        auto load = [&](int bi) {
            const int off = (BACK ? nb - 1 - bi : bi) * U;
#pragma unroll
            for (int u = 0; u < NL; ++u) {
                ra[u] = __builtin_nontemporal_load((const v2d_t*)(a.racc + ls[u] + off));
                rx[u] = *(const v2d_t*)(a.x + ls[u] + off);
            }
            ri = *(const v4u_t*)(a.id + c0 + off);
        };
        // stage slot of load piece u: rows 2 (lane % NL), + 1 of chunk (64 / NL) u + lane / NL
        auto slot_of = [&](int u) { return 2 * (lane % NL) * kSt + (64 / NL) * u + lane / NL; };
        load(0);
        for (int bi = 0; bi < nb; ++bi) {
#pragma unroll
            for (int u = 0; u < NL; ++u) {
                const int slot = slot_of(u);
                sacc[slot] = ra[u].x;
                sacc[slot + kSt] = ra[u].y;
                sx[slot] = rx[u].x;
                sx[slot + kSt] = rx[u].y;
            }
            *(v4u_t*)(sid + 4 * lane) = ri;
            __syncthreads();
            if (bi + 1 < nb) load(bi + 1);  // in flight during the walk below
            double out[U];
            const v4u_t iv = *(const v4u_t*)(sid + 4 * lane);
            const unsigned iw[4] = {iv.x, iv.y, iv.z, iv.w};
#pragma unroll
            for (int t = 0; t < U; ++t) {
                const int u = BACK ? U - 1 - t : t;
                const int tp = (int)((iw[u >> 2] >> (8 * (u & 3))) & 0xffu);
                double acc = sacc[u * kSt + lane];
                // the chunk's first row in sweep order has no chain neighbour; a template
                // without the neighbour entry (boundary row) has none either
                if ((bi > 0 || t > 0) && scf[tp]) acc -= scv[tp] * prev;
                prev = sx[u * kSt + lane] + acc * sdl[tp];
                out[u] = prev;
            }
            // x' back through the stage: whole 128-byte lines per 8 lanes, like the loads
#pragma unroll
            for (int u = 0; u < U; ++u) sacc[u * kSt + lane] = out[u];
            __syncthreads();
            const int off = (BACK ? nb - 1 - bi : bi) * U;
#pragma unroll
            for (int u = 0; u < NL; ++u) {
                const int slot = slot_of(u);
                *(v2d_t*)(a.y + ls[u] + off) = v2d_t{sacc[slot], sacc[slot + kSt]};
            }
            __syncthreads();  // the stage is rewritten by the next batch
        }
    } else if (live) {
        // clipped chunk (the rank's last rows), a partial wave, or B not a multiple of U
        for (int t = 0; t < c1 - c0; ++t) {
            const int i = BACK ? c1 - 1 - t : c0 + t;
            const int tp = a.id[i];
            double acc = a.racc[i];
            if (t > 0 && scf[tp]) acc -= scv[tp] * prev;
            prev = a.x[i] + acc * sdl[tp];
            a.y[i] = prev;
        }
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
__device__ __forceinline__ double block_sum_span(int n, const double* p, int g, double* red) {
    const int base = g * kRedSpan + threadIdx.x;
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
    return (red[0] + red[1]) + (red[2] + red[3]);  // meaningful in thread 0
}

__global__ __launch_bounds__(kTPB) void sum_partials_kernel(int n, const double* p, double* out) {
    __shared__ double red[kTPB / 64];
    const double s = block_sum_span(n, p, blockIdx.x, red);
    if (threadIdx.x == 0) out[blockIdx.x] = s;
}

// The same two stages (n <= kRedSpan^2) and the single-rank finish in ONE launch: each block
// writes its span's sum, then an agent-scope acq_rel counter picks the last block to arrive,
// which sums the block sums exactly as the second sum_partials_kernel would, appends sqrt to
// hist and resets the counter (bit-identical to reduce + finish, two launches fewer per norm).
// Visibility (MI355X_MICROARCH.md, inter-workgroup): the writer's release orders its store of
// tmp[g]; the last block's acquire (one lane) and barrier precede its plain loads.
__global__ __launch_bounds__(kTPB) void reduce_norm_kernel(int n, const double* p, double* tmp,
                                                           unsigned* done, double* out, double* hist,
                                                           int* counter) {
    __shared__ double red[kTPB / 64];
    __shared__ int last;
    const int g = gridDim.x;
    const double s = block_sum_span(n, p, blockIdx.x, red);
    if (threadIdx.x == 0) {
        tmp[blockIdx.x] = s;
        const unsigned prev = __hip_atomic_fetch_add(done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        last = prev == (unsigned)(g - 1);
    }
    __syncthreads();
    if (!last) return;  // workgroup-uniform
    __syncthreads();    // red[] is reused below
    const double t = block_sum_span(g, tmp, 0, red);
    if (threadIdx.x == 0) {
        *done = 0u;
        out[0] = t;
        double f = 0.0;
        f += t;  // finish_norm_kernel's sum over one rank
        hist[*counter] = sqrt(f);
        *counter += 1;
    }
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

// coarsest level: x_i = sum_j inv_ij b_j, one wavefront per row: lane l sums
// j = l, l + 64, ... in order from 0.0 (coalesced reads of the row-major inverse row), then a
// fixed xor butterfly -- the oracle's coarse_row() exactly.  (The round-1 kernel walked each row
// sequentially in one lane: 27 waves for the 1,709-row G3 substitute, 110 us on a 23 MB inverse.)
__global__ __launch_bounds__(256) void dense_gemv_kernel(long long nl, long long n, const double* inv,
                                                         const double* b, double* x) {
    const long long i = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (i >= nl) return;  // wave-uniform
    const double* row = inv + i * n;
    double s = 0.0;
    long long j = lane;
    // four products' loads in flight per step; the lane's sum stays sequential in j
    for (; j + 192 < n; j += 256) {
        const double p0 = row[j] * b[j], p1 = row[j + 64] * b[j + 64];
        const double p2 = row[j + 128] * b[j + 128], p3 = row[j + 192] * b[j + 192];
        s += p0;
        s += p1;
        s += p2;
        s += p3;
    }
    for (; j < n; j += 64) s += row[j] * b[j];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s = s + __shfl_xor(s, m, 64);
    if (lane == 0) x[i] = s;
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

int kernel_variant(const DevMatrix& A) {
    // variant bits: 2 = XCD-ordered blocks, 4 = gather path (no x tile), 8 = value-indexed
    // blocks (when any block qualifies), 32 = row templates (when built), 128 = z-marching
    // template windows (default when a
    // shift with enough reuse exists and the window is <= 2048 doubles: 7-pt level 0 74.5 vs
    // 80.6 us, profiles/r1u_march_ab.txt; the 27-pt window of 3078 doubles ran 204 vs 154 us,
    // profiles/r1u_sa27_kernel_stats.csv against r1t).  Default
    // (DevMatrix::default_variant): x tile for square operators, gather for rectangular ones
    // (stored without tiles), both in XCD order (profiles/r1m_variants.txt), VI and templates
    // where built.  AMG_KERNEL_VARIANT overrides the bits (experiments,
    // scripts/spmv_variants.py; results are identical).
    const char* ev = getenv("AMG_KERNEL_VARIANT");
    int var = ev ? atoi(ev) : (A.default_variant | (A.n_vi_blocks > 0 ? 8 : 0) | (A.n_tpl > 0 ? 32 : 0) |
                                (A.tpl_march_s > 0 && A.tpl_win <= 8 * kTPB ? 128 : 0));
    if (A.n_vi_blocks == 0) var &= ~8;
    if (A.n_tpl == 0) var &= ~32;
    // AMG_FORMAT_BLOCKS: the CSR block kernel on every row (no templates)
    if (A.format == AMG_FORMAT_BLOCKS) var &= ~(32 | 128);
    // each operator is stored for one kernel: square -> x tile, rectangular -> gather
    if (A.tiled) var &= ~4;
    else var |= 4;
    // 256: gather path with 16-bit column codes, where built (DevMatrix::col16; default on,
    // AMG_GATHER_C16=0 turns it off for A/B runs)
    if (!ev && !A.tiled && A.col16.p) {
        const char* e = std::getenv("AMG_GATHER_C16");
        if (!(e && std::atoi(e) == 0)) var |= 256;
    }
    if (!A.col16.p) var &= ~256;
    // 512: uniform-stencil template rows, default where the templates are
    // one master's subsequences (DevMatrix::tpl_mne; AMG_TPL_MASTER=0 at build turns it off)
    if (!ev && A.tpl_mne > 0) var |= 512;
    if (A.tpl_mne == 0) var &= ~512;
    return var;
}

bool DevMatrix::tpl_on() const { return n_tpl > 0 && (kernel_variant(*this) & 32); }

int DevMatrix::norm_parts() const {
    if (format == AMG_FORMAT_CSR) return plain_blocks() * kNormParts;
    return tpl_on() ? (tpl_blocks() + nb_int + nb_bnd - nb_skip) * kNormParts
                    : (nb_int + nb_bnd) * kNormParts;
}

// window path: the persistent kernel with a grid of exactly the resident workgroups (its
// blocks are split statically, so a workgroup that waited for a slot would double the tail),
// or one workgroup per block when that is no more
template <int M, bool N, int P, int K>
static void launch_tpl_window(hipStream_t s, const TplArgs& a, int g, size_t lds) {
    // larger windows: the one-block kernel (27-pt SpMV 146 us; the persistent form 164,
    // marching 153: profiles/r2w_wide_forms.txt)
    if (P > 8) {
        hipLaunchKernelGGL((tpl_kernel<M, N, P, K>), dim3(g), dim3(kTPB), lds, s, a);
        return;
    }
    thread_local int cus = 0, occ = 0;
    thread_local size_t occ_lds = 0;
    if (cus == 0) {
        int dev = 0;
        HIP_CHECK(hipGetDevice(&dev));
        HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    if (occ_lds != lds) {
        HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, tpl_persist_kernel<M, N, P, K>, kTPB, lds));
        occ_lds = lds;
    }
    const int gp = std::min(g, cus * occ) / 8 * 8;
    if (gp >= 8 && g > gp)
        hipLaunchKernelGGL((tpl_persist_kernel<M, N, P, K>), dim3(gp), dim3(kTPB), lds, s, a, g);
    else
        hipLaunchKernelGGL((tpl_kernel<M, N, P, K>), dim3(g), dim3(kTPB), lds, s, a);
}

// AMG_TPL_MARCH_CHUNKS caps the chains per column (tests: longer chains, so the LDS reuse
// branch runs on small grids; 0 = no cap)
int tpl_march_chunk_cap() {
    const char* e = std::getenv("AMG_TPL_MARCH_CHUNKS");
    return e ? std::max(0, std::atoi(e)) : 0;
}

template <int M, bool N, int P, int K>
static void launch_tpl_march(hipStream_t s, const TplArgs& a, int g, size_t lds, int S) {
    if constexpr (P > 0) {
        // CU count and occupancy per LDS size cached per instantiation (no runtime queries
        // on the eager multi-rank path)
        thread_local int ncu = 0, occ = 0;
        thread_local size_t occ_lds = 0;
        if (ncu == 0) {
            int dev = 0;
            HIP_CHECK(hipGetDevice(&dev));
            HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        }
        if (occ_lds != lds) {
            HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, tpl_march_kernel<M, N, P, K>, kTPB, lds));
            occ_lds = lds;
        }
        const int res = std::max(8, std::max(1, occ) * ncu / 8 * 8);  // resident workgroups
        int nchunk = std::max(1, res / S);                              // chains per column
        const int cap = tpl_march_chunk_cap();
        if (cap > 0) nchunk = std::min(nchunk, cap);
        const int gp = std::max(8, std::min(res, (S * nchunk + 7) / 8 * 8));
        hipLaunchKernelGGL((tpl_march_kernel<M, N, P, K>), dim3(gp), dim3(kTPB), lds, s, a, g, S, nchunk);
    }
}

void launch_tpl(hipStream_t s, int mode, bool norm, const DevMatrix& A, const double* x,
                const double* b, double* y, double omega, double* partial) {
    const int g = A.tpl_blocks();
    if (g <= 0) return;
    AMG_ASSERT(A.square && A.n_tpl > 0 && A.n_tpl <= kTplMax && A.n_tpl_ent <= kTplEntries);
    const bool win = A.tpl_win > 0;
    TplArgs a{};
    a.id = A.tpl_id.p;
    a.hdr = A.tpl_hdr.p;
    a.off = win ? A.tpl_ldo.p : A.tpl_off.p;
    a.val = A.tpl_val.p;
    a.pd = A.tpl_pd.p;
    a.ntpl = A.n_tpl;
    a.nent = A.n_tpl_ent;
    a.n = (int)A.n_rows;
    a.nband = win ? (int)A.tpl_blo.size() : 0;
    a.win = win ? A.tpl_win : 0;
    a.wend = win ? A.tpl_wend : 0;
    for (int q = 0; q < a.nband; ++q) a.blo[q] = A.tpl_blo[q], a.bbase[q] = A.tpl_bbase[q];
    a.bbase[a.nband] = a.win;
    for (int q = a.nband; q < kTplBands; ++q) a.blo[q] = 0, a.bbase[q + 1] = a.win;
    tpl_chunk_tables(a);
    a.x = x;
    a.b = b;
    a.y = y;
    a.omega = omega;
    a.partial = partial;
    // uniform stencil (variant bit 512): entry masks instead of the template tables
    const int mne = win && (kernel_variant(A) & 512) ? A.tpl_mne : 0;
    if (mne > 0) {
        AMG_ASSERT(mne <= kTplMasterMax && (int)A.tpl_mslot.size() == mne && A.tpl_mmask.n >= (size_t)A.n_tpl);
        a.hdr = (const int*)A.tpl_mmask.p;
        a.nent = 0;
        a.mdiag = A.tpl_mdiag;
        a.mpd = A.tpl_mpd;
        for (int e = 0; e < mne; ++e) a.mslot[e] = A.tpl_mslot[e], a.mval[e] = A.tpl_mval[e];
    }
    const int npl = !win ? 0 : a.win <= 4 * kTPB ? 4 : a.win <= 8 * kTPB ? 8 : a.win <= 12 * kTPB ? 12 : 16;
    AMG_ASSERT(a.win <= npl * kTPB && a.win <= kTplWin);
    const size_t lds = tpl_lds_bytes(a.win, a.nent, mode == KM_JACOBI);
    const bool march = win && A.tpl_march_s > 0 && (kernel_variant(A) & 128);
    if (march) a.wsrc = A.tpl_wsrc.p;
#define AMG_T3(M, N, P, K)                                                     \
    do {                                                                       \
        if (march) launch_tpl_march<M, N, P, K>(s, a, g, lds, A.tpl_march_s);  \
        else launch_tpl_window<M, N, P, K>(s, a, g, lds);                      \
    } while (0)
#define AMG_T2(M, N, P)                       \
    do {                                      \
        if (mne == 7) AMG_T3(M, N, P, 7);     \
        else if (mne == 27) AMG_T3(M, N, P, 27); \
        else AMG_T3(M, N, P, 0);              \
    } while (0)
#define AMG_T(M, N)                              \
    do {                                         \
        switch (npl) {                           \
            case 4: AMG_T2(M, N, 4); break;      \
            case 8: AMG_T2(M, N, 8); break;      \
            case 12: AMG_T2(M, N, 12); break;    \
            case 16: AMG_T2(M, N, 16); break;    \
            default: hipLaunchKernelGGL((tpl_kernel<M, N, 0>), dim3(g), dim3(kTPB), lds, s, a); break; \
        }                                        \
    } while (0)
    switch (mode) {
        case KM_SPMV: AMG_T(KM_SPMV, false); break;
        case KM_SPMV_ADD: AMG_T(KM_SPMV_ADD, false); break;
        case KM_RESID:
            if (norm) AMG_T(KM_RESID, true);
            else AMG_T(KM_RESID, false);
            break;
        case KM_JACOBI:
            if (norm) AMG_T(KM_JACOBI, true);
            else AMG_T(KM_JACOBI, false);
            break;
        default: throw Error(AMG_ERR_INTERNAL, "bad kernel mode");
    }
#undef AMG_T
#undef AMG_T2
#undef AMG_T3
    HIP_CHECK(hipGetLastError());
}

template <int M, bool N, bool X, bool T, bool V>
static void launch_block(hipStream_t s, dim3 g, const CsrArgs& a, int first_block, bool rpb4, int lw) {
    if constexpr (T) {
        if (lw == 4) {  // 32-byte x-tile lines
            if constexpr (!N && (M == KM_SPMV || M == KM_SPMV_ADD)) {
                if (rpb4) {
                    hipLaunchKernelGGL((csr_block_kernel<M, N, X, T, V, kGatherRPB, false, 4>), g, dim3(kTPB), 0, s, a, first_block);
                    return;
                }
            }
            hipLaunchKernelGGL((csr_block_kernel<M, N, X, T, V, 1, false, 4>), g, dim3(kTPB), 0, s, a, first_block);
            return;
        }
    }
    if constexpr (!N && (M == KM_SPMV || M == KM_SPMV_ADD)) {
        if (!T && a.col16) {
            if (rpb4) hipLaunchKernelGGL((csr_block_kernel<M, N, X, T, V, kGatherRPB, !T>), g, dim3(kTPB), 0, s, a, first_block);
            else hipLaunchKernelGGL((csr_block_kernel<M, N, X, T, V, 1, !T>), g, dim3(kTPB), 0, s, a, first_block);
            return;
        }
        if (rpb4) {
            hipLaunchKernelGGL((csr_block_kernel<M, N, X, T, V, kGatherRPB>), g, dim3(kTPB), 0, s, a, first_block);
            return;
        }
    }
    hipLaunchKernelGGL((csr_block_kernel<M, N, X, T, V>), g, dim3(kTPB), 0, s, a, first_block);
}

void launch_csr_stream(hipStream_t s, int mode, bool norm, const DevMatrix& A, int first_block,
                       int n_blocks, const double* x, const double* b, double* y, double omega,
                       double* partial, int part_off, double* y2, const double* d2) {
    if (n_blocks <= 0) return;
    const int ncl = (int)A.n_cols_local, nh = (int)A.n_halo();
    AMG_ASSERT(!y2 || (mode == KM_SPMV && d2));
    CsrArgs a{A.hdr.p, A.tile_fixed.p, A.lcol.p, A.vidx.p, A.vtab.p, A.rend.p, A.dvi.p,
              A.rp.p, A.col.p, A.val.p,
              x, A.halo.p, ncl, nh, (ncl + A.line_w - 1) / A.line_w, (ncl >= 2 && nh != 1) ? 1 : 0, A.tiled ? 0 : 1,
              b, y2 ? d2 : A.dinv.p, y, omega, partial, part_off, y2, nullptr, A.gband.p, n_blocks};
    const dim3 g(n_blocks);
    const int var = kernel_variant(A);
    if (var & 256) a.col16 = A.col16.p;
    const bool rpb4 = A.gather_rpb > 1;
#define AMG_L1(M, N, X, T, V) launch_block<M, N, X, T, V>(s, g, a, first_block, rpb4, A.line_w)
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
#if AMG_CSR_PHASES
    // diagnostic build: every launch of a tiled operator dumps its blocks' stamps
    const char* phase_file = A.tiled ? std::getenv("AMG_CSR_PHASES_FILE") : nullptr;
    // never freed: a static's hipFree at exit would run after the runtime's teardown
    static DevBuf<unsigned long long>& phase_buf = *new DevBuf<unsigned long long>();
    if (phase_file) {
        if (phase_buf.n < (size_t)n_blocks * 8) phase_buf.alloc((size_t)n_blocks * 8);
        HIP_CHECK(hipMemsetAsync(phase_buf.p, 0, sizeof(unsigned long long) * n_blocks * 8, s));
        unsigned long long* p = phase_buf.p;
        HIP_CHECK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_csr_phase), &p, sizeof(p), 0, hipMemcpyHostToDevice, s));
        HIP_CHECK(hipStreamSynchronize(s));
    }
#endif
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
        case KM_GSACC:
            AMG_CHECK(!norm && A.square, "GS acc pass: square operator, no norm");
            AMG_L(KM_GSACC, false);
            break;
        default: throw Error(AMG_ERR_INTERNAL, "bad kernel mode");
    }
#if AMG_CSR_PHASES
    if (phase_file) {
        HIP_CHECK(hipStreamSynchronize(s));
        std::vector<unsigned long long> h((size_t)n_blocks * 8);
        HIP_CHECK(hipMemcpy(h.data(), phase_buf.p, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
        unsigned long long* z = nullptr;
        HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_csr_phase), &z, sizeof(z)));
        if (FILE* fp = std::fopen(phase_file, "ab")) {
            const long long hdr[4] = {mode, n_blocks, (long long)A.n_rows, (long long)A.nnz};
            std::fwrite(hdr, sizeof(hdr), 1, fp);
            std::fwrite(h.data(), sizeof(unsigned long long), h.size(), fp);
            std::fclose(fp);
        }
    }
#endif
#undef AMG_L
#undef AMG_L2
#undef AMG_L1
    HIP_CHECK(hipGetLastError());
}

void launch_csr_plain(hipStream_t s, int mode, bool norm, const DevMatrix& A, const double* x,
                      const double* b, double* y, double omega, double* partial) {
    const int g = A.plain_blocks();
    if (g <= 0) return;
    AMG_ASSERT(A.pcol.p != nullptr && A.pval.p != nullptr);
    PlainArgs a{A.rp.p, A.pcol.p, A.pval.p, x, A.halo.p, (int)A.n_cols_local, (int)A.n_rows,
                b, A.dinv.p, y, omega, partial};
#define AMG_PL(M, N) hipLaunchKernelGGL((csr_plain_kernel<M, N>), dim3(g), dim3(kTPB), 0, s, a)
    switch (mode) {
        case KM_SPMV: AMG_PL(KM_SPMV, false); break;
        case KM_SPMV_ADD: AMG_PL(KM_SPMV_ADD, false); break;
        case KM_RESID:
            if (norm) AMG_PL(KM_RESID, true);
            else AMG_PL(KM_RESID, false);
            break;
        case KM_JACOBI:
            if (norm) AMG_PL(KM_JACOBI, true);
            else AMG_PL(KM_JACOBI, false);
            break;
        default: throw Error(AMG_ERR_INTERNAL, "bad kernel mode");
    }
#undef AMG_PL
    HIP_CHECK(hipGetLastError());
}

int64_t read_partials(int64_t n) { return std::max<int64_t>(1, (n / 2 + 4 * kTPB - 1) / (4 * kTPB)) * 4; }

void launch_read(hipStream_t s, int64_t n, const double* src, double* part) {
    AMG_CHECK(((uintptr_t)src & 15) == 0, "read: 16-byte aligned vector");
    const long long np = n / 2;
    if (np <= 0) return;
    const long long g = (np + 4 * kTPB - 1) / (4 * kTPB);
    AMG_CHECK(g < INT_MAX, "read: vector too long");
    hipLaunchKernelGGL(read_kernel, dim3((unsigned)g), dim3(kTPB), 0, s, np, (const v2d_t*)src, part);
    HIP_CHECK(hipGetLastError());
}

void launch_copy(hipStream_t s, int64_t n, const double* src, double* dst) {
    if (n <= 0) return;
    AMG_CHECK(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0, "copy: 16-byte aligned vectors");
    const long long np = n / 2;
    if (np > 0) {
        const long long g = (np + 4 * kTPB - 1) / (4 * kTPB);
        AMG_CHECK(g < INT_MAX, "copy: vector too long");
        hipLaunchKernelGGL(copy_kernel, dim3((unsigned)g), dim3(kTPB), 0, s, np, (const v2d_t*)src, (v2d_t*)dst);
        HIP_CHECK(hipGetLastError());
    }
    if (n & 1) HIP_CHECK(hipMemcpyAsync(dst + n - 1, src + n - 1, sizeof(double), hipMemcpyDeviceToDevice, s));
}

// acc kernel LDS: the template kernel's RESID layout + the entries' column offsets
// + the per-GS-template chain-entry table, sized by the templates in use: at kTplMax + 1 ints
// the 27-pt acc kernel needed 32.7 KiB and fit 4 workgroups per CU against the residual's 5
// (its LDS is 31.6 KiB): 205-211 vs 165-170 us per launch
inline size_t tpl_gs_lds_bytes(int win, int nent, int ntpl) {
    return tpl_lds_bytes(win, nent, false) + 4 * (((size_t)ntpl + 4) & ~(size_t)3);
}

static void launch_tpl_gs(hipStream_t s, const DevMatrix& A, const double* x, const double* b,
                          double* y, bool backward, double* partial) {
    AMG_ASSERT(A.n_gs_tblk > 0 && A.tpl_win > 0 && A.n_tpl_ent <= kTplEntries);
    AMG_ASSERT(A.gs_racc.n >= (size_t)A.n_rows);
    TplGsArgs g{};
    TplArgs& a = g.t;
    a.id = A.gs_tid.p;
    a.hdr = A.gs_thdr.p;
    a.off = A.tpl_ldo.p;
    a.val = A.tpl_val.p;
    a.pd = A.gs_tdl.p;
    a.ntpl = A.n_gs_tpl;
    a.nent = A.n_tpl_ent;
    a.n = (int)A.n_rows;
    a.nband = (int)A.tpl_blo.size();
    a.win = A.tpl_win;
    a.wend = A.tpl_wend;
    for (int q = 0; q < a.nband; ++q) a.blo[q] = A.tpl_blo[q], a.bbase[q] = A.tpl_bbase[q];
    a.bbase[a.nband] = a.win;
    for (int q = a.nband; q < kTplBands; ++q) a.blo[q] = 0, a.bbase[q + 1] = a.win;
    tpl_chunk_tables(a);
    a.x = x;
    a.b = b;
    a.y = A.gs_racc.p;
    a.partial = partial;
    g.ke = backward ? A.gs_tkep.p : A.gs_tkem.p;
    // every block on the template path (27-pt): no block list to load before the window
    const bool all_blocks = A.n_gs_tblk == A.tpl_blocks();
    g.blocks = all_blocks ? nullptr : A.gs_tblocks.p;
    g.nblk = A.n_gs_tblk;
    g.first_row = A.first_row;
    g.B = (int)A.gs_block;
    g.part_off = A.n_gs_slabs;
    // uniform stencil (variant bit 512): GS-template entry masks; the kernel's chain entry is
    // master entry 2 / 4 (7-pt) or 12 / 14 (27-pt): offsets -1 / +1
    const int mne = (kernel_variant(A) & 512) && A.gs_tmask.p &&
                            ((A.tpl_mne == 7 && A.tpl_mem == 2 && A.tpl_mep == 4) ||
                             (A.tpl_mne == 27 && A.tpl_mem == 12 && A.tpl_mep == 14))
                        ? A.tpl_mne
                        : 0;
    if (mne > 0) {
        a.hdr = (const int*)A.gs_tmask.p;
        a.nent = 0;
        a.mdiag = A.tpl_mdiag;
        a.mpd = A.tpl_mpd;
        for (int e = 0; e < mne; ++e) a.mslot[e] = A.tpl_mslot[e], a.mval[e] = A.tpl_mval[e];
    }
    const bool norm = partial != nullptr;
    const dim3 grid(g.nblk), blk(kTPB);
    const int npl = a.win <= 4 * kTPB ? 4 : a.win <= 8 * kTPB ? 8 : a.win <= 12 * kTPB ? 12 : 16;
    AMG_ASSERT(a.win <= npl * kTPB && a.win <= kTplWin);
    const size_t lds = tpl_gs_lds_bytes(a.win, a.nent, a.ntpl);
#define AMG_G3(BK, NM, P, K) hipLaunchKernelGGL((tpl_gs_acc_kernel<BK, NM, P, K>), grid, blk, lds, s, g)
#define AMG_G2(BK, NM, P)                          \
    do {                                           \
        if (mne == 7) AMG_G3(BK, NM, P, 7);        \
        else if (mne == 27) AMG_G3(BK, NM, P, 27); \
        else AMG_G3(BK, NM, P, 0);                 \
    } while (0)
#define AMG_G(BK, NM)                         \
    do {                                      \
        switch (npl) {                        \
            case 4: AMG_G2(BK, NM, 4); break;   \
            case 8: AMG_G2(BK, NM, 8); break;   \
            case 12: AMG_G2(BK, NM, 12); break; \
            default: AMG_G2(BK, NM, 16); break; \
        }                                     \
    } while (0)
    if (backward) AMG_G(true, false);
    else if (norm) AMG_G(false, true);
    else AMG_G(false, false);
#undef AMG_G
#undef AMG_G2
#undef AMG_G3
    HIP_CHECK(hipGetLastError());
    TplGsChainArgs c{A.gs_racc.p, x, A.gs_tid.p, A.gs_tdl.p, backward ? A.gs_tcvp.p : A.gs_tcvm.p,
                     A.gs_tcf.p, A.n_gs_tpl, g.blocks, A.n_gs_tblk, (int)A.gs_block, (int)A.n_rows,
                     (long long)A.first_row, y};
    const long long nch = (long long)A.n_gs_tblk * (kTplRows / A.gs_block);
    const dim3 cg((unsigned)((nch + 63) / 64)), cb(64);
    const size_t clds = (size_t)c.ntpl * (8 + 8 + 4);
    if (backward) hipLaunchKernelGGL((tpl_gs_chain_kernel<true>), cg, cb, clds, s, c);
    else hipLaunchKernelGGL((tpl_gs_chain_kernel<false>), cg, cb, clds, s, c);
    HIP_CHECK(hipGetLastError());
}

void launch_hybrid_gs(hipStream_t s, const DevMatrix& A, const double* x, const double* b,
                      double* y, bool backward, double* partial, int s0, int s1, bool tpl) {
    AMG_ASSERT(!(backward && partial));
    if (tpl && A.n_gs_tblk > 0) launch_tpl_gs(s, A, x, b, y, backward, partial);
    if (s1 <= s0) return;
    GsArgs a{A.gs_slabs.p, A.gs_col.p, A.gs_val.p, x, A.halo.p, (int)A.n_cols_local, b,
             A.gs_dinv.p, y, (long long)A.first_row, (long long)A.gs_block, (int)A.n_rows,
             s1, partial, A.gs_vid.p, A.gs_vtab.p, A.gs_ndict, s0};
    const bool wide = A.gs_wide;
    const int ns = s1 - s0;
    const dim3 grid(wide ? ns : (ns + 3) / 4), block(wide ? 64 : 256);
#define AMG_GS(BK, WD, NM)                                                                          \
    do {                                                                                            \
        if (A.gs_ndict > 0) hipLaunchKernelGGL((hybrid_gs_kernel<BK, WD, NM, true>), grid, block, 0, s, a); \
        else hipLaunchKernelGGL((hybrid_gs_kernel<BK, WD, NM, false>), grid, block, 0, s, a);      \
    } while (0)
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

// Chain walk of a split sweep: one wave per slab, lane = row.  The lane's
// in-chunk new-value couplings come from a sliced ELL stored in consumption order (forward:
// ascending j, backward: descending j; padding col -1) and are staged in the wave's LDS column
// `lane` first, so phase 2 -- hybrid_gs_kernel's column sweep: at step t the row j that is final
// now is broadcast with v_readlane, every lane whose next coupling is j subtracts a_ij x'_j --
// reads its next entry from LDS instead of waiting on a global load inside the step loop.
// acc comes from the KM_GSACC pass (b - old couplings), so the result is the oracle's.
template <bool BACK, int W>
__global__ __launch_bounds__(64) void gs_chain_kernel(GsArgs a) {
    __shared__ double qv[W * 64];
    __shared__ int qc[W * 64];
    const int wave = __builtin_amdgcn_readfirstlane((int)blockIdx.x) + a.slab0;
    if (wave >= a.nslab) return;
    const int lane = threadIdx.x;
    const int4 sl = a.slabs[wave];
    const int r = sl.x + lane;
    const bool live = lane < sl.y;
    double acc = 0.0, xi = 0.0, dinv = 0.0;
    if (live) {
        acc = a.b[r];
        xi = a.x[r];
        dinv = a.dinv[r];
    }
    const size_t base = (size_t)sl.z * 64 + lane;
    // the slab's couplings into the LDS queue: up to 32 entries per lane in flight at once (one
    // memory round for W <= 32, two for W = 64).  Loading 8 at a time put W / 8 dependent
    // rounds in every wave's life (~11 us per launch whatever the grid, profiles/r4f_*)
    constexpr int KR = W < 32 ? W : 32;  // entries per round
    for (int k0 = 0; k0 < sl.w; k0 += KR) {  // sl.w <= W (launch_gs_chain)
        int c[KR];
        double v[KR];
#pragma unroll
        for (int u = 0; u < KR; ++u) {
            const bool in = k0 + u < sl.w;  // uniform
            c[u] = in ? __builtin_nontemporal_load(a.col + base + (size_t)(k0 + u) * 64) : -1;
            v[u] = in ? __builtin_nontemporal_load(a.val + base + (size_t)(k0 + u) * 64) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < KR; ++u) {
            if (k0 + u < sl.w) {
                qc[(k0 + u) * 64 + lane] = c[u];
                qv[(k0 + u) * 64 + lane] = v[u];
            }
        }
    }
    // each lane reads back only its own LDS column: no barrier
    int p = 0;
    int cn = sl.w > 0 ? qc[lane] : -1;
    double vn = sl.w > 0 ? qv[lane] : 0.0;
    for (int t = 0; t < sl.y; ++t) {
        const int j = BACK ? sl.y - 1 - t : t;  // lane whose row is final now
        const double xj = bcast_lane(xi + acc * dinv, j);
        if (cn == sl.x + j) {
            acc -= vn * xj;
            ++p;
            cn = p < sl.w ? qc[p * 64 + lane] : -1;
            vn = p < sl.w ? qv[p * 64 + lane] : 0.0;
        }
    }
    if (live) a.y[r] = xi + acc * dinv;
}

void launch_gs_chain(hipStream_t s, const DevMatrix& A, const double* x, const double* acc,
                     double* y, bool backward) {
    const int d = backward ? 1 : 0;
    const int ns = A.n_gs_slabs;
    if (ns <= 0) return;
    GsArgs a{A.gs_cslabs[d].p, A.gs_ccol[d].p, A.gs_cval[d].p, x, A.halo.p, (int)A.n_cols_local, acc,
             A.gs_dinv.p, y, (long long)A.first_row, (long long)A.gs_block, (int)A.n_rows,
             ns, nullptr, nullptr, nullptr, 0, 0};
    AMG_ASSERT(A.gs_cmaxw[d] <= 64);  // <= 63: in-chunk couplings of a <= 64-row chunk
    AMG_ASSERT(A.gs_cbucket[d][kGsChainBuckets] == ns);
    // one launch, at the widest slab's width bucket (DevMatrix::gs_cbucket)
    for (int q = 0; q < kGsChainBuckets; ++q) {
        const int b0 = A.gs_cbucket[d][q], b1 = A.gs_cbucket[d][q + 1];
        if (b1 <= b0) continue;
        a.slab0 = b0;
        a.nslab = b1;
#define AMG_GC(W)                                                                                     \
    do {                                                                                              \
        if (backward) hipLaunchKernelGGL((gs_chain_kernel<true, W>), dim3(b1 - b0), dim3(64), 0, s, a); \
        else hipLaunchKernelGGL((gs_chain_kernel<false, W>), dim3(b1 - b0), dim3(64), 0, s, a);         \
    } while (0)
        static_assert(kGsChainW[0] == 8 && kGsChainW[1] == 16 && kGsChainW[2] == 32 && kGsChainW[3] == 64, "");
        if (q == 0) AMG_GC(8);
        else if (q == 1) AMG_GC(16);
        else if (q == 2) AMG_GC(32);
        else AMG_GC(64);
#undef AMG_GC
    }
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

bool launch_reduce_norm(hipStream_t s, int n, const double* partial, double* tmp, unsigned* done,
                        double* out, double* hist, int* counter) {
    if (n <= 0 || n > kRedSpan * kRedSpan || !done) return false;
    const int g = (n + kRedSpan - 1) / kRedSpan;
    hipLaunchKernelGGL(reduce_norm_kernel, dim3(g), dim3(kTPB), 0, s, n, partial, tmp, done, out, hist, counter);
    HIP_CHECK(hipGetLastError());
    return true;
}

void launch_finish_norm(hipStream_t s, int n, const double* in, double* hist, int* counter) {
    hipLaunchKernelGGL(finish_norm_kernel, dim3(1), dim3(64), 0, s, n, in, hist, counter);
    HIP_CHECK(hipGetLastError());
}

void launch_dense_gemv(hipStream_t s, int64_t n_local, int64_t n, const double* inv,
                       const double* bfull, double* x) {
    if (n_local <= 0) return;
    hipLaunchKernelGGL(dense_gemv_kernel, dim3((unsigned)((n_local + 3) / 4)), dim3(256), 0, s,
                       (long long)n_local, (long long)n, inv, bfull, x);
    HIP_CHECK(hipGetLastError());
}

void launch_uniform(hipStream_t s, int64_t n, int64_t first_gid, uint64_t seed, double* out) {
    if (n <= 0) return;
    hipLaunchKernelGGL(uniform_kernel, dim3(grid_for(n)), dim3(kTPB), 0, s, (long long)n,
                       (long long)first_gid, (unsigned long long)seed, out);
    HIP_CHECK(hipGetLastError());
}

}  // namespace amg
