// par_matrix.hip -- ParCSRMatrix on the GPU.
//
// Layout in HBM: rank-local rows, int32 row_ptr, int32 column ids
// renumbered [0, n_cols_local) local | [n_cols_local, +n_halo) halo, fp64 values, fp64
// 1/a_ii.  Columns stay in ascending GLOBAL order inside a row, so row sums are identical
// for any partition.  Row blocks are split into "interior" (no halo column) and
// "boundary" lists: the interior kernel runs while RCCL moves the halo on a second
// stream; the boundary kernel runs after the halo event.
#include <algorithm>
#include <atomic>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <unordered_map>

#include "device.hpp"

namespace amg {

// Zero-filled host staging buffer, written in parallel: std::vector's value-initialising
// constructor zeroes on one thread (0.1-0.2 s for the 1-2 GB of a 256^3 level's streams)
template <class T>
struct ParZeros {
    std::unique_ptr<T[]> p;
    size_t n = 0;
    explicit ParZeros(size_t count) : p(new T[count > 0 ? count : 1]), n(count) {
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < (int64_t)count; ++i) p[i] = T();
    }
    T* data() { return p.get(); }
    const T* data() const { return p.get(); }
    size_t size() const { return n; }
    T& operator[](size_t i) { return p[i]; }
    const T& operator[](size_t i) const { return p[i]; }
    T* begin() { return p.get(); }
};

// ---- staged host <-> device copies (device.hpp) ----------------------------------------
namespace {

constexpr size_t kStageChunk = size_t(32) << 20;

// two pinned chunks + a copy stream per (device, user); kept for the process lifetime
struct Stage {
    int device = -1;
    bool busy = false;
    hipStream_t s = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    char* buf[2] = {nullptr, nullptr};
};

std::mutex g_stage_mu;
std::vector<Stage*> g_stages;

Stage* stage_acquire() {
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> g(g_stage_mu);
    for (Stage* st : g_stages)
        if (!st->busy && st->device == dev) {
            st->busy = true;
            return st;
        }
    std::unique_ptr<Stage> st(new Stage());
    st->device = dev;
    HIP_CHECK(hipStreamCreateWithFlags(&st->s, hipStreamNonBlocking));
    for (int b = 0; b < 2; ++b) {
        HIP_CHECK(hipEventCreateWithFlags(&st->ev[b], hipEventDisableTiming));
        HIP_CHECK(hipHostMalloc((void**)&st->buf[b], kStageChunk, hipHostMallocDefault));
    }
    st->busy = true;
    g_stages.push_back(st.get());
    return st.release();
}

void stage_release(Stage* st) {
    std::lock_guard<std::mutex> g(g_stage_mu);
    st->busy = false;
}

struct StageLease {
    Stage* st;
    StageLease() : st(stage_acquire()) {}
    ~StageLease() { stage_release(st); }
};

void par_memcpy(void* dst, const void* src, size_t bytes) {
    const int64_t parts = (int64_t)std::max<size_t>(1, bytes >> 21);  // 2 MiB pieces
#pragma omp parallel for schedule(static)
    for (int64_t q = 0; q < parts; ++q) {
        const size_t a = bytes * (size_t)q / (size_t)parts, b = bytes * (size_t)(q + 1) / (size_t)parts;
        std::memcpy((char*)dst + a, (const char*)src + a, b - a);
    }
}

}  // namespace

void copy_to_device(void* dst, const void* src, size_t bytes) {
    if (bytes < (size_t(4) << 20)) {
        if (bytes) HIP_CHECK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
        return;
    }
    StageLease L;
    Stage& S = *L.st;
    size_t c = 0;
    for (size_t off = 0; off < bytes; off += kStageChunk, ++c) {
        const int b = (int)(c & 1);
        const size_t len = std::min(kStageChunk, bytes - off);
        if (c >= 2) HIP_CHECK(hipEventSynchronize(S.ev[b]));  // the DMA out of this buffer is done
        par_memcpy(S.buf[b], (const char*)src + off, len);
        HIP_CHECK(hipMemcpyAsync((char*)dst + off, S.buf[b], len, hipMemcpyHostToDevice, S.s));
        HIP_CHECK(hipEventRecord(S.ev[b], S.s));
    }
    HIP_CHECK(hipStreamSynchronize(S.s));
}

void copy_to_host(void* dst, const void* src, size_t bytes, hipStream_t after) {
    if (after) HIP_CHECK(hipStreamSynchronize(after));
    if (bytes < (size_t(4) << 20)) {
        if (bytes) HIP_CHECK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
        return;
    }
    StageLease L;
    Stage& S = *L.st;
    const size_t nc = (bytes + kStageChunk - 1) / kStageChunk;
    auto issue = [&](size_t c) {
        const size_t off = c * kStageChunk, len = std::min(kStageChunk, bytes - off);
        HIP_CHECK(hipMemcpyAsync(S.buf[c & 1], (const char*)src + off, len, hipMemcpyDeviceToHost, S.s));
        HIP_CHECK(hipEventRecord(S.ev[c & 1], S.s));
    };
    issue(0);
    for (size_t c = 0; c < nc; ++c) {
        if (c + 1 < nc) issue(c + 1);  // into the other buffer, emptied in the previous round
        HIP_CHECK(hipEventSynchronize(S.ev[c & 1]));
        const size_t off = c * kStageChunk, len = std::min(kStageChunk, bytes - off);
        par_memcpy((char*)dst + off, S.buf[c & 1], len);
    }
}

Context::~Context() {
    loopback_leave(*this);
    if (nccl) (void)ncclCommDestroy(nccl);
    if (ev_pack) (void)hipEventDestroy(ev_pack);
    if (ev_halo) (void)hipEventDestroy(ev_halo);
    if (comm_stream) (void)hipStreamDestroy(comm_stream);
    if (own_stream && stream) (void)hipStreamDestroy(stream);
}

// Row blocks of the CSR-stream kernel: <= kCAP nonzeros, <= kTPB rows, one class (interior /
// boundary), and <= kCAP / lw distinct lines of x (lw = 8 or 4 doubles; local lines first,
// then halo lines).  Each block gets its sorted line list ("x tile") and every nonzero a
// 16-bit index into the tile: slot * lw + (column mod lw).  A single row touching more lines
// than a tile holds becomes a block of its own and takes the untiled path.
struct BlockBuild {
    std::vector<int2> blocks;     // interior all-templated, other interior, then boundary blocks
    std::vector<int> tile_ptr;    // nb + 1
    std::vector<int> tile_lines;  // global line ids per block
    hvec<uint16_t> lcol;          // per nonzero (nnz + kPad)
    int nb_int = 0, nb_bnd = 0, nb_skip = 0;  // nb_skip: leading interior all-templated blocks
};

// tplf (optional): per row 1 = handled by the template kernel; blocks then also break where it
// changes, and all-templated interior blocks come first
// sample > 1: cut only every sample-th chunk (statistics for the format choices below; no
// tile indices)
static BlockBuild build_row_blocks(const std::vector<int>& rp, const hvec<int>& col,
                                   const std::vector<uint8_t>& cls, int64_t ncl, int64_t nhalo,
                                   const std::vector<uint8_t>* tplf = nullptr, int row_cap = kTPB,
                                   bool line_cap = true, bool want_lcol = true, int lw = 8, int sample = 1) {
    if (sample > 1) want_lcol = false;
    const int n = (int)rp.size() - 1;
    const int sh = lw == 8 ? 3 : 2, tl_cap = kCAP / lw;
    AMG_ASSERT(lw == 8 || lw == 4);
    const int64_t hl0 = (ncl + lw - 1) / lw;
    auto line_of = [&](int c) -> int64_t { return c < ncl ? c >> sh : hl0 + ((c - ncl) >> sh); };
    struct Rec {
        int r0, r1;
        std::vector<int> lines;
        bool bnd, tpl;
    };
    BlockBuild out;
    // every entry below col.size() is written by the block that holds it; the pad is zero.
    // want_lcol = false: the tile indices are built on the device (formats.hip)
    if (want_lcol) {
        out.lcol.resize(col.size() + kPad);
        std::fill(out.lcol.begin() + (int64_t)(rp.back()), out.lcol.end(), (uint16_t)0);
    }
    // The greedy cut runs independently on a fixed number of row chunks (each chunk starts a
    // block at its first row), in parallel: blocks never change the arithmetic (rows never
    // straddle a block), and a fixed chunk count keeps the cut independent of the thread count.
    // Sequential, the cut took 0.4-0.7 s per 256^3-level operator.
    // (r5: also operators of few but long rows -- sa27's R1, 49,492 rows of ~270 entries, took
    // 0.45 s in one chunk)
    const int nch = n >= (1 << 16) || (n >= (1 << 12) && rp.back() >= (1 << 20)) ? 64 : 1;
    std::vector<std::vector<Rec>> recs((size_t)nch);
    // Each thread keeps the open block's lines (and the current row's new ones) in an
    // open-addressing table with a generation per slot: a slot of an older generation (block)
    // reads as empty, so closing a block clears nothing.  Sized for one block's lines (<= its
    // entries: kCAP, or one longer row) plus one row's.  r5: per-thread arrays indexed by line
    // id (16 B per line of the column space, filled per call) cost more than the cut itself on
    // level-0 operators (0.54 s for a 16.7 M-column operator on 16 threads).
    int max_row = 0;
#pragma omp parallel for reduction(max : max_row) schedule(static)
    for (int i = 0; i < n; ++i) max_row = std::max(max_row, rp[i + 1] - rp[i]);
    int hb = 10;
    while (((size_t)1 << hb) < 2 * ((size_t)kCAP + 2 * (size_t)max_row)) ++hb;
    const size_t H = (size_t)1 << hb;
#pragma omp parallel if (nch > 1)
    {
        std::vector<int64_t> hkey(H), hrow(H);
        std::vector<int> hgen(H, -1), hpos(H);
        std::vector<char> hin(H);
        std::vector<int> lines, cand;
        std::vector<size_t> cslot;
        int blk = 0;  // per thread, never reset: generations stay unique across chunks
        size_t used = 0;
        // the slot of line L in the open block's generation (inserted: not in the block, no row)
        auto find = [&](int64_t L) -> size_t {
            size_t h = (size_t)(((uint64_t)L * 0x9E3779B97F4A7C15ull) >> (64 - hb));
            for (;;) {
                if (hgen[h] != blk) {
                    AMG_ASSERT(++used < H);
                    hgen[h] = blk;
                    hkey[h] = L;
                    hin[h] = 0;
                    hrow[h] = -1;
                    return h;
                }
                if (hkey[h] == L) return h;
                h = (h + 1) & (H - 1);
            }
        };
        auto next_block = [&] {
            ++blk;
            used = 0;
        };
#pragma omp for schedule(dynamic, 1)
        for (int ch = 0; ch < nch; ++ch) {
            if (ch % sample) continue;
            const int ra = (int)((int64_t)n * ch / nch), rb = (int)((int64_t)n * (ch + 1) / nch);
            std::vector<Rec>& rc = recs[(size_t)ch];
            int r0 = ra, nl = 0;
            long long acc = 0;
            lines.clear();
            next_block();
            auto emit = [&](int a, int b) {
                if (b <= a) return;
                std::sort(lines.begin(), lines.end());
                for (size_t q = 0; q < lines.size(); ++q) hpos[find(lines[q])] = (int)q;
                const bool tiled = (int)lines.size() <= tl_cap;
                if (want_lcol)
                    for (int k = rp[a]; k < rp[b]; ++k) {
                        const int c = col[k];
                        // element within its line
                        const int e = c < ncl ? (c & (lw - 1)) : (int)((c - ncl) & (lw - 1));
                        out.lcol[k] = tiled ? (uint16_t)(hpos[find(line_of(c))] * lw + e) : (uint16_t)0;
                    }
                rc.push_back({a, b, tiled ? lines : std::vector<int>(), cls[a] != 0,
                              tplf != nullptr && (*tplf)[a] != 0});
                if (!tiled) rc.back().lines.assign(tl_cap + 1, 0);  // marker: untiled
                lines.clear();
                next_block();
            };
            // distinct lines of row r not yet in the open block (marker keeps them distinct
            // per call)
            auto collect = [&](int r, int64_t marker) {
                cand.clear();
                cslot.clear();
                for (int k = rp[r]; k < rp[r + 1]; ++k) {
                    const int64_t L = line_of(col[k]);
                    const size_t h = find(L);
                    if (!hin[h] && hrow[h] != marker) {
                        hrow[h] = marker;
                        cand.push_back((int)L);
                        cslot.push_back(h);
                    }
                }
            };
            for (int r = ra; r < rb; ++r) {
                const long long len = rp[r + 1] - rp[r];
                collect(r, 2 * (int64_t)r);
                if (r > r0 && (cls[r] != cls[r0] || acc + len > kCAP || r - r0 >= row_cap ||
                               (line_cap && nl + (int)cand.size() > tl_cap) ||
                               (tplf && (*tplf)[r] != (*tplf)[r0]))) {
                    emit(r0, r);  // closes [r0, r); a new generation
                    r0 = r;
                    acc = 0;
                    nl = 0;
                    collect(r, 2 * (int64_t)r + 1);  // all of row r's lines are new to the new block
                }
                for (size_t q = 0; q < cand.size(); ++q) {
                    hin[cslot[q]] = 1;
                    lines.push_back(cand[q]);
                }
                nl += (int)cand.size();
                acc += len;
            }
            emit(r0, rb);
        }
    }
    for (int pass = 0; pass < 3; ++pass)
        for (const std::vector<Rec>& rc : recs)
            for (const Rec& R : rc) {
                const int p = R.bnd ? 2 : R.tpl ? 0 : 1;
                if (p != pass) continue;
                out.blocks.push_back(make_int2(R.r0, R.r1));
                out.tile_ptr.push_back((int)out.tile_lines.size());
                out.tile_lines.insert(out.tile_lines.end(), R.lines.begin(), R.lines.end());
                (pass == 2 ? out.nb_bnd : out.nb_int)++;
                if (pass == 0) out.nb_skip++;
            }
    out.tile_ptr.push_back((int)out.tile_lines.size());
    return out;
}

// Value-indexed CSR (Kourtis et al., CF'08): blocks whose nonzeros take <= 256 distinct
// values (exact bit patterns) get a table of those values and a 1-byte index per nonzero,
// lane-major like the tile indices (entry j of the block -> lane j % kTPB, slot j / kTPB).
// Returns per-block table offset (-1: value stream) and table size for the block headers.
// For square operators also the table index of each row's diagonal (dvi, 1 byte per row) and
// per block whether every row has one (then Jacobi forms 1 / a_ii from the table in-kernel
// instead of streaming dinv: 1 byte per row instead of 8).
// Lane-major position of entry j of a block whose lanes hold nu entries each, as pairs:
// entry j = 512 p + 2 t + h sits at lane t, slot 2 p + h (p < nu / 2).
static inline size_t lane_pos(int j, int nu) {
    return (size_t)((j & (2 * kTPB - 1)) >> 1) * (size_t)nu + 2 * (size_t)(j / (2 * kTPB)) + (size_t)(j & 1);
}

// Index layout.  Square operators (x-tile kernel, 8 slots, entry pairs: lane_pos): kCAP
// bytes per block at bid * kCAP.  Rectangular ones (gather kernel, entry j at lane j % kTPB,
// slot j / kTPB): NU = 2, 4 or 8 slots by block size (the kernel's choice), packed, block
// offset in vofs (header field 0, unused by the gather kernel otherwise).
static int gather_slots(int nz) { return nz > 4 * kTPB ? 8 : nz > 2 * kTPB ? 4 : 2; }

static void build_value_index(DevMatrix& M, const HostCSR& H, const std::vector<int>& hrp, const BlockBuild& bb,
                              std::vector<int>& vt_off, std::vector<int>& vt_len,
                              std::vector<uint8_t>& dvi, std::vector<char>& dvi_ok,
                              std::vector<int64_t>& vofs) {
    const size_t nbk = bb.blocks.size();
    PhaseTimer tm(M.ctx->host);
    std::vector<std::vector<uint64_t>> tabs(nbk);
#pragma omp parallel for schedule(dynamic, 64)
    for (size_t q = 0; q < nbk; ++q) {
        const int kb = hrp[bb.blocks[q].x], nz = hrp[bb.blocks[q].y] - kb;
        if (nz > kCAP || nz == 0) continue;
        std::vector<uint64_t> t(nz);
        std::memcpy(t.data(), H.val.data() + kb, sizeof(double) * (size_t)nz);
        std::sort(t.begin(), t.end());
        t.erase(std::unique(t.begin(), t.end()), t.end());
        if (t.size() <= 256) tabs[q] = std::move(t);
    }
    tm.lap("      vi: per-block sort / unique");
    std::vector<int> ptr(std::max<size_t>(nbk, 1), -1);
    int64_t total = 0, vin = 0;
    int nvi = 0;
    for (size_t q = 0; q < nbk; ++q)
        if (!tabs[q].empty()) {
            ptr[q] = (int)total;
            total += (int64_t)tabs[q].size();
            vin += hrp[bb.blocks[q].y] - hrp[bb.blocks[q].x];
            ++nvi;
        }
    M.n_vi_blocks = nvi;
    M.vi_nnz = vin;
    vt_off.assign(nbk, -1);
    vt_len.assign(nbk, 0);
    dvi.assign(M.square ? (size_t)M.n_rows + 1 : 0, 0);
    dvi_ok.assign(nbk, 0);
    for (size_t q = 0; q < nbk; ++q)
        if (!tabs[q].empty()) vt_off[q] = ptr[q], vt_len[q] = (int)tabs[q].size();
    if (nvi == 0) {
        M.vtab.reset();
        M.vidx.reset();
        return;
    }
    AMG_CHECK(total < INT_MAX, "value tables too large");
    std::vector<double> tab((size_t)total);
    vofs.assign(nbk + 1, 0);
    for (size_t q = 0; q < nbk; ++q) {
        const int nz = hrp[bb.blocks[q].y] - hrp[bb.blocks[q].x];
        vofs[q + 1] = vofs[q] + (M.tiled ? kCAP : tabs[q].empty() ? 0 : gather_slots(nz) * kTPB);
    }
    AMG_CHECK(vofs[nbk] < INT_MAX, "value index stream too large");
    ParZeros<uint8_t> idx((size_t)vofs[nbk] + 16);
    tm.lap("      vi: offsets");
#pragma omp parallel for schedule(dynamic, 64)
    for (size_t q = 0; q < nbk; ++q) {
        if (tabs[q].empty()) continue;
        const std::vector<uint64_t>& t = tabs[q];
        std::memcpy(tab.data() + ptr[q], t.data(), sizeof(double) * t.size());
        const int kb = hrp[bb.blocks[q].x], nz = hrp[bb.blocks[q].y] - kb;
        for (int j = 0; j < nz; ++j) {
            uint64_t bits;
            std::memcpy(&bits, H.val.data() + kb + j, sizeof(bits));
            const size_t at = std::lower_bound(t.begin(), t.end(), bits) - t.begin();
            // square (x-tile kernel): entry pairs; rectangular (gather kernel): entry j at
            // lane j % kTPB, slot j / kTPB, NU slots per lane
            const size_t pos = M.tiled ? lane_pos(j, kCAP / kTPB)
                                        : (size_t)(j % kTPB) * gather_slots(nz) + (size_t)(j / kTPB);
            idx[(size_t)vofs[q] + pos] = (uint8_t)at;
        }
        if (!M.square) continue;
        bool ok = true;
        for (int r = bb.blocks[q].x; r < bb.blocks[q].y; ++r) {
            int64_t k = H.rp[r], e = H.rp[r + 1];
            const int64_t g = M.first_row + r;
            while (k < e && H.col[k] < g) ++k;
            if (k == e || H.col[k] != g || H.val[k] == 0.0) {
                ok = false;
                continue;
            }
            uint64_t bits;
            std::memcpy(&bits, H.val.data() + k, sizeof(bits));
            dvi[r] = (uint8_t)(std::lower_bound(t.begin(), t.end(), bits) - t.begin());
        }
        dvi_ok[q] = ok;
    }
    tm.lap("      vi: indices + diagonal table slots");
    M.vtab.upload(tab.data(), tab.size());
    M.vidx.upload(idx.data(), idx.size());
    tm.lap("      vi: upload");
}


// Row templates.  A row qualifies when all its columns are local and it has
// 1..kTplMaxLen entries; its key is (column - row offsets, value bits, 1/a_ii bits).  Rows
// with equal keys share a template.  Each thread scans a contiguous chunk into a local
// dictionary; the chunk dictionaries merge in chunk order into <= kTplMax templates of
// <= kTplEntries entries (later shapes beyond either cap stay untemplated).
struct TplBuild {
    std::vector<uint8_t> id;  // per row, kTplNone = not templated
    std::vector<int> hdr, off;
    std::vector<double> val, pd;
    int64_t rows = 0;
};

static TplBuild build_templates(const std::vector<int>& rp, const hvec<int>& col,
                                const hvec<double>& val, const std::vector<double>& dinv,
                                int64_t ncl) {
    const int n = (int)rp.size() - 1;
    TplBuild T;
    T.id.assign((size_t)n, (uint8_t)kTplNone);
    if (n <= 0) return T;
    auto bits = [](double v) {
        uint64_t u;
        std::memcpy(&u, &v, sizeof(u));
        return u;
    };
    auto qualifies = [&](int r) {
        const int len = rp[r + 1] - rp[r];
        if (len <= 0 || len > kTplMaxLen) return false;
        for (int k = rp[r]; k < rp[r + 1]; ++k)
            if (col[k] >= ncl) return false;
        return true;
    };
    auto key_hash = [&](int r) {
        uint64_t h = 0x9E3779B97F4A7C15ull * (uint64_t)(rp[r + 1] - rp[r] + 1);
        auto mix = [&](uint64_t v) {
            h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
            h *= 0xBF58476D1CE4E5B9ull;
        };
        for (int k = rp[r]; k < rp[r + 1]; ++k) {
            mix((uint64_t)(uint32_t)(col[k] - r));
            mix(bits(val[k]));
        }
        mix(bits(dinv[r]));
        return h;
    };
    auto same = [&](int a, int b) {
        const int la = rp[a + 1] - rp[a];
        if (la != rp[b + 1] - rp[b] || bits(dinv[a]) != bits(dinv[b])) return false;
        for (int k = 0; k < la; ++k)
            if (col[rp[a] + k] - a != col[rp[b] + k] - b || bits(val[rp[a] + k]) != bits(val[rp[b] + k]))
                return false;
        return true;
    };
    // quick rejection (Galerkin coarse operators: nearly every row is its own shape): when
    // 4096 rows spread over the operator already show more than 2 kTplMax distinct keys,
    // the templates could not cover half the rows -- skip the full scan
    if (n > 65536) {
        std::vector<uint64_t> sk;
        for (int t = 0; t < 4096; ++t) {
            const int r = (int)((int64_t)n * t / 4096);
            if (qualifies(r)) sk.push_back(key_hash(r));
        }
        std::sort(sk.begin(), sk.end());
        sk.erase(std::unique(sk.begin(), sk.end()), sk.end());
        if ((int)sk.size() > 2 * kTplMax) return T;
    }
    const int nch = std::max(1, std::min(256, n / 16384));
    std::vector<std::vector<int>> reps(nch);       // representative row per local template
    std::vector<std::vector<uint64_t>> hashes(nch);
    std::vector<int16_t> lid((size_t)n, -1);
#pragma omp parallel for schedule(dynamic, 1)
    for (int c = 0; c < nch; ++c) {
        const int r0 = (int)((int64_t)n * c / nch), r1 = (int)((int64_t)n * (c + 1) / nch);
        std::unordered_map<uint64_t, std::vector<int>> m;
        std::vector<int>& R = reps[c];
        int last = -1;
        for (int r = r0; r < r1; ++r) {
            if (!qualifies(r)) continue;
            if (last >= 0 && same(R[last], r)) {
                lid[r] = (int16_t)last;
                continue;
            }
            const uint64_t h = key_hash(r);
            int found = -1;
            auto it = m.find(h);
            if (it != m.end())
                for (int t : it->second)
                    if (same(R[t], r)) {
                        found = t;
                        break;
                    }
            if (found < 0) {
                if ((int)R.size() >= kTplMax) continue;
                found = (int)R.size();
                R.push_back(r);
                hashes[c].push_back(h);
                m[h].push_back(found);
            }
            lid[r] = (int16_t)found;
            last = found;
        }
    }
    // merge (chunk order) into the global dictionary
    std::vector<std::vector<int>> gmap(nch);
    std::vector<int> grep;
    std::unordered_map<uint64_t, std::vector<int>> gm;
    int ent = 0;
    for (int c = 0; c < nch; ++c) {
        gmap[c].assign(reps[c].size(), -1);
        for (size_t t = 0; t < reps[c].size(); ++t) {
            const int r = reps[c][t];
            const uint64_t h = hashes[c][t];
            int g = -1;
            auto it = gm.find(h);
            if (it != gm.end())
                for (int q : it->second)
                    if (same(grep[q], r)) {
                        g = q;
                        break;
                    }
            const int len4 = (rp[r + 1] - rp[r] + 3) & ~3;  // padded run (below)
            if (g < 0 && (int)grep.size() < kTplMax && ent + len4 <= kTplEntries) {
                g = (int)grep.size();
                grep.push_back(r);
                gm[h].push_back(g);
                ent += len4;
            }
            gmap[c][t] = g;
        }
    }
    int64_t rows = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : rows)
    for (int c = 0; c < nch; ++c) {
        const int r0 = (int)((int64_t)n * c / nch), r1 = (int)((int64_t)n * (c + 1) / nch);
        for (int r = r0; r < r1; ++r)
            if (lid[r] >= 0 && gmap[c][lid[r]] >= 0) {
                T.id[r] = (uint8_t)gmap[c][lid[r]];
                ++rows;
            }
    }
    T.rows = rows;
    for (int r : grep) {
        const int start = (int)T.off.size(), len = rp[r + 1] - rp[r];
        int dk = 255;
        for (int k = 0; k < len; ++k) {
            T.off.push_back(col[rp[r] + k] - r);
            T.val.push_back(val[rp[r] + k]);
            if (col[rp[r] + k] == r && dk == 255) dk = k;
        }
        // runs start at multiples of 4 entries: the window kernels read 4 slots (16 bytes) and
        // 2 x 2 values per LDS instruction; padding repeats the run's first slot with value 0
        // and is never summed (entries >= len are masked)
        for (int k = len; k & 3; ++k) {
            T.off.push_back(col[rp[r]] - r);
            T.val.push_back(0.0);
        }
        T.hdr.push_back(start | len << 16 | (int)((unsigned)dk << 24));
        T.pd.push_back(dinv[r]);
    }
    return T;
}

// Uniform stencil: a constant-coefficient stencil's boundary templates are
// its interior template with entries removed.  When the longest template (the master) has a
// kernel instantiation (7 or 27 entries) and every template's (offset, value bits) entries are
// a subsequence of the master's -- in order, since offsets ascend -- and holds the master's
// diagonal with the same 1/a_ii, a row is (master, entry mask): the kernels take values and
// window slots from kernel arguments and skip the entries a row lacks.  The products and their
// order are the row's own, so results are unchanged (bit-identical).
static void find_master_template(DevMatrix& D, const TplBuild& tb, const std::vector<int>& ldo) {
    D.tpl_mne = 0;
    D.tpl_mdiag = D.tpl_mem = D.tpl_mep = -1;
    D.tpl_mslot.clear();
    D.tpl_mval.clear();
    D.tpl_mmask.reset();
    const char* env = std::getenv("AMG_TPL_MASTER");
    if (env && std::atoi(env) == 0) return;
    const int nt = (int)tb.hdr.size();
    if (nt == 0) return;
    auto start = [&](int t) { return tb.hdr[t] & 0xffff; };
    auto len = [&](int t) { return (tb.hdr[t] >> 16) & 0xff; };
    auto diag = [&](int t) { return (int)((unsigned)tb.hdr[t] >> 24); };
    auto bits = [](double v) {
        uint64_t u;
        std::memcpy(&u, &v, sizeof(u));
        return u;
    };
    int M = 0;
    for (int t = 1; t < nt; ++t)
        if (len(t) > len(M)) M = t;
    const int ne = len(M);
    if ((ne != 7 && ne != 27) || diag(M) == 255) return;
    const int sm = start(M);
    std::vector<unsigned> mask(nt, 0u);
    for (int t = 0; t < nt; ++t) {
        if (diag(t) == 255 || bits(tb.pd[t]) != bits(tb.pd[M])) return;
        int e = 0;
        for (int k = 0; k < len(t); ++k) {
            const int o = tb.off[start(t) + k];
            while (e < ne && tb.off[sm + e] != o) ++e;
            if (e == ne || bits(tb.val[start(t) + k]) != bits(tb.val[sm + e])) return;
            mask[t] |= 1u << e;
            ++e;
        }
        if (!(mask[t] >> diag(M) & 1u)) return;
    }
    D.tpl_mne = ne;
    D.tpl_mdiag = diag(M);
    D.tpl_mpd = tb.pd[M];
    for (int e = 0; e < ne; ++e) {
        D.tpl_mslot.push_back(ldo[sm + e]);
        D.tpl_mval.push_back(tb.val[sm + e]);
        if (tb.off[sm + e] == -1) D.tpl_mem = e;
        if (tb.off[sm + e] == 1) D.tpl_mep = e;
    }
    D.tpl_mmask.upload(mask.data(), mask.size());
}

void DevMatrix::build(Context* c, HostCSR&& h, bool replicated_view) {
    build_view(c, h, replicated_view);
    host = std::move(h);
}

void DevMatrix::defer(Context* c, HostCSR&& h) {
    ctx = c;
    replicated = false;
    host = std::move(h);
    const HostComm& comm = ctx->host;
    first_row = host.row_starts[comm.rank];
    n_rows = host.nrows();
    first_col = host.col_starts[comm.rank];
    n_cols_local = host.col_starts[comm.rank + 1] - first_col;
    nnz = host.nnz();
    square = host.n_global_rows == host.n_global_cols && host.row_starts == host.col_starts;
    deferred = true;
}

void DevMatrix::ensure_built() {
    if (!deferred) return;
    build_view(ctx, host);
    deferred = false;
}

// Every device format from a CSR the caller keeps (the member `host` is shadowed by the
// argument): Solver::setup runs this on a worker thread while the hierarchy thread still
// reads the same CSR, and moves it into `host` after both are done.
void DevMatrix::build_view(Context* c, const HostCSR& host, bool replicated_view) {
    ctx = c;
    replicated = replicated_view;
    static const HostComm serial;  // rank 0 of 1: replicated matrices have no halo
    const HostComm& comm = replicated ? serial : ctx->host;
    PhaseTimer tm(comm);
    AMG_CHECK((int)host.row_starts.size() == comm.nranks + 1, "matrix row partition size");
    AMG_CHECK((int)host.col_starts.size() == comm.nranks + 1, "matrix column partition size");
    first_row = host.row_starts[comm.rank];
    n_rows = host.nrows();
    AMG_CHECK(n_rows == host.row_starts[comm.rank + 1] - first_row, "local row count mismatch");
    first_col = host.col_starts[comm.rank];
    n_cols_local = host.col_starts[comm.rank + 1] - first_col;
    nnz = host.nnz();
    AMG_CHECK(nnz < INT_MAX && n_rows < INT_MAX, "local matrix exceeds int32 indexing");
    square = host.n_global_rows == host.n_global_cols && host.row_starts == host.col_starts;
    plan = halo_plan_for_cols(comm, host);
    if (send_map && !replicated)
        for (int64_t& v : plan.send_idx) v = (*send_map)[v];
    AMG_CHECK(n_cols_local + plan.n_halo() < INT_MAX, "too many columns for int32");
    tm.lap("    build: halo plan");

    std::vector<int> hrp(n_rows + 1);
    // every entry written below; capacity for the kPad zero entries appended after the
    // templates, so that resize does not reallocate and copy (0.4 s for a 449 M-entry operator)
    hvec<int> hcol;
    hcol.reserve((size_t)nnz + kPad);
    hcol.resize(nnz);
    std::vector<uint8_t> cls(n_rows, 0);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i <= n_rows; ++i) hrp[i] = (int)host.rp[i];
    const int64_t clo = first_col, chi = first_col + n_cols_local;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n_rows; ++i) {
        uint8_t b = 0;
        for (int64_t k = host.rp[i]; k < host.rp[i + 1]; ++k) {
            const int64_t g = host.col[k];
            if (g >= clo && g < chi) {
                hcol[k] = (int)(g - clo);
            } else {
                hcol[k] = (int)(n_cols_local + plan.find(g));
                b = 1;
            }
        }
        cls[i] = b;
    }
    rp.upload(hrp.data(), hrp.size());
    std::vector<double> di;
    if (square) {
        std::vector<double> d = diagonal(comm, host);
        di.resize(n_rows);
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < n_rows; ++i) di[i] = 1.0 / d[i];
        dinv.upload(di.data(), di.size());
    }
    // row templates: square operators whose templates cover every row, or at least half of
    // the rows of a large operator (AMG_TPL_MIN_ROWS, default 16384; tests lower it)
    TplBuild tb;
    n_tpl = n_tpl_ent = nb_skip = 0;
    tpl_rows = 0;
    if (square && n_rows > 0 && !blocks_only) {
        const char* e = std::getenv("AMG_TPL_MIN_ROWS");
        const int64_t min_rows = e ? std::atoll(e) : (int64_t)16384;
        tb = build_templates(hrp, hcol, host.val, di, n_cols_local);
        const bool use = tb.rows == n_rows || (n_rows >= min_rows && 2 * tb.rows >= n_rows);
        if (!use) tb = TplBuild();
    }
    tm.lap("    build: local columns, dinv, templates");
    hcol.resize(nnz + kPad, 0);
    {
        std::vector<uint8_t> tplf;
        if (!tb.hdr.empty()) {
            tplf.resize(n_rows);
            for (int64_t i = 0; i < n_rows; ++i) tplf[i] = tb.id[i] != kTplNone && cls[i] == 0;
        }
        // square operators: x tiles, one row per lane; short-row rectangular ones (gather
        // path): up to kGatherRPB rows per lane (profiles/r2n: P0 x += P e 162 -> 95 us; R
        // with 7+ entries per row was slower that way: R0 94 -> 106 us, sa27 R0 350 -> 415)
        gather_rpb = !square && nnz <= 4 * n_rows ? kGatherRPB : 1;
        const bool dev_fmt = device_formats();
        // The format choices below (x tile or gather, 64- or 32-byte lines) read statistics of
        // the 64-byte cut; r5 takes them from every 8th of its 64 row chunks (the whole
        // operator below 65,536 rows) and cuts the operator once, at the chosen width.  Before,
        // each choice cut the whole operator again: 0.6 s of sa27's setup.
        constexpr int kSample = 8;
        const BlockBuild s8 = build_row_blocks(hrp, hcol, cls, n_cols_local, plan.n_halo(),
                                               tplf.empty() ? nullptr : &tplf, kTPB * gather_rpb, true, false, 8,
                                               kSample);
        // rectangular operators take the x-tile kernel when their blocks reuse x lines: at most
        // 0.5 tile lines per nonzero.  Same-box A/B (profiles/r2y_rtile_*, r2z_rpb_*): 7-pt R0
        // 106 -> 79 us (0.23 lines / nnz), R1 66 -> 53 (0.34), P0 (4 rows per lane, 0.06)
        // 97 -> 80, P1 49 -> 39; sa27 P0 299 -> 234 (0.04), P1 33 -> 26; g3sub R0 24 -> 20
        // (0.33), P0 19 -> 15; sa27 R1 122 -> 158 at 0.70 (a 297-entry block loading 210
        // lines) stays on the gather kernel.
        // AMG_RECT_TILE=0 / 1: never / always (A/B runs)
        int64_t tile_lines_total = 0, tile_full = 0, sample_nnz = 0;
        for (size_t q = 0; q + 1 < s8.tile_ptr.size(); ++q) {
            const int nt = s8.tile_ptr[q + 1] - s8.tile_ptr[q];
            tile_lines_total += nt;
            tile_full += nt >= kTileLines;
            sample_nnz += hrp[s8.blocks[q].y] - hrp[s8.blocks[q].x];
        }
        {
            const char* e = std::getenv("AMG_RECT_TILE");
            const int mode = e ? std::atoi(e) : -1;
            tiled = square || (mode != 0 && (mode == 1 || 2 * tile_lines_total <= sample_nnz));
        }
        if (std::getenv("AMG_TRACE_BLOCKS")) {
            const int64_t lines = tile_lines_total, full = tile_full;
            std::fprintf(stderr, "[amg-blocks] %s rows %lld cols %lld nnz %lld sampled: blocks %zu lines %lld full %lld nnz %lld rpb %d\n",
                         square ? "square" : tiled ? "rect-tiled" : "rect-gather", (long long)n_rows, (long long)n_cols_local, (long long)nnz,
                         s8.blocks.size(), (long long)lines, (long long)full, (long long)sample_nnz, gather_rpb);
        }
        // x-tile line width: operators whose blocks, cut at 256 lines of
        // 64 B, run close to the cap (>= 3/4 full on average: Galerkin operators,
        // restrictions) are cut at 512 lines of 32 B (the 7-pt 256^3 A2: 40,250 -> 25,615
        // blocks; R0: same-box 76 -> 70 us); P-like operators (few lines per block) keep
        // 64-byte lines and their 1 KiB of line ids per block (sa27 P0: 234 us at 64 B, 263 at
        // 32 B), and so do square operators the 32-byte cut saves < 20 % of the blocks (the
        // 7-pt A1: 50,573 -> 46,841 blocks ran 144 -> 149 us; A2: 40,281 -> 25,640 ran 125 ->
        // 102 us); restrictions gain either way (R0 91 -> 88 us at -9 %, R1 61 -> 52 at -33 %).
        // AMG_TILE_LINE=8 / 4 forces the width.
        // The gather kernel reads x from global memory: its blocks need only the kCAP-entry and
        // row caps, not the 256-line tile cap.  sa27's R1 (270 entries per row over ~200 lines
        // each) was cut into blocks of ~1 row by that cap: one lane summing while 255 idled.
        int lw = 8;
        const bool line_cap = tiled;
        if (tiled && !s8.blocks.empty()) {
            const char* e = std::getenv("AMG_TILE_LINE");
            const int force = e ? std::atoi(e) : 0;
            const bool tryhalf = force == 4 || (force != 8 && 4 * tile_lines_total >= 3 * (int64_t)kTileLines *
                                                                                         (int64_t)s8.blocks.size());
            if (tryhalf) {
                bool take = force == 4 || !square;
                if (!take) {
                    const BlockBuild s4 = build_row_blocks(hrp, hcol, cls, n_cols_local, plan.n_halo(),
                                                           tplf.empty() ? nullptr : &tplf, kTPB * gather_rpb, true,
                                                           false, 4, kSample);
                    take = 5 * s4.blocks.size() <= 4 * s8.blocks.size();
                }
                if (take) lw = 4;
            }
        }
        tm.lap("    build: row blocks, sampled cuts");
        BlockBuild bb = build_row_blocks(hrp, hcol, cls, n_cols_local, plan.n_halo(),
                                         tplf.empty() ? nullptr : &tplf, kTPB * gather_rpb, line_cap, !dev_fmt, lw);
        line_w = lw;
        nb_int = bb.nb_int;
        nb_bnd = bb.nb_bnd;
        if (std::getenv("AMG_TRACE_BLOCKS"))
            std::fprintf(stderr, "[amg-blocks]   %s, lines of %d B: %zu blocks\n", tiled ? "x tile" : "gather",
                         8 * line_w, bb.blocks.size());
        tm.lap("    build: row blocks + x tiles");
        if (!tb.hdr.empty()) {
            // rows of blocks the CSR kernel still runs are not the template kernel's
            std::vector<char> keep(n_rows, 0);
            for (int q = 0; q < bb.nb_skip; ++q)
                for (int r = bb.blocks[q].x; r < bb.blocks[q].y; ++r) keep[r] = 1;
            int64_t rows = 0;
            for (int64_t i = 0; i < n_rows; ++i) {
                if (!keep[i]) tb.id[i] = (uint8_t)kTplNone;
                rows += tb.id[i] != kTplNone;
            }
            nb_skip = bb.nb_skip;
            tpl_rows = rows;
            n_tpl = (int)tb.hdr.size();
            n_tpl_ent = (int)tb.off.size();
            tpl_id.upload(tb.id.data(), tb.id.size());
            tpl_id_host = tb.id;
            tpl_hdr.upload(tb.hdr.data(), tb.hdr.size());
            tpl_off.upload(tb.off.data(), tb.off.size());
            tpl_val.upload(tb.val.data(), tb.val.size());
            tpl_pd.upload(tb.pd.data(), tb.pd.size());
            // x window: distinct offsets merged into bands while a gap is shorter than a
            // workgroup's rows (a new band would load kTplRows more doubles than the gap)
            std::vector<int> offs(tb.off);
            std::sort(offs.begin(), offs.end());
            offs.erase(std::unique(offs.begin(), offs.end()), offs.end());
            std::vector<int2> bands;  // {lo, hi}
            for (int o : offs) {
                if (!bands.empty() && (int64_t)o - bands.back().y < kTplRows) bands.back().y = o;
                else bands.push_back(make_int2(o, o));
            }
            // even band starts and lengths: slot pairs map to 16-byte aligned pairs of x
            for (int2& bd : bands) bd.x &= ~1;
            auto blen = [](const int2& bd) { return (int64_t)(kTplRows + bd.y - bd.x + 1) & ~(int64_t)1; };
            int64_t w = 0;
            for (const int2& bd : bands) w += blen(bd);
            tpl_blo.clear();
            tpl_bbase.clear();
            tpl_win = tpl_wend = 0;
            tpl_ldo.reset();
            if ((int)bands.size() <= kTplBands && w <= kTplWin) {
                std::vector<int> ldo(tb.off.size());
                int base = 0;
                for (const int2& bd : bands) {
                    tpl_blo.push_back(bd.x);
                    tpl_bbase.push_back(base);
                    base += (int)blen(bd);
                }
                tpl_wend = bands.back().x + (int)blen(bands.back());
                for (size_t k = 0; k < tb.off.size(); ++k) {
                    const int o = tb.off[k];
                    size_t q = 0;
                    while (q + 1 < bands.size() && o > bands[q].y) ++q;
                    ldo[k] = tpl_bbase[q] + (o - bands[q].x);
                }
                tpl_win = base;
                tpl_ldo.upload(ldo.data(), ldo.size());
                find_master_template(*this, tb, ldo);
                // z-marching: the shift D (a multiple of kTplRows, taken from the band
                // starts) under which the most window slots of a block are slots of the block
                // D rows back; used when at least a quarter of the window is reused
                const int nbd = (int)bands.size();
                auto reuse_map = [&](int64_t D, std::vector<int>* map) {
                    int cnt = 0;
                    for (int q = 0; q < nbd; ++q) {
                        const int len = (q + 1 < nbd ? tpl_bbase[q + 1] : base) - tpl_bbase[q];
                        for (int i = 0; i < len; ++i) {
                            const int64_t g = D + tpl_blo[q] + i;  // relative to the old r0
                            int src = -1;
                            for (int q2 = 0; q2 < nbd && src < 0; ++q2) {
                                const int len2 = (q2 + 1 < nbd ? tpl_bbase[q2 + 1] : base) - tpl_bbase[q2];
                                const int64_t j = g - tpl_blo[q2];
                                if (j >= 0 && j < len2) src = tpl_bbase[q2] + (int)j;
                            }
                            if (map) (*map)[tpl_bbase[q] + i] = src;
                            cnt += src >= 0;
                        }
                    }
                    return cnt;
                };
                int64_t bestD = 0;
                int best = 0;
                std::vector<int64_t> cand;
                for (int q = 0; q < nbd; ++q) {
                    cand.push_back(std::abs((int64_t)tpl_blo[q]));
                    for (int q2 = q + 1; q2 < nbd; ++q2) cand.push_back((int64_t)tpl_blo[q2] - tpl_blo[q]);
                }
                for (int64_t D : cand) {
                    D -= D % kTplRows;
                    if (D <= 0 || D / kTplRows > INT_MAX / 2) continue;
                    const int c = reuse_map(D, nullptr);
                    if (c > best) best = c, bestD = D;
                }
                tpl_march_s = 0;
                tpl_wsrc.reset();
                // 16-byte pair loads: an even row count keeps every pair inside or outside x
                if (bestD > 0 && 4 * best >= base && n_rows % 2 == 0) {
                    std::vector<int> map(base, -1);
                    reuse_map(bestD, &map);
                    tpl_march_s = (int)(bestD / kTplRows);
                    tpl_wsrc.upload(map.data(), map.size());
                }
            }
        } else {
            tpl_blo.clear();
            tpl_bbase.clear();
            tpl_win = tpl_wend = 0;
            tpl_ldo.reset();
            tpl_id.reset();
            tpl_id_host.clear();
            tpl_hdr.reset();
            tpl_off.reset();
            tpl_val.reset();
            tpl_pd.reset();
        }
        if (tpl_win == 0) {
            tpl_mne = 0;
            tpl_mmask.reset();
        }
        tm.lap("    build: template window / march");
        blocks.upload(bb.blocks.data(), bb.blocks.size());
        const size_t nbk = bb.blocks.size();
        // device col / val: block-aligned copies -- block q's entries at an even offset
        // koff[q] (16-byte aligned values), so the kernel reads them as (2t, 2t + 1) pairs
        std::vector<int64_t> koff(nbk + 1, 0);
        for (size_t q = 0; q < nbk; ++q)
            koff[q + 1] = koff[q] + (int64_t)(hrp[bb.blocks[q].y] - hrp[bb.blocks[q].x] + 1) / 2 * 2;
        AMG_CHECK(koff[nbk] + kPad < INT_MAX, "local matrix exceeds int32 indexing");
        std::vector<int> vt_off, vt_len;
        std::vector<char> dvi_ok;
        std::vector<int64_t> vofs;
        if (dev_fmt) {
            // per-nonzero streams built on the GPU from one upload of the CSR (formats.hip)
            FormatHeaderInfo fi;
            build_formats_device(*this, hrp, hcol, host.val, bb.blocks, bb.tile_ptr, bb.tile_lines, koff, fi);
            vt_off = std::move(fi.vt_off);
            vt_len = std::move(fi.vt_len);
            dvi_ok = std::move(fi.dvi_ok);
            vofs = std::move(fi.vofs);
            tm.lap("    build: device col / val / tiles / value index / row ends");
        } else {
            {
                ParZeros<int> cb((size_t)(koff[nbk] + kPad));
                ParZeros<double> vb(cb.size());
#pragma omp parallel for schedule(dynamic, 256)
                for (size_t q = 0; q < nbk; ++q) {
                    const int kb = hrp[bb.blocks[q].x], nz = hrp[bb.blocks[q].y] - kb;
                    std::copy(hcol.begin() + kb, hcol.begin() + kb + nz, cb.begin() + koff[q]);
                    std::copy(host.val.begin() + kb, host.val.begin() + kb + nz, vb.begin() + koff[q]);
                }
                col.upload(cb.data(), cb.size());
                val.upload(vb.data(), vb.size());
            }
            if (tiled) {  // x tiles: the x-tile kernel only
                // x-tile line ids at a fixed stride (kCAP / line_w per block, padded with the block's
                // last line), so the kernel loads them without waiting for the block header
                const int tlb = kCAP / line_w;
                ParZeros<int> fx(std::max<size_t>(nbk, 1) * tlb);
#pragma omp parallel for schedule(static)
                for (size_t q = 0; q < nbk; ++q) {
                    const int t0 = bb.tile_ptr[q], nt = bb.tile_ptr[q + 1] - t0;
                    if (nt <= 0 || nt > tlb) continue;
                    for (int j = 0; j < tlb; ++j)
                        fx[q * tlb + j] = bb.tile_lines[t0 + std::min(j, nt - 1)];
                }
                tile_fixed.upload(fx.data(), fx.size());
                // lane-major per block (lane_pos): lane t's 8 indices are 16 contiguous bytes,
                // one 16-byte load per lane
                ParZeros<uint16_t> perm(std::max<size_t>(nbk, 1) * kCAP);
#pragma omp parallel for schedule(static)
                for (size_t q = 0; q < nbk; ++q) {
                    const int kb = hrp[bb.blocks[q].x], nz = hrp[bb.blocks[q].y] - kb;
                    if (nz > kCAP) continue;
                    for (int j = 0; j < nz; ++j)
                        perm[q * kCAP + lane_pos(j, kCAP / kTPB)] = bb.lcol[kb + j];
                }
                lcol.upload(perm.data(), perm.size());
            } else {
                tile_fixed.reset();
                lcol.reset();
            }
            tm.lap("    build: col / val / tile layouts");
            std::vector<uint8_t> hdvi;
            build_value_index(*this, host, hrp, bb, vt_off, vt_len, hdvi, dvi_ok, vofs);
            if (n_vi_blocks > 0 && square) dvi.upload(hdvi.data(), hdvi.size());
            else dvi.reset();
            tm.lap("    build: value index");
            {
                // per row: end of its nonzeros relative to its block's first (<= kCAP: 16 bits)
                std::vector<uint16_t> re((size_t)n_rows + 1, 0);
                for (size_t q = 0; q < nbk; ++q) {
                    const int2 b = bb.blocks[q];
                    if (hrp[b.y] - hrp[b.x] > kCAP) continue;
                    for (int r = b.x; r < b.y; ++r) re[r] = (uint16_t)(hrp[r + 1] - hrp[b.x]);
                }
                rend.upload(re.data(), re.size());
            }
        }
        // gather operators: 16-bit column codes when every block's columns fit in <= 4
        // bands of kGatherBand: a structured P / R block reads three
        // planes' worth of columns, each a narrow band.  Lossless: the kernel decodes
        // base[code >> 14] + (code & 0x3fff), the same column.
        col16.reset();
        gband.reset();
        if (!tiled && nbk > 0) {
            ParZeros<uint16_t> c16((size_t)(koff[nbk] + kPad));
            std::vector<int4> gb(nbk, make_int4(0, 0, 0, 0));
            int bad = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : bad)
            for (size_t q = 0; q < nbk; ++q) {
                const int kb = hrp[bb.blocks[q].x], nz = hrp[bb.blocks[q].y] - kb;
                if (nz == 0 || nz > kCAP) continue;  // chunked path: int32 columns
                std::vector<int> u(hcol.begin() + kb, hcol.begin() + kb + nz);
                std::sort(u.begin(), u.end());
                int base[4] = {0, 0, 0, 0}, nbnd = 0;
                for (int c : u) {
                    if (nbnd == 0 || c - base[nbnd - 1] >= kGatherBand) {
                        if (nbnd == 4) {
                            nbnd = 5;
                            break;
                        }
                        base[nbnd++] = c;
                    }
                }
                if (nbnd > 4) {
                    ++bad;
                    continue;
                }
                for (int t = nbnd; t < 4; ++t) base[t] = base[nbnd - 1];
                gb[q] = make_int4(base[0], base[1], base[2], base[3]);
                for (int j = 0; j < nz; ++j) {
                    const int c = hcol[kb + j];
                    int t = nbnd - 1;
                    while (c < base[t]) --t;
                    c16[koff[q] + j] = (uint16_t)((t << 14) | (c - base[t]));
                }
            }
            if (bad == 0) {
                col16.upload(c16.data(), c16.size());
                gband.upload(gb.data(), gb.size());
            }
        }
        // 32-byte block headers (two scalar loads per block):
        //   {r0, r1, koff, nnz}, {diag slot, tile lines | dvi flag << 16, value-table offset (-1),
        //   table size}
        // diag slot (square operators): tile position of line r0 / line_w when the lines of the
        // block's own rows are consecutive in its tile, so x[r] is read from the tile; else -1
        std::vector<int4> hh(std::max<size_t>(2 * nbk, 2), make_int4(0, 0, 0, 0));
        jac_extra_all = jac_extra_csr = 0;
        for (size_t q = 0; q < nbk; ++q) {
            const int2 b = bb.blocks[q];
            const int t0 = bb.tile_ptr[q], nt = bb.tile_ptr[q + 1] - t0;
            int dslot = -1;
            if (square && nt > 0 && nt <= kCAP / line_w) {
                const int ls = line_w == 8 ? 3 : 2;
                const int l0 = b.x >> ls, l1 = (b.y - 1) >> ls;
                const int* tl = bb.tile_lines.data() + t0;
                const int pos = (int)(std::lower_bound(tl, tl + nt, l0) - tl);
                bool ok = pos + (l1 - l0) < nt;
                for (int k = 0; ok && k <= l1 - l0; ++k) ok = tl[pos + k] == l0 + k;
                if (ok) dslot = pos;
            }
            hh[2 * q] = make_int4(b.x, b.y, (int)koff[q], hrp[b.y] - hrp[b.x]);
            if (square) {  // Jacobi operands beyond b: 1/a_ii (table index or fp64), x[r]
                const int64_t rows = b.y - b.x;
                const int64_t e = rows * (dvi_ok[q] ? 1 : 8) + (dslot < 0 ? 8 * rows : 0);
                jac_extra_all += e;
                if ((int)q >= bb.nb_skip) jac_extra_csr += e;
            }
            // rectangular (gather) operators: field 0 = the block's offset in the VI index stream
            const int f0 = square ? dslot : tiled ? -1 : (vofs.empty() ? 0 : (int)vofs[q]);
            hh[2 * q + 1] = make_int4(f0, nt | (dvi_ok[q] ? kHdrDvi : 0), vt_off[q], vt_len[q]);
        }
        hdr.upload(hh.data(), hh.size());
        // measured (profiles/r1m_variants.txt): x tiles in XCD order on square operators (A0
        // -6..8%, A1 -6..8%, A2 +1% vs plain order; gathers are 1.3-1.9x slower); gathers in
        // XCD order on the rectangular P / R (R0 -10% vs plain order)
        default_variant = tiled ? 2 : (4 | 2);
        // format bytes of one default-variant SpMV (the kernel reads every lane slot of the
        // fixed-stride streams, so their padding counts)
        // with templates: the skipped blocks cost nothing; template rows cost 1 byte (id); the
        // table (offsets, values, headers, 1/a_ii) is read from HBM once -- every further
        // workgroup's staging copy of it is an L2 hit, not HBM traffic
        const int64_t xy = 8 * (n_cols_local + plan.n_halo()) + 8 * n_rows;
        int64_t fb = 2 * n_rows + xy, fb_tpl = xy;
        if (n_tpl > 0)
            fb_tpl += n_rows + 12 * (int64_t)n_tpl_ent + 12 * (int64_t)n_tpl;
        for (size_t q = 0; q < nbk; ++q) {
            const int nz = hh[2 * q].w, nt = hh[2 * q + 1].y & 0xffff;
            const int64_t fb0 = fb;
            fb += 32;
            if (nz == 0) continue;
            if (nz > kCAP || (tiled && nt > kCAP / line_w)) {  // long row: CSR stream
                fb += 12 * (int64_t)nz;
                continue;
            }
            if (tiled) fb += 4 * (kCAP / line_w) + 2 * kCAP;  // tile ids, tile indices
            else if (col16.p) fb += 2 * (int64_t)nz + 16;  // column codes, band bases
            else fb += 4 * (int64_t)nz;                     // columns
            if (hh[2 * q + 1].z >= 0)
                fb += (tiled ? kCAP : gather_slots(nz) * kTPB) + 8 * (int64_t)hh[2 * q + 1].w;
            else
                fb += 8 * (int64_t)nz;
            if ((int)q >= nb_skip) fb_tpl += fb - fb0 + 2 * (int64_t)(bb.blocks[q].y - bb.blocks[q].x);
        }
        csr_fmt_bytes = fb;
        spmv_fmt_bytes = n_tpl > 0 ? fb_tpl : fb;
        tm.lap("    build: row ends, headers");
    }
    std::vector<int> sidx(plan.send_idx.begin(), plan.send_idx.end());
    send_idx.upload(sidx.data(), sidx.size());
    send_buf.alloc(sidx.size());
    halo.alloc(plan.n_halo());
    // collective order: the same id on every rank.  Only the loopback transport matches
    // matrices by it, and only one rank's setup builds formats on worker threads (several at
    // once), so the counter is touched where it is used
    if (ctx->transport == TR_LOOPBACK && !replicated) {
        seq = ctx->mat_seq++;
        loopback_register(*ctx, seq, send_buf.p, plan.send_procs, plan.send_ptr);
    }
}

// The one-kernel sweep's sliced ELL (hybrid_gs_kernel): every entry of the ELL slabs, with a
// value dictionary when the local operator takes <= 256 distinct values.  Built with the GS
// blocks unless the operator runs split sweeps (4.2c), whose passes never read it; then on
// first use (a norm-carrying forward sweep: Solver::setup builds it for level 0).  r5: sa27's
// level-1 / level-2 GS builds spent ~1.9 s of an 8.1 s setup mostly here.
// The split sweep's old-value pass for direction d (0 forward, 1 backward): this operator
// without the sweep's in-chunk new-value couplings, as a CSR-block matrix of its own (4.2c).
// Collective on N ranks (its halo plan); never inside a graph capture (Solver::setup builds
// what the cycle needs).
void DevMatrix::ensure_gs_pass(int d) {
    if (gs_old[d]) return;
    const HostCSR& host = host_image();  // the member, or the CSR a worker builds from
    AMG_CHECK(gs_split && gs_block > 0, "hybrid GS: no split sweep for this operator");
    AMG_CHECK(!ctx->capturing, "hybrid GS: split pass requested inside a graph capture");
    const int64_t B = gs_block, clo = first_col, chi = first_col + n_cols_local;
    auto is_new = [&](int64_t i, int64_t gc) {
        if (gc < clo || gc >= chi) return false;
        const int64_t j = gc - clo, g = first_row + i;
        const int64_t cs = std::max<int64_t>(0, (g / B) * B - first_row);
        const int64_t ce = std::min<int64_t>(n_rows, (g / B + 1) * B - first_row);
        return d == 0 ? (j >= cs && j < i) : (j > i && j < ce);
    };
    HostCSR h;
    h.n_global_rows = host.n_global_rows;
    h.n_global_cols = host.n_global_cols;
    h.row_starts = host.row_starts;
    h.col_starts = host.col_starts;
    h.rp.assign((size_t)n_rows + 1, 0);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n_rows; ++i) {
        int64_t c = 0;
        for (int64_t k = host.rp[i]; k < host.rp[i + 1]; ++k) c += !is_new(i, host.col[k]);
        h.rp[i + 1] = c;
    }
    for (int64_t i = 0; i < n_rows; ++i) h.rp[i + 1] += h.rp[i];
    h.col.resize((size_t)h.rp[n_rows]);
    h.val.resize((size_t)h.rp[n_rows]);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n_rows; ++i) {
        int64_t o = h.rp[i];
        for (int64_t k = host.rp[i]; k < host.rp[i + 1]; ++k)
            if (!is_new(i, host.col[k])) {
                h.col[o] = host.col[k];
                h.val[o] = host.val[k];
                ++o;
            }
    }
    // CSR blocks only: no row templates (and so no windows, masks or march tables) are built
    // for the pass's operator, and its format is set before the build -- no
    // format_generation bump, no captured graph goes stale
    gs_old[d] = std::make_unique<DevMatrix>();
    gs_old[d]->blocks_only = true;
    gs_old[d]->format = AMG_FORMAT_BLOCKS;
    gs_old[d]->build(ctx, std::move(h), replicated);
}

void DevMatrix::ensure_gs_ell() {
    if (gs_ell_built) return;
    const HostCSR& host = host_image();  // the member, or the CSR a worker builds from
    AMG_CHECK(!ctx->capturing, "hybrid GS: sliced ELL requested inside a graph capture");
    const int64_t clo = first_col, chi = first_col + n_cols_local;
    auto local_col = [&](int64_t g) -> int {
        return g >= clo && g < chi ? (int)(g - clo) : (int)(n_cols_local + plan.find(g));
    };
    const std::vector<int4>& slabs = gs_slabs_host;
    const int64_t cells = gs_cells;
    std::vector<int> sc((size_t)(cells + 4) * 64, -1);
    std::vector<double> sv(sc.size(), 0.0);
#pragma omp parallel for schedule(dynamic, 64)
    for (size_t q = 0; q < slabs.size(); ++q) {
        const int4 sl = slabs[q];
        for (int l = 0; l < sl.y; ++l) {
            const int64_t i = sl.x + l;
            for (int64_t k = host.rp[i]; k < host.rp[i + 1]; ++k) {
                const size_t at = ((size_t)sl.z + (size_t)(k - host.rp[i])) * 64 + l;
                sc[at] = local_col(host.col[k]);
                sv[at] = host.val[k];
            }
        }
    }
    // value dictionary: <= 256 distinct values (bit patterns) in the local operator; each
    // thread scans a chunk into a small set and gives up past 256
    std::vector<uint64_t> dict;
    {
        const int64_t nz = (int64_t)host.val.size();
        std::atomic<bool> over{false};
#pragma omp parallel
        {
            std::vector<uint64_t> mine;
#pragma omp for schedule(static) nowait
            for (int64_t k = 0; k < nz; ++k) {
                if (over.load(std::memory_order_relaxed)) continue;
                uint64_t bits;
                std::memcpy(&bits, &host.val[k], sizeof(bits));
                if (std::find(mine.begin(), mine.end(), bits) == mine.end()) {
                    mine.push_back(bits);
                    if (mine.size() > 256) over.store(true, std::memory_order_relaxed);
                }
            }
#pragma omp critical
            if (!over.load()) dict.insert(dict.end(), mine.begin(), mine.end());
        }
        std::sort(dict.begin(), dict.end());
        dict.erase(std::unique(dict.begin(), dict.end()), dict.end());
        if (over.load() || dict.size() > 256) dict.clear();
    }
    gs_ndict = (int)dict.size();
    if (gs_ndict > 0) {
        std::vector<uint8_t> vid(sc.size(), 0);
#pragma omp parallel for schedule(dynamic, 64)
        for (size_t q = 0; q < slabs.size(); ++q) {
            const int4 sl = slabs[q];
            for (int l = 0; l < sl.y; ++l)
                for (int k = 0; k < sl.w; ++k) {
                    const size_t at = ((size_t)sl.z + (size_t)k) * 64 + (size_t)l;
                    if (sc[at] < 0) continue;
                    uint64_t bits;
                    std::memcpy(&bits, &sv[at], sizeof(bits));
                    vid[((size_t)sl.z + (size_t)(k & ~3)) * 64 + 4 * (size_t)l + (size_t)(k & 3)] =
                        (uint8_t)(std::lower_bound(dict.begin(), dict.end(), bits) - dict.begin());
                }
        }
        std::vector<double> tab(dict.size());
        std::memcpy(tab.data(), dict.data(), sizeof(double) * dict.size());
        gs_vid.upload(vid.data(), vid.size());
        gs_vtab.upload(tab.data(), tab.size());
        gs_val.reset();
    } else {
        gs_vid.reset();
        gs_vtab.reset();
        gs_val.upload(sv.data(), sv.size());
    }
    gs_col.upload(sc.data(), sc.size());
    gs_ell_built = true;
}

void DevMatrix::ensure_gs_blocks(int64_t B) {
    const HostCSR& host = host_image();  // the member, or the CSR a worker builds from
    AMG_CHECK(square, "hybrid GS needs a square matrix");
    AMG_CHECK(B >= 1 && B <= 64, "hybrid GS block must be in [1, 64]");
    if (gs_block == B) return;
    const int64_t clo = first_col, chi = first_col + n_cols_local;
    // l1 diagonal of every row: d_i = a_ii + sum of |a_ij| outside the row's chunk (global
    // multiples of B clipped to the rank), summed in CSR order like the oracle
    std::vector<double> di(n_rows);
    std::atomic<bool> zero_row{false};
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n_rows; ++i) {
        const int64_t g = first_row + i;
        const int64_t cs = std::max<int64_t>(first_row, g / B * B);
        const int64_t ce = std::min(first_row + n_rows, (g / B + 1) * B);
        double l1 = 0.0, d = 0.0;
        for (int64_t k = host.rp[i]; k < host.rp[i + 1]; ++k) {
            const int64_t gc = host.col[k];
            if (gc < cs || gc >= ce) l1 += std::fabs(host.val[k]);
            if (gc == g) d = host.val[k];
        }
        if (d == 0.0 && l1 == 0.0) zero_row.store(true, std::memory_order_relaxed);
        di[i] = 1.0 / (d + l1);
    }
    AMG_CHECK(!zero_row.load(), "hybrid GS: zero row");
    // GS templates: a 512-row block runs on tpl_gs_kernel when every row has
    // a row template (all columns local) and the (template, l1 diagonal) pairs fit the table.
    // Chunks must not straddle a wave's 64-row group: first_row % 64 == 0 and B | 64.
    std::vector<char> tblk;
    n_gs_tpl = n_gs_tblk = 0;
    gs_tid.reset();
    gs_thdr.reset();
    gs_tdl.reset();
    gs_tblocks.reset();
    gs_tcvm.reset();
    gs_tcvp.reset();
    gs_tcf.reset();
    gs_tkem.reset();
    gs_tkep.reset();
    gs_tmask.reset();
    gs_racc.reset();
    {
        const char* e = std::getenv("AMG_GS_TEMPLATES");
        const bool allow = !(e && std::atoi(e) == 0);
        // the template kernels take one chain coupling per row: every template's in-chunk
        // offsets (0 < |o| < B) must be -1 / +1 only
        std::vector<int> hdrs, toff;
        std::vector<double> tval;
        bool shape_ok = n_tpl > 0 && tpl_win > 0;
        if (shape_ok) {
            hdrs.resize(n_tpl);
            toff.resize(n_tpl_ent);
            tval.resize(n_tpl_ent);
            HIP_CHECK(hipMemcpy(hdrs.data(), tpl_hdr.p, sizeof(int) * n_tpl, hipMemcpyDeviceToHost));
            HIP_CHECK(hipMemcpy(toff.data(), tpl_off.p, sizeof(int) * n_tpl_ent, hipMemcpyDeviceToHost));
            HIP_CHECK(hipMemcpy(tval.data(), tpl_val.p, sizeof(double) * n_tpl_ent, hipMemcpyDeviceToHost));
            for (int o : toff)
                if (o != 0 && o != -1 && o != 1 && std::llabs(o) < B) shape_ok = false;
        }
        if (allow && shape_ok && first_row % 64 == 0 && 64 % B == 0 &&
            (int64_t)tpl_id_host.size() == n_rows) {
            std::vector<uint8_t> gid((size_t)n_rows, (uint8_t)kTplNone);
            std::vector<std::vector<std::pair<uint64_t, int>>> by_tpl(n_tpl);
            std::vector<int> gbase;
            std::vector<double> gdl;
            bool ok = true;
            for (int64_t i = 0; i < n_rows && ok; ++i) {
                const int t = tpl_id_host[i];
                if (t == kTplNone) continue;
                uint64_t bits;
                std::memcpy(&bits, &di[i], sizeof(bits));
                int found = -1;
                for (const auto& pr : by_tpl[t])
                    if (pr.first == bits) {
                        found = pr.second;
                        break;
                    }
                if (found < 0) {
                    if ((int)gbase.size() >= kTplMax) {
                        ok = false;
                        break;
                    }
                    found = (int)gbase.size();
                    gbase.push_back(t);
                    gdl.push_back(di[i]);
                    by_tpl[t].push_back({bits, found});
                }
                gid[i] = (uint8_t)found;
            }
            if (ok) {
                const int64_t nb = (n_rows + kTplRows - 1) / kTplRows;
                tblk.assign((size_t)nb, 0);
                std::vector<int> blist;
                for (int64_t q = 0; q < nb; ++q) {
                    bool all = true;
                    for (int64_t i = q * kTplRows; i < std::min(n_rows, (q + 1) * kTplRows) && all; ++i)
                        all = gid[i] != kTplNone;
                    if (all) {
                        tblk[q] = 1;
                        blist.push_back((int)q);
                    }
                }
                if (!blist.empty()) {
                    std::vector<int> gh(gbase.size()), cf(gbase.size(), 0);
                    std::vector<int> kem(gbase.size(), -1), kep(gbase.size(), -1);
                    std::vector<double> cvm(gbase.size(), 0.0), cvp(gbase.size(), 0.0);
                    for (size_t k = 0; k < gbase.size(); ++k) {
                        const int h = hdrs[gbase[k]];
                        gh[k] = h;
                        const int st = h & 0xffff, ln = (h >> 16) & 0xff;
                        for (int e = st; e < st + ln; ++e) {
                            if (toff[e] == -1) cvm[k] = tval[e], cf[k] |= 1, kem[k] = e - st;
                            if (toff[e] == 1) cvp[k] = tval[e], cf[k] |= 2, kep[k] = e - st;
                        }
                    }
                    gs_tcvm.upload(cvm.data(), cvm.size());
                    gs_tcvp.upload(cvp.data(), cvp.size());
                    gs_tcf.upload(cf.data(), cf.size());
                    gs_tkem.upload(kem.data(), kem.size());
                    gs_tkep.upload(kep.data(), kep.size());
                    gs_racc.alloc((size_t)n_rows);
                    gs_tid.upload(gid.data(), gid.size());
                    gs_thdr.upload(gh.data(), gh.size());
                    gs_tdl.upload(gdl.data(), gdl.size());
                    gs_tblocks.upload(blist.data(), blist.size());
                    if (tpl_mne > 0) {  // uniform stencil: a GS template's mask is its row template's
                        std::vector<unsigned> tm_(n_tpl), gm(gbase.size());
                        HIP_CHECK(hipMemcpy(tm_.data(), tpl_mmask.p, sizeof(unsigned) * n_tpl, hipMemcpyDeviceToHost));
                        for (size_t k = 0; k < gbase.size(); ++k) gm[k] = tm_[gbase[k]];
                        gs_tmask.upload(gm.data(), gm.size());
                    }
                    n_gs_tpl = (int)gbase.size();
                    n_gs_tblk = (int)blist.size();
                } else {
                    tblk.clear();
                }
            }
        }
    }
    auto on_tpl = [&](int64_t r) { return !tblk.empty() && tblk[(size_t)(r / kTplRows)] != 0; };
    // the other rows: chunks packed whole into <= 64-row slabs; interior slabs (no halo
    // column) first, so par_hybrid_gs runs them while the halo is in flight
    std::vector<int4> slabs;
    std::vector<char> sbnd;
    for (int64_t r = 0; r < n_rows;) {
        if (on_tpl(r)) {
            r = std::min(n_rows, (r / kTplRows + 1) * kTplRows);
            continue;
        }
        int64_t end = r;
        while (end < n_rows && !on_tpl(end)) {
            const int64_t g = first_row + end;
            const int64_t ce = std::min(n_rows, (g / B + 1) * B - first_row);
            if (ce - r > 64) break;
            end = ce;
        }
        AMG_ASSERT(end > r);
        int w = 0;
        char bnd = 0;
        for (int64_t i = r; i < end; ++i) {
            w = std::max<int>(w, (int)(host.rp[i + 1] - host.rp[i]));
            for (int64_t k = host.rp[i]; k < host.rp[i + 1] && !bnd; ++k)
                bnd = host.col[k] < first_col || host.col[k] >= first_col + n_cols_local;
        }
        slabs.push_back(make_int4((int)r, (int)(end - r), 0, w));
        sbnd.push_back(bnd);
        r = end;
    }
    {
        std::vector<int4> ordered;
        ordered.reserve(slabs.size());
        for (int pass = 0; pass < 2; ++pass)
            for (size_t q = 0; q < slabs.size(); ++q)
                if (sbnd[q] == pass) ordered.push_back(slabs[q]);
        n_gs_slabs_int = 0;
        for (char c : sbnd) n_gs_slabs_int += c == 0;
        slabs.swap(ordered);
    }
    int64_t cells = 0;
    for (int4& sl : slabs) {
        sl.z = (int)cells;
        cells += (sl.w + 3) & ~3;  // slabs start at multiples of 4 cells (dictionary dwords)
    }
    AMG_CHECK((cells + 4) * 64 < INT_MAX, "hybrid GS: sliced-ELL too large for int32 offsets");
    gs_slabs.upload(slabs.data(), slabs.size());
    gs_slabs_host = slabs;
    gs_cells = cells;
    gs_ell_built = false;
    gs_col.reset();
    gs_val.reset();
    gs_vid.reset();
    gs_vtab.reset();
    gs_ndict = 0;
    gs_dinv.upload(di.data(), di.size());
    n_gs_slabs = (int)slabs.size();
    gs_block = B;
    // bytes per sweep: ELL cells + slab headers + 32 B per ELL row (b, x, dinv, y)
    int64_t ell_rows = 0;
    for (const int4& sl : slabs) ell_rows += sl.y;
    gs_bytes = (gs_ndict > 0 ? 5 : 12) * 64 * cells + 16 * (int64_t)slabs.size() + 32 * ell_rows;
    // template rows: acc kernel 1 B id + b + x (window) + acc out; chain kernel acc + x + id + y
    if (n_gs_tblk > 0)
        gs_bytes += 50 * (n_rows - ell_rows) + 16 * (int64_t)n_tpl_ent + 12 * (int64_t)n_gs_tpl;
    gs_wide = !slabs.empty() && cells >= (int64_t)kGsWide * (int64_t)slabs.size();

    // Split sweeps: the old-value couplings as a CSR-block pass (KM_GSACC on A
    // without the sweep's in-chunk new-value couplings -- the same entries in the same order,
    // so acc is bit-identical) and the chain walk on a sliced ELL of the new-value couplings
    // only.  No GS template rows, and rows of >= AMG_GS_SPLIT_NPR entries on average (default
    // 12: g3sub's 5.5-entry level 0 ran 60 -> 72 us per sweep split, its 45-entry level 1
    // 121 -> 63 us; profiles/r3u_split_ab.txt; 0 forces it, tests).  On N ranks (r5) the pass
    // is a distributed matrix of its own: its off-rank columns are A's (chunks never cross a
    // rank cut, so every in-chunk coupling is local), par_apply exchanges their halo while the
    // interior blocks run, and the old values across ranks are the Jacobi-across-ranks half of
    // the oracle's rank-cut definition -- results unchanged.  The pass is built collectively,
    // so the ranks agree first: all split or none do.
    gs_split = false;
    for (int d = 0; d < 2; ++d) {
        gs_old[d].reset();
        gs_cslabs[d].reset();
        gs_ccol[d].reset();
        gs_cval[d].reset();
    }
    gs_acc.reset();
    {
        const char* e = std::getenv("AMG_GS_SPLIT_NPR");
        const int64_t npr = e ? std::atoll(e) : (int64_t)12;
        const char* off = std::getenv("AMG_GS_SPLIT");
        const bool allow = !(off && std::atoi(off) == 0);
        bool split = allow && n_gs_tblk == 0 && n_rows > 0 && nnz >= npr * n_rows;
        if (ctx->host.nranks > 1 && !replicated)
            for (int64_t v : ctx->host.allgather((int64_t)(split ? 1 : 0))) split = split && v != 0;
        if (split) {
            // in-chunk new-value coupling of row i (local ids): forward cs <= j < i, backward
            // i < j < ce (hybrid_gs_kernel's [lo, hi))
            auto chunk = [&](int64_t i, int64_t& cs, int64_t& ce) {
                const int64_t g = first_row + i;
                cs = std::max<int64_t>(0, (g / B) * B - first_row);
                ce = std::min<int64_t>(n_rows, (g / B + 1) * B - first_row);
            };
            auto is_new = [&](int d, int64_t i, int64_t gc) {
                if (gc < clo || gc >= chi) return false;
                const int64_t j = gc - clo;
                int64_t cs, ce;
                chunk(i, cs, ce);
                return d == 0 ? (j >= cs && j < i) : (j > i && j < ce);
            };
            int64_t ccells = 0;
            gs_split = true;  // (ensure_gs_pass checks it)
            for (int d = 0; d < 2; ++d) {
                // the backward pass (post-smoothing) is built now; the forward one on first
                // use (ensure_gs_pass): a coarse level's forward sweep starts from x = 0 and
                // skips it (par_hybrid_gs_from_zero)
                if (d == 1) ensure_gs_pass(1);
                // the chain ELL: same slabs, only the new-value couplings (CSR order)
                std::vector<int4> cs = slabs;
                int64_t cc = 0;
                for (int4& sl : cs) {
                    int w = 0;
                    for (int l = 0; l < sl.y; ++l) {
                        const int64_t i = sl.x + l;
                        int c = 0;
                        for (int64_t k = host.rp[i]; k < host.rp[i + 1]; ++k) c += is_new(d, i, host.col[k]);
                        w = std::max(w, c);
                    }
                    sl.z = (int)cc;
                    sl.w = w;
                    cc += (w + 3) & ~3;
                }
                std::vector<int> ccol((size_t)(cc + 4) * 64, -1);
                std::vector<double> cval(ccol.size(), 0.0);
#pragma omp parallel for schedule(dynamic, 64)
                for (size_t q = 0; q < cs.size(); ++q) {
                    const int4 sl = cs[q];
                    for (int l = 0; l < sl.y; ++l) {
                        const int64_t i = sl.x + l;
                        int c = 0;
                        // consumption order: forward ascending, backward descending column
                        for (int64_t kk = host.rp[i]; kk < host.rp[i + 1]; ++kk) {
                            const int64_t k = d == 0 ? kk : host.rp[i + 1] - 1 - (kk - host.rp[i]);
                            if (is_new(d, i, host.col[k])) {
                                const size_t at = ((size_t)sl.z + (size_t)c++) * 64 + l;
                                ccol[at] = (int)(host.col[k] - clo);
                                cval[at] = host.val[k];
                            }
                        }
                    }
                }
                // one chain launch: every slab in the widest slab's width bucket (one launch per
                // bucket measured slower, g3sub 1560 -> 1360 V-cycles/s: the coarse levels pay
                // the extra launches, profiles/r4f_g3sub_buckets.txt)
                int wmax = 0;
                for (const int4& sl : cs) wmax = std::max(wmax, sl.w);
                for (int q = 0; q <= kGsChainBuckets; ++q) gs_cbucket[d][q] = 0;
                gs_cbucket[d][gs_chain_bucket(wmax) + 1] = (int)cs.size();
                for (int q = 0; q < kGsChainBuckets; ++q) gs_cbucket[d][q + 1] += gs_cbucket[d][q];
                gs_cslabs[d].upload(cs.data(), cs.size());
                gs_ccol[d].upload(ccol.data(), ccol.size());
                gs_cval[d].upload(cval.data(), cval.size());
                gs_cmaxw[d] = 0;
                for (const int4& sl : cs) gs_cmaxw[d] = std::max(gs_cmaxw[d], sl.w);
                if (d == 0) ccells = cc;
            }
            gs_acc.alloc((size_t)n_rows);
            gs_split = true;
            // bytes per (forward) sweep: the pass (its stored format + b + acc out), then the
            // chain ELL cells + slab headers + acc, x, dinv in and y out
            gs_bytes = gs_old[1]->mode_bytes(KM_RESID) + 8 * n_rows + 12 * 64 * ccells +
                       16 * (int64_t)slabs.size() + 32 * n_rows;
        }
    }
    if (!gs_split) ensure_gs_ell();
}

int64_t DevMatrix::format_generation = 0;

int64_t DevMatrix::mode_bytes(int mode) const {
    const int64_t n = n_rows;
    if (format == AMG_FORMAT_CSR) {  // residual + 8 n (b), Jacobi + 16 n (b, dinv)
        const int64_t base = csr_plain_bytes();
        return base + (mode == KM_JACOBI ? 16 * n : mode == KM_SPMV ? 0 : 8 * n);
    }
    const bool tpl = tpl_on();
    int64_t b = tpl ? spmv_fmt_bytes : csr_fmt_bytes;
    if (mode != KM_SPMV) b += 8 * n;  // b, or y for y += A x
    // template rows take 1/a_ii and x[r] from LDS; CSR-kernel rows stream them
    if (mode == KM_JACOBI) b += tpl ? jac_extra_csr : jac_extra_all;
    return b;
}

void DevMatrix::set_format(int f) {
    AMG_CHECK(f == AMG_FORMAT_AUTO || f == AMG_FORMAT_CSR || f == AMG_FORMAT_BLOCKS, "bad format");
    if (f == AMG_FORMAT_CSR && !pcol.p && nnz + 2 > 0) {
        // plain arrays in local | halo numbering, in row order (row_ptr is `rp`); two padding
        // entries (column 0, value 0) keep the kernel's last 16-byte pair inside the buffer
        const int64_t clo = first_col, chi = first_col + n_cols_local;
        std::vector<int> pc((size_t)nnz + 2, 0);
        std::vector<double> pv((size_t)nnz + 2, 0.0);
#pragma omp parallel for schedule(static)
        for (int64_t k = 0; k < nnz; ++k) {
            const int64_t g = host.col[k];
            pc[k] = g >= clo && g < chi ? (int)(g - clo) : (int)(n_cols_local + plan.find(g));
            pv[k] = host.val[k];
        }
        pcol.upload(pc.data(), pc.size());
        pval.upload(pv.data(), pv.size());
    }
    if (f != AMG_FORMAT_CSR) {
        // the plain arrays (12 B per nonzero) are rebuilt when CSR is selected again; hipFree
        // waits for the kernels that may still read them
        pcol.reset();
        pval.reset();
    }
    if (format != f) ++format_generation;
    format = f;
}

bool DevMatrix::halo_begin(const double* x) {
    const HostComm& comm = ctx->host;
    if (comm.nranks == 1 || replicated) return false;
    hipStream_t s = ctx->stream, cs = ctx->comm_stream;
    if (ctx->transport == TR_LOOPBACK) {  // collective on every rank, even with no neighbours
        loopback_before_pack(*ctx, plan.send_procs);
        launch_pack(s, (int64_t)plan.send_idx.size(), send_idx.p, x, send_buf.p);
        loopback_halo(*ctx, seq, send_buf.p, halo.p, plan.send_procs, plan.recv_procs,
                      plan.recv_ptr, true);
        return true;
    }
    if (plan.send_idx.empty() && plan.halo_gid.empty()) return false;
    ctx->eager_rccl_fence();
    static const bool trace = std::getenv("AMG_TRACE_RCCL") != nullptr;
    if (trace) std::fprintf(stderr, "[amg] rank %d halo_begin seq %lld send %zu recv %lld\n", comm.rank,
                            (long long)seq, plan.send_idx.size(), (long long)plan.n_halo());
    launch_pack(s, (int64_t)plan.send_idx.size(), send_idx.p, x, send_buf.p);
    HIP_CHECK(hipEventRecord(ctx->ev_pack, s));
    HIP_CHECK(hipStreamWaitEvent(cs, ctx->ev_pack, 0));
    NCCL_CHECK(ncclGroupStart());
    for (size_t p = 0; p < plan.send_procs.size(); ++p)
        NCCL_CHECK(ncclSend(send_buf.p + plan.send_ptr[p], (size_t)(plan.send_ptr[p + 1] - plan.send_ptr[p]),
                            ncclDouble, plan.send_procs[p], ctx->nccl, cs));
    for (size_t p = 0; p < plan.recv_procs.size(); ++p)
        NCCL_CHECK(ncclRecv(halo.p + plan.recv_ptr[p], (size_t)(plan.recv_ptr[p + 1] - plan.recv_ptr[p]),
                            ncclDouble, plan.recv_procs[p], ctx->nccl, cs));
    NCCL_CHECK(ncclGroupEnd());
    if (trace) std::fprintf(stderr, "[amg] rank %d halo group enqueued\n", comm.rank);
    HIP_CHECK(hipEventRecord(ctx->ev_halo, cs));
    return true;
}

void DevMatrix::halo_wait() { HIP_CHECK(hipStreamWaitEvent(ctx->stream, ctx->ev_halo, 0)); }

void par_apply(DevMatrix& A, int mode, const double* x, const double* b, double* y, double omega,
               double* partial) {
    if (mode == KM_JACOBI || mode == KM_RESID) AMG_CHECK(A.square, "Jacobi/residual need a square matrix");
    const bool comm = A.halo_begin(x);
    hipStream_t s = A.ctx->stream;
    const bool norm = partial != nullptr;
    if (A.format == AMG_FORMAT_CSR) {  // plain CSR: one launch over every row, after the halo
        if (comm) A.halo_wait();
        launch_csr_plain(s, mode, norm, A, x, b, y, omega, partial);
        return;
    }
    // template rows never touch the halo: they run with the interior blocks; the CSR kernel's
    // partials follow the template kernel's
    const bool tp = A.tpl_on();
    const int c0 = tp ? A.nb_skip : 0;
    const int poff = tp ? (A.tpl_blocks() - A.nb_skip) * kNormParts : 0;
    if (tp) launch_tpl(s, mode, norm, A, x, b, y, omega, partial);
    launch_csr_stream(s, mode, norm, A, c0, A.nb_int - c0, x, b, y, omega, partial, poff);
    if (comm) A.halo_wait();
    launch_csr_stream(s, mode, norm, A, A.nb_int, A.nb_bnd, x, b, y, omega, partial, poff);
}

bool par_restrict_j0(DevMatrix& R, const double* r, double* bc, double* x0c, const double* dinvc,
                     double omega) {
    if (R.format == AMG_FORMAT_CSR || R.tpl_on()) return false;
    const bool comm = R.halo_begin(r);
    hipStream_t s = R.ctx->stream;
    launch_csr_stream(s, KM_SPMV, false, R, 0, R.nb_int, r, nullptr, bc, omega, nullptr, 0, x0c, dinvc);
    if (comm) R.halo_wait();
    launch_csr_stream(s, KM_SPMV, false, R, R.nb_int, R.nb_bnd, r, nullptr, bc, omega, nullptr, 0, x0c, dinvc);
    return true;
}

void par_hybrid_gs(DevMatrix& A, const double* x, const double* b, double* y, int64_t block,
                   bool backward, double* partial) {
    A.ensure_gs_blocks(block);
    if (A.gs_split && !partial) {  // split sweep: the pass exchanges its halo
        A.ensure_gs_pass(backward ? 1 : 0);
        par_apply(*A.gs_old[backward ? 1 : 0], KM_GSACC, x, b, A.gs_acc.p, 0.0, nullptr);
        launch_gs_chain(A.ctx->stream, A, x, A.gs_acc.p, y, backward);
        return;
    }
    A.ensure_gs_ell();
    const bool comm = A.halo_begin(x);
    hipStream_t s = A.ctx->stream;
    // template blocks and interior slabs never read the halo: they run while it is in flight
    launch_hybrid_gs(s, A, x, b, y, backward, partial, 0, A.n_gs_slabs_int, true);
    if (comm) A.halo_wait();
    launch_hybrid_gs(s, A, x, b, y, backward, partial, A.n_gs_slabs_int, A.n_gs_slabs, false);
}

// Forward sweep from x = 0 (the first pre-smoothing sweep of a coarse level): every old-value
// term is a_ij * 0.0 = +-0.0, so acc = b bit for bit (b - (+-0.0) == b, and where b is -0.0
// the new x_i = 0.0 + acc * d is +0.0 either way) -- the split sweep's old-value pass and its
// halo exchange are skipped and the chain walk starts from acc = b.  Other forms sweep as usual.
void par_hybrid_gs_from_zero(DevMatrix& A, const double* x0, const double* b, double* y, int64_t block) {
    A.ensure_gs_blocks(block);
    if (A.gs_split) {
        launch_gs_chain(A.ctx->stream, A, x0, b, y, false);
        return;
    }
    par_hybrid_gs(A, x0, b, y, block, false);
}

void norm_finish(DevMatrix& A, const NormSink& ns, int nparts) {
    Context* c = A.ctx;
    const int nb = nparts >= 0 ? nparts : A.norm_parts();
    const int nr = c->host.nranks;
    double* local = ns.gathered + nr;
    // one rank: the reduction and the finish in one launch
    if (nr == 1 && launch_reduce_norm(c->stream, nb, ns.partial, ns.tmp, ns.done, local, ns.hist, ns.counter))
        return;
    if (nb > 0) launch_reduce_partials(c->stream, nb, ns.partial, ns.tmp, local);
    else launch_zero(c->stream, 1, local);
    if (nr > 1) {
        c->allgather(local, ns.gathered, 1);
        launch_finish_norm(c->stream, nr, ns.gathered, ns.hist, ns.counter);
    } else {
        launch_finish_norm(c->stream, 1, local, ns.hist, ns.counter);
    }
}

void par_residual_norm(DevMatrix& A, const double* x, const double* b, double* r,
                       const NormSink& ns) {
    par_apply(A, KM_RESID, x, b, r, 0.0, ns.partial);
    norm_finish(A, ns);
}

}  // namespace amg
