// device.hpp -- device (gfx950) side of the product: context, ParCSRMatrix on the GPU,
// the CSR-stream level kernels and the V-cycle.  SURVEY.md 8a rows a1-a7, a11.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <initializer_list>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "host.hpp"

namespace amg {

#define HIP_CHECK(expr)                                                                   \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            throw ::amg::Error(AMG_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)
#define NCCL_CHECK(expr)                                                                  \
    do {                                                                                  \
        ncclResult_t r_ = (expr);                                                         \
        if (r_ != ncclSuccess)                                                            \
            throw ::amg::Error(AMG_ERR_RCCL, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

// kernel geometry shared by host-side block building and the kernels
constexpr int kTPB = 256;   // threads per workgroup (4 waves of 64)
constexpr int kCAP = 2048;
constexpr int kGatherBand = 1 << 14;  // gather column-code band width (col16)  // nonzeros staged in LDS per workgroup (16 KiB of products)
constexpr int kPad = kCAP;  // col/val padding (entries): unconditional loads past a block's end
// x tile per workgroup: 16 KiB of LDS = kCAP doubles in lines of 8 doubles (256 lines of 64 B)
// or, r3, 4 doubles (512 lines of 32 B): a Galerkin row block reads a few doubles of each line
// it touches, so half-lines fit more rows in the same tile (the 7-pt 256^3 level-2 operator:
// 40,250 -> 25,615 blocks).  Chosen per operator (DevMatrix::line_w)
constexpr int kTileLines = kCAP / 8;     // 64-byte lines per tile
constexpr int kTileLinesMax = kCAP / 4;  // 32-byte lines per tile
constexpr int kNormParts = kTPB / 64;  // norm partials per CSR block (one per wave)
constexpr int kGsWide = 128;     // sliced-ELL width from which hybrid GS uses the wide variant
// split-GS chain walk: LDS queue widths, W entries per lane (12 W * 64 bytes
// per 64-lane workgroup), and the bucket of a slab whose widest lane has w couplings
constexpr int kGsChainBuckets = 4;
constexpr int kGsChainW[kGsChainBuckets] = {8, 16, 32, 64};
inline int gs_chain_bucket(int w) { return w <= 8 ? 0 : w <= 16 ? 1 : w <= 32 ? 2 : 3; }
constexpr int kGatherRPB = 4;    // rows per lane of gather (rectangular-operator) row blocks
// CSR block header h1.y: tile lines (low 16 bits); bit kHdrDvi = a value-indexed square
// block whose Jacobi takes 1/a_ii from its value table
constexpr int kHdrDvi = 1 << 16;
// row templates: 1-byte template id per row (kTplNone = row not templated)
constexpr int kTplNone = 255;
constexpr int kTplMax = 255;       // templates per operator
constexpr int kTplEntries = 1024;  // entries over all templates (staged in LDS per workgroup)
constexpr int kTplMaxLen = 64;     // entries per template

#ifndef AMG_CSR_PRE_TILE  // build-time knob: x-tile blocks issue batch 1 with the header
#define AMG_CSR_PRE_TILE 1
#endif
#ifndef AMG_TPL_BATCH  // build-time knob: window entries per batch in the template kernel (0: one)
#define AMG_TPL_BATCH 0
#endif
#ifndef AMG_TPL_SPLIT_READS  // build-time knob: uniform-stencil rows read each row's x separately
#define AMG_TPL_SPLIT_READS 1
#endif
#ifndef AMG_TPL_MASK_BRANCH  // build-time knob: masked uniform-stencil rows add under exec masks
#define AMG_TPL_MASK_BRANCH 0
#endif
#ifndef AMG_TPL_RPL  // build-time knob for same-box A/B builds (scripts/gpu_libab.sh)
#define AMG_TPL_RPL 2
#endif
constexpr int kTplRPL = AMG_TPL_RPL;  // rows per lane of the template kernel
constexpr int kTplBands = 8;       // x-window bands
constexpr int kTplChunks = 16;     // window chunks of kTPB slots (kTplWin / kTPB)
constexpr int kTplWin = 16 * 256;  // x-window doubles per workgroup (32 KiB of LDS)
constexpr int kTplRows = kTPB * kTplRPL;  // rows per template-kernel workgroup
// uniform-stencil rows: every template a subsequence of one master
// template; the kernels are instantiated for masters of these entry counts
constexpr int kTplMasterMax = 27;

// Host <-> device copies of large pageable buffers (setup: operator uploads, Galerkin and
// P / R downloads) through pinned staging: OpenMP threads fill one 32 MiB buffer while the
// DMA engine drains the other.  Synchronous for the host.  Below 4 MiB, plain hipMemcpy.
// copy_to_host waits for `after` (the producing stream).
void copy_to_device(void* dst, const void* src, size_t bytes);
void copy_to_host(void* dst, const void* src, size_t bytes, hipStream_t after);

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr, o.n = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) {
            reset();
            p = o.p, n = o.n;
            o.p = nullptr, o.n = 0;
        }
        return *this;
    }
    ~DevBuf() { reset(); }
    void reset() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    void alloc(size_t count) {
        reset();
        if (count) HIP_CHECK(hipMalloc(&p, count * sizeof(T)));
        n = count;
    }
    // count may be padded to >= 1 for an empty host array (data() == nullptr): then only the
    // allocation is made (a halo plan with no ghost ids, an operator without nonzeros)
    void upload(const T* h, size_t count) {
        alloc(count);
        if (count && h) copy_to_device(p, h, count * sizeof(T));
    }
};

// AMG_SEGV_BACKTRACE=1: print the native stack on SIGSEGV / SIGABRT (debugging host crashes
// inside runtime calls); a no-op otherwise
void install_crash_handler();

struct LoopbackWorld;

// Solve-time data path between ranks.  RCCL over xGMI (one process per GPU) is the product
// transport; LOOPBACK joins N contexts of ONE process (threads) that share a device: the
// same plans, pack kernels and interior/boundary overlap, with D2D copies + events + host
// barriers as the wire.  It exists so the multi-rank device path can be tested on a
// 1-GPU machine (RCCL refuses two ranks on one GPU).
enum Transport { TR_NONE = 0, TR_RCCL = 1, TR_LOOPBACK = 2 };

struct Context {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    hipStream_t comm_stream = nullptr;
    hipEvent_t ev_pack = nullptr, ev_halo = nullptr;
    HostComm host;
    int transport = TR_NONE;
    ncclComm_t nccl = nullptr;
    std::shared_ptr<LoopbackWorld> lb;
    void* lb_user = nullptr;  // host-exchange callback state for the loopback world
    int lb_omp_threads = 0;   // the joining thread's OpenMP team size before the loopback share
    std::thread::id lb_thread;
    int64_t mat_seq = 0;      // collective creation counter: matches matrices across ranks
    // RCCL ordering between graph-launched and eager work on this communicator:
    // `capturing` while a V-cycle is captured; `graph_inflight` from a multi-rank replay until
    // the stream is known idle.  An eager RCCL enqueue while a replay's RCCL work is in flight
    // deadlocks on RCCL's proxy (profiles/r4_rccl_graph_probe.txt), so eager_rccl_fence()
    // waits for the replays first -- once per graph -> eager transition, not per cycle.
    bool capturing = false;
    bool graph_inflight = false;
    void eager_rccl_fence();
    ~Context();
    // recv[q*count ..] = rank q's send[0..count) for every q (device pointers, on `stream`)
    void allgather(const double* send, double* recv, size_t count);
};

// Device image of one host CSR of the hierarchy during setup:
// the same rows, global column ids, in whichever index widths the consumers need -- int32 for
// the strength / aggregation / interpolation kernels, the transpose and the left operand of a
// SpGEMM, int64 for the SpGEMM's right operand (B image) and its row pointers.  A width that
// is missing is derived on the device from the other (ensure_*).
struct DevCsr {
    int64_t n = 0, nnz = 0, ncols = 0;
    DevBuf<int> rp32, col32;
    DevBuf<long long> rp64, col64;
    DevBuf<double> val;
    void ensure_rp32(hipStream_t s);
    void ensure_rp64(hipStream_t s);
    void ensure_col32(hipStream_t s);
    void ensure_col64(hipStream_t s);
};

// The device images of one hierarchy setup (Solver::setup; any rank count, r5).  A matrix the setup
// computes on the device (P, R = P^T, A_{l+1} = R (A P)) is registered as it is downloaded,
// so its consumers in the same level (transpose, Galerkin product, the next level's strength
// and aggregation) read it where it already is instead of uploading the host copy back; the
// level-0 operator is uploaded once.  Keyed by the host image's row-pointer buffer, which
// moves with the HostCSR and is never reallocated; the level loop keeps only the next
// level's operator when a level is done (keep_only), so no entry outlives its host matrix.
struct SetupImages {
    std::vector<std::pair<const int64_t*, std::unique_ptr<DevCsr>>> e;
    DevCsr* find(const HostCSR& M);
    DevCsr& get(const HostCSR& M);  // find, or upload rp64 / col64 / val
    void put(const HostCSR& M, std::unique_ptr<DevCsr> d);  // n / nnz / ncols taken from M
    void keep_only(const HostCSR& M);
};

// Galerkin SpGEMM on the device (spgemm.hip); result downloaded as a host image
HostCSR spgemm_device(Context& ctx, const HostComm& comm, const HostCSR& A, const HostCSR& B);
// formats.hip: the per-nonzero device formats of DevMatrix::build_view built on the GPU
// (AMG_DEVICE_FORMATS=0: the host builders); what the host block headers need back
struct FormatHeaderInfo {
    std::vector<int> vt_off, vt_len;  // per block: value-table offset (-1) and size
    std::vector<char> dvi_ok;         // per block: every row's diagonal is a table slot
    std::vector<int64_t> vofs;        // per block: offset in the value-index stream (empty: none)
};
bool device_formats();
struct DevMatrix;
void build_formats_device(DevMatrix& M, const std::vector<int>& hrp, const hvec<int>& hcol, const hvec<double>& hval,
                          const std::vector<int2>& blocks, const std::vector<int>& tile_ptr,
                          const std::vector<int>& tile_lines, const std::vector<int64_t>& koff, FormatHeaderInfo& out);
// R (A P), A P kept on the device between the products where it can be (one rank)
// imgs (may be null): A, P and R read from their device images, R (A P) registered
HostCSR galerkin_device(Context& ctx, const HostComm& comm, const HostCSR& R, const HostCSR& A,
                        const HostCSR& P, SetupImages* imgs = nullptr);
// device setup of one level (setup_device.hip): strength, PMIS or MIS(2) aggregation,
// classical or smoothed-aggregation P; false where it does not apply.  imgs: A's device image,
// P registered (SA: one rank)
bool level_setup_device(Context& ctx, const HostComm& comm, const HostCSR& A, const amg_options& opt,
                        int level, HostCSR& P, std::vector<int32_t>& split, SetupImages* imgs = nullptr);
bool transpose_device(Context& ctx, const HostComm& comm, const HostCSR& P, HostCSR& R,
                      SetupImages* imgs = nullptr);
// coarse-operator drop tolerance (host_setup.cpp sparsify) on A's device image (one rank; the
// host sparsify otherwise); the result is registered in imgs
HostCSR sparsify_device(Context& ctx, const HostComm& comm, const HostCSR& A, double tau, SetupImages* imgs);
// C = A B with A on the device (DevCsr: rp64, col32, val; one rank, global = local columns)
// and B's image on the device; C left on the device (rp also on the host)
struct DevCSR64 {
    std::vector<long long> rp;  // host copy
    DevBuf<long long> d_rp, d_col;
    DevBuf<double> d_val;
    int64_t nnz() const { return rp.empty() ? 0 : rp.back(); }
};
// brp_host: B's row pointers on the host; Bh: B's host image for the rare host-computed rows
// (null: downloaded from the device image if such a row occurs)
void spgemm_images(Context& ctx, PhaseTimer& tm, const HostCSR& Ah, DevCsr& A, const long long* brp_host,
                   const HostCSR* Bh, DevCsr& B, int64_t bncol, DevCSR64& C);

void loopback_join(Context& c, int rank, int nranks, const std::string& world);
void loopback_leave(Context& c);
void loopback_before_pack(Context& c, const std::vector<int>& send_procs);
void loopback_register(Context& c, int64_t seq, const double* send_buf,
                       const std::vector<int>& send_procs, const std::vector<int64_t>& send_ptr);
void loopback_halo(Context& c, int64_t seq, const double* x_send_buf, double* halo,
                   const std::vector<int>& send_procs, const std::vector<int>& recv_procs,
                   const std::vector<int64_t>& recv_ptr, bool packed);

// ParCSRMatrix on the device: rank-local rows, columns renumbered [local | halo].
struct DevMatrix {
    Context* ctx = nullptr;
    HostCSR host;              // host image (global column ids), kept for export / setup
    // while Solver::setup's worker threads build this operator's formats (and its GS
    // structures) from the hierarchy's CSR in place, before it is moved into `host`
    const HostCSR* host_view = nullptr;
    const HostCSR& host_image() const { return host_view ? *host_view : host; }
    int64_t first_row = 0, n_rows = 0, first_col = 0, n_cols_local = 0, nnz = 0;
    bool square = false;
    // stored for the x-tile kernel (tile ids, 16-bit tile indices, kCAP-stride VI indices):
    // square operators, and restrictions (rectangular, one row per lane) under AMG_RECT_TILE=1
    bool tiled = false;
    DevBuf<int> rp, col;
    DevBuf<double> val, dinv;
    // CSR-stream row blocks: [0, nb_int) interior rows, [nb_int, nb_int+nb_bnd) rows that
    // touch halo columns.  Each block is {row begin, row end}.
    DevBuf<int2> blocks;
    int nb_int = 0, nb_bnd = 0;
    // per block 2 x int4 = {r0, r1, k0, nnz}, {diag slot, tile lines, value-table offset
    // (-1: value stream), value-table size}: everything a block needs before its bulk loads
    DevBuf<int4> hdr;
    // x tiles: per block the sorted distinct 64-byte lines of x it reads (tile_fixed:
    // kTileLines ids per block, padded with the last) and per nonzero a 16-bit index into
    // that tile (lcol, lane-major)
    DevBuf<int> tile_fixed;
    // per row: end of its nonzeros relative to its block's first (16 bits; the kernel's row
    // bounds) and, for value-indexed square operators, the table index of its diagonal
    DevBuf<uint16_t> rend;
    DevBuf<uint8_t> dvi;
    DevBuf<uint16_t> lcol;
    int line_w = 8;  // doubles per x-tile line: 8 (64 B) or 4 (32 B)
    // gather operators (P, R): 16-bit column codes band << 14 | (col - band base) when every
    // block's columns fit in <= 4 bands of kGatherBand (gband: the block's 4 band bases);
    // null otherwise (int32 col).  Blocks of more than kCAP entries read col either way.
    DevBuf<uint16_t> col16;
    DevBuf<int4> gband;
    // HBM bytes of one SpMV launch in the stored format with the default kernel variant
    // (headers, tile ids, 16-bit tile indices, VI indices + tables or values, columns for the
    // gather path, row_ptr, x once, y): the roofline numerator, DESIGN.md section 4
    int64_t spmv_fmt_bytes = 0;
    // value-indexed blocks (<= 256 distinct values): the tables (offsets in hdr) and
    // lane-major 1-byte indices (kCAP per block)
    DevBuf<double> vtab;
    DevBuf<uint8_t> vidx;
    int n_vi_blocks = 0;
    int64_t vi_nnz = 0;  // nonzeros in value-indexed blocks
    // csr-stream variant bits (kernels.hip): 2 = XCD block order, 4 = gather (no x tile).
    // Set at build: x tile for square operators; gather + XCD order for rectangular ones.
    int default_variant = 0;
    // rows per lane of gather blocks: kGatherRPB for short-row rectangular operators (avg <= 4
    // entries per row: P of the classical hierarchy), whose blocks then hold up to 1024 rows
    int gather_rpb = 1;
    // l1 hybrid GS (built on first use for a given block size B <= 64): GS chunks = global
    // multiples of B clipped to this rank, packed whole into slabs of <= 64 rows (one
    // wavefront each, lane = row).  Each slab's rows are stored sliced-ELL, column-major
    // (entry k of lane l at (off + k) * 64 + l; col -1 = padding) so a lane's walk of its
    // row is a coalesced stream.  gs_dinv = 1 / (a_ii + sum of |a_ij| outside the chunk).
    DevBuf<int4> gs_slabs;  // {first row, rows, offset / 64, width}
    DevBuf<int> gs_col;
    // the slabs on the host and their cell count (the sliced ELL is built by ensure_gs_ell, on
    // first use for split operators)
    std::vector<int4> gs_slabs_host;
    int64_t gs_cells = 0;
    bool gs_ell_built = false;
    void ensure_gs_ell();
    void ensure_gs_pass(int d);  // gs_old[d], built on first use (ensure_gs_blocks: d = 1)
    DevBuf<double> gs_val, gs_dinv;
    int n_gs_slabs = 0;
    int n_gs_slabs_int = 0;  // slabs [0, n_gs_slabs_int) touch no halo column (run before the wait)
    int64_t gs_block = 0;
    // hybrid GS on row templates: 512-row blocks whose rows all have a GS
    // template = (row template, l1 diagonal) pair run tpl_gs_kernel; the sliced-ELL slabs
    // above cover the other rows only
    DevBuf<uint8_t> gs_tid;      // per row: GS template (kTplNone: ELL row)
    DevBuf<int> gs_thdr;         // per GS template: its row template's header
    DevBuf<double> gs_tdl;       // per GS template: 1 / (a_ii + l1)
    DevBuf<int> gs_tblocks;      // the 512-row blocks on the template kernel
    DevBuf<double> gs_tcvm, gs_tcvp;  // per GS template: value of its -1 / +1 entry (or 0)
    DevBuf<int> gs_tcf;          // per GS template: bit 0 has a -1 entry, bit 1 a +1 entry
    DevBuf<int> gs_tkem, gs_tkep;  // per GS template: index in the row of its -1 / +1 entry (-1)
    DevBuf<double> gs_racc;      // per row: b - old-value couplings (acc kernel -> chain kernel)
    int n_gs_tpl = 0, n_gs_tblk = 0;
    int gs_norm_parts() const { return n_gs_slabs + kNormParts * n_gs_tblk; }
    int64_t gs_bytes = 0;  // sliced-ELL bytes streamed per sweep
    bool gs_wide = false;  // average slab width >= kGsWide: the LDS-chain kernel variant
    // value dictionary (the whole local operator takes <= 256 distinct values, e.g. a
    // constant-coefficient stencil): 1-byte indices instead of gs_val, four entries of a
    // lane per dword -- entry k of lane l at (off + (k & ~3)) * 64 + 4 l + (k & 3) -- and
    // the table (gs_ndict values) staged in LDS by the kernel
    DevBuf<uint8_t> gs_vid;
    DevBuf<double> gs_vtab;
    int gs_ndict = 0;
    // split GS sweep (one rank or a replicated operator, no GS templates):
    // gs_old[0 / 1] = this operator without the forward / backward sweep's in-chunk new-value
    // couplings, in CSR-block format (its KM_GSACC pass leaves acc in gs_acc); gs_cslabs /
    // gs_ccol / gs_cval[0 / 1] = the same slabs' sliced ELL holding only those couplings, in
    // consumption order (backward: descending column) for gs_chain_kernel
    std::unique_ptr<DevMatrix> gs_old[2];
    // r5: an operator the caller created (C-ABI constructors) keeps, on one rank, the CSR the
    // device format build uploaded (row pointers, columns, values in row order) until a solver
    // setup takes it as its level-0 image (SetupImages) instead of uploading the operator
    // again; 12 B per nonzero while it is held (r6: the first C-ABI computation on the matrix
    // frees it too, capi.hip release_setup_image)
    bool keep_setup_csr = false;
    std::unique_ptr<DevCsr> setup_csr;
    DevBuf<int4> gs_cslabs[2];
    DevBuf<int> gs_ccol[2];
    DevBuf<double> gs_cval[2];
    DevBuf<double> gs_acc;
    bool gs_split = false;
    int gs_cmaxw[2] = {0, 0};  // widest chain-ELL slab per direction
    // chain slabs ordered by width bucket (gs_chain_bucket): bucket q is slabs
    // [gs_cbucket[d][q], gs_cbucket[d][q + 1]), walked by gs_chain_kernel<., kGsChainW[q]>
    int gs_cbucket[2][kGsChainBuckets + 1] = {};
    // row templates (square operators): rows whose columns are all local, written as
    // (column - row) offsets, values and 1/a_ii; rows with identical triples share a template.
    // tpl_id per row (kTplNone: the CSR block kernel handles the row); per template
    // tpl_hdr = start | len << 16 | diag entry << 24 (255: none), tpl_pd = 1/a_ii; entries
    // tpl_off / tpl_val.  CSR blocks [0, nb_skip) hold only templated rows: the block kernel
    // skips them while templates are active (tpl_on()).
    DevBuf<uint8_t> tpl_id;
    std::vector<uint8_t> tpl_id_host;  // host copy (GS templates are derived from it)
    DevBuf<int> tpl_hdr, tpl_off;
    // x window: bands of template offsets; per entry its window slot (tpl_ldo);
    // tpl_win = window size in doubles, 0 = the bands do not fit (global x loads)
    std::vector<int> tpl_blo, tpl_bbase;
    DevBuf<int> tpl_ldo;
    // z-marching (variant bit 128): stride in blocks between a block and the one whose window
    // it reuses (0: no useful shift), and per window slot the source slot (-1: load)
    int tpl_march_s = 0;
    DevBuf<int> tpl_wsrc;
    int tpl_win = 0, tpl_wend = 0;
    DevBuf<double> tpl_val, tpl_pd;
    int n_tpl = 0, n_tpl_ent = 0, nb_skip = 0;
    int64_t tpl_rows = 0;  // rows the template kernel handles
    // uniform stencil: every template's (offset, value) entries are a
    // subsequence of the master template's (tpl_mne entries, window slots tpl_mslot, values
    // tpl_mval, diagonal entry tpl_mdiag), every template holds the diagonal and every 1/a_ii
    // is tpl_mpd; tpl_mmask / gs_tmask: per (GS) template, bit e = has master entry e.
    // tpl_mne = 0: not uniform.  tpl_mem / tpl_mep: master index of offset -1 / +1 (-1: none)
    int tpl_mne = 0, tpl_mdiag = -1, tpl_mem = -1, tpl_mep = -1;
    std::vector<int> tpl_mslot;
    std::vector<double> tpl_mval;
    double tpl_mpd = 0.0;
    DevBuf<unsigned> tpl_mmask, gs_tmask;
    int64_t csr_fmt_bytes = 0;  // spmv_fmt_bytes with templates off (AMG_KERNEL_VARIANT)
    // storage format the level kernels use (AMG_FORMAT_*, amg_par_csr_set_format):
    // AUTO = templates + CSR blocks (default), BLOCKS = CSR blocks only, CSR = plain CSR
    // (row_ptr / col / val exactly as SURVEY.md 8(d) prices them; pcol / pval are built when
    // the format is first selected: local | halo column numbering, 2 padding entries)
    int format = AMG_FORMAT_AUTO;
    bool blocks_only = false;  // build only the CSR-block formats (the split-GS pass operators)
    // local rows as a lexicographic box (x fastest) of these extents, when the operator came
    // from a grid (stencil constructors); 0: unknown.  Only a locality hint (cycle order)
    int64_t grid_local[3] = {0, 0, 0};
    // build-time only: this rank's send lists index its column level through this map (old
    // local position -> new; the cycle-order copies)
    const std::vector<int64_t>* send_map = nullptr;
    DevBuf<int> pcol;
    DevBuf<double> pval;
    int plain_blocks() const { return (int)((n_rows + kTPB - 1) / kTPB); }
    // SURVEY.md 8(d) plain-CSR SpMV bytes: 12 nnz + 4 (n + 1) + 8 (local + halo columns) + 8 n
    int64_t csr_plain_bytes() const {
        return 12 * nnz + 4 * (n_rows + 1) + 8 * (n_cols_local + plan.n_halo()) + 8 * n_rows;
    }
    void set_format(int f);
    // stored-format HBM bytes of one application in `mode` (KernelMode) with the format and
    // kernel variant in effect (the bench's per-kernel roofline table)
    int64_t mode_bytes(int mode) const;
    int64_t jac_extra_all = 0, jac_extra_csr = 0;  // Jacobi operand bytes of the CSR-kernel rows
    static int64_t format_generation;  // bumped by every set_format: captured graphs go stale
    bool tpl_on() const;
    int tpl_blocks() const { return n_tpl > 0 ? (int)((n_rows + kTplRows - 1) / kTplRows) : 0; }
    // norm partials one NORM-mode application leaves (and the most either path can leave)
    int norm_parts() const;
    int norm_parts_max() const {
        return std::max(nb_int + nb_bnd + tpl_blocks(), plain_blocks()) * kNormParts;
    }
    // halo (ParComm): RCCL neighbour exchange
    HaloPlan plan;
    DevBuf<int> send_idx;
    DevBuf<double> send_buf, halo;
    int64_t seq = -1;  // collective id (loopback transport)

    // replicated: a whole matrix held by every rank (one-rank view, no halo, no exchange)
    bool replicated = false;
    void build(Context* c, HostCSR&& h, bool replicated_view = false);
    // host CSR and shape only; the device formats wait for ensure_built() (a level operator
    // the V-cycle runs as a cycle-order copy: built when a caller asks for it)
    bool deferred = false;
    void defer(Context* c, HostCSR&& h);
    void ensure_built();
    // the same formats from a CSR that stays the caller's (moved into `host` afterwards)
    void build_view(Context* c, const HostCSR& h, bool replicated_view = false);
    void ensure_gs_blocks(int64_t block);
    // start the halo exchange of x (pack on the compute stream, RCCL on the comm stream);
    // returns true when a boundary phase is needed
    bool halo_begin(const double* x);
    void halo_wait();
    int64_t n_halo() const { return plan.n_halo(); }
};

// KM_GSACC (square, no norm): y_i = b_i - sum_j a_ij x_j, subtracted one product at a time in
// CSR order (acc = b; acc -= a_ij x_j) -- the old-value half of an l1 hybrid GS sweep
//  on an operator without the sweep's in-chunk couplings
enum KernelMode { KM_SPMV = 0, KM_SPMV_ADD = 1, KM_RESID = 2, KM_JACOBI = 3, KM_GSACC = 4 };

// launchers (kernels.hip); all enqueue on s
// csr-stream variant bits in effect for A (DevMatrix::default_variant, VI and template bits,
// or AMG_KERNEL_VARIANT): 2 XCD order, 4 gather, 8 value-indexed, 32 row templates
int kernel_variant(const DevMatrix& A);
// partial slot of block bid's wave w: part_off + bid * kNormParts + w
void launch_csr_stream(hipStream_t s, int mode, bool norm, const DevMatrix& A, int first_block,
                       int n_blocks, const double* x, const double* b, double* y, double omega,
                       double* partial, int part_off = 0,
                       double* y2 = nullptr, const double* d2 = nullptr);
// template rows of A (all of them, one launch); partials at [0, tpl_blocks() * kNormParts)
void launch_tpl(hipStream_t s, int mode, bool norm, const DevMatrix& A, const double* x,
                const double* b, double* y, double omega, double* partial);
// hybrid GS sweep over slabs [s0, s1) of the sliced-ELL copy, plus (tpl) the template blocks;
// partials: slab q at q, template block list entry t, wave w at n_gs_slabs + 4 t + w
void launch_hybrid_gs(hipStream_t s, const DevMatrix& A, const double* x, const double* b,
                      double* y, bool backward, double* partial, int s0, int s1, bool tpl);
// chain walk of a split GS sweep: every slab, acc (from the KM_GSACC pass of
// A.gs_old) minus the in-chunk new-value couplings in sweep order, y = x + acc * dinv_l1
void launch_gs_chain(hipStream_t s, const DevMatrix& A, const double* x, const double* acc,
                     double* y, bool backward);
// plain CSR (AMG_FORMAT_CSR): all rows, one launch; partials at [0, plain_blocks() * kNormParts)
void launch_csr_plain(hipStream_t s, int mode, bool norm, const DevMatrix& A, const double* x,
                      const double* b, double* y, double omega, double* partial);
// dst = src (16-byte nontemporal copy kernel; the bench's STREAM-copy ceiling)
void launch_copy(hipStream_t s, int64_t n, const double* src, double* dst);
// one read pass over src (16-byte loads), per-wave partial sums into part[read_partials(n)]
// (the bench's read-bandwidth ceiling)
int64_t read_partials(int64_t n);
void launch_read(hipStream_t s, int64_t n, const double* src, double* part);
int tpl_march_chunk_cap();
void launch_jacobi_zero(hipStream_t s, int64_t n, const double* b, const double* dinv, double* y,
                        double omega);
void launch_pack(hipStream_t s, int64_t n, const int* idx, const double* x, double* out);
// deterministic sum of n per-block partials into *out (tmp: >= n/4096 + 16 doubles)
void launch_reduce_partials(hipStream_t s, int n, const double* partial, double* tmp, double* out);
// hist[*counter] = sqrt(sum_{i<n} in[i]) (rank order); ++*counter
bool launch_reduce_norm(hipStream_t s, int n, const double* partial, double* tmp, unsigned* done,
                        double* out, double* hist, int* counter);
void launch_finish_norm(hipStream_t s, int n, const double* in, double* hist, int* counter);
// PCG helpers: deterministic dot partials (fixed block span), scalar finish, fused updates
int dot_partial_count(int64_t n);
void launch_dot_partials(hipStream_t s, int64_t n, const double* a, const double* b, double* partial);
void launch_finish_sum(hipStream_t s, int n, const double* in, double* out, bool take_sqrt);
void launch_pcg_xr(hipStream_t s, int64_t n, const double* rz, const double* pq, const double* p,
                   const double* q, double* x, double* r);
void launch_pcg_p(hipStream_t s, int64_t n, const double* rz_new, const double* rz_old,
                  const double* z, double* p);
void launch_append(hipStream_t s, const double* v, double* hist, int* counter);
// x_i = inv_i . b, one wavefront per row, lane-interleaved partial sums + xor butterfly
void launch_dense_gemv(hipStream_t s, int64_t n_local, int64_t n, const double* inv,
                       const double* b, double* x);
void launch_uniform(hipStream_t s, int64_t n, int64_t first_gid, uint64_t seed, double* out);
void launch_zero(hipStream_t s, int64_t n, double* y);

// ParCSRMatrix operations with halo exchange + interior/boundary overlap
void par_apply(DevMatrix& A, int mode, const double* x, const double* b, double* y, double omega,
               double* partial_or_null);
// partial (forward only): per-slab sums of (b - A x)^2 for a fused residual norm
void par_hybrid_gs(DevMatrix& A, const double* x, const double* b, double* y, int64_t block,
                   bool backward = false, double* partial = nullptr);
// the forward sweep from x0 = 0 (zeroed by the caller): the split form skips its old-value pass
void par_hybrid_gs_from_zero(DevMatrix& A, const double* x0, const double* b, double* y, int64_t block);
// Norm plumbing: a mode-NORM level kernel leaves per-block partial sums of (b - Ax)^2 in
// NormSink::partial; norm_finish() reduces them (fixed order), combines ranks (RCCL
// allgather, rank order) and appends sqrt to hist[*counter] -- all on the device.
struct NormSink {
    double* partial = nullptr;  // >= number of blocks of the matrix
    double* tmp = nullptr;      // reduction scratch
    double* gathered = nullptr; // nranks + 1
    double* hist = nullptr;
    int* counter = nullptr;
    unsigned* done = nullptr;   // zeroed arrival counter of reduce_norm_kernel (null: two launches)
};
// b_c = R r and, fused, x0_c = omega * (dinv_c * b_c) (the coarse level's first Jacobi sweep
// from x = 0); false (nothing launched) where R is not on the CSR block path
bool par_restrict_j0(DevMatrix& R, const double* r, double* bc, double* x0c, const double* dinvc,
                     double omega);
// reduce `nparts` partials (default: one per CSR-stream block) and append the norm
void norm_finish(DevMatrix& A, const NormSink& ns, int nparts = -1);
// r = b - A x and append ||r|| (device-side) through ns
void par_residual_norm(DevMatrix& A, const double* x, const double* b, double* r,
                       const NormSink& ns);

struct Level {
    std::unique_ptr<DevMatrix> A, P, R;
    // cycle-order copies: the same operators with this level's points (and
    // the next level's) in a private brick order, entries of each row in the hierarchy's order;
    // null where the cycle runs the operator above as it is
    std::unique_ptr<DevMatrix> Ac, Pc, Rc;
    std::vector<int32_t> split;  // C/F or aggregate id (local rows)
    DevBuf<double> x, b, r, t;
};

struct Solver {
    Context* ctx = nullptr;
    amg_options opt{};
    std::vector<Level> levels;
    DevMatrix* A0 = nullptr;  // borrowed fine matrix (levels[0].A is null)
    // coarsest level: dense inverse rows of this rank, row-major (invT[i * n + j]); b gathered
    // padded, then unpadded into global order (bfull)
    DevBuf<double> invT, bfull;
    std::vector<int64_t> coarse_starts;
    int64_t coarse_n = 0;
    std::vector<int> coarse_counts, coarse_displs;
    // replicated coarse levels: levels >= rep_level are whole on every rank (-1: none)
    int rep_level = -1;
    std::vector<int64_t> rep_starts;
    int64_t rep_cmax = 0;
    DevBuf<double> rep_pad;
    // solve state: residual history kept on the device, appended by finish_norm_kernel
    DevBuf<double> hist, norm_scratch;
    DevBuf<int> hist_counter;
    DevBuf<unsigned> norm_done;
    NormSink sink;
    bool use_graph = true;
    // multi-rank capture of whole cycles (RCCL groups inside the graph): allowed on the
    // runtime it was validated on; *why gets the reason when it is not
    static bool rccl_graph_allowed(std::string* why = nullptr);
    struct Graph {
        hipGraphExec_t exec = nullptr;
        const double* x = nullptr;
        const double* b = nullptr;
        int64_t fmt_gen = -1;
    } graphs[5];  // [0] plain cycle, [1] cycle that also appends ||b - A x_in||, [2] the
                  // residual norm alone (solve's last norm), [3] / [4] the two halves of a
                  // PCG iteration (Solver::pcg)
    enum { G_CYCLE = 0, G_CYCLE_NORM = 1, G_NORM = 2, G_PCG_STEP = 3, G_PCG_PREC = 4 };
    // the graph in `slot` captured for (x, b) -- recaptured by `body` when stale.  Multi-rank
    // with `agree`: the ranks decide together (host allgather of the stale flags, then of the
    // capture / instantiate status), so no rank captures while a peer replays.  false: the
    // solver fell back to eager cycles (every rank, together).
    bool graph_ready(int slot, const double* x, const double* b, const std::function<void()>& body,
                     bool agree);
    void agree_stale(std::initializer_list<int> slots, const double* x, const double* b);
    void graph_launch(int slot);
    void destroy_graphs();
    void drop_graph(Graph& G);  // destroy one exec once the stream has drained

    DevMatrix& Amat(size_t l) { return l == 0 ? *A0 : *levels[l].A; }
    // the operators the cycle runs (cycle-order copies where they exist)
    DevMatrix& CA(size_t l) { return l > 0 && levels[l].Ac ? *levels[l].Ac : Amat(l); }
    DevMatrix& CP(size_t l) { return levels[l].Pc ? *levels[l].Pc : *levels[l].P; }
    DevMatrix& CR(size_t l) { return levels[l].Rc ? *levels[l].Rc : *levels[l].R; }
    void setup(DevMatrix& A, const amg_options& o);
    // one V-cycle; with_norm: the first level-0 Jacobi sweep also appends ||b - A x_in||
    // to the device history (falls back to a separate residual when it cannot).  agree: the
    // multi-rank graph decision is collective (false only where the caller made it already)
    void cycle(double* x, const double* b, bool with_norm = false, bool agree = true);
    // ||b - A x|| appended to the device history (the norm graph where graphs are on)
    void residual_norm(double* x, const double* b, bool agree);
    // x0_in_t: level l's first pre-sweep from x = 0 already sits in levels[l].t (fused into
    // the restriction above, par_restrict_j0)
    void cycle_rec(size_t l, double* x, const double* b, bool x_zero, bool with_norm, bool x0_in_t = false);
    void smooth(size_t l, double*& x, const double* b, double*& tmp, bool x_zero, bool with_norm,
                bool post = false);
    void ensure_hist(int32_t n);
    bool can_fuse_norm() const;
    // ParMultilevel::solve; hist_host gets it+1 norms
    int32_t solve(double* x, const double* b, int32_t max_iter, double tol, double* hist_host);
    // AMG-preconditioned conjugate gradients (one V-cycle per iteration as M^-1)
    int32_t pcg(double* x, const double* b, int32_t max_iter, double tol, double* hist_host);
    DevBuf<double> pcg_vec, pcg_scratch;  // r | z | p | q ; dot partials | tmp | gathered | scalars
    void dot(const double* a, const double* b, double* dst, bool take_sqrt);
    // in-graph time of every operation of a cycle (amg_solver_cycle_timeline, one rank): while
    // tl_on, cycle_rec marks the end of each operation -- a timing event when eager, the end of
    // a captured segment (one graph per operation, replayed back to back) when capturing
    bool tl_on = false;
    int tl_mode = 0;  // 2: event-record nodes in one graph, 1: one graph per operation, 0: eager
    std::vector<hipEvent_t> tl_ev;
    std::vector<std::string> tl_label;
    std::vector<hipGraph_t> tl_graphs;  // the timeline's captured segments (one per operation)
    size_t tl_n = 0;
    void mark(size_t l, const char* what);
    // reps replays (eager cycles where graphs are off); per operation the median of the
    // event-to-event times in microseconds; returns the mode that timed them (tl_mode)
    int cycle_timeline(double* x, const double* b, int reps, std::vector<std::string>& labels,
                       std::vector<double>& us);
    int64_t bytes_per_cycle(size_t l) const;
    // the bytes level l's share of a cycle streams in the stored formats (<= what HBM can
    // move in the measured time)
    int64_t stored_bytes_per_cycle(size_t l) const;
    ~Solver();
};

}  // namespace amg
