// capi.hip -- extern "C" boundary (include/raptor_amd.h).  Every entry point catches
// exceptions and turns them into an error code + thread-local message.
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>

#include "device.hpp"

using namespace amg;

struct amg_context_s {
    Context c;
};
struct amg_matrix_s {
    std::unique_ptr<DevMatrix> own;  // null for borrowed level views
    DevMatrix* m = nullptr;
};
struct amg_solver_s {
    Solver s;
    std::vector<std::unique_ptr<amg_matrix_s>> views;  // borrowed level handles
};

static thread_local std::string g_err;

template <class F>
static int guard(F&& f) {
    OmpQuiet quiet;  // blocktime 0 for the library's parallel regions, restored on return
    try {
        f();
        return AMG_OK;
    } catch (const Error& e) {
        g_err = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        g_err = "out of host memory";
        return AMG_ERR_NOMEM;
    } catch (const std::exception& e) {
        g_err = e.what();
        return AMG_ERR_INTERNAL;
    }
}

static void set_device(Context& c) { HIP_CHECK(hipSetDevice(c.device)); }

static HostCSR make_host_csr(const HostComm& comm, int64_t n_global, int64_t first_row,
                             int64_t n_local, const int64_t* row_ptr, const int64_t* col_global,
                             const double* val) {
    AMG_CHECK(row_ptr, "null row_ptr");
    AMG_CHECK(n_local >= 0 && first_row >= 0 && first_row + n_local <= n_global, "bad row range");
    HostCSR h;
    h.n_global_rows = h.n_global_cols = n_global;
    std::vector<int64_t> counts = comm.allgather(n_local);
    h.row_starts.assign(comm.nranks + 1, 0);
    for (int r = 0; r < comm.nranks; ++r) h.row_starts[r + 1] = h.row_starts[r] + counts[r];
    AMG_CHECK(h.row_starts[comm.rank] == first_row, "first_row inconsistent with rank order");
    AMG_CHECK(h.row_starts[comm.nranks] == n_global, "local row counts do not sum to n_global");
    h.col_starts = h.row_starts;
    AMG_CHECK(row_ptr[0] == 0, "row_ptr[0] must be 0");
    const int64_t nnz = row_ptr[n_local];
    h.rp.assign(row_ptr, row_ptr + n_local + 1);
    h.col.assign(col_global, col_global + nnz);
    h.val.assign(val, val + nnz);
    for (int64_t i = 0; i < n_local; ++i) {
        AMG_CHECK(row_ptr[i + 1] >= row_ptr[i], "row_ptr not monotone");
        const int64_t b = row_ptr[i], e = row_ptr[i + 1];
        bool sorted = true;
        for (int64_t k = b; k < e; ++k) {
            AMG_CHECK(col_global[k] >= 0 && col_global[k] < n_global, "column id out of range");
            if (k > b && col_global[k] <= col_global[k - 1]) sorted = false;
        }
        if (!sorted) {
            std::vector<int64_t> idx(e - b);
            std::iota(idx.begin(), idx.end(), b);
            std::sort(idx.begin(), idx.end(), [&](int64_t x, int64_t y) { return col_global[x] < col_global[y]; });
            for (int64_t t = 0; t < e - b; ++t) {
                h.col[b + t] = col_global[idx[t]];
                h.val[b + t] = val[idx[t]];
                AMG_CHECK(t == 0 || h.col[b + t] != h.col[b + t - 1], "duplicate column in a row");
            }
        }
    }
    return h;
}

// AMG_SEGV_BACKTRACE=1 (debugging a host crash inside a runtime call, e.g. RCCL graph
// capture): print the native stack to stderr on SIGSEGV / SIGABRT, then re-raise
static void amg_crash_handler(int sig) {
    void* fr[64];
    const int n = backtrace(fr, 64);
    const char msg[] = "[amg] fatal signal, native backtrace:\n";
    (void)!write(2, msg, sizeof(msg) - 1);
    backtrace_symbols_fd(fr, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

// (re)installed at context creation and again right before a hipGraph capture: runtimes
// loaded later (RCCL, a framework) may have replaced the handler in between

void amg::install_crash_handler() {
    const char* e = std::getenv("AMG_SEGV_BACKTRACE");
    if (!(e && std::atoi(e) != 0)) return;
    signal(SIGSEGV, amg_crash_handler);
    signal(SIGABRT, amg_crash_handler);
}

extern "C" {

const char* amg_last_error(void) { return g_err.c_str(); }
int amg_version(void) { return 100; }

int amg_runtime_versions(int32_t* hip_runtime, int32_t* rccl) {
    return guard([&] {
        AMG_CHECK(hip_runtime && rccl, "null output");
        int hv = 0, nv = 0;
        HIP_CHECK(hipRuntimeGetVersion(&hv));
        NCCL_CHECK(ncclGetVersion(&nv));
        *hip_runtime = hv;
        *rccl = nv;
    });
}

int amg_context_create(int device, void* hip_stream, amg_context* out) {
    return guard([&] {
        AMG_CHECK(out, "null output");
        install_crash_handler();
        int ndev = 0;
        HIP_CHECK(hipGetDeviceCount(&ndev));
        AMG_CHECK(device >= 0 && device < ndev, "device index out of range");
        auto* h = new amg_context_s();
        h->c.device = device;
        try {
            set_device(h->c);
            if (hip_stream) {
                h->c.stream = (hipStream_t)hip_stream;
            } else {
                HIP_CHECK(hipStreamCreateWithFlags(&h->c.stream, hipStreamNonBlocking));
                h->c.own_stream = true;
            }
            HIP_CHECK(hipStreamCreateWithFlags(&h->c.comm_stream, hipStreamNonBlocking));
            HIP_CHECK(hipEventCreateWithFlags(&h->c.ev_pack, hipEventDisableTiming));
            HIP_CHECK(hipEventCreateWithFlags(&h->c.ev_halo, hipEventDisableTiming));
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
    });
}

int amg_rccl_unique_id(void* out128) {
    return guard([&] {
        AMG_CHECK(out128, "null output");
        static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
        ncclUniqueId id;
        NCCL_CHECK(ncclGetUniqueId(&id));
        std::memcpy(out128, &id, sizeof(id));
    });
}

int amg_context_set_comm(amg_context ctx, int rank, int nranks, const void* uid,
                         amg_alltoallv_fn exchange, void* user) {
    return guard([&] {
        AMG_CHECK(ctx, "null context");
        AMG_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank/nranks");
        Context& c = ctx->c;
        set_device(c);
        AMG_CHECK(!c.nccl && !c.lb, "communicator already set");
        c.host.rank = rank;
        c.host.nranks = nranks;
        c.host.fn = exchange;
        c.host.user = user;
        if (nranks > 1) {
            AMG_CHECK(uid && exchange, "multi-rank needs an RCCL unique id and a host exchange");
            ncclUniqueId id;
            std::memcpy(&id, uid, sizeof(id));
            NCCL_CHECK(ncclCommInitRank(&c.nccl, nranks, id, rank));
            c.transport = TR_RCCL;
        }
    });
}

int amg_context_set_loopback(amg_context ctx, int rank, int nranks, const char* world) {
    return guard([&] {
        AMG_CHECK(ctx && world, "null argument");
        AMG_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank/nranks");
        Context& c = ctx->c;
        AMG_CHECK(!c.nccl && !c.lb, "communicator already set");
        set_device(c);
        loopback_join(c, rank, nranks, world);
    });
}

int amg_context_stream(amg_context ctx, void** s) {
    return guard([&] {
        AMG_CHECK(ctx && s, "null argument");
        *s = (void*)ctx->c.stream;
    });
}

int amg_context_synchronize(amg_context ctx) {
    return guard([&] {
        AMG_CHECK(ctx, "null context");
        set_device(ctx->c);
        HIP_CHECK(hipStreamSynchronize(ctx->c.stream));
        HIP_CHECK(hipStreamSynchronize(ctx->c.comm_stream));
        ctx->c.graph_inflight = false;
    });
}

int amg_context_destroy(amg_context ctx) {
    return guard([&] {
        if (!ctx) return;
        (void)hipSetDevice(ctx->c.device);
        (void)hipStreamSynchronize(ctx->c.stream);
        delete ctx;
    });
}

int amg_par_csr_create(amg_context ctx, int64_t n_global, int64_t first_row, int64_t n_local,
                       const int64_t* row_ptr, const int64_t* col_global, const double* val,
                       amg_matrix* out) {
    return guard([&] {
        AMG_CHECK(ctx && out && row_ptr, "null argument");
        AMG_CHECK(n_local >= 0 && first_row >= 0 && first_row + n_local <= n_global, "bad row range");
        Context& c = ctx->c;
        set_device(c);
        HostCSR h = make_host_csr(c.host, n_global, first_row, n_local, row_ptr, col_global, val);
        std::unique_ptr<amg_matrix_s> m(new amg_matrix_s());
        m->own.reset(new DevMatrix());
        m->m = m->own.get();
        m->m->keep_setup_csr = true;  // the level-0 operator of a later solver setup
        m->m->build(&c, std::move(h));
        *out = m.release();
    });
}

int amg_par_stencil_create(amg_context ctx, int kind, int64_t nx, int64_t ny, int64_t nz,
                           const double* eps3, amg_matrix* out) {
    return guard([&] {
        AMG_CHECK(ctx && out, "null argument");
        AMG_CHECK(kind == AMG_STENCIL_5PT || kind == AMG_STENCIL_7PT || kind == AMG_STENCIL_27PT,
                  "unknown stencil");
        Context& c = ctx->c;
        set_device(c);
        HostCSR h = stencil_slab(c.host, kind, nx, ny, nz, eps3);
        std::unique_ptr<amg_matrix_s> m(new amg_matrix_s());
        m->own.reset(new DevMatrix());
        m->m = m->own.get();
        m->m->keep_setup_csr = true;  // the level-0 operator of a later solver setup
        m->m->grid_local[0] = nx;     // a z-slab of whole (nx, ny) planes
        m->m->grid_local[1] = ny;
        m->m->grid_local[2] = (h.nrows() + nx * ny - 1) / (nx * ny);
        m->m->build(&c, std::move(h));
        *out = m.release();
    });
}

int amg_par_stencil_create_boxes(amg_context ctx, int kind, int64_t nx, int64_t ny, int64_t nz, int64_t bx,
                                 int64_t by, int64_t bz, const double* eps3, amg_matrix* out) {
    return guard([&] {
        AMG_CHECK(ctx && out, "null argument");
        AMG_CHECK(kind == AMG_STENCIL_5PT || kind == AMG_STENCIL_7PT || kind == AMG_STENCIL_27PT,
                  "unknown stencil");
        Context& c = ctx->c;
        set_device(c);
        HostCSR h = stencil_boxes(c.host, kind, nx, ny, nz, bx, by, bz, eps3);
        std::unique_ptr<amg_matrix_s> m(new amg_matrix_s());
        m->own.reset(new DevMatrix());
        m->m = m->own.get();
        m->m->keep_setup_csr = true;  // the level-0 operator of a later solver setup
        if (bx * by * bz == c.host.nranks) {  // one box per rank: its extents (stencil_boxes' split)
            const int64_t b = c.host.rank, ix = b % bx, iy = (b / bx) % by, iz = b / (bx * by);
            m->m->grid_local[0] = nx * (ix + 1) / bx - nx * ix / bx;
            m->m->grid_local[1] = ny * (iy + 1) / by - ny * iy / by;
            m->m->grid_local[2] = nz * (iz + 1) / bz - nz * iz / bz;
        }
        m->m->build(&c, std::move(h));
        *out = m.release();
    });
}

static void upload(Context& c, HostCSR&& h, amg_matrix* out) {
    std::unique_ptr<amg_matrix_s> m(new amg_matrix_s());
    m->own.reset(new DevMatrix());
    m->m = m->own.get();
    m->m->keep_setup_csr = true;  // the level-0 operator of a later solver setup
    m->m->build(&c, std::move(h));
    *out = m.release();
}

int amg_par_graph_laplacian_create(amg_context ctx, int64_t nx, int64_t ny, uint64_t seed,
                                   amg_matrix* out) {
    return guard([&] {
        AMG_CHECK(ctx && out, "null argument");
        set_device(ctx->c);
        upload(ctx->c, graph_laplacian_slab(ctx->c.host, nx, ny, seed), out);
    });
}

int amg_par_csr_read(amg_context ctx, const char* path, amg_matrix* out) {
    return guard([&] {
        AMG_CHECK(ctx && path && out, "null argument");
        set_device(ctx->c);
        HostCSR h = read_par_matrix(ctx->c.host, path);
        AMG_CHECK(h.n_global_rows == h.n_global_cols, "ParCSRMatrix needs a square matrix");
        upload(ctx->c, std::move(h), out);
    });
}

int amg_par_csr_write(amg_matrix A, const char* path) {
    return guard([&] {
        AMG_CHECK(A && path, "null argument");
        write_par_matrix(A->m->ctx->host, A->m->host, path);
    });
}

int amg_par_csr_reorder(amg_matrix A, int method, amg_matrix* out, int64_t* new_to_old_local) {
    return guard([&] {
        AMG_CHECK(A && out && new_to_old_local, "null argument");
        AMG_CHECK(method == AMG_REORDER_RCM, "unknown reorder method");
        Context& c = *A->m->ctx;
        set_device(c);
        std::vector<int64_t> n2o;
        HostCSR h = reorder_rcm(c.host, A->m->host, n2o);
        std::copy(n2o.begin(), n2o.end(), new_to_old_local);
        upload(c, std::move(h), out);
    });
}

int amg_par_csr_info(amg_matrix A, amg_matrix_info* info) {
    return guard([&] {
        AMG_CHECK(A && info, "null argument");
        std::memset(info, 0, sizeof(*info));
        // a level operator the cycle runs as a cycle-order copy is not built by info (that
        // would undo the deferral and double the level's device memory): its shape
        // fields are valid, its format fields 0 with deferred = 1, until the first compute call
        const DevMatrix& m = *A->m;
        info->deferred = m.deferred ? 1 : 0;
        if (m.deferred) {  // shape only
            info->n_global_rows = m.host.n_global_rows;
            info->n_global_cols = m.host.n_global_cols;
            info->first_row = m.first_row;
            info->n_local_rows = m.n_rows;
            info->first_col = m.first_col;
            info->n_local_cols = m.n_cols_local;
            info->nnz_local = m.nnz;
            return;
        }
        info->n_global_rows = m.host.n_global_rows;
        info->n_global_cols = m.host.n_global_cols;
        info->first_row = m.first_row;
        info->n_local_rows = m.n_rows;
        info->first_col = m.first_col;
        info->n_local_cols = m.n_cols_local;
        info->nnz_local = m.nnz;
        info->n_halo = m.plan.n_halo();
        info->n_send = (int64_t)m.plan.send_idx.size();
        info->n_neighbors = (int32_t)std::max(m.plan.send_procs.size(), m.plan.recv_procs.size());
        info->n_blocks = m.nb_int + m.nb_bnd;
        info->n_vi_blocks = m.n_vi_blocks;
        info->spmv_bytes = m.mode_bytes(KM_SPMV);
        info->n_templates = m.n_tpl;
        info->template_rows = m.tpl_on() ? m.tpl_rows : 0;
        info->format = m.format;
        info->kernel_variant = kernel_variant(m);
        info->csr_bytes = m.csr_plain_bytes();
        if (m.format == AMG_FORMAT_CSR) info->template_rows = 0;
        const bool tpl = m.tpl_on();
        info->tpl_window = tpl ? m.tpl_win : 0;
        const int w = info->tpl_window;
        info->tpl_lanes = w <= 0 ? 0 : w <= 4 * kTPB ? 4 : w <= 8 * kTPB ? 8 : w <= 12 * kTPB ? 12 : 16;
        info->tpl_march_shift = tpl && (info->kernel_variant & 128) ? m.tpl_march_s : 0;
        info->mult_add_bytes = m.mode_bytes(KM_SPMV_ADD);
        info->residual_bytes = m.square ? m.mode_bytes(KM_RESID) : 0;
        info->jacobi_bytes = m.square ? m.mode_bytes(KM_JACOBI) : 0;
        info->gs_bytes = m.gs_block > 0 ? m.gs_bytes : 0;
        info->tpl_master = tpl && (info->kernel_variant & 512) ? m.tpl_mne : 0;
        info->tile_line_bytes = m.tiled && m.format != AMG_FORMAT_CSR ? 8 * m.line_w : 0;
        info->gs_split = m.gs_block > 0 && m.gs_split ? 1 : 0;
        info->gs_chain_maxw = info->gs_split ? m.gs_cmaxw[0] | m.gs_cmaxw[1] << 16 : 0;
    });
}

int amg_par_csr_set_format(amg_matrix A, int32_t format) {
    return guard([&] {
        AMG_CHECK(A, "null matrix");
        set_device(*A->m->ctx);
        HIP_CHECK(hipStreamSynchronize(A->m->ctx->stream));
        A->m->ensure_built();
        A->m->set_format(format);
    });
}

int amg_par_csr_format_digest(amg_matrix A, uint64_t* digest) {
    return guard([&] {
        AMG_CHECK(A && digest, "null argument");
        DevMatrix& M = *A->m;
        set_device(*M.ctx);
        HIP_CHECK(hipStreamSynchronize(M.ctx->stream));
        M.ensure_built();
        uint64_t h = 1469598103934665603ull;
        auto mix = [&](const void* p, size_t bytes) {
            std::vector<unsigned char> b(bytes);
            if (bytes) HIP_CHECK(hipMemcpy(b.data(), p, bytes, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < 8; ++i) h = (h ^ ((bytes >> (8 * i)) & 0xff)) * 1099511628211ull;
            for (unsigned char c : b) h = (h ^ c) * 1099511628211ull;
        };
        mix(M.rp.p, M.rp.n * sizeof(int));
        mix(M.col.p, M.col.n * sizeof(int));
        mix(M.val.p, M.val.n * sizeof(double));
        mix(M.blocks.p, M.blocks.n * sizeof(int2));
        mix(M.hdr.p, M.hdr.n * sizeof(int4));
        mix(M.tile_fixed.p, M.tile_fixed.n * sizeof(int));
        mix(M.lcol.p, M.lcol.n * sizeof(uint16_t));
        mix(M.col16.p, M.col16.n * sizeof(uint16_t));
        mix(M.gband.p, M.gband.n * sizeof(int4));
        mix(M.vtab.p, M.vtab.n * sizeof(double));
        mix(M.vidx.p, M.vidx.n);
        mix(M.dvi.p, M.dvi.n);
        mix(M.rend.p, M.rend.n * sizeof(uint16_t));
        *digest = h;
    });
}

int amg_par_csr_export(amg_matrix A, int64_t* rp, int64_t* col, double* val) {
    return guard([&] {
        AMG_CHECK(A && rp && col && val, "null argument");
        const HostCSR& h = A->m->host;
        std::copy(h.rp.begin(), h.rp.end(), rp);
        std::copy(h.col.begin(), h.col.end(), col);
        std::copy(h.val.begin(), h.val.end(), val);
    });
}

// an operator's setup image (DevMatrix::setup_csr, 12 B per nonzero) is held only
// until the matrix is set up as a solver's level 0 or used for a computation, whichever comes
// first (a later setup uploads the operator again)
static void release_setup_image(DevMatrix& M) {
    if (M.setup_csr) M.setup_csr.reset();
}

static int apply(amg_matrix A, int mode, const double* x, const double* b, double* y, double w) {
    return guard([&] {
        AMG_CHECK(A, "null matrix");
        AMG_CHECK((x || A->m->n_cols_local == 0) && (y || A->m->n_rows == 0), "null vector");
        set_device(*A->m->ctx);
        A->m->ensure_built();
        release_setup_image(*A->m);
        par_apply(*A->m, mode, x, b, y, w, nullptr);
    });
}

int amg_par_csr_mult(amg_matrix A, const double* x, double* y) { return apply(A, KM_SPMV, x, nullptr, y, 0.0); }
int amg_par_csr_mult_add(amg_matrix A, const double* x, double* y) {
    return apply(A, KM_SPMV_ADD, x, nullptr, y, 0.0);
}
int amg_par_csr_residual(amg_matrix A, const double* x, const double* b, double* r) {
    return apply(A, KM_RESID, x, b, r, 0.0);
}
int amg_par_csr_jacobi(amg_matrix A, const double* x, const double* b, double* xo, double omega) {
    return apply(A, KM_JACOBI, x, b, xo, omega);
}

int amg_par_csr_hybrid_gs(amg_matrix A, const double* x, const double* b, double* xo, int64_t block) {
    return guard([&] {
        AMG_CHECK(A, "null matrix");
        AMG_CHECK(x != xo, "hybrid GS is out of place: x and x_out must differ");
        set_device(*A->m->ctx);
        A->m->ensure_built();
        release_setup_image(*A->m);
        par_hybrid_gs(*A->m, x, b, xo, block);
    });
}

int amg_par_csr_hybrid_gs_backward(amg_matrix A, const double* x, const double* b, double* xo,
                                   int64_t block) {
    return guard([&] {
        AMG_CHECK(A, "null matrix");
        AMG_CHECK(x != xo, "hybrid GS is out of place: x and x_out must differ");
        set_device(*A->m->ctx);
        A->m->ensure_built();
        release_setup_image(*A->m);
        par_hybrid_gs(*A->m, x, b, xo, block, true);
    });
}

int amg_par_csr_matmat(amg_matrix A, amg_matrix B, amg_matrix* out) {
    return guard([&] {
        AMG_CHECK(A && B && out, "null argument");
        AMG_CHECK(A->m->ctx == B->m->ctx, "matrices belong to different contexts");
        Context& c = *A->m->ctx;
        set_device(c);
        HostCSR h = spgemm_device(c, c.host, A->m->host, B->m->host);
        std::unique_ptr<amg_matrix_s> m(new amg_matrix_s());
        m->own.reset(new DevMatrix());
        m->m = m->own.get();
        m->m->build(&c, std::move(h));
        *out = m.release();
    });
}

int amg_par_csr_residual_norm(amg_matrix A, const double* x, const double* b, double* out) {
    return guard([&] {
        AMG_CHECK(A && out, "null argument");
        Context& c = *A->m->ctx;
        set_device(c);
        A->m->ensure_built();
        release_setup_image(*A->m);
        const size_t nb = (size_t)A->m->norm_parts_max(), tmpn = nb / 4096 + 64;
        DevBuf<double> r, buf;
        DevBuf<int> cnt;
        r.alloc((size_t)std::max<int64_t>(A->m->n_rows, 1));
        buf.alloc(nb + tmpn + (size_t)c.host.nranks + 8);
        cnt.alloc(1);
        HIP_CHECK(hipMemsetAsync(cnt.p, 0, sizeof(int), c.stream));
        NormSink ns;
        ns.partial = buf.p;
        ns.tmp = buf.p + nb;
        ns.gathered = ns.tmp + tmpn;
        ns.hist = ns.gathered + c.host.nranks + 2;
        ns.counter = cnt.p;
        par_residual_norm(*A->m, x, b, r.p, ns);
        HIP_CHECK(hipMemcpyAsync(out, ns.hist, sizeof(double), hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipStreamSynchronize(c.stream));
    });
}

int amg_par_csr_destroy(amg_matrix A) {
    return guard([&] {
        if (!A) return;
        AMG_CHECK(A->own != nullptr, "cannot destroy a borrowed level matrix");
        (void)hipSetDevice(A->m->ctx->device);
        (void)hipStreamSynchronize(A->m->ctx->stream);
        delete A;
    });
}

int amg_options_default(int preset, amg_options* o) {
    return guard([&] {
        AMG_CHECK(o, "null argument");
        o->coarsen = AMG_COARSEN_PMIS;
        o->smoother = AMG_SMOOTH_JACOBI;
        o->strong_threshold = 0.25;
        o->jacobi_omega = 2.0 / 3.0;
        o->pre_sweeps = 1;
        o->post_sweeps = 1;
        o->max_levels = 25;
        o->max_coarse = 256;
        o->gs_block = 64;
        o->seed = 0x5EED;
        o->setup_device = 1;
        o->replicate_below = 262144;  // modelled N = 8 cycle
        o->interp = AMG_INTERP_CLASSICAL;
        o->p_max = 4;
        o->drop_tol = 0.0;
        if (preset == AMG_PRESET_RS_JACOBI) {
            o->coarsen = AMG_COARSEN_RS;
        } else if (preset == AMG_PRESET_SA_HYBRID_GS) {
            o->coarsen = AMG_COARSEN_SA;
            o->smoother = AMG_SMOOTH_HYBRID_GS;
            o->strong_threshold = 0.08;
        } else {
            AMG_CHECK(preset == AMG_PRESET_PMIS_JACOBI, "unknown preset");
        }
    });
}

int amg_solver_setup(amg_matrix A, const amg_options* opt, amg_solver* out) {
    return guard([&] {
        AMG_CHECK(A && opt && out, "null argument");
        set_device(*A->m->ctx);
        A->m->ensure_built();
        auto* s = new amg_solver_s();
        try {
            s->s.setup(*A->m, *opt);
        } catch (...) {
            delete s;
            throw;
        }
        *out = s;
    });
}

int amg_solver_num_levels(amg_solver S, int32_t* out) {
    return guard([&] {
        AMG_CHECK(S && out, "null argument");
        *out = (int32_t)S->s.levels.size();
    });
}

int amg_solver_level_info(amg_solver S, int32_t l, amg_level_info* info) {
    return guard([&] {
        AMG_CHECK(S && info, "null argument");
        AMG_CHECK(l >= 0 && l < (int32_t)S->s.levels.size(), "level out of range");
        DevMatrix& A = S->s.Amat(l);
        const HostComm& comm = S->s.ctx->host;
        info->n_global = A.host.n_global_rows;
        info->n_local = A.n_rows;
        info->nnz_local = A.nnz;
        // a replicated coarse level is whole on every rank: its nnz is not summed over ranks
        const int64_t nz = comm.allreduce_sum(A.nnz);
        info->nnz_global = A.replicated ? A.nnz : nz;
        const Level& L = S->s.levels[l];
        info->p_nnz_local = L.P ? L.P->nnz : 0;
        info->r_nnz_local = L.R ? L.R->nnz : 0;
        info->bytes_per_cycle_local = S->s.bytes_per_cycle(l);
        info->stored_bytes_per_cycle_local = S->s.stored_bytes_per_cycle(l);
    });
}

int amg_solver_level_matrix(amg_solver S, int32_t l, int32_t which, amg_matrix* out) {
    return guard([&] {
        AMG_CHECK(S && out, "null argument");
        AMG_CHECK(l >= 0 && l < (int32_t)S->s.levels.size(), "level out of range");
        AMG_CHECK(which >= 0 && which <= 5, "which must be 0 (A), 1 (P), 2 (R), or 3-5 (their cycle-order forms)");
        Solver& s = S->s;
        const bool coarsest = l + 1 == (int32_t)s.levels.size();
        AMG_CHECK(which % 3 == 0 || !coarsest, "no such matrix on this level (the coarsest level has no P/R)");
        DevMatrix* m = which == 0 ? &s.Amat(l)
                     : which == 1 ? s.levels[l].P.get()
                     : which == 2 ? s.levels[l].R.get()
                     : which == 3 ? &s.CA(l) : which == 4 ? &s.CP(l) : &s.CR(l);
        AMG_CHECK(m, "no such matrix on this level (the coarsest level has no P/R)");
        std::unique_ptr<amg_matrix_s> v(new amg_matrix_s());
        v->m = m;
        S->views.push_back(std::move(v));
        *out = S->views.back().get();
    });
}

int amg_solver_level_split(amg_solver S, int32_t l, int32_t* out) {
    return guard([&] {
        AMG_CHECK(S && out, "null argument");
        AMG_CHECK(l >= 0 && l + 1 < (int32_t)S->s.levels.size(), "level has no splitting");
        const auto& sp = S->s.levels[l].split;
        std::copy(sp.begin(), sp.end(), out);
    });
}

int amg_solver_cycle(amg_solver S, double* x, const double* b) {
    return guard([&] {
        AMG_CHECK(S, "null solver");
        set_device(*S->s.ctx);
        S->s.cycle(x, b);
    });
}

int amg_solver_solve(amg_solver S, double* x, const double* b, int32_t max_iter, double tol,
                     double* hist, int32_t* iters) {
    return guard([&] {
        AMG_CHECK(S && hist && iters, "null argument");
        AMG_CHECK(max_iter >= 0, "max_iter must be >= 0");
        set_device(*S->s.ctx);
        const int32_t it = S->s.solve(x, b, max_iter, tol, hist);
        *iters = it;
    });
}

int amg_solver_pcg(amg_solver S, double* x, const double* b, int32_t max_iter, double tol,
                   double* hist, int32_t* iters) {
    return guard([&] {
        AMG_CHECK(S && hist && iters, "null argument");
        set_device(*S->s.ctx);
        *iters = S->s.pcg(x, b, max_iter, tol, hist);
    });
}

int amg_solver_set_graph(amg_solver S, int32_t enable) {
    return guard([&] {
        AMG_CHECK(S, "null solver");
        AMG_CHECK(!enable || S->s.ctx->host.nranks == 1 || S->s.ctx->transport == TR_RCCL,
                  "hipGraph capture needs one rank or the RCCL transport (loopback ranks "
                  "synchronise on the host)");
        // capturing the RCCL groups of a multi-rank cycle: only on the runtime it was
        // validated on
        std::string why;
        if (enable && S->s.ctx->host.nranks > 1) AMG_CHECK(Solver::rccl_graph_allowed(&why), why);
        S->s.use_graph = enable != 0;
        S->s.destroy_graphs();
    });
}

int amg_solver_cycle_timeline(amg_solver S, double* x, const double* b, int32_t reps, int32_t n_max,
                              double* us, char* labels, int32_t label_bytes, int32_t* n_ops, int32_t* in_graph) {
    return guard([&] {
        AMG_CHECK(S && us && labels && n_ops && in_graph, "null argument");
        AMG_CHECK(n_max >= 0 && label_bytes >= 2, "bad buffer sizes");
        set_device(*S->s.ctx);
        std::vector<std::string> lab;
        std::vector<double> t;
        *in_graph = S->s.cycle_timeline(x, b, reps, lab, t);
        *n_ops = (int32_t)t.size();
        for (size_t k = 0; k < t.size() && (int32_t)k < n_max; ++k) {
            us[k] = t[k];
            char* dst = labels + k * (size_t)label_bytes;
            std::snprintf(dst, (size_t)label_bytes, "%s", lab[k].c_str());
        }
    });
}

int amg_solver_get_graph(amg_solver S, int32_t* enabled) {
    return guard([&] {
        AMG_CHECK(S && enabled, "null argument");
        *enabled = S->s.use_graph ? 1 : 0;
    });
}

int amg_solver_destroy(amg_solver S) {
    return guard([&] {
        if (!S) return;
        (void)hipSetDevice(S->s.ctx->device);
        (void)hipStreamSynchronize(S->s.ctx->stream);
        delete S;
    });
}

struct amg_host_hierarchy_s {
    HostComm comm;
    HostCSR A0;
    HostHierarchy H;
};

int amg_host_hierarchy_build(int rank, int nranks, amg_alltoallv_fn exchange, void* user,
                             int64_t n_global, int64_t first_row, int64_t n_local,
                             const int64_t* row_ptr, const int64_t* col_global, const double* val,
                             const amg_options* opt, amg_host_hierarchy* out) {
    return guard([&] {
        AMG_CHECK(opt && out, "null argument");
        AMG_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank/nranks");
        AMG_CHECK(nranks == 1 || exchange, "multi-rank needs a host exchange");
        std::unique_ptr<amg_host_hierarchy_s> h(new amg_host_hierarchy_s());
        h->comm.rank = rank;
        h->comm.nranks = nranks;
        h->comm.fn = exchange;
        h->comm.user = user;
        h->A0 = make_host_csr(h->comm, n_global, first_row, n_local, row_ptr, col_global, val);
        build_hierarchy(h->comm, h->A0, *opt, h->H);
        *out = h.release();
    });
}

static const HostCSR& host_level(amg_host_hierarchy H, int32_t l, int32_t which) {
    AMG_CHECK(H, "null hierarchy");
    AMG_CHECK(l >= 0 && l < (int32_t)H->H.levels.size(), "level out of range");
    AMG_CHECK(which >= 0 && which <= 2, "which must be 0 (A), 1 (P) or 2 (R)");
    AMG_CHECK(which == 0 || l + 1 < (int32_t)H->H.levels.size(), "coarsest level has no P/R");
    return which == 0 ? H->H.A(l) : which == 1 ? H->H.levels[l].P : H->H.levels[l].R;
}

int amg_host_hierarchy_num_levels(amg_host_hierarchy H, int32_t* out) {
    return guard([&] {
        AMG_CHECK(H && out, "null argument");
        *out = (int32_t)H->H.levels.size();
    });
}

int amg_host_hierarchy_level_size(amg_host_hierarchy H, int32_t l, int32_t which, int64_t* s) {
    return guard([&] {
        AMG_CHECK(s, "null argument");
        const HostCSR& M = host_level(H, l, which);
        s[0] = M.n_global_rows;
        s[1] = M.n_global_cols;
        s[2] = M.row_starts[H->comm.rank];
        s[3] = M.nrows();
        s[4] = M.nnz();
    });
}

int amg_host_hierarchy_level_export(amg_host_hierarchy H, int32_t l, int32_t which, int64_t* rp,
                                    int64_t* col, double* val) {
    return guard([&] {
        AMG_CHECK(rp && col && val, "null argument");
        const HostCSR& M = host_level(H, l, which);
        std::copy(M.rp.begin(), M.rp.end(), rp);
        std::copy(M.col.begin(), M.col.end(), col);
        std::copy(M.val.begin(), M.val.end(), val);
    });
}

int amg_host_hierarchy_level_split(amg_host_hierarchy H, int32_t l, int32_t* out) {
    return guard([&] {
        AMG_CHECK(H && out, "null argument");
        AMG_CHECK(l >= 0 && l + 1 < (int32_t)H->H.levels.size(), "level has no splitting");
        const auto& sp = H->H.levels[l].split;
        std::copy(sp.begin(), sp.end(), out);
    });
}

int amg_host_hierarchy_coarse_inverse(amg_host_hierarchy H, double* out) {
    return guard([&] {
        AMG_CHECK(H && out, "null argument");
        std::copy(H->H.coarse_inv.begin(), H->H.coarse_inv.end(), out);
    });
}

int amg_host_hierarchy_destroy(amg_host_hierarchy H) {
    return guard([&] { delete H; });
}

struct amg_host_csr_s {
    HostCSR A;
    int rank = 0;
};

static HostComm host_comm(int rank, int nranks, amg_alltoallv_fn exchange, void* user,
                          bool communicates = true) {
    AMG_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank/nranks");
    AMG_CHECK(nranks == 1 || exchange || !communicates, "multi-rank needs a host exchange");
    HostComm c;
    c.rank = rank, c.nranks = nranks, c.fn = exchange, c.user = user;
    return c;
}

static void host_out(HostCSR&& h, int rank, amg_host_csr* out) {
    std::unique_ptr<amg_host_csr_s> o(new amg_host_csr_s());
    o->A = std::move(h);
    o->rank = rank;
    *out = o.release();
}

int amg_host_csr_graph_laplacian(int rank, int nranks, int64_t nx, int64_t ny, uint64_t seed,
                                 amg_host_csr* out) {
    return guard([&] {
        AMG_CHECK(out, "null argument");
        host_out(graph_laplacian_slab(host_comm(rank, nranks, nullptr, nullptr, false), nx, ny, seed), rank, out);
    });
}

// the stencil generators need no communication either
int amg_host_csr_stencil(int rank, int nranks, int kind, int64_t nx, int64_t ny, int64_t nz, int64_t bx,
                         int64_t by, int64_t bz, const double* eps3, amg_host_csr* out) {
    return guard([&] {
        AMG_CHECK(out, "null argument");
        AMG_CHECK(kind == AMG_STENCIL_5PT || kind == AMG_STENCIL_7PT || kind == AMG_STENCIL_27PT,
                  "unknown stencil");
        host_out(stencil_boxes(host_comm(rank, nranks, nullptr, nullptr, false), kind, nx, ny, nz, bx, by, bz, eps3),
                 rank, out);
    });
}

// the reader needs no communication (even partition from the file header)
int amg_host_csr_read(int rank, int nranks, const char* path, amg_host_csr* out) {
    return guard([&] {
        AMG_CHECK(path && out, "null argument");
        host_out(read_par_matrix(host_comm(rank, nranks, nullptr, nullptr, false), path), rank, out);
    });
}

int amg_host_csr_write(int rank, int nranks, amg_alltoallv_fn exchange, void* user, amg_host_csr A,
                       const char* path) {
    return guard([&] {
        AMG_CHECK(A && path, "null argument");
        write_par_matrix(host_comm(rank, nranks, exchange, user), A->A, path);
    });
}

int amg_host_csr_reorder(int rank, int nranks, amg_alltoallv_fn exchange, void* user, amg_host_csr A,
                         int method, amg_host_csr* out, int64_t* new_to_old_local) {
    return guard([&] {
        AMG_CHECK(A && out && new_to_old_local, "null argument");
        AMG_CHECK(method == AMG_REORDER_RCM, "unknown reorder method");
        std::vector<int64_t> n2o;
        HostCSR h = reorder_rcm(host_comm(rank, nranks, exchange, user), A->A, n2o);
        std::copy(n2o.begin(), n2o.end(), new_to_old_local);
        host_out(std::move(h), rank, out);
    });
}

int amg_host_csr_size(amg_host_csr A, int64_t* s) {
    return guard([&] {
        AMG_CHECK(A && s, "null argument");
        const HostCSR& h = A->A;
        s[0] = h.n_global_rows, s[1] = h.n_global_cols;
        s[2] = h.row_starts[A->rank];
        s[3] = h.nrows(), s[4] = h.nnz();
    });
}

int amg_host_csr_export(amg_host_csr A, int64_t* row_ptr, int64_t* col_global, double* val) {
    return guard([&] {
        AMG_CHECK(A && row_ptr && col_global && val, "null argument");
        std::copy(A->A.rp.begin(), A->A.rp.end(), row_ptr);
        std::copy(A->A.col.begin(), A->A.col.end(), col_global);
        std::copy(A->A.val.begin(), A->A.val.end(), val);
    });
}

int amg_host_csr_destroy(amg_host_csr A) {
    return guard([&] { delete A; });
}

int amg_vector_copy(amg_context ctx, int64_t n, const double* src, double* dst) {
    return guard([&] {
        AMG_CHECK(ctx && n >= 0, "bad argument");
        AMG_CHECK(n == 0 || (src && dst), "null vector");
        set_device(ctx->c);
        launch_copy(ctx->c.stream, n, src, dst);
    });
}

int amg_vector_read(amg_context ctx, int64_t n, const double* src, double* partials, int64_t n_partials) {
    return guard([&] {
        AMG_CHECK(ctx && n >= 0, "bad argument");
        AMG_CHECK(n == 0 || (src && partials), "null vector");
        AMG_CHECK(n_partials >= read_partials(n), "read: too few partial slots");
        set_device(ctx->c);
        launch_read(ctx->c.stream, n, src, partials);
    });
}

int amg_device_malloc(amg_context ctx, int64_t bytes, void** out) {
    return guard([&] {
        AMG_CHECK(ctx && out && bytes >= 0, "bad argument");
        set_device(ctx->c);
        *out = nullptr;
        if (bytes == 0) return;
        const hipError_t e = hipMalloc(out, (size_t)bytes);
        if (e == hipErrorOutOfMemory) {
            (void)hipGetLastError();
            throw Error(AMG_ERR_NOMEM, "hipMalloc of " + std::to_string(bytes) + " bytes: out of device memory");
        }
        HIP_CHECK(e);
    });
}

int amg_device_free(amg_context ctx, void* p) {
    return guard([&] {
        AMG_CHECK(ctx, "null context");
        if (!p) return;
        set_device(ctx->c);
        HIP_CHECK(hipStreamSynchronize(ctx->c.stream));
        HIP_CHECK(hipFree(p));
    });
}

int amg_memcpy(amg_context ctx, void* dst, const void* src, int64_t bytes) {
    return guard([&] {
        AMG_CHECK(ctx && bytes >= 0, "bad argument");
        if (bytes == 0) return;
        AMG_CHECK(dst && src, "null pointer");
        set_device(ctx->c);
        HIP_CHECK(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDefault, ctx->c.stream));
        HIP_CHECK(hipStreamSynchronize(ctx->c.stream));
    });
}

int amg_memset_async(amg_context ctx, void* p, int value, int64_t bytes) {
    return guard([&] {
        AMG_CHECK(ctx && bytes >= 0, "bad argument");
        if (bytes == 0) return;
        AMG_CHECK(p, "null pointer");
        set_device(ctx->c);
        HIP_CHECK(hipMemsetAsync(p, value, (size_t)bytes, ctx->c.stream));
    });
}

struct amg_event_s {
    amg_context ctx = nullptr;
    hipEvent_t e = nullptr;
};

int amg_event_create(amg_context ctx, amg_event* out) {
    return guard([&] {
        AMG_CHECK(ctx && out, "null argument");
        set_device(ctx->c);
        std::unique_ptr<amg_event_s> ev(new amg_event_s());
        ev->ctx = ctx;
        HIP_CHECK(hipEventCreate(&ev->e));
        *out = ev.release();
    });
}

int amg_event_record(amg_event e) {
    return guard([&] {
        AMG_CHECK(e, "null event");
        set_device(e->ctx->c);
        HIP_CHECK(hipEventRecord(e->e, e->ctx->c.stream));
    });
}

int amg_event_elapsed_ms(amg_event start, amg_event end, float* ms) {
    return guard([&] {
        AMG_CHECK(start && end && ms, "null argument");
        set_device(end->ctx->c);
        HIP_CHECK(hipEventSynchronize(end->e));
        HIP_CHECK(hipEventElapsedTime(ms, start->e, end->e));
    });
}

int amg_event_destroy(amg_event e) {
    return guard([&] {
        if (!e) return;
        (void)hipEventDestroy(e->e);
        delete e;
    });
}

int amg_vector_uniform(amg_context ctx, int64_t n, int64_t first_gid, uint64_t seed, double* out) {
    return guard([&] {
        AMG_CHECK(ctx && (out || n == 0), "null argument");
        set_device(ctx->c);
        launch_uniform(ctx->c.stream, n, first_gid, seed, out);
    });
}

}  // extern "C"
