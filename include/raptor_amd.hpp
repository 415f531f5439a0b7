// raptor_amd.hpp -- header-only C++ facade over the C-ABI of raptor_amd.h.
//
// BASELINE.json:5 asks for "the ParMultilevel/ParCSRMatrix API surface ... C++ host code calls
// HIP through a thin extern-"C" layer" ("C++ facade: ParCSRMatrix ... and
// ParMultilevel ... Below it, a thin extern "C" C-ABI").  These classes are that facade: RAII
// owners of the opaque handles, C-ABI error codes turned into raptor_amd::Error on the C++ side only
// (no exception ever crosses the C-ABI itself).  Vectors are device pointers (hipMalloc) of
// the rank-local length, as in the C-ABI; all work runs on the context's HIP stream.
//
//   raptor_amd::Context ctx(0);
//   raptor_amd::ParCSRMatrix A = raptor_amd::ParCSRMatrix::stencil(ctx, AMG_STENCIL_7PT, 256, 256, 256);
//   raptor_amd::ParMultilevel ml(A, raptor_amd::ParMultilevel::options(AMG_PRESET_PMIS_JACOBI));
//   std::vector<double> hist = ml.solve(d_x, d_b, 20);
#ifndef RAPTOR_AMD_HPP
#define RAPTOR_AMD_HPP

#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "raptor_amd.h"

// The facade has its own namespace: the library's internals are namespace amg, and although
// libraptor_amd.so exports only the amg_* C entry points (linker version script), distinct
// names keep a caller's inline copies of these classes from ever meeting internal symbols.
namespace raptor_amd {

// a C-ABI error code and amg_last_error() of the failing call
class Error : public std::runtime_error {
public:
    Error(int code, const std::string& msg) : std::runtime_error(msg), code_(code) {}
    int code() const noexcept { return code_; }

private:
    int code_;
};

inline void check(int rc) {
    if (rc != AMG_OK) throw Error(rc, std::string("raptor_amd: ") + amg_last_error());
}

// one GPU / rank (amg_context_*)
class Context {
public:
    explicit Context(int device = 0, void* hip_stream = nullptr) { check(amg_context_create(device, hip_stream, &h_)); }
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;
    Context(Context&& o) noexcept : h_(std::exchange(o.h_, nullptr)) {}
    ~Context() {
        if (h_) amg_context_destroy(h_);
    }
    // multi-rank: RCCL id from rank 0's rccl_unique_id(), host exchange for setup metadata
    void set_comm(int rank, int nranks, const void* rccl_id128, amg_alltoallv_fn exchange, void* user) {
        check(amg_context_set_comm(h_, rank, nranks, rccl_id128, exchange, user));
    }
    static std::vector<char> rccl_unique_id() {
        std::vector<char> id(128);
        check(amg_rccl_unique_id(id.data()));
        return id;
    }
    void* stream() const {
        void* s = nullptr;
        check(amg_context_stream(h_, &s));
        return s;
    }
    void synchronize() const { check(amg_context_synchronize(h_)); }
    // out[i] = uniform(-1, 1) of splitmix64(seed, first_gid + i), on the device
    void uniform(int64_t n, int64_t first_gid, uint64_t seed, double* d_out) const {
        check(amg_vector_uniform(h_, n, first_gid, seed, d_out));
    }
    amg_context handle() const { return h_; }

private:
    amg_context h_ = nullptr;
};

// row-partitioned CSR on the GPU (RAPtor ParCSRMatrix analogue)
class ParCSRMatrix {
public:
    // rank-local rows [first_row, first_row + n_local) of an n_global x n_global matrix
    // (global column ids).  Collective.
    ParCSRMatrix(Context& ctx, int64_t n_global, int64_t first_row, int64_t n_local, const int64_t* row_ptr,
                 const int64_t* col_global, const double* val) {
        check(amg_par_csr_create(ctx.handle(), n_global, first_row, n_local, row_ptr, col_global, val, &h_));
    }
    // this rank's slab of a model problem (AMG_STENCIL_5PT / 7PT / 27PT).  Collective.
    static ParCSRMatrix stencil(Context& ctx, int kind, int64_t nx, int64_t ny, int64_t nz,
                                const double* eps3 = nullptr) {
        amg_matrix h = nullptr;
        check(amg_par_stencil_create(ctx.handle(), kind, nx, ny, nz, eps3, &h));
        return ParCSRMatrix(h, true);
    }
    // Matrix Market or binary CSR, even row partition.  Collective.
    static ParCSRMatrix read(Context& ctx, const std::string& path) {
        amg_matrix h = nullptr;
        check(amg_par_csr_read(ctx.handle(), path.c_str(), &h));
        return ParCSRMatrix(h, true);
    }
    ParCSRMatrix(const ParCSRMatrix&) = delete;
    ParCSRMatrix& operator=(const ParCSRMatrix&) = delete;
    ParCSRMatrix(ParCSRMatrix&& o) noexcept : h_(std::exchange(o.h_, nullptr)), own_(o.own_) {}
    ~ParCSRMatrix() {
        if (h_ && own_) amg_par_csr_destroy(h_);
    }

    amg_matrix_info info() const {
        amg_matrix_info i{};
        check(amg_par_csr_info(h_, &i));
        return i;
    }
    int64_t local_rows() const { return info().n_local_rows; }
    int64_t first_row() const { return info().first_row; }
    int64_t global_rows() const { return info().n_global_rows; }
    void set_format(int32_t format) { check(amg_par_csr_set_format(h_, format)); }

    // ParCSRMatrix::mult and the level kernels (device pointers, local length)
    void mult(const double* x, double* y) const { check(amg_par_csr_mult(h_, x, y)); }
    void mult_add(const double* x, double* y) const { check(amg_par_csr_mult_add(h_, x, y)); }
    void residual(const double* x, const double* b, double* r) const { check(amg_par_csr_residual(h_, x, b, r)); }
    void jacobi(const double* x, const double* b, double* x_out, double omega = 2.0 / 3.0) const {
        check(amg_par_csr_jacobi(h_, x, b, x_out, omega));
    }
    void hybrid_gs(const double* x, const double* b, double* x_out, int64_t block = 64, bool backward = false) const {
        check(backward ? amg_par_csr_hybrid_gs_backward(h_, x, b, x_out, block)
                       : amg_par_csr_hybrid_gs(h_, x, b, x_out, block));
    }
    double residual_norm(const double* x, const double* b) const {
        double v = 0.0;
        check(amg_par_csr_residual_norm(h_, x, b, &v));
        return v;
    }
    // C = this * B (Galerkin SpGEMM kernel).  Collective.
    ParCSRMatrix matmat(const ParCSRMatrix& B) const {
        amg_matrix c = nullptr;
        check(amg_par_csr_matmat(h_, B.h_, &c));
        return ParCSRMatrix(c, true);
    }
    amg_matrix handle() const { return h_; }

private:
    friend class ParMultilevel;
    ParCSRMatrix(amg_matrix h, bool own) : h_(h), own_(own) {}
    amg_matrix h_ = nullptr;
    bool own_ = true;
};

// AMG hierarchy + V-cycle (RAPtor ParMultilevel analogue)
class ParMultilevel {
public:
    static amg_options options(int preset) {
        amg_options o{};
        check(amg_options_default(preset, &o));
        return o;
    }
    // ParMultilevel::setup(A); A must outlive the solver.  Collective.
    ParMultilevel(const ParCSRMatrix& A, const amg_options& opt) { check(amg_solver_setup(A.handle(), &opt, &h_)); }
    ParMultilevel(const ParMultilevel&) = delete;
    ParMultilevel& operator=(const ParMultilevel&) = delete;
    ParMultilevel(ParMultilevel&& o) noexcept : h_(std::exchange(o.h_, nullptr)) {}
    ~ParMultilevel() {
        if (h_) amg_solver_destroy(h_);
    }

    int num_levels() const {
        int32_t n = 0;
        check(amg_solver_num_levels(h_, &n));
        return n;
    }
    amg_level_info level_info(int level) const {
        amg_level_info i{};
        check(amg_solver_level_info(h_, level, &i));
        return i;
    }
    // borrowed view of A_l / P_l / R_l (which = 0 / 1 / 2), valid while the solver lives
    ParCSRMatrix level_matrix(int level, int which) const {
        amg_matrix m = nullptr;
        check(amg_solver_level_matrix(h_, level, which, &m));
        return ParCSRMatrix(m, false);
    }
    std::vector<int32_t> level_split(int level) const {
        std::vector<int32_t> s((size_t)level_info(level).n_local);
        check(amg_solver_level_split(h_, level, s.data()));
        return s;
    }
    void set_graph(bool on) { check(amg_solver_set_graph(h_, on ? 1 : 0)); }
    bool graph() const {
        int32_t v = 0;
        check(amg_solver_get_graph(h_, &v));
        return v != 0;
    }
    // ParMultilevel::cycle: x <- cycle(x, b)
    void cycle(double* x, const double* b) { check(amg_solver_cycle(h_, x, b)); }
    // ParMultilevel::solve: the residual history ||b - A x_k||, k = 0 .. iterations
    std::vector<double> solve(double* x, const double* b, int max_iter, double tol = 0.0) {
        std::vector<double> hist((size_t)max_iter + 1);
        int32_t it = 0;
        check(amg_solver_solve(h_, x, b, max_iter, tol, hist.data(), &it));
        hist.resize((size_t)it + 1);
        return hist;
    }
    // conjugate gradients preconditioned by one V-cycle per iteration
    std::vector<double> pcg(double* x, const double* b, int max_iter, double tol = 0.0) {
        std::vector<double> hist((size_t)max_iter + 1);
        int32_t it = 0;
        check(amg_solver_pcg(h_, x, b, max_iter, tol, hist.data(), &it));
        hist.resize((size_t)it + 1);
        return hist;
    }
    amg_solver handle() const { return h_; }

private:
    amg_solver h_ = nullptr;
};

}  // namespace raptor_amd

#endif  // RAPTOR_AMD_HPP
