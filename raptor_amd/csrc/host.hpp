// host.hpp -- host-side (CPU) part of the product: row-partitioned CSR, the setup-time
// exchange layer and the AMG setup algorithms.
//
// Everything here works on the rank-local rows of a row-partitioned matrix with GLOBAL
// column ids (int64), sorted ascending per row.  Keeping global column order everywhere
// makes every row sum partition-independent: 1, 2, 4 or 8 ranks produce bit-identical
// hierarchies (integer AND fp64), and the same bits as the serial oracle.
//
// The setup exchange goes through HostComm::alltoallv (a C callback supplied over the
// C-ABI, torch.distributed/gloo in the Python host layer); the solve-time data path never
// touches it (RCCL, see device.hpp).
#pragma once
#include <cmath>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <type_traits>
#include <utility>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/raptor_amd.h"
#include <rocprofiler-sdk-roctx/roctx.h>

namespace amg {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// OpenMP teams the library's host loops start from this thread sleep as soon as a parallel
// region ends (kmp_set_blocktime(0) for this thread, once; KMP_BLOCKTIME in the environment
// wins): libomp's default keeps them spinning for 200 ms, and on a CPU-quota'd host two
// spinning teams -- the setup thread's and the format worker's -- exhausted the quota and
// stalled the launching thread for 5-10 ms inside timed V-cycles (profiles/r3i_cycle_gaps.txt).
// omp_quiet_thread() sets it for good on the library's own threads (the format worker);
// OmpQuiet, held by every C-ABI entry, sets it on the caller's thread for the call and
// restores the caller's value on return, so OpenMP teams the host application forks from
// that thread keep their own blocktime.
void omp_quiet_thread();
struct OmpQuiet {
    int saved = -1;
    OmpQuiet();
    ~OmpQuiet();
    OmpQuiet(const OmpQuiet&) = delete;
    OmpQuiet& operator=(const OmpQuiet&) = delete;
};
#define AMG_CHECK(cond, msg)                                                              \
    do {                                                                                  \
        if (!(cond)) throw ::amg::Error(AMG_ERR_INVALID, std::string(msg));               \
    } while (0)
#define AMG_ASSERT(cond)                                                                  \
    do {                                                                                  \
        if (!(cond))                                                                      \
            throw ::amg::Error(AMG_ERR_INTERNAL, std::string("invariant failed: ") + #cond \
                                                     + " at " + __FILE__ + ":" +           \
                                                     std::to_string(__LINE__));           \
    } while (0)

// ---------------------------------------------------------------------------------
// Setup-time communicator: rank/nranks + an all-to-all-v byte callback.
// ---------------------------------------------------------------------------------
struct HostComm {
    int rank = 0, nranks = 1;
    amg_alltoallv_fn fn = nullptr;
    void* user = nullptr;

    void alltoallv(const void* send, const std::vector<int64_t>& sbytes, void* recv,
                   const std::vector<int64_t>& rbytes) const;
    // every rank sends counts[r] to rank r; returns what each rank sent to us
    std::vector<int64_t> alltoall_counts(const std::vector<int64_t>& counts) const;
    // typed variable all-to-all: send[r] goes to rank r
    template <class T>
    std::vector<std::vector<T>> exchange(const std::vector<std::vector<T>>& send) const;
    std::vector<int64_t> allgather(int64_t v) const;
    std::vector<double> allgather(double v) const;
    int64_t allreduce_sum(int64_t v) const;
    double allreduce_max(double v) const;
};

// ---------------------------------------------------------------------------------
// Rank-local rows of a row-partitioned CSR matrix (ParCSRMatrix host image, row a1).
// ---------------------------------------------------------------------------------
// std::allocator whose resize(n) leaves new scalars uninitialised (default-init): the
// nonzero arrays of a HostCSR are written right after they are sized (device downloads,
// parallel fills), so value-initialising them first would be a serial pass over GBs
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = DefaultInitAlloc<U>;
    };
    DefaultInitAlloc() = default;
    template <class U>
    DefaultInitAlloc(const DefaultInitAlloc<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept(std::is_nothrow_default_constructible<U>::value) {
        ::new ((void*)p) U;
    }
    template <class U, class... Args>
    void construct(U* p, Args&&... args) {
        ::new ((void*)p) U(std::forward<Args>(args)...);
    }
};
template <class T>
using hvec = std::vector<T, DefaultInitAlloc<T>>;

struct HostCSR {
    int64_t n_global_rows = 0, n_global_cols = 0;
    std::vector<int64_t> row_starts;  // nranks+1: global row partition
    std::vector<int64_t> col_starts;  // nranks+1: partition of the column space (x owners)
    std::vector<int64_t> rp;          // n_local+1
    hvec<int64_t> col;                // global column ids, ascending per row
    hvec<double> val;

    int64_t first_row(int rank) const { return row_starts[rank]; }
    int64_t n_local(int rank) const { return row_starts[rank + 1] - row_starts[rank]; }
    int64_t nrows() const { return (int64_t)rp.size() - 1; }
    int64_t nnz() const { return rp.empty() ? 0 : rp.back(); }
};

// owner of global id g under a contiguous partition
int owner_of(const std::vector<int64_t>& starts, int64_t g);

// ---------------------------------------------------------------------------------
// Halo plan (ParComm): which off-process ids this rank receives and which local ids it
// sends.  Built collectively from the set of needed global ids (row a11).
// ---------------------------------------------------------------------------------
struct HaloPlan {
    std::vector<int64_t> halo_gid;     // sorted ascending (=> grouped by owner)
    std::vector<int> recv_procs;       // owners, ascending
    std::vector<int64_t> recv_ptr;     // recv_procs.size()+1 into halo_gid
    std::vector<int> send_procs;       // destinations, ascending
    std::vector<int64_t> send_ptr;     // send_procs.size()+1 into send_idx
    std::vector<int64_t> send_idx;     // local indices (gid - owner start)

    int64_t n_halo() const { return (int64_t)halo_gid.size(); }
    // index of gid in halo_gid (binary search), -1 if absent
    int64_t find(int64_t gid) const;

    template <class T>
    void forward(const HostComm& comm, const T* local, T* halo) const;
};

HaloPlan build_halo_plan(const HostComm& comm, const std::vector<int64_t>& starts,
                         std::vector<int64_t> needed_gids);
// halo plan for the off-process columns of A (columns partitioned by A.col_starts)
HaloPlan halo_plan_for_cols(const HostComm& comm, const HostCSR& A);

// ghost rows of B for plan.halo_gid (B rows partitioned like plan's partition)
struct GhostRows {
    std::vector<int64_t> rp, col;
    std::vector<double> val;
};
GhostRows fetch_rows(const HostComm& comm, const HaloPlan& plan, const HostCSR& B);

// ---------------------------------------------------------------------------------
// Setup algorithms (identical definitions to the oracle).
// ---------------------------------------------------------------------------------
HostCSR transpose(const HostComm& comm, const HostCSR& P);
HostCSR spgemm(const HostComm& comm, const HostCSR& A, const HostCSR& B);
std::vector<double> diagonal(const HostComm& comm, const HostCSR& A);  // local rows
// coarse-operator drop tolerance (oracle orc_sparsify): off-diagonals below
// tau sqrt(|a_ii a_jj|) are added to the diagonal in row order
HostCSR sparsify(const HostComm& comm, const HostCSR& A, double tau);
HostCSR strength_classical(const HostComm& comm, const HostCSR& A, double theta);
HostCSR strength_symmetric(const HostComm& comm, const HostCSR& A, double theta);
std::vector<int32_t> rs_split(const HostComm& comm, const HostCSR& S);
std::vector<int32_t> pmis_split(const HostComm& comm, const HostCSR& S, uint64_t seed);
HostCSR interp_classical(const HostComm& comm, const HostCSR& A, const HostCSR& S,
                         const std::vector<int32_t>& cf);
HostCSR interp_ext_i(const HostComm& comm, const HostCSR& A, const HostCSR& S, const std::vector<int32_t>& cf,
                     int p_max);
// returns global aggregate id per local row; *n_agg_global receives the count
std::vector<int64_t> mis2_aggregate(const HostComm& comm, const HostCSR& S, uint64_t seed,
                                    int64_t* n_agg_global, std::vector<int64_t>* agg_starts);
// SA: the signed strength test; theta of level l (theta_0 * 0.75 per level,
// rounded per level); the filtered operator; rho(D^-1 A_F) by kSaRhoIters max-norm power
// steps; P = T - (4/3 rho) (1/a_ii) A_F T
constexpr int kSaRhoIters = 10;
inline bool sa_strong(double aij, double di, double dj, double theta) {
    return -aij >= theta * std::sqrt(std::fabs(di * dj));
}
inline double sa_theta(double theta0, int level) {
    double t = theta0;
    for (int l = 0; l < level; ++l) t = t * 0.75;
    return t;
}
HostCSR sa_filter(const HostComm& comm, const HostCSR& A, double theta);
HostCSR sa_prolongator(const HostComm& comm, const HostCSR& A, const std::vector<int64_t>& agg,
                       int64_t n_agg, const std::vector<int64_t>& agg_starts, double theta, uint64_t seed);
// every rank receives the whole matrix (rows in global order); the result is a one-rank
// matrix (row_starts {0, n}, col_starts {0, n_cols}) for replicated coarse levels
HostCSR gather_global(const HostComm& comm, const HostCSR& M);
// Gauss-Jordan inverse of the whole (gathered) coarsest matrix, row-major n*n
std::vector<double> dense_inverse_gathered(const HostComm& comm, const HostCSR& A);

// model problems: this rank's slab (rows split evenly by planes)
HostCSR stencil_slab(const HostComm& comm, int kind, int64_t nx, int64_t ny, int64_t nz,
                     const double* eps3);
// the same problem numbered box by box (bx x by x bz boxes, ranks own contiguous box ranges)
HostCSR stencil_boxes(const HostComm& comm, int kind, int64_t nx, int64_t ny, int64_t nz, int64_t bx,
                      int64_t by, int64_t bz, const double* eps3);

// Whole hierarchy on the host (rows a7-a10): level l holds A_l (l >= 1), P_l, R_l and the
// integer splitting; the coarsest level's gathered dense inverse.  Same stopping rule and
// per-level seeds/thresholds as the oracle.
struct HostLevel {
    HostCSR A;  // empty for level 0 (the caller's matrix)
    HostCSR P, R;
    std::vector<int32_t> split;
};
struct HostHierarchy {
    // a deque: levels keep their addresses as the hierarchy grows (Solver::setup builds a
    // level's device formats on a worker thread while the next level is coarsened)
    std::deque<HostLevel> levels;
    std::vector<double> coarse_inv;  // row-major n_c x n_c
    const HostCSR* A0 = nullptr;
    const HostCSR& A(size_t l) const { return l == 0 ? *A0 : levels[l].A; }
};
// Galerkin SpGEMM hook: C = A * B for the local rows (the device SpGEMM of spgemm.hip when
// the hierarchy is built for a GPU solver; the host spgemm() otherwise).  Same results.
using SpgemmFn = std::function<HostCSR(const HostCSR&, const HostCSR&)>;
// Device hooks for the rest of a level's setup (setup_device.hip, single rank): P and the
// integer split of level l, and R = P^T.  Each returns false where it does not apply (the
// host algorithms below run instead); results are identical either way.
using LevelSetupFn = std::function<bool(int level, const HostCSR& A, HostCSR& P, std::vector<int32_t>& split)>;
using TransposeFn = std::function<bool(const HostCSR& P, HostCSR& R)>;
// called once level l is final (its P, R and the coarse operator A_{l+1}); none of the three
// is written again by build_hierarchy
using LevelDoneFn = std::function<void(int level)>;
// the whole Galerkin product R (A P) in one hook (the device keeps A P between the two
// products); when absent, two SpgemmFn / spgemm() calls.  It returns the level's coarse
// operator with opt.drop_tol already applied (sparsify)
using RapFn = std::function<HostCSR(const HostCSR& R, const HostCSR& A, const HostCSR& P)>;
void build_hierarchy(const HostComm& comm, const HostCSR& A0, const amg_options& opt,
                     HostHierarchy& H, const SpgemmFn& galerkin = nullptr,
                     const LevelSetupFn& level_fn = nullptr, const TransposeFn& transpose_fn = nullptr,
                     const LevelDoneFn& level_done = nullptr, const RapFn& rap_fn = nullptr);

uint64_t mix64(uint64_t z);
uint32_t hash32(int64_t gid, uint64_t seed);

// Setup phase timing: with AMG_TIMING=1 in the environment, rank 0 prints
// "[amg] <label> <ms>" to stderr for every phase (host wall clock).
// roctx range for the lifetime of the object (rocprofv3 --marker-trace shows the setup phases,
// solves and cycle replays on the host timeline)
struct RoctxRange {
    explicit RoctxRange(const char* name) { roctxRangePushA(name); }
    ~RoctxRange() { roctxRangePop(); }
    RoctxRange(const RoctxRange&) = delete;
    RoctxRange& operator=(const RoctxRange&) = delete;
};

struct PhaseTimer {
    static bool enabled();
    explicit PhaseTimer(const HostComm& comm);
    void lap(const std::string& label);  // time since construction / the previous lap
    int rank;
    double t0;
};

// ---- inputs beyond the stencils (host_io.cpp, row f2) ----------------------------
// seeded unstructured graph Laplacian (G3_circuit substitute), even row partition
HostCSR graph_laplacian_slab(const HostComm& comm, int64_t nx, int64_t ny, uint64_t seed);
// Matrix Market (coordinate real/integer/pattern; general/symmetric/skew) or binary CSR
// (magic "RAMGCSR1"), detected from the first bytes; this rank's rows of an even partition
HostCSR read_par_matrix(const HostComm& comm, const std::string& path);
// collective binary CSR writer (every rank writes its rows at their global offsets)
void write_par_matrix(const HostComm& comm, const HostCSR& A, const std::string& path);
// reverse Cuthill-McKee order (new_to_old) of a whole square matrix
std::vector<int64_t> rcm_order(const HostCSR& full);
// P A P^T by RCM; the result uses the even row partition; new_to_old_local[i] is the
// old global id of the new local row i
HostCSR reorder_rcm(const HostComm& comm, const HostCSR& A, std::vector<int64_t>& new_to_old_local);

}  // namespace amg
