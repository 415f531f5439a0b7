// multilevel.hip -- ParMultilevel: hierarchy setup (host, distributed) and the GPU V-cycle.
// SURVEY.md 8a rows a6-a10.  The cycle mirrors oracle/amg_oracle.c cycle_rec() operation
// for operation, so the iterates are bit-identical to the oracle's.
#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <mutex>
#include <thread>

#include "device.hpp"

namespace amg {

namespace {


// One worker thread that builds device formats (DevMatrix::build_view: host C++ format
// builds + uploads) in FIFO order while the setup thread coarsens the next level: level l's
// P and R and A_{l+1} are final once build_hierarchy reports level l done.  One rank only:
// a multi-rank build_view runs host collectives (the halo plan), which must not interleave
// with the hierarchy's.
class FormatWorker {
  public:
    explicit FormatWorker(int device) : th_([this, device] { run(device); }) {}
    ~FormatWorker() {
        if (th_.joinable()) stop();
    }
    void push(std::function<void()> job) {
        {
            std::lock_guard<std::mutex> g(mu_);
            q_.push_back(std::move(job));
        }
        cv_.notify_one();
    }
    // waits for every queued job; rethrows the first failure
    void finish() {
        stop();
        if (err_) std::rethrow_exception(err_);
    }

  private:
    void stop() {
        {
            std::lock_guard<std::mutex> g(mu_);
            done_ = true;
        }
        cv_.notify_one();
        th_.join();
    }
    void run(int device) {
        const hipError_t e = hipSetDevice(device);
        omp_quiet_thread();
        for (;;) {
            std::function<void()> job;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [this] { return done_ || !q_.empty(); });
                if (q_.empty()) return;
                job = std::move(q_.front());
                q_.pop_front();
            }
            if (err_) continue;  // after a failure: drain, report the first one
            try {
                HIP_CHECK(e);
                job();
            } catch (...) {
                err_ = std::current_exception();
            }
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
    bool done_ = false;
    std::exception_ptr err_;
    std::thread th_;
};

}  // namespace

// Cycle order.  A Jacobi-smoothed level's kernels form each row's products
// and sum them in the row's stored order; neither depends on where the row sits or on the
// numbering of its columns.  So the cycle may run a level's points in any order Pi, as long as
// every operator touching the level carries the same Pi: A_l (rows and columns), P_l (rows),
// R_l (columns), R_{l-1} (rows) and P_{l-1} (columns).  Each row keeps its entries in the
// hierarchy's order, so every sum is the hierarchy's, bit for bit.  The order chosen is 8x8x8
// bricks of the fine grid: a level point sits at the fine point of its restriction row's
// first local column (for PMIS / RS its C point; for SA a fine point at its aggregate).  A
// block of consecutive rows is then a compact piece of space, and its x tile holds fewer
// lines than a block of a lexicographic slab (tests/analysis_brick_cut.py).  Grid-built
// operators (stencil constructors: each rank knows its box or slab), Jacobi levels only
// (hybrid-GS chunks are defined on the hierarchy's order), distributed levels only (not the
// coarsest, not replicated ones).  On N ranks each rank orders its own points; its send lists
// index its vectors through that order (DevMatrix::send_map), halo columns keep their global
// ids.  AMG_CYCLE_ORDER=0 turns it off.
namespace {
// rows: new row -> old row, cols: old local column -> new (either empty: identity); halo
// columns (other ranks' points) keep their global ids
HostCSR permuted_csr(const HostCSR& M, int rank, const std::vector<int64_t>& rows, const std::vector<int64_t>& cols) {
    const int64_t clo = M.col_starts[rank], chi = M.col_starts[rank + 1];
    HostCSR B;
    B.n_global_rows = M.n_global_rows;
    B.n_global_cols = M.n_global_cols;
    B.row_starts = M.row_starts;
    B.col_starts = M.col_starts;
    const int64_t n = M.nrows();
    B.rp.assign((size_t)n + 1, 0);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        const int64_t o = rows.empty() ? i : rows[i];
        B.rp[i + 1] = M.rp[o + 1] - M.rp[o];
    }
    for (int64_t i = 0; i < n; ++i) B.rp[i + 1] += B.rp[i];
    B.col.resize((size_t)M.nnz());
    B.val.resize((size_t)M.nnz());
#pragma omp parallel for schedule(dynamic, 4096)
    for (int64_t i = 0; i < n; ++i) {
        const int64_t o = rows.empty() ? i : rows[i];
        int64_t d = B.rp[i];
        for (int64_t k = M.rp[o]; k < M.rp[o + 1]; ++k, ++d) {
            const int64_t c = M.col[k];
            B.col[d] = cols.empty() || c < clo || c >= chi ? c : clo + cols[c - clo];
            B.val[d] = M.val[k];
        }
    }
    return B;
}

// the brick orders of a hierarchy's levels, one level at a time as the setup produces them
struct CycleOrder {
    static constexpr int64_t kB = 8, kMinRows = 4096;
    bool open = false;                             // the next level may still be permuted
    int64_t g[3] = {0, 0, 0};                      // level-0 local grid extents
    std::vector<char> on;                          // per level: permuted (the same on every rank)
    std::vector<std::vector<int64_t>> perm, inv;   // this rank's points: new -> old, old -> new
    std::vector<int64_t> at;                       // fine point of each point of the last level seen

    void init(const DevMatrix& A, const amg_options& opt, const HostComm& comm, size_t maxl) {
        const char* e = std::getenv("AMG_CYCLE_ORDER");  // read per setup (tests compare both)
        std::copy(A.grid_local, A.grid_local + 3, g);
        const bool mine = g[0] > 0 && g[1] > 0 && g[0] * g[1] * std::max<int64_t>(g[2], 1) >= A.n_rows;
        open = !(e && std::atoi(e) == 0) && opt.smoother == AMG_SMOOTH_JACOBI &&
               comm.allreduce_sum(mine ? 0 : 1) == 0;  // every rank's operator came from a grid
        on.assign(maxl, 0);
        perm.assign(maxl, {});
        inv.assign(maxl, {});
        if (!open) return;
        at.resize((size_t)A.n_rows);
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < A.n_rows; ++i) at[i] = i;
    }
    bool any(size_t l) const { return l < on.size() && on[l]; }
    // level l + 1's order, from R_l (its rows are level l + 1's points, ascending fine columns)
    void next(size_t l, const HostCSR& R, const amg_options& opt, const HostComm& comm) {
        if (!open) return;
        const int64_t n = R.nrows(), ng = R.n_global_rows;
        const int64_t flo = R.col_starts[comm.rank], fhi = R.col_starts[comm.rank + 1];
        // large enough, not the coarsest level (dense-solved in the hierarchy's order) and not
        // replicated (multi-rank coarse levels held whole on every rank)
        if (ng < kMinRows || ng <= opt.max_coarse || (int)l + 2 >= opt.max_levels || l + 1 >= perm.size() ||
            (comm.nranks > 1 && opt.replicate_below > 0 && ng <= opt.replicate_below)) {
            open = false;
            return;
        }
        on[l + 1] = 1;
        std::vector<int64_t> up((size_t)n), key((size_t)n);
        const int64_t nbx = (g[0] + kB - 1) / kB, nby = (g[1] + kB - 1) / kB, nbz = (g[2] + kB - 1) / kB;
#pragma omp parallel for schedule(static)
        for (int64_t c = 0; c < n; ++c) {
            int64_t f = 0;  // the fine point of the row's first local column
            for (int64_t k = R.rp[c]; k < R.rp[c + 1]; ++k)
                if (R.col[k] >= flo && R.col[k] < fhi) {
                    f = at[R.col[k] - flo];
                    break;
                }
            const int64_t x = f % g[0], y = (f / g[0]) % g[1], z = f / (g[0] * g[1]);
            up[c] = f;
            key[c] = ((z / kB) * nby + y / kB) * nbx + x / kB;
        }
        at.swap(up);
        // stable counting sort by brick
        std::vector<int64_t> cnt((size_t)(nbx * nby * nbz) + 1, 0);
        for (int64_t c = 0; c < n; ++c) ++cnt[key[c] + 1];
        for (size_t b = 1; b < cnt.size(); ++b) cnt[b] += cnt[b - 1];
        std::vector<int64_t>& p = perm[l + 1];
        std::vector<int64_t>& q = inv[l + 1];
        p.resize((size_t)n);
        q.resize((size_t)n);
        for (int64_t c = 0; c < n; ++c) {
            const int64_t t = cnt[key[c]]++;
            p[t] = c;
            q[c] = t;
        }
    }
};
}  // namespace

Solver::~Solver() {
    for (auto& g : graphs)
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
    for (hipEvent_t e : tl_ev) (void)hipEventDestroy(e);
}

void Solver::setup(DevMatrix& A, const amg_options& o) {
    RoctxRange range("ParMultilevel::setup");
    AMG_CHECK(A.square, "AMG setup needs a square matrix");
    AMG_CHECK(o.pre_sweeps >= 0 && o.post_sweeps >= 0, "negative sweep count");
    AMG_CHECK(o.max_levels >= 1, "max_levels must be >= 1");
    AMG_CHECK(o.smoother == AMG_SMOOTH_JACOBI || o.smoother == AMG_SMOOTH_HYBRID_GS, "bad smoother");
    ctx = A.ctx;
    opt = o;
    A0 = &A;

    const HostComm& comm = ctx->host;
    HostHierarchy H;
    SpgemmFn galerkin = nullptr;
    LevelSetupFn level_fn = nullptr;
    TransposeFn transpose_fn = nullptr;
    RapFn rap_fn = nullptr;
    // the level operators, P and R stay on the device between the setup steps that read them
    // (SetupImages); only the next level's operator is carried over
    SetupImages images;
    SetupImages* im = opt.setup_device ? &images : nullptr;
    // the level-0 operator's CSR left on the device by its format build (one rank)
    // (a host-side setup has no use for it: freed here either way)
    if (im && A.setup_csr) images.put(A.host, std::move(A.setup_csr));
    A.setup_csr.reset();
    if (opt.setup_device) {
        galerkin = [this, &comm](const HostCSR& X, const HostCSR& Y) {
            return spgemm_device(*ctx, comm, X, Y);
        };
        rap_fn = [this, &comm, im](const HostCSR& R, const HostCSR& Am, const HostCSR& P) {
            HostCSR Ac = galerkin_device(*ctx, comm, R, Am, P, im);
            // the drop tolerance before keep_only: the Galerkin product's device image goes
            // (images are keyed by the host arrays' address)
            if (opt.drop_tol > 0.0) Ac = sparsify_device(*ctx, comm, Ac, opt.drop_tol, im);
            if (im) im->keep_only(Ac);
            return Ac;
        };
        // setup_device == 1: the whole level setup on the GPU where it applies;
        // 2: Galerkin products only (the round-1 split, for A/B and tests)
        if (opt.setup_device == 1) {
            level_fn = [this, &comm, im](int l, const HostCSR& A, HostCSR& P, std::vector<int32_t>& split) {
                return level_setup_device(*ctx, comm, A, opt, l, P, split, im);
            };
            transpose_fn = [this, &comm, im](const HostCSR& P, HostCSR& R) {
                return transpose_device(*ctx, comm, P, R, im);
            };
        }
    }
    PhaseTimer tm(comm);
    // device formats of finished levels, built on a worker thread during the hierarchy
    const bool overlap = comm.nranks == 1;
    const size_t maxl = (size_t)std::max(opt.max_levels, 1) + 1;
    std::vector<std::unique_ptr<DevMatrix>> preA(maxl), preP(maxl), preR(maxl), preAc(maxl), prePc(maxl), preRc(maxl);
    const bool hgs = opt.smoother == AMG_SMOOTH_HYBRID_GS;
    // cycle order: the brick order of level l + 1 is fixed once R_l exists; the operators that
    // touch a permuted level are built as cycle-order copies (their hierarchy-order formats wait
    // for a caller that asks for them: DevMatrix::defer)
    CycleOrder co;
    co.init(A, opt, comm, maxl);
    auto copy = [this, &comm](const HostCSR& M, const std::vector<int64_t>& rows, const std::vector<int64_t>& cols) {
        std::unique_ptr<DevMatrix> d(new DevMatrix());
        d->blocks_only = true;  // row templates assume ascending offsets
        // what this rank sends of its column level: positions in that level's order
        d->send_map = cols.empty() ? nullptr : &cols;
        d->build(ctx, permuted_csr(M, comm.rank, rows, cols));
        d->send_map = nullptr;
        return d;
    };
    // a level operator's hybrid-GS structures: l1 diagonals, slabs, templates,
    // the split sweep's old-value pass (built by ensure_gs_blocks), level 0's sliced ELL
    auto gs_build = [this](DevMatrix& Al, int l) {
        Al.ensure_gs_blocks(opt.gs_block);
        // level 0's norm-carrying forward sweep runs the one-kernel form, inside captured
        // cycles: its sliced ELL is built now even where the other sweeps run split
        if (l == 0) Al.ensure_gs_ell();
        // a forward split sweep on x != 0: level 0's (tol > 0 solves), a second pre-sweep
        if (Al.gs_split && (l == 0 || opt.pre_sweeps >= 2)) Al.ensure_gs_pass(0);
    };
    {
        RoctxRange r("setup: hierarchy (strength, split / aggregates, P, R, Galerkin)");
        // r5: a second worker builds each operator's GS structures as soon as its formats
        // exist (level 0 from the start), beside the format worker (sa27: 0.9 s of GS builds
        // after the hierarchy before)
        // gs_worker first: members are destroyed in reverse order, so when build_hierarchy
        // throws, worker and worker2 drain (their A_{l+1} jobs push onto gs_worker) before
        // gs_worker itself is joined and freed
        std::unique_ptr<FormatWorker> gs_worker, worker, worker2;
        LevelDoneFn done = nullptr;
        if (overlap) {
            worker.reset(new FormatWorker(ctx->device));
            worker2.reset(new FormatWorker(ctx->device));
            if (hgs) {
                gs_worker.reset(new FormatWorker(ctx->device));
                DevMatrix* a0 = &A;
                gs_worker->push([gs_build, a0] { gs_build(*a0, 0); });
            }
            done = [&](int l) {
                auto job = [this, &gs_worker, &gs_build](std::unique_ptr<DevMatrix>& slot, const HostCSR& M,
                                                         int gs_level) {
                    return [this, &slot, &M, &gs_worker, &gs_build, gs_level] {
                        std::unique_ptr<DevMatrix> d(new DevMatrix());
                        d->build_view(ctx, M);
                        if (gs_level >= 0 && gs_worker) {
                            DevMatrix* dm = d.get();
                            dm->host_view = &M;
                            gs_worker->push([gs_build, dm, gs_level] { gs_build(*dm, gs_level); });
                        }
                        slot = std::move(d);
                    };
                };
                // A_{l+1} first: its GS structures start on the second worker while P_l and
                // R_l are built
                // (r5: P_l and R_l on a second format worker beside A_{l+1})
                co.next((size_t)l, H.levels[l].R, opt, comm);
                const size_t a = (size_t)l + 1, p = (size_t)l;
                if (co.any(a)) {
                    const HostCSR* M = &H.levels[a].A;
                    worker->push([&, a, M] { preAc[a] = copy(*M, co.perm[a], co.inv[a]); });
                } else {
                    worker->push(job(preA[a], H.levels[a].A, (int)a));
                }
                if (co.any(p) || co.any(a)) {
                    const HostCSR *Ph = &H.levels[p].P, *Rh = &H.levels[p].R;
                    worker2->push([&, a, p, Ph] { prePc[p] = copy(*Ph, co.perm[p], co.inv[a]); });
                    worker2->push([&, a, p, Rh] { preRc[p] = copy(*Rh, co.perm[a], co.inv[p]); });
                } else {
                    worker2->push(job(preP[p], H.levels[p].P, -1));
                    worker2->push(job(preR[p], H.levels[p].R, -1));
                }
            };
        }
        build_hierarchy(comm, A.host, opt, H, galerkin, level_fn, transpose_fn, done, rap_fn);
        images.e.clear();
        tm.lap("hierarchy (host + SpGEMM)");
        if (worker) worker->finish();  // before gs_worker: its jobs push GS jobs
        if (worker2) worker2->finish();
        if (gs_worker) gs_worker->finish();
        if (overlap) tm.lap("format builds still running after the hierarchy");
    }
    // replicated coarse levels (multi-rank): from the first level with <= replicate_below
    // global rows on, every rank holds the whole operators and cycles them locally
    rep_level = -1;
    if (comm.nranks > 1 && opt.replicate_below > 0)
        for (size_t l = 1; l < H.levels.size(); ++l)
            if (H.A(l).n_global_rows <= opt.replicate_below) {
                rep_level = (int)l;
                break;
            }
    if (!overlap)  // the brick orders (overlapped setups fixed them level by level)
        for (size_t l = 0; l + 1 < H.levels.size(); ++l) co.next(l, H.levels[l].R, opt, comm);
    levels.clear();
    levels.resize(H.levels.size());
    RoctxRange rbuild("setup: device level formats");
    for (size_t l = 0; l < H.levels.size(); ++l) {
        HostLevel& hl = H.levels[l];
        const bool rep = rep_level >= 0 && (int)l >= rep_level;
        auto make = [&](HostCSR& M, std::unique_ptr<DevMatrix>& pre, bool cycle_copy) {
            std::unique_ptr<DevMatrix> d(std::move(pre));
            if (d) {
                d->host = std::move(M);  // built from M on the worker
                d->host_view = nullptr;
                return d;
            }
            d.reset(new DevMatrix());
            if (rep) d->build(ctx, gather_global(comm, M), true);
            else if (cycle_copy) d->defer(ctx, std::move(M));  // the cycle runs its copy
            else d->build(ctx, std::move(M));
            return d;
        };
        const bool pa = l > 0 && co.any(l), pr = co.any(l) || co.any(l + 1);
        if (l > 0) levels[l].A = make(hl.A, preA[l], pa);
        if (!overlap) tm.lap("L" + std::to_string(l) + " device A build");
        if (l + 1 < H.levels.size()) {
            levels[l].split = std::move(hl.split);
            if (rep) {  // a replicated level is whole on every rank: so is its splitting
                const std::vector<std::vector<int32_t>> all =
                    comm.exchange(std::vector<std::vector<int32_t>>(comm.nranks, levels[l].split));
                levels[l].split.clear();
                for (const auto& v : all) levels[l].split.insert(levels[l].split.end(), v.begin(), v.end());
            }
            levels[l].P = make(hl.P, preP[l], pr);
            levels[l].R = make(hl.R, preR[l], pr);
            if (!overlap) tm.lap("L" + std::to_string(l) + " device P/R build");
        }
    }
    // cycle-order copies (built on the workers where the setup overlaps, here otherwise)
    if (co.any(levels.size() - 1)) {
        // the coarsening stalled on a permuted level, which became the (dense-solved) coarsest:
        // the cycle runs the hierarchy's order
        for (auto& L : levels)
            for (DevMatrix* m : {L.A.get(), L.P.get(), L.R.get()})
                if (m) m->ensure_built();
    } else {
        for (size_t l = 0; l < levels.size(); ++l) {
            const bool pa = l > 0 && co.any(l), pr = l + 1 < levels.size() && (co.any(l) || co.any(l + 1));
            if (pa) levels[l].Ac = preAc[l] ? std::move(preAc[l]) : copy(levels[l].A->host, co.perm[l], co.inv[l]);
            if (pr) {
                levels[l].Pc = prePc[l] ? std::move(prePc[l]) : copy(levels[l].P->host, co.perm[l], co.inv[l + 1]);
                levels[l].Rc = preRc[l] ? std::move(preRc[l]) : copy(levels[l].R->host, co.perm[l + 1], co.inv[l]);
            }
        }
        if (!overlap) tm.lap("cycle-order copies");
    }
    if (rep_level > 0) {  // transition: distributed R output -> whole vector on every rank
        const HostCSR& Rh = levels[rep_level - 1].R->host;
        rep_starts = Rh.row_starts;
        rep_cmax = 0;
        for (int r = 0; r < comm.nranks; ++r)
            rep_cmax = std::max(rep_cmax, rep_starts[r + 1] - rep_starts[r]);
        rep_pad.alloc((size_t)rep_cmax * (comm.nranks + 1));
        HIP_CHECK(hipMemset(rep_pad.p, 0, rep_pad.n * sizeof(double)));
    }
    // per-level work vectors
    size_t max_blocks = 0;
    for (size_t l = 0; l < levels.size(); ++l) {
        DevMatrix& Al = Amat(l);
        const size_t n = (size_t)Al.n_rows;
        if (l > 0) {
            levels[l].x.alloc(n);
            levels[l].b.alloc(n);
        }
        levels[l].r.alloc(n);
        levels[l].t.alloc(n);
        max_blocks = std::max({max_blocks, (size_t)Al.norm_parts_max(), (size_t)CA(l).norm_parts_max()});
        if (hgs) {
            gs_build(Al, (int)l);  // done on the GS worker already where the setup overlaps
            tm.lap("L" + std::to_string(l) + " GS structures");
            max_blocks = std::max(max_blocks, (size_t)Al.gs_norm_parts());
        }
    }
    // norm plumbing: partials | reduction scratch | gathered rank sums
    const size_t tmpn = max_blocks / 4096 + 64;
    norm_scratch.alloc(max_blocks + tmpn + (size_t)comm.nranks + 8);
    sink.partial = norm_scratch.p;
    sink.tmp = sink.partial + max_blocks;
    sink.gathered = sink.tmp + tmpn;
    hist_counter.alloc(1);
    sink.counter = hist_counter.p;
    norm_done.alloc(1);
    HIP_CHECK(hipMemset(norm_done.p, 0, sizeof(unsigned)));
    sink.done = norm_done.p;
    ensure_hist(1024);
    // coarsest level: this rank's rows of the gathered dense inverse, row-major (one
    // wavefront per row reads its row coalesced).  With several ranks b is
    // allgathered into a padded [nranks x cmax] layout and unpadded into the global order
    // before the solve (the lanes' interleaving is defined on the global index j).
    DevMatrix& Ac = Amat(levels.size() - 1);
    coarse_n = Ac.host.n_global_rows;
    const std::vector<double>& inv = H.coarse_inv;
    const int64_t nl = Ac.n_rows, f = Ac.first_row;
    const bool serial_coarse = comm.nranks == 1 || Ac.replicated;
    const int nparts = serial_coarse ? 1 : comm.nranks;
    int64_t cmax = 0;
    coarse_starts.assign(Ac.host.row_starts.begin(), Ac.host.row_starts.end());
    for (int r = 0; r < nparts; ++r)
        cmax = std::max(cmax, Ac.host.row_starts[r + 1] - Ac.host.row_starts[r]);
    this->invT.upload(inv.data() + (size_t)(f * coarse_n), (size_t)std::max<int64_t>(nl * coarse_n, 0));
    if (nl * coarse_n == 0) this->invT.alloc(1);
    tm.lap("coarse inverse upload");
    coarse_counts.assign(1, (int)cmax);
    if (!serial_coarse) {
        // gathered (nranks x cmax) + local padded send slot + the unpadded global vector
        bfull.alloc((size_t)cmax * comm.nranks + (size_t)cmax + (size_t)coarse_n);
        HIP_CHECK(hipMemset(bfull.p, 0, bfull.n * sizeof(double)));
    }
    // multi-rank cycles: loopback ranks meet at host barriers, which a graph cannot replay;
    // RCCL ranks capture whole cycles where the runtime is the one capture was validated on
    use_graph = comm.nranks == 1 || (ctx->transport == TR_RCCL && rccl_graph_allowed());
}

// Whole-cycle capture with RCCL groups inside: on HIP 7.0.51831 + RCCL 2.26.6
// (the copies torch bundles, which a torch-first process binds) hipStreamEndCapture segfaults;
// on ROCm 7.2's HIP 7.2.26015 + RCCL 2.27.7 (torch-free callers) captured cycles replay
// bit-exact.  AMG_RCCL_GRAPH=0 / 1 overrides the version check either way.
bool Solver::rccl_graph_allowed(std::string* why) {
    static const int forced = [] {
        const char* e = std::getenv("AMG_RCCL_GRAPH");
        return e && *e ? (std::atoi(e) != 0 ? 1 : 0) : -1;
    }();
    int hv = 0, nv = 0;
    (void)hipRuntimeGetVersion(&hv);
    (void)ncclGetVersion(&nv);
    const bool ok = forced >= 0 ? forced == 1 : hv >= 70200000 && nv >= 22707;
    if (!ok && why)
        *why = "multi-rank hipGraph capture of RCCL cycles is validated on HIP >= 7.2 with RCCL >= "
               "2.27.7; this process runs HIP " + std::to_string(hv) + " with RCCL " +
               std::to_string(nv) + (forced == 0 ? " (AMG_RCCL_GRAPH=0)" : " (AMG_RCCL_GRAPH=1 overrides)");
    return ok;
}

void Solver::ensure_hist(int32_t n) {
    if (hist.n >= (size_t)n) return;
    hist.alloc((size_t)n);
    sink.hist = hist.p;
    destroy_graphs();  // captured graphs baked the old pointer (collective: every rank's solve
                       // sizes the history from the same max_iter)
}

// Hybrid GS sweeps forward before the coarse correction and backward after it (post):
// the V-cycle is then a symmetric operator, as CG requires (oracle smooth()).
void Solver::smooth(size_t l, double*& x, const double* b, double*& tmp, bool x_zero,
                    bool with_norm, bool post) {
    DevMatrix& A = CA(l);
    if (with_norm && opt.smoother == AMG_SMOOTH_HYBRID_GS) {
        // forward GS sweep that also leaves the partials of ||b - A x|| (old x)
        AMG_ASSERT(!x_zero && !post);
        par_hybrid_gs(A, x, b, tmp, opt.gs_block, false, sink.partial);
        norm_finish(A, sink, A.gs_norm_parts());
    } else if (with_norm) {  // Jacobi sweep that also leaves the partials of ||b - A x||
        AMG_ASSERT(opt.smoother == AMG_SMOOTH_JACOBI && !x_zero);
        par_apply(A, KM_JACOBI, x, b, tmp, opt.jacobi_omega, sink.partial);
        norm_finish(A, sink);
    } else if (opt.smoother == AMG_SMOOTH_HYBRID_GS) {
        if (x_zero) launch_zero(ctx->stream, A.n_rows, x);
        if (x_zero && !post) par_hybrid_gs_from_zero(A, x, b, tmp, opt.gs_block);
        else par_hybrid_gs(A, x, b, tmp, opt.gs_block, post);
    } else if (x_zero) {
        launch_jacobi_zero(ctx->stream, A.n_rows, b, A.dinv.p, tmp, opt.jacobi_omega);
    } else {
        par_apply(A, KM_JACOBI, x, b, tmp, opt.jacobi_omega, nullptr);
    }
    std::swap(x, tmp);
    mark(l, post ? "post-smooth" : with_norm ? "pre-smooth + norm" : x_zero ? "pre-smooth from 0" : "pre-smooth");
}

// Timeline marks (amg_solver_cycle_timeline).  tl_mode 2, inside the timeline's capture: an
// event-record node is added behind the capture's current tail and becomes the new tail, so one
// graph of the whole cycle timestamps every operation as it replays (HIP captures a plain
// event record only as a dependency marker).  tl_mode 1, inside the capture: the capture is
// closed there and reopened (one graph per operation, replayed back to back with timing events
// between them; each time then includes a graph launch).  Eager: a timing event.
void Solver::mark(size_t l, const char* what) {
    if (!tl_on) return;
    hipStream_t s = ctx->stream;
    const std::string label = "L" + std::to_string(l) + " " + what;
    if (ctx->capturing && tl_mode == 1) {
        hipGraph_t g = nullptr;
        HIP_CHECK(hipStreamEndCapture(s, &g));
        tl_graphs.push_back(g);
        tl_label.push_back(label);
        HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        return;
    }
    if (tl_n == tl_ev.size()) {
        hipEvent_t e;
        HIP_CHECK(hipEventCreate(&e));  // timing enabled
        tl_ev.push_back(e);
    }
    if (tl_label.size() <= tl_n) tl_label.resize(tl_n + 1);
    tl_label[tl_n] = label;
    if (ctx->capturing) {  // tl_mode 2
        hipStreamCaptureStatus st;
        hipGraph_t g = nullptr;
        const hipGraphNode_t* deps = nullptr;
        size_t nd = 0;
        HIP_CHECK(hipStreamGetCaptureInfo_v2(s, &st, nullptr, &g, &deps, &nd));
        hipGraphNode_t en;
        HIP_CHECK(hipGraphAddEventRecordNode(&en, g, deps, nd, tl_ev[tl_n]));
        HIP_CHECK(hipStreamUpdateCaptureDependencies(s, &en, 1, hipStreamSetCaptureDependencies));
    } else {
        HIP_CHECK(hipEventRecord(tl_ev[tl_n], s));
    }
    ++tl_n;
}

int Solver::cycle_timeline(double* x, const double* b, int reps, std::vector<std::string>& labels,
                           std::vector<double>& us) {
    AMG_CHECK(ctx->host.nranks == 1, "cycle timeline: one rank");
    AMG_CHECK(reps >= 1, "cycle timeline: reps must be >= 1");
    hipStream_t s = ctx->stream;
    auto ensure_events = [&](size_t n) {
        while (tl_ev.size() < n) {
            hipEvent_t e;
            HIP_CHECK(hipEventCreate(&e));
            tl_ev.push_back(e);
        }
    };
    // capture the cycle with marks in mode m; the instantiated graphs (one, or one per
    // operation) and their labels; false where the runtime refuses
    std::vector<hipGraphExec_t> execs;
    std::vector<std::string> seg_label;
    auto capture = [&](int m) {
        tl_mode = m;
        tl_graphs.clear();
        tl_label.clear();
        tl_n = 0;
        tl_on = true;
        HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        ctx->capturing = true;
        std::string err;
        try {
            if (m == 2) mark(0, "begin");
            cycle_rec(0, x, b, false, false);
        } catch (const std::exception& e) {
            err = e.what();
        }
        ctx->capturing = false;
        tl_on = false;
        hipGraph_t last = nullptr;
        const hipError_t ce = hipStreamEndCapture(s, &last);
        (void)hipGetLastError();
        bool ok = err.empty() && ce == hipSuccess;
        if (m == 2) {
            if (last) tl_graphs.push_back(last);
            seg_label.assign(tl_label.begin() + (tl_n > 0 ? 1 : 0), tl_label.begin() + tl_n);
        } else {
            if (last) (void)hipGraphDestroy(last);  // after the last mark: nothing
            seg_label = tl_label;
        }
        for (hipGraph_t g : tl_graphs) {
            hipGraphExec_t e = nullptr;
            if (ok && hipGraphInstantiate(&e, g, nullptr, nullptr, 0) == hipSuccess) execs.push_back(e);
            else ok = false;
            (void)hipGraphDestroy(g);
        }
        tl_graphs.clear();
        (void)hipGetLastError();
        if (!ok) {
            for (hipGraphExec_t e : execs) (void)hipGraphExecDestroy(e);
            execs.clear();
        }
        return ok;
    };
    // one replay: a vector of event-to-event times (ms), empty where the runtime did not time them
    auto replay = [&](int m) {
        std::vector<float> t;
        size_t n = 0;
        if (m == 2) {
            HIP_CHECK(hipGraphLaunch(execs[0], s));
            n = tl_n;
        } else if (m == 1) {
            ensure_events(execs.size() + 1);
            HIP_CHECK(hipEventRecord(tl_ev[0], s));
            for (size_t k = 0; k < execs.size(); ++k) {
                HIP_CHECK(hipGraphLaunch(execs[k], s));
                HIP_CHECK(hipEventRecord(tl_ev[k + 1], s));
            }
            n = execs.size() + 1;
        } else {
            tl_mode = 0;
            tl_on = true;
            tl_n = 0;
            try {
                mark(0, "begin");
                cycle_rec(0, x, b, false, false);
            } catch (...) {
                tl_on = false;
                throw;
            }
            tl_on = false;
            n = tl_n;
            seg_label.assign(tl_label.begin() + 1, tl_label.begin() + (n > 0 ? n : 1));
        }
        HIP_CHECK(hipStreamSynchronize(s));
        for (size_t k = 1; k < n; ++k) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, tl_ev[k - 1], tl_ev[k]) != hipSuccess) {
                (void)hipGetLastError();
                return std::vector<float>();
            }
            t.push_back(ms);
        }
        return t;
    };
    int mode = 0;
    std::vector<std::vector<float>> t;
    for (int m = use_graph ? 2 : 0; m >= 0 && mode == 0; --m) {
        if (m > 0 && !capture(m)) continue;
        std::vector<float> first = replay(m);
        if (first.empty() && m > 0) {  // not timed: the next mode
            for (hipGraphExec_t e : execs) (void)hipGraphExecDestroy(e);
            execs.clear();
            continue;
        }
        mode = m > 0 ? m : -1;
        t.assign(first.size(), {});
        for (size_t k = 0; k < first.size(); ++k) t[k].push_back(first[k]);
        for (int r = 1; r < reps; ++r) {
            const std::vector<float> v = replay(m);
            for (size_t k = 0; k < v.size() && k < t.size(); ++k) t[k].push_back(v[k]);
        }
    }
    for (hipGraphExec_t e : execs) HIP_CHECK(hipGraphExecDestroy(e));
    execs.clear();
    labels = seg_label;
    labels.resize(t.size());
    if (mode == 2) {
        // calibration: two event-record nodes with nothing between them -- the time a node adds
        // to the operation before it (reported as a last pseudo-operation "event-node gap")
        tl_mode = 2;
        tl_graphs.clear();
        tl_n = 0;
        tl_on = true;
        HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        ctx->capturing = true;
        std::string err;
        try {
            mark(0, "gap a");
            mark(0, "gap b");
        } catch (const std::exception& e) {
            err = e.what();
        }
        ctx->capturing = false;
        tl_on = false;
        hipGraph_t g = nullptr;
        const hipError_t ce = hipStreamEndCapture(s, &g);
        hipGraphExec_t e = nullptr;
        if (err.empty() && ce == hipSuccess && g && hipGraphInstantiate(&e, g, nullptr, nullptr, 0) == hipSuccess) {
            std::vector<float> gv;
            for (int r = 0; r < reps; ++r) {
                HIP_CHECK(hipGraphLaunch(e, s));
                HIP_CHECK(hipStreamSynchronize(s));
                float ms = 0.f;
                if (hipEventElapsedTime(&ms, tl_ev[0], tl_ev[1]) == hipSuccess) gv.push_back(ms);
            }
            if (!gv.empty()) {
                labels.push_back("event-node gap");
                t.push_back(gv);
            }
            HIP_CHECK(hipGraphExecDestroy(e));
        }
        if (g) (void)hipGraphDestroy(g);
        (void)hipGetLastError();
    }
    tl_mode = 0;
    us.clear();
    for (auto& v : t) {
        std::sort(v.begin(), v.end());
        us.push_back(1e3 * (double)v[v.size() / 2]);
    }
    return mode > 0 ? mode : 0;
}

void Solver::cycle_rec(size_t l, double* x, const double* b, bool x_zero, bool with_norm, bool x0_in_t) {
    DevMatrix& A = CA(l);
    hipStream_t s = ctx->stream;
    const HostComm& comm = ctx->host;
    if (l + 1 == levels.size()) {
        const double* bf = b;
        if (comm.nranks > 1 && !A.replicated) {
            const int64_t cmax = coarse_counts[0];
            double* slot = bfull.p + cmax * comm.nranks;
            if (A.n_rows > 0)
                HIP_CHECK(hipMemcpyAsync(slot, b, A.n_rows * sizeof(double), hipMemcpyDeviceToDevice, s));
            ctx->allgather(slot, bfull.p, (size_t)cmax);
            double* glob = bfull.p + cmax * (comm.nranks + 1);
            for (int q = 0; q < comm.nranks; ++q) {
                const int64_t c = coarse_starts[q + 1] - coarse_starts[q];
                if (c)
                    HIP_CHECK(hipMemcpyAsync(glob + coarse_starts[q], bfull.p + q * cmax, c * sizeof(double),
                                             hipMemcpyDeviceToDevice, s));
            }
            launch_dense_gemv(s, A.n_rows, coarse_n, invT.p, glob, x);
        } else {
            launch_dense_gemv(s, A.n_rows, coarse_n, invT.p, bf, x);
        }
        mark(l, "coarse solve");
        return;
    }
    Level& L = levels[l];
    double* cur = x;
    double* tmp = L.t.p;
    bool zero = x_zero;
    for (int k = 0; k < opt.pre_sweeps; ++k) {
        if (k == 0 && x0_in_t) std::swap(cur, tmp);  // the sweep from zero is in tmp already
        else smooth(l, cur, b, tmp, zero, with_norm && k == 0);
        zero = false;
    }
    if (zero) launch_zero(s, A.n_rows, cur);
    par_apply(A, KM_RESID, cur, b, L.r.p, 0.0, nullptr);
    mark(l, "residual");
    Level& C = levels[l + 1];
    if ((int)l + 1 == rep_level) {
        // distributed R output -> whole b_{l+1} on every rank (padded allgather + unpad)
        const int64_t cmax = rep_cmax, me = comm.rank;
        double* slot = rep_pad.p + cmax * comm.nranks;
        par_apply(CR(l), KM_SPMV, L.r.p, nullptr, slot, 0.0, nullptr);
        ctx->allgather(slot, rep_pad.p, (size_t)cmax);
        for (int q = 0; q < comm.nranks; ++q) {
            const int64_t cnt = rep_starts[q + 1] - rep_starts[q];
            if (cnt)
                HIP_CHECK(hipMemcpyAsync(C.b.p + rep_starts[q], rep_pad.p + q * cmax,
                                         cnt * sizeof(double), hipMemcpyDeviceToDevice, s));
        }
        (void)me;
        mark(l, "restrict + allgather");
        cycle_rec(l + 1, C.x.p, C.b.p, true, false);
        // this rank's slice of the whole correction feeds the distributed interpolation
        par_apply(CP(l), KM_SPMV_ADD, C.x.p + L.P->first_col, nullptr, cur, 0.0, nullptr);
    } else {
        // Jacobi: the coarse level's first sweep from x = 0 (omega dinv b) rides along with
        // the restriction that produces b (one pass over b and a launch fewer per level)
        const bool j0 = opt.smoother == AMG_SMOOTH_JACOBI && opt.pre_sweeps >= 1 && l + 2 < levels.size() &&
                        par_restrict_j0(CR(l), L.r.p, C.b.p, C.t.p, CA(l + 1).dinv.p, opt.jacobi_omega);
        if (!j0) par_apply(CR(l), KM_SPMV, L.r.p, nullptr, C.b.p, 0.0, nullptr);
        mark(l, j0 ? "restrict + next pre-smooth from 0" : "restrict");
        cycle_rec(l + 1, C.x.p, C.b.p, true, false, j0);
        par_apply(CP(l), KM_SPMV_ADD, C.x.p, nullptr, cur, 0.0, nullptr);
    }
    mark(l, "interp");
    for (int k = 0; k < opt.post_sweeps; ++k) smooth(l, cur, b, tmp, false, false, true);
    if (cur != x) {
        HIP_CHECK(hipMemcpyAsync(x, cur, A.n_rows * sizeof(double), hipMemcpyDeviceToDevice, s));
        mark(l, "copy");
    }
}

bool Solver::can_fuse_norm() const {
    return (opt.smoother == AMG_SMOOTH_JACOBI || opt.smoother == AMG_SMOOTH_HYBRID_GS) &&
           opt.pre_sweeps >= 1 && levels.size() >= 2;
}

// An exec is destroyed only once the stream has drained: a replay enqueued without a host
// wait (graph_launch) may still be running, and HIP does not document a deferred free of an
// executing graph the way CUDA does.  Recaptures are rare, so one wait is cheap.
void Solver::drop_graph(Graph& G) {
    if (!G.exec) return;
    if (!ctx->capturing) HIP_CHECK(hipStreamSynchronize(ctx->stream));
    ctx->graph_inflight = false;
    HIP_CHECK(hipGraphExecDestroy(G.exec));
    G.exec = nullptr;
}

void Solver::destroy_graphs() {
    for (auto& g : graphs) drop_graph(g);
}

// Capture `body` (enqueues on ctx->stream, RCCL groups included) into graphs[slot] unless the
// graph for (x, b) and the current formats exists.  Multi-rank, the decision is collective:
//  1. with `agree`, every rank's stale flag goes through the host exchange and all ranks
//     recapture if any must (a caching allocator handing x a new address on one rank only
//     would otherwise leave that rank capturing -- and waiting in the host exchange below --
//     while its peers replay RCCL groups it never joins);
//  2. the capture + instantiate status is exchanged: one rank's failure sends every rank to
//     eager launches (an exception during capture raises on every rank).
bool Solver::graph_ready(int slot, const double* x, const double* b, const std::function<void()>& body,
                         bool agree) {
    Graph& G = graphs[slot];
    const HostComm& comm = ctx->host;
    const bool multi = comm.nranks > 1;
    bool stale = !G.exec || G.x != x || G.b != b || G.fmt_gen != DevMatrix::format_generation;
    if (multi && agree) {
        bool any = false;
        for (int64_t v : comm.allgather((int64_t)(stale ? 1 : 0))) any = any || v != 0;
        stale = any;
    }
    if (!stale) return true;
    drop_graph(G);
    hipStream_t s = ctx->stream;
    static const bool trace = std::getenv("AMG_TRACE_RCCL") != nullptr;
    if (trace) std::fprintf(stderr, "[amg] rank %d capture begin (slot %d)\n", comm.rank, slot);
    RoctxRange r("cycle: hipGraph capture");
    install_crash_handler();
    // a capture starts from an idle stream: RCCL work of earlier replays still in flight
    // stays ordered before the captured groups by the stream, and nothing eager is pending
    if (multi) ctx->eager_rccl_fence();
    hipGraph_t g = nullptr;
    std::string err;
    int err_code = AMG_ERR_INTERNAL;  // the amg::Error code of a failing body, rethrown below
    HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    ctx->capturing = true;
    try {
        body();
    } catch (const Error& e) {
        err = e.what();
        err_code = e.code;
    } catch (const std::exception& e) {
        err = e.what();
    }
    ctx->capturing = false;
    const hipError_t ce = hipStreamEndCapture(s, &g);
    if (ce != hipSuccess && err.empty()) err = std::string("hipStreamEndCapture: ") + hipGetErrorString(ce);
    if (trace) std::fprintf(stderr, "[amg] rank %d capture end\n", comm.rank);
    hipError_t ie = hipErrorUnknown;
    if (err.empty() && g) ie = hipGraphInstantiate(&G.exec, g, nullptr, nullptr, 0);
    if (g) (void)hipGraphDestroy(g);
    if (ie != hipSuccess) {
        (void)hipGetLastError();
        G.exec = nullptr;
    }
    // 1 = ready, 0 = instantiate refused, -1 = the capture itself failed
    const int64_t mine = !err.empty() ? -1 : ie == hipSuccess ? 1 : 0;
    int64_t worst = mine;
    if (multi)
        for (int64_t v : comm.allgather(mine)) worst = std::min(worst, v);
    if (worst == -1) {
        destroy_graphs();
        use_graph = false;
        // the failing rank keeps its own error code (NOMEM, INVALID, ...); its peers report
        // the generic failure
        throw Error(err.empty() ? AMG_ERR_INTERNAL : err_code,
                    "V-cycle capture failed" + (err.empty() ? std::string(" on another rank") : ": " + err));
    }
    if (worst == 0) {
        // a graph some rank's runtime cannot instantiate: every rank runs eagerly from now on
        // (identical results; only the launch overhead differs)
        AMG_CHECK(multi, std::string("hipGraphInstantiate: ") + hipGetErrorString(ie));
        destroy_graphs();
        use_graph = false;
        return false;
    }
    G.x = x;
    G.b = b;
    G.fmt_gen = DevMatrix::format_generation;
    return true;
}

// One collective staleness decision for every graph slot a call will replay (multi-rank): a
// slot stale on any rank is dropped on every rank, so the later graph_ready(.., agree = false)
// calls capture -- and meet in the capture's status exchange -- on all ranks or on none.
// (Deciding per slot inside the loop hung: solve's last-norm graph was stale on the rank whose
// x had moved and fresh on the others, so one rank waited in the status exchange.)
void Solver::agree_stale(std::initializer_list<int> slots, const double* x, const double* b) {
    const HostComm& comm = ctx->host;
    if (!use_graph || comm.nranks <= 1) return;
    bool stale = false;
    for (int slot : slots) {
        const Graph& G = graphs[slot];
        stale = stale || !G.exec || G.x != x || G.b != b || G.fmt_gen != DevMatrix::format_generation;
    }
    bool any = false;
    for (int64_t v : comm.allgather((int64_t)(stale ? 1 : 0))) any = any || v != 0;
    if (!any) return;
    if (ctx->graph_inflight) ctx->eager_rccl_fence();  // replays of the graphs dropped below
    for (int slot : slots) drop_graph(graphs[slot]);
}

void Solver::graph_launch(int slot) {
    RoctxRange r("cycle: hipGraph replay");
    HIP_CHECK(hipGraphLaunch(graphs[slot].exec, ctx->stream));
    static const bool trace = std::getenv("AMG_TRACE_RCCL") != nullptr;
    if (trace) std::fprintf(stderr, "[amg] rank %d graph launched (slot %d)\n", ctx->host.rank, slot);
    // no host wait: the next replay orders behind this one on the stream, and the next eager
    // RCCL enqueue waits once (Context::eager_rccl_fence)
    if (ctx->host.nranks > 1) ctx->graph_inflight = true;
}

void Solver::cycle(double* x, const double* b, bool with_norm, bool agree) {
    AMG_ASSERT(!with_norm || can_fuse_norm());
    const int slot = with_norm ? G_CYCLE_NORM : G_CYCLE;
    if (use_graph && graph_ready(slot, x, b, [&] { cycle_rec(0, x, b, false, with_norm); }, agree)) {
        graph_launch(slot);
        return;
    }
    RoctxRange r("cycle: eager");
    cycle_rec(0, x, b, false, with_norm);
}

void Solver::residual_norm(double* x, const double* b, bool agree) {
    DevMatrix& A = *A0;
    double* r = levels[0].r.p;
    // AMG_RCCL_NORM_GRAPH=0: the norm eager after graph-replayed cycles (probe of the eager
    // fence)
    static const bool norm_graph = [] {
        const char* e = std::getenv("AMG_RCCL_NORM_GRAPH");
        return !(e && *e && std::atoi(e) == 0);
    }();
    if (use_graph && (norm_graph || ctx->host.nranks == 1) &&
        graph_ready(G_NORM, x, b, [&] { par_residual_norm(A, x, b, r, sink); }, agree)) {
        graph_launch(G_NORM);
        return;
    }
    par_residual_norm(A, x, b, r, sink);
}

int32_t Solver::solve(double* x, const double* b, int32_t max_iter, double tol, double* hist_host) {
    AMG_CHECK(max_iter >= 0, "max_iter must be >= 0");
    RoctxRange range("ParMultilevel::solve");
    hipStream_t s = ctx->stream;
    ensure_hist(max_iter + 1);
    if (ctx->host.nranks > 1) ctx->eager_rccl_fence();
    HIP_CHECK(hipMemsetAsync(hist_counter.p, 0, sizeof(int), s));
    int32_t it = 0;
    // one collective graph decision per solve, over every slot it replays (x and b stay put
    // for its cycles)
    if (tol <= 0.0 && can_fuse_norm()) {
        // ||b - A x_k|| comes out of cycle k+1's first Jacobi sweep (same b - Ax values);
        // only the last norm needs its own residual pass.  No host sync in the loop, and with
        // graphs on, no eager work at all: cycles and the last norm replay captured graphs.
        agree_stale({G_CYCLE_NORM, G_NORM}, x, b);
        for (; it < max_iter; ++it) cycle(x, b, true, false);
        residual_norm(x, b, false);
    } else {
        agree_stale({G_CYCLE, G_NORM}, x, b);
        residual_norm(x, b, false);
        double r0 = 0.0;
        if (tol > 0.0) {
            HIP_CHECK(hipMemcpyAsync(&r0, hist.p, sizeof(double), hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
            ctx->graph_inflight = false;
        }
        while (it < max_iter) {
            cycle(x, b, false, false);
            residual_norm(x, b, false);
            ++it;
            if (tol > 0.0) {
                double rn = 0.0;
                HIP_CHECK(hipMemcpyAsync(&rn, hist.p + it, sizeof(double), hipMemcpyDeviceToHost, s));
                HIP_CHECK(hipStreamSynchronize(s));
                ctx->graph_inflight = false;
                if (r0 > 0.0 && rn / r0 < tol) break;
            }
        }
    }
    HIP_CHECK(hipMemcpyAsync(hist_host, hist.p, sizeof(double) * (size_t)(it + 1),
                             hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    ctx->graph_inflight = false;
    return it;
}

// ---- AMG-preconditioned CG ------------------------------------
// Scalars never leave the device (alpha/beta are formed inside the update kernels), so an
// iteration has no host synchronisation unless a tolerance is requested.  Dot products use
// a fixed block span + fixed trees + rank-ordered sums: deterministic for a given partition.
enum { SC_RZ = 0, SC_RZN, SC_PQ, SC_RN, SC_N };

void Solver::dot(const double* a, const double* b, double* dst, bool take_sqrt) {
    DevMatrix& A = *A0;
    const int g = dot_partial_count(A.n_rows);
    double* partial = pcg_scratch.p;
    double* tmp = partial + g;
    double* gathered = tmp + g / 4096 + 64;
    double* local = gathered + ctx->host.nranks;
    launch_dot_partials(ctx->stream, A.n_rows, a, b, partial);
    launch_reduce_partials(ctx->stream, g, partial, tmp, local);
    if (ctx->host.nranks > 1) {
        ctx->allgather(local, gathered, 1);
        launch_finish_sum(ctx->stream, ctx->host.nranks, gathered, dst, take_sqrt);
    } else {
        launch_finish_sum(ctx->stream, 1, local, dst, take_sqrt);
    }
}

// With graphs on, an iteration is two captured graphs: G_PCG_STEP (q = A p, p.q, the x / r
// update, ||r|| appended) and G_PCG_PREC (z = M^-1 r by one V-cycle from z = 0, r.z, the p
// update).  Multi-rank, their RCCL halo groups and dot allgathers replay inside the graphs, so
// nothing eager follows a replay inside the loop and Context::eager_rccl_fence never waits
// there (the eager dot allgathers synchronised the host once per
// iteration).  The set-up (r = b - A x, ||r||, the first z, r.z) runs eagerly, before any
// replay.  tol > 0 waits for the norm each iteration anyway.
int32_t Solver::pcg(double* x, const double* b, int32_t max_iter, double tol, double* hist_host) {
    AMG_CHECK(max_iter >= 0, "max_iter must be >= 0");
    RoctxRange range("ParMultilevel::pcg");
    DevMatrix& A = *A0;
    const int64_t n = A.n_rows;
    hipStream_t s = ctx->stream;
    const int g = dot_partial_count(n);
    const size_t need = (size_t)g + g / 4096 + 64 + ctx->host.nranks + 2 + SC_N;
    if (pcg_vec.n < (size_t)(4 * n + 4) || pcg_scratch.n < need) {
        // the captured iteration graphs hold these addresses
        drop_graph(graphs[G_PCG_STEP]);
        drop_graph(graphs[G_PCG_PREC]);
        if (pcg_vec.n < (size_t)(4 * n + 4)) pcg_vec.alloc((size_t)(4 * n + 4));
        if (pcg_scratch.n < need) pcg_scratch.alloc(need);
    }
    double* r = pcg_vec.p;
    double* z = r + n;
    double* p = z + n;
    double* q = p + n;
    double* sc = pcg_scratch.p + (need - SC_N);
    ensure_hist(max_iter + 1);
    if (ctx->host.nranks > 1) ctx->eager_rccl_fence();  // replays of earlier calls
    HIP_CHECK(hipMemsetAsync(hist_counter.p, 0, sizeof(int), s));
    auto record_norm = [&] {
        dot(r, r, sc + SC_RN, true);
        launch_append(s, sc + SC_RN, hist.p, hist_counter.p);
    };
    auto step = [&] {  // q = A p; alpha = rz / pq; x += alpha p; r -= alpha q; ||r||
        par_apply(A, KM_SPMV, p, nullptr, q, 0.0, nullptr);
        dot(p, q, sc + SC_PQ, false);
        launch_pcg_xr(s, n, sc + SC_RZ, sc + SC_PQ, p, q, x, r);
        record_norm();
    };
    auto prec = [&] {  // z = M^-1 r (one V-cycle from z = 0); beta = rz_new / rz; p = z + beta p
        launch_zero(s, n, z);
        cycle_rec(0, z, r, false, false);
        dot(r, z, sc + SC_RZN, false);
        launch_pcg_p(s, n, sc + SC_RZN, sc + SC_RZ, z, p);
        HIP_CHECK(hipMemcpyAsync(sc + SC_RZ, sc + SC_RZN, sizeof(double), hipMemcpyDeviceToDevice, s));
    };
    par_apply(A, KM_RESID, x, b, r, 0.0, nullptr);
    record_norm();
    double r0 = 0.0;
    if (tol > 0.0) {
        HIP_CHECK(hipMemcpyAsync(&r0, hist.p, sizeof(double), hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
    }
    launch_zero(s, n, z);
    cycle_rec(0, z, r, false, false);
    if (n) HIP_CHECK(hipMemcpyAsync(p, z, n * sizeof(double), hipMemcpyDeviceToDevice, s));
    dot(r, z, sc + SC_RZ, false);
    // one collective graph decision for both iteration graphs (keyed by the caller's x, b)
    agree_stale({G_PCG_STEP, G_PCG_PREC}, x, b);
    auto run = [&](int slot, const std::function<void()>& body) {
        if (use_graph && graph_ready(slot, x, b, body, false)) graph_launch(slot);
        else body();
    };
    int32_t it = 0;
    while (it < max_iter) {
        run(G_PCG_STEP, step);
        ++it;
        if (tol > 0.0) {
            double rn = 0.0;
            HIP_CHECK(hipMemcpyAsync(&rn, hist.p + it, sizeof(double), hipMemcpyDeviceToHost, s));
            HIP_CHECK(hipStreamSynchronize(s));
            ctx->graph_inflight = false;
            if (r0 > 0.0 && rn / r0 < tol) break;
        }
        if (it == max_iter) break;
        run(G_PCG_PREC, prec);
    }
    HIP_CHECK(hipMemcpyAsync(hist_host, hist.p, sizeof(double) * (size_t)(it + 1),
                             hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    ctx->graph_inflight = false;
    return it;
}

static int64_t spmv_bytes(const DevMatrix& M) {
    return 12 * M.nnz + 4 * (M.n_rows + 1) + 8 * M.n_cols_local + 8 * M.n_rows;
}

int64_t Solver::bytes_per_cycle(size_t l) const {
    Solver& me = *const_cast<Solver*>(this);
    const DevMatrix& A = me.CA(l);
    const int64_t n = A.n_rows;
    if (l + 1 == levels.size()) return 8 * coarse_n * n + 8 * coarse_n + 8 * n;
    const int64_t base = 12 * A.nnz + 4 * (n + 1);
    const int64_t jac = base + 32 * n;
    int64_t b = 0;
    bool zero = l > 0;
    int64_t sweeps = 0;
    for (int k = 0; k < opt.pre_sweeps; ++k, ++sweeps) {
        if (zero && opt.smoother == AMG_SMOOTH_JACOBI) b += 24 * n;
        else b += jac + (zero ? 8 * n : 0);
        zero = false;
    }
    if (zero) b += 8 * n;
    b += base + 24 * n;                                   // residual
    b += spmv_bytes(me.CR(l));                            // restriction
    b += spmv_bytes(me.CP(l)) + 8 * n;                    // interpolation (reads x)
    b += opt.post_sweeps * jac;
    sweeps += opt.post_sweeps;
    if (sweeps % 2 == 1) b += 16 * n;                     // copy back
    return b;
}

}  // namespace amg

namespace amg {

// Mirrors cycle_rec(): per operation the stored-format bytes of the kernel that runs it
// (DevMatrix::mode_bytes, the sliced-ELL stream for hybrid GS), plus the vector-only passes.
int64_t Solver::stored_bytes_per_cycle(size_t l) const {
    Solver& me = *const_cast<Solver*>(this);
    const DevMatrix& A = me.CA(l);  // the operators the cycle runs
    const int64_t n = A.n_rows;
    if (l + 1 == levels.size()) return 8 * coarse_n * n + 8 * coarse_n + 8 * n;
    const bool gs = opt.smoother == AMG_SMOOTH_HYBRID_GS;
    const int64_t sweep = gs ? A.gs_bytes : A.mode_bytes(KM_JACOBI);
    int64_t b = 0;
    bool zero = l > 0;
    int64_t sweeps = 0;
    // the sweep from zero fused into the restriction above (cycle_rec): dinv read + x write
    const DevMatrix* Rup = l > 0 ? &me.CR(l - 1) : nullptr;
    const bool j0 = !gs && Rup && (int)l != rep_level && Rup->format != AMG_FORMAT_CSR &&
                    !Rup->tpl_on();
    // a split GS sweep from zero is its chain walk alone (par_hybrid_gs_from_zero)
    const int64_t sweep0 = gs && A.gs_split ? sweep - A.gs_old[1]->mode_bytes(KM_RESID) - 8 * n : sweep;
    for (int k = 0; k < opt.pre_sweeps; ++k, ++sweeps) {
        if (zero && !gs) b += (j0 ? 16 : 24) * n;  // omega * dinv * b
        else b += (zero ? sweep0 : sweep) + (zero ? 8 * n : 0);  // (zero fill of x first)
        zero = false;
    }
    if (zero) b += 8 * n;
    b += A.mode_bytes(KM_RESID);
    b += me.CR(l).mode_bytes(KM_SPMV);
    b += me.CP(l).mode_bytes(KM_SPMV_ADD);
    b += opt.post_sweeps * sweep;
    sweeps += opt.post_sweeps;
    if (sweeps % 2 == 1) b += 16 * n;  // copy back
    return b;
}

}  // namespace amg
