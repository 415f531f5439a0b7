// loopback.hip -- in-process multi-rank transport (testing the multi-rank device path on
// one GPU).  N contexts in one process, one thread each, share a device; the halo
// exchange and allgathers are D2D copies ordered by events, with host barriers making the
// events of every rank visible; the setup exchange is an in-process all-to-all-v.
// The RCCL transport (par_matrix.hip) is the production path; both drive the same halo
// plans, pack kernels, interior/boundary overlap and coarse/norm allgathers.
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>

#include <cstdio>
#include <cstdlib>
#include <omp.h>

#include "device.hpp"

namespace amg {

struct LoopbackWorld {
    int nranks = 0;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    std::vector<hipEvent_t> ev_pack, ev_done;
    std::vector<const char*> h_send;
    std::vector<std::vector<int64_t>> h_sbytes;
    std::vector<const double*> ag_send;
    struct Reg {
        const double* send_buf = nullptr;
        std::vector<int> send_procs;
        std::vector<int64_t> send_ptr;
    };
    std::map<std::pair<int64_t, int>, Reg> mats;

    void barrier() {
        std::unique_lock<std::mutex> lk(m);
        const uint64_t g = gen;
        if (++arrived == nranks) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return;
        }
        // AMG_LOOPBACK_TIMEOUT (seconds, default 120): full-size runs (512^3 over 8 ranks)
        // spend minutes in the host setup between two collectives
        const char* e = std::getenv("AMG_LOOPBACK_TIMEOUT");
        const int secs = e && std::atoi(e) > 0 ? std::atoi(e) : 120;
        if (!cv.wait_for(lk, std::chrono::seconds(secs), [&] { return gen != g; }))
            throw Error(AMG_ERR_COMM, "loopback barrier timed out (a peer rank failed?)");
    }
};

namespace {
std::mutex g_worlds_m;
std::map<std::string, std::weak_ptr<LoopbackWorld>> g_worlds;

struct LbUser {
    LoopbackWorld* w;
    int rank;
};

int lb_alltoallv(void* user, const void* send, const int64_t* sb, void* recv, const int64_t* rb) {
    try {
        LbUser* u = static_cast<LbUser*>(user);
        LoopbackWorld& W = *u->w;
        const int r = u->rank, n = W.nranks;
        W.h_send[r] = static_cast<const char*>(send);
        W.h_sbytes[r].assign(sb, sb + n);
        W.barrier();
        char* out = static_cast<char*>(recv);
        int rc = 0;
        for (int q = 0; q < n; ++q) {
            int64_t off = 0;
            for (int t = 0; t < r; ++t) off += W.h_sbytes[q][t];
            const int64_t len = W.h_sbytes[q][r];
            if (len != rb[q]) rc = 1;
            else if (len) std::memcpy(out, W.h_send[q] + off, (size_t)len);
            out += rb[q];
        }
        W.barrier();
        return rc;
    } catch (...) {
        return 1;
    }
}
}  // namespace

void loopback_join(Context& c, int rank, int nranks, const std::string& name) {
    std::shared_ptr<LoopbackWorld> w;
    {
        std::lock_guard<std::mutex> lk(g_worlds_m);
        w = g_worlds[name].lock();
        if (!w) {
            w = std::make_shared<LoopbackWorld>();
            w->nranks = nranks;
            w->ev_pack.assign(nranks, nullptr);
            w->ev_done.assign(nranks, nullptr);
            w->h_send.assign(nranks, nullptr);
            w->h_sbytes.assign(nranks, {});
            w->ag_send.assign(nranks, nullptr);
            g_worlds[name] = w;
        }
    }
    AMG_CHECK(w->nranks == nranks, "loopback world joined with a different size");
    {
        std::lock_guard<std::mutex> lk(w->m);
        AMG_CHECK(w->ev_pack[rank] == nullptr, "loopback rank joined twice");
        HIP_CHECK(hipEventCreateWithFlags(&w->ev_pack[rank], hipEventDisableTiming));
        HIP_CHECK(hipEventCreateWithFlags(&w->ev_done[rank], hipEventDisableTiming));
    }
    HIP_CHECK(hipEventRecord(w->ev_pack[rank], c.stream));
    HIP_CHECK(hipEventRecord(w->ev_done[rank], c.stream));
    c.lb = w;
    c.lb_user = new LbUser{w.get(), rank};
    c.host.rank = rank;
    c.host.nranks = nranks;
    c.host.fn = lb_alltoallv;
    c.host.user = c.lb_user;
    c.transport = TR_LOOPBACK;
    // the ranks' host loops share the process's cores: each rank thread forks teams of
    // 1/nranks of them (this thread's OpenMP setting only), not nranks full teams
    c.lb_omp_threads = omp_get_max_threads();
    c.lb_thread = std::this_thread::get_id();
    omp_set_num_threads(std::max(1, c.lb_omp_threads / nranks));
    w->barrier();  // every rank's events exist before anyone waits on them
}

void loopback_leave(Context& c) {
    if (!c.lb) return;
    if (c.lb_omp_threads > 0 && c.lb_thread == std::this_thread::get_id()) omp_set_num_threads(c.lb_omp_threads);
    delete static_cast<LbUser*>(c.lb_user);
    c.lb_user = nullptr;
    c.lb.reset();
}

void loopback_register(Context& c, int64_t seq, const double* send_buf,
                       const std::vector<int>& send_procs, const std::vector<int64_t>& send_ptr) {
    LoopbackWorld& W = *c.lb;
    std::lock_guard<std::mutex> lk(W.m);
    auto& r = W.mats[{seq, c.host.rank}];
    r.send_buf = send_buf;
    r.send_procs = send_procs;
    r.send_ptr = send_ptr;
}

// called after the caller packed x into send_buf on c.stream
void loopback_halo(Context& c, int64_t seq, const double* /*send_buf*/, double* halo,
                   const std::vector<int>& send_procs, const std::vector<int>& recv_procs,
                   const std::vector<int64_t>& recv_ptr, bool /*packed*/) {
    LoopbackWorld& W = *c.lb;
    const int me = c.host.rank;
    (void)send_procs;
    HIP_CHECK(hipEventRecord(W.ev_pack[me], c.stream));
    W.barrier();
    // my previous boundary kernels (before my pack on c.stream) finish before halo is reused
    HIP_CHECK(hipStreamWaitEvent(c.comm_stream, W.ev_pack[me], 0));
    for (size_t i = 0; i < recv_procs.size(); ++i) {
        const int p = recv_procs[i];
        const LoopbackWorld::Reg* reg;
        {
            std::lock_guard<std::mutex> lk(W.m);
            auto it = W.mats.find({seq, p});
            AMG_ASSERT(it != W.mats.end());
            reg = &it->second;
        }
        size_t j = 0;
        while (j < reg->send_procs.size() && reg->send_procs[j] != me) ++j;
        AMG_ASSERT(j < reg->send_procs.size());
        const int64_t cnt = recv_ptr[i + 1] - recv_ptr[i];
        AMG_ASSERT(cnt == reg->send_ptr[j + 1] - reg->send_ptr[j]);
        HIP_CHECK(hipStreamWaitEvent(c.comm_stream, W.ev_pack[p], 0));
        if (cnt)
            HIP_CHECK(hipMemcpyAsync(halo + recv_ptr[i], reg->send_buf + reg->send_ptr[j],
                                     (size_t)cnt * sizeof(double), hipMemcpyDeviceToDevice,
                                     c.comm_stream));
    }
    HIP_CHECK(hipEventRecord(W.ev_done[me], c.comm_stream));
    HIP_CHECK(hipEventRecord(c.ev_halo, c.comm_stream));
    W.barrier();
}

// before re-packing a send buffer: readers of my previous round must be done with it
void loopback_before_pack(Context& c, const std::vector<int>& send_procs) {
    LoopbackWorld& W = *c.lb;
    for (int q : send_procs) HIP_CHECK(hipStreamWaitEvent(c.stream, W.ev_done[q], 0));
}

// Graph-launched and eager RCCL work on one communicator: an eager group or
// allgather enqueued while replayed groups are still in flight never completed on ROCm 7.2's
// RCCL (profiles/r4_rccl_graph_probe.txt), so the first eager RCCL enqueue after replays waits
// for them.  AMG_RCCL_EAGER_FENCE=0 drops the wait (the probe that reproduces the hang).
void Context::eager_rccl_fence() {
    if (!graph_inflight || capturing) return;
    static const bool on = [] {
        const char* e = std::getenv("AMG_RCCL_EAGER_FENCE");
        return !(e && *e && std::atoi(e) == 0);
    }();
    graph_inflight = false;
    if (!on) return;
    static const bool trace = std::getenv("AMG_TRACE_RCCL") != nullptr;
    if (trace) std::fprintf(stderr, "[amg] rank %d eager fence (waiting for replays)\n", host.rank);
    HIP_CHECK(hipStreamSynchronize(stream));
}

void Context::allgather(const double* send, double* recv, size_t count) {
    if (transport == TR_RCCL) {
        eager_rccl_fence();
        static const bool trace = std::getenv("AMG_TRACE_RCCL") != nullptr;
        if (trace) std::fprintf(stderr, "[amg] rank %d allgather %zu\n", host.rank, count);
        NCCL_CHECK(ncclAllGather(send, recv, count, ncclDouble, nccl, stream));
        if (trace) std::fprintf(stderr, "[amg] rank %d allgather enqueued\n", host.rank);
        return;
    }
    if (transport != TR_LOOPBACK) {
        if (count) HIP_CHECK(hipMemcpyAsync(recv, send, count * sizeof(double), hipMemcpyDeviceToDevice, stream));
        return;
    }
    LoopbackWorld& W = *lb;
    const int me = host.rank;
    W.ag_send[me] = send;
    HIP_CHECK(hipEventRecord(W.ev_pack[me], stream));
    W.barrier();
    for (int q = 0; q < W.nranks; ++q) {
        HIP_CHECK(hipStreamWaitEvent(stream, W.ev_pack[q], 0));
        if (count)
            HIP_CHECK(hipMemcpyAsync(recv + (size_t)q * count, W.ag_send[q], count * sizeof(double),
                                     hipMemcpyDeviceToDevice, stream));
    }
    HIP_CHECK(hipEventRecord(W.ev_done[me], stream));
    W.barrier();
    // nobody overwrites its send slot before every rank copied it
    for (int q = 0; q < W.nranks; ++q) HIP_CHECK(hipStreamWaitEvent(stream, W.ev_done[q], 0));
}

}  // namespace amg
