// host_comm.cpp -- setup-time exchange layer, halo plans (ParComm), ghost rows,
// distributed transpose and SpGEMM, model-problem slabs.  SURVEY.md 8a rows a1, a10, a11.
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "host.hpp"


// LLVM libomp extension (the library links libomp); weak, so a host-only build against
// another OpenMP runtime (the sanitizer build with libgomp) just skips it
extern "C" void kmp_set_blocktime(int) __attribute__((weak));
extern "C" int kmp_get_blocktime(void) __attribute__((weak));

namespace amg {

static bool omp_quiet_wanted() {
    static const bool on = [] {
        const char* e = std::getenv("KMP_BLOCKTIME");
        return !(e && *e) && kmp_set_blocktime && kmp_get_blocktime;
    }();
    return on;
}

void omp_quiet_thread() {
    thread_local bool done = false;
    if (done || !omp_quiet_wanted()) return;
    done = true;
    kmp_set_blocktime(0);
}

OmpQuiet::OmpQuiet() {
    if (!omp_quiet_wanted()) return;
    saved = kmp_get_blocktime();
    if (saved != 0) kmp_set_blocktime(0);
}

OmpQuiet::~OmpQuiet() {
    if (saved > 0) kmp_set_blocktime(saved);
}


uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
uint32_t hash32(int64_t gid, uint64_t seed) {
    return (uint32_t)(mix64((uint64_t)gid ^ (seed * 0x9E3779B97F4A7C15ull)) >> 32);
}

static double wall_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}
bool PhaseTimer::enabled() {
    static const bool on = [] {
        const char* e = std::getenv("AMG_TIMING");
        return e && *e && *e != '0';
    }();
    return on;
}
PhaseTimer::PhaseTimer(const HostComm& comm) : rank(comm.rank), t0(wall_ms()) {}
void PhaseTimer::lap(const std::string& label) {
    const double t = wall_ms();
    if (enabled() && rank == 0) std::fprintf(stderr, "[amg] %-28s %9.1f ms\n", label.c_str(), t - t0);
    t0 = t;
}

// ----------------------------------------------------------------------------------
// HostComm
// ----------------------------------------------------------------------------------
void HostComm::alltoallv(const void* send, const std::vector<int64_t>& sbytes, void* recv,
                         const std::vector<int64_t>& rbytes) const {
    AMG_ASSERT((int)sbytes.size() == nranks && (int)rbytes.size() == nranks);
    if (nranks == 1) {
        AMG_ASSERT(sbytes[0] == rbytes[0]);
        if (sbytes[0]) std::memcpy(recv, send, (size_t)sbytes[0]);
        return;
    }
    if (!fn) throw Error(AMG_ERR_COMM, "multi-rank setup needs a host exchange callback");
    int rc = fn(user, send, sbytes.data(), recv, rbytes.data());
    if (rc != 0) throw Error(AMG_ERR_COMM, "host exchange callback failed");
}

std::vector<int64_t> HostComm::alltoall_counts(const std::vector<int64_t>& counts) const {
    std::vector<int64_t> out(nranks), b(nranks, 8);
    alltoallv(counts.data(), b, out.data(), b);
    return out;
}

template <class T>
std::vector<std::vector<T>> HostComm::exchange(const std::vector<std::vector<T>>& send) const {
    AMG_ASSERT((int)send.size() == nranks);
    std::vector<int64_t> cnt(nranks), sb(nranks), rb(nranks);
    size_t tot = 0;
    for (int r = 0; r < nranks; ++r) cnt[r] = (int64_t)send[r].size(), tot += send[r].size();
    std::vector<int64_t> rc = alltoall_counts(cnt);
    std::vector<T> sbuf(tot);
    size_t o = 0;
    for (int r = 0; r < nranks; ++r) {
        std::copy(send[r].begin(), send[r].end(), sbuf.begin() + o);
        o += send[r].size();
        sb[r] = cnt[r] * (int64_t)sizeof(T);
        rb[r] = rc[r] * (int64_t)sizeof(T);
    }
    size_t rtot = 0;
    for (int r = 0; r < nranks; ++r) rtot += (size_t)rc[r];
    std::vector<T> rbuf(rtot);
    alltoallv(sbuf.data(), sb, rbuf.data(), rb);
    std::vector<std::vector<T>> out(nranks);
    o = 0;
    for (int r = 0; r < nranks; ++r) {
        out[r].assign(rbuf.begin() + o, rbuf.begin() + o + rc[r]);
        o += (size_t)rc[r];
    }
    return out;
}
template std::vector<std::vector<int64_t>> HostComm::exchange(
    const std::vector<std::vector<int64_t>>&) const;
template std::vector<std::vector<double>> HostComm::exchange(
    const std::vector<std::vector<double>>&) const;
template std::vector<std::vector<int32_t>> HostComm::exchange(
    const std::vector<std::vector<int32_t>>&) const;

std::vector<int64_t> HostComm::allgather(int64_t v) const {
    std::vector<int64_t> s(nranks, v);
    return alltoall_counts(s);
}
std::vector<double> HostComm::allgather(double v) const {
    std::vector<double> s(nranks, v), out(nranks);
    std::vector<int64_t> b(nranks, 8);
    alltoallv(s.data(), b, out.data(), b);
    return out;
}
int64_t HostComm::allreduce_sum(int64_t v) const {
    int64_t s = 0;
    for (int64_t x : allgather(v)) s += x;
    return s;
}
double HostComm::allreduce_max(double v) const {
    std::vector<double> a = allgather(v);
    double m = a[0];
    for (double x : a) m = x > m ? x : m;
    return m;
}

int owner_of(const std::vector<int64_t>& starts, int64_t g) {
    // starts is nondecreasing; owner = last r with starts[r] <= g < starts[r+1]
    auto it = std::upper_bound(starts.begin(), starts.end(), g);
    int r = (int)(it - starts.begin()) - 1;
    while (r + 1 < (int)starts.size() - 1 && starts[r + 1] <= g) ++r;
    AMG_ASSERT(r >= 0 && r < (int)starts.size() - 1 && g < starts[r + 1]);
    return r;
}

// ----------------------------------------------------------------------------------
// HaloPlan
// ----------------------------------------------------------------------------------
int64_t HaloPlan::find(int64_t gid) const {
    auto it = std::lower_bound(halo_gid.begin(), halo_gid.end(), gid);
    if (it == halo_gid.end() || *it != gid) return -1;
    return (int64_t)(it - halo_gid.begin());
}

HaloPlan build_halo_plan(const HostComm& comm, const std::vector<int64_t>& starts,
                         std::vector<int64_t> needed) {
    HaloPlan P;
    std::sort(needed.begin(), needed.end());
    needed.erase(std::unique(needed.begin(), needed.end()), needed.end());
    P.halo_gid = std::move(needed);
    std::vector<std::vector<int64_t>> req(comm.nranks);
    P.recv_ptr.push_back(0);
    for (size_t t = 0; t < P.halo_gid.size(); ++t) {
        int o = owner_of(starts, P.halo_gid[t]);
        AMG_ASSERT(o != comm.rank);
        if (P.recv_procs.empty() || P.recv_procs.back() != o) {
            if (!P.recv_procs.empty()) P.recv_ptr.push_back((int64_t)t);
            P.recv_procs.push_back(o);
        }
        req[o].push_back(P.halo_gid[t]);
    }
    if (!P.recv_procs.empty()) P.recv_ptr.push_back((int64_t)P.halo_gid.size());
    auto got = comm.exchange(req);
    P.send_ptr.push_back(0);
    int64_t lo = starts[comm.rank];
    for (int r = 0; r < comm.nranks; ++r) {
        if (got[r].empty()) continue;
        P.send_procs.push_back(r);
        for (int64_t g : got[r]) {
            AMG_ASSERT(g >= lo && g < starts[comm.rank + 1]);
            P.send_idx.push_back(g - lo);
        }
        P.send_ptr.push_back((int64_t)P.send_idx.size());
    }
    return P;
}

HaloPlan halo_plan_for_cols(const HostComm& comm, const HostCSR& A) {
    int64_t lo = A.col_starts[comm.rank], hi = A.col_starts[comm.rank + 1];
    // off-process columns, collected per chunk in parallel and concatenated in order
    const int64_t nz = (int64_t)A.col.size();
    const int nch = (int)std::max<int64_t>(1, std::min<int64_t>(256, nz / (1 << 20)));
    std::vector<std::vector<int64_t>> part((size_t)nch);
#pragma omp parallel for schedule(dynamic, 1)
    for (int c = 0; c < nch; ++c)
        for (int64_t k = nz * c / nch; k < nz * (c + 1) / nch; ++k)
            if (A.col[k] < lo || A.col[k] >= hi) part[(size_t)c].push_back(A.col[k]);
    std::vector<int64_t> need;
    for (auto& p : part) need.insert(need.end(), p.begin(), p.end());
    return build_halo_plan(comm, A.col_starts, std::move(need));
}

template <class T>
void HaloPlan::forward(const HostComm& comm, const T* local, T* halo) const {
    std::vector<int64_t> sb(comm.nranks, 0), rb(comm.nranks, 0);
    std::vector<T> sbuf(send_idx.size());
    for (size_t t = 0; t < send_idx.size(); ++t) sbuf[t] = local[send_idx[t]];
    for (size_t p = 0; p < send_procs.size(); ++p)
        sb[send_procs[p]] = (send_ptr[p + 1] - send_ptr[p]) * (int64_t)sizeof(T);
    for (size_t p = 0; p < recv_procs.size(); ++p)
        rb[recv_procs[p]] = (recv_ptr[p + 1] - recv_ptr[p]) * (int64_t)sizeof(T);
    comm.alltoallv(sbuf.data(), sb, halo, rb);
}
template void HaloPlan::forward(const HostComm&, const int32_t*, int32_t*) const;
template void HaloPlan::forward(const HostComm&, const int64_t*, int64_t*) const;
template void HaloPlan::forward(const HostComm&, const uint64_t*, uint64_t*) const;
template void HaloPlan::forward(const HostComm&, const double*, double*) const;

GhostRows fetch_rows(const HostComm& comm, const HaloPlan& plan, const HostCSR& B) {
    GhostRows G;
    int64_t nl = B.nrows();
    std::vector<int64_t> len(nl);
    for (int64_t i = 0; i < nl; ++i) len[i] = B.rp[i + 1] - B.rp[i];
    std::vector<int64_t> hlen(plan.n_halo());
    plan.forward(comm, len.data(), hlen.data());
    G.rp.assign(plan.n_halo() + 1, 0);
    for (int64_t t = 0; t < plan.n_halo(); ++t) G.rp[t + 1] = G.rp[t] + hlen[t];
    // entries: one exchange of (col, val) pairs packed as 16-byte records
    struct Rec {
        int64_t c;
        double v;
    };
    std::vector<int64_t> sb(comm.nranks, 0), rb(comm.nranks, 0);
    std::vector<Rec> sbuf;
    for (size_t p = 0; p < plan.send_procs.size(); ++p) {
        size_t before = sbuf.size();
        for (int64_t t = plan.send_ptr[p]; t < plan.send_ptr[p + 1]; ++t) {
            int64_t i = plan.send_idx[t];
            for (int64_t k = B.rp[i]; k < B.rp[i + 1]; ++k) sbuf.push_back({B.col[k], B.val[k]});
        }
        sb[plan.send_procs[p]] = (int64_t)((sbuf.size() - before) * sizeof(Rec));
    }
    for (size_t p = 0; p < plan.recv_procs.size(); ++p)
        rb[plan.recv_procs[p]] =
            (G.rp[plan.recv_ptr[p + 1]] - G.rp[plan.recv_ptr[p]]) * (int64_t)sizeof(Rec);
    std::vector<Rec> rbuf(G.rp.back());
    comm.alltoallv(sbuf.data(), sb, rbuf.data(), rb);
    G.col.resize(rbuf.size());
    G.val.resize(rbuf.size());
    for (size_t t = 0; t < rbuf.size(); ++t) G.col[t] = rbuf[t].c, G.val[t] = rbuf[t].v;
    return G;
}

// ----------------------------------------------------------------------------------
// Distributed transpose: R = P^T.  Entries (J, i, v) go to owner(J) as 24-byte records in ONE
// exchange; each rank's records leave in ascending i, the received buffers are placed in rank
// order => every row of R is in ascending global column.  Bucketing and placement run as
// OpenMP loops (per-thread counts, then exclusive offsets: the record order equals the serial
// loop's), so the host part stays a small fraction of the exchange on N ranks.
// ----------------------------------------------------------------------------------
HostCSR transpose(const HostComm& comm, const HostCSR& P) {
    struct Rec {
        int64_t j, i;
        double v;
    };
    HostCSR R;
    R.n_global_rows = P.n_global_cols;
    R.n_global_cols = P.n_global_rows;
    R.row_starts = P.col_starts;
    R.col_starts = P.row_starts;
    const int nr = comm.nranks;
    const int64_t i0 = P.row_starts[comm.rank], n = P.nrows();
    const int nt = std::max(1, std::min(omp_get_max_threads(), (int)(n / 4096 + 1)));
    // owner of every entry, and per (thread, owner) counts over contiguous row ranges
    std::vector<int> own((size_t)P.nnz());
    std::vector<int64_t> tc((size_t)nt * nr, 0);
#pragma omp parallel num_threads(nt)
    {
        const int t = omp_get_thread_num();
        const int64_t r0 = n * t / nt, r1 = n * (t + 1) / nt;
        int64_t* c = tc.data() + (size_t)t * nr;
        for (int64_t k = P.rp[r0]; k < P.rp[r1]; ++k) {
            const int o = owner_of(P.col_starts, P.col[k]);
            own[k] = o;
            ++c[o];
        }
    }
    // record offsets: owner-major, thread order inside an owner (= ascending i)
    std::vector<int64_t> off((size_t)nt * nr), sb(nr, 0);
    int64_t pos = 0;
    for (int o = 0; o < nr; ++o) {
        for (int t = 0; t < nt; ++t) {
            off[(size_t)t * nr + o] = pos;
            pos += tc[(size_t)t * nr + o];
        }
        sb[o] = 0;
    }
    std::vector<Rec> sbuf((size_t)pos);
#pragma omp parallel num_threads(nt)
    {
        const int t = omp_get_thread_num();
        const int64_t r0 = n * t / nt, r1 = n * (t + 1) / nt;
        int64_t* w = off.data() + (size_t)t * nr;
        for (int64_t i = r0; i < r1; ++i)
            for (int64_t k = P.rp[i]; k < P.rp[i + 1]; ++k) sbuf[(size_t)w[own[k]]++] = {P.col[k], i0 + i, P.val[k]};
    }
    std::vector<int64_t> cnt(nr, 0);
    for (int o = 0; o < nr; ++o)
        for (int t = 0; t < nt; ++t) cnt[o] += tc[(size_t)t * nr + o];
    const std::vector<int64_t> rcnt = comm.alltoall_counts(cnt);
    std::vector<int64_t> rb(nr);
    int64_t rtot = 0;
    for (int o = 0; o < nr; ++o) {
        sb[o] = cnt[o] * (int64_t)sizeof(Rec);
        rb[o] = rcnt[o] * (int64_t)sizeof(Rec);
        rtot += rcnt[o];
    }
    std::vector<Rec> rbuf((size_t)rtot);
    comm.alltoallv(sbuf.data(), sb, rbuf.data(), rb);
    std::vector<Rec>().swap(sbuf);
    const int64_t lo = R.row_starts[comm.rank], m = R.row_starts[comm.rank + 1] - lo;
    R.rp.assign(m + 1, 0);
    for (const Rec& e : rbuf) R.rp[e.j - lo + 1]++;
    for (int64_t t = 0; t < m; ++t) R.rp[t + 1] += R.rp[t];
    R.col.resize(R.rp[m]);
    R.val.resize(R.rp[m]);
    // placement in received order (rank order, ascending i inside a rank)
    std::vector<int64_t> at(R.rp.begin(), R.rp.end() - 1);
    for (const Rec& e : rbuf) {
        const int64_t p = at[e.j - lo]++;
        R.col[p] = e.i;
        R.val[p] = e.v;
    }
    return R;
}

// ----------------------------------------------------------------------------------
// SpGEMM C = A * B (local rows of A; rows of B partitioned by A.col_starts).
// Canonical order: acc_j = 0.0; for k in A row (ascending global col), for j
// in B row k (ascending): acc_j += a_ik * b_kj.  Pattern = structural union, cols sorted.
// ----------------------------------------------------------------------------------
HostCSR spgemm(const HostComm& comm, const HostCSR& A, const HostCSR& B) {
    AMG_CHECK(A.col_starts == B.row_starts, "spgemm: A columns and B rows partitioned differently");
    HaloPlan plan = halo_plan_for_cols(comm, A);
    GhostRows G = fetch_rows(comm, plan, B);
    int64_t n = A.nrows(), lo = B.row_starts[comm.rank], hi = B.row_starts[comm.rank + 1];
    // locate B row of every A entry: >= 0 local row, < 0 ghost -(t+1)
    std::vector<int64_t> loc(A.nnz());
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < A.nnz(); ++k) {
        int64_t c = A.col[k];
        loc[k] = (c >= lo && c < hi) ? c - lo : -(plan.find(c) + 1);
    }
    int nt = omp_get_max_threads();
    std::vector<std::vector<int64_t>> tcol(nt), tlen(nt);
    std::vector<std::vector<double>> tval(nt);
#pragma omp parallel num_threads(nt)
    {
        int t = omp_get_thread_num(), T = omp_get_num_threads();
        int64_t r0 = n * t / T, r1 = n * (t + 1) / T;
        std::vector<int64_t> hkey, hslot, order;
        std::vector<double> acc;
        auto& oc = tcol[t];
        auto& ov = tval[t];
        auto& ol = tlen[t];
        for (int64_t i = r0; i < r1; ++i) {
            int64_t ub = 0;
            for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
                int64_t l = loc[k];
                ub += l >= 0 ? B.rp[l + 1] - B.rp[l] : G.rp[-l] - G.rp[-l - 1];
            }
            size_t cap = 16;
            while (cap < (size_t)(2 * ub)) cap <<= 1;
            if (hkey.size() < cap) hkey.resize(cap), hslot.resize(cap);
            std::fill(hkey.begin(), hkey.begin() + cap, (int64_t)-1);
            order.clear();
            acc.clear();
            for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
                int64_t l = loc[k];
                double a = A.val[k];
                const int64_t* bc;
                const double* bv;
                int64_t bl;
                if (l >= 0) {
                    bc = &B.col[B.rp[l]], bv = &B.val[B.rp[l]], bl = B.rp[l + 1] - B.rp[l];
                } else {
                    int64_t g = -l - 1;
                    bc = &G.col[G.rp[g]], bv = &G.val[G.rp[g]], bl = G.rp[g + 1] - G.rp[g];
                }
                for (int64_t q = 0; q < bl; ++q) {
                    int64_t j = bc[q];
                    size_t h = (size_t)(mix64((uint64_t)j) & (cap - 1));
                    while (hkey[h] != -1 && hkey[h] != j) h = (h + 1) & (cap - 1);
                    if (hkey[h] == -1) {
                        hkey[h] = j;
                        hslot[h] = (int64_t)acc.size();
                        order.push_back(j);
                        acc.push_back(0.0);
                    }
                    acc[hslot[h]] += a * bv[q];
                }
            }
            // emit sorted by column
            std::vector<int64_t> idx(order.size());
            std::iota(idx.begin(), idx.end(), 0);
            std::sort(idx.begin(), idx.end(), [&](int64_t x, int64_t y) { return order[x] < order[y]; });
            for (int64_t s : idx) {
                oc.push_back(order[s]);
                ov.push_back(acc[s]);
            }
            ol.push_back((int64_t)idx.size());
        }
    }
    HostCSR C;
    C.n_global_rows = A.n_global_rows;
    C.n_global_cols = B.n_global_cols;
    C.row_starts = A.row_starts;
    C.col_starts = B.col_starts;
    C.rp.assign(n + 1, 0);
    int64_t r = 0;
    for (int t = 0; t < nt; ++t)
        for (int64_t l : tlen[t]) C.rp[r + 1] = C.rp[r] + l, ++r;
    AMG_ASSERT(r == n);
    C.col.reserve(C.rp[n]);
    C.val.reserve(C.rp[n]);
    for (int t = 0; t < nt; ++t) {
        C.col.insert(C.col.end(), tcol[t].begin(), tcol[t].end());
        C.val.insert(C.val.end(), tval[t].begin(), tval[t].end());
    }
    return C;
}

// ----------------------------------------------------------------------------------
// Model problems: rank r owns planes [r*nz/N, (r+1)*nz/N) (2D: lines of y).
// Values identical to oracle/amg_oracle.c generators.
// ----------------------------------------------------------------------------------
static double stencil27(int dx, int dy, int dz, double ex, double ey, double ez) {
    static const double K[3] = {-1.0, 2.0, -1.0};
    static const double m[3] = {1.0, 4.0, 1.0};
    double t1 = ex * K[dx + 1] * m[dy + 1] * m[dz + 1];
    double t2 = ey * m[dx + 1] * K[dy + 1] * m[dz + 1];
    double t3 = ez * m[dx + 1] * m[dy + 1] * K[dz + 1];
    return t1 + t2 + t3;
}

HostCSR stencil_slab(const HostComm& comm, int kind, int64_t nx, int64_t ny, int64_t nz,
                     const double* eps3) {
    AMG_CHECK(nx > 0 && ny > 0 && nz > 0, "stencil: grid dims must be positive");
    AMG_CHECK(kind != AMG_STENCIL_5PT || nz == 1, "5-pt stencil is 2D: nz must be 1");
    int64_t planes = kind == AMG_STENCIL_5PT ? ny : nz;
    int64_t pl = kind == AMG_STENCIL_5PT ? nx : nx * ny;
    HostCSR A;
    A.n_global_rows = A.n_global_cols = nx * ny * nz;
    A.row_starts.resize(comm.nranks + 1);
    for (int r = 0; r <= comm.nranks; ++r) A.row_starts[r] = (planes * r / comm.nranks) * pl;
    A.col_starts = A.row_starts;
    int64_t p0 = planes * comm.rank / comm.nranks, p1 = planes * (comm.rank + 1) / comm.nranks;
    int64_t nloc = (p1 - p0) * pl;
    int per = kind == AMG_STENCIL_5PT ? 5 : kind == AMG_STENCIL_7PT ? 7 : 27;
    A.rp.assign(nloc + 1, 0);
    // row lengths first (parallel fill needs offsets)
    auto inside = [&](int64_t i, int64_t j, int64_t k) {
        return i >= 0 && i < nx && j >= 0 && j < ny && k >= 0 && k < nz;
    };
    std::vector<int64_t> len(nloc);
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < nloc; ++t) {
        int64_t g = A.row_starts[comm.rank] + t;
        int64_t i = g % nx, j = (g / nx) % ny, k = g / (nx * ny);
        int64_t c = 0;
        if (kind == AMG_STENCIL_27PT) {
            for (int dz = -1; dz <= 1; ++dz)
                for (int dy = -1; dy <= 1; ++dy)
                    for (int dx = -1; dx <= 1; ++dx) c += inside(i + dx, j + dy, k + dz);
        } else {
            c = 1 + (i > 0) + (i < nx - 1) + (j > 0) + (j < ny - 1);
            if (kind == AMG_STENCIL_7PT) c += (k > 0) + (k < nz - 1);
        }
        len[t] = c;
    }
    for (int64_t t = 0; t < nloc; ++t) A.rp[t + 1] = A.rp[t] + len[t];
    A.col.resize(A.rp[nloc]);
    A.val.resize(A.rp[nloc]);
    double ex = eps3 ? eps3[0] : 1.0, ey = eps3 ? eps3[1] : 1.0, ez = eps3 ? eps3[2] : 1e-3;
    (void)per;
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < nloc; ++t) {
        int64_t g = A.row_starts[comm.rank] + t;
        int64_t i = g % nx, j = (g / nx) % ny, k = g / (nx * ny);
        int64_t q = A.rp[t];
        auto put = [&](int64_t c, double v) { A.col[q] = c, A.val[q] = v, ++q; };
        if (kind == AMG_STENCIL_27PT) {
            for (int dz = -1; dz <= 1; ++dz)
                for (int dy = -1; dy <= 1; ++dy)
                    for (int dx = -1; dx <= 1; ++dx)
                        if (inside(i + dx, j + dy, k + dz))
                            put(g + dx + nx * dy + nx * ny * dz, stencil27(dx, dy, dz, ex, ey, ez));
        } else if (kind == AMG_STENCIL_7PT) {
            if (k > 0) put(g - nx * ny, -1.0);
            if (j > 0) put(g - nx, -1.0);
            if (i > 0) put(g - 1, -1.0);
            put(g, 6.0);
            if (i < nx - 1) put(g + 1, -1.0);
            if (j < ny - 1) put(g + nx, -1.0);
            if (k < nz - 1) put(g + nx * ny, -1.0);
        } else {
            if (j > 0) put(g - nx, -1.0);
            if (i > 0) put(g - 1, -1.0);
            put(g, 4.0);
            if (i < nx - 1) put(g + 1, -1.0);
            if (j < ny - 1) put(g + nx, -1.0);
        }
    }
    return A;
}

// Box-ordered model problem (bench.py --gpus 8: 2 x 2 x 2 cubes of 256^3 instead of z-slabs
// of 512 x 512 x 64).  The grid is cut into bx x by x bz boxes (box (ix, iy, iz) covers
// x in [nx ix / bx, nx (ix + 1) / bx), ...), boxes are numbered x fastest, and each box's
// points get consecutive global ids in lexicographic order inside the box; rank r owns boxes
// [nb r / P, nb (r + 1) / P).  The matrix is P A P^T of the natural-order stencil (same
// values, rows with their columns sorted); boxes (1, 1, P) give exactly stencil_slab's rows.
HostCSR stencil_boxes(const HostComm& comm, int kind, int64_t nx, int64_t ny, int64_t nz, int64_t bx,
                      int64_t by, int64_t bz, const double* eps3) {
    AMG_CHECK(nx > 0 && ny > 0 && nz > 0, "stencil: grid dims must be positive");
    AMG_CHECK(kind != AMG_STENCIL_5PT || nz == 1, "5-pt stencil is 2D: nz must be 1");
    AMG_CHECK(bx >= 1 && by >= 1 && bz >= 1 && bx <= nx && by <= ny && bz <= nz, "stencil: bad box grid");
    const int64_t nb = bx * by * bz;
    AMG_CHECK(nb >= comm.nranks, "stencil: fewer boxes than ranks");
    // per axis: box of each coordinate and the coordinate inside it; box starts and widths
    auto axis = [](int64_t n, int64_t b, std::vector<int64_t>& box, std::vector<int64_t>& loc,
                   std::vector<int64_t>& start) {
        start.resize(b + 1);
        for (int64_t q = 0; q <= b; ++q) start[q] = n * q / b;
        box.resize(n);
        loc.resize(n);
        for (int64_t q = 0; q < b; ++q)
            for (int64_t i = start[q]; i < start[q + 1]; ++i) box[i] = q, loc[i] = i - start[q];
    };
    std::vector<int64_t> xb, xl, xs, yb, yl, ys, zb, zl, zs;
    axis(nx, bx, xb, xl, xs);
    axis(ny, by, yb, yl, ys);
    axis(nz, bz, zb, zl, zs);
    std::vector<int64_t> off(nb + 1, 0);
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t ix = b % bx, iy = (b / bx) % by, iz = b / (bx * by);
        off[b + 1] = off[b] + (xs[ix + 1] - xs[ix]) * (ys[iy + 1] - ys[iy]) * (zs[iz + 1] - zs[iz]);
    }
    auto gid = [&](int64_t i, int64_t j, int64_t k) {
        const int64_t ix = xb[i], iy = yb[j], iz = zb[k], b = ix + bx * (iy + by * iz);
        const int64_t wx = xs[ix + 1] - xs[ix], wy = ys[iy + 1] - ys[iy];
        return off[b] + xl[i] + wx * (yl[j] + wy * zl[k]);
    };
    HostCSR A;
    A.n_global_rows = A.n_global_cols = nx * ny * nz;
    A.row_starts.resize(comm.nranks + 1);
    for (int r = 0; r <= comm.nranks; ++r) A.row_starts[r] = off[nb * r / comm.nranks];
    A.col_starts = A.row_starts;
    const int64_t b0 = nb * comm.rank / comm.nranks, b1 = nb * (comm.rank + 1) / comm.nranks;
    const int64_t nloc = off[b1] - off[b0];
    // local row t -> (i, j, k): walk this rank's boxes
    std::vector<int64_t> pt((size_t)nloc);
    for (int64_t b = b0; b < b1; ++b) {
        const int64_t ix = b % bx, iy = (b / bx) % by, iz = b / (bx * by);
        const int64_t wx = xs[ix + 1] - xs[ix], wy = ys[iy + 1] - ys[iy], wz = zs[iz + 1] - zs[iz];
#pragma omp parallel for schedule(static)
        for (int64_t t = 0; t < wx * wy * wz; ++t) {
            const int64_t i = xs[ix] + t % wx, j = ys[iy] + (t / wx) % wy, k = zs[iz] + t / (wx * wy);
            pt[off[b] - off[b0] + t] = i + nx * (j + ny * k);  // natural id: decoded below
        }
    }
    auto inside = [&](int64_t i, int64_t j, int64_t k) {
        return i >= 0 && i < nx && j >= 0 && j < ny && k >= 0 && k < nz;
    };
    const double ex = eps3 ? eps3[0] : 1.0, ey = eps3 ? eps3[1] : 1.0, ez = eps3 ? eps3[2] : 1e-3;
    std::vector<int64_t> len((size_t)nloc);
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < nloc; ++t) {
        const int64_t g = pt[t], i = g % nx, j = (g / nx) % ny, k = g / (nx * ny);
        int64_t c = 0;
        if (kind == AMG_STENCIL_27PT) {
            for (int dz = -1; dz <= 1; ++dz)
                for (int dy = -1; dy <= 1; ++dy)
                    for (int dx = -1; dx <= 1; ++dx) c += inside(i + dx, j + dy, k + dz);
        } else {
            c = 1 + (i > 0) + (i < nx - 1) + (j > 0) + (j < ny - 1);
            if (kind == AMG_STENCIL_7PT) c += (k > 0) + (k < nz - 1);
        }
        len[t] = c;
    }
    A.rp.assign(nloc + 1, 0);
    for (int64_t t = 0; t < nloc; ++t) A.rp[t + 1] = A.rp[t] + len[t];
    A.col.resize(A.rp[nloc]);
    A.val.resize(A.rp[nloc]);
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < nloc; ++t) {
        const int64_t g = pt[t], i = g % nx, j = (g / nx) % ny, k = g / (nx * ny);
        int64_t q = A.rp[t];
        auto put = [&](int64_t ii, int64_t jj, int64_t kk, double v) { A.col[q] = gid(ii, jj, kk), A.val[q] = v, ++q; };
        if (kind == AMG_STENCIL_27PT) {
            for (int dz = -1; dz <= 1; ++dz)
                for (int dy = -1; dy <= 1; ++dy)
                    for (int dx = -1; dx <= 1; ++dx)
                        if (inside(i + dx, j + dy, k + dz)) put(i + dx, j + dy, k + dz, stencil27(dx, dy, dz, ex, ey, ez));
        } else if (kind == AMG_STENCIL_7PT) {
            if (k > 0) put(i, j, k - 1, -1.0);
            if (j > 0) put(i, j - 1, k, -1.0);
            if (i > 0) put(i - 1, j, k, -1.0);
            put(i, j, k, 6.0);
            if (i < nx - 1) put(i + 1, j, k, -1.0);
            if (j < ny - 1) put(i, j + 1, k, -1.0);
            if (k < nz - 1) put(i, j, k + 1, -1.0);
        } else {
            if (j > 0) put(i, j - 1, k, -1.0);
            if (i > 0) put(i - 1, j, k, -1.0);
            put(i, j, k, 4.0);
            if (i < nx - 1) put(i + 1, j, k, -1.0);
            if (j < ny - 1) put(i, j + 1, k, -1.0);
        }
        // columns ascending (a neighbour in another box may sit anywhere in the numbering)
        const int64_t b = A.rp[t], e = A.rp[t + 1];
        for (int64_t u = b + 1; u < e; ++u)
            for (int64_t w = u; w > b && A.col[w - 1] > A.col[w]; --w) {
                std::swap(A.col[w - 1], A.col[w]);
                std::swap(A.val[w - 1], A.val[w]);
            }
    }
    return A;
}

// ----------------------------------------------------------------------------------
// Replicated coarse levels: every rank gets all rows (rank order = global row order).
// ----------------------------------------------------------------------------------
HostCSR gather_global(const HostComm& comm, const HostCSR& M) {
    const int64_t n = M.nrows();
    std::vector<std::vector<int64_t>> sl(comm.nranks), sc(comm.nranks);
    std::vector<std::vector<double>> sv(comm.nranks);
    for (int r = 0; r < comm.nranks; ++r) {
        for (int64_t i = 0; i < n; ++i) sl[r].push_back(M.rp[i + 1] - M.rp[i]);
        sc[r].assign(M.col.begin(), M.col.end());
        sv[r].assign(M.val.begin(), M.val.end());
    }
    auto gl = comm.exchange(sl);
    auto gc = comm.exchange(sc);
    auto gv = comm.exchange(sv);
    HostCSR G;
    G.n_global_rows = M.n_global_rows;
    G.n_global_cols = M.n_global_cols;
    G.row_starts = {0, M.n_global_rows};
    G.col_starts = {0, M.n_global_cols};
    G.rp.assign(1, 0);
    for (int r = 0; r < comm.nranks; ++r) {
        for (int64_t l : gl[r]) G.rp.push_back(G.rp.back() + l);
        G.col.insert(G.col.end(), gc[r].begin(), gc[r].end());
        G.val.insert(G.val.end(), gv[r].begin(), gv[r].end());
    }
    AMG_ASSERT(G.nrows() == M.n_global_rows);
    return G;
}

}  // namespace amg
