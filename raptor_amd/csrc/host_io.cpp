// host_io.cpp -- inputs beyond the model stencils: the seeded
// unstructured graph-Laplacian that stands in for SuiteSparse G3_circuit
// (BASELINE.json:11; the real matrix is not available offline), Matrix Market and binary
// CSR readers with a contiguous row partition, a collective binary writer, and the reverse
// Cuthill-McKee reordering that turns a randomly numbered graph back into a banded one.
//
// Every function is deterministic and partition-independent: the rows a rank holds are
// bit-identical to the same rows of the serial result (oracle: orc_gen_graph_laplacian,
// orc_rcm, orc_permute in oracle/amg_oracle.c).
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <numeric>

#include "host.hpp"

namespace amg {

// ----------------------------------------------------------------------------------
// Graph-Laplacian substitute for G3_circuit.  Spec (restated in the oracle):
//   nodes q = i + nx*j on an nx*ny lattice; candidate edges, in this enumeration order,
//     west, east, south, north   kept with probability 0.85  (salt GRID)
//     south-west, north-east     kept with probability 0.30  (salt DIAG)
//     the node's "partner"       kept with probability 0.50  (salt LONG) unless it is
//                                already a kept lattice neighbour; partners pair up the
//                                nodes of each 32x32 lattice tile: the tile's nodes in
//                                row-major order, shuffled (seed ^ PAIR mixed with the tile
//                                index), paired (2t, 2t+1) -- medium-range "nets"
//   weight w = 0.1 + 9.9 u^3 (u from salt W): conductances spread over two decades
//   a_qp = -w,  a_qq = (sum of w in enumeration order) + g,  g = 1 for 1% of nodes
//   ("grounded", salt GND) and 1e-6 otherwise, so every row is strictly dominant
//   rows/cols renumbered by a second seeded permutation pi: new id = pi[q]
// All uniforms are symmetric in (q, p), so A is exactly symmetric.
// ----------------------------------------------------------------------------------
namespace {
constexpr uint64_t kSaltOrder = 0x0A11CE5ull, kSaltPair = 0xBA5E1ull, kSaltGrid = 0x6121Dull,
                   kSaltDiag = 0xD1A6ull, kSaltLong = 0x10A6ull, kSaltW = 0x3E16ull,
                   kSaltGnd = 0x6A0DDull;

inline double edge_u(int64_t a, int64_t b, uint64_t salt, uint64_t seed) {
    if (a > b) std::swap(a, b);
    uint64_t z = mix64(mix64((uint64_t)a * 0x9E3779B97F4A7C15ull ^ salt ^ (seed * 0xD1B54A32D192ED03ull))
                       + (uint64_t)b);
    return (double)(z >> 11) * 0x1.0p-53;
}

// Fisher-Yates with splitmix64 draws: out[k] for k in [0, n)
std::vector<int64_t> seeded_permutation(int64_t n, uint64_t seed) {
    std::vector<int64_t> p(n);
    std::iota(p.begin(), p.end(), 0);
    for (int64_t i = n - 1; i > 0; --i) {
        uint64_t j = mix64(seed * 0xD1B54A32D192ED03ull + (uint64_t)i) % (uint64_t)(i + 1);
        std::swap(p[i], p[(int64_t)j]);
    }
    return p;
}

std::vector<int64_t> inverse_of(const std::vector<int64_t>& p) {
    std::vector<int64_t> q(p.size());
    for (size_t k = 0; k < p.size(); ++k) q[p[k]] = (int64_t)k;
    return q;
}

constexpr int64_t kTile = 32;

std::vector<int64_t> tile_partners(int64_t nx, int64_t ny, uint64_t seed) {
    std::vector<int64_t> partner(nx * ny, -1);
    const int64_t tx = (nx + kTile - 1) / kTile, ty = (ny + kTile - 1) / kTile;
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t t = 0; t < tx * ty; ++t) {
        const int64_t a = t % tx, b = t / tx;
        std::vector<int64_t> mem;
        for (int64_t j = b * kTile; j < std::min(ny, (b + 1) * kTile); ++j)
            for (int64_t i = a * kTile; i < std::min(nx, (a + 1) * kTile); ++i) mem.push_back(i + nx * j);
        const std::vector<int64_t> s = seeded_permutation((int64_t)mem.size(), mix64((seed ^ kSaltPair) + (uint64_t)t));
        for (size_t k = 0; k + 1 < s.size(); k += 2) {
            partner[mem[s[k]]] = mem[s[k + 1]];
            partner[mem[s[k + 1]]] = mem[s[k]];
        }
    }
    return partner;
}

struct Lattice {
    int64_t nx, ny;
    uint64_t seed;
    std::vector<int64_t> partner;  // -1: none

    // kept neighbours of q in enumeration order; returns the count (<= 7)
    int neighbours(int64_t q, int64_t* nb, double* w) const {
        const int64_t i = q % nx, j = q / nx;
        int c = 0;
        auto cand = [&](bool inside, int64_t p, uint64_t salt, double prob) {
            if (inside && edge_u(q, p, salt, seed) < prob) nb[c++] = p;
        };
        cand(i > 0, q - 1, kSaltGrid, 0.85);
        cand(i < nx - 1, q + 1, kSaltGrid, 0.85);
        cand(j > 0, q - nx, kSaltGrid, 0.85);
        cand(j < ny - 1, q + nx, kSaltGrid, 0.85);
        cand(i > 0 && j > 0, q - nx - 1, kSaltDiag, 0.30);
        cand(i < nx - 1 && j < ny - 1, q + nx + 1, kSaltDiag, 0.30);
        const int64_t p = partner[q];
        if (p >= 0) {
            bool dup = false;
            for (int t = 0; t < c; ++t) dup |= nb[t] == p;
            if (!dup && edge_u(q, p, kSaltLong, seed) < 0.5) nb[c++] = p;
        }
        for (int t = 0; t < c; ++t) {
            double u = edge_u(q, nb[t], kSaltW, seed);
            w[t] = 0.1 + 9.9 * (u * u * u);
        }
        return c;
    }
    double ground(int64_t q) const { return edge_u(q, q, kSaltGnd, seed) < 0.01 ? 1.0 : 1e-6; }
};
}  // namespace

HostCSR graph_laplacian_slab(const HostComm& comm, int64_t nx, int64_t ny, uint64_t seed) {
    AMG_CHECK(nx > 0 && ny > 0, "graph laplacian: lattice dims must be positive");
    const int64_t n = nx * ny;
    Lattice L{nx, ny, seed, tile_partners(nx, ny, seed)};
    const std::vector<int64_t> pi = seeded_permutation(n, seed ^ kSaltOrder);  // q -> new id
    const std::vector<int64_t> pinv = inverse_of(pi);
    HostCSR A;
    A.n_global_rows = A.n_global_cols = n;
    A.row_starts.resize(comm.nranks + 1);
    for (int r = 0; r <= comm.nranks; ++r) A.row_starts[r] = n * r / comm.nranks;
    A.col_starts = A.row_starts;
    const int64_t r0 = A.row_starts[comm.rank], m = A.row_starts[comm.rank + 1] - r0;
    std::vector<int64_t> len(m);
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < m; ++t) {
        int64_t nb[7];
        double w[7];
        len[t] = 1 + L.neighbours(pinv[r0 + t], nb, w);
    }
    A.rp.assign(m + 1, 0);
    for (int64_t t = 0; t < m; ++t) A.rp[t + 1] = A.rp[t] + len[t];
    A.col.resize(A.rp[m]);
    A.val.resize(A.rp[m]);
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < m; ++t) {
        const int64_t q = pinv[r0 + t];
        int64_t nb[8];
        double w[8];
        const int c = L.neighbours(q, nb, w);
        double d = 0.0;
        for (int k = 0; k < c; ++k) d += w[k];
        d += L.ground(q);
        std::pair<int64_t, double> e[8];
        for (int k = 0; k < c; ++k) e[k] = {pi[nb[k]], -w[k]};
        e[c] = {r0 + t, d};
        std::sort(e, e + c + 1, [](const auto& a, const auto& b) { return a.first < b.first; });
        for (int k = 0; k <= c; ++k) A.col[A.rp[t] + k] = e[k].first, A.val[A.rp[t] + k] = e[k].second;
    }
    return A;
}

// ----------------------------------------------------------------------------------
// Readers.  Row partition: rank r holds rows [n r / P, n (r+1) / P).
// ----------------------------------------------------------------------------------
namespace {
constexpr char kMagic[8] = {'R', 'A', 'M', 'G', 'C', 'S', 'R', '1'};

struct File {
    FILE* f = nullptr;
    explicit File(const std::string& path, const char* mode) : f(std::fopen(path.c_str(), mode)) {
        if (!f) throw Error(AMG_ERR_INVALID, "cannot open " + path + ": " + std::strerror(errno));
    }
    ~File() {
        if (f) std::fclose(f);
    }
};

void partition(const HostComm& comm, int64_t n_rows, int64_t n_cols, HostCSR& A) {
    A.n_global_rows = n_rows;
    A.n_global_cols = n_cols;
    A.row_starts.resize(comm.nranks + 1);
    A.col_starts.resize(comm.nranks + 1);
    for (int r = 0; r <= comm.nranks; ++r) {
        A.row_starts[r] = n_rows * r / comm.nranks;
        A.col_starts[r] = n_cols * r / comm.nranks;
    }
}

std::string lower(std::string s) {
    for (auto& ch : s) ch = (char)std::tolower((unsigned char)ch);
    return s;
}

HostCSR read_mm(const HostComm& comm, const std::string& path) {
    File F(path, "rb");
    std::fseek(F.f, 0, SEEK_END);
    const long size = std::ftell(F.f);
    std::fseek(F.f, 0, SEEK_SET);
    std::string buf((size_t)size, '\0');
    AMG_CHECK(std::fread(&buf[0], 1, (size_t)size, F.f) == (size_t)size, "short read: " + path);
    size_t pos = buf.find('\n');
    AMG_CHECK(pos != std::string::npos, "matrix market: no header line");
    char obj[64] = {}, fmt[64] = {}, field[64] = {}, sym[64] = {};
    AMG_CHECK(std::sscanf(buf.c_str(), "%%%%MatrixMarket %63s %63s %63s %63s", obj, fmt, field, sym) == 4,
              "matrix market: bad banner");
    const std::string o = lower(obj), f = lower(fmt), fl = lower(field), sy = lower(sym);
    AMG_CHECK(o == "matrix" && f == "coordinate", "matrix market: only 'matrix coordinate' is supported");
    AMG_CHECK(fl == "real" || fl == "integer" || fl == "pattern" || fl == "double",
              "matrix market: field must be real, integer or pattern");
    AMG_CHECK(sy == "general" || sy == "symmetric" || sy == "skew-symmetric",
              "matrix market: symmetry must be general, symmetric or skew-symmetric");
    const bool pattern = fl == "pattern", mirror = sy != "general", skew = sy == "skew-symmetric";
    const char* p = buf.c_str() + pos + 1;
    const char* end = buf.c_str() + buf.size();
    for (;;) {  // blank and comment lines
        while (p < end && std::isspace((unsigned char)*p)) ++p;
        if (p >= end || *p != '%') break;
        const char* nl = (const char*)std::memchr(p, '\n', end - p);
        p = nl ? nl + 1 : end;
    }
    char* q;
    const int64_t nr = std::strtoll(p, &q, 10), nc = std::strtoll(q, &q, 10), ne = std::strtoll(q, &q, 10);
    AMG_CHECK(q != p && nr > 0 && nc > 0 && ne >= 0, "matrix market: bad size line");
    AMG_CHECK(!mirror || nr == nc, "matrix market: symmetric matrix must be square");
    p = q;
    HostCSR A;
    partition(comm, nr, nc, A);
    const int64_t lo = A.row_starts[comm.rank], hi = A.row_starts[comm.rank + 1];
    struct Ent {
        int64_t r, c, seq;
        double v;
    };
    std::vector<Ent> ent;
    for (int64_t k = 0; k < ne; ++k) {
        const int64_t i = std::strtoll(p, &q, 10) - 1;
        AMG_CHECK(q != p, "matrix market: truncated entry list");
        p = q;
        const int64_t j = std::strtoll(p, &q, 10) - 1;
        AMG_CHECK(q != p, "matrix market: truncated entry list");
        p = q;
        double v = 1.0;
        if (!pattern) {
            v = std::strtod(p, &q);
            AMG_CHECK(q != p, "matrix market: missing value");
            p = q;
        }
        AMG_CHECK(i >= 0 && i < nr && j >= 0 && j < nc, "matrix market: index out of range");
        if (i >= lo && i < hi) ent.push_back({i, j, 2 * k, v});
        if (mirror && i != j && j >= lo && j < hi) ent.push_back({j, i, 2 * k + 1, skew ? -v : v});
    }
    // (row, col) order; duplicates summed in file order
    std::sort(ent.begin(), ent.end(), [](const Ent& a, const Ent& b) {
        return a.r != b.r ? a.r < b.r : a.c != b.c ? a.c < b.c : a.seq < b.seq;
    });
    A.rp.assign(hi - lo + 1, 0);
    for (size_t k = 0; k < ent.size(); ++k) {
        if (k > 0 && ent[k].r == ent[k - 1].r && ent[k].c == ent[k - 1].c) {
            A.val.back() += ent[k].v;
            continue;
        }
        A.col.push_back(ent[k].c);
        A.val.push_back(ent[k].v);
        A.rp[ent[k].r - lo + 1]++;
    }
    for (int64_t t = 0; t < hi - lo; ++t) A.rp[t + 1] += A.rp[t];
    return A;
}

void read_at(FILE* f, int64_t off, void* dst, size_t bytes, const std::string& path) {
    AMG_CHECK(std::fseek(f, (long)off, SEEK_SET) == 0, "seek failed: " + path);
    AMG_CHECK(std::fread(dst, 1, bytes, f) == bytes, "short read: " + path);
}

HostCSR read_bin(const HostComm& comm, const std::string& path) {
    File F(path, "rb");
    char magic[8];
    int64_t hdr[3];
    read_at(F.f, 0, magic, 8, path);
    AMG_CHECK(std::memcmp(magic, kMagic, 8) == 0, "binary csr: bad magic");
    read_at(F.f, 8, hdr, sizeof(hdr), path);
    const int64_t nr = hdr[0], nc = hdr[1], nnz = hdr[2];
    AMG_CHECK(nr > 0 && nc > 0 && nnz >= 0, "binary csr: bad header");
    HostCSR A;
    partition(comm, nr, nc, A);
    const int64_t lo = A.row_starts[comm.rank], m = A.row_starts[comm.rank + 1] - lo;
    const int64_t o_rp = 32, o_col = o_rp + 8 * (nr + 1), o_val = o_col + 8 * nnz;
    A.rp.resize(m + 1);
    read_at(F.f, o_rp + 8 * lo, A.rp.data(), 8 * (m + 1), path);
    const int64_t b = A.rp[0], e = A.rp[m];
    AMG_CHECK(b >= 0 && b <= e && e <= nnz, "binary csr: bad row pointer");
    for (auto& v : A.rp) v -= b;
    A.col.resize(e - b);
    A.val.resize(e - b);
    if (e > b) {
        read_at(F.f, o_col + 8 * b, A.col.data(), 8 * (e - b), path);
        read_at(F.f, o_val + 8 * b, A.val.data(), 8 * (e - b), path);
    }
    for (int64_t t = 0; t < m; ++t) {
        AMG_CHECK(A.rp[t + 1] >= A.rp[t], "binary csr: row pointer not monotone");
        for (int64_t k = A.rp[t]; k < A.rp[t + 1]; ++k) {
            AMG_CHECK(A.col[k] >= 0 && A.col[k] < nc, "binary csr: column out of range");
            AMG_CHECK(k == A.rp[t] || A.col[k] > A.col[k - 1], "binary csr: columns not ascending");
        }
    }
    return A;
}
}  // namespace

HostCSR read_par_matrix(const HostComm& comm, const std::string& path) {
    char head[16] = {};
    {
        File F(path, "rb");
        size_t got = std::fread(head, 1, sizeof(head), F.f);
        AMG_CHECK(got >= 8, "file too short: " + path);
    }
    if (std::memcmp(head, kMagic, 8) == 0) return read_bin(comm, path);
    AMG_CHECK(std::strncmp(head, "%%MatrixMarket", 14) == 0,
              "unknown matrix file format (expected Matrix Market or binary CSR): " + path);
    return read_mm(comm, path);
}

// Collective: rank 0 writes the header and truncates; every rank then writes its rows at
// their global offsets (shared file system; one node here).
void write_par_matrix(const HostComm& comm, const HostCSR& A, const std::string& path) {
    const int64_t m = A.nrows(), nnz = A.nnz();
    std::vector<int64_t> nnzs = comm.allgather(nnz);
    int64_t before = 0, total = 0;
    for (int r = 0; r < comm.nranks; ++r) {
        if (r < comm.rank) before += nnzs[r];
        total += nnzs[r];
    }
    int ok = 1;
    if (comm.rank == 0) {
        int fd = ::open(path.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
        if (fd < 0) {
            ok = 0;
        } else {
            int64_t hdr[3] = {A.n_global_rows, A.n_global_cols, total};
            ok = ::pwrite(fd, kMagic, 8, 0) == 8 && ::pwrite(fd, hdr, sizeof(hdr), 8) == (ssize_t)sizeof(hdr);
            ::close(fd);
        }
    }
    AMG_CHECK(comm.allreduce_sum(ok) == comm.nranks, "cannot create " + path);
    ok = 1;
    int fd = ::open(path.c_str(), O_WRONLY);
    if (fd < 0) {
        ok = 0;
    } else {
        const int64_t lo = A.row_starts[comm.rank], nr = A.n_global_rows;
        std::vector<int64_t> rp(m + 1);
        for (int64_t t = 0; t <= m; ++t) rp[t] = A.rp[t] + before;
        // the last rank also writes rp[n]; others stop at their last row
        const int64_t cnt = comm.rank == comm.nranks - 1 ? m + 1 : m;
        auto put = [&](const void* src, int64_t bytes, int64_t off) {
            const char* s = (const char*)src;
            while (bytes > 0 && ok) {
                ssize_t w = ::pwrite(fd, s, (size_t)bytes, off);
                if (w <= 0) ok = 0;
                s += w, bytes -= w, off += w;
            }
        };
        const int64_t o_rp = 32, o_col = o_rp + 8 * (nr + 1), o_val = o_col + 8 * total;
        put(rp.data(), 8 * cnt, o_rp + 8 * lo);
        put(A.col.data(), 8 * nnz, o_col + 8 * before);
        put(A.val.data(), 8 * nnz, o_val + 8 * before);
        ::close(fd);
    }
    AMG_CHECK(comm.allreduce_sum(ok) == comm.nranks, "write failed: " + path);
}

// ----------------------------------------------------------------------------------
// Reverse Cuthill-McKee on the symmetrised pattern of a GATHERED matrix (the whole graph
// on every rank; fine up to ~1e8 nnz of host memory).  Spec, restated in orc_rcm:
//   G = pattern(A + A^T) minus the diagonal; deg = |G(v)|
//   components in order of their first node in the (deg, id)-sorted node list; each
//   starts from a pseudo-peripheral node (George-Liu: BFS, move to the (deg, id)-minimal
//   node of the last level while the eccentricity grows), then BFS appending each
//   node's unvisited neighbours in (deg, id) order; the final order is reversed.
// ----------------------------------------------------------------------------------
std::vector<int64_t> rcm_order(const HostCSR& A) {
    const int64_t n = A.n_global_rows;
    AMG_CHECK(A.n_global_cols == n && A.nrows() == n, "rcm: needs the whole square matrix");
    std::vector<int64_t> cnt(n + 1, 0);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k)
            if (A.col[k] != i) cnt[i + 1]++, cnt[A.col[k] + 1]++;
    for (int64_t i = 0; i < n; ++i) cnt[i + 1] += cnt[i];
    std::vector<int64_t> adj(cnt[n]), fill(cnt.begin(), cnt.end() - 1);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
            const int64_t j = A.col[k];
            if (j != i) adj[fill[i]++] = j, adj[fill[j]++] = i;
        }
    std::vector<int64_t> gp(n + 1, 0);
    std::vector<int64_t> deg(n);
#pragma omp parallel for schedule(dynamic, 4096)
    for (int64_t i = 0; i < n; ++i) {
        std::sort(adj.begin() + cnt[i], adj.begin() + cnt[i + 1]);
        deg[i] = std::unique(adj.begin() + cnt[i], adj.begin() + cnt[i + 1]) - (adj.begin() + cnt[i]);
    }
    auto before = [&](int64_t a, int64_t b) { return deg[a] != deg[b] ? deg[a] < deg[b] : a < b; };
    // neighbour lists in (deg, id) order, used by every BFS below
#pragma omp parallel for schedule(dynamic, 4096)
    for (int64_t i = 0; i < n; ++i) std::sort(adj.begin() + cnt[i], adj.begin() + cnt[i] + deg[i], before);
    std::vector<int64_t> nodes(n);
    std::iota(nodes.begin(), nodes.end(), 0);
    std::stable_sort(nodes.begin(), nodes.end(), [&](int64_t a, int64_t b) { return deg[a] < deg[b]; });

    std::vector<int64_t> level(n, -1), order;
    order.reserve(n);
    std::vector<char> done(n, 0);
    std::vector<int64_t> queue;
    queue.reserve(n);
    // BFS from s over the not-yet-ordered component: returns eccentricity, fills queue
    auto bfs = [&](int64_t s) {
        queue.clear();
        queue.push_back(s);
        level[s] = 0;
        for (size_t h = 0; h < queue.size(); ++h) {
            const int64_t v = queue[h];
            for (int64_t k = cnt[v]; k < cnt[v] + deg[v]; ++k)
                if (level[adj[k]] < 0) level[adj[k]] = level[v] + 1, queue.push_back(adj[k]);
        }
        const int64_t ecc = level[queue.back()];
        return ecc;
    };
    auto reset = [&]() {
        for (int64_t v : queue) level[v] = -1;
    };
    for (int64_t s : nodes) {
        if (done[s]) continue;
        int64_t r = s, ecc = bfs(r);
        for (;;) {
            int64_t best = -1;
            for (size_t h = queue.size(); h-- > 0 && level[queue[h]] == ecc;)
                if (best < 0 || before(queue[h], best)) best = queue[h];
            reset();
            const int64_t e2 = bfs(best);
            if (e2 > ecc) {
                r = best, ecc = e2;
                continue;
            }
            reset();
            break;
        }
        // Cuthill-McKee from r: BFS order with (deg, id)-sorted neighbour lists
        (void)bfs(r);
        for (int64_t v : queue) order.push_back(v), done[v] = 1;
        reset();
    }
    AMG_ASSERT((int64_t)order.size() == n);
    std::reverse(order.begin(), order.end());
    return order;  // new_to_old
}

// B = P A P^T (B[k, :] = A[new_to_old[k], :] renumbered), this rank's rows of the even
// row partition; full = gathered A
HostCSR permute_symmetric(const HostComm& comm, const HostCSR& full, const std::vector<int64_t>& new_to_old) {
    const int64_t n = full.n_global_rows;
    std::vector<int64_t> old_to_new = inverse_of(new_to_old);
    HostCSR B;
    partition(comm, n, n, B);
    const int64_t lo = B.row_starts[comm.rank], m = B.row_starts[comm.rank + 1] - lo;
    B.rp.assign(m + 1, 0);
    for (int64_t t = 0; t < m; ++t) {
        const int64_t o = new_to_old[lo + t];
        B.rp[t + 1] = B.rp[t] + full.rp[o + 1] - full.rp[o];
    }
    B.col.resize(B.rp[m]);
    B.val.resize(B.rp[m]);
#pragma omp parallel for schedule(dynamic, 1024)
    for (int64_t t = 0; t < m; ++t) {
        const int64_t o = new_to_old[lo + t];
        const int64_t len = full.rp[o + 1] - full.rp[o];
        std::vector<std::pair<int64_t, double>> e(len);
        for (int64_t k = 0; k < len; ++k)
            e[k] = {old_to_new[full.col[full.rp[o] + k]], full.val[full.rp[o] + k]};
        std::sort(e.begin(), e.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
        for (int64_t k = 0; k < len; ++k) B.col[B.rp[t] + k] = e[k].first, B.val[B.rp[t] + k] = e[k].second;
    }
    return B;
}

HostCSR reorder_rcm(const HostComm& comm, const HostCSR& A, std::vector<int64_t>& new_to_old_local) {
    AMG_CHECK(A.n_global_rows == A.n_global_cols, "reorder: matrix must be square");
    HostCSR full = gather_global(comm, A);
    std::vector<int64_t> n2o = rcm_order(full);
    HostCSR B = permute_symmetric(comm, full, n2o);
    const int64_t lo = B.row_starts[comm.rank];
    new_to_old_local.assign(n2o.begin() + lo, n2o.begin() + B.row_starts[comm.rank + 1]);
    return B;
}

}  // namespace amg
