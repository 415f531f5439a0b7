/*
 * io_oracle.c -- serial restatement of the unstructured-input path:
 * the G3_circuit-substitute graph Laplacian, reverse Cuthill-McKee and the symmetric
 * permutation.  TEST INFRASTRUCTURE ONLY (see amg_oracle.h).  PARITY UNPINNED against the
 * reference (no such code there); the generator and RCM specs are fixed in DESIGN.md 8
 * and the RCM quality is cross-checked against scipy.sparse.csgraph in the tests.
 *
 * Written independently of raptor_amd/csrc/host_io.cpp: plain arrays, explicit loops,
 * insertion sorts, one serial pass per row.
 */
#include <stdlib.h>
#include <string.h>

#include "amg_oracle.h"

static uint64_t sm64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* symmetric uniform in [0, 1) attached to the unordered pair {a, b} */
static double pair_uniform(int64_t a, int64_t b, uint64_t salt, uint64_t seed) {
    int64_t lo = a < b ? a : b, hi = a < b ? b : a;
    uint64_t h = sm64((uint64_t)lo * 0x9E3779B97F4A7C15ull ^ salt ^ (seed * 0xD1B54A32D192ED03ull));
    h = sm64(h + (uint64_t)hi);
    return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}

static int64_t* shuffled(int64_t n, uint64_t seed) {
    int64_t* p = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) p[i] = i;
    for (int64_t i = n - 1; i >= 1; --i) {
        int64_t j = (int64_t)(sm64(seed * 0xD1B54A32D192ED03ull + (uint64_t)i) % (uint64_t)(i + 1));
        int64_t t = p[i];
        p[i] = p[j];
        p[j] = t;
    }
    return p;
}

#define SALT_ORDER 0x0A11CE5ull
#define SALT_PAIR 0xBA5E1ull
#define SALT_GRID 0x6121Dull
#define SALT_DIAG 0xD1A6ull
#define SALT_LONG 0x10A6ull
#define SALT_W 0x3E16ull
#define SALT_GND 0x6A0DDull

/* kept neighbours of node q (lattice numbering) in enumeration order */
static int lattice_edges(int64_t q, int64_t nx, int64_t ny, uint64_t seed, const int64_t* partner,
                         int64_t* nb, double* w) {
    int64_t i = q % nx, j = q / nx;
    int c = 0;
    int64_t cand[6] = {q - 1, q + 1, q - nx, q + nx, q - nx - 1, q + nx + 1};
    int ok[6] = {i > 0, i + 1 < nx, j > 0, j + 1 < ny, i > 0 && j > 0, i + 1 < nx && j + 1 < ny};
    for (int t = 0; t < 6; ++t) {
        if (!ok[t]) continue;
        int grid = t < 4;
        double u = pair_uniform(q, cand[t], grid ? SALT_GRID : SALT_DIAG, seed);
        if (u < (grid ? 0.85 : 0.30)) nb[c++] = cand[t];
    }
    int64_t p = partner[q];
    if (p >= 0) {
        int seen = 0;
        for (int t = 0; t < c; ++t)
            if (nb[t] == p) seen = 1;
        if (!seen && pair_uniform(q, p, SALT_LONG, seed) < 0.5) nb[c++] = p;
    }
    for (int t = 0; t < c; ++t) {
        double u = pair_uniform(q, nb[t], SALT_W, seed);
        w[t] = 0.1 + 9.9 * (u * u * u);
    }
    return c;
}

orc_csr* orc_gen_graph_laplacian(int64_t nx, int64_t ny, uint64_t seed) {
    int64_t n = nx * ny;
    /* partners: each 32x32 tile's nodes (row-major), shuffled, paired (2t, 2t+1) */
    int64_t* partner = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
    int64_t* mem = (int64_t*)malloc(sizeof(int64_t) * 32 * 32);
    for (int64_t k = 0; k < n; ++k) partner[k] = -1;
    int64_t tx = (nx + 31) / 32, ty = (ny + 31) / 32;
    for (int64_t t = 0; t < tx * ty; ++t) {
        int64_t a = t % tx, b = t / tx, sz = 0;
        for (int64_t j = b * 32; j < ny && j < (b + 1) * 32; ++j)
            for (int64_t i = a * 32; i < nx && i < (a + 1) * 32; ++i) mem[sz++] = i + nx * j;
        int64_t* s = shuffled(sz, sm64((seed ^ SALT_PAIR) + (uint64_t)t));
        for (int64_t k = 0; k + 1 < sz; k += 2) {
            partner[mem[s[k]]] = mem[s[k + 1]];
            partner[mem[s[k + 1]]] = mem[s[k]];
        }
        free(s);
    }
    free(mem);
    int64_t* pi = shuffled(n, seed ^ SALT_ORDER); /* lattice node -> row id */
    int64_t* pinv = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
    for (int64_t k = 0; k < n; ++k) pinv[pi[k]] = k;

    int64_t* rp = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 1));
    int64_t* col = (int64_t*)malloc(sizeof(int64_t) * (size_t)(8 * n));
    double* val = (double*)malloc(sizeof(double) * (size_t)(8 * n));
    rp[0] = 0;
    for (int64_t r = 0; r < n; ++r) {
        int64_t q = pinv[r], nb[7];
        double w[7];
        int c = lattice_edges(q, nx, ny, seed, partner, nb, w);
        double d = 0.0;
        for (int t = 0; t < c; ++t) d = d + w[t];
        d = d + (pair_uniform(q, q, SALT_GND, seed) < 0.01 ? 1.0 : 1e-6);
        int64_t cc[8];
        double vv[8];
        for (int t = 0; t < c; ++t) {
            cc[t] = pi[nb[t]];
            vv[t] = -w[t];
        }
        cc[c] = r;
        vv[c] = d;
        /* insertion sort by column */
        for (int a = 1; a <= c; ++a) {
            int64_t kc = cc[a];
            double kv = vv[a];
            int b = a - 1;
            while (b >= 0 && cc[b] > kc) {
                cc[b + 1] = cc[b];
                vv[b + 1] = vv[b];
                --b;
            }
            cc[b + 1] = kc;
            vv[b + 1] = kv;
        }
        for (int t = 0; t <= c; ++t) {
            col[rp[r] + t] = cc[t];
            val[rp[r] + t] = vv[t];
        }
        rp[r + 1] = rp[r] + c + 1;
    }
    orc_csr* A = orc_csr_new(n, n, rp, col, val);
    free(rp), free(col), free(val), free(partner), free(pi), free(pinv);
    return A;
}

/* ------------------------------------------------------------------------------ */
/* Reverse Cuthill-McKee: G = pattern(A + A^T) without the diagonal;  */
/* components started in (deg, id) order from a George-Liu pseudo-peripheral node; */
/* BFS visiting neighbours in (deg, id) order; whole order reversed.               */
/* ------------------------------------------------------------------------------ */
static const int64_t* g_deg;
static int by_deg_id(const void* a, const void* b) {
    int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    if (g_deg[x] != g_deg[y]) return g_deg[x] < g_deg[y] ? -1 : 1;
    return x < y ? -1 : x > y;
}
static int by_id(const void* a, const void* b) {
    int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    return x < y ? -1 : x > y;
}

/* BFS from s; fills q[0..len) and lev[]; returns the eccentricity */
static int64_t bfs_levels(int64_t s, const int64_t* gp, const int64_t* g, int64_t* lev, int64_t* q,
                          int64_t* len) {
    int64_t head = 0, tail = 0;
    q[tail++] = s;
    lev[s] = 0;
    while (head < tail) {
        int64_t v = q[head++];
        for (int64_t k = gp[v]; k < gp[v + 1]; ++k)
            if (lev[g[k]] < 0) {
                lev[g[k]] = lev[v] + 1;
                q[tail++] = g[k];
            }
    }
    *len = tail;
    return lev[q[tail - 1]];
}

void orc_rcm(const orc_csr* A, int64_t* new_to_old) {
    int64_t n = A->n_rows;
    /* symmetrised adjacency, deduplicated */
    int64_t* cnt = (int64_t*)calloc((size_t)(n + 1), sizeof(int64_t));
    for (int64_t i = 0; i < n; ++i)
        for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k)
            if (A->col[k] != i) {
                cnt[i + 1]++;
                cnt[A->col[k] + 1]++;
            }
    for (int64_t i = 0; i < n; ++i) cnt[i + 1] += cnt[i];
    int64_t* raw = (int64_t*)malloc(sizeof(int64_t) * (size_t)(cnt[n] > 0 ? cnt[n] : 1));
    int64_t* pos = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) pos[i] = cnt[i];
    for (int64_t i = 0; i < n; ++i)
        for (int64_t k = A->rp[i]; k < A->rp[i + 1]; ++k) {
            int64_t j = A->col[k];
            if (j == i) continue;
            raw[pos[i]++] = j;
            raw[pos[j]++] = i;
        }
    int64_t* gp = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 1));
    int64_t* g = (int64_t*)malloc(sizeof(int64_t) * (size_t)(cnt[n] > 0 ? cnt[n] : 1));
    int64_t* deg = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    gp[0] = 0;
    for (int64_t i = 0; i < n; ++i) {
        int64_t b = cnt[i], e = cnt[i + 1];
        qsort(raw + b, (size_t)(e - b), sizeof(int64_t), by_id);
        int64_t m = 0;
        for (int64_t k = b; k < e; ++k)
            if (k == b || raw[k] != raw[k - 1]) g[gp[i] + m++] = raw[k];
        gp[i + 1] = gp[i] + m;
        deg[i] = m;
    }
    g_deg = deg;
    for (int64_t i = 0; i < n; ++i) qsort(g + gp[i], (size_t)deg[i], sizeof(int64_t), by_deg_id);
    int64_t* start = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) start[i] = i;
    qsort(start, (size_t)n, sizeof(int64_t), by_deg_id);

    int64_t* lev = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    int64_t* q = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    char* placed = (char*)calloc((size_t)(n > 0 ? n : 1), 1);
    for (int64_t i = 0; i < n; ++i) lev[i] = -1;
    int64_t out = 0, len = 0;
    for (int64_t t = 0; t < n; ++t) {
        int64_t root = start[t];
        if (placed[root]) continue;
        int64_t ecc = bfs_levels(root, gp, g, lev, q, &len);
        for (;;) {
            int64_t cand = -1;
            for (int64_t h = 0; h < len; ++h) {
                int64_t v = q[h];
                if (lev[v] != ecc) continue;
                if (cand < 0 || deg[v] < deg[cand] || (deg[v] == deg[cand] && v < cand)) cand = v;
            }
            for (int64_t h = 0; h < len; ++h) lev[q[h]] = -1;
            int64_t e2 = bfs_levels(cand, gp, g, lev, q, &len);
            for (int64_t h = 0; h < len; ++h) lev[q[h]] = -1;
            if (e2 <= ecc) break;
            root = cand;
            ecc = bfs_levels(root, gp, g, lev, q, &len);
        }
        bfs_levels(root, gp, g, lev, q, &len);
        for (int64_t h = 0; h < len; ++h) {
            new_to_old[out++] = q[h];
            placed[q[h]] = 1;
            lev[q[h]] = -1;
        }
    }
    for (int64_t a = 0, b = n - 1; a < b; ++a, --b) {
        int64_t t = new_to_old[a];
        new_to_old[a] = new_to_old[b];
        new_to_old[b] = t;
    }
    free(cnt), free(raw), free(pos), free(gp), free(g), free(deg), free(start), free(lev), free(q),
        free(placed);
}

orc_csr* orc_permute(const orc_csr* A, const int64_t* new_to_old) {
    int64_t n = A->n_rows, nnz = A->rp[n];
    int64_t* inv = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t k = 0; k < n; ++k) inv[new_to_old[k]] = k;
    int64_t* rp = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 1));
    int64_t* col = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nnz > 0 ? nnz : 1));
    double* val = (double*)malloc(sizeof(double) * (size_t)(nnz > 0 ? nnz : 1));
    rp[0] = 0;
    for (int64_t r = 0; r < n; ++r) {
        int64_t o = new_to_old[r], b = rp[r];
        for (int64_t k = A->rp[o]; k < A->rp[o + 1]; ++k) {
            /* insert keeping columns ascending */
            int64_t c = inv[A->col[k]], at = rp[r] + (k - A->rp[o]);
            double v = A->val[k];
            while (at > b && col[at - 1] > c) {
                col[at] = col[at - 1];
                val[at] = val[at - 1];
                --at;
            }
            col[at] = c;
            val[at] = v;
        }
        rp[r + 1] = b + (A->rp[o + 1] - A->rp[o]);
    }
    orc_csr* B = orc_csr_new(n, n, rp, col, val);
    free(inv), free(rp), free(col), free(val);
    return B;
}
