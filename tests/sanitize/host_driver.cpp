// host_driver.cpp -- AddressSanitizer / UBSan run of the product's host code (SURVEY.md 5:
// host sanitizer build).  Built by tests/sanitize/Makefile from raptor_amd/csrc/host_*.cpp
// with -fsanitize=address,undefined (no HIP: the host setup is plain C++ + OpenMP); exercises
// the setup paths the GPU solver runs before uploading: stencil slabs, strength, RS / PMIS
// splits + classical interpolation, MIS(2) aggregation + smoothed prolongator, transposes,
// Galerkin SpGEMM, extended+i and the coarse drop tolerance (r6), the coarse dense inverse,
// the graph-Laplacian generator, RCM reordering
// and the Matrix Market / binary CSR readers and writer.
#include <cstdio>
#include <cstdlib>
#include <string>

#include "../../raptor_amd/csrc/host.hpp"

using namespace amg;

static amg_options opts(int coarsen, int smoother, double theta) {
    amg_options o{};
    o.coarsen = coarsen;
    o.smoother = smoother;
    o.strong_threshold = theta;
    o.jacobi_omega = 2.0 / 3.0;
    o.pre_sweeps = o.post_sweeps = 1;
    o.max_levels = 25;
    o.max_coarse = 64;
    o.gs_block = 64;
    o.seed = 0x5EED;
    o.setup_device = 0;
    o.replicate_below = 0;
    return o;
}

int main(int argc, char** argv) {
    const std::string tmp = argc > 1 ? argv[1] : "/tmp";
    HostComm serial;
    const double eps[3] = {1.0, 1.0, 1e-3};
    int levels = 0;
    struct Case {
        int kind;
        int64_t nx, ny, nz;
        int coarsen, smoother;
        double theta;
        int interp;       // r6 options: extended+i interpolation (P_max 4)
        double drop_tol;  // and the coarse drop tolerance
    } cases[] = {{AMG_STENCIL_7PT, 14, 13, 12, AMG_COARSEN_PMIS, AMG_SMOOTH_JACOBI, 0.25, AMG_INTERP_CLASSICAL, 0.0},
                 {AMG_STENCIL_5PT, 40, 33, 1, AMG_COARSEN_RS, AMG_SMOOTH_JACOBI, 0.25, AMG_INTERP_CLASSICAL, 0.0},
                 {AMG_STENCIL_27PT, 11, 10, 9, AMG_COARSEN_SA, AMG_SMOOTH_HYBRID_GS, 0.08, AMG_INTERP_CLASSICAL, 0.0},
                 {AMG_STENCIL_7PT, 14, 13, 12, AMG_COARSEN_PMIS, AMG_SMOOTH_JACOBI, 0.25, AMG_INTERP_EXT_I, 0.05},
                 {AMG_STENCIL_27PT, 11, 10, 9, AMG_COARSEN_SA, AMG_SMOOTH_HYBRID_GS, 0.08, AMG_INTERP_CLASSICAL, 0.02}};
    for (const Case& c : cases) {
        HostCSR A = stencil_slab(serial, c.kind, c.nx, c.ny, c.nz, eps);
        HostHierarchy H;
        amg_options o = opts(c.coarsen, c.smoother, c.theta);
        o.interp = c.interp;
        o.p_max = 4;
        o.drop_tol = c.drop_tol;
        build_hierarchy(serial, A, o, H);
        levels += (int)H.levels.size();
        if (H.levels.size() < 2 || H.coarse_inv.empty()) {
            std::fprintf(stderr, "hierarchy too shallow\n");
            return 1;
        }
    }
    HostCSR G = graph_laplacian_slab(serial, 60, 50, 3);
    std::vector<int64_t> order = rcm_order(G);
    if ((int64_t)order.size() != G.n_global_rows) return 1;
    const std::string bin = tmp + "/host_driver_g.bin";
    write_par_matrix(serial, G, bin);
    HostCSR G2 = read_par_matrix(serial, bin);
    if (G2.nnz() != G.nnz() || G2.val != G.val) return 1;
    const std::string mm = tmp + "/host_driver.mtx";
    FILE* f = std::fopen(mm.c_str(), "w");
    std::fprintf(f, "%%%%MatrixMarket matrix coordinate real symmetric\n%% comment\n3 3 4\n1 1 2\n2 1 -1\n2 2 2\n3 3 5.5\n");
    std::fclose(f);
    HostCSR M = read_par_matrix(serial, mm);
    if (M.nnz() != 5) return 1;
    std::printf("host sanitizer driver ok: %d levels over 3 hierarchies, graph %lld rows\n", levels,
                (long long)G.n_global_rows);
    return 0;
}
