// copy_probe.hip -- STREAM-copy ceiling probe (1 GiB fp64, 16-byte lanes): load/store policy
// and grid size variants, HIP-event timed.  Used to pick the bench's copy kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v2d __attribute__((ext_vector_type(2)));
template <int NTL, int NTS, int U>
__global__ __launch_bounds__(256) void cp(long long np, const v2d* __restrict__ s, v2d* __restrict__ d) {
    const long long stride = (long long)gridDim.x * 256;
    long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < np; i += U * stride) {
        v2d v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NTL ? __builtin_nontemporal_load(s + i + u * stride) : s[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) { if (NTS) __builtin_nontemporal_store(v[u], d + i + u * stride); else d[i + u * stride] = v[u]; }
    }
    for (; i < np; i += stride) d[i] = s[i];
}
// one pass, no grid-stride: every thread copies U consecutive-block pairs
template <int U>
__global__ __launch_bounds__(256) void cp1(long long np, const v2d* __restrict__ s, v2d* __restrict__ d) {
    long long i = ((long long)blockIdx.x * U) * 256 + threadIdx.x;
    v2d v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = s[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u) d[i + u * 256] = v[u];
}
#define CK(x) do { if ((x) != hipSuccess) { printf("err %s\n", #x); return 1; } } while (0)
int main() {
    const long long n = 1ll << 27, np = n / 2;
    double *a, *b;
    CK(hipMalloc(&a, n * 8)); CK(hipMalloc(&b, n * 8));
    CK(hipMemset(a, 0, n * 8)); CK(hipMemset(b, 0, n * 8));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        hipEventRecord(e0);
        for (int r = 0; r < 20; ++r) launch();
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("%-40s %8.1f GB/s  %7.1f us\n", name, 2.0 * n * 8 / (ms / 20 * 1e-3) / 1e9, ms / 20 * 1e3);
    };
    for (int g : {1024, 2048, 4096, 8192, 16384}) {
        char nm[64];
        snprintf(nm, 64, "plain U4 grid %d", g);
        run(nm, [&] { hipLaunchKernelGGL((cp<0, 0, 4>), dim3(g), dim3(256), 0, 0, np, (const v2d*)a, (v2d*)b); });
        snprintf(nm, 64, "nt-load U4 grid %d", g);
        run(nm, [&] { hipLaunchKernelGGL((cp<1, 0, 4>), dim3(g), dim3(256), 0, 0, np, (const v2d*)a, (v2d*)b); });
        snprintf(nm, 64, "nt-both U4 grid %d", g);
        run(nm, [&] { hipLaunchKernelGGL((cp<1, 1, 4>), dim3(g), dim3(256), 0, 0, np, (const v2d*)a, (v2d*)b); });
    }
    run("one-pass U4", [&] { hipLaunchKernelGGL((cp1<4>), dim3(np / 1024), dim3(256), 0, 0, np, (const v2d*)a, (v2d*)b); });
    run("one-pass U8", [&] { hipLaunchKernelGGL((cp1<8>), dim3(np / 2048), dim3(256), 0, 0, np, (const v2d*)a, (v2d*)b); });
    run("one-pass U16", [&] { hipLaunchKernelGGL((cp1<16>), dim3(np / 4096), dim3(256), 0, 0, np, (const v2d*)a, (v2d*)b); });
    run("hipMemcpyAsync D2D", [&] { hipMemcpyAsync(b, a, n * 8, hipMemcpyDeviceToDevice, 0); });
    return 0;
}
