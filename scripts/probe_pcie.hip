// Host link probe: H2D alone, D2H alone and both at once (pinned host memory,
// hipMemcpyAsync in 256 MiB pieces on one stream per direction), and H2D beside a
// kernel that writes to mapped pinned memory (as k_rows_to_host does); and a kernel that
// pulls mapped pinned host memory into device memory (instead of the copy engine), alone
// and beside the copy engine's D2H or the host-writing kernel.
//   hipcc --offload-arch=gfx950 -O2 scripts/probe_pcie.hip -o /tmp/probe_pcie && /tmp/probe_pcie
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_write_host(uint4* __restrict__ h, const uint4* __restrict__ d, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) h[i] = d[i];
}

__global__ void k_read_host(uint4* __restrict__ d, const uint4* __restrict__ h, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        d[i] = h[i];
}

int main() {
    const size_t N = 4ull << 30, P = 256ull << 20;
    void *h1, *h2, *d1, *d2;
    CK(hipHostMalloc(&h1, N, hipHostMallocDefault));
    CK(hipHostMalloc(&h2, N, hipHostMallocDefault));
    CK(hipMalloc(&d1, N));
    CK(hipMalloc(&d2, N));
    memset(h1, 1, N);
    memset(h2, 2, N);
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    auto run = [&](bool up, bool down, int kern_wg, int pull_wg = 0) -> double {
        CK(hipDeviceSynchronize());
        auto t0 = std::chrono::steady_clock::now();
        if (pull_wg) k_read_host<<<pull_wg, 256, 0, a>>>((uint4*)d1, (const uint4*)h1, N / 16);
        for (size_t o = 0; o < N; o += P) {
            if (up) CK(hipMemcpyAsync((char*)d1 + o, (char*)h1 + o, P, hipMemcpyHostToDevice, a));
            if (down) CK(hipMemcpyAsync((char*)h2 + o, (char*)d2 + o, P, hipMemcpyDeviceToHost, b));
        }
        if (kern_wg) k_write_host<<<kern_wg, 256, 0, b>>>((uint4*)h2, (const uint4*)d2, N / 16);
        CK(hipDeviceSynchronize());
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    };
    for (int rep = 0; rep < 2; ++rep) {
        double t;
        t = run(true, false, 0);  printf("H2D alone          %6.1f GB/s\n", N / t / 1e9);
        t = run(false, true, 0);  printf("D2H alone          %6.1f GB/s\n", N / t / 1e9);
        t = run(true, true, 0);   printf("H2D + D2H          %6.1f GB/s each (both end at %.3f s)\n", N / t / 1e9, t);
        t = run(false, false, 256); printf("kernel writes host %6.1f GB/s (256 WGs)\n", N / t / 1e9);
        t = run(false, false, 2048); printf("kernel writes host %6.1f GB/s (2048 WGs)\n", N / t / 1e9);
        t = run(true, false, 256); printf("H2D + kernel wr    %6.1f GB/s each (both end at %.3f s)\n", N / t / 1e9, t);
        for (int wg : {256, 1024, 4096}) {
            t = run(false, false, 0, wg); printf("kernel pulls host  %6.1f GB/s (%d WGs)\n", N / t / 1e9, wg);
        }
        t = run(false, true, 0, 1024); printf("pull + D2H         %6.1f GB/s each (both end at %.3f s)\n", N / t / 1e9, t);
        t = run(false, false, 256, 1024); printf("pull + kernel wr   %6.1f GB/s each (both end at %.3f s)\n", N / t / 1e9, t);
    }
    return 0;
}
