// probe_gather.hip — what rate can random 128-byte record gathers reach on this GPU?
// (the pileup reads one 128-B record line per piled read, in cell-major order, so
// from random places of the BAM-ordered payload). Experiment only, not product.
//   build: hipcc --offload-arch=gfx950 -O3 scripts/probe_gather.hip -o scripts/probe_gather
//   run:   scripts/probe_gather [GB] [M lines] [alloc mode]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ unsigned long long mix(unsigned long long z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// V = 16-byte vectors per line (8: 128 B, 4: 64 B), U = lines per lane in flight,
// mode 0 random lines, 1 sequential lines (lane-contiguous), 2 random 2 KiB pages
template <int V, int U>
__global__ void __launch_bounds__(256) k_gather(const uint4* __restrict__ buf, unsigned long long nlines,
                                                unsigned long long nreq, int mode, uint4* out,
                                                unsigned long long rlines) {
    const unsigned long long tid = blockIdx.x * 256ull + threadIdx.x;
    const unsigned long long nth = (unsigned long long)gridDim.x * 256ull;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (unsigned long long i0 = tid; i0 < nreq; i0 += nth * U) {
        uint4 v[U][V];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned long long i = i0 + u * nth;
            unsigned long long line;
            if (mode == 1) line = i % nlines;
            else if (mode == 2) line = ((mix(i >> 4) % (nlines >> 4)) << 4) + (i & 15);
            else if (mode == 3)  // random inside a region of rlines that slides once per grid pass
                line = ((i / nth) * rlines) % (nlines - rlines) + mix(i) % rlines;
            else line = mix(i) % nlines;
            const uint4* p = buf + line * 8;
#pragma unroll
            for (int k = 0; k < V; ++k) v[u][k] = i < nreq ? p[k] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < V; ++k) {
                acc.x ^= v[u][k].x;
                acc.y ^= v[u][k].y;
                acc.z ^= v[u][k].z;
                acc.w ^= v[u][k].w;
            }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) out[0] = acc;
}

template <int V, int U>
static void run(const char* name, const uint4* buf, unsigned long long nlines, unsigned long long nreq, int mode,
                uint4* out, int grid, unsigned long long rlines = 1) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k_gather<V, U><<<grid, 256>>>(buf, nlines, nreq, mode, out, rlines);
    hipEventRecord(a);
    const int reps = 3;
    for (int r = 0; r < reps; ++r) k_gather<V, U><<<grid, 256>>>(buf, nlines, nreq, mode, out, rlines);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    const double bytes = (double)nreq * V * 16;
    printf("%-40s grid %6d  %8.3f ms  %7.0f GB/s\n", name, grid, ms, bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const double gb = argc > 1 ? atof(argv[1]) : 25.6;
    const unsigned long long nreq = (unsigned long long)((argc > 2 ? atof(argv[2]) : 128.0) * 1e6);
    const unsigned long long nlines = (unsigned long long)(gb * 1e9 / 128);
    // allocation: 0 hipMalloc, 1 hipExtMallocWithFlags(contiguous), 2 one VMM handle
    // (hipMemCreate + hipMemMap) at the largest granularity the driver offers
    const int amode = argc > 3 ? atoi(argv[3]) : 0;
    uint4* buf = nullptr;
    uint4* out = nullptr;
    size_t bytes = nlines * 128;
    hipError_t e = hipSuccess;
    if (amode == 1) {
        e = hipExtMallocWithFlags((void**)&buf, bytes, hipDeviceMallocContiguous);
    } else if (amode == 2) {
        hipMemAllocationProp prop = {};
        prop.type = hipMemAllocationTypePinned;
        prop.location.type = hipMemLocationTypeDevice;
        prop.location.id = 0;
        size_t gmin = 0, grec = 0;
        hipMemGetAllocationGranularity(&gmin, &prop, hipMemAllocationGranularityMinimum);
        hipMemGetAllocationGranularity(&grec, &prop, hipMemAllocationGranularityRecommended);
        printf("VMM granularity min %zu recommended %zu\n", gmin, grec);
        const size_t gr = grec > gmin ? grec : gmin;
        bytes = (bytes + gr - 1) / gr * gr;
        hipMemGenericAllocationHandle_t h;
        void* va = nullptr;
        e = hipMemCreate(&h, bytes, &prop, 0);
        if (e == hipSuccess) e = hipMemAddressReserve(&va, bytes, 1ull << 30, nullptr, 0);
        if (e == hipSuccess) e = hipMemMap(va, bytes, 0, h, 0);
        hipMemAccessDesc acc = {};
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        if (e == hipSuccess) e = hipMemSetAccess(va, bytes, &acc, 1);
        buf = (uint4*)va;
    } else {
        e = hipMalloc(&buf, bytes);
    }
    if (e != hipSuccess || hipMalloc(&out, 64) != hipSuccess) {
        printf("alloc failed (mode %d): %s\n", amode, hipGetErrorString(e));
        return 1;
    }
    printf("allocation mode %d at %p\n", amode, (void*)buf);
    hipMemset(buf, 1, nlines * 128);
    hipDeviceSynchronize();
    printf("buffer %.1f GB, %llu lines gathered per pass\n", nlines * 128 / 1e9, nreq);
    const int grid = 2048;
    run<8, 2>("random 128B lines, whole buffer", buf, nlines, nreq, 0, out, grid);
    run<8, 2>("sequential 128B lines", buf, nlines, nreq, 1, out, grid);
    for (double mb : {64.0, 128.0, 256.0, 512.0, 1024.0, 2048.0, 4096.0}) {
        char name[64];
        snprintf(name, sizeof name, "random 128B in sliding %5.0f MB region", mb);
        run<8, 2>(name, buf, nlines, nreq, 3, out, grid, (unsigned long long)(mb * 1048576.0 / 128));
    }
    if (amode != 2) hipFree(buf);  // (the VMM mapping is released at exit)
    hipFree(out);
    return 0;
}
