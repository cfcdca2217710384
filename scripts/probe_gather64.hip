// probe_gather64.hip — can a random 64-byte record gather cost 64 bytes of HBM
// traffic instead of a whole 128-byte line? (k_pileup gathers one 64-byte packed
// record per piled read; every such gather was a 128-B fabric read request at v16,
// profiles/r01/rdreq_v16.txt). Experiment only, not product.
//
// The buffer stays below 4 GiB (one buffer descriptor, 32-bit offsets): far larger
// than the 256 MiB Infinity Cache, so uniform random gathers miss it.
// For each allocation kind (hipMalloc, hipDeviceMallocUncached,
// hipDeviceMallocFinegrained) and each load cache policy (plain, nt, sc0, sc1,
// sc0 sc1, sc0 sc1 nt) it times U=4 records in flight per lane, 4 x 16-B loads per
// record, under three access patterns: uniform random over the whole buffer,
// random inside a sliding 1 GiB region (the pileup's window), sequential records.
//   build: hipcc --offload-arch=gfx950 -O3 scripts/probe_gather64.hip -o scripts/probe_gather64
//   run:   scripts/probe_gather64 [GB]
// PMC: rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum
//      TCC_EA0_RDREQ_128B_sum -- scripts/probe_gather64 (kernel names carry the mode)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ unsigned long long mix(unsigned long long z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// load cache policy POL -> buffer-load aux bits (gfx950: sc0 = 1, nt = 2, sc1 = 16);
// compiler-tracked builtin loads (no inline asm: an asm load's destination is not
// protected until its own wait, cdna_hip_programming.md §5.7 item 1)
template <int POL>
struct Aux {
    static constexpr int v = POL == 0 ? 0 : POL == 1 ? 2 : POL == 2 ? 1 : POL == 3 ? 16 : POL == 4 ? 17 : 19;
};

// PAT 0: uniform random records over the buffer; 1: random inside a region of
// rrecs records that slides once per grid pass; 2: sequential records
// ALLOC only labels the kernel name (allocation kind of the buffer)
template <int POL, int PAT, int ALLOC>
__global__ void __launch_bounds__(256) k_g64(uint4* __restrict__ buf, unsigned long long nrec,
                                             unsigned long long nreq, unsigned long long rrecs, uint4* out) {
    constexpr int U = 4;
    const unsigned long long tid = blockIdx.x * 256ull + threadIdx.x;
    const unsigned long long nth = (unsigned long long)gridDim.x * 256ull;
    // one descriptor over the whole buffer (< 4 GiB: 32-bit offsets), wave-uniform
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(buf, 0, (int)(unsigned)(nrec * 64), 0x00020000);
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (unsigned long long i0 = tid; i0 < nreq; i0 += nth * U) {
        uint4 v[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned long long i = i0 + u * nth;
            const unsigned long long j = i < nreq ? i : nreq - 1;
            unsigned long long r;
            if (PAT == 0) r = mix(j) % nrec;
            else if (PAT == 1) r = ((j / nth) * (rrecs / 64)) % (nrec - rrecs) + mix(j) % rrecs;
            else r = j % nrec;
            const unsigned off = (unsigned)(r * 64);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(off + 16u * k), 0, Aux<POL>::v);
                v[u][k] = make_uint4(x[0], x[1], x[2], x[3]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                acc.x ^= v[u][k].x;
                acc.y ^= v[u][k].y;
                acc.z ^= v[u][k].z;
                acc.w ^= v[u][k].w;
            }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) out[0] = acc;
}

static const char* kPol[] = {"plain", "nt", "sc0", "sc1", "sc0 sc1", "sc0 sc1 nt"};
static const char* kPat[] = {"random, whole buffer", "random, sliding 1 GiB", "sequential"};
static const char* kAlloc[] = {"hipMalloc", "Uncached", "Finegrained"};

template <int POL, int PAT, int ALLOC>
static void run(uint4* buf, unsigned long long nrec, unsigned long long nreq, uint4* out) {
    const int grid = 4096;
    const unsigned long long rrecs = (1ull << 30) / 64;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k_g64<POL, PAT, ALLOC><<<grid, 256>>>(buf, nrec, nreq, rrecs, out);
    hipEventRecord(a);
    const int reps = 3;
    for (int r = 0; r < reps; ++r) k_g64<POL, PAT, ALLOC><<<grid, 256>>>(buf, nrec, nreq, rrecs, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    const double bytes = (double)nreq * 64;
    printf("%-12s %-11s %-22s %8.3f ms  %7.0f GB/s of records\n", kAlloc[ALLOC], kPol[POL], kPat[PAT], ms,
           bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
    hipEventDestroy(a);
    hipEventDestroy(b);
}

template <int POL, int ALLOC>
static void pats(uint4* buf, unsigned long long nrec, unsigned long long nreq, uint4* out) {
    run<POL, 0, ALLOC>(buf, nrec, nreq, out);
    run<POL, 1, ALLOC>(buf, nrec, nreq, out);
    run<POL, 2, ALLOC>(buf, nrec, nreq, out);
}

template <int ALLOC>
static int one_alloc(double gb, unsigned long long nreq, uint4* out) {
    const unsigned long long nrec = (unsigned long long)(gb * 1e9 / 64);
    const size_t bytes = nrec * 64;
    uint4* buf = nullptr;
    hipError_t e = ALLOC == 0 ? hipMalloc(&buf, bytes)
                              : hipExtMallocWithFlags((void**)&buf, bytes,
                                                      ALLOC == 1 ? hipDeviceMallocUncached : hipDeviceMallocFinegrained);
    if (e != hipSuccess) {
        printf("%s: allocation of %.1f GB failed: %s\n", kAlloc[ALLOC], bytes / 1e9, hipGetErrorString(e));
        (void)hipGetLastError();
        return 1;
    }
    hipMemset(buf, 1, bytes);
    hipDeviceSynchronize();
    pats<0, ALLOC>(buf, nrec, nreq, out);
    pats<1, ALLOC>(buf, nrec, nreq, out);
    pats<2, ALLOC>(buf, nrec, nreq, out);
    pats<3, ALLOC>(buf, nrec, nreq, out);
    pats<4, ALLOC>(buf, nrec, nreq, out);
    pats<5, ALLOC>(buf, nrec, nreq, out);
    hipFree(buf);
    return 0;
}

int main(int argc, char** argv) {
    const double gb = argc > 1 ? atof(argv[1]) : 3.2;  // < 4 GiB: one buffer descriptor
    const unsigned long long nreq = 150000000ull;  // ~ the piled reads of one C4 pileup launch
    if (!(gb > 1.2 && gb * 1e9 < 4294967295.0)) {
        printf("buffer size must lie in (1.2, 4.29) GB (one buffer descriptor)\n");
        return 1;
    }
    uint4* out = nullptr;
    if (hipMalloc(&out, 64) != hipSuccess) return 1;
    printf("buffer %.1f GB, %llu random 64-B records per pass\n", gb, nreq);
    one_alloc<0>(gb, nreq, out);
    one_alloc<1>(gb, nreq, out);
    one_alloc<2>(gb, nreq, out);
    hipFree(out);
    return 0;
}
