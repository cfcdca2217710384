// probe_coop.hip — does a random 64-byte record gather get cheaper when the four
// lanes of a quad load one record together (16 lines per wave-instruction) instead
// of every lane loading its own record (64 lines per wave-instruction)? k_pileup
// gathers one 64-byte packed record per piled read, one record per lane.
// Experiment only, not product.
//
// Modes (each: 150M records of a 3.2 GB buffer, U groups of 64 records in flight per wave):
//   0 lane   : lane l loads record l with 4 x 16-B loads (k_pileup today)
//   1 quad   : lane l loads 16 B (part l&3) of record 16k + l/4 in instruction k; data
//              stays in the loading lanes (no transpose: the load cost alone)
//   2 quad+ds: mode 1, then ds_write_b128 into a swizzled per-wave LDS image and 4 x
//              ds_read_b128 so lane l holds record l (the full cost of a quad gather)
//   3 glds   : LDS-DMA (global_load_lds_dwordx4, source address pre-swizzled) then
//              4 x ds_read_b128 so lane l holds record l
// Patterns: random over the whole buffer, random inside a sliding 1 GiB region.
//   build: hipcc --offload-arch=gfx950 -O3 scripts/probe_coop.hip -o scripts/probe_coop
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ unsigned long long mix(unsigned long long z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// cheap per-lane record index (power-of-two buffer and region): the index math must
// not dominate the quad modes, which compute four indices per lane per group
__device__ __forceinline__ unsigned hash32(unsigned x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    return x ^ (x >> 16);
}
template <int PAT>
__device__ __forceinline__ unsigned long long rec_of(unsigned long long j, unsigned long long rbase,
                                                     unsigned long long nrec, unsigned long long rrecs) {
    if (PAT == 0) return hash32((unsigned)j) & (unsigned)(nrec - 1);
    return rbase + (hash32((unsigned)j) & (unsigned)(rrecs - 1));
}

// swizzled slot of part p of record s in a 64-record image: conflict-free
// ds_read_b128 of a whole record per lane (lane groups of MI355X_MICROARCH.md §LDS)
__device__ __forceinline__ unsigned slot_of(unsigned s, unsigned p) { return (p + (s >> 2)) & 3u; }

template <int MODE, int PAT, int U>
__global__ void __launch_bounds__(256) k_coop(const uint4* __restrict__ buf, unsigned long long nrec,
                                              unsigned long long ngrp, unsigned long long rrecs, uint4* out) {
    __shared__ uint4 img[(MODE >= 2) ? 4 * U * 64 * 4 : 1];  // [wave][u][record][4 x 16 B]
    const unsigned lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const unsigned long long gw = blockIdx.x * 4ull + wid;  // global wave
    const unsigned long long nw = gridDim.x * 4ull;
    uint4 acc = make_uint4(0, 0, 0, 0);
    const char* base = reinterpret_cast<const char*>(buf);
    for (unsigned long long g0 = gw; g0 < ngrp; g0 += nw * U) {
        const unsigned long long pass = g0 / nw;  // region slides once per grid pass
        const unsigned long long pass_base = (pass * (rrecs / 64)) % (nrec - rrecs);
        uint4 v[U][4];
        if (MODE == 0) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const unsigned long long g = g0 + u * nw < ngrp ? g0 + u * nw : ngrp - 1;
                const unsigned long long r = rec_of<PAT>(g * 64 + lane, pass_base, nrec, rrecs);
                const uint4* p = reinterpret_cast<const uint4*>(base + r * 64);
#pragma unroll
                for (int k = 0; k < 4; ++k) v[u][k] = p[k];
            }
        } else if (MODE == 1 || MODE == 2) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const unsigned long long g = g0 + u * nw < ngrp ? g0 + u * nw : ngrp - 1;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const unsigned s = 16u * k + (lane >> 2);
                    const unsigned long long r = rec_of<PAT>(g * 64 + s, pass_base, nrec, rrecs);
                    v[u][k] = *reinterpret_cast<const uint4*>(base + r * 64 + 16 * (lane & 3));
                }
            }
            if (MODE == 2) {
                uint4* my = img + (size_t)wid * U * 256;
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const unsigned s = 16u * k + (lane >> 2);
                        my[u * 256 + s * 4 + slot_of(s, lane & 3)] = v[u][k];
                    }
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int q = 0; q < 4; ++q) v[u][q] = my[u * 256 + lane * 4 + slot_of(lane, q)];
                __builtin_amdgcn_wave_barrier();
            }
        } else {  // MODE 3: LDS-DMA, lane l lands at base + 16 l = record s slot l&3
            uint4* my = img + (size_t)wid * U * 256;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const unsigned long long g = g0 + u * nw < ngrp ? g0 + u * nw : ngrp - 1;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const unsigned s = 16u * k + (lane >> 2);
                    const unsigned p = ((lane & 3u) - (s >> 2)) & 3u;  // slot_of(s, p) == lane & 3
                    const unsigned long long r = rec_of<PAT>(g * 64 + s, pass_base, nrec, rrecs);
                    __builtin_amdgcn_global_load_lds(
                        reinterpret_cast<const void*>(base + r * 64 + 16 * p),
                        (__attribute__((address_space(3))) void*)(my + u * 256 + k * 64), 16, 0, 0);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int q = 0; q < 4; ++q) v[u][q] = my[u * 256 + lane * 4 + slot_of(lane, q)];
            __builtin_amdgcn_wave_barrier();
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                acc.x ^= v[u][k].x;
                acc.y ^= v[u][k].y + k;
                acc.z ^= v[u][k].z;
                acc.w ^= v[u][k].w;
            }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) out[0] = acc;
}

// Region sweep: quad-style loads of RS-byte records (RS/16 lanes per record), random
// inside a sliding region of rmib MiB (rmib 0: sequential records)
template <int RS>
__global__ void __launch_bounds__(256) k_region(const uint4* __restrict__ buf, unsigned long long nrec,
                                                unsigned long long ngrp, unsigned long long rrecs, uint4* out) {
    constexpr int LPR = RS / 16;          // lanes per record
    constexpr int NI = 64 * LPR / 64;     // instructions per 64 records
    const unsigned lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const unsigned long long gw = blockIdx.x * 4ull + wid;
    const unsigned long long nw = gridDim.x * 4ull;
    uint4 acc = make_uint4(0, 0, 0, 0);
    const char* base = reinterpret_cast<const char*>(buf);
    constexpr int U = 2;
    for (unsigned long long g0 = gw; g0 < ngrp; g0 += nw * U) {
        const unsigned long long pass = g0 / nw;
        const unsigned long long pass_base = rrecs ? (pass * (rrecs / 64)) % (nrec - rrecs) : 0;
        uint4 v[U][NI];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned long long g = g0 + u * nw < ngrp ? g0 + u * nw : ngrp - 1;
#pragma unroll
            for (int k = 0; k < NI; ++k) {
                const unsigned s = (64u / LPR) * k + lane / LPR;
                const unsigned long long j = g * 64 + s;
                const unsigned long long r = rrecs ? pass_base + (hash32((unsigned)j) & (unsigned)(rrecs - 1))
                                                   : j % nrec;
                v[u][k] = *reinterpret_cast<const uint4*>(base + r * RS + 16 * (lane % LPR));
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < NI; ++k) {
                acc.x ^= v[u][k].x;
                acc.y ^= v[u][k].y + k;
                acc.z ^= v[u][k].z;
                acc.w ^= v[u][k].w;
            }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) out[0] = acc;
}

template <int RS>
static void region(const uint4* buf, unsigned long long nreq, int rmib, uint4* out) {
    const unsigned long long nrec = (4ull << 30) / RS;
    const unsigned long long rrecs = rmib ? ((unsigned long long)rmib << 20) / RS : 0;
    const unsigned long long ngrp = nreq / 64;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k_region<RS><<<4096, 256>>>(buf, nrec, ngrp, rrecs, out);
    hipEventRecord(a);
    for (int r = 0; r < 3; ++r) k_region<RS><<<4096, 256>>>(buf, nrec, ngrp, rrecs, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= 3;
    printf("region RS=%d  %5d MiB %s %8.3f ms  %7.0f GB/s of records\n", RS, rmib, rmib ? "random    " : "sequential", ms,
           (double)ngrp * 64 * RS / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

static const char* kMode[] = {"lane", "quad", "quad+ds", "glds"};
static const char* kPat[] = {"random, whole buffer", "random, sliding 1 GiB"};

template <int MODE, int PAT, int U>
static void run(const uint4* buf, unsigned long long nrec, unsigned long long nreq, uint4* out) {
    const int grid = 4096;
    const unsigned long long rrecs = (1ull << 30) / 64;
    const unsigned long long ngrp = nreq / 64;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k_coop<MODE, PAT, U><<<grid, 256>>>(buf, nrec, ngrp, rrecs, out);
    hipEventRecord(a);
    const int reps = 3;
    for (int r = 0; r < reps; ++r) k_coop<MODE, PAT, U><<<grid, 256>>>(buf, nrec, ngrp, rrecs, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    const double bytes = (double)ngrp * 64 * 64;
    printf("%-8s U=%d  %-22s %8.3f ms  %7.0f GB/s of records\n", kMode[MODE], U, kPat[PAT], ms,
           bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
    hipEventDestroy(a);
    hipEventDestroy(b);
}

template <int MODE, int U>
static void pats(const uint4* buf, unsigned long long nrec, unsigned long long nreq, uint4* out) {
    run<MODE, 0, U>(buf, nrec, nreq, out);
    run<MODE, 1, U>(buf, nrec, nreq, out);
}

int main(int argc, char** argv) {
    const double gb = 4.0;  // 2^26 records of 64 B (power of two: mask, no modulo)
    const unsigned long long nreq = 150000000ull;  // ~ the piled reads of one C4 pileup launch
    const unsigned long long nrec = 1ull << 26;
    uint4* buf = nullptr;
    uint4* out = nullptr;
    if (hipMalloc(&buf, nrec * 64) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) {
        printf("allocation failed\n");
        return 1;
    }
    hipMemset(buf, 1, nrec * 64);
    hipDeviceSynchronize();
    printf("buffer %.1f GB, %llu random 64-B records per pass\n", gb, nreq);
    for (int rs = 0; rs < 2; ++rs)
        for (int rmib : {0, 64, 128, 256, 384, 512, 768, 1024, 2048}) {
            if (rs == 0) region<64>(buf, nreq, rmib, out);
            else region<32>(buf, nreq, rmib, out);
        }
    if (argc > 1) return 0;
    pats<0, 4>(buf, nrec, nreq, out);
    pats<0, 2>(buf, nrec, nreq, out);
    pats<1, 4>(buf, nrec, nreq, out);
    pats<1, 2>(buf, nrec, nreq, out);
    pats<2, 2>(buf, nrec, nreq, out);
    pats<2, 1>(buf, nrec, nreq, out);
    pats<3, 2>(buf, nrec, nreq, out);
    pats<3, 1>(buf, nrec, nreq, out);
    hipFree(buf);
    hipFree(out);
    return 0;
}
