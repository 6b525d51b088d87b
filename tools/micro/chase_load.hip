// Diagnostic: dependent-load latency under the replay kernel's concurrency.  Each one-wave
// workgroup owns a region of R bytes of one big buffer and chases pointers through it (every lane
// loads 4 bytes of a 256-byte record, the next record's index comes from lane 0, as a walk's leaf
// rows do); cycles per dependent step (s_memtime) are averaged over the waves.  Sweeps the region
// size (footprint = waves * R) and the wave count.  Build: hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

// every region's records link into one cycle through all of them (the same permutation per region)
__global__ void fill(int* buf, long long regionInts, const int* perm, int nrec) {
    int* base = buf + (long long)blockIdx.x * regionInts;
    for (int i = threadIdx.x; i < nrec; i += 64) base[(long long)i * 64] = perm[i];
}
__global__ void chase(const int* buf, long long regionInts, int steps, unsigned long long* cyc) {
    const int* base = buf + (long long)blockIdx.x * regionInts;
    const int nrec = (int)(regionInts / 64);
    int p = (blockIdx.x * 7919) % nrec;
    int acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < steps; i++) {
        const int v = base[(long long)p * 64 + threadIdx.x];
        acc += v;
        p = __builtin_amdgcn_readfirstlane(v);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = (t1 - t0) + (acc == 0x7fffffff ? 1 : 0);
}

int main(int argc, char** argv) {
    const int steps = 2000;
    const long long maxBytes = 8ll << 30;
    int* d = nullptr;
    if (hipMalloc(&d, maxBytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
    unsigned long long* c = nullptr;
    int* dperm = nullptr;
    (void)hipMalloc(&dperm, 4 << 20);
    (void)hipMalloc(&c, 8 * 8192);
    std::vector<unsigned long long> hc(8192);
    printf("waves  region_KB  footprint_MB  cycles/step (s_memtime units, mean over waves)\n");
    for (int waves : {256, 1024, 4096}) {
        for (long long rk : {16ll, 256ll, 1024ll, 2048ll}) {
            const long long regionInts = rk * 1024 / 4;
            if ((long long)waves * rk * 1024 > maxBytes) continue;
            const int nrec = (int)(regionInts / 64);
            std::vector<int> perm(nrec), order(nrec);
            for (int i = 0; i < nrec; i++) order[i] = i;
            unsigned s = 12345u + (unsigned)rk;
            for (int i = nrec - 1; i > 0; i--) { s = s * 1103515245u + 12345u; const int j = (int)((s >> 8) % (unsigned)i); std::swap(order[i], order[j]); }
            for (int i = 0; i < nrec; i++) perm[order[i]] = order[(i + 1) % nrec];   // one cycle through every record
            (void)hipMemcpy(dperm, perm.data(), 4ull * nrec, hipMemcpyHostToDevice);
            hipLaunchKernelGGL(fill, dim3(waves), dim3(64), 0, 0, d, regionInts, dperm, nrec);
            hipLaunchKernelGGL(chase, dim3(waves), dim3(64), 0, 0, d, regionInts, steps, c);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(hc.data(), c, 8 * waves, hipMemcpyDeviceToHost);
            double m = 0;
            for (int i = 0; i < waves; i++) m += (double)hc[i];
            printf("%5d  %9lld  %12lld  %.0f\n", waves, rk, (long long)waves * rk / 1024, m / waves / steps);
        }
    }
    return 0;
}
