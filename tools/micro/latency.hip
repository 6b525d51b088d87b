// Diagnostic micro-benchmark: dependent-load latency seen by one wave on gfx950
// (pointer chase over a small L2-resident ring), with and without an
// interleaved store, plus the s_memtime / s_memrealtime tick ratio.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void chase(const int* ring, int* sink, int steps, int mode, unsigned long long* out) {
    int p = 0;
    // warm
    for (int i = 0; i < steps; i++) p = __builtin_amdgcn_readfirstlane(ring[p]);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < steps; i++) {
        p = __builtin_amdgcn_readfirstlane(ring[p]);
        if (mode == 1) sink[(i & 63) * 16 + 8192] = p;     // store to another line, then next dependent load
        if (mode == 2) { sink[(i & 63) * 16 + 8192] = p; __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; out[2] = p; }
}

int main() {
    const int N = 1 << 20;   // ints
    std::vector<int> h(N);
    for (int span : {1024, 16384, 262144, 1 << 20}) {
        // ring with stride of 97 lines within span ints
        for (int i = 0; i < N; i++) h[i] = 0;
        int cur = 0;
        const int nodes = span / 32;
        for (int k = 0; k < nodes; k++) { int nxt = ((k + 1) * 37 % nodes) * 32; h[cur] = nxt; cur = nxt; }
        int *d, *sink; unsigned long long* o;
        hipMalloc(&d, N * 4); hipMalloc(&sink, N * 4 * 2); hipMalloc(&o, 64);
        hipMemcpy(d, h.data(), N * 4, hipMemcpyHostToDevice);
        for (int mode = 0; mode < 3; mode++) {
            for (int blocks : {1, 1024}) {
                chase<<<blocks, 64>>>(d, sink, 2000, mode, o);
                hipDeviceSynchronize();
                unsigned long long r[3]; hipMemcpy(r, o, 24, hipMemcpyDeviceToHost);
                printf("span %7d B mode %d blocks %4d: %.0f memtime ticks/load, %.1f ns/load, tick ratio %.1f\n",
                       span * 4, mode, blocks, r[0] / 2000.0, r[1] * 10.0 / 2000.0, (double)r[0] / r[1]);
            }
        }
        hipFree(d); hipFree(sink); hipFree(o);
    }
    return 0;
}
