// Diagnostic: does a line written by the wave stay L2-resident for later dependent loads?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) (void)(x)

__global__ void chase2(int* ring, int steps, int mode, unsigned long long* out) {
    int p = 0;
    for (int i = 0; i < steps; i++) p = __builtin_amdgcn_readfirstlane(ring[p]);   // warm (reads)
    if (mode >= 1) {               // write a field in every node's line (same line as the pointer)
        int q = 0;
        for (int i = 0; i < steps; i++) { const int n = __builtin_amdgcn_readfirstlane(ring[q]); ring[q + 4] = i; q = n; }
    }
    if (mode == 2) __builtin_amdgcn_s_sleep(127);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    p = 0;
    for (int i = 0; i < steps; i++) p = __builtin_amdgcn_readfirstlane(ring[p]);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    // loads of the written field only (data dependency through the value)
    int acc = 0; p = 0;
    const unsigned long long t2 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < steps; i++) { p = __builtin_amdgcn_readfirstlane(ring[p]); acc += ring[p + 4]; }
    const unsigned long long t3 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) { out[0] = t1 - t0; out[1] = t3 - t2; out[2] = acc; }
}

int main() {
    const int N = 1 << 20;
    std::vector<int> h(N);
    for (int span : {16384, 262144}) {
        for (int i = 0; i < N; i++) h[i] = 0;
        const int nodes = span / 32;
        int cur = 0;
        for (int k = 0; k < nodes; k++) { int nxt = ((k + 1) * 37 % nodes) * 32; h[cur] = nxt; cur = nxt; }
        for (int mode = 0; mode < 3; mode++) {
            for (int blocks : {1, 256}) {
                int* d; unsigned long long* o;
                CK(hipMalloc(&d, (size_t)N * 4 * blocks)); CK(hipMalloc(&o, 64));
                for (int b = 0; b < blocks; b++) CK(hipMemcpy(d + (size_t)b * N, h.data(), N * 4, hipMemcpyHostToDevice));
                chase2<<<1, 64>>>(d, nodes, mode, o);
                CK(hipDeviceSynchronize());
                unsigned long long r[3]; CK(hipMemcpy(r, o, 24, hipMemcpyDeviceToHost));
                printf("span %7d B nodes %5d mode %d: chase %.0f ticks/load, chase+field %.0f ticks/step\n",
                       span * 4, nodes, mode, r[0] / (double)nodes, r[1] / (double)nodes);
                CK(hipFree(d)); CK(hipFree(o));
                break;
            }
        }
    }
    return 0;
}
