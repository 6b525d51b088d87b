// Reproducer attempt for the round-2/3 device-only INSERT_FAILED: a per-lane
// short-circuit visibility test whose last term holds a loop, feeding `vis ? len : 0`.
// Rows: removed (rseq = 9) by client 1; perspective r = 5, c = 2 has not seen the removal,
// so every row is visible and must give its length.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <stdio.h>
struct Row { int len, seq, rseq, meta, rcl, pad; unsigned long long ovl; };
struct Ovx { int row, rseq, client, pad; };
__host__ __device__ inline bool ovl_sc(const Ovx* ox, int n, unsigned long long ovl, int s, int rs, int c) {
    if (c < 63) return (ovl >> c) & 1ull;
    if (!(ovl >> 63)) return false;
    for (int i = 0; i < n; i++) if (ox[i].row == s && ox[i].client == c && ox[i].rseq == rs) return true;
    return false;
}
__host__ __device__ inline bool vis_sc(const Row& f, int r, int c, const Ovx* ox, int n, int s) {   // round-3 shape
    if (!((f.meta & 0xFFFF) == c || f.seq <= r)) return false;
    if (f.meta & 0x10000) { if (f.rcl == c || f.rseq <= r || ovl_sc(ox, n, f.ovl, s, f.rseq, c)) return false; }
    return true;
}
__global__ void k(const Row* R, const int* ch, int nch, int r, int c, const Ovx* ox, int n, int* out) {
    const int j = threadIdx.x;
    if (j >= nch) return;
    const Row f = R[ch[j]];
    out[j] = vis_sc(f, r, c, ox, n, ch[j]) ? f.len : 0;
}
int main() {
    Row h[8]; int ch[8], want[8], got[8]; Ovx ox[1] = {{99, 9, 70, 0}};
    for (int i = 0; i < 8; i++) { h[i] = {i + 1, 1, 9, 0x10000 | 3, 1, 0, 0}; ch[i] = 7 - i; }
    Row* dR; int *dc, *dout; Ovx* dox;
    hipMalloc(&dR, sizeof h); hipMalloc(&dc, sizeof ch); hipMalloc(&dout, sizeof got); hipMalloc(&dox, sizeof ox);
    hipMemcpy(dR, h, sizeof h, hipMemcpyHostToDevice); hipMemcpy(dc, ch, sizeof ch, hipMemcpyHostToDevice);
    hipMemcpy(dox, ox, sizeof ox, hipMemcpyHostToDevice);
    for (int c : {2, 70}) {                          // c < 63: bit test; c >= 63: the side-list loop
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dR, dc, 8, 5, c, dox, 1, dout);
        hipMemcpy(got, dout, sizeof got, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int j = 0; j < 8; j++) { want[j] = vis_sc(h[ch[j]], 5, c, ox, 1, ch[j]) ? h[ch[j]].len : 0; bad += got[j] != want[j]; }
        printf("c=%d device %s: got", c, bad ? "WRONG" : "right");
        for (int j = 0; j < 8; j++) printf(" %d", got[j]);
        printf(" | host");
        for (int j = 0; j < 8; j++) printf(" %d", want[j]);
        printf("\n");
    }
    return 0;
}
