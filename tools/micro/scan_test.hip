// block_excl_scan (enc_bits.inc) against a host scan: max and sum, random inputs with -1s
#include "../../openh264-wasm_amd/csrc/h264mi_kernels.hip"
#include <cstdio>
#include <vector>
using namespace h264mi;
__global__ __launch_bounds__(1024) void scan_k(const int *in, int *outm, int *outs, int *tot) {
    __shared__ int s_w[PACK_WAVES];
    int t1, t2;
    int v = in[threadIdx.x];
    outm[threadIdx.x] = block_excl_scan<true>(v, s_w, &t1);
    outs[threadIdx.x] = block_excl_scan<false>(v < 0 ? 0 : v, s_w, &t2);
    if (threadIdx.x == 0) { tot[0] = t1; tot[1] = t2; }
}
int main() {
    std::vector<int> in(1024), m(1024), s(1024);
    srand(1);
    for (int i = 0; i < 1024; i++) in[i] = (rand() % 3 == 0) ? i : -1;
    int *di, *dm, *ds, *dt; int ht[2];
    hipMalloc(&di, 4096); hipMalloc(&dm, 4096); hipMalloc(&ds, 4096); hipMalloc(&dt, 8);
    hipMemcpy(di, in.data(), 4096, hipMemcpyHostToDevice);
    scan_k<<<1, 1024>>>(di, dm, ds, dt);
    hipMemcpy(m.data(), dm, 4096, hipMemcpyDeviceToHost); hipMemcpy(s.data(), ds, 4096, hipMemcpyDeviceToHost); hipMemcpy(ht, dt, 8, hipMemcpyDeviceToHost);
    int em = -1, es = 0, bad = 0;
    for (int i = 0; i < 1024; i++) {
        if (m[i] != em || s[i] != es) { if (bad < 10) printf("i %d max %d/%d sum %d/%d\n", i, m[i], em, s[i], es); bad++; }
        em = std::max(em, in[i]); es += in[i] < 0 ? 0 : in[i];
    }
    printf("bad %d totals %d/%d %d/%d\n", bad, ht[0], em, ht[1], es);
    return bad != 0;
}
