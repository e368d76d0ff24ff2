// DPP direction check: prints which source lane each DPP control reads (lane 5 and lane 17).
#include <hip/hip_runtime.h>
#include <cstdio>
template <int C> __device__ int dpp(int v) { return __builtin_amdgcn_update_dpp(0, v, C, 0xF, 0xF, false); }
__global__ void k(int *o) {
    int l = threadIdx.x;
    o[0 * 64 + l] = dpp<0x124>(l);  // row_ror:4
    o[1 * 64 + l] = dpp<0x111>(l);  // row_shr:1
    o[2 * 64 + l] = dpp<0x101>(l);  // row_shl:1
    o[3 * 64 + l] = dpp<0x141>(l);  // row_half_mirror
    o[4 * 64 + l] = dpp<0x140>(l);  // row_mirror
    o[5 * 64 + l] = dpp<0xE4 ^ 0xE4 | 0x55>(l);  // quad_perm [1,1,1,1]
}
int main() {
    int *d, h[6 * 64];
    hipMalloc(&d, sizeof(h));
    k<<<1, 64>>>(d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char *n[] = {"row_ror:4", "row_shr:1", "row_shl:1", "row_half_mirror", "row_mirror", "quad_perm[1,1,1,1]"};
    for (int i = 0; i < 6; i++) printf("%-20s lane5<-%d lane17<-%d lane0<-%d lane15<-%d\n", n[i], h[i * 64 + 5], h[i * 64 + 17], h[i * 64], h[i * 64 + 15]);
    return 0;
}
