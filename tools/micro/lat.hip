// Latency microbenchmarks for the serial parse chain on gfx950 (one wave): dependent SALU ops,
// dependent scalar loads from a constant table, dependent LDS read + readfirstlane, v_readlane.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__constant__ uint32_t c_tab[4096];
__global__ void k(uint64_t *out, uint32_t seed, int n) {
    __shared__ uint32_t lds[4096];
    for (int i = threadIdx.x; i < 4096; i += 64) lds[i] = (i * 2654435761u) & 4095;
    __syncthreads();
    uint32_t x = seed;
    uint64_t t0 = clock64();
    for (int i = 0; i < n; i++) {  // 8 dependent SALU ops per iteration
        x = x * 3 + 1; x ^= x >> 7; x = x * 5 + 3; x ^= x >> 9; x += 11; x ^= x << 3; x = x * 7; x += i;
    }
    uint64_t t1 = clock64();
    uint32_t y = __builtin_amdgcn_readfirstlane(x) & 4095;
    for (int i = 0; i < n; i++) y = c_tab[y] & 4095;   // dependent scalar loads (K$)
    uint64_t t2 = clock64();
    uint32_t z = y;
    for (int i = 0; i < n; i++) z = __builtin_amdgcn_readfirstlane(lds[z]) & 4095;  // LDS + readfirstlane
    uint64_t t3 = clock64();
    int v = threadIdx.x;
    uint32_t w = z;
    for (int i = 0; i < n; i++) w = (uint32_t)__builtin_amdgcn_readlane(v + (int)w, (int)(w & 63)) & 4095;
    uint64_t t4 = clock64();
    uint32_t a0 = w, a1 = w + 1, a2 = w + 2, a3 = w + 3, a4 = w + 4, a5 = w + 5, a6 = w + 6, a7 = w + 7;
    for (int i = 0; i < n; i++) {  // 8 independent SALU adds+xors per iteration (16 ops)
        a0 += 0x9e37; a1 += 0x7f4a; a2 += 0x1234; a3 += 0x4321; a4 += 0x1111; a5 += 0x2222; a6 += 0x3333; a7 += 0x4444;
        a0 ^= a0 >> 3; a1 ^= a1 >> 5; a2 ^= a2 >> 7; a3 ^= a3 >> 9; a4 ^= a4 >> 11; a5 ^= a5 >> 13; a6 ^= a6 >> 2; a7 ^= a7 >> 4;
    }
    uint64_t t5 = clock64();
    uint32_t bsum = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    // dependent chain with a 64-bit shift + clz, like the bit reader
    uint64_t cache = ((uint64_t)bsum << 32) | 0x12345u;
    int av = 64;
    for (int i = 0; i < n; i++) {
        uint32_t p = (uint32_t)(cache >> 32);
        int lz = __clz(p | 1);
        int len = (lz & 7) + 1;
        cache = (cache << len) | (uint64_t)(p & 0xff);
        av -= len; if (av < 32) av += 32;
    }
    uint64_t t6 = clock64();
    int tv[8];
#pragma unroll
    for (int j = 0; j < 8; j++) tv[j] = (int)(((threadIdx.x + 64 * j) * 2654435761u) & 511);
    uint32_t q = (uint32_t)av & 511;
    for (int i = 0; i < n; i++) q = (uint32_t)__builtin_amdgcn_readlane(tv[(q >> 6) & 7], (int)(q & 63)) & 511;
    uint64_t t7 = clock64();
    uint32_t q2 = q;
    for (int i = 0; i < n; i++) {  // select by branch tree on 2 bits x readlane (4 regs)
        const uint32_t r = q2 >> 6 & 3;
        int sel = r == 0 ? tv[0] : (r == 1 ? tv[1] : (r == 2 ? tv[2] : tv[3]));
        q2 = (uint32_t)__builtin_amdgcn_readlane(sel, (int)(q2 & 63)) & 255;
    }
    uint64_t t8 = clock64();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = t2 - t1; out[2] = t3 - t2; out[3] = t4 - t3; out[4] = x + y + z + w + bsum + (uint32_t)cache + av;
                            out[5] = t5 - t4; out[6] = t6 - t5; out[7] = t7 - t6; out[8] = t8 - t7; out[9] = q + q2; }
}
int main() {
    uint32_t h[4096];
    for (int i = 0; i < 4096; i++) h[i] = (i * 40503u + 17) & 4095;
    hipMemcpyToSymbol(HIP_SYMBOL(c_tab), h, sizeof(h));
    uint64_t *d; hipMalloc(&d, 128);
    uint64_t r[10];
    int n = 10000;
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, 12345u, n);
        hipMemcpy(r, d, 80, hipMemcpyDeviceToHost);
        printf("per iter cycles: 8 SALU chain %.1f | s_load dep %.1f | lds+rfl dep %.1f | readlane dep %.1f | 16 indep SALU %.1f | bitreader step %.1f | vgpr-table(movrel) %.1f | vgpr-table(select4) %.1f\n",
               r[0] / (double)n, r[1] / (double)n, r[2] / (double)n, r[3] / (double)n, r[5] / (double)n, r[6] / (double)n, r[7] / (double)n, r[8] / (double)n);
    }
    return 0;
}
