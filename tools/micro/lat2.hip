// Issue/latency microbenchmarks for a single wave (gfx950): VALU vs SALU chains, VALU table lookups
// from LDS (lane-varying address, no readfirstlane), v_bfe bit extraction, VALU->SALU branch round trips.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__global__ void k(uint64_t *out, uint32_t seed, int n, uint32_t *sink) {
    __shared__ uint32_t lds[4096];
    for (int i = threadIdx.x; i < 4096; i += 64) lds[i] = (i * 2654435761u) & 4095;
    __syncthreads();
    uint32_t v = seed + threadIdx.x;          // VGPR
    uint64_t t0 = clock64();
    for (int i = 0; i < n; i++) {  // 8 dependent VALU ops
        v = v * 3u + 1u; v ^= v >> 7; v = v * 5u + 3u; v ^= v >> 9; v += 11u; v ^= v << 3; v = v * 7u; v += (uint32_t)i;
    }
    uint64_t t1 = clock64();
    uint32_t a0 = v, a1 = v + 1, a2 = v + 2, a3 = v + 3, a4 = v + 4, a5 = v + 5, a6 = v + 6, a7 = v + 7;
    for (int i = 0; i < n; i++) {  // 16 independent VALU ops
        a0 += 0x9e37u; a1 += 0x7f4au; a2 += 0x1234u; a3 += 0x4321u; a4 += 0x1111u; a5 += 0x2222u; a6 += 0x3333u; a7 += 0x4444u;
        a0 ^= a0 >> 3; a1 ^= a1 >> 5; a2 ^= a2 >> 7; a3 ^= a3 >> 9; a4 ^= a4 >> 11; a5 ^= a5 >> 13; a6 ^= a6 >> 2; a7 ^= a7 >> 4;
    }
    uint64_t t2 = clock64();
    uint32_t z = (a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) & 4095;
    for (int i = 0; i < n; i++) z = lds[z] & 4095;  // dependent LDS lookups, VGPR address
    uint64_t t3 = clock64();
    uint32_t w = z, pos = 0;
    for (int i = 0; i < n; i++) {  // bit reader step on VALU: bfe + clz + add (dependent)
        uint32_t x = __builtin_amdgcn_alignbit(w, w * 0x9e3779b9u, pos & 31);
        uint32_t lz = __builtin_clz(x | 1u);
        pos += (lz & 7) + 1;
        w ^= x;
    }
    uint64_t t4 = clock64();
    uint32_t u = w;
    int cnt = 0;
    for (int i = 0; i < n; i++) {  // VALU value -> uniform SGPR -> scalar branch
        uint32_t s = (uint32_t)__builtin_amdgcn_readfirstlane((int)(u * 3u + 1u));
        if (s & 1) cnt++;
        u = s >> 1;
    }
    uint64_t t5 = clock64();
    uint32_t q = u & 4095;
    for (int i = 0; i < n; i++) q = (uint32_t)__builtin_amdgcn_readfirstlane((int)lds[q]) & 4095;  // LDS + rfl (ref)
    uint64_t t6 = clock64();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0; out[1] = t2 - t1; out[2] = t3 - t2; out[3] = t4 - t3; out[4] = t5 - t4; out[5] = t6 - t5;
    }
    sink[threadIdx.x] = v + z + w + u + pos + cnt + q;
}
int main() {
    uint64_t *d; hipMalloc(&d, 128);
    uint32_t *s; hipMalloc(&s, 4096);
    uint64_t r[6];
    int n = 10000;
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, 12345u, n, s);
        hipMemcpy(r, d, 48, hipMemcpyDeviceToHost);
        printf("per iter: 8 dep VALU %.1f | 16 indep VALU %.1f | LDS dep (vgpr addr) %.1f | valu bitstep(alignbit,clz,add) %.1f | valu->rfl->branch %.1f | lds+rfl %.1f\n",
               r[0] / (double)n, r[1] / (double)n, r[2] / (double)n, r[3] / (double)n, r[4] / (double)n, r[5] / (double)n);
    }
    return 0;
}
