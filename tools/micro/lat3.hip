// Scalar-chain cost model on gfx950 (one wave): cycles per instruction for dependent / independent
// SALU, 64-bit shifts, v_readlane -> SALU, M0 + v_writelane, taken / not-taken branches.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define REP10(x) x x x x x x x x x x
__global__ void k(uint64_t *out, uint32_t seed) {
    uint32_t a = __builtin_amdgcn_readfirstlane(seed), b = a + 1, c = a + 2;
    uint64_t w = ((uint64_t)a << 32) | b;
    int v = threadIdx.x;
    uint64_t t[10];
    t[0] = clock64();
    for (int i = 0; i < 100; i++) asm volatile(REP10("s_add_u32 %0, %0, 1\n\t") : "+s"(a) :: "scc");   // dependent
    t[1] = clock64();
    for (int i = 0; i < 100; i++) asm volatile(REP10("s_add_u32 %0, %0, 1\n\ts_add_u32 %1, %1, 1\n\t") : "+s"(a), "+s"(b) :: "scc"); // 2 chains
    t[2] = clock64();
    for (int i = 0; i < 100; i++) asm volatile(REP10("s_lshl_b64 %0, %0, 1\n\t") : "+s"(w) :: "scc");
    t[3] = clock64();
    for (int i = 0; i < 100; i++) asm volatile(REP10("v_readlane_b32 %0, %1, %0\n\ts_and_b32 %0, %0, 63\n\t") : "+s"(c) : "v"(v) : "scc");
    t[4] = clock64();
    for (int i = 0; i < 100; i++) asm volatile(REP10("s_mov_b32 m0, %1\n\ts_nop 0\n\tv_writelane_b32 %0, %1, m0\n\t") : "+v"(v) : "s"(a & 63) : "m0");
    t[5] = clock64();
    for (int i = 0; i < 100; i++) asm volatile(REP10("s_branch 1f\n1:\n\t") ::: );
    t[6] = clock64();
    for (int i = 0; i < 100; i++) asm volatile(REP10("s_cmp_eq_u32 %0, 12345\n\ts_cbranch_scc1 1f\n1:\n\t") :: "s"(a) : "scc");
    t[7] = clock64();
    for (int i = 0; i < 100; i++) asm volatile(REP10("s_flbit_i32_b32 %0, %0\n\ts_or_b32 %0, %0, 0x100\n\t") : "+s"(b) :: "scc");
    t[8] = clock64();
    for (int i = 0; i < 100; i++) asm volatile(REP10("s_cmp_lt_u32 %0, 7\n\ts_cselect_b32 %0, %0, 9\n\t") : "+s"(c) :: "scc");
    t[9] = clock64();
    if (threadIdx.x == 0) {
        for (int j = 0; j < 9; j++) out[j] = t[j + 1] - t[j];
        out[9] = a + b + c + (uint32_t)w + v;
    }
}
int main() {
    uint64_t *d; (void)hipMalloc(&d, 128);
    uint64_t r[10];
    const char *nm[9] = {"dep s_add", "2 indep chains (per op)", "dep s_lshl_b64", "readlane->s_and (per pair)", "m0+nop+writelane (per triple)",
                         "s_branch taken", "cmp+cbranch not taken (per pair)", "flbit+or dep (per pair)", "cmp+cselect dep (per pair)"};
    const double per[9] = {1000, 2000, 1000, 1000, 1000, 1000, 1000, 1000, 1000};
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, 12345u);
        (void)hipMemcpy(r, d, 80, hipMemcpyDeviceToHost);
    }
    for (int j = 0; j < 9; j++) printf("%-34s %.2f cycles\n", nm[j], r[j] / per[j]);
    return 0;
}
