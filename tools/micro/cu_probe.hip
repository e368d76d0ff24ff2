// Which CUs do a stream's workgroups land on? Launches 2048 one-wave workgroups on a stream created with
// a CU mask (bits [lo, hi) of the mask, or its complement) and counts the distinct (XCC, SE, SH, CU)
// placements read from HW_REG_HW_ID / HW_REG_XCC_ID. Used to check that hipExtStreamCreateWithCUMask
// partitions the chip the way the decoder's reserved parse CUs assume (runtime_dec.inc).
// usage: cu_probe <lo> <hi>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <set>
#include <vector>
__global__ void probe(uint32_t *out) {
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_REG_HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
    const uint64_t t0 = clock64();
    while (clock64() - t0 < 200000) {}  // keep the slot busy so later workgroups spread out
    if (threadIdx.x == 0) out[blockIdx.x] = (xcc << 16) | (((hw >> 13) & 3) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15);
}
static std::set<uint32_t> run(const std::vector<uint32_t> &mask, uint32_t *d, int n) {
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) { printf("mask stream failed\n"); exit(1); }
    hipLaunchKernelGGL(probe, dim3(n), dim3(64), 0, s, d);
    std::vector<uint32_t> h(n);
    if (hipStreamSynchronize(s) != hipSuccess || hipMemcpy(h.data(), d, 4 * n, hipMemcpyDeviceToHost) != hipSuccess) exit(1);
    hipStreamDestroy(s);
    return std::set<uint32_t>(h.begin(), h.end());
}
int main(int argc, char **argv) {
    const int lo = atoi(argv[1]), hi = atoi(argv[2]);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int ncu = p.multiProcessorCount, words = (ncu + 31) / 32, n = 2048;
    std::vector<uint32_t> in(words, 0), out(words, 0);
    for (int i = 0; i < ncu; i++) ((i >= lo && i < hi) ? in : out)[i / 32] |= 1u << (i % 32);
    uint32_t *d;
    hipMalloc(&d, 4 * n);
    auto a = run(in, d, n), b = run(out, d, n);
    int common = 0;
    for (uint32_t x : a) common += b.count(x);
    std::set<uint32_t> xa;
    for (uint32_t x : a) xa.insert(x >> 16);
    printf("CUs %d; mask bits [%d,%d): %zu distinct CUs on %zu XCCs; complement: %zu CUs; shared: %d\n", ncu, lo, hi, a.size(), xa.size(),
           b.size(), common);
    return 0;
}
