// Micro-benchmark of the slice-data chain's residual_block_cavlc (dec_parse.inc read_block) on one
// wave: cycles per block for a synthetic block stream (tools/micro/cavlc_gen.py), decoded
// coefficients checked against the generator's. usage: cavlc_bench <stream.bin>
#include "../../openh264-wasm_amd/csrc/h264mi_dev.h"
#include "../../openh264-wasm_amd/csrc/vlc_tables.inc"
#include "../../openh264-wasm_amd/csrc/dec_parse.inc"
#include <stdio.h>
#include <vector>
using namespace h264mi;
__global__ __launch_bounds__(64) void k(const uint32_t *rb, int ndw, int nblocks, int maxnum, int16_t *coefs, uint64_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[RING_BYTES];
    __shared__ Ring RS;
    const int lane = threadIdx.x;
    for (int i = lane; i < RING_BYTES / 4; i += 64) ((uint32_t *)ring)[i] = i < ndw ? rb[i] : 0u;
    __syncthreads();
    PT T;
    pt_load(T);
    VR r;
    r.err = 0;
    vr_seek(r, (const uint32_t *)ring, 0);
    uint32_t refill_at = ~0u;
    const int base = maxnum == 15 ? 1 : 0;
    uint64_t sum = 0;
    GLOBAL int16_t *gc = (GLOBAL int16_t *)(uint64_t)coefs;
    const uint64_t t0 = clock64();
    for (int i = 0; i < nblocks; i++) {
        vr_slide(r, RS, ring, refill_at);
        int val;
        const int tc = read_block(r, T, maxnum, 0, base, val);
        sum += tc;
        if (tc && lane < 16) gc[i * 16 + lane] = (int16_t)val;
    }
    const uint64_t t1 = clock64();
    if (lane == 0) { out[0] = t1 - t0; out[1] = sum; out[2] = vr_pos(r); out[3] = r.err; }
}
int main(int argc, char **argv) {
    FILE *f = fopen(argv[1], "rb");
    int hdr[4];
    if (!f || fread(hdr, 4, 4, f) != 4) return 2;
    const int nb = hdr[0], maxnum = hdr[1], ndw = hdr[3];
    std::vector<uint32_t> rb(ndw);
    std::vector<int16_t> exp((size_t)nb * 16), got((size_t)nb * 16, 0);
    if (fread(rb.data(), 4, ndw, f) != (size_t)ndw || fread(exp.data(), 2, exp.size(), f) != exp.size()) return 2;
    fclose(f);
    uint32_t *d_rb; int16_t *d_c; uint64_t *d_o;
    if (hipMalloc(&d_rb, 4 * ndw) || hipMalloc(&d_c, 2 * exp.size()) || hipMalloc(&d_o, 64)) return 3;
    if (hipMemcpy(d_rb, rb.data(), 4 * ndw, hipMemcpyHostToDevice)) return 3;
    uint64_t o[4] = {0, 0, 0, 0};
    for (int rep = 0; rep < 3; rep++) {
        if (hipMemset(d_c, 0, 2 * exp.size())) return 3;
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d_rb, ndw, nb, maxnum, d_c, d_o);
        if (hipMemcpy(o, d_o, 32, hipMemcpyDeviceToHost) || hipMemcpy(got.data(), d_c, 2 * got.size(), hipMemcpyDeviceToHost)) return 3;
    }
    size_t bad = 0;
    for (size_t i = 0; i < exp.size(); i++) bad += exp[i] != got[i];
    printf("%s: %d blocks maxnum %d: %.1f cycles/block, sum tc %llu, bits %llu, err %llu, coefficient mismatches %zu\n", argv[1], nb, maxnum,
           (double)o[0] / nb, (unsigned long long)o[1], (unsigned long long)o[2], (unsigned long long)o[3], bad);
    return bad || o[3] ? 1 : 0;
}
