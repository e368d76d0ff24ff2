// Checks the parse kernel's asm residual-block decoder (csrc/cavlc_blk.inc blk_decode) against the C++
// one (dec_parse.inc read_block) and the generator's coefficients on random blocks of every nC class
// (tools/micro/blk_gen.py). One wave walks the stream once per decoder. usage: blk_check <blocks.bin>
#include "../../openh264-wasm_amd/csrc/h264mi_dev.h"
#include "../../openh264-wasm_amd/csrc/vlc_tables.inc"
#include "../../openh264-wasm_amd/csrc/dec_parse.inc"
#include <stdio.h>
#include <vector>
using namespace h264mi;
// out per block: [0] tc, [1] bit position after, [2] err, [3] L byte, [4] T byte, [5..20] coefficients
__global__ __launch_bounds__(64) void k(const uint32_t *rb, int ndw, const int *meta, int nb, int use_asm, int *out, uint64_t *cyc) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[RING_BYTES];
    const int lane = threadIdx.x;
    for (int i = lane; i < RING_BYTES / 4; i += 64) ((uint32_t *)ring)[i] = i < ndw ? rb[i] : 0u;
    __syncthreads();
    PT T;
    pt_load(T);
    VR r;
    r.err = 0;
    vr_seek(r, (const uint32_t *)ring, 0);
    GLOBAL int *go = (GLOBAL int *)(uint64_t)out;
    const uint32_t off2 = 2u * (uint32_t)lane;
    uint64_t t = 0;
    for (int b = 0; b < nb; b++) {
        if (r.wi - r.wb >= 16) { r.wb = r.wi & ~15u; vr_load_windows(r, (const uint32_t *)ring); }
        const int na = (int)uni((uint32_t)meta[4 * b]), nbb = (int)uni((uint32_t)meta[4 * b + 1]), maxnum = (int)uni((uint32_t)meta[4 * b + 2]);
        const int base = (int)uni(maxnum == 15 ? 1u : 0u);
        uint32_t L = (uint32_t)na << 8, Tc = (uint32_t)nbb << 16;  // bytes at ys = 8, xs = 16
        r.err = 0;
        GLOBAL int *o = go + (size_t)b * 24;
        int tc;
        const uint64_t t0 = clock64();
        if (use_asm) {
            uint64_t nz = 0;
            GLOBAL int16_t *dst = uni_ptr((int16_t *)(uint64_t)(o + 8));
            if (lane < 8) o[8 + lane] = 0;
            tc = blk_decode(r, T, L, Tc, 8, 16, maxnum, base, dst, off2, nz, 8);
            if (lane == 0) o[6] = (int)(nz >> 8);
        } else {
            int val;
            tc = read_block(r, T, maxnum, nc_of((uint32_t)na, (uint32_t)nbb), base, val);
            L = (L & ~(255u << 8)) | ((uint32_t)tc << 8);
            Tc = (Tc & ~(255u << 16)) | ((uint32_t)tc << 16);
            if (lane < 16) ((GLOBAL int16_t *)(o + 8))[lane] = tc ? (int16_t)val : 0;
            if (lane == 0) o[6] = tc;
        }
        t += clock64() - t0;
        if (lane == 0) { o[0] = tc; o[1] = (int)vr_pos(r); o[2] = (int)r.err; o[3] = (int)((L >> 8) & 255); o[4] = (int)((Tc >> 16) & 255); }
    }
    if (lane == 0) cyc[use_asm] = t;
}
int main(int argc, char **argv) {
    FILE *f = fopen(argv[1], "rb");
    int hdr[2];
    if (!f || fread(hdr, 4, 2, f) != 2) return 2;
    const int nb = hdr[0], ndw = hdr[1];
    std::vector<int> meta(4 * nb);
    std::vector<uint32_t> rb(ndw);
    std::vector<int16_t> exp((size_t)nb * 16);
    if (fread(meta.data(), 4, meta.size(), f) != meta.size() || fread(rb.data(), 4, ndw, f) != (size_t)ndw ||
        fread(exp.data(), 2, exp.size(), f) != exp.size()) return 2;
    fclose(f);
    uint32_t *d_rb; int *d_meta, *d_out[2]; uint64_t *d_cyc;
    if (hipMalloc(&d_rb, 4 * ndw) || hipMalloc(&d_meta, 4 * meta.size()) || hipMalloc(&d_out[0], 96 * nb) || hipMalloc(&d_out[1], 96 * nb) ||
        hipMalloc(&d_cyc, 16)) return 3;
    hipMemcpy(d_rb, rb.data(), 4 * ndw, hipMemcpyHostToDevice);
    hipMemcpy(d_meta, meta.data(), 4 * meta.size(), hipMemcpyHostToDevice);
    for (int m = 0; m < 2; m++) hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d_rb, ndw, d_meta, nb, m, d_out[m], d_cyc);
    std::vector<int> o[2] = {std::vector<int>(24 * nb), std::vector<int>(24 * nb)};
    uint64_t cyc[2];
    for (int m = 0; m < 2; m++) hipMemcpy(o[m].data(), d_out[m], 96 * nb, hipMemcpyDeviceToHost);
    hipMemcpy(cyc, d_cyc, 16, hipMemcpyDeviceToHost);
    int bad = 0, pos = 0;
    for (int b = 0; b < nb && bad < 10; b++) {
        pos += meta[4 * b + 3];
        const int *a = &o[1][24 * b], *c = &o[0][24 * b];
        const int16_t *ac = (const int16_t *)(a + 8), *cc = (const int16_t *)(c + 8), *e = &exp[16 * b];
        bool ok = a[0] == c[0] && a[1] == c[1] && a[2] == c[2] && a[3] == c[3] && a[4] == c[4] && a[6] == a[0] && a[1] == pos && c[2] == 0;
        for (int i = 0; i < 16; i++) ok = ok && ac[i] == cc[i] && cc[i] == e[i];
        if (!ok) {
            bad++;
            printf("block %d (na %d nb %d maxnum %d, %d bits): asm tc %d pos %d err %d L %d T %d nz %d | c++ tc %d pos %d err %d L %d T %d | want pos %d\n  asm:", b,
                   meta[4 * b], meta[4 * b + 1], meta[4 * b + 2], meta[4 * b + 3], a[0], a[1], a[2], a[3], a[4], a[6], c[0], c[1], c[2], c[3], c[4], pos);
            for (int i = 0; i < 16; i++) printf(" %d", ac[i]);
            printf("\n  c++:");
            for (int i = 0; i < 16; i++) printf(" %d", cc[i]);
            printf("\n  exp:");
            for (int i = 0; i < 16; i++) printf(" %d", e[i]);
            printf("\n");
            pos = a[1];  // resynchronise expectations on the asm decoder
        }
    }
    printf("%s: %d blocks, mismatches %d; cycles per block: asm %.1f, c++ %.1f\n", argv[1], nb, bad, (double)cyc[1] / nb, (double)cyc[0] / nb);
    return bad ? 1 : 0;
}
