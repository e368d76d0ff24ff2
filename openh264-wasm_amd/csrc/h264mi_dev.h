// h264mi_dev.h -- gfx950 device helpers shared by the encoder, decoder and deblocking kernels.
//
// Spec tables are constexpr so that fully-unrolled per-lane code folds them into immediates;
// tables indexed by runtime values live in __constant__ memory (scalar-cache resident).
// Every function restates an ITU-T H.264 clause (cited) or the encoder rule of DESIGN.md §3.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "h264mi_types.h"

#define DEV __device__ __forceinline__
// Global-address-space pointers. Pointers loaded from descriptors are generic, and generic (flat)
// accesses count against LGKM_CNT as well as VM_CNT: every LDS wait after a flat store would also
// wait for the store to reach memory. Kernels that mix LDS traffic with global stores use these.
#define GLOBAL __attribute__((address_space(1)))
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));  // plain vector types: HIP's uint2/uint4
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // classes cannot live in address space 1
template <class T> __device__ __forceinline__ GLOBAL T *gbl(T *p) { return (GLOBAL T *)(uint64_t)p; }

namespace h264mi {

// ---------------------------------------------------------------- tables (spec)
constexpr uint8_t ZZ[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};       // Table 8-13
constexpr uint8_t BLK2RAS[16] = {0, 1, 4, 5, 2, 3, 6, 7, 8, 9, 12, 13, 10, 11, 14, 15};  // 6.4.3
constexpr uint8_t POSCLS[16] = {0, 2, 0, 2, 2, 1, 2, 1, 0, 2, 0, 2, 2, 1, 2, 1};
__constant__ const int32_t c_MF[6][3] = {{13107, 5243, 8066}, {11916, 4660, 7490}, {10082, 4194, 6554},
                                        {9362, 3647, 5825},  {8192, 3355, 5243},  {7282, 2893, 4559}};
__constant__ const int32_t c_V[6][3] = {{10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};
__constant__ const uint8_t c_CHROMA_QP[52] = {
    0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25,
    26, 27, 28, 29, 29, 30, 31, 32, 32, 33, 34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};
__constant__ const uint8_t c_LAMBDA[52] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 4, 4, 4,
                                           5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 23, 25, 29, 32, 36, 40, 45, 51, 57, 64, 72, 81, 91};

DEV int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
DEV int clip1(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
DEV int iabs(int v) { return v < 0 ? -v : v; }
DEV int median3(int a, int b, int c) { return max(min(a, b), min(max(a, b), c)); }
DEV int ue_len(uint32_t v) { return 2 * (31 - __clz(v + 1)) + 1; }   // v < 2^31
DEV int se_len(int v) { return ue_len(v > 0 ? (uint32_t)(2 * v - 1) : (uint32_t)(-2 * v)); }

// Quantisation constants for one QP (uniform per frame)
struct QuantQP {
    int mf0, mf1, mf2, v0, v1, v2, q6, qbits, fintra, finter;
};
DEV QuantQP make_qqp(int qp) {
    QuantQP q;
    int r = qp % 6;
    q.mf0 = c_MF[r][0]; q.mf1 = c_MF[r][1]; q.mf2 = c_MF[r][2];
    q.v0 = c_V[r][0]; q.v1 = c_V[r][1]; q.v2 = c_V[r][2];
    q.q6 = qp / 6; q.qbits = 15 + q.q6;
    q.fintra = (1 << q.qbits) / 3; q.finter = (1 << q.qbits) / 6;
    return q;
}
template <int POS> DEV int mf_of(const QuantQP &q) { return POSCLS[POS] == 0 ? q.mf0 : (POSCLS[POS] == 1 ? q.mf1 : q.mf2); }
template <int POS> DEV int v_of(const QuantQP &q) { return POSCLS[POS] == 0 ? q.v0 : (POSCLS[POS] == 1 ? q.v1 : q.v2); }
// 32-bit is exact here: |c| <= 9180 (4x4 transform of 8-bit residuals), mf <= 13107, f < 2^23
DEV int quant1(int c, int mf, int qbits, int f) {
    int l = (int)(((uint32_t)iabs(c) * (uint32_t)mf + (uint32_t)f) >> qbits);
    return c < 0 ? -l : l;
}

// ---------------------------------------------------------------- per-lane 4x4 transforms
// forward core transform (exact integer), d/c raster
DEV void fdct4(const int d[16], int c[16]) {
    int t[16];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int s0 = d[4 * i] + d[4 * i + 3], s1 = d[4 * i + 1] + d[4 * i + 2], s2 = d[4 * i + 1] - d[4 * i + 2], s3 = d[4 * i] - d[4 * i + 3];
        t[4 * i + 0] = s0 + s1; t[4 * i + 2] = s0 - s1; t[4 * i + 1] = 2 * s3 + s2; t[4 * i + 3] = s3 - 2 * s2;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        int s0 = t[j] + t[12 + j], s1 = t[4 + j] + t[8 + j], s2 = t[4 + j] - t[8 + j], s3 = t[j] - t[12 + j];
        c[j] = s0 + s1; c[8 + j] = s0 - s1; c[4 + j] = 2 * s3 + s2; c[12 + j] = s3 - 2 * s2;
    }
}
// 8.5.12.2 inverse transform: rows then columns, (x+32)>>6; returns residual r (raster)
DEV void idct4(const int c[16], int r[16]) {
    int t[16];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int e0 = c[4 * i] + c[4 * i + 2], e1 = c[4 * i] - c[4 * i + 2];
        int e2 = (c[4 * i + 1] >> 1) - c[4 * i + 3], e3 = c[4 * i + 1] + (c[4 * i + 3] >> 1);
        t[4 * i + 0] = e0 + e3; t[4 * i + 1] = e1 + e2; t[4 * i + 2] = e1 - e2; t[4 * i + 3] = e0 - e3;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        int e0 = t[j] + t[8 + j], e1 = t[j] - t[8 + j];
        int e2 = (t[4 + j] >> 1) - t[12 + j], e3 = t[4 + j] + (t[12 + j] >> 1);
        r[j] = (e0 + e3 + 32) >> 6; r[4 + j] = (e1 + e2 + 32) >> 6; r[8 + j] = (e1 - e2 + 32) >> 6; r[12 + j] = (e0 - e3 + 32) >> 6;
    }
}
// SATD = (sum |H d H| + 1) >> 1
DEV int satd4(const int d[16]) {
    int t[16], s = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int a0 = d[4 * i] + d[4 * i + 1], a1 = d[4 * i] - d[4 * i + 1], a2 = d[4 * i + 2] + d[4 * i + 3], a3 = d[4 * i + 2] - d[4 * i + 3];
        t[4 * i] = a0 + a2; t[4 * i + 1] = a1 + a3; t[4 * i + 2] = a0 - a2; t[4 * i + 3] = a1 - a3;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        int a0 = t[j] + t[4 + j], a1 = t[j] - t[4 + j], a2 = t[8 + j] + t[12 + j], a3 = t[8 + j] - t[12 + j];
        s += iabs(a0 + a2) + iabs(a1 + a3) + iabs(a0 - a2) + iabs(a1 - a3);
    }
    return (s + 1) >> 1;
}
// quantise a raster coefficient block into scan-ordered levels (positions >= first); returns TotalCoeff
DEV int quant_block(const int c[16], const QuantQP &q, int f, int first, int16_t lv[16]) {
    int n = 0;
#define QK(K)                                                                          \
    {                                                                                  \
        int l = (K) >= first ? quant1(c[ZZ[K]], mf_of<ZZ[K]>(q), q.qbits, f) : 0;      \
        lv[K] = (int16_t)l; n += l != 0;                                               \
    }
    QK(0) QK(1) QK(2) QK(3) QK(4) QK(5) QK(6) QK(7) QK(8) QK(9) QK(10) QK(11) QK(12) QK(13) QK(14) QK(15)
#undef QK
    return n;
}
// 8.5.12.1 flat-matrix scaling: raster coefficients from scan-ordered levels
DEV void dequant_block(const int16_t lv[16], const QuantQP &q, int c[16]) {
#define DK(K) c[ZZ[K]] = (lv[K] * v_of<ZZ[K]>(q)) << q.q6;
    DK(0) DK(1) DK(2) DK(3) DK(4) DK(5) DK(6) DK(7) DK(8) DK(9) DK(10) DK(11) DK(12) DK(13) DK(14) DK(15)
#undef DK
}
// DC terms: |v| <= 32640 (luma, after >> 1) or 16320 (chroma): |v| * mf0 + 2f < 2^32
DEV int quant_dc(int v, int mf0, int qbits, int f) {
    int l = (int)(((uint32_t)iabs(v) * (uint32_t)mf0 + 2u * (uint32_t)f) >> (qbits + 1));
    return v < 0 ? -l : l;
}
// 8.5.10 luma DC scaling of one inverse-Hadamard output
DEV int luma_dc_scale(int f, const QuantQP &q) {
    int x = f * q.v0;
    return q.q6 >= 2 ? (x << (q.q6 - 2)) : ((x + (1 << (1 - q.q6))) >> (2 - q.q6));
}

// ---------------------------------------------------------------- wave helpers (wave64)
DEV int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
DEV int group16_sum(int v) {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// ---------------------------------------------------------------- intra-workgroup LDS hand-offs
// __syncthreads() is a release/acquire fence at workgroup scope: it waits for every outstanding
// global load AND store (vmcnt(0)) before the barrier. The wavefront kernels only hand data to each
// other through LDS, so they use these instead: global traffic stays in flight across them.
// lds_barrier: multi-wave workgroups (this wave's LDS operations done, then s_barrier).
DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// wave_lds_sync: single-wave workgroups -- one wave's LDS requests complete in issue order, so
// only the compiler must not move LDS accesses across this point.
DEV void wave_lds_sync() { asm volatile("" ::: "memory"); }

// ---------------------------------------------------------------- inter-workgroup hand-off (R2 granules)
// 8-byte {tag = epoch, payload} granules written by ONE sc1 (agent-scope atomic) store each and
// polled with agent-scope relaxed loads (MI355X_MICROARCH.md § visibility, R2). Spins are bounded
// and abort on a per-launch error word.
template <class P> DEV void gran_store(P g, uint32_t epoch, uint32_t v) {
    __hip_atomic_store(g, ((uint64_t)epoch << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// lanes [0, n) each poll one granule; returns false on abort/timeout. Payload of lane's granule in *v.
template <class P> DEV bool gran_wait(P g, int n, uint32_t epoch, uint32_t *v, int32_t *abort_word) {
    int lane = threadIdx.x & 63;
    uint32_t val = 0;
    for (unsigned spins = 0;; spins++) {
        bool ok = true;
        if (lane < n) {
            uint64_t x = __hip_atomic_load(g + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            val = (uint32_t)x;
            ok = (uint32_t)(x >> 32) == epoch;
        }
        if (__all(ok)) break;
        if ((spins & 255) == 255) {
            int ab = __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (ab || spins > (1u << 24)) {
                if (lane == 0) __hip_atomic_store(abort_word, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return false;
            }
        }
        __builtin_amdgcn_s_sleep(1);
    }
    *v = val;
    return true;
}

}  // namespace h264mi
