// h264mi_dev.h -- gfx950 device helpers shared by the encoder, decoder and deblocking kernels.
//
// Spec tables are constexpr so that fully-unrolled per-lane code folds them into immediates;
// tables indexed by runtime values live in __constant__ memory (scalar-cache resident).
// Every function restates an ITU-T H.264 clause (cited) or the encoder rule of DESIGN.md §3.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <atomic>
#include "h264mi_types.h"

#define DEV __device__ __forceinline__
// Global-address-space pointers. Pointers loaded from descriptors are generic, and generic (flat)
// accesses count against LGKM_CNT as well as VM_CNT: every LDS wait after a flat store would also
// wait for the store to reach memory. Kernels that mix LDS traffic with global stores use these.
#define GLOBAL __attribute__((address_space(1)))
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));  // plain vector types: HIP's uint2/uint4
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // classes cannot live in address space 1
template <class T> __device__ __forceinline__ GLOBAL T *gbl(T *p) { return (GLOBAL T *)(uint64_t)p; }
// Constant-address-space view of read-only launch data (descriptors, tables): uniform addresses then
// load through the scalar cache into SGPRs instead of per-lane vector loads.
#define CONSTANT __attribute__((address_space(4)))
template <class T> __device__ __forceinline__ CONSTANT const T *cst(const T *p) { return (CONSTANT const T *)(uint64_t)p; }

namespace h264mi {

// ---------------------------------------------------------------- tables (spec)
constexpr uint8_t ZZ[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};       // Table 8-13
constexpr uint8_t BLK2RAS[16] = {0, 1, 4, 5, 2, 3, 6, 7, 8, 9, 12, 13, 10, 11, 14, 15};  // 6.4.3
constexpr uint8_t POSCLS[16] = {0, 2, 0, 2, 2, 1, 2, 1, 0, 2, 0, 2, 2, 1, 2, 1};
// OpenH264's quantiser tables (g_kiQuantMF / g_kiQuantInterFF as the reference's h264.wasm holds them,
// tests/golden/openh264_tables.json), one entry per coefficient class
// {even/even, odd/odd, mixed} = positions {0, 5, 1} of the 8-wide rows. FF: inter rows qp, intra qp + 6.
__constant__ const int32_t c_QMF[52][3] = {{26214, 10486, 16132}, {23832, 9320, 14980}, {20164, 8388, 13108}, {18724, 7294, 11650}, {16384, 6710, 10486}, {14564, 5786, 9118}, {13107, 5243, 8066}, {11916, 4660, 7490}, {10082, 4194, 6554}, {9362, 3647, 5825}, {8192, 3355, 5243}, {7282, 2893, 4559}, {6554, 2622, 4033}, {5958, 2330, 3745}, {5041, 2097, 3277}, {4681, 1824, 2913}, {4096, 1678, 2622}, {3641, 1447, 2280}, {3277, 1311, 2017}, {2979, 1165, 1873}, {2521, 1049, 1639}, {2341, 912, 1456}, {2048, 839, 1311}, {1821, 723, 1140}, {1638, 655, 1008}, {1490, 583, 936}, {1260, 524, 819}, {1170, 456, 728}, {1024, 419, 655}, {910, 362, 570}, {819, 328, 504}, {745, 291, 468}, {630, 262, 410}, {585, 228, 364}, {512, 210, 328}, {455, 181, 285}, {410, 164, 252}, {372, 146, 234}, {315, 131, 205}, {293, 114, 182}, {256, 105, 164}, {228, 90, 142}, {205, 82, 126}, {186, 73, 117}, {158, 66, 102}, {146, 57, 91}, {128, 52, 82}, {114, 45, 71}, {102, 41, 63}, {93, 36, 59}, {79, 33, 51}, {73, 28, 46}};
__constant__ const int32_t c_QFF[58][3] = {{0, 1, 1}, {0, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 2, 1}, {1, 2, 1}, {1, 2, 1}, {1, 2, 1}, {1, 3, 2}, {1, 3, 2}, {1, 3, 2}, {1, 4, 2}, {2, 4, 3}, {2, 5, 3}, {2, 5, 3}, {2, 6, 4}, {3, 7, 4}, {3, 8, 5}, {3, 8, 5}, {4, 9, 6}, {4, 10, 7}, {5, 12, 8}, {5, 13, 8}, {6, 15, 10}, {7, 17, 11}, {7, 19, 12}, {9, 21, 13}, {9, 24, 15}, {11, 26, 17}, {12, 30, 19}, {13, 33, 22}, {15, 38, 23}, {17, 42, 27}, {19, 48, 30}, {21, 52, 33}, {24, 60, 38}, {27, 67, 43}, {29, 75, 47}, {35, 83, 53}, {37, 96, 60}, {43, 104, 67}, {48, 121, 77}, {53, 133, 87}, {59, 150, 93}, {69, 167, 107}, {75, 192, 120}, {85, 208, 133}, {96, 242, 153}, {107, 267, 173}, {117, 300, 187}, {139, 333, 213}, {149, 383, 240}, {171, 417, 267}, {192, 483, 307}, {213, 533, 347}, {235, 600, 373}, {277, 667, 427}, {299, 767, 480}};
__constant__ const int32_t c_V[6][3] = {{10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};
__constant__ const uint8_t c_CHROMA_QP[52] = {
    0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25,
    26, 27, 28, 29, 29, 30, 31, 32, 32, 33, 34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};
__constant__ const uint8_t c_LAMBDA[52] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 4, 4, 4,
                                           5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 23, 25, 29, 32, 36, 40, 45, 51, 57, 64, 72, 81, 91};

// Rate control: OpenH264's g_kiQpToQstepTable (h264.wasm linear address 43696, pinned by
// tests/golden/openh264_tables.json "rc_qstep"), and RcConvertQStep2Qp as thresholds: QP k >= 1 for a QStep at or
// above THR[k - 1]. The wasm computes trunc(6 * logf(QStep / 100.0f) / ln 2 + 4.5) with musl's logf (func 483);
// tests/test_rc.py checks these thresholds against the oracle's restatement of that function over every QStep up
// to 400000. QPs above 52 are never used: every result is clipped into the camera range [12, 42].
#define H264MI_RC_QSTEP_LIST 63, 71, 79, 89, 100, 112, 126, 141, 159, 178, 200, 224, 252, 283, 317, 356, 400, 449, 504, \
    566, 635, 713, 800, 898, 1008, 1131, 1270, 1425, 1600, 1796, 2016, 2263, 2540, 2851, 3200, 3592, 4032, 4525, 5080, \
    5702, 6400, 7184, 8063, 9051, 10159, 11404, 12800, 14368, 16127, 18102, 20319, 22807
#define H264MI_RC_QP_THR_LIST 67, 75, 85, 95, 106, 119, 134, 150, 169, 189, 212, 238, 267, 300, 337, 378, 424, 476, 534, \
    600, 673, 756, 848, 952, 1068, 1199, 1346, 1511, 1696, 1903, 2136, 2398, 2691, 3021, 3391, 3806, 4272, 4795, 5382, \
    6041, 6781, 7611, 8543, 9590, 10764, 12082, 13562, 15222, 17086, 19179, 21527, 24164
__constant__ const int32_t c_RC_QSTEP[52] = {H264MI_RC_QSTEP_LIST};
__constant__ const int32_t c_RC_QP_THR[52] = {H264MI_RC_QP_THR_LIST};

DEV int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
DEV int clip1(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
// Clip1(x >> s) for byte-packed results. Clamp-first form: hipcc (ROCm 7.2, gfx950) selects
// v_ashr_pk_u8_i32 for "shift, saturate, pack two bytes" and then assumes the instruction's upper 16
// bits are zero, corrupting the neighbouring bytes.
DEV int clip1_shr(int x, int s) { return min(max(x, 0), (256 << s) - 1) >> s; }
DEV int iabs(int v) { return v < 0 ? -v : v; }
DEV int median3(int a, int b, int c) { return max(min(a, b), min(max(a, b), c)); }
DEV int ue_len(uint32_t v) { return 2 * (31 - __clz(v + 1)) + 1; }   // v < 2^31
DEV int se_len(int v) { return ue_len(v > 0 ? (uint32_t)(2 * v - 1) : (uint32_t)(-2 * v)); }

// Quantisation constants for one QP (uniform per frame)
struct QuantQP {
    int mf0, mf1, mf2, fi0, fi1, fi2, fp0, fp1, fp2, v0, v1, v2, q6;
};
DEV QuantQP make_qqp(int qp) {
    QuantQP q;
    int r = qp % 6;
    q.mf0 = c_QMF[qp][0]; q.mf1 = c_QMF[qp][1]; q.mf2 = c_QMF[qp][2];
    q.fi0 = c_QFF[qp + 6][0]; q.fi1 = c_QFF[qp + 6][1]; q.fi2 = c_QFF[qp + 6][2];
    q.fp0 = c_QFF[qp][0]; q.fp1 = c_QFF[qp][1]; q.fp2 = c_QFF[qp][2];
    q.v0 = c_V[r][0]; q.v1 = c_V[r][1]; q.v2 = c_V[r][2];
    q.q6 = qp / 6;
    return q;
}
// per-lane class selects of single fields (a select of the struct or of an array would go through scratch)
DEV int qmf(const QuantQP &q, int cls) { return cls == 0 ? q.mf0 : (cls == 1 ? q.mf1 : q.mf2); }
DEV int qff(const QuantQP &q, int cls, int intra) {
    const int f0 = intra ? q.fi0 : q.fp0, f1 = intra ? q.fi1 : q.fp1, f2 = intra ? q.fi2 : q.fp2;  // uniform
    return cls == 0 ? f0 : (cls == 1 ? f1 : f2);
}
template <int POS> DEV int mf_of(const QuantQP &q) { return POSCLS[POS] == 0 ? q.mf0 : (POSCLS[POS] == 1 ? q.mf1 : q.mf2); }
template <int POS> DEV int ff_of(const QuantQP &q, int intra) { return qff(q, POSCLS[POS], intra); }
template <int POS> DEV int v_of(const QuantQP &q) { return POSCLS[POS] == 0 ? q.v0 : (POSCLS[POS] == 1 ? q.v1 : q.v2); }
// OpenH264's quantiser (WelsQuant4x4_c): level = sign(c) * (((|c| + ff) * mf) >> 16). 32-bit exact:
// |c| <= 9180 (4x4 transform of 8-bit residuals), ff <= 767, mf <= 26214
DEV int quant1(int c, int mf, int ff) {
    int l = (int)((((uint32_t)iabs(c) + (uint32_t)ff) * (uint32_t)mf) >> 16);
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
DEV int quant_block(const int c[16], const QuantQP &q, int intra, int first, int16_t lv[16]) {
    int n = 0;
#define QK(K)                                                                                   \
    {                                                                                           \
        int l = (K) >= first ? quant1(c[ZZ[K]], mf_of<ZZ[K]>(q), ff_of<ZZ[K]>(q, intra)) : 0;   \
        lv[K] = (int16_t)l; n += l != 0;                                                        \
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
// DC levels (I16x16 luma DC after the Hadamard, chroma 2x2 DC): OpenH264 quantises them with
// (int16)(FF[0] << 1) and MF[0] >> 1 (WelsQuant4x4Dc / WelsHadamardQuant2x2). |v| <= 32640 (luma) or
// 16320 (chroma): (|v| + 2 ff0) * (mf0 >> 1) < 2^31
DEV int quant_dc(int v, int mf0, int ff0) {
    int l = (int)((((uint32_t)iabs(v) + 2u * (uint32_t)ff0) * ((uint32_t)mf0 >> 1)) >> 16);
    return v < 0 ? -l : l;
}
// 8.5.10 luma DC scaling of one inverse-Hadamard output
DEV int luma_dc_scale(int f, const QuantQP &q) {
    int x = f * q.v0;
    return q.q6 >= 2 ? (x << (q.q6 - 2)) : ((x + (1 << (1 - q.q6))) >> (2 - q.q6));
}

// ---------------------------------------------------------------- wave helpers (wave64)
// A value every lane holds identically (read from LDS, reduced across lanes, ...) moved to an SGPR:
// the compiler then treats what depends on it as uniform -- scalar branches and scalar table loads
// instead of exec-mask juggling and per-lane global loads.
DEV int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
// Cross-lane reductions on DPP (data-parallel primitives: an operand modifier of the VALU, no LDS
// round trip; __shfl_* lowers to ds_bpermute, ~100+ cycles each on a dependent chain).
// DPP controls: quad_perm [1,0,3,2] = 0xB1 (xor 1), [2,3,0,1] = 0x4E (xor 2), row_ror:4 = 0x124,
// row_ror:8 = 0x128, row_half_mirror = 0x141 (lane i <-> 7-i within 8). All lanes read a valid source.
template <int CTRL> DEV int dpp(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }
DEV int lane_read(int v, int l) { return __builtin_amdgcn_readlane(v, l); }  // l uniform
// total of each 16-lane row (lanes 16r..16r+15), in every lane of the row
DEV int group16_sum(int v) {
    v += dpp<0xB1>(v); v += dpp<0x4E>(v); v += dpp<0x124>(v); v += dpp<0x128>(v);
    return v;
}
DEV int group16_min(int v) {
    v = min(v, dpp<0xB1>(v)); v = min(v, dpp<0x4E>(v)); v = min(v, dpp<0x124>(v)); v = min(v, dpp<0x128>(v));
    return v;
}
// total of each 8-lane group, in every lane of the group
DEV int group8_sum(int v) {
    v += dpp<0xB1>(v); v += dpp<0x4E>(v); v += dpp<0x141>(v);
    return v;
}
// wave64 total / minimum, returned uniform (SGPR)
DEV int wave_sum(int v) {
    v = group16_sum(v);
    return lane_read(v, 0) + lane_read(v, 16) + lane_read(v, 32) + lane_read(v, 48);
}
DEV int wave_min(int v) {
    v = group16_min(v);
    return min(min(lane_read(v, 0), lane_read(v, 16)), min(lane_read(v, 32), lane_read(v, 48)));
}

// ---------------------------------------------------------------- lane-per-coefficient 4x4 transforms
// A 4x4 block lives on 16 consecutive lanes, lane & 15 = 4r + c (raster). A 1-D pass along a row
// reads the other three samples of its quad with quad_perm DPP; a pass along a column reads rows
// (r+1)&3, (r+2)&3, (r+3)&3 with row_ror:12/8/4 (lane l <- lane (l - n) mod 16; checked on gfx950,
// tools/micro/dpp.hip), so the column pass uses lane-constant coefficients in rotated order. The
// coefficients of each pass are packed as 4 signed bytes in one VGPR (Xf), built once per kernel.
DEV int sbyte(uint32_t p, int k) { return __builtin_amdgcn_sbfe((int)p, 8 * k, 8); }
DEV int m24(int a, int b) { return __mul24(a, b); }  // v_mul_i32_i24: both operands |x| < 2^23
// out = sum_k m_k x_(row r, column k)
DEV int xf_row(int x, uint32_t m) {
    return m24(sbyte(m, 0), dpp<0x00>(x)) + m24(sbyte(m, 1), dpp<0x55>(x)) + m24(sbyte(m, 2), dpp<0xAA>(x)) + m24(sbyte(m, 3), dpp<0xFF>(x));
}
// out = sum_j m_j x_(row (r+j)&3, column c)
DEV int xf_col(int x, uint32_t m) {
    return m24(sbyte(m, 0), x) + m24(sbyte(m, 1), dpp<0x12C>(x)) + m24(sbyte(m, 2), dpp<0x128>(x)) + m24(sbyte(m, 3), dpp<0x124>(x));
}
// inverse core transform pass (8.5.12.2): coefficient k enters halved where the matrix has 1/2;
// sh holds one shift bit per k (same order as m)
DEV int xf_row_inv(int x, uint32_t m, uint32_t sh) {
    return m24(sbyte(m, 0), dpp<0x00>(x) >> (sh & 1)) + m24(sbyte(m, 1), dpp<0x55>(x) >> ((sh >> 1) & 1)) +
           m24(sbyte(m, 2), dpp<0xAA>(x) >> ((sh >> 2) & 1)) + m24(sbyte(m, 3), dpp<0xFF>(x) >> ((sh >> 3) & 1));
}
DEV int xf_col_inv(int x, uint32_t m, uint32_t sh) {
    return m24(sbyte(m, 0), x >> (sh & 1)) + m24(sbyte(m, 1), dpp<0x12C>(x) >> ((sh >> 1) & 1)) +
           m24(sbyte(m, 2), dpp<0x128>(x) >> ((sh >> 2) & 1)) + m24(sbyte(m, 3), dpp<0x124>(x) >> ((sh >> 3) & 1));
}
constexpr int XF_FWD[4][4] = {{1, 1, 1, 1}, {2, 1, -1, -2}, {1, -1, -1, 1}, {1, -2, 2, -1}};   // 8.5 core transform
constexpr int XF_HAD[4][4] = {{1, 1, 1, 1}, {1, 1, -1, -1}, {1, -1, -1, 1}, {1, -1, 1, -1}};   // 8-320 / 8-326
constexpr int XF_INV[4][4] = {{1, 1, 1, 1}, {1, 1, -1, -1}, {1, -1, -1, 1}, {1, -1, 1, -1}};   // signs of 8-338..8-345
constexpr int XF_INVSH[4][4] = {{0, 0, 0, 1}, {0, 1, 0, 0}, {0, 1, 0, 0}, {0, 0, 0, 1}};        // the 1/2 factors
constexpr uint8_t XF_INVZZ[16] = {0, 1, 5, 6, 2, 4, 7, 12, 3, 8, 11, 13, 9, 10, 14, 15};         // raster -> scan (Table 8-13)
struct Xf {
    uint32_t fr, fc, hr, hc, ir, ic;  // packed coefficient bytes per pass
    uint32_t irs, ics;                // inverse shift bits per pass
    int cls, zz;                      // quantiser position class (0: even/even, 1: odd/odd, 2: mixed), scan index
};
DEV Xf xf_consts(int pos) {
    const int r = pos >> 2, c = pos & 3;
    Xf x{};
    for (int k = 0; k < 4; k++) {
        const int j = (r + k) & 3;
        x.fr |= (uint32_t)(XF_FWD[c][k] & 255) << (8 * k);
        x.fc |= (uint32_t)(XF_FWD[r][j] & 255) << (8 * k);
        x.hr |= (uint32_t)(XF_HAD[c][k] & 255) << (8 * k);
        x.hc |= (uint32_t)(XF_HAD[r][j] & 255) << (8 * k);
        x.ir |= (uint32_t)(XF_INV[c][k] & 255) << (8 * k);
        x.ic |= (uint32_t)(XF_INV[r][j] & 255) << (8 * k);
        x.irs |= (uint32_t)XF_INVSH[c][k] << k;
        x.ics |= (uint32_t)XF_INVSH[r][j] << k;
    }
    x.cls = ((r | c) & 1) == 0 ? 0 : (((r & c) & 1) ? 1 : 2);
    x.zz = XF_INVZZ[pos];
    return x;
}
DEV int xf_fwd(int d, const Xf &x) { return xf_col(xf_row(d, x.fr), x.fc); }
DEV int xf_had(int d, const Xf &x) { return xf_col(xf_row(d, x.hr), x.hc); }
DEV int xf_inv(int w, const Xf &x) { return xf_col_inv(xf_row_inv(w, x.ir, x.irs), x.ic, x.ics); }
DEV uint32_t popc(uint64_t m) { return (uint32_t)__builtin_popcountll(m); }

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
// two consecutive granules {epoch, a}, {epoch, b} from one lane: one 16-byte write-through (sc1) store
// (cdna_hip_programming.md Guideline 16 R1 store form; each 8-byte half is a complete granule, which
// consumers poll as before). Halves the store instructions of a granule hand-off. base: wave-uniform
// (the buffer descriptor lives in SGPRs), idx: the lane's first granule, even.
#ifndef H264MI_GRAN16
#define H264MI_GRAN16 1
#endif
template <class P> DEV void gran_store2(P base, int idx, uint32_t epoch, uint32_t a, uint32_t b) {
#if H264MI_GRAN16
    const u32x4 v = {a, epoch, b, epoch};
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)(uint64_t)base, (short)0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, idx * 8, 0, 16);
#else
    gran_store(base + idx, epoch, a);
    gran_store(base + idx + 1, epoch, b);
#endif
}
// Every GPU-side hand-off wait gives up (abort) after H264MI_WAIT_LIMIT_MS of the constant 100 MHz clock,
// checked every 256 polls (the clock starts at the first check): a time budget rather than a spin count, so
// contention that slows the polls cannot turn a legitimately long wait into an abort, and the budget does not
// depend on the poll's latency (round 4: spins > 2^24).
#ifndef H264MI_WAIT_LIMIT_MS
#define H264MI_WAIT_LIMIT_MS 2000
#endif
// The budget is a device global (ticks of the 100 MHz clock): the host sets it from the environment variable
// H264MI_WAIT_LIMIT_MS when an encoder or decoder is created (wait_limit_from_env), e.g. for a GPU shared with
// other processes. One WaitClock bounds one whole wait: gran_wait / the deblocking rows' get() pass theirs to
// gran_wait1, so a wait over a set of granules is bounded by one budget, not one per stale granule.
__device__ uint64_t g_wait_limit_ticks = (uint64_t)H264MI_WAIT_LIMIT_MS * 100000u;
struct WaitClock {
    uint64_t t0 = 0;
    DEV bool expired() {
        const uint64_t t = __builtin_amdgcn_s_memrealtime();
        if (t0 == 0) { t0 = t; return false; }
        return t - t0 > __hip_atomic_load(&g_wait_limit_ticks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
};

// Wait until the granule at g carries epoch, polling it alone (one 8-byte load, the same address on every
// lane: one request). gran_wait / DbkSrcGranules use it on the first stale granule of a set instead of
// re-polling the whole set: a stale poll of a 128-granule record was ~1.3 KB of fabric reads. false on
// abort/timeout; spins carries the caller's poll count (abort check every 256).
#ifndef H264MI_GRAN_WAIT1
#define H264MI_GRAN_WAIT1 1
#endif
template <class P> DEV bool gran_wait1(P g, uint32_t epoch, int32_t *abort_word, unsigned &spins, WaitClock &wc) {
    for (;; spins++) {
        if ((spins & 255) == 255) {
            int ab = __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (ab || wc.expired()) {
                if ((threadIdx.x & 63) == 0) __hip_atomic_store(abort_word, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return false;
            }
        }
        __builtin_amdgcn_s_sleep(1);
        const uint64_t y = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(y >> 32) == epoch) return true;
    }
}

// lanes [0, n) each poll one granule; returns false on abort/timeout. Payload of lane's granule in *v.
// A stale set waits on its first stale granule alone, then reloads the set.
template <class P> DEV bool gran_wait(P g, int n, uint32_t epoch, uint32_t *v, int32_t *abort_word) {
    int lane = threadIdx.x & 63;
    uint32_t val = 0;
    WaitClock wc;
    for (unsigned spins = 0;; spins++) {
        bool ok = true;
        if (lane < n) {
            uint64_t x = __hip_atomic_load(g + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            val = (uint32_t)x;
            ok = (uint32_t)(x >> 32) == epoch;
        }
        const uint64_t bad = __ballot(!ok);
        if (bad == 0) break;
#if H264MI_GRAN_WAIT1
        if (!gran_wait1(g + (int)__builtin_ctzll(bad), epoch, abort_word, spins, wc)) return false;
#else
        if ((spins & 255) == 255) {
            int ab = __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (ab || wc.expired()) {
                if (lane == 0) __hip_atomic_store(abort_word, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return false;
            }
        }
        __builtin_amdgcn_s_sleep(1);
#endif
    }
    *v = val;
    return true;
}

// one granule per lane, already loaded into x (e.g. one step ahead); lanes with need poll it until its
// tag is epoch. Returns false on abort/timeout.
// Every exit is preceded by an explicit vmcnt(0) wait, free at run time (the test that ends the loop has just waited
// for the last reload, the youngest memory operation). Without it the compiler's wait analysis saw a path that left
// the loop with a reload still in flight (the exits share a block) and charged its destination registers as pending
// to the rest of the MB loop: a vmcnt(0) on the P path's first write of them, next MB, which then also waited for that
// MB's window prefetch and the previous MB's output stores (~1 us a MB; profiles/round6/eprof/README).
#define H264MI_WAIT_VM0() __builtin_amdgcn_s_waitcnt(0x0F70)  // s_waitcnt vmcnt(0) (gfx9 encoding: expcnt 7, lgkmcnt 15)
// The first test is outside the loop: a granule set loaded well ahead (and already waited for) is used with no wait
// at all -- a test at the loop's head waited for whatever the loop's reload left pending, i.e. vmcnt(0) on entry too.
template <class P> DEV bool gran_poll(P g, bool need, uint32_t epoch, uint64_t &x, int32_t *abort_word) {
    if (__all(!need || (uint32_t)(x >> 32) == epoch)) return true;
    WaitClock wc;
    for (unsigned spins = 0;; spins++) {
        if (spins > 0 && __all(!need || (uint32_t)(x >> 32) == epoch)) { H264MI_WAIT_VM0(); return true; }
        if ((spins & 255) == 255) {
            int ab = __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (ab || wc.expired()) {
                if ((threadIdx.x & 63) == 0) __hip_atomic_store(abort_word, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                H264MI_WAIT_VM0();
                return false;
            }
        }
        __builtin_amdgcn_s_sleep(1);
        if (need) x = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// QPY entering MB row r of an encoder frame: the slice QP for row 0, else the value
// row r - 1 publishes in rowq[r] (its row QP as soon as it codes an MB carrying mb_qp_delta, or the
// QPY it entered with if it codes none). Wave-uniform; false on abort/timeout.
template <class P> DEV bool row_entry_qp(P rowq, int r, int slice_qp, uint32_t epoch, int32_t *abort_word, int *qp) {
    if (r == 0) { *qp = slice_qp; return true; }
    uint32_t v = 0;
    if (!gran_wait(rowq + r, 1, epoch, &v, abort_word)) return false;
    *qp = __builtin_amdgcn_readfirstlane((int)v);
    return true;
}

}  // namespace h264mi
