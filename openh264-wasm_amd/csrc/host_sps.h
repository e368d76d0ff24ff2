// host_sps.h -- host-side SPS peek (plain C++, no HIP: also compiled into the sanitizer harness
// tests/native/host_fuzz.cc).
//
// The C-ABI decoder is created without dimensions (openh264_wrapper.cpp:253-280); its buffers are
// sized from the first SPS seen in the caller's access unit. Only pic_width/height_in_mbs are read
// here; the full SPS/PPS/slice parse runs on the GPU (dec_parse.inc). The input is untrusted caller
// memory: every read is bounds-checked, the Exp-Golomb reader saturates instead of overflowing, and a
// geometry outside 1..H264MI_MAX_MBS macroblocks per side is rejected.
#pragma once
#include <cstdint>
#include <vector>

namespace h264mi {

// per side: 4096 luma samples. The one limit for the peek and the decoder's allocation (dec_create):
// an SPS the peek accepts is one the decoder can be created for.
constexpr int H264MI_MAX_MBS = 256;

inline bool host_peek_sps(const uint8_t *d, int n, int *mbw, int *mbh) {
    if (!d || n <= 0) return false;
    for (int i = 0; i + 4 < n; i++) {
        if (!(d[i] == 0 && d[i + 1] == 0 && d[i + 2] == 1)) continue;
        const int s = i + 3;
        if ((d[s] & 31) != 7) continue;
        std::vector<uint8_t> rb;  // RBSP of the SPS (emulation-prevention bytes removed), first 256 bytes
        int z = 0;
        for (int k = s + 1; k < n && rb.size() < 256; k++) {
            if (z >= 2 && d[k] == 3) { z = 0; continue; }
            if (z >= 2 && d[k] == 1) break;  // next start code
            rb.push_back(d[k]);
            z = d[k] == 0 ? z + 1 : 0;
        }
        size_t pos = 0;
        auto bit = [&]() -> uint32_t {
            if (pos >= rb.size() * 8) return 0;
            const uint32_t v = (rb[pos >> 3] >> (7 - (pos & 7))) & 1u;
            pos++;
            return v;
        };
        auto bits = [&](int k) { uint32_t v = 0; for (int q = 0; q < k; q++) v = (v << 1) | bit(); return v; };
        auto ue = [&]() -> uint32_t {  // saturates at 2^31 - 1 (any larger value is invalid here anyway)
            int lz = 0;
            while (lz < 32 && bit() == 0) lz++;
            if (lz >= 31) return 0x7fffffffu;
            return ((1u << lz) - 1u) + bits(lz);
        };
        const uint32_t profile = bits(8);
        bits(16);
        ue();
        if (profile == 100 || profile == 110 || profile == 122 || profile == 244) return false;
        ue();
        const uint32_t poc_type = ue();
        if (poc_type == 0) ue();
        else if (poc_type == 1) {
            bit(); ue(); ue();
            const uint32_t c = ue();
            for (uint32_t q = 0; q < c && q < 256; q++) ue();
        }
        ue(); bit();
        const uint32_t w = ue(), h = ue();
        if (w >= (uint32_t)H264MI_MAX_MBS || h >= (uint32_t)H264MI_MAX_MBS) return false;
        *mbw = (int)w + 1;
        *mbh = (int)h + 1;
        return true;
    }
    return false;
}

}  // namespace h264mi
