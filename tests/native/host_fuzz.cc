// tests/native/host_fuzz.cc -- sanitizer harness (AddressSanitizer + UndefinedBehaviorSanitizer, built
// and run by tests/test_sanitizers.py) for the host code of the product that handles caller-supplied
// bytes and offsets without a GPU:
//   * h264mi::host_peek_sps (csrc/host_sps.h): the C-ABI decoder's geometry peek over untrusted
//     access units -- real SPS NAL units (written by the oracle's h264o_write_sps), truncated,
//     bit-flipped and random buffers; a peeked geometry must be 1..H264MI_MAX_MBS and, for an intact
//     SPS, the one that was written;
//   * the N-API heap (napi/heap.h): random _malloc/_free sequences against a shadow model (blocks
//     never overlap, stay inside the heap, 16-byte aligned, coalescing returns the whole heap), and
//     the bounds check `ok(off, n)` at extreme arguments.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>
#include "../../openh264-wasm_amd/csrc/host_sps.h"
#include "../../openh264-wasm_amd/napi/heap.h"

extern "C" size_t h264o_write_sps(int w, int h, int bitrate, uint8_t *out);  // oracle (linked in by the harness build)

static uint32_t rs = 0x9E3779B9u;
static uint32_t rnd() { rs ^= rs << 13; rs ^= rs >> 17; rs ^= rs << 5; return rs; }
static int fails = 0;
#define CHECK(c, ...) do { if (!(c)) { std::fprintf(stderr, "FAIL: " __VA_ARGS__); std::fprintf(stderr, "\n"); fails++; } } while (0)

static void fuzz_sps() {
    static const int geo[][2] = {{16, 16}, {176, 144}, {1920, 1080}, {98, 62}, {4096, 2160}};
    for (auto &g : geo) {
        uint8_t sps[128];
        const int n = (int)h264o_write_sps(g[0], g[1], 1000000, sps);
        int w = 0, h = 0;
        CHECK(h264mi::host_peek_sps(sps, n, &w, &h) && w == (g[0] + 15) / 16 && h == (g[1] + 15) / 16,
              "intact SPS %dx%d -> %dx%d MBs", g[0], g[1], w, h);
        for (int t = 0; t < 20000; t++) {
            std::vector<uint8_t> b(sps, sps + n);
            switch (t % 3) {
            case 0: b.resize(1 + rnd() % (uint32_t)n); break;
            case 1: for (int k = 0; k < 1 + t % 7; k++) b[4 + rnd() % (uint32_t)(n - 4)] ^= (uint8_t)(1u << (rnd() & 7)); break;
            case 2: for (size_t k = 4; k < b.size(); k++) b[k] = (uint8_t)rnd(); break;
            }
            // exact-size heap copy, so any over-read is an ASan report
            uint8_t *p = (uint8_t *)std::malloc(b.size());
            std::memcpy(p, b.data(), b.size());
            int pw = -1, ph = -1;
            if (h264mi::host_peek_sps(p, (int)b.size(), &pw, &ph))
                CHECK(pw >= 1 && ph >= 1 && pw <= h264mi::H264MI_MAX_MBS && ph <= h264mi::H264MI_MAX_MBS, "peeked %dx%d", pw, ph);
            std::free(p);
        }
    }
    {  // wider than the decoder supports: the peek must refuse it (the C-ABI keeps its working decoder)
        uint8_t sps[128];
        const int n = (int)h264o_write_sps(16 * (h264mi::H264MI_MAX_MBS + 1), 64, 1000000, sps);
        int w = 0, h = 0;
        CHECK(!h264mi::host_peek_sps(sps, n, &w, &h), "SPS of %d MBs per side accepted", h264mi::H264MI_MAX_MBS + 1);
    }
    for (int t = 0; t < 20000; t++) {  // random buffers with start codes sprinkled in
        const size_t len = rnd() % 300;
        uint8_t *p = (uint8_t *)std::malloc(len ? len : 1);
        for (size_t k = 0; k < len; k++) p[k] = (rnd() & 3) ? (uint8_t)rnd() : 0;
        if (len > 4 && (t & 1)) { p[0] = 0; p[1] = 0; p[2] = 1; p[3] = 0x67; }
        int pw, ph;
        (void)h264mi::host_peek_sps(p, (int)len, &pw, &ph);
        std::free(p);
    }
    int pw, ph;
    CHECK(!h264mi::host_peek_sps(nullptr, 10, &pw, &ph), "null buffer");
}

static void fuzz_heap() {
    const size_t N = 1 << 20;
    std::vector<uint8_t> mem(N);
    Heap h;
    h.init(mem.data(), N);
    std::map<uint32_t, uint32_t> live;  // offset -> requested bytes
    for (int t = 0; t < 200000; t++) {
        if (live.empty() || (rnd() % 3)) {
            const size_t want = (rnd() & 15) == 0 ? rnd() % N : rnd() % 4096;
            const uint32_t off = h.alloc(want);
            if (!off) continue;
            CHECK(off % 16 == 0 && off >= 16 && (size_t)off + want <= N, "alloc %zu -> %u", want, off);
            auto nx = live.lower_bound(off);
            if (nx != live.end()) CHECK((size_t)off + (want ? want : 1) <= nx->first, "overlap with next block");
            if (nx != live.begin()) { auto pv = std::prev(nx); CHECK((size_t)pv->first + pv->second <= off, "overlap with previous block"); }
            std::memset(mem.data() + off, 0xA5, want);
            live[off] = (uint32_t)(want ? want : 1);
        } else {
            auto it = live.begin();
            std::advance(it, rnd() % live.size());
            h.release(it->first);
            live.erase(it);
        }
        if ((t & 1023) == 0) h.release((uint32_t)rnd());  // freeing a non-block is a no-op
    }
    for (auto &kv : live) h.release(kv.first);
    CHECK(h.free_.size() == 1 && h.free_.begin()->first == 16 && h.free_.begin()->second == N - 16, "heap not fully coalesced");
    CHECK(!h.ok(0, 4) && !h.ok(-1, 4) && !h.ok(16, -1), "ok() accepts NULL / negative");
    CHECK(!h.ok((int64_t)N, 1) && h.ok((int64_t)N - 4, 4) && !h.ok((int64_t)N - 3, 4), "ok() at the end of the heap");
    CHECK(!h.ok(INT64_MAX, INT64_MAX) && !h.ok(16, INT64_MAX) && !h.ok(INT64_MAX - 8, 16), "ok() overflow");
    CHECK(h.alloc(N + 1) == 0 && h.alloc((size_t)-1) == 0, "oversized alloc");
}

int main() {
    fuzz_sps();
    fuzz_heap();
    std::printf("host_fuzz: %s (%d failures)\n", fails ? "FAIL" : "ok", fails);
    return fails ? 1 : 0;
}
