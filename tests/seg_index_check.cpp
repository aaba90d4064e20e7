// Host check of the trace launches' queue indexing (nori-ray-tracer_amd/csrc/
// seg_index.h), compiled with g++ by tests/test_seg_index.py.  For segment
// counts G = 1..67 (multiples of kTraceGroup and not) and count patterns with
// empty, partial, full and trailing segments, it walks every (work-group,
// thread, ray) of each trace launch shape exactly as the kernels do and
// asserts: every index a thread loads lies inside the queue (< G * kSeg) and
// inside its segment's count, and the live rays cover every queued entry
// exactly once.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "seg_index.h"

using namespace nori;

static int fails = 0;
#define CHECK(c, ...)                                  \
    do {                                               \
        if (!(c)) {                                    \
            if (fails++ < 20) std::printf(__VA_ARGS__); \
        }                                              \
    } while (0)

static void run(const std::vector<uint32_t> &cnt, uint32_t per, uint32_t B, uint32_t K, const char *name) {
    const uint32_t G = (uint32_t)cnt.size();
    std::vector<int> seen((size_t)G * kSeg, 0);
    const uint32_t grid = seg_grid(G, per);
    for (uint32_t bid = 0; bid < grid; ++bid) {
        const SegRange sr = seg_group(cnt.data(), G, bid, per);
        const uint32_t n = sr.pre[kTraceGroup];
        CHECK(sr.s0 < G, "%s G=%u bid=%u: group start %u past the queue\n", name, G, bid, sr.s0);
        for (uint32_t t = 0; t < B; ++t) {
            const uint32_t i0 = seg_first(bid, per, B, K, t);
            if (i0 >= n) continue;  // the kernels return here
            for (uint32_t k = 0; k < K; ++k) {
                const uint32_t i = i0 + k * B;
                const bool live = i < n;
                const uint32_t q = seg_entry(sr, live ? i : i0);
                CHECK(q < G * kSeg, "%s G=%u bid=%u t=%u k=%u: index %u >= %u\n", name, G, bid, t, k, q, G * kSeg);
                if (q >= G * kSeg) continue;
                CHECK(q % kSeg < cnt[q / kSeg], "%s G=%u bid=%u t=%u k=%u: slot %u of segment %u past its count %u\n",
                      name, G, bid, t, k, q % kSeg, q / kSeg, cnt[q / kSeg]);
                if (live) ++seen[q];
            }
        }
    }
    for (uint32_t s = 0; s < G; ++s)
        for (uint32_t j = 0; j < kSeg; ++j) {
            const int want = j < cnt[s] ? 1 : 0;
            CHECK(seen[(size_t)s * kSeg + j] == want, "%s G=%u: entry %u of segment %u traced %d times (want %d)\n",
                  name, G, j, s, seen[(size_t)s * kSeg + j], want);
        }
}

int main() {
    // the launch shapes of kernels.hip: BVH walks (kTraceBlock = 128 threads,
    // one ray), k_extend_scan (256 threads, 2 rays), k_shadow_scan (256, 1)
    struct Shape {
        uint32_t B, K;
        const char *name;
    } shapes[] = {{128, 1, "k_extend/k_shadow"}, {256, 2, "k_extend_scan"}, {256, 1, "k_shadow_scan"}};
    unsigned seed = 12345u;
    auto rnd = [&](uint32_t m) {
        seed = seed * 1103515245u + 12345u;
        return (seed >> 8) % m;
    };
    long cases = 0;
    for (uint32_t G = 1; G <= 67; ++G) {
        for (int pat = 0; pat < 8; ++pat) {
            std::vector<uint32_t> cnt(G);
            for (uint32_t s = 0; s < G; ++s) {
                switch (pat) {
                case 0: cnt[s] = 0; break;                               // all empty
                case 1: cnt[s] = kSeg; break;                            // all full
                case 2: cnt[s] = rnd(kSeg + 1); break;                   // random
                case 3: cnt[s] = s + 1 == G ? rnd(kSeg) + 1 : 0; break;  // only the last
                case 4: cnt[s] = s % 2 ? kSeg : 0; break;                // alternating
                case 5: cnt[s] = s == 0 ? 1 : 0; break;                  // one entry
                case 6: cnt[s] = (s % kTraceGroup == kTraceGroup - 1) ? 0 : rnd(3) * 128; break;  // slice edges
                default: cnt[s] = s + 1 == G ? 0 : kSeg - rnd(2); break;  // full but an empty last
                }
            }
            for (const Shape &sh : shapes) {
                const uint32_t per = kTraceGroup * kSeg / (sh.B * sh.K);
                run(cnt, per, sh.B, sh.K, sh.name);
                ++cases;
            }
        }
    }
    std::printf("seg_index: %ld launches checked, %d failures\n", cases, fails);
    return fails ? 1 : 0;
}
