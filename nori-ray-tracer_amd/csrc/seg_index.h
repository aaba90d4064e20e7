// seg_index.h -- how the trace launches number the entries of the segmented
// queues (dev_scene.h): plain integer arithmetic, host-compilable, so that
// tests/test_seg_index.py can check with g++ that every entry a launch's
// threads address lies inside the queue (an index past G * kSeg is an
// illegal access on the GPU; round 5's persistent scans faulted that way).
//
// Trace work-groups are dealt out over groups of kTraceGroup consecutive
// segments: the entries of a group are numbered through a prefix over its
// segment counts, and work-group j of the group takes the next B * K of them
// (B threads, K rays per thread, the k-th ray of thread t is entry
// j B K + t + k B).  Partly filled segments (a segment's shadow queue is about
// half full; the drain phase empties them) therefore do not leave waves
// partly idle.
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define NORI_SEG_FN __host__ __device__ __forceinline__
#else
#define NORI_SEG_FN inline
#endif

namespace nori {

constexpr uint32_t kSeg = 256;  // queue entries per segment (= shade work-group size)
#ifndef NORI_TRACE_GROUP
#define NORI_TRACE_GROUP 4
#endif
constexpr int kTraceGroup = NORI_TRACE_GROUP;  // segments per group of trace work-groups

struct SegRange {
    uint32_t pre[kTraceGroup + 1];  // prefix of the group's segment counts
    uint32_t s0;                    // first segment of the group
};
// Work-groups of a trace launch over G segments, `per` work-groups per group.
NORI_SEG_FN uint32_t seg_grid(uint32_t G, uint32_t per) { return (G + kTraceGroup - 1) / kTraceGroup * per; }
// The group of work-group `bid` (segments past G count as empty).
NORI_SEG_FN SegRange seg_group(const uint32_t *cnt, uint32_t G, uint32_t bid, uint32_t per) {
    SegRange r;
    r.s0 = (bid / per) * kTraceGroup;
    r.pre[0] = 0;
#pragma unroll
    for (int k = 0; k < kTraceGroup; ++k) r.pre[k + 1] = r.pre[k] + (r.s0 + k < G ? cnt[r.s0 + k] : 0u);
    return r;
}
// The group's entry number i of thread t's first ray in work-group `bid`
// (B threads, K rays per thread); ray k is entry seg_first + k B.  A thread
// with seg_first >= pre[kTraceGroup] has no ray (the work-group's slice of
// the group is past its last entry); the kernels return before any load.
NORI_SEG_FN uint32_t seg_first(uint32_t bid, uint32_t per, uint32_t B, uint32_t K, uint32_t t) {
    return (bid % per) * B * K + t;
}
// Queue index of the group's entry i < pre[kTraceGroup]: segment s0 + k with
// pre[k] <= i < pre[k + 1], slot i - pre[k].
NORI_SEG_FN uint32_t seg_entry(const SegRange &r, uint32_t i) {
    uint32_t k = 0;
#pragma unroll
    for (int j = 1; j < kTraceGroup; ++j) k += i >= r.pre[j] ? 1u : 0u;
    uint32_t base = r.pre[0];
#pragma unroll
    for (int j = 1; j < kTraceGroup; ++j) base = k == (uint32_t)j ? r.pre[j] : base;
    return (r.s0 + k) * kSeg + (i - base);
}

}  // namespace nori
