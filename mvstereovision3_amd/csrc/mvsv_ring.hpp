// mvsv_ring.hpp — slot bookkeeping of the frame stream (mvsv_stream.cpp), kept
// free of HIP so the CPU suite can drive it under AddressSanitizer + UBSan.
//
// Frames are numbered by push order; frame f lives in slot f % depth.  head =
// frames pushed, tail = frames popped, launched = frames whose compute is
// enqueued (tail <= launched <= head, head - tail <= depth).  Pushed frames are
// launched as runs of consecutive slots; a run never wraps past the ring's end,
// so its slots are one contiguous [frame][H][W] block of the device arrays.
#pragma once

#include <algorithm>

namespace mvsv {

struct RingRun {
    long i0;  // first slot
    int n;    // slots
};

// The next run to launch, or false when every pushed frame is launched.
inline bool ring_next_run(long launched, long head, long depth, RingRun* r)
{
    if (launched >= head) return false;
    r->i0 = launched % depth;
    r->n = (int)std::min(head - launched, depth - r->i0);
    return true;
}

// After a push: launch when a full group of `batch` frames is pending, or when
// the group would otherwise wrap past the ring's end.
inline bool ring_launch_after_push(long head, long launched, int batch, long depth)
{
    return head - launched >= batch || head % depth == 0;
}

inline bool ring_full(long head, long tail, long depth) { return head - tail >= depth; }

}  // namespace mvsv
