// Cross-stream hand-off: the consumer stream waits for everything the producer stream has
// enqueued so far.
//
// Default (PDT_STREAM_SYNC unset / "event"): hipEventRecord on the producer + hipStreamWaitEvent on
// the consumer.  PDT_STREAM_SYNC=value: HIP stream memory operations instead -- the producer
// writes a monotonically increasing 64-bit ticket into signal memory (hipStreamWriteValue64) and
// the consumer waits for it (hipStreamWaitValue64, >=).  VERDICT r3 item 3: with a high-priority
// compute stream, a handful of event hand-offs per step to the normal-priority comm stream made
// every small compute kernel ~35 us longer (profiles/r3z_priority_vs_sync.md); scripts/prio_repro.hip
// measures both primitives in isolation.  A stream that is being captured into a HIP graph always
// takes the event path.
#pragma once
#include <hip/hip_runtime.h>

namespace pdt {

bool stream_sync_value();  // PDT_STREAM_SYNC=value
// consumer waits for producer's enqueued work; `ev` is the event used by the event path
void stream_handoff(hipStream_t producer, hipStream_t consumer, hipEvent_t ev);

}  // namespace pdt
