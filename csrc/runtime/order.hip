// The stream-order guard: ONE communicator's collectives run in the order they were issued, on
// every rank, whatever streams the caller issued them on.
//
// Why: every cross-rank protocol of the IPC kernels assumes that one instance's kernels execute
// one after the other on each rank — the double-buffered slots of the latency tier (a slot is
// rewritten two calls later, ipc_ar.hip), the "one call ahead" start-barrier rule, the epoch
// flags (ipc_common.hpp block_barrier).  Two calls issued back to back from two streams could
// otherwise run concurrently on one rank and overwrite each other's flags or slots.  The
// reference gets the same total order from its one send queue and one receive queue per process
// (/root/reference/src/main/java/com/fenbi/mp4j/comm/ProcessCommSlave.java:84-127) and the barrier
// that ends every collective (:1367); RCCL from its per-communicator stream.
//
// How: the guard remembers the stream of the communicator's previous launch.  A launch on the
// SAME stream costs one pointer compare (the steady state: the latency fast path stays a single
// native call).  A launch on ANOTHER stream first records an event on the previous stream and
// makes the new stream wait for it — the event captures everything queued there so far, the
// previous collective included.  No cycle can form: the old stream's tail only waits for work
// that was queued before this call.
//
// Contract (DESIGN.md §"Stream order"): a stream handed to a collective should stay alive until
// the communicator's next collective was issued (torch's pooled streams always do); if it was
// destroyed, the event cannot be recorded there and the join falls back to a device-wide
// synchronisation (ROCclr validates stream handles and returns an error).  Graph capture:
// the captured launches of one capture must all be on one stream (a switch inside a capture is
// refused: MP4X_E_STREAM_SWITCH; callers that cannot rule a capture out pass capturing = -1 and
// the status is queried); a capture does not move the eager order, and replays are ordered by the
// stream they are launched on, like any graph.
#include "ipc_common.hpp"

using namespace mp4x;

// `capturing`: 0 = the caller knows the stream is not being captured (the fast paths checked it),
// 1 = it is, -1 = unknown (queried here).  The steady state (same stream as the previous launch,
// not capturing) is one compare.
extern "C" int mp4x_order_enter_ex(StreamOrder* o, void* stream, int capturing) {
  if (!o) return 0;
  if (capturing == 0 && o->have_last && o->last == stream) return 0;      // the steady state
  hipStream_t s = (hipStream_t)stream;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  if (hipError_t e = hipStreamGetCaptureInfo(s, &cs, &id)) {
    (void)hipGetLastError();
    return (int)e;
  }
  if (cs != hipStreamCaptureStatusActive && o->have_last && o->last == stream) return 0;
  if (cs == hipStreamCaptureStatusActive) {
    if (o->cap_have && o->cap_id == id && o->cap_stream != stream) return MP4X_E_STREAM_SWITCH;
    o->cap_have = 1;
    o->cap_id = id;
    o->cap_stream = stream;
    return 0;
  }
  if (o->have_last && !o->disabled) {
    if (!o->ev) {
      hipEvent_t ev = nullptr;
      if (hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) {
        (void)hipGetLastError();
        return (int)e;
      }
      o->ev = ev;
    }
    if (hipEventRecord((hipEvent_t)o->ev, (hipStream_t)o->last) != hipSuccess) {
      // the previous stream is gone (destroyed by its owner since the last collective): order the
      // new launch after everything queued on the device instead — slow, but never unordered
      (void)hipGetLastError();
      if (hipError_t e = hipDeviceSynchronize()) {
        (void)hipGetLastError();
        return (int)e;
      }
    } else if (hipError_t e = hipStreamWaitEvent(s, (hipEvent_t)o->ev, 0)) {
      (void)hipGetLastError();
      return (int)e;
    }
    ++o->switches;
  }
  o->last = stream;
  o->have_last = 1;
  return 0;
}

extern "C" int mp4x_order_enter(StreamOrder* o, void* stream) { return mp4x_order_enter_ex(o, stream, 0); }

// Release the guard's event (the communicator is closing; its streams were drained).
extern "C" int mp4x_order_release(StreamOrder* o) {
  if (!o || !o->ev) return 0;
  hipError_t e = hipEventDestroy((hipEvent_t)o->ev);
  o->ev = nullptr;
  o->have_last = 0;
  if (e) (void)hipGetLastError();
  return (int)e;
}
