// stream_device.h -- internal to libcadence_replay.so (not part of the C ABI).
//
// Every entry point of include/cadence_replay.h / cadence_ingest.h that takes a stream runs on that
// stream's device whatever device the calling thread has selected: a cgo goroutine may migrate to an
// OS thread that never called crr_set_device.  The thread's selection is restored on return.  A NULL
// stream means the calling thread's current device and its null stream.
#ifndef CADENCE_STREAM_DEVICE_H_
#define CADENCE_STREAM_DEVICE_H_

#include <hip/hip_runtime.h>

namespace crr_internal {

struct StreamDevice {
  int prev = -1;
  bool ok = true;
  explicit StreamDevice(hipStream_t s) {
    if (!s) return;
    int cur = 0, dev = 0;
    if (hipGetDevice(&cur) != hipSuccess || hipStreamGetDevice(s, &dev) != hipSuccess) { ok = false; return; }
    if (dev != cur) {
      if (hipSetDevice(dev) != hipSuccess) { ok = false; return; }
      prev = cur;
    }
  }
  ~StreamDevice() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  StreamDevice(const StreamDevice&) = delete;
  StreamDevice& operator=(const StreamDevice&) = delete;
};

}  // namespace crr_internal

#endif  // CADENCE_STREAM_DEVICE_H_
