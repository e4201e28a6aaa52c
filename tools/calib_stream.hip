// calib_stream.hip -- profiling aid (not product code): streams a known byte count with the access
// widths the replay kernels use, so rocprofv3 FETCH_SIZE / WRITE_SIZE can be converted to bytes
// (MI355X_MICROARCH.md, "HBM": only 16-B/lane streams are calibrated; every other width must be
// calibrated on a known byte count in the kernel's own pattern).
//
// Pattern = the replay kernels' column loads: lane l of a wavefront reads element (base + l), the
// wavefront walks consecutive 64-element runs (wave-interleaved layout, one run per step).
#include <hip/hip_runtime.h>

#include <cstdint>

template <typename T>
__global__ void __launch_bounds__(256) calib_read(const T* __restrict__ p, uint64_t n, uint64_t* __restrict__ out, uint64_t magic) {
  uint64_t acc = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) acc ^= (uint64_t)p[i];
  // a store that never happens for these inputs (magic is a runtime value the compiler cannot see
  // through) keeps the loads live without write traffic
  if (acc == magic) out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// one u64 per `stride_words`-word row (a field gathered from AoS rows, e.g. an activity row's ScheduleID:
// 112-byte rows, stride 14): lane l reads row (base + l), as the checksum's per-lane row gathers do
__global__ void __launch_bounds__(256) calib_gather(const uint64_t* __restrict__ p, uint64_t rows, uint32_t stride_words,
                                                    uint64_t* __restrict__ out, uint64_t magic) {
  uint64_t acc = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows; i += stride) acc ^= p[i * stride_words];
  if (acc == magic) out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <typename T>
__global__ void __launch_bounds__(256) calib_write(T* __restrict__ p, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = (T)i;
}

extern "C" {

// kind: 1, 4, 8 = read u8 / u32 / u64 per lane; 108 = write u64 per lane; 1000 + w = gather one u64 per
// w-word row (1014: 112-byte rows, 1026: 208-byte rows, 1002: 16-byte rows)
int calib_stream(int kind, void* buf, uint64_t bytes, void* scratch, void* stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid(4096), block(256);
  uint64_t* out = reinterpret_cast<uint64_t*>(scratch);
  switch (kind) {
    case 1: hipLaunchKernelGGL(calib_read<uint8_t>, grid, block, 0, s, (const uint8_t*)buf, bytes, out, 0x5a5a5a5a5a5a5a5aull ^ (uint64_t)kind); break;
    case 4: hipLaunchKernelGGL(calib_read<uint32_t>, grid, block, 0, s, (const uint32_t*)buf, bytes / 4, out, 0x5a5a5a5a5a5a5a5aull ^ (uint64_t)kind); break;
    case 8: hipLaunchKernelGGL(calib_read<uint64_t>, grid, block, 0, s, (const uint64_t*)buf, bytes / 8, out, 0x5a5a5a5a5a5a5a5aull ^ (uint64_t)kind); break;
    case 108: hipLaunchKernelGGL(calib_write<uint64_t>, grid, block, 0, s, (uint64_t*)buf, bytes / 8); break;
    default:
      if (kind > 1000 && kind < 1100) {
        const uint32_t w = (uint32_t)(kind - 1000);
        hipLaunchKernelGGL(calib_gather, grid, block, 0, s, (const uint64_t*)buf, bytes / (8ull * w), w, out,
                           0x5a5a5a5a5a5a5a5aull ^ (uint64_t)kind);
        break;
      }
      return -1;
  }
  return (int)hipGetLastError();
}

}  // extern "C"
