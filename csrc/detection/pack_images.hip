// One-launch packing of per-image detection tensors into flat state buffers (MeanAveragePrecision.update).
//
// The reference appends 9 tensors per image to Python lists (S/detection/mean_ap.py:470-511) and converts the boxes
// image by image; a torch formulation still costs one `cat` launch per state plus the box conversion.  Here the host
// packer (csrc/bindings/fastcall.cpp map_pack) validates the batch and lays out one segment per (image, state), and
// this kernel runs every segment -- plain copies, zero fills for missing `iscrowd` / `area`, and the xyxy -> xywh box
// conversion fused into the copy -- one block per segment, up to kPackSegs segments per launch.
#include <c10/core/DeviceGuard.h>

#include "../common/pack.h"
#include "../common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kPackSegs = 128;
constexpr int kPackThreads = 128;

struct PackTable {
  PackSeg s[kPackSegs];
};

template <typename T>
__device__ __forceinline__ void box_rows(const T* __restrict__ src, T* __restrict__ dst, int rows) {
  for (int r = threadIdx.x; r < rows; r += kPackThreads) {
    const T x1 = src[4 * r], y1 = src[4 * r + 1], x2 = src[4 * r + 2], y2 = src[4 * r + 3];
    dst[4 * r] = x1;
    dst[4 * r + 1] = y1;
    dst[4 * r + 2] = x2 - x1;
    dst[4 * r + 3] = y2 - y1;
  }
}

__global__ void __launch_bounds__(kPackThreads) pack_segments_kernel(PackTable tab) {
  const PackSeg sg = tab.s[blockIdx.x];
  if (sg.mode == kPackXyxyToXywh) {
    if (sg.esize == 4) box_rows(static_cast<const float*>(sg.src), static_cast<float*>(sg.dst), sg.n);
    else box_rows(static_cast<const double*>(sg.src), static_cast<double*>(sg.dst), sg.n);
    return;
  }
  const long long bytes = static_cast<long long>(sg.n) * sg.esize;
  unsigned char* d = static_cast<unsigned char*>(sg.dst);
  const bool words = (reinterpret_cast<uintptr_t>(sg.dst) % 4 == 0) && (bytes % 4 == 0) &&
                     (sg.mode == kPackZero || reinterpret_cast<uintptr_t>(sg.src) % 4 == 0);
  if (words) {
    uint32_t* dw = reinterpret_cast<uint32_t*>(d);
    const uint32_t* sw = static_cast<const uint32_t*>(sg.src);
    for (long long i = threadIdx.x; i < bytes / 4; i += kPackThreads) dw[i] = sg.mode == kPackZero ? 0u : sw[i];
  } else {
    const unsigned char* s = static_cast<const unsigned char*>(sg.src);
    for (long long i = threadIdx.x; i < bytes; i += kPackThreads) d[i] = sg.mode == kPackZero ? 0 : s[i];
  }
}

}  // namespace

void pack_segments(const PackSeg* segs, int n, int device) {
  if (n <= 0) return;
  c10::DeviceGuard guard(c10::Device(c10::kCUDA, static_cast<c10::DeviceIndex>(device)));
  auto s = stream();
  for (int i = 0; i < n; i += kPackSegs) {
    PackTable tab;
    const int k = std::min(kPackSegs, n - i);
    for (int j = 0; j < k; ++j) tab.s[j] = segs[i + j];
    hipLaunchKernelGGL(pack_segments_kernel, dim3(k), dim3(kPackThreads), 0, s, tab);
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

}  // namespace tm_amd
