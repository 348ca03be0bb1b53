// compute() of a whole MetricCollection in ONE launch.
//
// Per compute() a 20-metric classification + regression collection runs ~16 one-block reduction kernels (stat-score
// family, confusion-matrix family, binned AUROC / AP, streaming regression ratios).  Each is a few microseconds of
// work but costs a full launch / graph-node dispatch.  Here the Python side records the members' reductions as task
// descriptors (torchmetrics_amd.ops.fused_compute) and this kernel runs them all: block b looks up its task by the
// descriptor's block prefix and executes the same block body (common/compute_bodies.h) the standalone kernel runs.
// Descriptors travel by value in the kernel arguments (no device table to keep alive; capturable into a HIP graph).
#include "common/compute_bodies.h"

#include <atomic>
#include <chrono>
#include <mutex>
#include <vector>

namespace tm_amd {
namespace {

constexpr int kMaxTasks = 32;

enum TaskType : int {
  kTaskStat = 0,
  kTaskConfmat = 1,
  kTaskCurve = 2,
  kTaskRegF32 = 3,
  kTaskRegF64 = 4,
  kTaskRatioF32 = 5,
  kTaskRatioF64 = 6,
  kTaskStatScores = 7
};

struct Task {
  int type;
  int blocks;
  int i[6];
  double f[2];
  const void* p[8];
};

struct TaskTable {
  int n;
  int first[kMaxTasks + 1];
  Task t[kMaxTasks];
};

__global__ void __launch_bounds__(cbody::kThreads) compute_tasks_kernel(TaskTable tab) {
  extern __shared__ double dyn[];
  __shared__ double red[cbody::kThreads / kWave];
  const int b = blockIdx.x;
  // the block's task: every lane loads one block prefix (one round trip), a ballot counts the tasks starting at or
  // before this block.  (A serial scan of the prefixes was up to n dependent kernel-argument loads, ~0.3-1 us each
  // from a kernel-argument buffer the host has just written: 1.7-12 us per launch in config #5's traces.)
  const int lane = threadIdx.x & (kWave - 1);
  const bool starts = lane < tab.n && tab.first[lane] <= b;
  const int ti = __builtin_amdgcn_readfirstlane(__popcll(__ballot(starts)) - 1);
  const Task& t = tab.t[ti];
  const int local = b - tab.first[ti];
  switch (t.type) {
    case kTaskStat:
      cbody::stat_reduce_row(static_cast<const int64_t*>(t.p[0]), static_cast<const int64_t*>(t.p[1]),
                             static_cast<const int64_t*>(t.p[2]), static_cast<const int64_t*>(t.p[3]), t.i[0], t.i[1],
                             t.i[2], t.i[3] != 0, static_cast<float>(t.f[0]),
                             static_cast<float*>(const_cast<void*>(t.p[4])), local, red);
      break;
    case kTaskConfmat:
      cbody::confmat_reduce_block(static_cast<const int64_t*>(t.p[0]), t.i[0], t.i[1], t.i[2], t.i[3], t.i[4],
                                  static_cast<float*>(const_cast<void*>(t.p[1])), dyn, red);
      break;
    case kTaskCurve:
      cbody::curve_score_block(static_cast<const int64_t*>(t.p[0]), t.i[0], t.i[1], t.i[2], t.i[3],
                               static_cast<float*>(const_cast<void*>(t.p[1])),
                               static_cast<int*>(const_cast<void*>(t.p[2])), reinterpret_cast<float*>(dyn));
      break;
    case kTaskRegF32:
      cbody::regression_compute_block<float>(
          t.i[0], t.i[1], static_cast<const float*>(t.p[0]), static_cast<const float*>(t.p[1]),
          static_cast<const float*>(t.p[2]), static_cast<const float*>(t.p[3]), static_cast<const float*>(t.p[4]),
          t.p[5], t.i[2], t.i[3], t.f[0], t.i[4], static_cast<float>(t.f[1]),
          static_cast<float*>(const_cast<void*>(t.p[6])), reinterpret_cast<float*>(red));
      break;
    case kTaskRatioF32:
      cbody::ratio_block<float>(static_cast<const float*>(t.p[0]), t.p[1], t.i[1], t.i[2], t.i[0], t.i[3],
                                static_cast<float*>(const_cast<void*>(t.p[2])));
      break;
    case kTaskRatioF64:
      cbody::ratio_block<double>(static_cast<const double*>(t.p[0]), t.p[1], t.i[1], t.i[2], t.i[0], t.i[3],
                                 static_cast<double*>(const_cast<void*>(t.p[2])));
      break;
    case kTaskStatScores:
      cbody::stat_scores_block(static_cast<const int64_t*>(t.p[0]), static_cast<const int64_t*>(t.p[1]),
                               static_cast<const int64_t*>(t.p[2]), static_cast<const int64_t*>(t.p[3]), t.i[0],
                               t.i[1], const_cast<void*>(t.p[4]), red);
      break;
    default:
      cbody::regression_compute_block<double>(
          t.i[0], t.i[1], static_cast<const double*>(t.p[0]), static_cast<const double*>(t.p[1]),
          static_cast<const double*>(t.p[2]), static_cast<const double*>(t.p[3]), static_cast<const double*>(t.p[4]),
          t.p[5], t.i[2], t.i[3], t.f[0], t.i[4], t.f[1], static_cast<double*>(const_cast<void*>(t.p[6])), red);
      break;
  }
}

// ---------------------------------------------------------------------------------------- status-word gather
// Collects the members' validation words and device-side warning flags (int32 / int64 / f32 / f64 / u8 scalars)
// into an int32 vector in pinned host memory, written straight from the kernel: after the stream synchronises, the
// host reads every word with no copy operation.  Float flags map to 1 when non-zero (NaN included).
constexpr int kMaxWords = 128;

struct WordTable {
  int n;
  int code[kMaxWords];
  const void* p[kMaxWords];
};

__global__ void __launch_bounds__(kMaxWords) gather_words_kernel(WordTable tab, int* __restrict__ dst) {
  const int i = threadIdx.x;
  if (i < tab.n) {
    int v = 0;
    switch (tab.code[i]) {
      case 0: v = *static_cast<const int*>(tab.p[i]); break;
      case 1: v = *static_cast<const float*>(tab.p[i]) != 0.f ? 1 : 0; break;
      case 2: v = *static_cast<const double*>(tab.p[i]) != 0.0 ? 1 : 0; break;
      case 3: v = *static_cast<const int64_t*>(tab.p[i]) != 0 ? 1 : 0; break;
      default: v = *static_cast<const uint8_t*>(tab.p[i]) != 0 ? 1 : 0; break;
    }
    dst[i] = v;
  }
  __threadfence_system();
}

// read_words: the gather above, then a sequence number stored after every word is visible to the host (each storing
// lane's system-scope fence, the block barrier, then lane 0's store)
__global__ void __launch_bounds__(kMaxWords) gather_words_seq_kernel(WordTable tab, int* __restrict__ dst,
                                                                      int* __restrict__ seq, int seq_val) {
  const int i = threadIdx.x;
  if (i < tab.n) {
    int v = 0;
    switch (tab.code[i]) {
      case 0: v = *static_cast<const int*>(tab.p[i]); break;
      case 1: v = *static_cast<const float*>(tab.p[i]) != 0.f ? 1 : 0; break;
      case 2: v = *static_cast<const double*>(tab.p[i]) != 0.0 ? 1 : 0; break;
      case 3: v = *static_cast<const int64_t*>(tab.p[i]) != 0 ? 1 : 0; break;
      default: v = *static_cast<const uint8_t*>(tab.p[i]) != 0 ? 1 : 0; break;
    }
    dst[i] = v;
  }
  __threadfence_system();
  __syncthreads();
  if (i == 0) *reinterpret_cast<volatile int*>(seq) = seq_val;
  __threadfence_system();
}

// one word of device memory copied into mapped host memory (vector store by lane 0) -- read_word_sync
__global__ void __launch_bounds__(64) publish_word_kernel(const int* __restrict__ src, int* __restrict__ dst) {
  if (threadIdx.x == 0) dst[0] = src[0];
  __threadfence_system();
}

}  // namespace

// The value of an int32 device word, read without a device->host copy: one 1-thread kernel stores it into mapped
// (fine-grained, coherent) pinned host memory, the CURRENT STREAM is synchronised, the host reads the word.  Against
// `.item()` (a blit + wait) this leaves the stream known-idle to the runtime, so a following
// hipDeviceSynchronize / torch.cuda.synchronize() returns at once instead of issuing its own marker round trip
// (profiles/r05_region_tail.jsonl: 0.2 us vs 14 us after the read).  The caller (metric.py _raise_device_errors)
// releases nothing it holds; the GIL is released by the fastcall wrapper around this call.
int64_t read_word_sync(const at::Tensor& word) {
  TM_CHECK_CUDA(word);
  TORCH_CHECK(word.scalar_type() == at::kInt && word.numel() >= 1, "read_word_sync: an int32 word");
  const int dev = word.get_device();
  TORCH_CHECK(dev >= 0 && dev < 64, "read_word_sync: device index");
  static std::mutex mu;
  static int* host[64] = {};
  static int* mapped[64] = {};
  std::lock_guard<std::mutex> lock(mu);  // one slot per device: serialise readers of one device
  const c10::DeviceGuard guard(word.device());
  if (host[dev] == nullptr) {
    int* h = nullptr;
    TORCH_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h), 64, hipHostMallocMapped | hipHostMallocCoherent) ==
                    hipSuccess, "read_word_sync: pinned allocation failed");
    void* d = nullptr;
    TORCH_CHECK(hipHostGetDevicePointer(&d, h, 0) == hipSuccess, "read_word_sync: unmapped pinned memory");
    host[dev] = h;
    mapped[dev] = static_cast<int*>(d);
  }
  hipStream_t s = stream();
  hipLaunchKernelGGL(publish_word_kernel, dim3(1), dim3(64), 0, s, word.data_ptr<int>(), mapped[dev]);
  C10_HIP_KERNEL_LAUNCH_CHECK();
  TORCH_CHECK(hipStreamSynchronize(s) == hipSuccess, "read_word_sync: stream synchronisation failed");
  return static_cast<int64_t>(*static_cast<volatile int*>(host[dev]));
}

// words: CPU int64 [n, 2] rows (device pointer, code: 0 i32 raw / 1 f32 / 2 f64 / 3 i64 / 4 u8|bool as 0-1);
// dst: device-side address of a pinned int32 [>= n] buffer (mapped_device_ptr); anchor: a tensor on the device.
// Capturable: no allocation and no runtime query happens here.
void gather_words(const at::Tensor& words, int64_t dst, const at::Tensor& anchor) {
  TM_CHECK_CUDA(anchor);
  TORCH_CHECK(!words.is_cuda() && words.scalar_type() == at::kLong && words.dim() == 2 && words.size(1) == 2,
              "gather_words: words must be a CPU int64 [n, 2] table");
  const int n = static_cast<int>(words.size(0));
  TORCH_CHECK(n >= 1 && n <= kMaxWords, "gather_words: 1..", kMaxWords, " words");
  TORCH_CHECK(dst != 0, "gather_words: null destination");
  const at::Tensor w = words.contiguous();
  const int64_t* r = w.data_ptr<int64_t>();
  WordTable tab{};
  tab.n = n;
  for (int k = 0; k < n; ++k) {
    tab.p[k] = reinterpret_cast<const void*>(r[2 * k]);
    tab.code[k] = static_cast<int>(r[2 * k + 1]);
    TORCH_CHECK(tab.p[k] != nullptr && tab.code[k] >= 0 && tab.code[k] <= 4, "gather_words: bad word ", k);
  }
  hipLaunchKernelGGL(gather_words_kernel, dim3(1), dim3(kMaxWords), 0, stream(), tab, reinterpret_cast<int*>(dst));
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

// Every status word of a collection compute() in ONE native call: the gather kernel stores the words and then a
// sequence number into mapped pinned host memory; the host spins on the sequence number (the kernel is the last
// work of the stream, typically landing within a few us) instead of a hipStreamSynchronize round trip, and falls
// back to that sync after `spin_us` (a busy queue ahead of it).  words: CPU int64 [n, 2] (pointer, code) rows as for
// gather_words; anchor: a tensor on the device (device + current stream).  The caller releases the GIL.
std::vector<int64_t> read_words(const at::Tensor& words, const at::Tensor& anchor, int64_t spin_us) {
  TM_CHECK_CUDA(anchor);
  TORCH_CHECK(!words.is_cuda() && words.scalar_type() == at::kLong && words.dim() == 2 && words.size(1) == 2,
              "read_words: words must be a CPU int64 [n, 2] table");
  const int n = static_cast<int>(words.size(0));
  TORCH_CHECK(n >= 1 && n <= kMaxWords, "read_words: 1..", kMaxWords, " words");
  const int dev = anchor.get_device();
  TORCH_CHECK(dev >= 0 && dev < 64, "read_words: device index");
  static std::mutex mu;
  static int* host[64] = {};
  static int* mapped[64] = {};
  static int counter[64] = {};
  std::lock_guard<std::mutex> lock(mu);  // one buffer per device: serialise readers of one device
  if (host[dev] == nullptr) {
    int* h = nullptr;
    TORCH_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h), (kMaxWords + 64) * sizeof(int),
                              hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess,
                "read_words: pinned allocation failed");
    void* d = nullptr;
    TORCH_CHECK(hipHostGetDevicePointer(&d, h, 0) == hipSuccess, "read_words: unmapped pinned memory");
    host[dev] = h;
    mapped[dev] = static_cast<int*>(d);
    h[kMaxWords] = 0;
  }
  const at::Tensor w = words.contiguous();
  const int64_t* r = w.data_ptr<int64_t>();
  WordTable tab{};
  tab.n = n;
  for (int k = 0; k < n; ++k) {
    tab.p[k] = reinterpret_cast<const void*>(r[2 * k]);
    tab.code[k] = static_cast<int>(r[2 * k + 1]);
    TORCH_CHECK(tab.p[k] != nullptr && tab.code[k] >= 0 && tab.code[k] <= 4, "read_words: bad word ", k);
  }
  int seq_val = counter[dev] = (counter[dev] % 0x3fffffff) + 1;
  volatile int* seq = host[dev] + kMaxWords;
  hipStream_t s = stream();
  hipLaunchKernelGGL(gather_words_seq_kernel, dim3(1), dim3(kMaxWords), 0, s, tab, mapped[dev], mapped[dev] + kMaxWords,
                     seq_val);
  C10_HIP_KERNEL_LAUNCH_CHECK();
  const auto t0 = std::chrono::steady_clock::now();
  bool seen = false;
  while (true) {
    if (*seq == seq_val) {
      seen = true;
      break;
    }
    if (std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count() >
        spin_us)
      break;
  }
  if (!seen) TORCH_CHECK(hipStreamSynchronize(s) == hipSuccess, "read_words: stream synchronisation failed");
  std::atomic_thread_fence(std::memory_order_acquire);
  std::vector<int64_t> out(n);
  for (int k = 0; k < n; ++k) out[k] = static_cast<volatile int*>(host[dev])[k];
  return out;
}

// device-side address of pinned host memory (kernels write it directly)
int64_t mapped_device_ptr(const at::Tensor& pinned) {
  TORCH_CHECK(!pinned.is_cuda() && pinned.is_pinned(), "mapped_device_ptr: expected a pinned CPU tensor");
  void* dptr = nullptr;
  TORCH_CHECK(hipHostGetDevicePointer(&dptr, pinned.data_ptr(), 0) == hipSuccess,
              "mapped_device_ptr: memory is not mapped");
  return reinterpret_cast<int64_t>(dptr);
}

// desc: CPU int64 [n, 18] rows: type, blocks, i0..i5, bits(f0), bits(f1), p0..p7 (see ops.fused_compute);
// anchor: any tensor on the target device (selects device and stream); lds_bytes: dynamic LDS of the largest task.
void compute_tasks(const at::Tensor& desc, const at::Tensor& anchor, int64_t lds_bytes) {
  TM_CHECK_CUDA(anchor);
  TORCH_CHECK(!desc.is_cuda() && desc.scalar_type() == at::kLong && desc.dim() == 2 && desc.size(1) == 18,
              "compute_tasks: desc must be a CPU int64 [n, 18] table");
  const int n = static_cast<int>(desc.size(0));
  TORCH_CHECK(n >= 1 && n <= kMaxTasks, "compute_tasks: 1..", kMaxTasks, " tasks per launch");
  TORCH_CHECK(lds_bytes >= 0 && lds_bytes <= 160 * 1024, "compute_tasks: dynamic LDS exceeds 160 KiB");
  const at::Tensor d = desc.contiguous();
  const int64_t* r = d.data_ptr<int64_t>();
  TaskTable tab{};
  tab.n = n;
  int total = 0;
  for (int k = 0; k < n; ++k, r += 18) {
    Task& t = tab.t[k];
    t.type = static_cast<int>(r[0]);
    t.blocks = static_cast<int>(r[1]);
    TORCH_CHECK(t.type >= kTaskStat && t.type <= kTaskStatScores && t.blocks >= 1, "compute_tasks: bad task ", k);
    for (int j = 0; j < 6; ++j) t.i[j] = static_cast<int>(r[2 + j]);
    std::memcpy(&t.f[0], &r[8], sizeof(double));
    std::memcpy(&t.f[1], &r[9], sizeof(double));
    for (int j = 0; j < 8; ++j) t.p[j] = reinterpret_cast<const void*>(r[10 + j]);
    tab.first[k] = total;
    total += t.blocks;
  }
  tab.first[n] = total;
  hipLaunchKernelGGL(compute_tasks_kernel, dim3(total), dim3(cbody::kThreads), static_cast<size_t>(lds_bytes),
                     stream(), tab);
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

int64_t compute_tasks_max() { return kMaxTasks; }

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  m.def("compute_tasks(Tensor desc, Tensor anchor, int lds_bytes) -> ()");
  m.def("compute_tasks_max() -> int", &compute_tasks_max);
  m.def("gather_words(Tensor words, int dst, Tensor anchor) -> ()");
  m.def("mapped_device_ptr(Tensor pinned) -> int", &mapped_device_ptr);
  m.def("read_word_sync(Tensor word) -> int");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) {
  m.impl("compute_tasks", &compute_tasks);
  m.impl("gather_words", &gather_words);
  m.impl("read_word_sync", &read_word_sync);
}

}  // namespace tm_amd
