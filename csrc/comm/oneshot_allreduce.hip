// One-shot intra-node all-reduce over xGMI peer reads, for the tiny metric-state buckets.
//
// Why: a classification / regression collection syncs a few hundred bytes to a few KiB per compute() (tp/fp/tn/fn of
// 20 metrics, regression moments).  A ring all-reduce over W ranks is 2(W-1) latency-bound steps; on MI355X every
// GPU has a direct xGMI link to every other GPU of the node, so one step suffices: each rank publishes its bucket in
// a buffer the peers have mapped (hipIpcGetMemHandle / hipIpcOpenMemHandle), raises a flag in every peer's flag
// array, waits for all W flags, and reads the W buckets straight out of the peers' HBM.  Reference behaviour being
// replaced: S/utilities/distributed.py:97-147 (per-state barrier + all_gather + local reduce).
//
// Buffer layout (one uncached fine-grained allocation per rank, identical on every rank):
//   [ data parity 0 : slot ][ data parity 1 : slot ][ ready flags: 2 x kMaxBlocks x kMaxRanks u32 ]
//   [ done flags: 2 x kMaxBlocks x kMaxRanks u32 ]
// Call number `epoch` (1, 2, ...) uses parity epoch & 1.
//
// Two-phase protocol per block b (block b owns elements [b*chunk, (b+1)*chunk) on every rank):
//   1. publish the chunk in this rank's buffer; store `epoch` into ready[parity][b][rank] of EVERY rank (xGMI store);
//      wait until ready[parity][b][p] == epoch for all p; reduce the W copies (rank order, identical rounding);
//   2. store `epoch` into done[parity][b][rank] of every rank (this rank has finished READING the peers' copies);
//      wait until every done[parity][b][p] is `epoch` or `epoch | kAbort`.
// A phase-1 wait that runs out of time (timeout_ticks of the 100 MHz wall clock) never reduces: the block stores
// `epoch | kAbort` into every rank's done slot instead and sets status bit kTimedOut.  Every rank that got through
// phase 1 then finds that abort in its phase-2 wait and sets kPeerAborted, so a timeout is reported on EVERY rank
// (nobody is left holding a result its peers disowned) and the host raises before the values are used (reference
// semantics: collectives block and never return partial results, S/utilities/distributed.py:97-147).  The phase-2
// wait also makes the double-buffer proof local: a rank leaves call e only after every peer finished reading its
// e-parity copy, so call e+2 can never overwrite data a late peer still reads.
// Status bits are OR-ed into `status` (the communicator's word) and, when given, into `err` (the metric's deferred
// validation word, read once by compute()).
#include "common/tm_common.h"

namespace tm_amd {
namespace {

constexpr int kMaxRanks = 16;
constexpr int kMaxBlocks = 64;
constexpr int kThreads = 256;
constexpr uint32_t kAbort = 0x80000000u;
constexpr int kTimedOut = 1;     // this rank's phase-1 wait for a peer ran out of time
constexpr int kPeerAborted = 2;  // a peer timed out (or never finished phase 2): results disowned

struct PeerPtrs {
  char* p[kMaxRanks];
};

enum : int { kOpSum = 0, kOpMax = 1, kOpMin = 2 };

template <typename T>
__device__ __forceinline__ T combine(T a, T b, int op) {
  if (op == kOpSum) return a + b;
  if (op == kOpMax) return a > b ? a : b;
  return a < b ? a : b;
}

__device__ __forceinline__ uint32_t* flag_slot(char* base, long long slot_bytes, int which, int parity, int block,
                                               int src) {
  uint32_t* flags = reinterpret_cast<uint32_t*>(base + 2 * slot_bytes) + which * (2 * kMaxBlocks * kMaxRanks);
  return flags + (static_cast<long long>(parity) * kMaxBlocks + block) * kMaxRanks + src;
}

// lanes p < world poll slot (which, parity, b, p) of this rank until it holds `epoch` (or `epoch | kAbort` when
// accept_abort); returns 0 = all arrived, 1 = timeout, 2 = a peer aborted
__device__ __forceinline__ int wait_peers(char* own, long long slot_bytes, int which, int parity, int b, int world,
                                          uint32_t epoch, bool accept_abort, long long timeout_ticks) {
  __shared__ int outcome;
  if (threadIdx.x == 0) outcome = 0;
  __syncthreads();
  if (threadIdx.x < world) {
    uint32_t* f = flag_slot(own, slot_bytes, which, parity, b, threadIdx.x);
    const long long t0 = wall_clock64();
    while (true) {
      const uint32_t v = __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (v == epoch) break;
      if (accept_abort && v == (epoch | kAbort)) {
        atomicOr(&outcome, 2);
        break;
      }
      if (wall_clock64() - t0 > timeout_ticks) {
        atomicOr(&outcome, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  return outcome;
}

__device__ __forceinline__ void signal_peers(const PeerPtrs& peers, long long slot_bytes, int which, int parity, int b,
                                             int rank, int world, uint32_t value) {
  if (threadIdx.x < world) {
    __hip_atomic_store(flag_slot(peers.p[threadIdx.x], slot_bytes, which, parity, b, rank), value, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__device__ __forceinline__ void report(int* status, int* err, int bits) {
  if (threadIdx.x == 0) {
    atomicOr(status, bits);
    if (err != nullptr) atomicOr(err, kErrOneshot);
  }
}

template <typename T>
__global__ void __launch_bounds__(kThreads) oneshot_allreduce_kernel(const T* __restrict__ inp, T* __restrict__ out,
                                                                     long long n, long long chunk, PeerPtrs peers,
                                                                     int rank, int world, long long slot_bytes,
                                                                     uint32_t epoch, int op, int publish,
                                                                     long long timeout_ticks, int* __restrict__ status,
                                                                     int* __restrict__ err) {
  const int b = blockIdx.x;
  const int parity = static_cast<int>(epoch & 1u);
  const long long lo = static_cast<long long>(b) * chunk;
  const long long hi = lo + chunk < n ? lo + chunk : n;
  char* own = peers.p[rank];
  // phase 1: publish this rank's chunk in its own (peer-visible) buffer, signal, wait for every peer's chunk
  T* mine = reinterpret_cast<T*>(own + parity * slot_bytes);
  if (publish) {
    for (long long i = lo + threadIdx.x; i < hi; i += kThreads) mine[i] = inp[i];
  }
  __threadfence_system();
  __syncthreads();
  signal_peers(peers, slot_bytes, 0, parity, b, rank, world, epoch);
  if (wait_peers(own, slot_bytes, 0, parity, b, world, epoch, false, timeout_ticks) != 0) {
    // never reduce a partial set: disown the call on every rank (their phase-2 waits see the abort)
    signal_peers(peers, slot_bytes, 1, parity, b, rank, world, epoch | kAbort);
    report(status, err, kTimedOut);
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // peers' data is visible to every lane of the block
  // reduce the W copies of chunk b, always in rank order (identical rounding on every rank)
  for (long long i = lo + threadIdx.x; i < hi; i += kThreads) {
    T acc = reinterpret_cast<const T*>(peers.p[0] + parity * slot_bytes)[i];
    for (int r = 1; r < world; ++r) acc = combine(acc, reinterpret_cast<const T*>(peers.p[r] + parity * slot_bytes)[i], op);
    out[i] = acc;
  }
  // phase 2: every lane's peer reads have returned (their values were stored above) -> tell the peers, wait for theirs
  __syncthreads();
  signal_peers(peers, slot_bytes, 1, parity, b, rank, world, epoch);
  const int r2 = wait_peers(own, slot_bytes, 1, parity, b, world, epoch, true, timeout_ticks);
  if (r2 != 0) report(status, err, kPeerAborted);
}

}  // namespace

// ---------------------------------------------------------------------------------------------------- host side
int64_t ipc_buffer_alloc(int64_t nbytes, int64_t device) {
  TORCH_CHECK(nbytes > 0, "ipc_buffer_alloc: nbytes must be positive");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(c10::Device(c10::DeviceType::CUDA, static_cast<int>(device)));
  void* p = nullptr;
  // uncached fine-grained memory: the peers poll flags and read data that another GPU writes while both kernels run;
  // coarse-grained hipMalloc memory is only coherent at kernel boundaries (a peer's flag store could sit behind a
  // stale line of this GPU's L2 for the whole wait)
  TORCH_CHECK(hipExtMallocWithFlags(&p, nbytes, hipDeviceMallocUncached) == hipSuccess,
              "ipc_buffer_alloc: hipExtMallocWithFlags(hipDeviceMallocUncached) failed");
  TORCH_CHECK(hipMemset(p, 0, nbytes) == hipSuccess, "ipc_buffer_alloc: hipMemset failed");
  TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "ipc_buffer_alloc: sync failed");
  return reinterpret_cast<int64_t>(p);
}

void ipc_buffer_free(int64_t ptr, int64_t device) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(c10::Device(c10::DeviceType::CUDA, static_cast<int>(device)));
  (void)hipFree(reinterpret_cast<void*>(ptr));
}

at::Tensor ipc_get_handle(int64_t ptr, int64_t device) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(c10::Device(c10::DeviceType::CUDA, static_cast<int>(device)));
  hipIpcMemHandle_t h;
  TORCH_CHECK(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(ptr)) == hipSuccess, "ipc_get_handle failed");
  at::Tensor out = at::empty({static_cast<int64_t>(sizeof(h))}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(out.data_ptr<uint8_t>(), &h, sizeof(h));
  return out;
}

int64_t ipc_open_handle(const at::Tensor& handle, int64_t device) {
  TORCH_CHECK(!handle.is_cuda() && handle.scalar_type() == at::kByte && handle.numel() == sizeof(hipIpcMemHandle_t),
              "ipc_open_handle: expected a CPU uint8 tensor of ", sizeof(hipIpcMemHandle_t), " bytes");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(c10::Device(c10::DeviceType::CUDA, static_cast<int>(device)));
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.contiguous().data_ptr<uint8_t>(), sizeof(h));
  void* p = nullptr;
  const hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
  TORCH_CHECK(e == hipSuccess, "ipc_open_handle: hipIpcOpenMemHandle failed: ", hipGetErrorString(e));
  return reinterpret_cast<int64_t>(p);
}

void ipc_close_handle(int64_t ptr, int64_t device) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(c10::Device(c10::DeviceType::CUDA, static_cast<int>(device)));
  (void)hipIpcCloseMemHandle(reinterpret_cast<void*>(ptr));
}

// uint8 view of `nbytes` at a raw device pointer (no ownership): lets tests and tools fill / inspect the buffers
at::Tensor ipc_view(int64_t ptr, int64_t nbytes, int64_t device) {
  return at::from_blob(reinterpret_cast<void*>(ptr), {nbytes},
                       at::TensorOptions().dtype(at::kByte).device(c10::Device(c10::DeviceType::CUDA,
                                                                               static_cast<int>(device))));
}

// out = reduce_op over ranks of inp (1-D, <= slot_bytes).  peers: CPU int64 [world] of device pointers (this rank's
// own buffer at index `rank`).  publish=false skips step 1 (tests that pre-fill the buffers).
void oneshot_allreduce(const at::Tensor& inp, at::Tensor out, const at::Tensor& peers, int64_t rank, int64_t slot_bytes,
                       int64_t epoch, int64_t op, bool publish, double timeout_s, at::Tensor status,
                       const c10::optional<at::Tensor>& err) {
  TM_CHECK_CUDA(inp);
  TM_SAME_DEVICE(inp, out);
  TM_SAME_DEVICE(inp, status);
  TM_CHECK_CONTIG(inp);
  TM_CHECK_CONTIG(out);
  TORCH_CHECK(out.scalar_type() == inp.scalar_type() && out.numel() == inp.numel(), "oneshot_allreduce: bad out");
  TORCH_CHECK(status.scalar_type() == at::kInt && status.numel() >= 1, "oneshot_allreduce: bad status");
  TORCH_CHECK(!peers.is_cuda() && peers.scalar_type() == at::kLong && peers.dim() == 1, "oneshot_allreduce: peers");
  const int world = static_cast<int>(peers.numel());
  TORCH_CHECK(world >= 1 && world <= kMaxRanks, "oneshot_allreduce: world size must be in [1, ", kMaxRanks, "]");
  TORCH_CHECK(rank >= 0 && rank < world, "oneshot_allreduce: bad rank");
  TORCH_CHECK(op >= 0 && op <= 2, "oneshot_allreduce: op must be sum/max/min");
  TORCH_CHECK(epoch > 0 && epoch < (1LL << 31), "oneshot_allreduce: epoch out of range");
  TORCH_CHECK(timeout_s > 0, "oneshot_allreduce: timeout must be positive");
  int* errp = nullptr;
  if (err.has_value()) {
    TM_SAME_DEVICE(inp, *err);
    TORCH_CHECK(err->scalar_type() == at::kInt && err->numel() >= 1, "oneshot_allreduce: bad err word");
    errp = err->data_ptr<int>();
  }
  const double ticks = timeout_s * 1.0e8;  // wall_clock64: 100 MHz
  const long long timeout_ticks = ticks > 9.0e18 ? static_cast<long long>(9.0e18) : static_cast<long long>(ticks);
  const long long n = inp.numel();
  TORCH_CHECK(static_cast<long long>(n * inp.element_size()) <= slot_bytes, "oneshot_allreduce: bucket exceeds slot");
  if (n == 0) return;
  PeerPtrs pp{};
  const int64_t* pv = peers.data_ptr<int64_t>();
  for (int r = 0; r < world; ++r) {
    TORCH_CHECK(pv[r] != 0, "oneshot_allreduce: null peer pointer");
    pp.p[r] = reinterpret_cast<char*>(pv[r]);
  }
  // >= 4 KiB per block, at most kMaxBlocks blocks, chunk a multiple of 64 elements
  const long long bytes = n * inp.element_size();
  long long blocks = (bytes + 4095) / 4096;
  if (blocks > kMaxBlocks) blocks = kMaxBlocks;
  long long chunk = (n + blocks - 1) / blocks;
  chunk = (chunk + 63) / 64 * 64;
  blocks = (n + chunk - 1) / chunk;
  switch (inp.scalar_type()) {
#define TM_ONESHOT_CASE(ATYPE, CTYPE)                                                                              \
  case ATYPE:                                                                                                      \
    hipLaunchKernelGGL((oneshot_allreduce_kernel<CTYPE>), dim3(blocks), dim3(kThreads), 0, stream(),               \
                       inp.data_ptr<CTYPE>(), out.data_ptr<CTYPE>(), n, chunk, pp, static_cast<int>(rank), world,    \
                       slot_bytes, static_cast<uint32_t>(epoch), static_cast<int>(op), publish ? 1 : 0,            \
                       timeout_ticks, status.data_ptr<int>(), errp);                                               \
    break;
    TM_ONESHOT_CASE(at::kFloat, float)
    TM_ONESHOT_CASE(at::kDouble, double)
    TM_ONESHOT_CASE(at::kLong, int64_t)
    TM_ONESHOT_CASE(at::kInt, int32_t)
#undef TM_ONESHOT_CASE
    default:
      TORCH_CHECK(false, "oneshot_allreduce: unsupported dtype ", inp.scalar_type());
  }
}

int64_t oneshot_buffer_bytes(int64_t slot_bytes) {
  return 2 * slot_bytes + 2LL * 2 * kMaxBlocks * kMaxRanks * static_cast<int64_t>(sizeof(uint32_t));
}

TORCH_LIBRARY_FRAGMENT(tm_amd, m) {
  // pointer / handle management takes no device tensor: catch-all kernels
  m.def("ipc_buffer_alloc(int nbytes, int device) -> int", &ipc_buffer_alloc);
  m.def("ipc_buffer_free(int ptr, int device) -> ()", &ipc_buffer_free);
  m.def("ipc_get_handle(int ptr, int device) -> Tensor", &ipc_get_handle);
  m.def("ipc_open_handle(Tensor handle, int device) -> int", &ipc_open_handle);
  m.def("ipc_close_handle(int ptr, int device) -> ()", &ipc_close_handle);
  m.def("oneshot_buffer_bytes(int slot_bytes) -> int", &oneshot_buffer_bytes);
  m.def("ipc_view(int ptr, int nbytes, int device) -> Tensor", &ipc_view);
  m.def(
      "oneshot_allreduce(Tensor inp, Tensor(a!) out, Tensor peers, int rank, int slot_bytes, int epoch, int op, "
      "bool publish, float timeout_s, Tensor(b!) status, Tensor(c!)? err=None) -> ()");
}
TORCH_LIBRARY_IMPL(tm_amd, CUDA, m) { m.impl("oneshot_allreduce", &oneshot_allreduce); }

}  // namespace tm_amd
