// One-shot all-gather of the decode (M = 1) output shards over peer memory ("at M = 1 the all-gather
// moves KB and is latency-bound (~10-20 us on RCCL); prefer a custom hipIPC one-shot all-gather").  Not in the
// reference (it has no multi-GPU code); additive C-ABI beside the RCCL path, which stays the prefill all-gather.
//
// Each rank owns ONE exchange buffer in its own HBM, exported by hipIpcGetMemHandle and opened by every peer:
//   [0, 512)                    flags[2][64]  u32: flags[p][j] = the epoch of source rank j's last push into parity p
//   [512, 512 + 2 * g * bytes)  slots[2][g]   rank j's shard output of the step (bytes = n * sizeof(T), 16-B padded)
// allocated uncached (hipDeviceMallocUncached): a peer's stores land in the owner's memory and the owner's loads read
// memory, so no cache holds a stale copy of another GPU's bytes.  One step (k_ipc_allgather_push, one workgroup):
//   1. push: every lane stores 16-B pieces of this rank's [n] slice into slot (p, rank) of EVERY rank's buffer, then
//      waits for its own stores (vmcnt(0)); a workgroup barrier; lane 0 issues a system-scope release and stores the
//      epoch into flags[p][rank] of every rank's buffer (system-scope release stores);
//   2. wait: lane j < g polls flags[p][j] of its own buffer (system-scope acquire loads, s_sleep between polls) until
//      it holds the epoch -- BOUNDED: after ~kSpinLimit polls it records a timeout in `state` and stops waiting, so a
//      lost peer can never leave the kernel (and the GPU) spinning;
//   3. a workgroup barrier, then the g slots of parity p, which ARE the assembled [1, g * n] row (rank j's columns at
//      j * n), are copied to `rows` (an ordinary tensor).
// epoch (state[0], this rank's own device word) counts the steps, parity p = epoch & 1: a rank can only push parity p
// of step e + 2 after it saw every peer's step e + 1 flag, i.e. after every peer's stream finished step e's copy-out,
// so two parities suffice.  Kernels of one rank run in stream order, so state[0] needs no atomics.
// Failure is fail-stop: a step whose wait timed out writes NaN (0xFFFF in every 16-bit element, NaN in bf16 and fp16)
// to `rows` instead of the slots, whose contents are then stale; the timeout count state[1] is sticky, and every later
// step of this exchange only writes the NaN row (no push, no epoch advance) -- so the peers time out in turn and a lost
// rank never yields a silently wrong row on any rank.  The host reads state[1] (IpcAllGather.timeouts / check).
#include "common.hpp"

#include <cstring>

namespace bnb {

constexpr int IPC_FLAG_BYTES = 512;        // flags[2][64] u32
constexpr int IPC_MAX_RANKS = 64;
constexpr unsigned kSpinLimit = 1u << 22;  // ~0.5-1 s of polling with s_sleep 1

__host__ __device__ inline long long ipc_slot_bytes(int n, int elem) { return ((long long)n * elem + 15) / 16 * 16; }

__device__ __forceinline__ unsigned ld_acquire_sys(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_release_sys(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// state: [0] epoch of the last completed step (0 before the first), [1] timeouts seen (sticky), [2] last timed-out
// source rank + 1
__global__ void __launch_bounds__(256)
k_ipc_allgather_push(const unsigned long long* __restrict__ bufs, int rank, int world, long long slot_bytes,
                     const uint4* __restrict__ y, long long y_pieces, uint4* __restrict__ rows, unsigned* __restrict__ state) {
  __shared__ int s_fail;
  const int tid = threadIdx.x;
  const long long row_pieces = (long long)world * y_pieces;
  auto poison = [&]() {
    for (long long i = tid; i < row_pieces; i += blockDim.x) rows[i] = make_uint4(~0u, ~0u, ~0u, ~0u);
  };
  if (tid == 0) s_fail = state[1] != 0u;
  __syncthreads();
  if (s_fail) {                 // latched: an earlier step timed out, the exchange is out of step for good
    poison();
    return;
  }
  const unsigned e = state[0] + 1;
  const int p = e & 1;
  // 1. push this rank's slice into slot (p, rank) of every rank's buffer
  for (int j = 0; j < world; ++j) {
    uint8_t* dst = reinterpret_cast<uint8_t*>(bufs[j]) + IPC_FLAG_BYTES + ((long long)p * world + rank) * slot_bytes;
    for (long long i = tid; i < y_pieces; i += blockDim.x) reinterpret_cast<uint4*>(dst)[i] = y[i];
  }
  // (the peer pointers are generic: flat stores, counted on vmcnt AND lgkmcnt)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // this lane's pushes are done ...
  __syncthreads();                                    // ... and every lane's
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");     // system scope
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    for (int j = 0; j < world; ++j)
      st_release_sys(reinterpret_cast<unsigned*>(bufs[j]) + p * IPC_MAX_RANKS + rank, e);
  }
  // 2. wait for every source rank's flag of this step in this rank's own buffer (bounded)
  if (tid < world) {
    const unsigned* flag = reinterpret_cast<const unsigned*>(bufs[rank]) + p * IPC_MAX_RANKS + tid;
    unsigned it = 0;
    while (ld_acquire_sys(flag) != e) {
      if (++it >= kSpinLimit) {
        state[1] += 1;          // (a racy count is fine: any non-zero value reports the failure)
        state[2] = tid + 1;
        s_fail = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  if (s_fail) {                 // a source never pushed this step: its slot is stale, the row is not valid
    poison();
    return;
  }
  // 3. the g slots of parity p are the assembled row
  const uint8_t* own = reinterpret_cast<const uint8_t*>(bufs[rank]) + IPC_FLAG_BYTES + (long long)p * world * slot_bytes;
  for (int j = 0; j < world; ++j) {
    const uint4* src = reinterpret_cast<const uint4*>(own + (long long)j * slot_bytes);
    for (long long i = tid; i < y_pieces; i += blockDim.x) rows[(long long)j * y_pieces + i] = src[i];
  }
  __syncthreads();
  if (tid == 0) state[0] = e;
}

}  // namespace bnb

extern "C" {

// [additive] bytes of one rank's exchange buffer for `world` ranks and n elements of `elem` bytes per shard
long long cipc_allgather_buffer_bytes(int world, int n, int elem) {
  BNB_RANGE("cipc_allgather_buffer_bytes");
  return bnb::IPC_FLAG_BYTES + 2LL * world * bnb::ipc_slot_bytes(n, elem);
}

// [additive] allocate a zeroed exchange buffer: uncached device memory (*kind = 2), else fine-grained (*kind = 1) --
// both keep a peer's stores visible to the owner's system-scope acquire loads.  Plain coarse-grained memory is NOT a
// fallback: the owner's L2 could serve stale lines of the slots and flags the peers write over xGMI, so the gather
// could return an earlier step's row; when neither kind can be allocated this fails (NULL, cget_last_error*) and the
// caller keeps the RCCL gather.
void* cipc_alloc(long long bytes, int* kind) {
  BNB_RANGE("cipc_alloc");
  void* p = nullptr;
  int k = 2;
  if (hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached) != hipSuccess) {
    (void)hipGetLastError();
    k = 1;
    if (hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocFinegrained) != hipSuccess) {
      (void)hipGetLastError();
      bnb::set_error(2, "cipc_alloc: neither uncached nor fine-grained device memory could be allocated");
      return nullptr;
    }
  }
  if (hipMemset(p, 0, (size_t)bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    bnb::set_error(2, "cipc_alloc: memset failed");
    (void)hipFree(p);
    return nullptr;
  }
  if (kind) *kind = k;
  return p;
}

void cipc_free(void* p) {
  BNB_RANGE("cipc_free");
  if (p) (void)hipFree(p);
}

int cipc_handle_size() { return HIP_IPC_HANDLE_SIZE; }

// [additive] the IPC handle of a cipc_alloc buffer into `handle` (cipc_handle_size() bytes); 0 = ok
int cipc_get_handle(void* p, void* handle) {
  BNB_RANGE("cipc_get_handle");
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) {
    bnb::set_error((int)e, "cipc_get_handle: hipIpcGetMemHandle failed");
    return 1;
  }
  std::memcpy(handle, &h, sizeof(h));
  return 0;
}

// [additive] open a peer's handle; the mapped device pointer goes to *out; 0 = ok
int cipc_open_handle(const void* handle, void** out) {
  BNB_RANGE("cipc_open_handle");
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  const hipError_t e = hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
  if (e != hipSuccess) {
    bnb::set_error((int)e, "cipc_open_handle: hipIpcOpenMemHandle failed");
    return 1;
  }
  return 0;
}

int cipc_close_handle(void* p) { return hipIpcCloseMemHandle(p) == hipSuccess ? 0 : 1; }

// [additive] one decode all-gather step on the current stream: y [n] (this rank's shard, 16-bit elements, 16-B
// aligned) -> rows [world * n] (16-B aligned) through the exchange buffers `bufs` (device array of `world` pointers:
// this rank's own buffer at index `rank`, the opened peers' at theirs).  state: a device u32[4] zeroed once (epoch,
// timeouts).  Returns 0 = launched, 1 = shape / alignment not supported, 2 = launch error.  n * 2 must be a multiple of
// 16 (whole 16-B pieces; n % 8 == 0).
int callgather_ipc_16(const unsigned long long* bufs, int rank, int world, int n, const void* y, void* rows,
                      unsigned* state) {
  BNB_RANGE("callgather_ipc_16");
  if (world < 1 || world > bnb::IPC_MAX_RANKS || rank < 0 || rank >= world || n <= 0 || n % 8 ||
      ((uintptr_t)y & 15) || ((uintptr_t)rows & 15))
    return 1;
  const long long slot = bnb::ipc_slot_bytes(n, 2);
  hipLaunchKernelGGL(bnb::k_ipc_allgather_push, dim3(1), dim3(256), 0, bnb::current_stream(), bufs, rank, world, slot,
                     reinterpret_cast<const uint4*>(y), (long long)n * 2 / 16, reinterpret_cast<uint4*>(rows), state);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    bnb::set_error((int)e, "callgather_ipc_16 launch");
    return 2;
  }
  return 0;
}

}  // extern "C"
