// allreduce_p2p.hip — one-shot peer-to-peer gradient all-reduce over xGMI (single node).
//
// The reference averaged gradients through TF parameter servers or Horovod's NCCL all-reduce
// (resnet_model.py:108-116). RCCL rings are per-link bound and pay a multi-step
// latency that dominates small buckets (CIFAR ResNet's 3 MB of fp32 gradients). Here every GPU
// maps its peers' gradient buffers (HIP IPC, opened by the host runtime) and reduces a bucket in
// ONE kernel: out[i] = sum over ranks r of in_r[i], reading all 7 peers' slices concurrently
// over the 7 point-to-point xGMI links (one-shot: each GPU reads (W-1)/W more bytes than a
// ring but in one hop).
//
// Synchronisation (no host round trips, HIP-graph capturable; the epoch lives in device memory):
//   ready: after a bucket's gradient is complete on the stream, drn_p2p_signal writes the epoch
//          into slot [bucket][READY][my rank] of every peer's flag array (system-scope release,
//          preceded by an L2 write-back so peers read the gradient from memory);
//   reduce: every block polls its LOCAL flag array until all ranks' READY >= epoch, performs a
//          system-scope acquire (cache invalidate), then reduces with 16-byte loads;
//   done:   after all buckets, drn_p2p_signal(DONE); before the next step writes the gradient
//          buffer, drn_p2p_wait(DONE) — no rank overwrites an input a peer may still be reading.
// Every poll is bounded in TIME (P2PArgs::timeout_ms, measured on the 100 MHz s_memrealtime
// clock): on timeout the kernel records an error code and exits, so a missing peer can never
// hang the GPU. The error word also gates the optimizer: sgd_momentum_kernel skips the update
// when it is set, so a step whose exchange failed leaves weights and momentum untouched; the
// host reads a pinned copy of the word after every step (parallel/p2p.py) and aborts.
//
// Memory: the flag arrays and the output buffers (the two-shot all-gather reads the peers'
// outputs) are allocated UNCACHED (hipExtMallocWithFlags(hipDeviceMallocUncached), drn_p2p_alloc)
// and exported by IPC: a peer's system-scope store over xGMI and the owner's polling load then
// meet in memory, with no stale copy in either XCD L2 -- the coherence a coarse-grained hipMalloc
// buffer only gives at kernel boundaries.
//
// Two-shot variant for large buckets (reduce-scatter + all-gather): after READY,
// rank r reduces only its 1/W shard of the bucket (reading that shard from all peers) into its
// own output, publishes RS_DONE, and then copies every peer's reduced shard out of the peer's
// output buffer. Each GPU pulls 2(W-1)/W of the bucket over xGMI instead of (W-1)x: 1.75x vs 7x
// the bucket at W = 8, all 7 links busy in both phases.
#include "drn_common.h"


namespace drn {

constexpr int P2P_MAX_RANKS = 8;
constexpr int P2P_READY = 0, P2P_DONE = 1, P2P_RS_DONE = 2, P2P_KINDS = 3;

struct P2PArgs {
  float* out;                           // local output (never aliases an input)
  const float* in[P2P_MAX_RANKS];       // every rank's gradient bucket (index = rank), mapped
  const float* out_peer[P2P_MAX_RANKS]; // every rank's output bucket (two-shot all-gather)
  unsigned* flags_local;                // this rank's flag array [slots][3][8]
  unsigned* flags_peer[P2P_MAX_RANKS];  // every rank's flag array (remote mappings)
  const unsigned* epoch;                // device-resident step epoch (>= 1)
  int* err;                             // error word (0 = ok)
  int64_t n;                            // elements in the bucket (multiple of 4)
  int world, rank, slot;
  int timeout_ms;                       // bound of every device-side wait (<= 0: 60 s)
};

__device__ __forceinline__ unsigned flag_load(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ bool wait_all(const P2PArgs& a, int kind, unsigned e) {
  const unsigned* f = a.flags_local + (size_t)(a.slot * P2P_KINDS + kind) * P2P_MAX_RANKS;
  const unsigned long long ticks = 100000ull * (unsigned long long)(a.timeout_ms > 0 ? a.timeout_ms : 60000);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz, independent of the shader clock
  for (;;) {
    bool ok = true;
    for (int r = 0; r < a.world; ++r) ok = ok && flag_load(f + r) >= e;
    if (ok) return true;
    if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) return false;
    __builtin_amdgcn_s_sleep(2);
  }
}

// publish this rank's epoch e for (slot, kind) to every rank (incl. itself); one thread. The
// system-scope release makes every earlier write of this device (the gradient kernels, the bf16
// wire cast) visible to the peers reading it over xGMI.
__device__ __forceinline__ void publish(const P2PArgs& a, int kind, unsigned e) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  for (int r = 0; r < a.world; ++r) {
    unsigned* f = a.flags_peer[r] + (size_t)(a.slot * P2P_KINDS + kind) * P2P_MAX_RANKS + a.rank;
    __hip_atomic_store(f, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// kind = READY or DONE: publish this rank's epoch for `slot` (kept for the two-shot RS_DONE).
__global__ void p2p_signal_kernel(P2PArgs a, int kind) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  publish(a, kind, *a.epoch);
}

// wire element -> fp32 accumulate
template <typename W>
__device__ __forceinline__ float4 load4(const W* p, int64_t i);
template <>
__device__ __forceinline__ float4 load4<float>(const float* p, int64_t i) {
  return reinterpret_cast<const float4*>(p)[i];
}
template <>
__device__ __forceinline__ float4 load4<bf16_t>(const bf16_t* p, int64_t i) {
  const uint2 u = reinterpret_cast<const uint2*>(p)[i];
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}

// Signal + wait + reduce of one bucket in ONE launch: workgroup 0 publishes this rank's READY
// (the bucket is complete: the launch is stream-ordered after its producers), every workgroup
// polls its local flags for all ranks, acquires, and reduces out[i] = sum_r in_r[i] (fp32
// accumulate in rank order: identical on every rank, bitwise reproducible). W = wire type of the
// inputs (fp32, or bf16 shadows written by drn_p2p_cast).
template <typename W>
__global__ __launch_bounds__(256) void p2p_reduce_kernel(P2PArgs a) {
  __shared__ int ok;
  const unsigned e = *a.epoch;
  if (threadIdx.x == 0) {
    if (blockIdx.x == 0) publish(a, P2P_READY, e);
    ok = wait_all(a, P2P_READY, e) ? 1 : 0;
    if (!ok) atomicExch(a.err, 1);
  }
  __syncthreads();
  if (!ok) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // peers' gradient bytes, not stale cached lines
  const int64_t n4 = a.n / 4;
  const W* const* in = reinterpret_cast<const W* const*>(a.in);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 s = load4<W>(in[0], i);
    for (int r = 1; r < a.world; ++r) {
      const float4 v = load4<W>(in[r], i);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    reinterpret_cast<float4*>(a.out)[i] = s;
  }
}

// two-shot: shard of rank r = float4 range [r*sh, min((r+1)*sh, n4))
__device__ __forceinline__ void shard_of(const P2PArgs& a, int r, int64_t& lo, int64_t& hi) {
  const int64_t n4 = a.n / 4;
  const int64_t sh = (n4 + a.world - 1) / a.world;
  lo = r * sh < n4 ? r * sh : n4;
  hi = lo + sh < n4 ? lo + sh : n4;
}

// reduce-scatter (+ READY publish): my shard = sum over ranks of their inputs' shard
template <typename W>
__global__ __launch_bounds__(256) void p2p_rs_kernel(P2PArgs a) {
  __shared__ int ok;
  const unsigned e = *a.epoch;
  if (threadIdx.x == 0) {
    if (blockIdx.x == 0) publish(a, P2P_READY, e);
    ok = wait_all(a, P2P_READY, e) ? 1 : 0;
    if (!ok) atomicExch(a.err, 1);
  }
  __syncthreads();
  if (!ok) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  int64_t lo, hi;
  shard_of(a, a.rank, lo, hi);
  const W* const* in = reinterpret_cast<const W* const*>(a.in);
  for (int64_t i = lo + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < hi; i += (int64_t)gridDim.x * blockDim.x) {
    float4 s = load4<W>(in[0], i);
    for (int r = 1; r < a.world; ++r) {
      const float4 v = load4<W>(in[r], i);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    reinterpret_cast<float4*>(a.out)[i] = s;
  }
}

// all-gather: copy every peer's reduced shard out of the peer's output buffer
__global__ __launch_bounds__(256) void p2p_ag_kernel(P2PArgs a) {
  __shared__ int ok;
  if (threadIdx.x == 0) {
    ok = wait_all(a, P2P_RS_DONE, *a.epoch) ? 1 : 0;
    if (!ok) atomicExch(a.err, 3);
  }
  __syncthreads();
  if (!ok) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  for (int r = 0; r < a.world; ++r) {
    if (r == a.rank) continue;
    int64_t lo, hi;
    shard_of(a, r, lo, hi);
    const float4* src = reinterpret_cast<const float4*>(a.out_peer[r]);
    float4* dst = reinterpret_cast<float4*>(a.out);
    for (int64_t i = lo + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < hi; i += (int64_t)gridDim.x * blockDim.x)
      dst[i] = src[i];
  }
}

// Step boundary, one thread, ONE launch per step (before the step writes the gradient buffer):
// publish DONE for the finished epoch e (this rank's reductions of step e were stream-ordered
// before this launch, so it no longer reads any peer's buffers), wait until every rank published
// DONE >= e (no rank overwrites an input or output buffer a peer may still be reading), then
// advance the device epoch.
__global__ void p2p_step_kernel(P2PArgs a, unsigned* epoch_rw) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const unsigned e = *epoch_rw;
  if (e > 0) {
    publish(a, P2P_DONE, e);
    if (!wait_all(a, P2P_DONE, e)) atomicExch(a.err, 2);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "");
  *epoch_rw = e + 1;
}

// fp32 bucket -> bf16 wire shadow (round to nearest even), 4 elements per thread
__global__ __launch_bounds__(256) void p2p_cast_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, int64_t n4) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    reinterpret_cast<uint2*>(y)[i] = make_uint2(pack2bf(v.x, v.y), pack2bf(v.z, v.w));
  }
}

}  // namespace drn

static bool p2p_check(const drn::P2PArgs* a) {
  if (a->world < 1 || a->world > drn::P2P_MAX_RANKS || a->rank < 0 || a->rank >= a->world) return false;
  if (a->n % 4) return false;
  for (int r = 0; r < a->world; ++r)
    if (a->in[r] == nullptr || a->flags_peer[r] == nullptr || a->out_peer[r] == nullptr) return false;
  return a->out != nullptr && a->flags_local != nullptr && a->epoch != nullptr && a->err != nullptr;
}

DRN_API int drn_p2p_signal(const drn::P2PArgs* a, int kind, hipStream_t s) {
  if (!p2p_check(a) || kind < 0 || kind >= drn::P2P_KINDS) return (int)hipErrorInvalidValue;
  drn::launch(drn::p2p_signal_kernel, dim3(1), dim3(64), 0, s, *a, kind);
  return (int)hipGetLastError();
}

// one-shot all-reduce of one bucket (publish + wait + reduce in one launch); wire_bf16: the
// peers' inputs are bf16 shadows (drn_p2p_cast), accumulated in fp32
DRN_API int drn_p2p_reduce(const drn::P2PArgs* a, int blocks, int wire_bf16, hipStream_t s) {
  if (!p2p_check(a)) return (int)hipErrorInvalidValue;
  if (blocks < 1) blocks = 1;
  if (wire_bf16)
    drn::launch(drn::p2p_reduce_kernel<bf16_t>, dim3(blocks), dim3(256), 0, s, *a);
  else
    drn::launch(drn::p2p_reduce_kernel<float>, dim3(blocks), dim3(256), 0, s, *a);
  return (int)hipGetLastError();
}

// two-shot all-reduce of one bucket: reduce-scatter (with the READY publish), publish RS_DONE,
// all-gather of the peers' fp32 shards
DRN_API int drn_p2p_reduce2(const drn::P2PArgs* a, int blocks, int wire_bf16, hipStream_t s) {
  if (!p2p_check(a)) return (int)hipErrorInvalidValue;
  if (blocks < 1) blocks = 1;
  if (wire_bf16)
    drn::launch(drn::p2p_rs_kernel<bf16_t>, dim3(blocks), dim3(256), 0, s, *a);
  else
    drn::launch(drn::p2p_rs_kernel<float>, dim3(blocks), dim3(256), 0, s, *a);
  drn::launch(drn::p2p_signal_kernel, dim3(1), dim3(64), 0, s, *a, (int)drn::P2P_RS_DONE);
  drn::launch(drn::p2p_ag_kernel, dim3(blocks), dim3(256), 0, s, *a);
  return (int)hipGetLastError();
}

DRN_API int drn_p2p_step(const drn::P2PArgs* a, unsigned* epoch_rw, hipStream_t s) {
  if (!p2p_check(a)) return (int)hipErrorInvalidValue;
  drn::launch(drn::p2p_step_kernel, dim3(1), dim3(64), 0, s, *a, epoch_rw);
  return (int)hipGetLastError();
}

DRN_API int drn_p2p_cast(const float* x, void* y, int64_t n, hipStream_t s) {
  if (n % 4) return (int)hipErrorInvalidValue;
  int64_t b = (n / 4 + 255) / 256;
  if (b > 1024) b = 1024;
  if (b < 1) b = 1;
  drn::launch(drn::p2p_cast_kernel, dim3((unsigned)b), dim3(256), 0, s, x, (bf16_t*)y, n / 4);
  return (int)hipGetLastError();
}

DRN_API int drn_p2p_args_size() { return (int)sizeof(drn::P2PArgs); }

// Zeroed UNCACHED device memory for the flag arrays / output buffers that peers access over
// xGMI (exportable with hipIpcGetMemHandle like any device allocation); freed by drn_p2p_free.
DRN_API int drn_p2p_alloc(void** p, size_t bytes) {
  *p = nullptr;
  hipError_t e = hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(*p, 0, bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  return (int)e;
}

DRN_API int drn_p2p_free(void* p) { return (int)hipFree(p); }
