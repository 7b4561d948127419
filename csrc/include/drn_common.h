// drn_common.h — shared device helpers for the gfx950 (CDNA4) kernel library.
//
// Storage conventions used across every kernel in csrc/kernels/:
//   * activations are NHWC bf16 (raw uint16 storage, round-to-nearest-even on store);
//   * conv weights are KRSC bf16 ([Cout][R][S][Cin]) so the GEMM reduction dim is contiguous;
//   * statistics, master weights, momentum and gradients are fp32.
// Wave width is 64 everywhere (CDNA wavefront), never 32.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define DRN_API extern "C" __attribute__((visibility("default")))

#include <tuple>
#include <type_traits>
#include <utility>

typedef uint16_t bf16_t;
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

namespace drn {

__device__ __forceinline__ float bf2f(uint32_t u16) { return __uint_as_float(u16 << 16); }

__device__ __forceinline__ uint16_t f2bf(float f) {
  // hipcc lowers this to v_cvt_pk_bf16_f32 (RNE, NaN-preserving) on gfx950.
  __hip_bfloat16 h = __float2bfloat16(f);
  return __builtin_bit_cast(uint16_t, h);
}

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// Two floats -> packed bf16 pair: one v_cvt_pk_bf16_f32 (RNE, NaN-preserving) instead of two
// conversions plus a shift/or.
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  const f32x2_t f = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, bf16x2_t));
}

// 8 bf16 held in a uint4 (16 bytes) <-> 8 floats.
__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack2bf(f[0], f[1]); v.y = pack2bf(f[2], f[3]);
  v.z = pack2bf(f[4], f[5]); v.w = pack2bf(f[6], f[7]);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// 16-byte LDS read / write in inline asm, for LDS rewritten in place while LDS-DMAs of later
// pipeline stages are still in flight: hipcc assumes a plain ds_read may alias a pending
// global_load_lds and waits vmcnt(0) before its use, draining the pipeline. The caller orders
// the reads with lds_wait_all() (and the writes with an lgkmcnt wait before its barrier).
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)reinterpret_cast<uintptr_t>(p); }

__device__ __forceinline__ u32x4_t lds_read16(uint32_t addr) {
  u32x4_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}

__device__ __forceinline__ void lds_write16(uint32_t addr, u32x4_t v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(v) : "memory");
}

// s_waitcnt lgkmcnt(0) that the N registers it retires depend on (their consumers cannot be
// scheduled above it).
template <int N>
__device__ __forceinline__ void lds_wait_all(u32x4_t (&v)[N]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[i]));
}

__device__ __forceinline__ void unpack8v(const u32x4_t& v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ u32x4_t pack8v(const float* f) {
  u32x4_t v;
  v.x = pack2bf(f[0], f[1]); v.y = pack2bf(f[2], f[3]);
  v.z = pack2bf(f[4], f[5]); v.w = pack2bf(f[6], f[7]);
  return v;
}

typedef short s16x2_t __attribute__((ext_vector_type(2)));

// relu(x * sc + sh) of 8 bf16 (one 16-byte piece), packed: per pair one v_pk_fma_f32, one
// v_cvt_pk_bf16_f32 and the ReLU as ONE v_pk_max_i16 against 0 on the packed result (a bf16
// with its sign bit set is a negative int16; -0 becomes +0). sc2/sh2 hold the 4 channel pairs.
template <bool RELU>
__device__ __forceinline__ u32x4_t bn_relu_piece(const u32x4_t& v, const f32x2_t* sc2, const f32x2_t* sh2) {
  u32x4_t o;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const uint32_t u = v[p];
    f32x2_t f = {__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
    f = f * sc2[p] + sh2[p];
    uint32_t r = __builtin_bit_cast(uint32_t, __builtin_convertvector(f, bf16x2_t));
    if (RELU) {
      const s16x2_t z = {0, 0};
      r = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2_t, r), z));
    }
    o[p] = r;
  }
  return o;
}

// The same for N pieces in LDS (v[] already read and lds_wait_all'ed), written back in place;
// piece i keeps its (zero) contents unless bit i of `ok` is set -- pieces loaded from the zero
// page stay zero. Branch-free. Ends with the lgkmcnt wait that completes the writes before the
// caller's barrier.
template <int N, bool RELU>
__device__ __forceinline__ void lds_bn_relu_store(const uint32_t (&addr)[N], const u32x4_t* v, uint32_t ok,
                                                  const f32x2_t* sc2, const f32x2_t* sh2) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    u32x4_t o = bn_relu_piece<RELU>(v[i], sc2, sh2);
    const unsigned m = ((ok >> i) & 1u) ? 0xffffffffu : 0u;
    o.x &= m;
    o.y &= m;
    o.z &= m;
    o.w &= m;
    lds_write16(addr[i], o);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// XCD-aware bijective remap of a linear workgroup id: consecutive logical tiles land on the
// same XCD (blocks b, b+8, b+16 ... share an XCD under round-robin dispatch), so neighbouring
// tiles that share an operand panel share that XCD's L2. Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// ---------------------------------------------------------------------------------------------
// Kernel launch + native step plans (csrc/kernels/plan.hip). Every kernel of the library is
// launched through drn::launch: normally a plain hipLaunchKernelGGL; while the CALLING thread
// records a step plan, the launch (kernel, grid, block, LDS bytes, stream and a by-value copy of
// every argument) is appended to the plan instead, to be replayed later by drn_plan_replay with
// one host call per plan segment (no Python, no argument marshalling per launch).
// ---------------------------------------------------------------------------------------------
struct Plan;
extern thread_local Plan* g_plan_rec;
void plan_add_launch(Plan* p, const void* fn, dim3 grid, dim3 block, size_t shm, hipStream_t s, void* blob,
                     void** argv, void (*del)(void*));

template <typename T, size_t... I>
inline void plan_argv(T* t, void** argv, std::index_sequence<I...>) {
  ((argv[I] = static_cast<void*>(&std::get<I>(*t))), ...);
}

template <typename... KArgs, typename... Args>
inline void launch(void (*kern)(KArgs...), dim3 grid, dim3 block, size_t shm, hipStream_t s, Args&&... args) {
  static_assert(sizeof...(KArgs) == sizeof...(Args), "kernel argument count");
  if (g_plan_rec != nullptr) {
    using T = std::tuple<std::remove_cv_t<std::remove_reference_t<KArgs>>...>;
    T* t = new T(std::forward<Args>(args)...);  // converted to the kernel's parameter types
    void** argv = new void*[sizeof...(KArgs) + 1];
    plan_argv(t, argv, std::index_sequence_for<KArgs...>{});
    plan_add_launch(g_plan_rec, reinterpret_cast<const void*>(kern), grid, block, shm, s, t, argv,
                    [](void* q) { delete static_cast<T*>(q); });
    return;
  }
  hipLaunchKernelGGL(kern, grid, block, shm, s, std::forward<Args>(args)...);
}

}  // namespace drn

#define DRN_RET_LAST_ERR() return (int)hipGetLastError()
