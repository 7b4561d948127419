// conv_wgrad.hip — weight gradient of an NHWC bf16 convolution on CDNA4 MFMA (gfx950).
//
// Replaces the Conv2DBackpropFilter the reference graph gets from autodiff of every
// `conv2d_fixed_padding` (reference resnet_model_official.py:87-91).
//
// GEMM view:  dW[cout][k] = sum_{pixels m} dY[m][cout] * Patch[m][k],  k = (r, s, ci).
// Both operands are stored with the NON-reduction dim contiguous (NHWC rows), so the
// fragments are read out of LDS with the gfx950 hardware transpose `ds_read_b64_tr_b16`
// (4 rows x 16 cols per 16-lane group, delivered column-major). MFMA operand A = patches
// (rows = k), operand B = dY (cols = cout): the accumulator holds 4 consecutive k of one output
// channel per lane -> 16-byte fp32 stores into the KRSC gradient.
//
// Block = 4 waves in a 2x2 arrangement over a BKK(k) x BCO(cout) output tile (each wave
// BKK/2 x BCO/2); every step stages 64 output pixels (two 32-deep MFMA k-slices) of both
// operands, register-staged and double-buffered, one barrier per step. The thread->vector
// assignment keeps each thread on ONE 8-channel chunk of k for the whole kernel (r,s,ci decoded
// once; the pixel decode per vector uses magic-number division).
// LDS rows are BKK*2 / BCO*2 bytes with a 32-byte-slot XOR swizzle h(row) chosen so that the
// 8 rows a 32-lane half reads per transposed read hit 8 distinct bank slots (conflict-free) and
// every 8-lane ds_write_b128 group stays inside one 128-byte bank window.
// Grid y splits the pixel range (split-K) into fp32 partial slabs reduced deterministically by
// drn_splitk_reduce (no float atomics: bitwise-reproducible weight gradients).
#include "drn_common.h"
#include "drn_conv.h"
#include <stdlib.h>

namespace drn {

// Per-workgroup timeline of the LDS-DMA weight-gradient kernel, compiled in only with
// -DDRN_CONV_TRACE (the diagnostics build, as for the forward conv): b = {start, main-loop end,
// end} in s_memrealtime ticks (100 MHz) + HW_ID / XCC_ID, at the workgroup's linear launch index.
#ifdef DRN_CONV_TRACE
__device__ unsigned long long* g_wgrad_trace = nullptr;
__device__ __forceinline__ unsigned long long wg_realtime() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
  return t;
}
#endif

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const DrnFastDiv& f) { return drn_fdiv(n, f); }

// 32-byte-slot swizzle for rows of W bytes (W = 64, 128 or 256). W = 64 (the narrow 32-channel
// dY image of the K <= 32 weight gradients): 2 slots per row; the transposed fragment reads of
// one 32-lane half touch rows {r..r+3, r+8..r+11} at 4 byte offsets each, rows r and r+8 share
// their banks (4 rows per 256-byte bank row), so bit 3 of the row flips the slot.
template <int W>
__device__ __forceinline__ int slot_swz(int row) {
  if constexpr (W == 256) return (row & 3) | (((row >> 3) & 1) << 2);
  if constexpr (W == 64) return (row >> 3) & 1;
  return ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
}

// byte offset of element column `col` (bf16) of `row` in a swizzled image with W-byte rows
template <int W>
__device__ __forceinline__ int swz_off(int row, int col) {
  return row * W + ((((col >> 4) ^ slot_swz<W>(row))) << 5) + (col & 15) * 2;
}

typedef short s16x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4v lds_s16x4;

__device__ __forceinline__ s16x4v tr_read(const char* base, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + byte_off));
}

// Weight-gradient tile out: the split's fp32 partial slab (reduced by drn_splitk_reduce), or with
// atomic_out the fp32 adds straight into the (pre-zeroed) gradient -- no slab, no reduce
// launch; for layers with few weights (CIFAR) the reduce launch costs more than the atomics.
// Not bitwise reproducible across runs (the deterministic mode never selects it).
template <int MI, int MJ>
__device__ __forceinline__ void wgrad_store(const DrnConvWgradArgs& a, f32x4_t (&acc)[MI][MJ], int split, int cb,
                                            int kb, int Ktot, int lane) {
  float* out = a.out + (a.atomic_out ? (size_t)0 : (size_t)split * a.K * Ktot);
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      const int co = cb + 16 * j + (lane & 15);
      const int kr = kb + 16 * i + 4 * (lane >> 4);
      if (co < a.K && kr < Ktot) {
        float* p = out + (size_t)co * Ktot + kr;
        if (a.atomic_out) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            __hip_atomic_fetch_add(p + e, acc[i][j][e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          *reinterpret_cast<f32x4_t*>(p) = acc[i][j];
        }
      }
    }
}

template <int BKK, int BCO, bool PRO, int NST>
__global__ __launch_bounds__(256, NST == 1 ? 4 : 2) void conv_wgrad_kernel(DrnConvWgradArgs a) {
  constexpr int BP = 64;                 // pixels per step
  constexpr int WA = BKK * 2;            // patch image row bytes
  constexpr int WB = BCO * 2;            // dY image row bytes
  constexpr int A_BYTES = BP * WA;
  constexpr int STAGE = A_BYTES + BP * WB;
  constexpr int CHA = BKK / 8, CHB = BCO / 8;          // 16-byte chunks per row
  constexpr int NVA = BP * CHA / 256, NVB = BP * CHB / 256;
  constexpr int RPA = 64 / CHA, RPB = 64 / CHB;        // rows per wave-instruction group
  constexpr int WKK = BKK / 2, WCO = BCO / 2;          // wave tile
  constexpr int MI = WKK / 16, MJ = WCO / 16;
  static_assert(NVA >= 1 && NVB >= 1, "tiles must cover 256 threads");

  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Ktot = a.R * a.S * a.C;
  const int M = a.N * a.P * a.Q;
  const int nkt = (Ktot + BKK - 1) / BKK;
  // XCD-aware order: workgroups are dispatched round-robin over the 8 XCDs by linear id, so the
  // (k-tile, channel-tile) blocks of one pixel split -- which all read the same pixels of x and
  // dY -- would land on different XCDs and fetch them into 8 different L2s. Remapping the linear
  // id keeps consecutive logical blocks (the tiles of a split) on one XCD and its L2.
  const int ntile = gridDim.x;
  const int lin = xcd_remap(blockIdx.x + blockIdx.y * ntile, ntile * gridDim.y);
  const int tile = lin % ntile;
  const int split = lin / ntile;
  const int kt = tile % nkt;
  const int ct = tile / nkt;
  const int k0 = kt * BKK, c0 = ct * BCO;
  const int mbeg = split * a.pix_per_split;
  const int mend = min(M, mbeg + a.pix_per_split);

  // patch loader: fixed chunk per thread
  const int pchunk = lane % CHA;
  const int prow0 = lane / CHA;
  const int kk = k0 + pchunk * 8;
  const bool kvalid = kk < Ktot;
  int ci = 0, rr = 0, ss = 0;
  if (kvalid) {
    const int tap = kk / a.C;
    ci = kk - tap * a.C;
    rr = tap / a.S;
    ss = tap - rr * a.S;
  }
  float sc[8], sh[8];
  if constexpr (PRO) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = kvalid ? a.in_scale[ci + j] : 0.f;
      sh[j] = kvalid ? a.in_shift[ci + j] : 0.f;
    }
  }
  const int dchunk = lane % CHB;
  const int drow0 = lane / CHB;
  const int dc = c0 + dchunk * 8;
  const bool dvalid_c = dc < a.K;
  const uint32_t PQ = (uint32_t)(a.P * a.Q);

  uint4 rp[NVA], rd[NVB];
  auto load_stage = [&](int mstep) {
#pragma unroll
    for (int i = 0; i < NVA; ++i) {
      const int row = prow0 + RPA * (wave + 4 * i);
      const int m = mstep + row;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (kvalid && m < mend) {
        const uint32_t n = fdiv((uint32_t)m, a.fd_pq);
        const uint32_t rem = (uint32_t)m - n * PQ;
        const uint32_t p = fdiv(rem, a.fd_q);
        const uint32_t q = rem - p * (uint32_t)a.Q;
        const int h = (int)p * a.stride - a.pad_h + rr;
        const int w = (int)q * a.stride - a.pad_w + ss;
        if (h >= 0 && w >= 0 && h < a.H && w < a.W) {
          v = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(a.x) +
                                              ((size_t)((int)n * a.H + h) * a.W + w) * a.C + ci);
          if constexpr (PRO) {
            float f[8];
            unpack8(v, f);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              f[j] = f[j] * sc[j] + sh[j];
              if (a.relu_in) f[j] = fmaxf(f[j], 0.f);
            }
            v = pack8(f);
          }
        }
      }
      rp[i] = v;
    }
#pragma unroll
    for (int i = 0; i < NVB; ++i) {
      const int row = drow0 + RPB * (wave + 4 * i);
      const int m = mstep + row;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (dvalid_c && m < mend)
        v = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(a.dy) + (size_t)m * a.K + dc);
      rd[i] = v;
    }
  };
  auto store_stage = [&](char* st) {
#pragma unroll
    for (int i = 0; i < NVA; ++i) {
      const int row = prow0 + RPA * (wave + 4 * i);
      *reinterpret_cast<uint4*>(st + swz_off<WA>(row, pchunk * 8)) = rp[i];
    }
    char* sd = st + A_BYTES;
#pragma unroll
    for (int i = 0; i < NVB; ++i) {
      const int row = drow0 + RPB * (wave + 4 * i);
      *reinterpret_cast<uint4*>(sd + swz_off<WB>(row, dchunk * 8)) = rd[i];
    }
  };

  f32x4_t acc[MI][MJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < MJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int T = (mend > mbeg) ? (mend - mbeg + BP - 1) / BP : 0;
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int wk = wave & 1, wc = wave >> 1;

  if (T > 0) {
    load_stage(mbeg);
    if constexpr (NST == 2) {
      store_stage(smem);
      __syncthreads();
    }
  }
  for (int t = 0; t < T; ++t) {
    const char* cur = smem + (NST == 2 ? (t & 1) * STAGE : 0);
    const bool more = (t + 1) < T;
    if constexpr (NST == 1) {
      // single LDS stage (half the LDS -> 2x the resident workgroups): write the registers
      // loaded during the previous step, then immediately issue the next step's loads
      store_stage(smem);
      __syncthreads();
    }
    if (more) load_stage(mbeg + (t + 1) * BP);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8_t af[MI], bfr[MJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int col = wk * WKK + 16 * i + 4 * p4;
        const int r0 = 32 * ks + 8 * g + q4;
        const s16x4v lo = tr_read(cur, swz_off<WA>(r0, col));
        const s16x4v hi = tr_read(cur, swz_off<WA>(r0 + 4, col));
        af[i] = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        const int col = wc * WCO + 16 * j + 4 * p4;
        const int r0 = 32 * ks + 8 * g + q4;
        const s16x4v lo = tr_read(cur + A_BYTES, swz_off<WB>(r0, col));
        const s16x4v hi = tr_read(cur + A_BYTES, swz_off<WB>(r0 + 4, col));
        bfr[j] = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < MJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if constexpr (NST == 2) {
      if (more) store_stage(smem + ((t + 1) & 1) * STAGE);
    }
    __syncthreads();
  }

  wgrad_store<MI, MJ>(a, acc, split, c0 + wc * WCO, k0 + wk * WKK, Ktot, lane);
}

template <int BKK, int BCO, bool PRO>
static int launch_wgrad(DrnConvWgradArgs* a, hipStream_t s) {
  constexpr int NST = 2;
  constexpr int LDS = NST * (64 * BKK * 2 + 64 * BCO * 2);
  static bool attr_set = false;
  auto kern = conv_wgrad_kernel<BKK, BCO, PRO, NST>;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr_set = true;
  }
  const int Ktot = a->R * a->S * a->C;
  const int nkt = (Ktot + BKK - 1) / BKK;
  const int nct = (a->K + BCO - 1) / BCO;
  drn::launch(kern, dim3(nkt * nct, a->splits), dim3(256), LDS, s, *a);
  return (int)hipGetLastError();
}

template <bool PRO>
static int dispatch_wgrad(DrnConvWgradArgs* a, hipStream_t s) {
  const int Ktot = a->R * a->S * a->C;
  const bool wide_k = Ktot > 64;
  const bool wide_c = a->K > 64;
  if (wide_k && wide_c) return launch_wgrad<128, 128, PRO>(a, s);
  if (wide_k) return launch_wgrad<128, 64, PRO>(a, s);
  if (wide_c) return launch_wgrad<64, 128, PRO>(a, s);
  return launch_wgrad<64, 64, PRO>(a, s);
}

// ---------------------------------------------------------------------------------------
// LDS-DMA variant (no fused prologue): both operand images are filled by
// `global_load_lds_dwordx4` NS stages deep (counted vmcnt + raw barrier, like the forward
// kernel), so the 64-pixel steps no longer wait on a register round trip. The images keep the
// exact swizzled layout the transposed reads above expect; an LDS-DMA writes lane-linear, so
// the 32-byte-slot swizzle is applied to the per-lane SOURCE address instead: lane i of a
// wave-instruction fills physical 16-byte chunk (i mod W/16) of row (i div W/16) and therefore
// loads logical chunk 2*(slot ^ h(row)) + half. With wave w issuing instructions w, w+4, ...
// the swizzle bit that varies between instructions is wave-uniform, so each lane decodes its
// (tap, channel) chunk once. Out-of-image taps, pixels past the split and channels past K
// read the zero page.
// ---------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void wg_lds_void;
typedef __attribute__((address_space(1))) const void wg_gbl_void;

template <int N>
__device__ __forceinline__ void wg_wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int V>
struct drn_int_c {
  static constexpr int value = V;
};
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(drn_int_c<B>{});
    static_for<B + 1, E>(f);
  }
}

template <int OFF>
__device__ __forceinline__ s16x4v tr_read_asm(uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
  s16x4v r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}

// s_waitcnt lgkmcnt(N) that the fragments it retires depend on (so no MFMA reading them can be
// scheduled above it).
template <int N, int MI, int MJ>
__device__ __forceinline__ void lgkm_fence(s16x4v (&a)[MI][2], s16x4v (&b)[MJ][2]) {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
#pragma unroll
  for (int i = 0; i < MI; ++i) asm volatile("" : "+v"(a[i][0]), "+v"(a[i][1]));
#pragma unroll
  for (int j = 0; j < MJ; ++j) asm volatile("" : "+v"(b[j][0]), "+v"(b[j][1]));
}

// PRO: x is the RAW pre-BN input of a conv whose forward applied relu(x * in_scale + in_shift)
// in its prologue; the same transform is applied here to the patch image in LDS: after its
// counted vmcnt wait each lane rewrites the pieces its own LDS-DMAs landed for the stage (the
// lane's channels are fixed for the whole kernel, so scale/shift stay in registers) and the
// stage's barrier publishes them. Zero-page pieces (padding, pixels past the split) stay zero.
//
// IL: the next stage's LDS-DMA pieces are issued one at a time between this stage's MFMAs
// (instead of all right after the barrier, where every wave issues in lockstep and the matrix
// pipe idles for the DMA issue time).
//
// Loader address arithmetic (measured per-workgroup timelines, profiles/r3_wgrad_timelines.txt:
// 1.4 us per 64-pixel step at 2 workgroups/CU, i.e. ~35 % of the MFMA rate; the main loop issued
// ~170 VALU/SALU instructions per wave and step for 32 MFMAs, most of them the per-piece pixel
// decode and zero-page selects): every source address is a WAVE-UNIFORM stage base (SGPRs) plus a
// per-lane offset fixed for the whole kernel, and a stage whose pieces are all in range (every
// stage but a split's partial last one, when the tile's channel ranges are full) issues with no
// per-lane test at all.
// LIN: 1x1 stride-1 unpadded convolutions (33 of ResNet-50's 53 weight gradients): the patch row
// of pixel m is x[m][k0..] itself, so the patch loader is as cheap as the dY loader (no pixel
// decode, no padding test).
template <int BKK, int BCO, int NS, int BP = 64, bool PRO = false, bool IL = false, bool LIN = false>
__global__ __launch_bounds__(256) void conv_wgrad_glds_kernel(DrnConvWgradArgs a, const void* __restrict__ zero) {
  static_assert(BP == 32 || BP == 64, "pixels per stage");
  constexpr int KS = BP / 32;  // 32-deep MFMA k-slices per stage
  constexpr int WA = BKK * 2, WB = BCO * 2;       // image row bytes
  constexpr int A_BYTES = BP * WA;
  constexpr int STAGE = A_BYTES + BP * WB;
  constexpr int LPA = WA / 16, LPB = WB / 16;     // lanes per row in one wave-instruction
  constexpr int RIA = 64 / LPA, RIB = 64 / LPB;   // rows per wave-instruction
  constexpr int IA = BP / RIA / 4, IB = BP / RIB / 4;  // instructions per wave per stage
  constexpr int G = IA + IB;
  constexpr int D = NS - 1;
  constexpr int WKK = BKK / 2, WCO = BCO / 2;
  constexpr int MI = WKK / 16, MJ = WCO / 16;
  static_assert(IA >= 1 && IB >= 1 && NS >= 2, "geometry");

  extern __shared__ __attribute__((aligned(1024))) char smem[];
#ifdef DRN_CONV_TRACE
  unsigned long long* const trace = g_wgrad_trace;
  unsigned long long t_start = 0;
  if (trace != nullptr) t_start = wg_realtime();
#endif

  // (wave index made provably wave-uniform: LDS-DMA destinations then stay in SGPRs / M0)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Ktot = a.R * a.S * a.C;
  const int M = a.N * a.P * a.Q;
  const int nkt = (Ktot + BKK - 1) / BKK;
  // XCD-aware order: workgroups are dispatched round-robin over the 8 XCDs by linear id, so the
  // (k-tile, channel-tile) blocks of one pixel split -- which all read the same pixels of x and
  // dY -- would land on different XCDs and fetch them into 8 different L2s. Remapping the linear
  // id keeps consecutive logical blocks (the tiles of a split) on one XCD and its L2.
  const int ntile = gridDim.x;
  const int lin = xcd_remap(blockIdx.x + blockIdx.y * ntile, ntile * gridDim.y);
  const int tile = lin % ntile;
  const int split = lin / ntile;
  const int kt = tile % nkt;
  const int ct = tile / nkt;
  const int k0 = kt * BKK, c0 = ct * BCO;
  const int mbeg = split * a.pix_per_split;
  const int mend = min(M, mbeg + a.pix_per_split);

  // ---- A (patches) loader: row-in-instruction and logical chunk of this lane ----
  const int arow = lane / LPA;                 // + RIA * instruction
  int alc;
  {
    const int pc = lane % LPA;
    // row of the first instruction of this wave; the swizzle of later ones is identical
    const int row = RIA * wave + arow;
    alc = 2 * ((pc >> 1) ^ slot_swz<WA>(row)) + (pc & 1);
  }
  const int kk = k0 + alc * 8;
  const bool kvalid = kk < Ktot;
  int ci = 0, rr = 0, ss = 0;
  if (kvalid) {
    const int tap = kk / a.C;
    ci = kk - tap * a.C;
    rr = tap / a.S;
    ss = tap - rr * a.S;
  }
  const int roff = rr - a.pad_h, soff = ss - a.pad_w;
  f32x2_t psc2[4], psh2[4];  // fused BN of this lane's 8 input channels (channel pairs)
  if constexpr (PRO) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      psc2[p] = kvalid ? f32x2_t{a.in_scale[ci + 2 * p], a.in_scale[ci + 2 * p + 1]} : f32x2_t{0.f, 0.f};
      psh2[p] = kvalid ? f32x2_t{a.in_shift[ci + 2 * p], a.in_shift[ci + 2 * p + 1]} : f32x2_t{0.f, 0.f};
    }
    // retire these loads now, before any LDS-DMA is in flight (a use inside the pipelined
    // loop would otherwise make hipcc wait vmcnt(0) there every stage)
#pragma unroll
    for (int p = 0; p < 4; ++p) asm volatile("" : "+v"(psc2[p]), "+v"(psh2[p]));
  }
  static_assert(!PRO || IA * NS <= 32, "validity mask bits");
  uint32_t okm = 0;  // PRO: bit (slot * IA + i) = piece i of that stage came from the image
  // ---- B (dY) loader ----
  const int brow = lane / LPB;
  int blc;
  {
    const int pc = lane % LPB;
    const int row = RIB * wave + brow;
    blc = 2 * ((pc >> 1) ^ slot_swz<WB>(row)) + (pc & 1);
  }
  const int dc = c0 + blc * 8;
  const bool cvalid = dc < a.K;
  const bf16_t* __restrict__ xg = reinterpret_cast<const bf16_t*>(a.x);
  const bf16_t* __restrict__ dyg = reinterpret_cast<const bf16_t*>(a.dy) + dc;
  static_assert(!(LIN && IL), "LIN: plain stage issue only");
  // uniform fast-path conditions (every lane's k / output-channel chunk in range) and the per-lane
  // element offsets of the pieces inside a stage (stage base = uniform pixel offset)
  const bool a_full = k0 + BKK <= Ktot, b_full = c0 + BCO <= a.K;
  const bf16_t* __restrict__ dy0 = reinterpret_cast<const bf16_t*>(a.dy);
  uint32_t offB[IB], offA[LIN ? IA : 1];
#pragma unroll
  for (int i = 0; i < IB; ++i) offB[i] = (uint32_t)((RIB * (wave + 4 * i) + brow) * a.K + dc);
  if constexpr (LIN) {
#pragma unroll
    for (int i = 0; i < IA; ++i) offA[i] = (uint32_t)((RIA * (wave + 4 * i) + arow) * a.C + kk);
  }
  // Pixel coordinates of this lane's A rows, decoded once and then advanced by 64 pixels per
  // stage with adds/compares (a magic-number division per row per stage made the loader
  // VALU-bound: mul_hi/mul_lo/64-bit mads are quarter rate). Offsets use 24-bit multiplies
  // (every ResNet activation dimension product is < 2^24).
  const int HWC = a.H * a.W * a.C, WC = a.W * a.C;
  const int dq = BP % a.Q, dp = BP / a.Q;
  int am[IA], an[IA], ap[IA], aq[IA];
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    const int m = mbeg + RIA * (wave + 4 * i) + arow;
    am[i] = m;
    const uint32_t n = fdiv((uint32_t)m, a.fd_pq);
    const uint32_t rem = (uint32_t)m - n * (uint32_t)(a.P * a.Q);
    const uint32_t p = fdiv(rem, a.fd_q);
    an[i] = (int)n;
    ap[i] = (int)p;
    aq[i] = (int)(rem - p * (uint32_t)a.Q);
  }
  // Generic patch loader state, advanced incrementally (no multiplies in the loop): the input row
  // / column of the lane's tap (hh, ww) and the element offset po of (n, hh, ww, ci); the q wrap is
  // a select, p wraps (an image boundary inside the 64-pixel step) a short loop.
  int hh[IA], ww[IA], po[IA];
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    hh[i] = ap[i] * a.stride + roff;
    ww[i] = aq[i] * a.stride + soff;
    po[i] = (an[i] * a.H + hh[i]) * WC + ww[i] * a.C + ci;
  }
  const int Qs = a.Q * a.stride, Ps = a.P * a.stride;
  const int w_lim = Qs + soff, h_lim = Ps + roff;
  const int d_w = dq * a.stride, d_h = dp * a.stride;
  const int d_po = d_h * WC + d_w * a.C;               // plain step
  const int wrap_q = a.stride * WC - Qs * a.C;         // q wrapped: next input row band
  const int wrap_p = HWC - Ps * WC;                     // p wrapped: next image

  // one generic patch piece i of a stage (slot st): load, then advance the lane's pixel state by
  // one 64-pixel step (shared by issue() and the interleaved issue_piece())
  auto a_piece = [&](char* st, int slot, int i, bool full) {
    const int r0 = RIA * (wave + 4 * i);
    // (bitwise, not short-circuit: one select per piece instead of exec-mask branches)
    const bool ok = kvalid & (full | (am[i] < mend)) & ((unsigned)hh[i] < (unsigned)a.H) &
                    ((unsigned)ww[i] < (unsigned)a.W);
    const bf16_t* const pa = xg + (uint32_t)po[i];
    const void* src = ok ? (const void*)pa : zero;
    if constexpr (PRO) {
      const uint32_t bit = 1u << (slot * IA + i);
      okm = ok ? (okm | bit) : (okm & ~bit);
    }
    __builtin_amdgcn_global_load_lds((wg_gbl_void*)src, (wg_lds_void*)(st + r0 * WA), 16, 0, 0);
    am[i] += BP;
    ww[i] += d_w;
    hh[i] += d_h;
    po[i] += d_po;
    const bool wq = ww[i] >= w_lim;
    ww[i] = wq ? ww[i] - Qs : ww[i];
    hh[i] = wq ? hh[i] + a.stride : hh[i];
    po[i] += wq ? wrap_q : 0;
    while (hh[i] >= h_lim) {
      hh[i] -= Ps;
      po[i] += wrap_p;
    }
  };

  auto issue = [&](int slot, int mstep) {
    char* st = smem + slot * STAGE;
    const bool full = mstep + BP <= mend;  // wave-uniform: no piece of this stage is past the split
    if constexpr (LIN) {
      const bf16_t* __restrict__ xs = xg + (size_t)mstep * a.C;
      if (full && a_full) {
#pragma unroll
        for (int i = 0; i < IA; ++i)
          __builtin_amdgcn_global_load_lds((wg_gbl_void*)(xs + offA[i]), (wg_lds_void*)(st + RIA * (wave + 4 * i) * WA),
                                           16, 0, 0);
        if constexpr (PRO) okm |= ((1u << IA) - 1u) << (slot * IA);
      } else {
#pragma unroll
        for (int i = 0; i < IA; ++i) {
          const bool ok = kvalid && mstep + RIA * (wave + 4 * i) + arow < mend;
          if constexpr (PRO) {
            const uint32_t bit = 1u << (slot * IA + i);
            okm = ok ? (okm | bit) : (okm & ~bit);
          }
          __builtin_amdgcn_global_load_lds((wg_gbl_void*)(ok ? (const void*)(xs + offA[i]) : zero),
                                           (wg_lds_void*)(st + RIA * (wave + 4 * i) * WA), 16, 0, 0);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < (LIN ? 0 : IA); ++i) a_piece(st, slot, i, full);
    const bf16_t* __restrict__ ds = dy0 + (size_t)mstep * a.K;
    if (full && b_full) {
#pragma unroll
      for (int i = 0; i < IB; ++i)
        __builtin_amdgcn_global_load_lds((wg_gbl_void*)(ds + offB[i]), (wg_lds_void*)(st + A_BYTES + RIB * (wave + 4 * i) * WB),
                                         16, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < IB; ++i) {
        const int r0 = RIB * (wave + 4 * i);
        const bool ok = cvalid && mstep + r0 + brow < mend;
        __builtin_amdgcn_global_load_lds((wg_gbl_void*)(ok ? (const void*)(ds + offB[i]) : zero),
                                         (wg_lds_void*)(st + A_BYTES + r0 * WB), 16, 0, 0);
      }
    }
  };

  // one piece of issue(): g < IA: patch piece g (and its pixel-state advance); then the dY pieces
  auto issue_piece = [&](int slot, int mstep, int gp) {
    char* st = smem + slot * STAGE;
    if (gp < IA) {
      a_piece(st, slot, gp, false);
      return;
    }
    const int i = gp - IA;
    const int r0 = RIB * (wave + 4 * i);
    const int m = mstep + r0 + brow;
    const bool ok = cvalid && m < mend;
    __builtin_amdgcn_global_load_lds((wg_gbl_void*)(ok ? (const void*)(dyg + (uint32_t)__mul24(m, a.K)) : zero),
                                     (wg_lds_void*)(st + A_BYTES + r0 * WB), 16, 0, 0);
  };


  f32x4_t acc[MI][MJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < MJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int T = (mend > mbeg) ? (mend - mbeg + BP - 1) / BP : 0;
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int wk = wave & 1, wc = wave >> 1;
  const uint32_t lds_base = (uint32_t)reinterpret_cast<uintptr_t>(smem);  // LDS offset of the image
  // Fragment addresses: swz_off(32ks + 4hi + 8g + q4, col) = swz_off(8g + q4, col) + (32ks + 4hi) * W,
  // because the row swizzle only looks at row bits 0,1,3 (unchanged by +4 and +32): the
  // k-slice / half part is an immediate offset of the read.
  uint32_t a_lane[MI], b_lane[MJ];
#pragma unroll
  for (int i = 0; i < MI; ++i) a_lane[i] = (uint32_t)swz_off<WA>(8 * g + q4, wk * WKK + 16 * i + 4 * p4);
#pragma unroll
  for (int j = 0; j < MJ; ++j) b_lane[j] = (uint32_t)swz_off<WB>(8 * g + q4, wc * WCO + 16 * j + 4 * p4);

#pragma unroll
  for (int s = 0; s < D; ++s)
    if (s < T) issue(s, mbeg + s * BP);

  for (int t = 0; t < T; ++t) {
    if (t + D - 1 < T) wg_wait_vmcnt<G * (D - 1)>();
    else wg_wait_vmcnt<0>();
    if constexpr (PRO) {
      const int slot = t % NS;
      char* sw = smem + slot * STAGE;
      uint32_t pa[IA];
      u32x4_t v[IA];
#pragma unroll
      for (int i = 0; i < IA; ++i) {
        pa[i] = lds_addr(sw + RIA * (wave + 4 * i) * WA + lane * 16);
        v[i] = lds_read16(pa[i]);
      }
      lds_wait_all<IA>(v);
      lds_bn_relu_store<IA, true>(pa, v, (okm >> (slot * IA)) & ((1u << IA) - 1u), psc2, psh2);
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (!IL && t + D < T) issue((t + D) % NS, mbeg + (t + D) * BP);
    const bool more = IL && t + D < T;
    const int nslot = (t + D) % NS, nstep = mbeg + (t + D) * BP;
    // Transposed fragment reads in inline asm: hipcc treats its ds_read_tr intrinsic as
    // possibly aliasing the LDS-DMA just issued and would wait vmcnt(0) (serialising the
    // pipeline); the asm reads are ordered by hand instead: both k-slices' reads are issued,
    // lgkmcnt(16) retires the first 16 (LDS returns in order), lgkmcnt(0) the rest.
    const uint32_t cur = lds_base + (uint32_t)((t % NS) * STAGE);
    uint32_t ba[MI], bb[MJ];
#pragma unroll
    for (int i = 0; i < MI; ++i) ba[i] = cur + a_lane[i];
#pragma unroll
    for (int j = 0; j < MJ; ++j) bb[j] = cur + b_lane[j];
    s16x4v fa[KS][MI][2], fb[KS][MJ][2];
    static_for<0, KS>([&](auto KSI) {
      constexpr int ks = decltype(KSI)::value;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        fa[ks][i][0] = tr_read_asm<(32 * ks) * WA>(ba[i]);
        fa[ks][i][1] = tr_read_asm<(32 * ks + 4) * WA>(ba[i]);
      }
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        fb[ks][j][0] = tr_read_asm<A_BYTES + (32 * ks) * WB>(bb[j]);
        fb[ks][j][1] = tr_read_asm<A_BYTES + (32 * ks + 4) * WB>(bb[j]);
      }
    });
    constexpr int Q = KS * MI * MJ;
    constexpr int STEP = Q / (G + 1) > 0 ? Q / (G + 1) : 1;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) lgkm_fence<(2 * (MI + MJ) > 15 ? 15 : 2 * (MI + MJ))>(fa[ks], fb[ks]);  // 4-bit counter
      else lgkm_fence<0>(fa[ks], fb[ks]);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < MJ; ++j) {
          const bf16x8_t af = __builtin_bit_cast(
              bf16x8_t, __builtin_shufflevector(fa[ks][i][0], fa[ks][i][1], 0, 1, 2, 3, 4, 5, 6, 7));
          const bf16x8_t bfr = __builtin_bit_cast(
              bf16x8_t, __builtin_shufflevector(fb[ks][j][0], fb[ks][j][1], 0, 1, 2, 3, 4, 5, 6, 7));
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[i][j], 0, 0, 0);
          if constexpr (IL) {
            const int q = (ks * MI + i) * MJ + j + 1;
            if (q % STEP == 0 && q / STEP <= G && more) {
              __builtin_amdgcn_sched_barrier(0);
              issue_piece(nslot, nstep, q / STEP - 1);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
        }
    }
    if constexpr (IL) {
      if (Q / STEP < G && more) {
#pragma unroll
        for (int gp = Q / STEP; gp < G; ++gp) issue_piece(nslot, nstep, gp);
      }
    }
    asm volatile("" ::: "memory");
  }

#ifdef DRN_CONV_TRACE
  unsigned long long t_loop = 0;
  if (trace != nullptr) t_loop = wg_realtime();
#endif
  wgrad_store<MI, MJ>(a, acc, split, c0 + wc * WCO, k0 + wk * WKK, Ktot, lane);
#ifdef DRN_CONV_TRACE
  if (trace != nullptr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
      const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);
      unsigned long long* r = trace + 4 * (size_t)(blockIdx.x + blockIdx.y * gridDim.x);
      r[0] = t_start;
      r[1] = t_loop;
      r[2] = wg_realtime();
      r[3] = ((unsigned long long)xcc << 32) | hw;
    }
  }
#endif
}

// ---------------------------------------------------------------------------------------
// Packed-stem weight gradient from an LDS input halo (the ImageNet 7x7/2 stem in the layout of
// csrc/kernels/stem.hip: xp[n][h][W + 2][4], filter rows of 8 taps x 4 channels = 32 k).
// The generic kernel's im2col loader fetches every input piece ~4x per k-tile: a 64-pixel stage
// is 64 patch rows of 256 B, and adjacent output pixels' 64-byte row segments overlap by 48 B;
// the kernel is bound by those loads (its loads-only variant runs as long as the kernel itself,
// profiles/r6_experiments.md). Here a stage is one half output row (QH = Q / 2 <= 61 pixels,
// padded to 64 MFMA rows): the tile's 4 filter rows of input are loaded ONCE into LDS, 128
// columns x 8 B = 1 KB per row (one LDS-DMA instruction per row, out-of-image pieces from the zero
// page), and the transposed fragment reads address the virtual patch image directly: patch
// (pixel i, k = 32 r + 4 s + c) sits at byte r * 1024 + 16 i + 2 (k mod 32) -- adjacent pixels'
// patch rows overlap in LDS instead of being fetched again (4 KB of input per stage instead of
// 16 KB). dY: the stage's QH rows of 128 B (64 channels), loaded and swizzled as by the generic
// kernel; rows >= QH read the zero page (their patch rows are finite input data, so their
// products are exact zeros). Grid, splits, slabs and the store are the generic kernel's (2 k-tiles
// of 128 x channel tiles of 64, split-K over pixels); a split takes the half rows whose first
// pixel lies in its pixel range, so every pixel is reduced exactly once.
// ---------------------------------------------------------------------------------------
template <int NS>
__global__ __launch_bounds__(256) void stem_wgrad_halo_kernel(DrnConvWgradArgs a, const void* __restrict__ zero) {
  constexpr int BKK = 128, BCO = 64, BP = 64;
  constexpr int WB = BCO * 2;                      // dY image row bytes
  constexpr int A_BYTES = 4 * 1024;                // 4 filter rows x 128 input columns x 8 B
  constexpr int STAGE = A_BYTES + BP * WB;
  constexpr int LPB = WB / 16, RIB = 64 / LPB;     // lanes per dY row, dY rows per wave-instruction
  constexpr int IB = BP / RIB / 4;                 // dY instructions per wave per stage
  constexpr int G = 1 + IB;                        // LDS-DMA instructions per wave per stage
  constexpr int D = NS - 1;
  constexpr int WKK = BKK / 2, WCO = BCO / 2;
  constexpr int MI = WKK / 16, MJ = WCO / 16;
  static_assert(NS >= 2 && IB >= 1, "geometry");
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Ktot = a.R * a.S * a.C;
  const int M = a.N * a.P * a.Q;
  const int QH = a.Q / 2;
  const int nkt = (Ktot + BKK - 1) / BKK;
  const int ntile = gridDim.x;
  const int lin = xcd_remap(blockIdx.x + blockIdx.y * ntile, ntile * gridDim.y);
  const int tile = lin % ntile, split = lin / ntile;
  const int kt = tile % nkt, ct = tile / nkt;
  const int k0 = kt * BKK, c0 = ct * BCO;
  const int mbeg = split * a.pix_per_split;
  const int mend = min(M, mbeg + a.pix_per_split);
  const int hbeg = (mbeg + QH - 1) / QH, hend = (mend + QH - 1) / QH;
  const int T = hend > hbeg ? hend - hbeg : 0;
  const bf16_t* __restrict__ xg = reinterpret_cast<const bf16_t*>(a.x);
  const bf16_t* __restrict__ dyg = reinterpret_cast<const bf16_t*>(a.dy);
  // A (input halo): wave w loads filter row r = k0 / 32 + w, lane l the piece at input column
  // 2 q0 - pad_w + 2 l (two pixels x 4 channels)
  const int fr = k0 / 32 + wave;
  // B (dY): as the generic kernel's loader (logical chunk of the lane, swizzle of its rows)
  const int brow = lane / LPB;
  int blc;
  {
    const int pc = lane % LPB;
    blc = 2 * ((pc >> 1) ^ slot_swz<WB>(RIB * wave + brow)) + (pc & 1);
  }
  const int dc = c0 + blc * 8;
  const bool cvalid = dc < a.K;

  auto issue = [&](int slot, int hr) {
    char* st = smem + slot * STAGE;
    const int np = hr >> 1, hf = hr & 1;
    const int n = np / a.P, p = np - n * a.P;
    const int q0 = hf * QH;
    const int h = p * a.stride - a.pad_h + fr;
    const int col = q0 * a.stride - a.pad_w + 2 * lane;
    const bool ok = fr < a.R && (unsigned)h < (unsigned)a.H && col >= 0 && col + 1 < a.W;
    const bf16_t* src = xg + ((size_t)(n * a.H + h) * a.W + col) * a.C;
    __builtin_amdgcn_global_load_lds((wg_gbl_void*)(ok ? (const void*)src : zero), (wg_lds_void*)(st + wave * 1024),
                                     16, 0, 0);
    const int m0 = np * a.Q + q0;
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const int r0 = RIB * (wave + 4 * i);
      const bool okb = cvalid && r0 + brow < QH && m0 + r0 + brow < M;
      const bf16_t* bs = dyg + (size_t)(m0 + r0 + brow) * a.K + dc;
      __builtin_amdgcn_global_load_lds((wg_gbl_void*)(okb ? (const void*)bs : zero),
                                       (wg_lds_void*)(st + A_BYTES + r0 * WB), 16, 0, 0);
    }
  };

  f32x4_t acc[MI][MJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < MJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int wk = wave & 1, wc = wave >> 1;
  const uint32_t lds_base = (uint32_t)reinterpret_cast<uintptr_t>(smem);
  // fragment addresses: A (virtual patch image) row = pixel 8g + q4 (+4, +32 ks: immediates),
  // columns k = wk * WKK + 16 i + 4 p4 .. +3 (inside one 32-k filter row)
  uint32_t a_lane[MI], b_lane[MJ];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int kl = wk * WKK + 16 * i + 4 * p4;
    a_lane[i] = (uint32_t)((kl >> 5) * 1024 + 2 * (kl & 31) + 16 * (8 * g + q4));
  }
#pragma unroll
  for (int j = 0; j < MJ; ++j) b_lane[j] = (uint32_t)swz_off<WB>(8 * g + q4, wc * WCO + 16 * j + 4 * p4);

#pragma unroll
  for (int s = 0; s < D; ++s)
    if (s < T) issue(s, hbeg + s);

  for (int t = 0; t < T; ++t) {
    if (t + D - 1 < T) wg_wait_vmcnt<G * (D - 1)>();
    else wg_wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + D < T) issue((t + D) % NS, hbeg + t + D);
    const uint32_t cur = lds_base + (uint32_t)((t % NS) * STAGE);
    uint32_t ba[MI], bb[MJ];
#pragma unroll
    for (int i = 0; i < MI; ++i) ba[i] = cur + a_lane[i];
#pragma unroll
    for (int j = 0; j < MJ; ++j) bb[j] = cur + b_lane[j];
    s16x4v fa[2][MI][2], fb[2][MJ][2];
    static_for<0, 2>([&](auto KSI) {
      constexpr int ks = decltype(KSI)::value;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        fa[ks][i][0] = tr_read_asm<16 * (32 * ks)>(ba[i]);
        fa[ks][i][1] = tr_read_asm<16 * (32 * ks + 4)>(ba[i]);
      }
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        fb[ks][j][0] = tr_read_asm<A_BYTES + (32 * ks) * WB>(bb[j]);
        fb[ks][j][1] = tr_read_asm<A_BYTES + (32 * ks + 4) * WB>(bb[j]);
      }
    });
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (ks == 0) lgkm_fence<2 * (MI + MJ)>(fa[0], fb[0]);
      else lgkm_fence<0>(fa[1], fb[1]);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < MJ; ++j) {
          const bf16x8_t af = __builtin_bit_cast(
              bf16x8_t, __builtin_shufflevector(fa[ks][i][0], fa[ks][i][1], 0, 1, 2, 3, 4, 5, 6, 7));
          const bf16x8_t bfr = __builtin_bit_cast(
              bf16x8_t, __builtin_shufflevector(fb[ks][j][0], fb[ks][j][1], 0, 1, 2, 3, 4, 5, 6, 7));
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[i][j], 0, 0, 0);
        }
    }
    asm volatile("" ::: "memory");
  }
  wgrad_store<MI, MJ>(a, acc, split, c0 + wc * WCO, k0 + wk * WKK, Ktot, lane);
}

template <int NS>
static int launch_stem_wgrad_halo(DrnConvWgradArgs* a, const void* zero, hipStream_t s) {
  constexpr int LDS = NS * (4 * 1024 + 64 * 64 * 2);
  const int Ktot = a->R * a->S * a->C;
  drn::launch(stem_wgrad_halo_kernel<NS>, dim3(((Ktot + 127) / 128) * ((a->K + 63) / 64), a->splits), dim3(256), LDS,
              s, *a, zero);
  return (int)hipGetLastError();
}

// the packed-stem geometry the halo kernel covers (host check)
static bool stem_halo_ok(const DrnConvWgradArgs* a, const void* zero) {
  const int QH = a->Q / 2;
  return zero != nullptr && a->C == 4 && a->S == 8 && a->R <= 8 && a->stride == 2 && a->pad_w % 2 == 0 &&
         a->Q % 2 == 0 && QH >= 1 && 2 * QH + a->S - 2 <= 128 && a->K % 64 == 0 && a->in_scale == nullptr &&
         a->splits >= 1 && a->pix_per_split % 64 == 0;
}

template <int BKK, int BCO, int NS, int BP, bool PRO, bool IL = false, bool LIN = false>
static int launch_wgrad_glds_p(DrnConvWgradArgs* a, const void* zero, hipStream_t s) {
  constexpr int LDS = NS * (BP * BKK * 2 + BP * BCO * 2);
  static bool attr_set = false;
  auto kern = conv_wgrad_glds_kernel<BKK, BCO, NS, BP, PRO, IL, LIN>;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr_set = true;
  }
  const int Ktot = a->R * a->S * a->C;
  const int nkt = (Ktot + BKK - 1) / BKK;
  const int nct = (a->K + BCO - 1) / BCO;
  drn::launch(kern, dim3(nkt * nct, a->splits), dim3(256), LDS, s, *a, zero);
  return (int)hipGetLastError();
}

template <int BKK, int BCO, int NS, int BP, bool IL>
static int launch_wgrad_glds_ok(DrnConvWgradArgs* a, const void* zero, hipStream_t s);

template <int BKK, int BCO, int NS, int BP = 64, bool IL = false>
static int launch_wgrad_glds(DrnConvWgradArgs* a, const void* zero, hipStream_t s) {
  // (every wave issues >= 1 dY LDS-DMA instruction per stage: BP rows of 2*BCO bytes)
  if constexpr (BP * BCO * 2 < 4 * 1024) {
    return (int)hipErrorInvalidValue;
  } else {
    return launch_wgrad_glds_ok<BKK, BCO, NS, BP, IL>(a, zero, s);
  }
}

template <int BKK, int BCO, int NS, int BP, bool IL>
static int launch_wgrad_glds_ok(DrnConvWgradArgs* a, const void* zero, hipStream_t s) {
  const bool lin = !IL && a->R == 1 && a->S == 1 && a->stride == 1 && a->pad_h == 0 && a->pad_w == 0 &&
                   a->C % 8 == 0;
  if constexpr (!IL) {
    if (lin) {
      if (a->in_scale != nullptr) return launch_wgrad_glds_p<BKK, BCO, NS, BP, true, false, true>(a, zero, s);
      return launch_wgrad_glds_p<BKK, BCO, NS, BP, false, false, true>(a, zero, s);
    }
  }
  if (a->in_scale != nullptr) return launch_wgrad_glds_p<BKK, BCO, NS, BP, true, IL>(a, zero, s);
  return launch_wgrad_glds_p<BKK, BCO, NS, BP, false, IL>(a, zero, s);
}

template <int NS, int BP, bool IL = false>
static int dispatch_wgrad_tile(DrnConvWgradArgs* a, const void* zero, hipStream_t s) {
  const int Ktot = a->R * a->S * a->C;
  const bool wide_k = Ktot > 64;
  const bool wide_c = a->K > 64;
  if (a->K <= 32) {
    // narrow output (CIFAR stages 1-2: 16 / 32 filters, reference resnet_model_official.py:
    // 255-266): 32-channel dY tiles (a 64-wide tile wasted 50-75 % of the MFMA work) and the
    // k tile that pads R*S*C least (144 -> 192 instead of 256, 288 -> 320 instead of 384)
    const bool k128 = wide_k && ((Ktot + 127) / 128) * 128 <= ((Ktot + 63) / 64) * 64;
    if (k128) return launch_wgrad_glds<128, 32, NS, BP, IL>(a, zero, s);
    return launch_wgrad_glds<64, 32, NS, BP, IL>(a, zero, s);
  }
  if (wide_k && wide_c) return launch_wgrad_glds<128, 128, NS, BP, IL>(a, zero, s);
  if (wide_k) return launch_wgrad_glds<128, 64, NS, BP, IL>(a, zero, s);
  if (wide_c) return launch_wgrad_glds<64, 128, NS, BP, IL>(a, zero, s);
  return launch_wgrad_glds<64, 64, NS, BP, IL>(a, zero, s);
}

// pipeline id: 2 / 3 = 2 / 3 stages of 64 pixels; 4 / 5 / 6 = 2 / 3 / 4 stages of 32 pixels
// (half the LDS per stage: more resident workgroups per CU); 7 / 8 = 2 / 3 stages of 64 pixels
// with the interleaved LDS-DMA issue (IL)
static int dispatch_wgrad_glds(DrnConvWgradArgs* a, const void* zero, int ns, hipStream_t s) {
  switch (ns) {
    case 3: return dispatch_wgrad_tile<3, 64>(a, zero, s);
    case 4: return dispatch_wgrad_tile<2, 32>(a, zero, s);
    case 5: return dispatch_wgrad_tile<3, 32>(a, zero, s);
    case 6: return dispatch_wgrad_tile<4, 32>(a, zero, s);
    case 7: return dispatch_wgrad_tile<2, 64, true>(a, zero, s);
    case 8: return dispatch_wgrad_tile<3, 64, true>(a, zero, s);
    default: return dispatch_wgrad_tile<2, 64>(a, zero, s);
  }
}

// out[i] (+)= scale * sum_k ws[k][i]: block = COLS float4 columns x (256/COLS) split-groups;
// every thread keeps 4 independent loads in flight (the split loop is the latency chain for
// small tensors with many splits), then the groups are combined by a fixed-order LDS tree
// (deterministic). Small outputs with many splits (early-stage layers: 1-9K float4 x 100-500
// splits) take COLS = 4/16 so the grid still spreads over the CUs instead of a few blocks
// walking hundreds of splits each.
__device__ __forceinline__ void f4_add(float4& s, const float4 a) {
  s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
}

template <int COLS>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, float* __restrict__ out,
                                                            int n4, int splits, size_t stride4, float scale,
                                                            int accumulate) {
  constexpr int G = 256 / COLS;
  __shared__ float4 red[G][COLS];
  const int tx = threadIdx.x % COLS, ty = threadIdx.x / COLS;
  const int i = blockIdx.x * COLS + tx;
  float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0, s2 = s0, s3 = s0;
  if (i < n4) {
    const float4* p = reinterpret_cast<const float4*>(ws) + i;
    int k = ty;
    for (; k + 3 * G < splits; k += 4 * G) {
      const float4 a = p[(size_t)k * stride4], b = p[(size_t)(k + G) * stride4];
      const float4 c = p[(size_t)(k + 2 * G) * stride4], d = p[(size_t)(k + 3 * G) * stride4];
      f4_add(s0, a);
      f4_add(s1, b);
      f4_add(s2, c);
      f4_add(s3, d);
    }
    for (; k < splits; k += G) f4_add(s0, p[(size_t)k * stride4]);
  }
  float4 t;
  t.x = (s0.x + s1.x) + (s2.x + s3.x);
  t.y = (s0.y + s1.y) + (s2.y + s3.y);
  t.z = (s0.z + s1.z) + (s2.z + s3.z);
  t.w = (s0.w + s1.w) + (s2.w + s3.w);
  red[ty][tx] = t;
  __syncthreads();
#pragma unroll
  for (int w = G / 2; w >= 1; w >>= 1) {
    if (ty < w) {
      float4 u = red[ty][tx];
      f4_add(u, red[ty + w][tx]);
      red[ty][tx] = u;
    }
    __syncthreads();
  }
  if (ty == 0 && i < n4) {
    float4 r = red[0][tx];
    r.x *= scale; r.y *= scale; r.z *= scale; r.w *= scale;
    if (accumulate) {
      const float4 o = reinterpret_cast<float4*>(out)[i];
      r.x += o.x; r.y += o.y; r.z += o.z; r.w += o.w;
    }
    reinterpret_cast<float4*>(out)[i] = r;
  }
}

}  // namespace drn

#ifdef DRN_CONV_TRACE
// diagnostics: per-workgroup timeline buffer for the LDS-DMA weight-gradient kernel
DRN_API int drn_wgrad_trace_set(unsigned long long* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(drn::g_wgrad_trace), &buf, sizeof(buf));
}
#endif

// Block-tile shape the dispatcher picks (host mirror used to size the split-K grid).
DRN_API int drn_wgrad_tiles(int Ktot, int K) {
  int bkk = Ktot > 64 ? 128 : 64, bco = K > 64 ? 128 : 64;
  if (K <= 32) {  // (dispatch_wgrad_tile's narrow-output tiles)
    bco = 32;
    bkk = (Ktot > 64 && ((Ktot + 127) / 128) * 128 <= ((Ktot + 63) / 64) * 64) ? 128 : 64;
  }
  return ((Ktot + bkk - 1) / bkk) * ((K + bco - 1) / bco);
}

DRN_API int drn_conv_wgrad(DrnConvWgradArgs* a, hipStream_t s) {
  if ((a->C % 8) != 0 || (a->K % 8) != 0 || a->splits < 1 || (a->pix_per_split % 64) != 0)
    return (int)hipErrorInvalidValue;
  return a->in_scale != nullptr ? drn::dispatch_wgrad<true>(a, s) : drn::dispatch_wgrad<false>(a, s);
}

// LDS-DMA wgrad; ns = pipeline (dispatch_wgrad_glds), 0 = register-staged kernel, 9 / 10 = the
// packed stem's input-halo kernel with 3 / 4 stages.
DRN_API int drn_conv_wgrad2(DrnConvWgradArgs* a, const void* zero, int ns, hipStream_t s) {
  // C == 4: the packed stem (stem.hip) -- every 16-byte k piece is a tap pair x 4 channels, so the
  // tap count must be even (S padded to 8); LDS-DMA kernels, no fused prologue
  const bool packed = a->C == 4 && a->S % 2 == 0 && a->in_scale == nullptr && zero != nullptr && ns != 0;
  if (((a->C % 8) != 0 && !packed) || (a->K % 8) != 0 || a->splits < 1 || (a->pix_per_split % 64) != 0)
    return (int)hipErrorInvalidValue;
  if (ns == 9 || ns == 10) {  // packed-stem input halo (3 / 4 stages)
    if (!drn::stem_halo_ok(a, zero)) return (int)hipErrorInvalidValue;
    return ns == 9 ? drn::launch_stem_wgrad_halo<3>(a, zero, s) : drn::launch_stem_wgrad_halo<4>(a, zero, s);
  }
  // (the LDS-DMA kernels' fused BN prologue always applies the ReLU: pre-activation v2)
  if (zero == nullptr || ns == 0 || (a->in_scale != nullptr && a->relu_in == 0)) return drn_conv_wgrad(a, s);
  return drn::dispatch_wgrad_glds(a, zero, ns, s);
}

// out[i] (+)= scale * sum_k ws[k][i]  over n floats (n % 4 == 0), deterministic order.
DRN_API int drn_splitk_reduce(const float* ws, float* out, int64_t n, int splits, float scale, int accumulate,
                              hipStream_t s) {
  if (n % 4) return (int)hipErrorInvalidValue;
  const int n4 = (int)(n / 4);
  // widest column tile that still gives >= 512 blocks (2 per CU), or whose split-groups
  // would otherwise idle (splits <= groups)
  const int cols = (n4 >= 512 * 64 || splits <= 8) ? 64 : (n4 >= 512 * 16 || splits <= 32) ? 16 : 4;
  const int blocks = n4 > 0 ? (n4 + cols - 1) / cols : 1;
  if (cols == 64)
    drn::launch(drn::splitk_reduce_kernel<64>, dim3(blocks), dim3(256), 0, s, ws, out, n4, splits, (size_t)n4,
                       scale, accumulate);
  else if (cols == 16)
    drn::launch(drn::splitk_reduce_kernel<16>, dim3(blocks), dim3(256), 0, s, ws, out, n4, splits, (size_t)n4,
                       scale, accumulate);
  else
    drn::launch(drn::splitk_reduce_kernel<4>, dim3(blocks), dim3(256), 0, s, ws, out, n4, splits, (size_t)n4,
                       scale, accumulate);
  return (int)hipGetLastError();
}
