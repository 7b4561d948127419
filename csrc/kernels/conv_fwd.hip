// conv_fwd.hip — NHWC bf16 implicit-GEMM convolution on CDNA4 MFMA (gfx950).
//
// Replaces the cuDNN/MKL-DNN Conv2D the reference graph runs for every
// `conv2d_fixed_padding` (reference resnet_model_official.py:80-91) and its backprop-input.
//
// GEMM view (forward):   D[cout][pixel] = sum_k  W[cout][k] * Patch[pixel][k],
//   k = (r, s, ci) over R*S*C (KRSC weights make k contiguous; NHWC makes ci contiguous).
// MFMA operand A = weights (rows = output channels), operand B = im2col patches gathered on
// the fly (cols = output pixels), so each lane's 4 accumulator registers are 4 consecutive
// output channels of one pixel (one 16-byte fp32 chunk for the LDS-staged epilogue).
//
// Structure: 256 threads = 4 waves; block tile BP pixels x BC channels x BK reduction,
// register-staged double-buffered LDS (loads for step t+1 in flight while step t computes,
// one barrier per step). LDS image is chunk-major [BK/8][rows][8 x bf16]: the MFMA fragment
// reads (ds_read_b128, 16 rows x 16 B per 16-lane group) and the 8-lane ds_write_b128 groups
// are both bank-conflict free (checked against the gfx950 lane-group tables).
//
// Fusions: (1) optional BN-apply+ReLU of the INPUT in the load prologue (pre-activation v2:
// every conv consumes relu(bn(x)), reference resnet_model_official.py:113-119), zero padding
// stays zero; (2) optional residual add in the epilogue (block output `inputs + shortcut`,
// :130/:175); (3) optional per-channel partial sum / sum-of-squares of the stored output for
// the NEXT BatchNorm's batch statistics.
#include "drn_common.h"
#include "drn_conv.h"

namespace drn {

template <int BP, int BC, int BK, int WP, int WC, bool PRO, bool DIL2>
__global__ __launch_bounds__(256, 2) void conv_fwd_kernel(DrnConvFwdArgs a) {
  constexpr int CH = BK / 8;                  // 16-byte chunks per row per stage
  constexpr int RPG = 64 / CH;                // rows per wave-instruction group
  constexpr int NB = (BP * CH) / 256;         // pixel-operand vectors per thread
  constexpr int NA = (BC * CH + 255) / 256;   // weight-operand vectors per thread
  constexpr int WAVES_P = BP / WP;
  constexpr int WAVES_C = BC / WC;
  static_assert(WAVES_P * WAVES_C == 4, "4 waves per block");
  static_assert(NB >= 1 && (BP * CH) % 256 == 0, "pixel tile must be covered by 256 threads");
  constexpr int MI = WC / 16;                 // mfma tiles along channels
  constexpr int MJ = WP / 16;                 // mfma tiles along pixels
  constexpr int A_BYTES = BC * BK * 2;
  constexpr int STAGE = A_BYTES + BP * BK * 2;

  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int M = a.N * a.P * a.Q;
  const int Ktot = a.R * a.S * a.C;
  const int ntc = (a.K + BC - 1) / BC;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tc = bid % ntc;
  const int tp = bid / ntc;
  const int m0 = tp * BP;
  const int c0 = tc * BC;

  // ---------------- loader geometry ----------------
  const int chunk = (lane >> 3) % CH;
  const int rsub = (lane & 7) + 8 * ((lane >> 3) / CH);

  int b_base[NB], b_h[NB], b_w[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int row = rsub + RPG * (wave + 4 * i);
    const int m = m0 + row;
    if (m < M) {
      const int pq = a.P * a.Q;
      const int n = m / pq;
      const int rem = m - n * pq;
      const int p = rem / a.Q;
      const int q = rem - p * a.Q;
      b_base[i] = n * a.H * a.W * a.C;
      b_h[i] = p * a.stride - a.pad_h;
      b_w[i] = q * a.stride - a.pad_w;
    } else {
      b_base[i] = 0;
      b_h[i] = -(1 << 28);  // forces the bounds test to fail
      b_w[i] = -(1 << 28);
    }
  }
  // this thread's chunk position in (r, s, ci); advanced by BK each step
  int ci, rr, ss;
  {
    const int kk = chunk * 8;
    const int tap = kk / a.C;
    ci = kk - tap * a.C;
    rr = tap / a.S;
    ss = tap - rr * a.S;
  }
  int kw = chunk * 8;  // weight-operand k offset of this thread's chunk

  uint4 rb[NB];
  uint4 ra[NA];
  unsigned bvalid = 0;

  auto load_stage = [&]() {
    bvalid = 0;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (rr < a.R) {
        int h = b_h[i] + rr;
        int w = b_w[i] + ss;
        bool ok;
        if constexpr (DIL2) {
          ok = h >= 0 && w >= 0 && ((h | w) & 1) == 0;
          h >>= 1;
          w >>= 1;
          ok = ok && h < a.H && w < a.W;
        } else {
          ok = h >= 0 && w >= 0 && h < a.H && w < a.W;
        }
        if (ok) {
          v = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(a.x) + b_base[i] +
                                              (h * a.W + w) * a.C + ci);
          bvalid |= 1u << i;
        }
      }
      rb[i] = v;
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int row = rsub + RPG * (wave + 4 * i);
      const int c = c0 + row;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (row < BC && c < a.K && kw < Ktot)
        v = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(a.w) + (size_t)c * Ktot + kw);
      ra[i] = v;
    }
  };

  auto advance = [&]() {
    kw += BK;
    ci += BK;
    while (ci >= a.C) {
      ci -= a.C;
      if (++ss == a.S) {
        ss = 0;
        ++rr;
      }
    }
  };

  auto store_stage = [&](char* st, int ci_of_stage) {
    if constexpr (PRO) {
      if (bvalid) {
        float sc[8], sh[8];
        const float4* s4 = reinterpret_cast<const float4*>(a.in_scale + ci_of_stage);
        const float4* h4 = reinterpret_cast<const float4*>(a.in_shift + ci_of_stage);
        float4 t0 = s4[0], t1 = s4[1], u0 = h4[0], u1 = h4[1];
        sc[0] = t0.x; sc[1] = t0.y; sc[2] = t0.z; sc[3] = t0.w;
        sc[4] = t1.x; sc[5] = t1.y; sc[6] = t1.z; sc[7] = t1.w;
        sh[0] = u0.x; sh[1] = u0.y; sh[2] = u0.z; sh[3] = u0.w;
        sh[4] = u1.x; sh[5] = u1.y; sh[6] = u1.z; sh[7] = u1.w;
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          if (bvalid & (1u << i)) {
            float f[8];
            unpack8(rb[i], f);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              f[j] = f[j] * sc[j] + sh[j];
              if (a.relu_in) f[j] = fmaxf(f[j], 0.f);
            }
            rb[i] = pack8(f);
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int row = rsub + RPG * (wave + 4 * i);
      if (row < BC) *reinterpret_cast<uint4*>(st + (chunk * BC + row) * 16) = ra[i];
    }
    char* sb = st + A_BYTES;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int row = rsub + RPG * (wave + 4 * i);
      *reinterpret_cast<uint4*>(sb + (chunk * BP + row) * 16) = rb[i];
    }
  };

  // ---------------- main loop ----------------
  const int wp = wave % WAVES_P;
  const int wc = wave / WAVES_P;
  f32x4_t acc[MI][MJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < MJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int T = (Ktot + BK - 1) / BK;
  int ci_cur = ci;
  load_stage();
  store_stage(smem, ci_cur);
  __syncthreads();

  for (int t = 0; t < T; ++t) {
    char* cur = smem + (t & 1) * STAGE;
    const bool more = (t + 1) < T;
    if (more) {
      advance();
      ci_cur = ci;
      load_stage();
    }
    const char* sA = cur;
    const char* sB = cur + A_BYTES;
#pragma unroll
    for (int kh = 0; kh < BK / 32; ++kh) {
      bf16x8_t af[MI], bfr[MJ];
      const int kc = kh * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < MI; ++i)
        af[i] = *reinterpret_cast<const bf16x8_t*>(sA + (kc * BC + wc * WC + i * 16 + (lane & 15)) * 16);
#pragma unroll
      for (int j = 0; j < MJ; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8_t*>(sB + (kc * BP + wp * WP + j * 16 + (lane & 15)) * 16);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < MJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) store_stage(smem + ((t + 1) & 1) * STAGE, ci_cur);
    __syncthreads();
  }

  // ---------------- epilogue ----------------
  // The fp32 accumulator tile is staged through LDS ([BP][BC] fp32, 16-byte chunks XOR-swizzled
  // by row: conflict-free 8-lane ds_write_b128 groups and 16-lane ds_read_b128 groups), then
  // every lane owns 8 consecutive channels of one pixel: 16-byte residual loads and 16-byte
  // bf16 stores, whole 2*BC-byte pixel rows per wave instruction (fully coalesced).
  constexpr int CF = BC / 4;   // fp32 16-byte chunks per staged row
  constexpr int CHR = BC / 8;  // output 16-byte (8 x bf16) chunks per pixel row
  constexpr int RPI = 256 / CHR;
  constexpr int SWM = CF >= 8 ? 7 : CF - 1;  // swizzle mask stays inside a staged row
  static_assert(BP * BC * 4 <= 2 * STAGE, "epilogue tile must fit the staging LDS");
  float* tile = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int cf = (wc * WC + i * 16) / 4 + (lane >> 4);  // fp32 chunk of these 4 channels
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      const int row = wp * WP + j * 16 + (lane & 15);
      *reinterpret_cast<f32x4_t*>(tile + row * BC + ((cf ^ (row & SWM)) * 4)) = acc[i][j];
    }
  }
  __syncthreads();
  const bool want_stats = a.stats != nullptr;
  bf16_t* __restrict__ y = reinterpret_cast<bf16_t*>(a.y);
  const bf16_t* __restrict__ res = reinterpret_cast<const bf16_t*>(a.residual);
  const int ch = tid % CHR;
  const int c = c0 + ch * 8;
  const bool mapped = a.out_stride != 0;
  const int pq = a.P * a.Q;
  float ssum[8], ssq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) ssum[j] = ssq[j] = 0.f;
#pragma unroll
  for (int it = 0; it < BP / RPI; ++it) {
    const int row = it * RPI + tid / CHR;
    const int m = m0 + row;
    const f32x4_t lo = *reinterpret_cast<const f32x4_t*>(tile + row * BC + (((2 * ch) ^ (row & SWM)) * 4));
    const f32x4_t hi = *reinterpret_cast<const f32x4_t*>(tile + row * BC + (((2 * ch + 1) ^ (row & SWM)) * 4));
    if (m < M && c < a.K) {
      float f[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      size_t off;
      if (mapped) {
        const int n = m / pq;
        const int rem = m - n * pq;
        const int i = rem / a.Q;
        const int j = rem - i * a.Q;
        off = ((size_t)(n * a.out_H + i * a.out_stride + a.out_oh) * a.out_W + j * a.out_stride + a.out_ow) * a.K + c;
      } else {
        off = (size_t)m * a.K + c;
      }
      if (res) {
        float r8[8];
        unpack8(*reinterpret_cast<const uint4*>(res + off), r8);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] += r8[j];
      }
      const uint4 o = pack8(f);
      *reinterpret_cast<uint4*>(y + off) = o;
      if (want_stats) {
        float q8[8];
        unpack8(o, q8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          ssum[j] += q8[j];
          ssq[j] += q8[j] * q8[j];
        }
      }
    }
  }
  if (want_stats) {
    __syncthreads();
    float* red = tile;  // [256][16]
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[tid * 16 + j] = ssum[j];
      red[tid * 16 + 8 + j] = ssq[j];
    }
    __syncthreads();
    if (tid < 2 * BC) {
      const int cl = tid >> 1, which = tid & 1;
      const int chh = cl >> 3, j = cl & 7;
      float s = 0.f;
      for (int t2 = chh; t2 < 256; t2 += CHR) s += red[t2 * 16 + which * 8 + j];
      if (c0 + cl < a.K) atomicAdd(a.stats + (size_t)which * a.K + c0 + cl, s);
    }
  }
}

template <int BP, int BC, int BK, int WP, int WC, bool PRO, bool DIL2>
static int launch_conv_fwd(DrnConvFwdArgs* a, hipStream_t stream) {
  constexpr int STAGE = BC * BK * 2 + BP * BK * 2;
  constexpr int LDS = 2 * STAGE;
  static bool attr_set = false;
  auto kern = conv_fwd_kernel<BP, BC, BK, WP, WC, PRO, DIL2>;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr_set = true;
  }
  const int M = a->N * a->P * a->Q;
  const int tiles_p = (M + BP - 1) / BP;
  const int tiles_c = (a->K + BC - 1) / BC;
  a->tiles_p = tiles_p;
  hipLaunchKernelGGL(kern, dim3(tiles_p * tiles_c), dim3(256), LDS, stream, *a);
  return (int)hipGetLastError();
}

template <bool PRO, bool DIL2>
static int dispatch_conv_fwd(DrnConvFwdArgs* a, hipStream_t s) {
  if (a->K >= 128) return launch_conv_fwd<128, 128, 64, 64, 64, PRO, DIL2>(a, s);
  if (a->K > 32) return launch_conv_fwd<256, 64, 64, 64, 64, PRO, DIL2>(a, s);
  if (a->K > 16) return launch_conv_fwd<256, 32, 64, 64, 32, PRO, DIL2>(a, s);
  return launch_conv_fwd<256, 16, 32, 64, 16, PRO, DIL2>(a, s);
}

}  // namespace drn

// Host-side pixel-tile count for a given output-channel count (sizing of the stats buffer).
DRN_API int drn_conv_fwd_tiles_p(int M, int K) {
  const int BP = (K >= 128) ? 128 : 256;
  return (M + BP - 1) / BP;
}

DRN_API int drn_conv_fwd(DrnConvFwdArgs* a, hipStream_t s) {
  if ((a->C % 8) != 0 || (a->K % 8) != 0) return (int)hipErrorInvalidValue;
  if (a->dil != 1 && a->dil != 2) return (int)hipErrorInvalidValue;
  const bool pro = a->in_scale != nullptr;
  const bool dil2 = a->dil == 2;
  if (pro) return dil2 ? drn::dispatch_conv_fwd<true, true>(a, s) : drn::dispatch_conv_fwd<true, false>(a, s);
  return dil2 ? drn::dispatch_conv_fwd<false, true>(a, s) : drn::dispatch_conv_fwd<false, false>(a, s);
}
