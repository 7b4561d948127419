// conv_wgrad.hip — weight gradient of an NHWC bf16 convolution on CDNA4 MFMA (gfx950).
//
// Replaces the Conv2DBackpropFilter the reference graph gets from autodiff of every
// `conv2d_fixed_padding` (reference resnet_model_official.py:87-91).
//
// GEMM view:  dW[cout][k] = sum_{pixels m} dY[m][cout] * Patch[m][k],  k = (r, s, ci).
// Both operands are stored with the NON-reduction dim contiguous (NHWC rows), so the
// fragments are read out of LDS with the gfx950 hardware transpose `ds_read_b64_tr_b16`
// (4 rows x 16 cols per 16-lane group, delivered column-major). MFMA operand A = patches
// (rows = k), operand B = dY (cols = cout): the accumulator then holds 4 consecutive k of
// one output channel per lane -> 16-byte fp32 stores into the KRSC gradient.
//
// Block = 4 waves over a 64(k) x BC(cout) tile; each step stages 128 output pixels, every
// wave owning a 32-pixel MFMA k-slice (intra-block split-K), summed through LDS at the end.
// Grid z-splits the pixel range (split-K) into fp32 partial slabs reduced deterministically
// by drn_splitk_reduce (no float atomics: bitwise-reproducible gradients).
// LDS rows are 128 B with a 16-B chunk XOR swizzle f(row) that makes the transposed reads
// conflict-free (simulated against the tr_b16 bank rule) and keeps 128-B ds_write groups.
#include "drn_common.h"
#include "drn_conv.h"

namespace drn {

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const DrnFastDiv& f) {
  return (__umulhi(n, f.m) + n) >> f.s;
}

__device__ __forceinline__ int swz(int row) { return (((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2); }

typedef short s16x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4v lds_s16x4;

__device__ __forceinline__ s16x4v tr_read(const char* base, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + byte_off));
}

template <int BC, bool PRO>
__global__ __launch_bounds__(256, 2) void conv_wgrad_kernel(DrnConvWgradArgs a) {
  constexpr int BKK = 64;          // k (r,s,ci) columns per block
  constexpr int BM = 128;          // pixels per step
  constexpr int TILE = BM * 128;   // bytes per operand image (128-B rows)
  constexpr int STAGE = 2 * TILE;
  constexpr int CHD = BC / 8;      // dY chunks per row
  constexpr int ND = (BM * CHD) / 256;
  constexpr int MJ = BC / 16;      // cout subtiles
  static_assert(ND >= 1, "dY tile must cover 256 threads");

  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Ktot = a.R * a.S * a.C;
  const int M = a.N * a.P * a.Q;
  const int nkt = (Ktot + BKK - 1) / BKK;
  const int bid = blockIdx.x;
  const int kt = bid % nkt;
  const int ct = bid / nkt;
  const int k0 = kt * BKK, c0 = ct * BC;
  const int split = blockIdx.y;
  const int mbeg = split * a.pix_per_split;
  const int mend = min(M, mbeg + a.pix_per_split);

  // patch loader: lane -> (chunk = lane&7, row = lane>>3 + 8*(wave+4i)), 4 vectors/thread
  const int pchunk = lane & 7;
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
  // dY loader: lane -> (chunk = lane % CHD, row = lane / CHD + (64/CHD)*(wave+4i))
  const int dchunk = lane % CHD;
  const int dc = c0 + dchunk * 8;
  const bool dvalid_c = dc < a.K;

  uint4 rp[4], rd[ND];
  auto load_stage = [&](int mstep) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (lane >> 3) + 8 * (wave + 4 * i);
      const int m = mstep + row;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (kvalid && m < mend) {
        const uint32_t n = fdiv((uint32_t)m, a.fd_pq);
        const uint32_t rem = (uint32_t)m - n * (uint32_t)(a.P * a.Q);
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
    for (int i = 0; i < ND; ++i) {
      const int row = lane / CHD + (64 / CHD) * (wave + 4 * i);
      const int m = mstep + row;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (dvalid_c && m < mend)
        v = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(a.dy) + (size_t)m * a.K + dc);
      rd[i] = v;
    }
  };
  auto store_stage = [&](char* st) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (lane >> 3) + 8 * (wave + 4 * i);
      *reinterpret_cast<uint4*>(st + row * 128 + ((pchunk ^ swz(row)) & 7) * 16) = rp[i];
    }
    char* sd = st + TILE;
#pragma unroll
    for (int i = 0; i < ND; ++i) {
      const int row = lane / CHD + (64 / CHD) * (wave + 4 * i);
      *reinterpret_cast<uint4*>(sd + row * 128 + ((dchunk ^ swz(row)) & 7) * 16) = rd[i];
    }
  };

  f32x4_t acc[4][MJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < MJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int T = (mend > mbeg) ? (mend - mbeg + BM - 1) / BM : 0;
  // per-lane transposed-read geometry: group g = lane>>4 owns k-rows 8g..8g+7 of the wave slice
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;

  if (T > 0) {
    load_stage(mbeg);
    store_stage(smem);
    __syncthreads();
  }
  for (int t = 0; t < T; ++t) {
    const char* cur = smem + (t & 1) * STAGE;
    const bool more = (t + 1) < T;
    if (more) load_stage(mbeg + (t + 1) * BM);
    bf16x8_t af[4], bfr[MJ];
    {
      s16x4v alo[4], ahi[4], blo[MJ], bhi[MJ];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int row = 32 * wave + 8 * g + 4 * hh + q4;
        const int rbase = row * 128;
        const int sw = swz(row);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int col = 16 * i + 4 * p4;
          const int off = rbase + (((col >> 3) ^ sw) & 7) * 16 + (col & 7) * 2;
          if (hh == 0) alo[i] = tr_read(cur, off); else ahi[i] = tr_read(cur, off);
        }
#pragma unroll
        for (int j = 0; j < MJ; ++j) {
          const int col = 16 * j + 4 * p4;
          const int off = TILE + rbase + (((col >> 3) ^ sw) & 7) * 16 + (col & 7) * 2;
          if (hh == 0) blo[j] = tr_read(cur, off); else bhi[j] = tr_read(cur, off);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(alo[i], ahi[i], 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
      for (int j = 0; j < MJ; ++j)
        bfr[j] = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(blo[j], bhi[j], 0, 1, 2, 3, 4, 5, 6, 7));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < MJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (more) store_stage(smem + ((t + 1) & 1) * STAGE);
    __syncthreads();
  }

  // ---- intra-block reduction of the 4 waves' partial tiles (each 64 x BC fp32) ----
  float* red = reinterpret_cast<float*>(smem);  // [3 waves][4][MJ][64 lanes][4]
  if (wave > 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < MJ; ++j)
        *reinterpret_cast<f32x4_t*>(red + ((((wave - 1) * 4 + i) * MJ + j) * 64 + lane) * 4) = acc[i][j];
  }
  __syncthreads();
  if (wave == 0) {
    float* out = a.out + (size_t)split * a.K * Ktot;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        f32x4_t v = acc[i][j];
#pragma unroll
        for (int w = 0; w < 3; ++w)
          v += *reinterpret_cast<const f32x4_t*>(red + (((w * 4 + i) * MJ + j) * 64 + lane) * 4);
        const int co = c0 + 16 * j + (lane & 15);
        const int kr = k0 + 16 * i + 4 * (lane >> 4);
        if (co < a.K && kr < Ktot) *reinterpret_cast<f32x4_t*>(out + (size_t)co * Ktot + kr) = v;
      }
  }
}

template <int BC, bool PRO>
static int launch_wgrad(DrnConvWgradArgs* a, hipStream_t s) {
  constexpr int LDS_MAIN = 2 * 2 * 128 * 128;
  constexpr int LDS_RED = 3 * 4 * (BC / 16) * 64 * 4 * 4;
  constexpr int LDS = LDS_MAIN > LDS_RED ? LDS_MAIN : LDS_RED;
  static bool attr_set = false;
  auto kern = conv_wgrad_kernel<BC, PRO>;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr_set = true;
  }
  const int Ktot = a->R * a->S * a->C;
  const int nkt = (Ktot + 63) / 64;
  const int nct = (a->K + BC - 1) / BC;
  hipLaunchKernelGGL(kern, dim3(nkt * nct, a->splits), dim3(256), LDS, s, *a);
  return (int)hipGetLastError();
}

__global__ void splitk_reduce_kernel(const float* __restrict__ ws, float* __restrict__ out, int n4, int splits,
                                     size_t stride4, float scale, int accumulate) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    float4 s = reinterpret_cast<const float4*>(ws)[i];
    for (int k = 1; k < splits; ++k) {
      const float4 v = reinterpret_cast<const float4*>(ws)[i + k * stride4];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    s.x *= scale; s.y *= scale; s.z *= scale; s.w *= scale;
    if (accumulate) {
      const float4 o = reinterpret_cast<float4*>(out)[i];
      s.x += o.x; s.y += o.y; s.z += o.z; s.w += o.w;
    }
    reinterpret_cast<float4*>(out)[i] = s;
  }
}

}  // namespace drn

DRN_API int drn_conv_wgrad(DrnConvWgradArgs* a, hipStream_t s) {
  if ((a->C % 8) != 0 || (a->K % 8) != 0 || a->splits < 1) return (int)hipErrorInvalidValue;
  const bool pro = a->in_scale != nullptr;
  if (a->K >= 64) return pro ? drn::launch_wgrad<64, true>(a, s) : drn::launch_wgrad<64, false>(a, s);
  if (a->K > 16) return pro ? drn::launch_wgrad<32, true>(a, s) : drn::launch_wgrad<32, false>(a, s);
  return pro ? drn::launch_wgrad<16, true>(a, s) : drn::launch_wgrad<16, false>(a, s);
}

// out[i] (+)= scale * sum_k ws[k][i]  over n floats (n % 4 == 0), deterministic order.
DRN_API int drn_splitk_reduce(const float* ws, float* out, int64_t n, int splits, float scale, int accumulate,
                              hipStream_t s) {
  if (n % 4) return (int)hipErrorInvalidValue;
  const int n4 = (int)(n / 4);
  int blocks = (n4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(drn::splitk_reduce_kernel, dim3(blocks), dim3(256), 0, s, ws, out, n4, splits, (size_t)n4,
                     scale, accumulate);
  return (int)hipGetLastError();
}
