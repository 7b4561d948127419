// drn_conv_epi.h -- device helpers of the implicit-GEMM convolution kernels (conv_fwd.hip,
// stem.hip): the fused
// epilogue (LDS-staged fp32 tile -> coalesced bf16 rows, residual add, strided output map,
// next-BN statistics or fused BN-backward reduction), the LDS-DMA issue helpers and the
// swizzle of the 128-byte LDS rows.
#pragma once
#include "drn_common.h"
#include "drn_conv.h"

namespace drn {

__device__ __forceinline__ unsigned long long drn_realtime() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
  return t;
}

// Sum of x over the lanes of a wave that are congruent mod CHR (CHR = 2..32, a power of two):
// row rotations by CHR, 2*CHR .. 8 inside each 16-lane DPP row, then the cross-row partners via
// v_permlane16_swap (lane ^ 16) and v_permlane32_swap (lane ^ 32). Every such lane gets the sum.
template <int S>
__device__ __forceinline__ float dpp_row_ror(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x120 | S, 0xF, 0xF, false));
}

template <int CHR>
__device__ __forceinline__ float chunk_lane_sum(float x) {
  static_assert(CHR >= 2 && CHR <= 32 && (CHR & (CHR - 1)) == 0, "chunk count");
  if constexpr (CHR <= 2) x += dpp_row_ror<2>(x);
  if constexpr (CHR <= 4) x += dpp_row_ror<4>(x);
  if constexpr (CHR <= 8) x += dpp_row_ror<8>(x);
  if constexpr (CHR <= 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// ---------------- shared epilogue ----------------
// Every lane owns 8 consecutive channels (one 16-byte bf16 chunk) of BP/RPI pixel rows.
// epi_prefetch() computes those output offsets and issues the 16-byte loads of the residual
// and of the fused-BN-backward input BEFORE the main loop, so their latency hides behind the
// MFMA work instead of stalling the epilogue (short-K launches are otherwise dominated by it).
// PF = false: nothing is prefetched (no residual / BN-backward operand; saves the 64 VGPRs
// that would otherwise cap the occupancy).
template <int BP, int BC, int NT = 256, bool PF = true>
struct EpiPre {
  static constexpr int CHR = BC / 8;  // output 16-byte chunks per pixel row
  static constexpr int RPI = NT / CHR;
  static constexpr int IT = BP / RPI;
  static constexpr int NPF = PF ? IT : 1;
  int off[IT];     // element offset of the chunk, -1 when outside the output
  uint4 res[NPF];
  uint4 bx[NPF];
};

template <int BP, int BC, int NT = 256, bool PF = true>
__device__ __forceinline__ void epi_prefetch(const DrnConvFwdArgs& a, int m0, int c0, int M,
                                             EpiPre<BP, BC, NT, PF>& e) {
  using E = EpiPre<BP, BC, NT, PF>;
  const int tid = threadIdx.x;
  const int ch = tid % E::CHR;
  const int c = c0 + ch * 8;
  const bool mapped = a.out_stride != 0;
  const int pq = a.P * a.Q;
  const bf16_t* __restrict__ res = reinterpret_cast<const bf16_t*>(a.residual);
  const bf16_t* __restrict__ bx = reinterpret_cast<const bf16_t*>(a.bn_x);
#pragma unroll
  for (int it = 0; it < E::IT; ++it) {
    const int m = m0 + it * E::RPI + tid / E::CHR;
    int off = -1;
    if (m < M && c < a.K) {
      if (mapped) {
        const int n = (int)drn_fdiv((uint32_t)m, a.fd_pq);
        const int rem = m - n * pq;
        const int i = (int)drn_fdiv((uint32_t)rem, a.fd_q);
        const int j = rem - i * a.Q;
        off = ((n * a.out_H + i * a.out_stride + a.out_oh) * a.out_W + j * a.out_stride + a.out_ow) * a.K + c;
      } else {
        off = m * a.K + c;
      }
    }
    e.off[it] = off;
    if constexpr (PF) {
      e.res[it] = (res && off >= 0) ? *reinterpret_cast<const uint4*>(res + off) : make_uint4(0u, 0u, 0u, 0u);
      e.bx[it] = (bx && off >= 0) ? *reinterpret_cast<const uint4*>(bx + off) : make_uint4(0u, 0u, 0u, 0u);
    }
  }
}

// Last-arriving workgroup of a channel column finalizes that column's BatchNorm (see
// DrnConvFwdArgs::fin_cnt). The statistics atomics and the arrival counter are agent-scope
// atomics, performed past the per-XCD L2s; every thread waits for its own atomics to complete
// (vmcnt(0)) before the barrier and thread 0's counter increment, and the last workgroup reads
// the replicas with agent-scope loads. No agent-scope fence: on gfx950 that writes back the
// whole L2 (buffer_wbl2), which, issued by every workgroup, costs several times the conv.
// The flag word lives in the (by now free) epilogue staging LDS: a static __shared__ variable
// would add an LDS allocation granule to every instantiation and cost the 32 KB configurations
// their fifth workgroup per CU.
template <int BP, int BC, int NT>
__device__ __forceinline__ void bn_fin_column(const DrnConvFwdArgs& a, int c0, int M, int* s_last) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // also: every thread is done with the staging LDS
  const int col = c0 / BC;
  if (threadIdx.x == 0) {
    const unsigned tiles = (unsigned)((M + BP - 1) / BP);
    *s_last = __hip_atomic_fetch_add(a.fin_cnt + col, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u == tiles;
  }
  __syncthreads();
  if (!*s_last) return;
  const int rep = a.stats_rep > 1 ? a.stats_rep : 1;
  const int K = a.K;
  for (int cl = threadIdx.x; cl < BC; cl += NT) {
    const int c = c0 + cl;
    if (c >= K) break;
    float s = 0.f, q = 0.f;
    for (int r = 0; r < rep; ++r) {
      s += __hip_atomic_load(a.stats + (size_t)(2 * r) * K + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      q += __hip_atomic_load(a.stats + (size_t)(2 * r + 1) * K + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (a.bn_x != nullptr) {
      a.fin_dbeta[c] = s;
      a.fin_dgamma[c] = q;
      a.fin_coef[c] = a.fin_gamma[c] * a.bn_invstd[c];
      a.fin_coef[K + c] = s / a.fin_count;
      a.fin_coef[2 * K + c] = q / a.fin_count;
    } else {
      const double mean = (double)s / a.fin_count;
      double var = (double)q / a.fin_count - mean * mean;
      if (var < 0.0) var = 0.0;
      const float invstd = (float)(1.0 / sqrt(var + (double)a.fin_eps));
      const float sc = a.fin_gamma[c] * invstd;
      a.fin_scale[c] = sc;
      a.fin_shift[c] = a.fin_beta[c] - (float)mean * sc;
      a.fin_mean[c] = (float)mean;
      a.fin_invstd[c] = invstd;
      if (a.fin_run_mean != nullptr) {  // TF fused BN: the unbiased batch variance feeds the moving variance
        const float n = a.fin_count;
        const float unbiased = n > 1.f ? (float)(var * n / (n - 1.0)) : (float)var;
        const float mo = a.fin_momentum;
        a.fin_run_mean[c] = mo * a.fin_run_mean[c] + (1.f - mo) * (float)mean;
        a.fin_run_var[c] = mo * a.fin_run_var[c] + (1.f - mo) * unbiased;
      }
    }
  }
  if (threadIdx.x == 0)  // re-arm: the next launch is stream-ordered after this one
    __hip_atomic_store(a.fin_cnt + col, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The fp32 accumulator tile is staged through LDS ([BP][BC] fp32, 16-byte chunks XOR-swizzled
// by row: conflict-free 8-lane ds_write_b128 groups and 16-lane ds_read_b128 groups), then
// written as whole 2*BC-byte pixel rows per wave instruction (fully coalesced). Optional
// residual add, optional strided output map, optional per-channel sum/sumsq for the next BN,
// or (bn_x set) the fused BN-backward reduction with ReLU-masked output.
//
// conv_epilogue_pass handles ONE channel slice [c0, c0 + BC) of the block tile: the waves that
// own it (stage == true) write their accumulators, then every thread stores / reduces it. The
// big-tile kernels (256 x 256) run it in NH slices because the whole fp32 tile (256 KB) does
// not fit the 160 KB LDS; wcs = the wave's channel offset inside the slice.
// element offset of output pixel m, channel c (-1 outside the output): epi_prefetch's map
__device__ __forceinline__ int epi_off(const DrnConvFwdArgs& a, int m, int c, int M) {
  if (m >= M || c >= a.K) return -1;
  if (a.out_stride == 0) return m * a.K + c;
  const int pq = a.P * a.Q;
  const int n = (int)drn_fdiv((uint32_t)m, a.fd_pq);
  const int rem = m - n * pq;
  const int i = (int)drn_fdiv((uint32_t)rem, a.fd_q);
  const int j = rem - i * a.Q;
  return ((n * a.out_H + i * a.out_stride + a.out_oh) * a.out_W + j * a.out_stride + a.out_ow) * a.K + c;
}

// Row map of the staged tile: staged row -> output pixel m (>= M: not an output pixel); the
// implicit-GEMM kernels' tiles are consecutive pixels.
struct EpiRowId {
  __device__ __forceinline__ int operator()(int m0, int row) const { return m0 + row; }
};

// LAZY: output offsets computed per row here instead of held in e.off (no registers across the
// main loop / the other slices)
template <int BP, int BC, int WP, int MI, int MJ, int NT = 256, bool PF = true, bool LAZY = false,
          typename RM = EpiRowId>
__device__ __forceinline__ void conv_epilogue_pass(const DrnConvFwdArgs& a, char* smem, f32x4_t (&acc)[MI][MJ],
                                                   bool stage, int wp, int wcs, int m0, int c0, int M,
                                                   const EpiPre<BP, BC, NT, PF>& e, RM rmap = RM()) {
  static_assert(!(LAZY && PF), "lazy offsets: no prefetched operands");
  using E = EpiPre<BP, BC, NT, PF>;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  constexpr int CF = BC / 4;   // fp32 16-byte chunks per staged row
  constexpr int CHR = E::CHR;
  constexpr int RPI = E::RPI;
  constexpr int SWM = CF >= 8 ? 7 : CF - 1;  // swizzle mask stays inside a staged row
  float* tile = reinterpret_cast<float*>(smem);
  if (stage) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int cf = (wcs + i * 16) / 4 + (lane >> 4);  // fp32 chunk of these 4 channels
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        const int row = wp * WP + j * 16 + (lane & 15);
        *reinterpret_cast<f32x4_t*>(tile + row * BC + ((cf ^ (row & SWM)) * 4)) = acc[i][j];
      }
    }
  }
  __syncthreads();
  const bool want_stats = a.stats != nullptr;
  bf16_t* __restrict__ y = reinterpret_cast<bf16_t*>(a.y);
  const bool has_res = a.residual != nullptr;
  const int ch = tid % CHR;
  const int c = c0 + ch * 8;
  const bool bwd = a.bn_x != nullptr;
  float ssum[8], ssq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) ssum[j] = ssq[j] = 0.f;
  float bsc[8], bsh[8], bmu[8], bis[8];
  if (bwd && c < a.K) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bsc[j] = a.bn_scale[c + j];
      bsh[j] = a.bn_shift[c + j];
      bmu[j] = a.bn_mean[c + j];
      bis[j] = a.bn_invstd[c + j];
    }
  }
#pragma unroll(LAZY ? 2 : E::IT)
  for (int it = 0; it < E::IT; ++it) {
    const int row = it * RPI + tid / CHR;
    const f32x4_t lo = *reinterpret_cast<const f32x4_t*>(tile + row * BC + (((2 * ch) ^ (row & SWM)) * 4));
    const f32x4_t hi = *reinterpret_cast<const f32x4_t*>(tile + row * BC + (((2 * ch + 1) ^ (row & SWM)) * 4));
    const int off = LAZY ? epi_off(a, rmap(m0, row), c, M) : e.off[it];
    if (off >= 0) {
      float f[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if (has_res) {
        float r8[8];
        if constexpr (PF) unpack8(e.res[it], r8);
        else unpack8(*reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(a.residual) + off), r8);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] += r8[j];
      }
      const uint4 o = pack8(f);
      float q8[8];
      unpack8(o, q8);
      if (bwd) {
        // BN-backward: mask by the forward ReLU, accumulate sum g and sum g * xhat
        float xb[8];
        if constexpr (PF) unpack8(e.bx[it], xb);
        else unpack8(*reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(a.bn_x) + off), xb);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float g = (xb[j] * bsc[j] + bsh[j] > 0.f) ? q8[j] : 0.f;
          f[j] = g;
          ssum[j] += g;
          ssq[j] += g * ((xb[j] - bmu[j]) * bis[j]);
        }
        *reinterpret_cast<uint4*>(y + off) = pack8(f);
      } else {
        *reinterpret_cast<uint4*>(y + off) = o;
        if (a.out_fill && a.out_stride > 1) {
          // zeros at this pixel's sibling phase positions (single-phase strided output)
          const int m = rmap(m0, row);
          const int pq = a.P * a.Q;
          const int n = (int)drn_fdiv((uint32_t)m, a.fd_pq);
          const int rem = m - n * pq;
          const int i = (int)drn_fdiv((uint32_t)rem, a.fd_q);
          const int j = rem - i * a.Q;
          for (int ph = 0; ph < a.out_stride; ++ph)
            for (int pw = 0; pw < a.out_stride; ++pw) {
              const int hh = i * a.out_stride + ph, ww = j * a.out_stride + pw;
              if ((ph != a.out_oh || pw != a.out_ow) && hh < a.out_H && ww < a.out_W)
                *reinterpret_cast<uint4*>(y + ((n * a.out_H + hh) * a.out_W + ww) * a.K + c) = make_uint4(0u, 0u, 0u, 0u);
            }
        }
        if (want_stats) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            ssum[j] += q8[j];
            ssq[j] += q8[j] * q8[j];
          }
        }
      }
    }
  }
  if (want_stats) {
    // (1) within the wave: the lanes holding the same 8-channel chunk are lane = ch (mod CHR);
    //     DPP row rotations inside each 16-lane row, then permlane16/32 swaps across rows
    float v[16];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = chunk_lane_sum<CHR>(ssum[j]);
      v[8 + j] = chunk_lane_sum<CHR>(ssq[j]);
    }
    // (2) across the waves through LDS: [wave][chunk][16] wave totals
    constexpr int NWV = NT / 64;
    __syncthreads();  // every thread is done reading the staged tile
    float* red = tile;
    const int wv = tid >> 6, ln = tid & 63;
    if (ln < CHR) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<float4*>(red + (wv * CHR + ln) * 16 + 4 * q) =
            make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    }
    __syncthreads();
    for (int t = tid; t < 2 * BC; t += NT) {  // 2*BC may exceed the thread count (BC = 256)
      const int cl = t >> 1, which = t & 1;
      const int chh = cl >> 3, j = cl & 7;
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; ++w) s += red[(w * CHR + chh) * 16 + which * 8 + j];
      const int rep = a.stats_rep > 1 ? a.stats_rep : 1;
      if (c0 + cl < a.K) atomicAdd(a.stats + ((size_t)(blockIdx.x % rep) * 2 + which) * a.K + c0 + cl, s);
    }
  }
}

template <int BP, int BC, int WP, int WC, int MI, int MJ, int NT = 256, bool PF = true>
__device__ __forceinline__ void conv_epilogue(const DrnConvFwdArgs& a, char* smem, f32x4_t (&acc)[MI][MJ], int wp,
                                              int wc, int m0, int c0, int M, const EpiPre<BP, BC, NT, PF>& e) {
  conv_epilogue_pass<BP, BC, WP, MI, MJ, NT, PF>(a, smem, acc, true, wp, wc * WC, m0, c0, M, e);
  if (a.stats != nullptr && a.fin_cnt != nullptr) bn_fin_column<BP, BC, NT>(a, c0, M, reinterpret_cast<int*>(smem));
}

// NH channel slices of BC / NH (each wave's WC channels lie inside one slice); no prefetched
// epilogue operands (the big tiles spend their registers on accumulators)
template <int BP, int BC, int WP, int WC, int MI, int MJ, int NT, int NH, typename RM = EpiRowId>
__device__ __forceinline__ void conv_epilogue_sliced(const DrnConvFwdArgs& a, char* smem, f32x4_t (&acc)[MI][MJ],
                                                     int wp, int wc, int m0, int c0, int M, RM rmap = RM()) {
  constexpr int BCH = BC / NH;
  static_assert(BC % NH == 0 && BCH % WC == 0, "a wave's channels must lie inside one slice");
#pragma unroll 1
  for (int h = 0; h < NH; ++h) {
    if (h > 0) __syncthreads();  // the previous slice's LDS reads / reductions are done
    EpiPre<BP, BCH, NT, false> e;  // unused (LAZY offsets)
    const int wcs = wc * WC - h * BCH;
    conv_epilogue_pass<BP, BCH, WP, MI, MJ, NT, false, true, RM>(a, smem, acc, wcs >= 0 && wcs < BCH, wp, wcs, m0,
                                                                 c0 + h * BCH, M, e, rmap);
  }
  if (a.stats != nullptr && a.fin_cnt != nullptr) bn_fin_column<BP, BC, NT>(a, c0, M, reinterpret_cast<int*>(smem));
}

typedef __attribute__((address_space(3))) void drn_lds_void;
typedef __attribute__((address_space(1))) const void drn_gbl_void;

__device__ __forceinline__ void glds16(const void* src, char* lds_base) {
  __builtin_amdgcn_global_load_lds((drn_gbl_void*)src, (drn_lds_void*)lds_base, 16, 0, 0);
}


template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// BK = 64: 128-byte LDS rows, slot(chunk c of row r) = c ^ ((r >> 1) & 7)
// BK = 32: 64-byte LDS rows (a stage holds one 32-deep MFMA k-slice; twice the stages in the same
//          LDS, i.e. a deeper pipeline), slot = c ^ (((r >> 2) & 1) << 1); both conflict-free for
//          the ds_read_b128 fragment reads (exhaustive check over the gfx950 lane groups).
template <int BK>
__device__ __forceinline__ int glds_swz(int row) {
  if constexpr (BK == 64) return (row >> 1) & 7;
  return ((row >> 2) & 1) << 1;
}

}  // namespace drn
