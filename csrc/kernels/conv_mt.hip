// conv_mt.hip — multi-tile LDS-DMA implicit-GEMM convolution (NHWC bf16, gfx950 MFMA).
//
// Same GEMM view, operand images and fused prologue as conv_fwd_glds_kernel (conv_fwd.hip):
// D[cout][pixel] = sum_k W[cout][k] * Patch[pixel][k], k = (r, s, ci), 64-deep LDS-DMA stages,
// v_mfma_f32_16x16x32_bf16, optional BN-apply+ReLU of the input applied in LDS (pre-activation
// v2, reference resnet_model_official.py:113-119).
//
// What differs is how a workgroup spends its lifetime. Per-workgroup timelines of the one-tile
// kernel (scripts/trace_conv.py) showed every block spending ~2.5 us waiting for its first
// stage and ~2.3 us in an epilogue during which nothing was loading, at 2 blocks per CU: the
// memory-bound 1x1 convolutions reached ~3-4 TB/s. Here a workgroup walks TPB consecutive
// output tiles through ONE continuous LDS-DMA pipeline: the next tile's first stages are in
// flight while the current tile's epilogue runs, so the DMA queue never drains between tiles.
//
// The epilogue writes straight from the MFMA accumulators (no LDS staging tile, so the LDS holds
// only the pipeline stages): lane l owns output channels 4*(l>>4)..+3 of pixel (l&15) of every
// 16x16 fragment, i.e. one 8-byte bf16 store per fragment. Per-channel statistics are summed
// over the lane's pixels, then across the 16 lanes of a DPP row (quad_perm / half-mirror /
// mirror butterfly: all 16 lanes end with the row total) and added with one buffer atomic per
// fragment row. Every epilogue memory operation is an UNCONDITIONAL buffer instruction whose
// out-of-range lanes carry an offset past the descriptor's size (the range check drops them),
// so the number of vector-memory instructions a tile's epilogue issues is a compile-time
// constant and the counted `s_waitcnt vmcnt` of the following stages can account for it
// exactly (vmcnt counts loads, LDS-DMAs, stores and atomics together, in issue order).
//
// Epilogue variants (compile-time): RES adds a residual (block output `inputs + shortcut`,
// reference :130/:175, or the accumulating data gradient), ST = 1 accumulates (sum, sumsq) of
// the stored output for the next BatchNorm, ST = 2 is the fused BN-backward reduction (output
// ReLU-masked by the forward pre-activation, sums of g and g * xhat). Optional strided output
// map (phase-decomposed data gradient).
#include "drn_common.h"
#include "drn_conv.h"

namespace drn {
namespace mt {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_void;
typedef int i32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void glds16(const void* src, char* lds) {
  __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)lds, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void vmwait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// 128-byte LDS rows: 16-byte chunk c of row r lives in slot c ^ ((r >> 1) & 7)
__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// sum over the 16 lanes of a DPP row; every lane of the row receives the total
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  v += dpp<0x140>(v);  // row_mirror
  return v;
}

constexpr uint32_t OOB = 0x80000000u;  // offset past every descriptor: the buffer op is dropped

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

template <int BP, int BC, int WAVES_P, int NS, bool PRO, bool RES, int ST>
__global__ __launch_bounds__(256, 2) void conv_mt_kernel(DrnConvFwdArgs a, const void* __restrict__ zero,
                                                         int ntiles, int tpb) {
  constexpr int NW = 4, NT = 256, BK = 64, ROWB = 128, CPR = 8, RPG = 8;
  constexpr int WAVES_C = NW / WAVES_P;
  constexpr int WP = BP / WAVES_P, WC = BC / WAVES_C;
  constexpr int MI = WC / 16, MJ = WP / 16;
  constexpr int STAGE = (BC + BP) * ROWB;
  constexpr int GA = BC / (RPG * NW), GB = BP / (RPG * NW);
  constexpr int G = GA + GB;
  constexpr int D = NS - 1;
  // vector-memory instructions of one tile's epilogue that can still be in flight when the
  // next tile's stages are waited for: the stores and the statistics atomics
  constexpr int NWR = MI * MJ + (ST ? MI : 0);
  constexpr int W0 = G * (D - 1);
  constexpr int W1 = (W0 + NWR) < 63 ? (W0 + NWR) : 63;
  static_assert(WAVES_P * WAVES_C == NW && MI >= 1 && MJ >= 1, "wave layout");
  static_assert(GA * RPG * NW == BC && GB * RPG * NW == BP, "rows must split evenly over the waves");
  static_assert(NS >= 2 && W0 < 64, "pipeline depth");
  static_assert(!(PRO && ST == 2), "the BN-backward epilogue runs on data gradients (no input BN)");

  extern __shared__ __attribute__((aligned(1024))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int M = a.N * a.P * a.Q;
  const int C = a.C;
  const int K = a.K;
  const int Ktot = a.R * a.S * C;
  const int T = Ktot / BK;  // stages per tile (host guarantees T >= D)
  const int ntc = (K + BC - 1) / BC;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile0 = bid * tpb;
  const int ntile = min(tpb, ntiles - tile0);
  if (ntile <= 0) return;
  const int total = ntile * T;

  const int lrow = lane / CPR;
  const int lpc = lane % CPR;
  const bf16_t* __restrict__ xg = reinterpret_cast<const bf16_t*>(a.x);
  const bf16_t* __restrict__ wg = reinterpret_cast<const bf16_t*>(a.w);
  const int pq = a.P * a.Q;

  // ---- issue-side state (the tile whose stages are being issued) ----
  const bf16_t* wsrc[GA];
  int bh[GB], bw[GB], boff[GB];
  int ik = 0, ir = 0, is = 0, ici = 0, itile = 0;
  auto set_issue_tile = [&](int t) {
    const int tt = tile0 + t;
    const int c0 = (tt % ntc) * BC;
    const int m0 = (tt / ntc) * BP;
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const int row = RPG * NW * i + RPG * wave + lrow;
      const int c = c0 + row;
      wsrc[i] = c < K ? wg + (size_t)c * Ktot + (lpc ^ swz(row)) * 8 : nullptr;
    }
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      const int row = RPG * NW * i + RPG * wave + lrow;
      const int m = m0 + row;
      if (m < M) {
        const int n = (int)drn_fdiv((uint32_t)m, a.fd_pq);
        const int rem = m - n * pq;
        const int p = (int)drn_fdiv((uint32_t)rem, a.fd_q);
        const int q = rem - p * a.Q;
        bh[i] = p * a.stride - a.pad_h;
        bw[i] = q * a.stride - a.pad_w;
        boff[i] = ((n * a.H + bh[i]) * a.W + bw[i]) * C + (lpc ^ swz(row)) * 8;
      } else {
        bh[i] = -(1 << 28);
        bw[i] = 0;
        boff[i] = 0;
      }
    }
    ik = ir = is = ici = 0;
  };
  auto issue = [&](int slot) {
    char* st = smem + slot * STAGE;
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const void* src = wsrc[i] ? (const void*)(wsrc[i] + ik) : zero;
      glds16(src, st + (RPG * NW * i + RPG * wave) * ROWB);
    }
    const int tap_off = (ir * a.W + is) * C + ici;
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      const int h = bh[i] + ir, w = bw[i] + is;
      const bool ok = (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
      const void* src = ok ? (const void*)(xg + (boff[i] + tap_off)) : zero;
      glds16(src, st + (BC + RPG * NW * i + RPG * wave) * ROWB);
    }
    ik += BK;
    ici += BK;
    if (ici == C) {
      ici = 0;
      if (++is == a.S) {
        is = 0;
        ++ir;
      }
    }
    if (ik == Ktot && ++itile < ntile) set_issue_tile(itile);
  };

  const int wp = wave % WAVES_P;
  const int wc = wave / WAVES_P;
  f32x4_t acc[MI][MJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < MJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fk = lane >> 4;
  int aoff[MI], boffl[MJ];
#pragma unroll
  for (int i = 0; i < MI; ++i) aoff[i] = (wc * WC + i * 16 + fr) * ROWB;
#pragma unroll
  for (int j = 0; j < MJ; ++j) boffl[j] = (BC + wp * WP + j * 16 + fr) * ROWB;
  const int fswz = swz(fr);

  // fused-BN operands [scale C][shift C] behind the stages (PRO)
  float* const ssl = reinterpret_cast<float*>(smem + NS * STAGE);
  const int lcb = lpc ^ swz(RPG * wave + lrow);
  // compute-side state for the PRO transform: tap / channel offset of the stage being
  // transformed and the pixel geometry of its tile
  int xr = 0, xs = 0, xci = 0;
  int cbh[GB], cbw[GB];
  auto set_compute_geom = [&](int t) {
    if constexpr (PRO) {
      const int tt = tile0 + t;
      const int m0 = (tt / ntc) * BP;
#pragma unroll
      for (int i = 0; i < GB; ++i) {
        const int m = m0 + RPG * NW * i + RPG * wave + lrow;
        if (m < M) {
          const int n = (int)drn_fdiv((uint32_t)m, a.fd_pq);
          const int rem = m - n * pq;
          const int p = (int)drn_fdiv((uint32_t)rem, a.fd_q);
          cbh[i] = p * a.stride - a.pad_h;
          cbw[i] = (rem - p * a.Q) * a.stride - a.pad_w;
        } else {
          cbh[i] = -(1 << 28);
          cbw[i] = 0;
        }
      }
    }
  };

  set_issue_tile(0);
#pragma unroll
  for (int s = 0; s < D; ++s)
    if (s < total) issue(s);
  if constexpr (PRO) {
    set_compute_geom(0);
    if (a.in_fin.stats != nullptr) {
      const bool pub = a.in_fin.publish && blockIdx.x == 0;
      for (int c = tid; c < C; c += NT) drn_bn_fin_fwd(a.in_fin, c, pub, ssl[c], ssl[C + c]);
    } else {
      for (int c = tid * 4; c < C; c += NT * 4) {
        *reinterpret_cast<float4*>(ssl + c) = *reinterpret_cast<const float4*>(a.in_scale + c);
        *reinterpret_cast<float4*>(ssl + C + c) = *reinterpret_cast<const float4*>(a.in_shift + c);
      }
    }
    __syncthreads();
  }

  // ---- epilogue descriptors ----
  const uint32_t ybytes = (uint32_t)((a.out_stride ? (size_t)a.N * a.out_H * a.out_W : (size_t)M) * K * 2);
  const __amdgpu_buffer_rsrc_t ry = rsrc(a.y, ybytes);
  const __amdgpu_buffer_rsrc_t rr = rsrc(RES ? a.residual : a.y, ybytes);
  const __amdgpu_buffer_rsrc_t rx = rsrc(ST == 2 ? a.bn_x : a.y, ybytes);
  const int rep = a.stats_rep > 1 ? a.stats_rep : 1;
  const __amdgpu_buffer_rsrc_t rs = rsrc(a.stats, ST ? (uint32_t)(rep * 2 * K * 4) : 0u);
  const uint32_t rep_off = (uint32_t)((blockIdx.x % rep) * 2 * K) * 4u;

  auto epilogue = [&](int t) {
    const int tt = tile0 + t;
    const int c0 = (tt % ntc) * BC;
    const int m0 = (tt / ntc) * BP;
    // byte offset of this lane's pixel row of fragment column j (OOB when past M)
    uint32_t poff[MJ];
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      const int m = m0 + wp * WP + j * 16 + fr;
      uint32_t o = OOB;
      if (m < M) {
        if (a.out_stride) {
          const int n = (int)drn_fdiv((uint32_t)m, a.fd_pq);
          const int rem = m - n * pq;
          const int i = (int)drn_fdiv((uint32_t)rem, a.fd_q);
          const int jj = rem - i * a.Q;
          o = (uint32_t)(((n * a.out_H + i * a.out_stride + a.out_oh) * a.out_W + jj * a.out_stride + a.out_ow) * K) * 2u;
        } else {
          o = (uint32_t)(m * K) * 2u;
        }
      }
      poff[j] = o;
    }
    uint32_t coff[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int c = c0 + wc * WC + i * 16 + 4 * fk;
      coff[i] = c < K ? (uint32_t)c * 2u : OOB;
    }
    // residual / BN-backward input of fragment row i (loaded per row: all rows at once would
    // not fit the 256 registers of a 2-workgroups-per-CU launch)
    auto ld_row = [&](int i, i32x2 (&res)[MJ], i32x2 (&bx)[MJ]) {
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        const uint32_t o = (poff[j] | coff[i]) >= OOB ? OOB : poff[j] + coff[i];
        if constexpr (RES) res[j] = __builtin_amdgcn_raw_buffer_load_b64(rr, (int)o, 0, 0);
        if constexpr (ST == 2) bx[j] = __builtin_amdgcn_raw_buffer_load_b64(rx, (int)o, 0, 0);
      }
    };
    i32x2 resn[MJ], bxn[MJ];
    ld_row(0, resn, bxn);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      float s4[4] = {0.f, 0.f, 0.f, 0.f}, q4[4] = {0.f, 0.f, 0.f, 0.f};
      i32x2 res[MJ], bx[MJ];
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        res[j] = resn[j];
        bx[j] = bxn[j];
      }
      if (i + 1 < MI) ld_row(i + 1, resn, bxn);  // next row's loads in flight during this row
      float4 bsc, bsh, bmu, bis;
      if constexpr (ST == 2) {
        const int c = min(c0 + wc * WC + i * 16 + 4 * fk, K - 4);
        bsc = *reinterpret_cast<const float4*>(a.bn_scale + c);
        bsh = *reinterpret_cast<const float4*>(a.bn_shift + c);
        bmu = *reinterpret_cast<const float4*>(a.bn_mean + c);
        bis = *reinterpret_cast<const float4*>(a.bn_invstd + c);
      }
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        float f[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if constexpr (RES) {
          const uint32_t lo = (uint32_t)res[j][0], hi = (uint32_t)res[j][1];
          f[0] += __uint_as_float(lo << 16);
          f[1] += __uint_as_float(lo & 0xffff0000u);
          f[2] += __uint_as_float(hi << 16);
          f[3] += __uint_as_float(hi & 0xffff0000u);
        }
        uint32_t o0 = pack2bf(f[0], f[1]), o1 = pack2bf(f[2], f[3]);
        const bool live = (poff[j] | coff[i]) < OOB;
        if constexpr (ST == 1) {
          const float v[4] = {__uint_as_float(o0 << 16), __uint_as_float(o0 & 0xffff0000u),
                              __uint_as_float(o1 << 16), __uint_as_float(o1 & 0xffff0000u)};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float ve = live ? v[e] : 0.f;
            s4[e] += ve;
            q4[e] = fmaf(ve, ve, q4[e]);
          }
        } else if constexpr (ST == 2) {
          const uint32_t xl = (uint32_t)bx[j][0], xh = (uint32_t)bx[j][1];
          const float xv[4] = {__uint_as_float(xl << 16), __uint_as_float(xl & 0xffff0000u), __uint_as_float(xh << 16),
                               __uint_as_float(xh & 0xffff0000u)};
          const float v[4] = {__uint_as_float(o0 << 16), __uint_as_float(o0 & 0xffff0000u),
                              __uint_as_float(o1 << 16), __uint_as_float(o1 & 0xffff0000u)};
          const float sc[4] = {bsc.x, bsc.y, bsc.z, bsc.w};
          const float sh[4] = {bsh.x, bsh.y, bsh.z, bsh.w};
          const float mu[4] = {bmu.x, bmu.y, bmu.z, bmu.w};
          const float is4[4] = {bis.x, bis.y, bis.z, bis.w};
          float g[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            g[e] = (live && xv[e] * sc[e] + sh[e] > 0.f) ? v[e] : 0.f;
            s4[e] += g[e];
            q4[e] = fmaf(g[e], (xv[e] - mu[e]) * is4[e], q4[e]);
          }
          o0 = pack2bf(g[0], g[1]);
          o1 = pack2bf(g[2], g[3]);
        }
        const uint32_t o = live ? poff[j] + coff[i] : OOB;
        __builtin_amdgcn_raw_buffer_store_b64(i32x2{(int)o0, (int)o1}, ry, (int)o, 0, 0);
      }
      if constexpr (ST != 0) {
        float tot[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          tot[e] = row_sum16(s4[e]);
          tot[4 + e] = row_sum16(q4[e]);
        }
        // lane fr < 8 of each row adds value fr: (sum | sumsq) of channel c + (fr & 3)
        float v = tot[0];
#pragma unroll
        for (int e = 1; e < 8; ++e) v = fr == e ? tot[e] : v;
        const uint32_t so = (fr < 8 && coff[i] < OOB)
                                ? rep_off + (uint32_t)(((fr >> 2) * K) * 4) + (coff[i] >> 1) * 4u + (uint32_t)(fr & 3) * 4u
                                : OOB;
        __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v, rs, (int)so, 0, 0);
      }
    }
  };

  int kst = 0, ctile = 0;
  for (int f = 0; f < total; ++f) {
    // retire stage f: what was issued after it may stay in flight (the D-1 later stages and,
    // right after an epilogue, that epilogue's stores / atomics)
    if (f + D - 1 < total) {
      if (kst < D && ctile > 0) vmwait<W1>();
      else vmwait<W0>();
    } else {
      vmwait<0>();
    }
    if constexpr (PRO) {
      char* sw = smem + (f % NS) * STAGE;
      const uint32_t sp = lds_addr(ssl + xci + lcb * 8);
      u32x4_t v[GB + 4];
      v[GB] = lds_read16(sp);
      v[GB + 1] = lds_read16(sp + 16);
      v[GB + 2] = lds_read16(sp + 4 * C);
      v[GB + 3] = lds_read16(sp + 4 * C + 16);
      uint32_t pa[GB], ok = 0;
#pragma unroll
      for (int i = 0; i < GB; ++i) {
        const int h = cbh[i] + xr, w = cbw[i] + xs;
        ok |= ((unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W) ? (1u << i) : 0u;
        pa[i] = lds_addr(sw + (BC + RPG * NW * i + RPG * wave) * ROWB + lane * 16);
        v[i] = lds_read16(pa[i]);
      }
      lds_wait_all<GB + 4>(v);
      f32x2_t sc2[4], sh2[4];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        sc2[2 * q] = f32x2_t{__uint_as_float(v[GB + q][0]), __uint_as_float(v[GB + q][1])};
        sc2[2 * q + 1] = f32x2_t{__uint_as_float(v[GB + q][2]), __uint_as_float(v[GB + q][3])};
        sh2[2 * q] = f32x2_t{__uint_as_float(v[GB + 2 + q][0]), __uint_as_float(v[GB + 2 + q][1])};
        sh2[2 * q + 1] = f32x2_t{__uint_as_float(v[GB + 2 + q][2]), __uint_as_float(v[GB + 2 + q][3])};
      }
      lds_bn_relu_store<GB, true>(pa, v, ok, sc2, sh2);
      if ((xci += BK) == C) {
        xci = 0;
        if (++xs == a.S) {
          xs = 0;
          ++xr;
        }
      }
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (f + D < total) issue((f + D) % NS);
    const char* st = smem + (f % NS) * STAGE;
#pragma unroll
    for (int kh = 0; kh < BK / 32; ++kh) {
      const int slot = ((kh * 4 + fk) ^ fswz) * 16;
      bf16x8_t af[MI], bfr[MJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = *reinterpret_cast<const bf16x8_t*>(st + aoff[i] + slot);
#pragma unroll
      for (int j = 0; j < MJ; ++j) bfr[j] = *reinterpret_cast<const bf16x8_t*>(st + boffl[j] + slot);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < MJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("" ::: "memory");
    if (++kst == T) {
      epilogue(ctile);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < MJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      kst = 0;
      if (++ctile < ntile) {
        set_compute_geom(ctile);
        xr = xs = xci = 0;
      }
    }
  }
}

template <int BP, int BC, int WAVES_P, int NS, bool PRO, bool RES, int ST>
static int launch(DrnConvFwdArgs* a, const void* zero, int tpb, hipStream_t stream) {
  constexpr int LDS0 = NS * (BC + BP) * 128;
  const int lds = LDS0 + (PRO ? 8 * a->C : 0);
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  auto kern = conv_mt_kernel<BP, BC, WAVES_P, NS, PRO, RES, ST>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  const int M = a->N * a->P * a->Q;
  const int tiles_p = (M + BP - 1) / BP;
  const int ntiles = tiles_p * ((a->K + BC - 1) / BC);
  a->tiles_p = tiles_p;
  const int grid = (ntiles + tpb - 1) / tpb;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, stream, *a, zero, ntiles, tpb);
  return (int)hipGetLastError();
}

template <int BP, int BC, int WAVES_P, int NS>
static int dispatch(DrnConvFwdArgs* a, const void* zero, int tpb, hipStream_t s) {
  const bool pro = a->in_scale != nullptr;
  const bool res = a->residual != nullptr;
  const int st = a->stats == nullptr ? 0 : (a->bn_x != nullptr ? 2 : 1);
  if (pro && st == 2) return (int)hipErrorInvalidValue;
  // stages per tile must cover the pipeline depth (the next tile's first D stages are issued
  // while the current tile computes)
  if ((a->R * a->S * a->C) / 64 < NS - 1) return (int)hipErrorInvalidValue;
#define DRN_MT_ST(P, R)                                                 \
  switch (st) {                                                         \
    case 0: return launch<BP, BC, WAVES_P, NS, P, R, 0>(a, zero, tpb, s); \
    case 1: return launch<BP, BC, WAVES_P, NS, P, R, 1>(a, zero, tpb, s); \
    default: return launch<BP, BC, WAVES_P, NS, false, R, 2>(a, zero, tpb, s); \
  }
  if (pro) {
    if (res) { DRN_MT_ST(true, true) }
    DRN_MT_ST(true, false)
  }
  if (res) { DRN_MT_ST(false, true) }
  DRN_MT_ST(false, false)
#undef DRN_MT_ST
}

}  // namespace mt
}  // namespace drn

// Multi-tile configurations {BP, BC, WAVES_P, NS, tiles per block}; ids continue after the
// one-tile LDS-DMA configurations of conv_fwd.hip (DRN_GLDS_CONFIGS) in the autotuner's space.
#define DRN_MT_CONFIGS(X) \
  X(0, 128, 128, 2, 2, 4) \
  X(1, 128, 128, 2, 3, 4) \
  X(2, 64, 128, 1, 2, 4)  \
  X(3, 64, 128, 1, 3, 4)  \
  X(4, 128, 64, 2, 3, 4)  \
  X(5, 256, 64, 4, 2, 4)  \
  X(6, 64, 128, 1, 2, 8)  \
  X(7, 128, 128, 2, 2, 8) \
  X(8, 64, 64, 2, 3, 4)

DRN_API int drn_conv_mt_num_cfgs() { return 9; }

// Whether the multi-tile kernel family supports this convolution (LDS-DMA constraints plus the
// register epilogue's feature set: no in-kernel BN finalize, no sibling-phase zero fill).
DRN_API int drn_conv_mt_ok(const DrnConvFwdArgs* a) {
  return a->C % 64 == 0 && a->K % 8 == 0 && a->dil == 1 && a->fin_cnt == nullptr && a->out_fill == 0 &&
         (a->in_scale == nullptr || (a->C <= 4096 && a->relu_in != 0)) &&
         !(a->in_scale != nullptr && a->bn_x != nullptr) && a->bnb_x == nullptr;
}

DRN_API int drn_conv_mt(int cfg, DrnConvFwdArgs* a, const void* zero, hipStream_t s) {
  if (!drn_conv_mt_ok(a) || zero == nullptr) return (int)hipErrorInvalidValue;
  if (a->in_fin.stats != nullptr &&
      (a->in_scale == nullptr || a->in_fin.C != a->C || a->in_fin.G < 1 || a->in_fin.G > DRN_BN_FIN_GMAX))
    return (int)hipErrorInvalidValue;
  switch (cfg) {
#define DRN_X(id, bp, bc, wpv, ns, tpb) \
  case id:                              \
    return drn::mt::dispatch<bp, bc, wpv, ns>(a, zero, tpb, s);
    DRN_MT_CONFIGS(DRN_X)
#undef DRN_X
    default:
      return (int)hipErrorInvalidValue;
  }
}
