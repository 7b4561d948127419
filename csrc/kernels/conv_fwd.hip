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
#include "drn_conv_epi.h"
#include <stdlib.h>

namespace drn {

// Optional per-workgroup timeline of the LDS-DMA conv kernel, compiled in only with
// -DDRN_CONV_TRACE (even a never-taken check costs ~2.5 % of the ResNet-50 step): record
// b = {start, main-loop end, end} in s_memrealtime ticks (100 MHz) + HW_ID / XCC_ID.
#ifdef DRN_CONV_TRACE
__device__ unsigned long long* g_conv_trace = nullptr;
#endif

// Nontemporal output stores / epilogue loads / operand DMA (scripts/nt_ab.py, runtime switches
// in an earlier revision): 2-5 % per conv in isolation for nt stores, no gain in the full step
// (the next layer reads the output), nt DMA of the reused operands slower everywhere -- and the
// runtime branches alone cost ~1 % of the step. Plain stores / loads.

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
      const int n = (int)drn_fdiv((uint32_t)m, a.fd_pq);
      const int rem = m - n * pq;
      const int p = (int)drn_fdiv((uint32_t)rem, a.fd_q);
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

  static_assert(BP * BC * 4 <= 2 * STAGE, "epilogue tile must fit the staging LDS");
  EpiPre<BP, BC> epre;
  epi_prefetch<BP, BC>(a, m0, c0, M, epre);
  conv_epilogue<BP, BC, WP, WC, MI, MJ>(a, smem, acc, wp, wc, m0, c0, M, epre);
}

// ---------------------------------------------------------------------------------------
// LDS-DMA pipelined variant (C % 64 == 0, no fused prologue, dil 1): the main path of every
// ResNet convolution except the 8-channel stem and the narrow CIFAR stages.
//
// Operand tiles go global -> LDS directly with `global_load_lds_dwordx4` (no VGPR staging, no
// ds_write pass), NS LDS stages deep: stage t+NS-1 is in flight while stage t computes, retired
// by a counted `s_waitcnt vmcnt` + raw `s_barrier` (a __syncthreads() would drain the DMA
// queue). A stage is one 64-deep slice of k = (r, s, ci): since C % 64 == 0 it lies inside a
// single filter tap, so the tap / channel offset is wave-uniform and every lane only adds its
// pixel base; out-of-image taps and out-of-range rows read a 16-byte zero page (no branches).
// LDS image per stage: [BC + BP rows][128 B], 16-byte chunk j of row r stored at slot
// j ^ ((r >> 1) & 7) — the swizzle is applied on the per-lane SOURCE address (an LDS-DMA
// writes lane-linear), and makes the 16x16x32 fragment reads (ds_read_b128, 4 lane groups)
// bank-conflict free (checked exhaustively against the gfx950 lane-group table).
// ---------------------------------------------------------------------------------------
// Order of the k-stages (tap r, tap s, channel chunk ci) of the LDS-DMA kernels: taps outer,
// channel chunks inner (KRSC order; the chunk-outer order measured identical, profiles/r2_experiments.md).
template <int BK>
__device__ __forceinline__ void kstep_next(int& r, int& s, int& ci, int R, int S, int C) {
  if ((ci += BK) == C) {
    ci = 0;
    if (++s == S) {
      s = 0;
      ++r;
    }
  }
}

// PRO: the input is the RAW pre-BN tensor and the kernel applies relu(x * in_scale + in_shift)
// itself (pre-activation v2, reference resnet_model_official.py:113-119): after its counted
// vmcnt wait every lane rewrites the 16-byte pieces its own LDS-DMAs landed for the stage
// (ds_read_b128 -> 8 FMA + max -> ds_write_b128) before the stage's barrier, so no extra
// barrier and no extra HBM pass; pieces read from the zero page (padding, rows past M) are
// skipped and stay zero. The per-channel scale/shift are staged once into LDS behind the
// pipeline stages. Used for 1x1 consumers, where it replaces a full streaming BN-apply pass.
//
// SROW: narrow-input convolutions (C == 8: the ImageNet 7x7/2 stem on RGB padded to 8 channels;
// C == 16: the CIFAR first stage) stage ONE FILTER ROW r per step: the 8 16-byte chunks of a
// 64-deep stage are that row's S taps x C channels in KRSC / NHWC order (chunk lc = tap
// lc*8/C, channels (lc*8)%C ..+7; chunks past S*C/8 are zero-page pieces on both operands), so
// k = (r, s, c) keeps the reduction on the LDS-DMA path (per-lane pixel / tap validity) at
// 64/(S*C) of the work instead of falling back to the register-staged kernel. With PRO the
// fused BN prologue uses the lane's fixed chunk channel offset.
//
// KS (split-K, a.ksplit = S > 1): the grid is tiles x S; workgroup (tile, s) runs k-stages
// [s*T/S, (s+1)*T/S) of its tile, stores its fp32 partial accumulators to a.ks_ws and takes a
// ticket; the LAST arriver of a tile sums the S partials in split order (fixed order: bitwise
// reproducible whatever the arrival order) and runs the fused epilogue. No workgroup ever waits
// on another (no deadlock at any residency); the hand-off is the agent-scope release / acquire
// pair of the CDNA4 guide (G16). For under-filled grids (e.g. 196 tiles of a 7x7-stage 3x3
// conv on 256 CUs) it trades 64 KB of partial traffic per extra split for a full chip.
template <int BP, int BC, int WAVES_P, int NS, int NW = 4, bool PF = true, int BK = 64, bool PRO = false,
          bool SROW = false, int NH = 1, bool KS = false, bool IL = false>
__device__ __forceinline__ void conv_fwd_glds_tile(const DrnConvFwdArgs& a, const void* __restrict__ zero, char* smem,
                                                   int bid, int ksn, int ksi, int ks_stride, int t_beg_in,
                                                   int t_cnt_in) {
  static_assert(BK == 64 || BK == 32, "k per stage");
  static_assert(!SROW || BK == 64, "row-staged narrow convs: 64-deep stages");
  constexpr int NT = NW * 64;
  constexpr int WAVES_C = NW / WAVES_P;
  constexpr int WP = BP / WAVES_P, WC = BC / WAVES_C;
  constexpr int MI = WC / 16, MJ = WP / 16;
  constexpr int ROWB = BK * 2;              // bytes of one LDS row (BK bf16 of k)
  constexpr int CPR = BK / 8;               // 16-byte chunks per row
  constexpr int RPG = 1024 / ROWB;          // rows per glds wave-instruction (1 KiB)
  constexpr int STAGE = (BC + BP) * ROWB;
  constexpr int GA = BC / (RPG * NW), GB = BP / (RPG * NW);  // glds wave-instructions per stage
  constexpr int G = GA + GB;
  constexpr int D = NS - 1;                 // stages in flight ahead of the computing one
  static_assert(WAVES_P * WAVES_C == NW && MI >= 1 && MJ >= 1, "wave layout");
  static_assert(GA * RPG * NW == BC && GB * RPG * NW == BP, "rows must split evenly over the waves");
  static_assert(NS >= 2 && G * (D > 1 ? D - 1 : 1) < 64, "pipeline depth");
  static_assert(NH == 1 || (!PF && !SROW), "sliced epilogue: big-tile plain / PRO kernels only");

#ifdef DRN_CONV_TRACE
  unsigned long long* const trace = g_conv_trace;
  unsigned long long t_start = 0;
  if (trace != nullptr) t_start = drn_realtime();
#endif
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably uniform: LDS-DMA destinations stay scalar
  const int M = a.N * a.P * a.Q;
  const int C = a.C;
  const int Ktot = a.R * a.S * C;
  const int ntc = (a.K + BC - 1) / BC;
  static_assert(!KS || !SROW, "split-K: plain / fused-BN-prologue inputs");
  const int tc = bid % ntc;
  const int tp = bid / ntc;
  const int m0 = tp * BP;
  const int c0 = tc * BC;

  // ---- per-lane loader state ----
  const int lrow = lane / CPR;
  const int lpc = lane % CPR;
  const bf16_t* __restrict__ xg = reinterpret_cast<const bf16_t*>(a.x);
  const bf16_t* wsrc[GA];
  int alc[GA];  // SROW: the lane's logical chunk = filter tap s of its weight rows
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int row = RPG * NW * i + RPG * wave + lrow;
    const int lc = lpc ^ glds_swz<BK>(row);
    const int c = c0 + row;
    alc[i] = lc;
    wsrc[i] = c < a.K ? reinterpret_cast<const bf16_t*>(a.w) + (size_t)c * Ktot + (SROW ? 0 : lc * 8) : nullptr;
  }
  int boff[GB], bh[GB], bw[GB], blc[GB];
#pragma unroll
  for (int i = 0; i < GB; ++i) {
    const int row = RPG * NW * i + RPG * wave + lrow;
    const int lc = lpc ^ glds_swz<BK>(row);  // (BC + row) has the same swizzle bits
    blc[i] = lc;
    const int m = m0 + row;
    if (m < M) {
      const int pq = a.P * a.Q;
      const int n = (int)drn_fdiv((uint32_t)m, a.fd_pq);
      const int rem = m - n * pq;
      const int p = (int)drn_fdiv((uint32_t)rem, a.fd_q);
      const int q = rem - p * a.Q;
      bh[i] = p * a.stride - a.pad_h;
      bw[i] = q * a.stride - a.pad_w;
      boff[i] = ((n * a.H + bh[i]) * a.W + bw[i]) * C + (SROW ? 0 : lc * 8);
    } else {
      bh[i] = -(1 << 28);
      bw[i] = 0;
      boff[i] = 0;
    }
  }
  // Uniform-base fast path (cf. conv_wgrad.hip: per-piece address arithmetic, not the matrix
  // pipe, bounded the main loop): for a 1x1 unpadded convolution every B row of a tile that lies
  // wholly inside the output is a valid pixel for the whole reduction, and with a full channel
  // tile every A row is a real filter -- such stages issue each piece as a wave-uniform stage base
  // plus a per-lane offset fixed for the whole kernel, with no per-lane test.
  const bool fast_b = !SROW && a.R == 1 && a.S == 1 && a.pad_h == 0 && a.pad_w == 0 && m0 + BP <= M;
  const bool fast_a = !SROW && c0 + BC <= a.K;
  uint32_t aoff_w[GA], boff_x[GB];
#pragma unroll
  for (int i = 0; i < GA; ++i)
    aoff_w[i] = (uint32_t)((RPG * NW * i + RPG * wave + lrow) * Ktot + (lpc ^ glds_swz<BK>(RPG * NW * i + RPG * wave + lrow)) * 8);
#pragma unroll
  for (int i = 0; i < GB; ++i) boff_x[i] = (uint32_t)boff[i];
  const bf16_t* __restrict__ w0 = reinterpret_cast<const bf16_t*>(a.w) + (size_t)c0 * Ktot;
  // wave-uniform k iterator of the next stage to issue: k offset, tap (r, s), channel offset
  int ik = 0, ir = 0, is = 0, ici = 0;
  int t_beg = 0, t_cnt = 0;  // KS: this split's / stream-K segment's k-stage range
  if constexpr (KS) {
    t_beg = t_beg_in;
    t_cnt = t_cnt_in;
    ik = t_beg * BK;
    const int tap = ik / C;
    ici = ik - tap * C;
    ir = tap / a.S;
    is = tap - ir * a.S;
  }

  auto issue = [&](int slot) {
    char* st = smem + slot * STAGE;
    if constexpr (SROW) {  // stage = filter row ir; chunk lc = (tap lc*8/C, channels (lc*8)%C)
      // (C == 4, packed stem: stage = filter rows 2ir, 2ir+1, chunks 0-3 / 4-7 = their 4 tap pairs)
      const int SC = a.S * C;
      const int rps = C == 4 ? 2 : 1;
#pragma unroll
      for (int i = 0; i < GA; ++i) {
        const int sub = rps == 2 ? alc[i] >> 2 : 0, lc = rps == 2 ? alc[i] & 3 : alc[i];
        const int row = ir * rps + sub;
        const void* src = (wsrc[i] && lc * 8 < SC && row < a.R) ? (const void*)(wsrc[i] + row * SC + lc * 8) : zero;
        glds16(src, st + (RPG * NW * i + RPG * wave) * ROWB);
      }
#pragma unroll
      for (int i = 0; i < GB; ++i) {
        const int sub = rps == 2 ? blc[i] >> 2 : 0, lc = rps == 2 ? blc[i] & 3 : blc[i];
        const int row = ir * rps + sub;
        const int h = bh[i] + row, w = bw[i] + lc * 8 / C;
        const bool ok = lc * 8 < SC && row < a.R && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
        const void* src = ok ? (const void*)(xg + (boff[i] + row * a.W * C + lc * 8)) : zero;
        glds16(src, st + (BC + RPG * NW * i + RPG * wave) * ROWB);
      }
      ++ir;
      return;
    }
    if (fast_a) {
      const bf16_t* __restrict__ ws_ = w0 + ik;
#pragma unroll
      for (int i = 0; i < GA; ++i) glds16(ws_ + aoff_w[i], st + (RPG * NW * i + RPG * wave) * ROWB);
    } else {
#pragma unroll
      for (int i = 0; i < GA; ++i) {
        const void* src = wsrc[i] ? (const void*)(wsrc[i] + ik) : zero;
        glds16(src, st + (RPG * NW * i + RPG * wave) * ROWB);
      }
    }
    const int tap_off = (ir * a.W + is) * C + ici;
    if (fast_b) {
      const bf16_t* __restrict__ xs_ = xg + tap_off;
#pragma unroll
      for (int i = 0; i < GB; ++i) glds16(xs_ + boff_x[i], st + (BC + RPG * NW * i + RPG * wave) * ROWB);
    } else {
#pragma unroll
      for (int i = 0; i < GB; ++i) {
        const int h = bh[i] + ir, w = bw[i] + is;
        const bool ok = (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
        const void* src = ok ? (const void*)(xg + (boff[i] + tap_off)) : zero;
        glds16(src, st + (BC + RPG * NW * i + RPG * wave) * ROWB);
      }
    }
    kstep_next<BK>(ir, is, ici, a.R, a.S, C);
    ik = (ir * a.S + is) * C + ici;
  };
  // IL: the same stage issued one LDS-DMA piece at a time (g = 0 .. G-1, A pieces then B pieces),
  // interleaved with the MFMAs of the computing stage by the main loop; then
  // issue_advance() moves the k iterator
  auto issue_piece = [&](int slot, int g) {
    char* st = smem + slot * STAGE;
    if (g < GA) {
      const void* src = wsrc[g] ? (const void*)(wsrc[g] + ik) : zero;
      glds16(src, st + (RPG * NW * g + RPG * wave) * ROWB);
      return;
    }
    const int i = g - GA;
    const int h = bh[i] + ir, w = bw[i] + is;
    const bool ok = (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
    const int off = boff[i] + (ir * a.W + is) * C + ici;
    glds16(ok ? (const void*)(xg + off) : zero, st + (BC + RPG * NW * i + RPG * wave) * ROWB);
  };
  auto issue_advance = [&]() {
    kstep_next<BK>(ir, is, ici, a.R, a.S, C);
    ik = (ir * a.S + is) * C + ici;
  };

  const int wp = wave % WAVES_P;
  const int wc = wave / WAVES_P;
  f32x4_t acc[MI][MJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < MJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets (bytes, within a stage): row r, logical chunk kc -> slot kc ^ ((r>>1)&7)
  const int fr = lane & 15, fk = lane >> 4;
  int aoff[MI], boffl[MJ];
#pragma unroll
  for (int i = 0; i < MI; ++i) aoff[i] = (wc * WC + i * 16 + fr) * ROWB;
#pragma unroll
  for (int j = 0; j < MJ; ++j) boffl[j] = (BC + wp * WP + j * 16 + fr) * ROWB;
  const int swz = glds_swz<BK>(fr);  // fragment row groups are 16-aligned: the swizzle bits are fr's

  const int T = KS ? t_cnt : SROW ? (C == 4 ? (a.R + 1) / 2 : a.R) : Ktot / BK;
  // fused-BN operands: [scale C][shift C] fp32 behind the stages, written AFTER the first
  // pipeline stages are issued (their LDS-DMA latency covers the parameter loads / finalize)
  // (behind the stages actually used: a convolution with fewer k-stages than NS - e.g. a 1x1
  // over 64 channels, T = 1 - gets only T stage slots, so more workgroups fit a CU)
  float* const ssl = reinterpret_cast<float*>(smem + (T < NS ? T : NS) * STAGE);
  // the lane's logical 16-byte chunk of the B rows it loads: identical for every piece i
  // (RPG * NW rows apart leave the swizzle bits unchanged)
  static_assert((RPG * NW) % 16 == 0, "piece stride must preserve the swizzle bits");
  const int lcb = lpc ^ glds_swz<BK>(RPG * wave + lrow);
  int xr = 0, xs = 0, xci = 0;  // tap / channel offset of the stage being transformed
  if constexpr (KS) {
    xr = ir;
    xs = is;
    xci = ici;
  }
  EpiPre<BP, BC / NH, NT, PF> epre;
  if constexpr (NH == 1)
    epi_prefetch<BP, BC, NT, PF>(a, m0, c0, M, epre);  // residual / BN inputs in flight during the main loop
#pragma unroll
  for (int s = 0; s < D; ++s)
    if (s < T) issue(s);
  if constexpr (PRO) {
    if (a.in_fin.stats != nullptr) {
      // consumer-side BN finalize: scale/shift straight from the statistics replicas (the
      // first workgroup of the publishing launch also writes them out for later kernels)
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
  for (int t = 0; t < T; ++t) {
    // retire stage t: the stages issued after it (up to D-1) may stay in flight
    if (t + D - 1 < T) wait_vmcnt<G * (D - 1)>();
    else wait_vmcnt<0>();
    if constexpr (PRO) {
      char* sw = smem + (t % NS) * STAGE;
      // one LDS round trip: this stage's scale/shift and the lane's landed pieces together
      // (SROW: the lane's chunk maps to a fixed tap / channel group in every stage)
      const uint32_t sp = lds_addr(ssl + (SROW ? (lcb * 8) % C : xci + lcb * 8));
      u32x4_t v[GB + 4];
      v[GB] = lds_read16(sp);
      v[GB + 1] = lds_read16(sp + 16);
      v[GB + 2] = lds_read16(sp + 4 * C);
      v[GB + 3] = lds_read16(sp + 4 * C + 16);
      uint32_t pa[GB], ok = 0;
#pragma unroll
      for (int i = 0; i < GB; ++i) {
        const int h = bh[i] + xr, w = bw[i] + (SROW ? lcb * 8 / C : xs);
        const bool chunk_ok = !SROW || lcb * 8 < a.S * C;
        ok |= (chunk_ok && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W) ? (1u << i) : 0u;
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
      if (SROW) ++xr;
      else kstep_next<BK>(xr, xs, xci, a.R, a.S, C);
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const char* st = smem + (t % NS) * STAGE;
    if constexpr (IL && !SROW) {
      // the next stage's LDS-DMA pieces spread between this stage's MFMAs: the DMA issue cost
      // (~0.1 us per piece per wave) hides under the matrix pipe instead of idling it after
      // every barrier while all waves issue in lockstep
      const bool more = t + D < T;
      const int nslot = (t + D) % NS;
      constexpr int Q = (BK / 32) * MI * MJ;
      constexpr int STEP = Q / (G + 1) > 0 ? Q / (G + 1) : 1;
#pragma unroll
      for (int kh = 0; kh < BK / 32; ++kh) {
        const int slot = ((kh * 4 + fk) ^ swz) * 16;
        bf16x8_t af[MI], bfr[MJ];
#pragma unroll
        for (int i = 0; i < MI; ++i) af[i] = *reinterpret_cast<const bf16x8_t*>(st + aoff[i] + slot);
#pragma unroll
        for (int j = 0; j < MJ; ++j) bfr[j] = *reinterpret_cast<const bf16x8_t*>(st + boffl[j] + slot);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < MJ; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
            const int q = (kh * MI + i) * MJ + j + 1;
            if (q % STEP == 0 && q / STEP <= G && more) {
              __builtin_amdgcn_sched_barrier(0);
              issue_piece(nslot, q / STEP - 1);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
      }
      if (Q / STEP < G && more) {  // (fewer MFMAs than pieces: the rest now)
#pragma unroll
        for (int g = Q / STEP; g < G; ++g) issue_piece(nslot, g);
      }
      if (more) issue_advance();
      asm volatile("" ::: "memory");
      continue;
    }
    if (t + D < T) issue((t + D) % NS);
#pragma unroll
    for (int kh = 0; kh < BK / 32; ++kh) {
      const int slot = ((kh * 4 + fk) ^ swz) * 16;
      bf16x8_t af[MI], bfr[MJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = *reinterpret_cast<const bf16x8_t*>(st + aoff[i] + slot);
#pragma unroll
      for (int j = 0; j < MJ; ++j) bfr[j] = *reinterpret_cast<const bf16x8_t*>(st + boffl[j] + slot);
      if constexpr (NW == 8) __builtin_amdgcn_s_setprio(1);  // keeps the MFMA cluster together (guide T5)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < MJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      if constexpr (NW == 8) __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("" ::: "memory");
  }
  __syncthreads();  // all fragment reads done before the epilogue reuses the LDS
  if constexpr (KS) {
    if (ksn > 1) {
      // publish this split's partial tile (lane-linear: 1 KB per wave-instruction), ticket
      constexpr int PER = NT * MI * MJ * 4;  // floats per partial tile (= BP * BC)
      float* ws = a.ks_ws + (size_t)bid * ks_stride * PER;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < MJ; ++j)
          *reinterpret_cast<f32x4_t*>(ws + (size_t)ksi * PER + ((i * MJ + j) * NT + tid) * 4) = acc[i][j];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      int* flag = reinterpret_cast<int*>(smem);
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned t = __hip_atomic_fetch_add(a.ks_tickets + bid, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = t + 1u == (unsigned)ksn;
        if (last) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __hip_atomic_store(a.ks_tickets + bid, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
        }
        *flag = last;
      }
      __syncthreads();
      if (!*flag) return;
      __syncthreads();  // every wave has read the flag before the epilogue reuses this LDS word
      // the tile's sum in split order (fixed: bitwise reproducible)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < MJ; ++j) {
          f32x4_t sum = f32x4_t{0.f, 0.f, 0.f, 0.f};
          for (int s = 0; s < ksn; ++s)
            sum += s == ksi ? acc[i][j]
                            : *reinterpret_cast<const f32x4_t*>(ws + (size_t)s * PER + ((i * MJ + j) * NT + tid) * 4);
          acc[i][j] = sum;
        }
    }
  }
#ifdef DRN_CONV_TRACE
  unsigned long long t_loop = 0;
  if (trace != nullptr) t_loop = drn_realtime();
#endif
  // (the launcher sizes the dynamic LDS for max(NS * STAGE, BP * BC * 4 / NH))
  if constexpr (NH == 1) conv_epilogue<BP, BC, WP, WC, MI, MJ, NT, PF>(a, smem, acc, wp, wc, m0, c0, M, epre);
  else conv_epilogue_sliced<BP, BC, WP, WC, MI, MJ, NT, NH>(a, smem, acc, wp, wc, m0, c0, M);
#ifdef DRN_CONV_TRACE
  if (trace != nullptr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
      const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);
      unsigned long long* r = trace + 4 * (size_t)blockIdx.x;
      r[0] = t_start;
      r[1] = t_loop;
      r[2] = drn_realtime();
      r[3] = ((unsigned long long)xcc << 32) | hw;
    }
  }
#endif
}

template <int BP, int BC, int WAVES_P, int NS, int NW = 4, bool PF = true, int BK = 64, bool PRO = false,
          bool SROW = false, int NH = 1, bool KS = false, bool IL = false>
__global__ __launch_bounds__(NW * 64) void conv_fwd_glds_kernel(DrnConvFwdArgs a, const void* __restrict__ zero) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int lin = xcd_remap(blockIdx.x, gridDim.x);  // (a tile's splits stay on one XCD)
  if constexpr (KS) {
    const int ksn = a.ksplit;
    const int bid = lin / ksn, ksi = lin - bid * ksn;
    const int t_all = (a.R * a.S * a.C) / BK;
    const int t_beg = (int)((long)ksi * t_all / ksn);
    const int t_cnt = (int)((long)(ksi + 1) * t_all / ksn) - t_beg;
    conv_fwd_glds_tile<BP, BC, WAVES_P, NS, NW, PF, BK, PRO, SROW, NH, KS, IL>(a, zero, smem, bid, ksn, ksi, ksn, t_beg,
                                                                             t_cnt);
  } else {
    conv_fwd_glds_tile<BP, BC, WAVES_P, NS, NW, PF, BK, PRO, SROW, NH, KS, IL>(a, zero, smem, lin, 1, 0, 1, 0, 0);
  }
}

// Stream-K (a.sk_blocks = gridDim.x > 0): the U = tiles x k-stages units are cut into gridDim.x
// equal contiguous ranges, one per workgroup; a workgroup walks the tile segments of its range
// (tile-major, k-minor). A tile whose units span several workgroups is finished by its last
// arriving contributor (partials summed in contributor order: bitwise reproducible); nobody
// waits. Every CU gets the same number of MFMA k-stages whatever the tile count (98 / 196 / 392
// tiles of the ResNet-50 layers against 256 CUs).
template <int BP, int BC, int WAVES_P, int NS, int NW = 4, int BK = 64, bool PRO = false, int NH = 1, bool IL = false>
__global__ __launch_bounds__(NW * 64) void conv_fwd_glds_sk_kernel(DrnConvFwdArgs a, const void* __restrict__ zero) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  // (32-bit unit arithmetic: the launcher checks tiles x k-stages x grid < 2^31)
  const unsigned G = gridDim.x;
  const unsigned b = xcd_remap(blockIdx.x, G);  // consecutive ranges (shared tiles) on one XCD
  const unsigned M = a.N * a.P * a.Q;
  const unsigned tiles = ((M + BP - 1) / BP) * ((a.K + BC - 1) / BC);
  const unsigned t_all = (a.R * a.S * a.C) / BK;
  const unsigned U = tiles * t_all;
  auto owner = [&](unsigned u) { return ((u + 1) * G - 1) / U; };  // workgroup whose range holds unit u
  unsigned u = __builtin_amdgcn_readfirstlane(b * U / G);
  const unsigned uend = __builtin_amdgcn_readfirstlane((b + 1) * U / G);
  bool first = true;
  while (u < uend) {
    const unsigned tile = __builtin_amdgcn_readfirstlane(u / t_all);
    const unsigned tbase = tile * t_all;
    const unsigned tend = tbase + t_all;
    const unsigned t0 = u - tbase, t1 = (tend < uend ? tend : uend) - tbase;  // (uniform)
    const unsigned bf = __builtin_amdgcn_readfirstlane(owner(tbase));
    const unsigned bl = __builtin_amdgcn_readfirstlane(owner(tend - 1));
    if (!first) {
      __syncthreads();  // the previous segment's LDS use is over
      // a consumer-side BN finalize publishes (and moves the moving averages) once: in the
      // first segment of workgroup 0, not again if that workgroup's range spans several tiles
      if constexpr (PRO) a.in_fin.publish = 0;
    }
    // (no epilogue-operand prefetch: most segments end in a partial tile, not an epilogue)
    conv_fwd_glds_tile<BP, BC, WAVES_P, NS, NW, false, BK, PRO, false, NH, true, IL>(
        a, zero, smem, (int)tile, (int)(bl - bf + 1), (int)(b - bf), a.ksplit, (int)t0, (int)(t1 - t0));
    first = false;
    u = tend;
  }
}

// ---------------- narrow-output convs (K = 16 / 32): operands straight to registers ----------------
// The CIFAR stage-1 convs (64 -> 16 1x1, 16 -> 16 3x3 and their data gradients; reference
// resnet_model_official.py:255-266, 16 filters per stage-1 bottleneck) have so few output channels
// that an LDS-staged tile is mostly overhead: the weights are 2-9 KB and each pixel row feeds one
// 16-channel MFMA column. Here a wave owns WP = 16 MJ output pixels x 16 MI channels; the A
// fragments (weights, every k-step) are loaded into registers once, the B fragments (8 channels
// of one pixel per lane: one 16-byte load, zero for padding) come straight from global memory,
// every k-step issued before the first MFMA (the kernel is bandwidth-bound: bytes in flight
// decide). A k-step is 32 k; with C < 32 it spans 32 / C taps (taps paired, not channels padded).
// The fused BN-apply (+ReLU) prologue runs on the fragments in registers (its per-channel
// parameters staged in LDS behind the epilogue tile); the epilogue is the shared LDS-staged one
// (residual, statistics, BN-backward reduction, finalize).
template <int MI, int MJ, int NW, int KMAX, bool PRO>
__global__ __launch_bounds__(NW * 64) void conv_fwd_nk_kernel(DrnConvFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NT = NW * 64, WP = 16 * MJ, BP = WP * NW, BC = 16 * MI;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4;
  const int M = a.N * a.P * a.Q;
  const int C = a.C, RS = a.R * a.S;
  const int Ktot = RS * C;
  const int ksteps = (Ktot + 31) >> 5;
  const int cshift = __builtin_ctz(C);  // (the launcher requires a power-of-two C)
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * BP;
  const bf16_t* __restrict__ xg = reinterpret_cast<const bf16_t*>(a.x);
  const bf16_t* __restrict__ wg = reinterpret_cast<const bf16_t*>(a.w);
  float* ssl = reinterpret_cast<float*>(smem + BP * BC * 4);  // [scale C][shift C]
  if constexpr (PRO) {
    if (a.in_fin.stats != nullptr) {
      // consumer-side BN finalize straight from the statistics replicas (the first workgroup of
      // a publishing launch also writes scale / shift out for later kernels)
      const bool pub = a.in_fin.publish && blockIdx.x == 0;
      for (int c = tid; c < C; c += NT) drn_bn_fin_fwd(a.in_fin, c, pub, ssl[c], ssl[C + c]);
    } else {
      for (int c = tid; c < C; c += NT) {
        ssl[c] = a.in_scale[c];
        ssl[C + c] = a.in_shift[c];
      }
    }
  }
  // this lane's output pixels
  int pb[MJ], ph[MJ], pw[MJ];
#pragma unroll
  for (int j = 0; j < MJ; ++j) {
    const int m = m0 + wave * WP + j * 16 + (lane & 15);
    if (m < M) {
      const int n = (int)drn_fdiv((uint32_t)m, a.fd_pq);
      const int rem = m - n * (a.P * a.Q);
      const int p = (int)drn_fdiv((uint32_t)rem, a.fd_q);
      const int q = rem - p * a.Q;
      ph[j] = p * a.stride - a.pad_h;
      pw[j] = q * a.stride - a.pad_w;
      pb[j] = ((n * a.H + ph[j]) * a.W + pw[j]) * C;
    } else {
      ph[j] = -(1 << 28);
      pw[j] = 0;
      pb[j] = 0;
    }
  }
  // every k-step's B fragments in flight first, then the weights
  uint4 xb[KMAX][MJ];
  unsigned long long okm = 0;  // bit t * MJ + j: fragment (t, j) inside the input (PRO: transform it)
#pragma unroll
  for (int t = 0; t < KMAX; ++t) {
    if (t < ksteps) {
      const int k = t * 32 + g * 8;
      const int tap = k >> cshift;
      const int ci = k - (tap << cshift);
      const int r = tap / a.S, sx = tap - r * a.S;
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        const int h = ph[j] + r, w = pw[j] + sx;
        const bool ok = tap < RS && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
        xb[t][j] = ok ? *reinterpret_cast<const uint4*>(xg + pb[j] + (r * a.W + sx) * C + ci)
                      : make_uint4(0u, 0u, 0u, 0u);
        if (ok) okm |= 1ull << (t * MJ + j);
      }
    }
  }
  bf16x8_t wa[MI][KMAX];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int t = 0; t < KMAX; ++t) {
      const int k = t * 32 + g * 8;
      const uint4 v = (t < ksteps && k < Ktot)
                          ? *reinterpret_cast<const uint4*>(wg + (size_t)(i * 16 + (lane & 15)) * Ktot + k)
                          : make_uint4(0u, 0u, 0u, 0u);
      wa[i][t] = __builtin_bit_cast(bf16x8_t, v);
    }
  if constexpr (PRO) __syncthreads();  // BN parameters staged
  f32x4_t acc[MI][MJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < MJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < KMAX; ++t) {
    if (t < ksteps) {
      bf16x8_t bv[MJ];
      if constexpr (PRO) {
        const int k = t * 32 + g * 8;
        const int ci = k & (C - 1);
        float sc[8], sh[8];
#pragma unroll
        for (int e = 0; e < 8; e += 4) {
          const float4 s4 = *reinterpret_cast<const float4*>(ssl + ci + e);
          const float4 h4 = *reinterpret_cast<const float4*>(ssl + C + ci + e);
          sc[e] = s4.x, sc[e + 1] = s4.y, sc[e + 2] = s4.z, sc[e + 3] = s4.w;
          sh[e] = h4.x, sh[e + 1] = h4.y, sh[e + 2] = h4.z, sh[e + 3] = h4.w;
        }
#pragma unroll
        for (int j = 0; j < MJ; ++j) {
          float f[8];
          unpack8(xb[t][j], f);
          const bool ok = (okm >> (t * MJ + j)) & 1ull;  // padding stays zero (BN-apply first)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float v = f[e] * sc[e] + sh[e];
            if (a.relu_in) v = v > 0.f ? v : 0.f;
            f[e] = ok ? v : 0.f;
          }
          bv[j] = __builtin_bit_cast(bf16x8_t, pack8(f));
        }
      } else {
#pragma unroll
        for (int j = 0; j < MJ; ++j) bv[j] = __builtin_bit_cast(bf16x8_t, xb[t][j]);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < MJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i][t], bv[j], acc[i][j], 0, 0, 0);
    }
  }
  EpiPre<BP, BC, NT, false> e;
  epi_prefetch<BP, BC, NT, false>(a, m0, 0, M, e);
  conv_epilogue<BP, BC, WP, BC, MI, MJ, NT, false>(a, smem, acc, wave, 0, m0, 0, M, e);
}

static int cfin_max_blocks();

// id -> (MI, MJ): 16-channel outputs with 32 / 64 pixels per wave, 32-channel with 16 / 32 / 64
#define DRN_NK_CONFIGS(X) X(0, 1, 2) X(1, 1, 4) X(2, 2, 1) X(3, 2, 2) X(4, 2, 4)
#define DRN_NK_NCFG 5
#define DRN_NK_CFG0 200  // configuration id of NK config 0 (DrnConvFwdArgs::cfg)

template <int MI, int MJ, bool PRO, int KMAX>
static int launch_conv_nk_k(DrnConvFwdArgs* a, hipStream_t stream) {
  constexpr int NW = 4, BP = 16 * MJ * NW, BC = 16 * MI;
  static_assert(BP % (NW * 64 / (BC / 8)) == 0, "epilogue rows per pass must divide the tile");
  const int M = a->N * a->P * a->Q;
  const int LDS = BP * BC * 4 + (PRO ? 8 * a->C : 0);
  if (LDS > 160 * 1024) return (int)hipErrorInvalidValue;
  auto kern = conv_fwd_nk_kernel<MI, MJ, NW, KMAX, PRO>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  a->tiles_p = (M + BP - 1) / BP;
  drn::launch(kern, dim3(a->tiles_p), dim3(NW * 64), LDS, stream, *a);
  return (int)hipGetLastError();
}

template <int MI, int MJ, bool PRO>
static int launch_conv_nk_p(DrnConvFwdArgs* a, hipStream_t stream) {
  const int ksteps = (a->R * a->S * a->C + 31) / 32;
  if (ksteps <= 2) return launch_conv_nk_k<MI, MJ, PRO, 2>(a, stream);
  if (ksteps <= 5) return launch_conv_nk_k<MI, MJ, PRO, 5>(a, stream);
  if (ksteps <= 9) return launch_conv_nk_k<MI, MJ, PRO, 9>(a, stream);
  return (int)hipErrorInvalidValue;
}

static int nk_cfg_mi(int id) {
  switch (id) {
#define DRN_X(id, mi, mj) \
  case id:                \
    return mi;
    DRN_NK_CONFIGS(DRN_X)
#undef DRN_X
    default:
      return 0;
  }
}

static int nk_cfg_mj(int id) {
  switch (id) {
#define DRN_X(id, mi, mj) \
  case id:                \
    return mj;
    DRN_NK_CONFIGS(DRN_X)
#undef DRN_X
    default:
      return 1;
  }
}

static int launch_conv_nk(int id, DrnConvFwdArgs* a, hipStream_t stream) {
  const int mi = nk_cfg_mi(id);
  if (mi == 0 || a->K != 16 * mi || a->dil != 1 || a->ksplit > 1 || a->sk_blocks > 0 ||
      a->C < 8 || (a->C & (a->C - 1)) != 0 || (a->R * a->S * a->C + 31) / 32 > 9)
    return (int)hipErrorInvalidValue;
  if (a->in_fin.stats != nullptr && (a->N * a->P * a->Q + 16 * 4 * nk_cfg_mj(id) - 1) / (16 * 4 * nk_cfg_mj(id)) >
                                         cfin_max_blocks()) {  // big grid: the finalize as its own launch
    if (a->in_fin.publish) {
      const int rc = drn_bn_fin_fwd_launch(&a->in_fin, stream);
      if (rc) return rc;
    }
    DrnConvFwdArgs b = *a;
    b.in_fin.stats = nullptr;
    const int rc = launch_conv_nk(id, &b, stream);
    a->tiles_p = b.tiles_p;
    return rc;
  }
  const bool pro = a->in_scale != nullptr;
  switch (id) {
#define DRN_X(id, mi, mj) \
  case id:                \
    return pro ? launch_conv_nk_p<mi, mj, true>(a, stream) : launch_conv_nk_p<mi, mj, false>(a, stream);
    DRN_NK_CONFIGS(DRN_X)
#undef DRN_X
    default:
      return (int)hipErrorInvalidValue;
  }
}

// partial-tile slots a stream-K launch needs per tile: the most workgroup ranges one tile's T
// units touch (the kernel's owner() map, tile by tile); 0 = invalid (more workgroups than units:
// empty ranges, or 32-bit unit arithmetic overflow)
static int sk_slots(int tiles, int T, int G) {
  const long U = (long)tiles * T;
  if (G < 1 || T < 1 || U < G || U * (long)(G + 1) >= (1l << 31)) return 0;
  auto owner = [&](long u) { return ((u + 1) * G - 1) / U; };
  long n = 1;
  for (long t = 0; t < tiles; ++t) {
    const long c = owner(t * T + T - 1) - owner(t * T) + 1;
    n = c > n ? c : n;
  }
  return (int)n;
}

// largest grid that finalizes its input BatchNorm in the prologue (profiles/r4_cfin_work_ab.txt)
static int cfin_max_blocks() { return 2048; }

// ... and a grid whose workgroups would each re-derive many channels: the prologue finalize
// reads G replicas x C channels per workgroup from L2 (ResNet-50 stage 4: 392 workgroups x 2048
// channels x 64 B = 51 MB, 8 dependent channel rounds per thread)
static long cfin_max_work() { return 1L << 19; }

template <int BP, int BC, int WAVES_P, int NS, int NW, bool PF, int BK, bool PRO, bool SROW = false, int NH = 1,
          bool KS = false, bool IL = false>
static int launch_conv_glds_pf(DrnConvFwdArgs* a, const void* zero, hipStream_t stream) {
  const int T = a->C == 4 ? (a->R + 1) / 2 : a->C == 8 || a->C == 16 ? a->R : (a->R * a->S * a->C) / BK;  // k-stages
                                                          // (SROW: filter rows; packed stem: row pairs)
  const int LDS0 = (T < NS ? T : NS) * (BC + BP) * BK * 2;  // stage slots actually used
  const int lds_main = LDS0 + (PRO ? 8 * a->C : 0);           // + fused-BN parameters
  const int LDS = lds_main > BP * BC * 4 / NH ? lds_main : BP * BC * 4 / NH;  // epilogue staging slice
  if (LDS > 160 * 1024) return (int)hipErrorInvalidValue;
  static bool attr_set = false;
  auto kern = conv_fwd_glds_kernel<BP, BC, WAVES_P, NS, NW, PF, BK, PRO, SROW, NH, KS, IL>;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  const int M = a->N * a->P * a->Q;
  const int tiles_p = (M + BP - 1) / BP;
  const int tiles_c = (a->K + BC - 1) / BC;
  a->tiles_p = tiles_p;
  if constexpr (KS) {
    if (a->sk_blocks > 0) {  // stream-K: sk_blocks workgroups, ksplit = partial slots per tile
      if (a->ks_ws == nullptr || a->ks_tickets == nullptr) return (int)hipErrorInvalidValue;
      const int need = sk_slots(tiles_p * tiles_c, T, a->sk_blocks);
      if (need == 0 || need > a->ksplit) return (int)hipErrorInvalidValue;
      auto skern = conv_fwd_glds_sk_kernel<BP, BC, WAVES_P, NS, NW, BK, PRO, NH, IL>;
      static bool sk_attr_set = false;
      if (!sk_attr_set) {
        hipFuncSetAttribute(reinterpret_cast<const void*>(skern), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
        sk_attr_set = true;
      }
      drn::launch(skern, dim3(a->sk_blocks), dim3(NW * 64), LDS, stream, *a, zero);
      return (int)hipGetLastError();
    }
  }
  const int ks = KS ? a->ksplit : 1;
  if (KS && (ks < 2 || T < ks || a->ks_ws == nullptr || a->ks_tickets == nullptr)) return (int)hipErrorInvalidValue;
  if (PRO && a->in_fin.stats != nullptr &&
      (tiles_p * tiles_c * ks > cfin_max_blocks() || (long)a->C * tiles_p * tiles_c * ks > cfin_max_work())) {
    // a large grid pays the in-prologue finalize once per workgroup wave: measured slower than
    // one separate finalize launch (ResNet-50 stage 1, 12544 workgroups: +11 us vs ~6 us)
    if (a->in_fin.publish) {
      const int rc = drn_bn_fin_fwd_launch(&a->in_fin, stream);
      if (rc) return rc;
    }
    DrnConvFwdArgs b = *a;
    b.in_fin.stats = nullptr;
    drn::launch(kern, dim3(tiles_p * tiles_c * ks), dim3(NW * 64), LDS, stream, b, zero);
    return (int)hipGetLastError();
  }
  drn::launch(kern, dim3(tiles_p * tiles_c * ks), dim3(NW * 64), LDS, stream, *a, zero);
  return (int)hipGetLastError();
}

template <int BP, int BC, int WAVES_P, int NS, int NW, int BK, bool IL>
static int launch_conv_glds_nh1(DrnConvFwdArgs* a, const void* zero, hipStream_t stream);

// split-K launch (a->ksplit > 1): plain / fused-BN-prologue inputs only
template <int BP, int BC, int WAVES_P, int NS, int NW, int BK, int NH, bool IL>
static int launch_conv_glds_ks(DrnConvFwdArgs* a, const void* zero, hipStream_t stream) {
  if (a->C == 4 || a->C == 8 || a->C == 16 || a->C % BK) return (int)hipErrorInvalidValue;
  // epilogue operands: prefetched by the (NH == 1) kernels that keep them in registers
  constexpr bool PFOK = NH == 1;
  const bool pf = PFOK && (a->residual != nullptr || a->bn_x != nullptr);
  if (a->in_scale != nullptr)
    return pf ? launch_conv_glds_pf<BP, BC, WAVES_P, NS, NW, PFOK, BK, true, false, NH, true, IL>(a, zero, stream)
              : launch_conv_glds_pf<BP, BC, WAVES_P, NS, NW, false, BK, true, false, NH, true, IL>(a, zero, stream);
  return pf ? launch_conv_glds_pf<BP, BC, WAVES_P, NS, NW, PFOK, BK, false, false, NH, true, IL>(a, zero, stream)
            : launch_conv_glds_pf<BP, BC, WAVES_P, NS, NW, false, BK, false, false, NH, true, IL>(a, zero, stream);
}

// epilogue operands (residual / BN-backward input) are prefetched only when present
template <int BP, int BC, int WAVES_P, int NS, int NW = 4, int BK = 64, int NH = 1, bool IL = false, bool KSOK = false>
static int launch_conv_glds(DrnConvFwdArgs* a, const void* zero, hipStream_t stream) {
  if (a->ksplit > 1 || a->sk_blocks > 0) {
    if constexpr (KSOK) return launch_conv_glds_ks<BP, BC, WAVES_P, NS, NW, BK, NH, IL>(a, zero, stream);
    return (int)hipErrorInvalidValue;
  }
  if constexpr (NH > 1) {  // big tiles: plain / fused-BN-prologue input, sliced epilogue, no prefetch
    if (a->C == 4 || a->C == 8 || a->C == 16 || a->C % BK) return (int)hipErrorInvalidValue;
    if (a->in_scale != nullptr)
      return launch_conv_glds_pf<BP, BC, WAVES_P, NS, NW, false, BK, true, false, NH, false, IL>(a, zero, stream);
    return launch_conv_glds_pf<BP, BC, WAVES_P, NS, NW, false, BK, false, false, NH, false, IL>(a, zero, stream);
  } else {
    return launch_conv_glds_nh1<BP, BC, WAVES_P, NS, NW, BK, IL>(a, zero, stream);
  }
}

template <int BP, int BC, int WAVES_P, int NS, int NW, int BK, bool IL>
static int launch_conv_glds_nh1(DrnConvFwdArgs* a, const void* zero, hipStream_t stream) {
  const bool pf = a->residual != nullptr || a->bn_x != nullptr;
  if (a->C == 4 || a->C == 8 || a->C == 16) {  // row-staged narrow conv (the stem, the CIFAR first stage)
    if constexpr (BK == 64 && !IL) {
      if (a->S * a->C > (a->C == 4 ? 32 : 64)) return (int)hipErrorInvalidValue;
      if (a->C == 4 && (a->S % 2 || a->in_scale != nullptr)) return (int)hipErrorInvalidValue;
      if (a->in_scale != nullptr)
        return pf ? launch_conv_glds_pf<BP, BC, WAVES_P, NS, NW, true, BK, true, true>(a, zero, stream)
                  : launch_conv_glds_pf<BP, BC, WAVES_P, NS, NW, false, BK, true, true>(a, zero, stream);
      return pf ? launch_conv_glds_pf<BP, BC, WAVES_P, NS, NW, true, BK, false, true>(a, zero, stream)
                : launch_conv_glds_pf<BP, BC, WAVES_P, NS, NW, false, BK, false, true>(a, zero, stream);
    }
    return (int)hipErrorInvalidValue;
  }
  if (a->C % BK) return (int)hipErrorInvalidValue;
  if (a->in_scale != nullptr)
    return pf ? launch_conv_glds_pf<BP, BC, WAVES_P, NS, NW, true, BK, true, false, 1, false, IL>(a, zero, stream)
              : launch_conv_glds_pf<BP, BC, WAVES_P, NS, NW, false, BK, true, false, 1, false, IL>(a, zero, stream);
  return pf ? launch_conv_glds_pf<BP, BC, WAVES_P, NS, NW, true, BK, false, false, 1, false, IL>(a, zero, stream)
            : launch_conv_glds_pf<BP, BC, WAVES_P, NS, NW, false, BK, false, false, 1, false, IL>(a, zero, stream);
}

// Tile configurations of the LDS-DMA kernel (index = DRN conv config id, also used by the
// host-side autotuner): {BP, BC, WAVES_P, NS, NW, BK, NH, IL, KS}. 25-30: 8-wave big tiles with
// 32-deep stages and 3-4 stages in flight (one workgroup per CU): a 128 x 128 tile needs 64 B per
// MFMA cycle from L2 -- the per-CU L2 read rate -- 256 x 256 half that. IL = the next stage's
// LDS-DMA pieces interleaved with the MFMAs (31-37 = IL twins of the most used configs).
// KS = split-K capable (DrnConvFwdArgs::ksplit > 1, last-arriver epilogue).
#define DRN_GLDS_CONFIGS(X)                 \
  X(0, 128, 128, 2, 2, 4, 64, 1, false, true)  \
  X(1, 128, 128, 2, 3, 4, 64, 1, false, false) \
  X(2, 128, 128, 2, 4, 4, 64, 1, false, false) \
  X(3, 256, 64, 4, 2, 4, 64, 1, false, false)  \
  X(4, 256, 64, 4, 3, 4, 64, 1, false, false)  \
  X(5, 128, 64, 2, 3, 4, 64, 1, false, false)  \
  X(6, 64, 128, 1, 3, 4, 64, 1, false, false)  \
  X(7, 64, 64, 2, 4, 4, 64, 1, false, false)   \
  X(8, 256, 128, 4, 2, 8, 64, 1, false, false) \
  X(9, 256, 128, 4, 3, 8, 64, 1, false, false) \
  X(10, 128, 256, 2, 2, 8, 64, 1, false, false) \
  X(11, 128, 256, 2, 3, 8, 64, 1, false, false) \
  X(12, 128, 64, 2, 2, 4, 64, 1, false, false) \
  X(13, 64, 128, 1, 2, 4, 64, 1, false, true)  \
  X(14, 64, 64, 2, 2, 4, 64, 1, false, false)  \
  X(15, 64, 256, 1, 2, 4, 64, 1, false, false) \
  X(16, 32, 128, 1, 2, 4, 64, 1, false, false) \
  X(17, 128, 128, 2, 4, 4, 32, 1, false, false) \
  X(18, 64, 128, 1, 4, 4, 32, 1, false, false) \
  X(19, 128, 64, 2, 4, 4, 32, 1, false, false) \
  X(20, 128, 128, 2, 3, 4, 32, 1, false, false) \
  X(21, 64, 128, 1, 3, 4, 32, 1, false, false) \
  X(22, 256, 64, 4, 4, 4, 32, 1, false, false) \
  X(23, 256, 32, 4, 2, 4, 64, 1, false, false) \
  X(24, 128, 32, 4, 3, 4, 64, 1, false, false) \
  X(25, 256, 256, 4, 4, 8, 32, 2, false, true) \
  X(26, 256, 256, 4, 2, 8, 64, 2, false, false) \
  X(27, 256, 128, 4, 5, 8, 32, 1, false, false) \
  X(28, 128, 256, 2, 5, 8, 32, 1, false, false) \
  X(29, 256, 256, 2, 4, 8, 32, 2, false, false) \
  X(30, 256, 128, 2, 4, 8, 32, 1, false, false) \
  X(31, 128, 128, 2, 2, 4, 64, 1, true, true)   \
  X(32, 64, 128, 1, 2, 4, 64, 1, true, true)    \
  X(33, 256, 256, 4, 4, 8, 32, 2, true, true)   \
  X(34, 256, 128, 4, 2, 8, 64, 1, true, false)  \
  X(35, 64, 256, 1, 2, 4, 64, 1, true, false)   \
  X(36, 128, 64, 2, 4, 4, 32, 1, true, false)   \
  X(37, 64, 128, 1, 3, 4, 32, 1, true, false)

static int launch_glds_cfg(int cfg, DrnConvFwdArgs* a, const void* zero, hipStream_t s) {
  switch (cfg) {
#define DRN_X(id, bp, bc, wpv, ns, nw, bk, nh, il, ks) \
  case id:                                             \
    return launch_conv_glds<bp, bc, wpv, ns, nw, bk, nh, il, ks>(a, zero, s);
    DRN_GLDS_CONFIGS(DRN_X)
#undef DRN_X
    default:
      return (int)hipErrorInvalidValue;
  }
}

static int glds_cfg_bp(int cfg) {
  switch (cfg) {
#define DRN_X(id, bp, bc, wpv, ns, nw, bk, nh, il, ks) \
  case id:                                             \
    return bp;
    DRN_GLDS_CONFIGS(DRN_X)
#undef DRN_X
    default:
      return 0;
  }
}

static int glds_cfg_bk(int cfg) {
  switch (cfg) {
#define DRN_X(id, bp, bc, wpv, ns, nw, bk, nh, il, ks) \
  case id:                                             \
    return ks ? bk : 0;
    DRN_GLDS_CONFIGS(DRN_X)
#undef DRN_X
    default:
      return 0;
  }
}

static int glds_cfg_bc(int cfg) {
  switch (cfg) {
#define DRN_X(id, bp, bc, wpv, ns, nw, bk, nh, il, ks) \
  case id:                                             \
    return bc;
    DRN_GLDS_CONFIGS(DRN_X)
#undef DRN_X
    default:
      return 0;
  }
}

// Default choice when the host did not autotune (measured on the ResNet-50 layer set): the
// 2-stage pipelines keep 2 blocks per CU resident, which beat deeper single-block pipelines;
// 64 x 128 tiles once the 128 x 128 grid stops filling the chip.
static int glds_default_cfg(const DrnConvFwdArgs* a) {
  const long M = (long)a->N * a->P * a->Q;
  if (a->C == 4 || a->C == 8 || a->C == 16) return a->K <= 32 ? 23 : a->K <= 64 ? 3 : 0;  // row-staged
  if (a->C % 64) return 18;  // 32-channel inputs: the 32-deep-stage family
  auto blocks = [&](int bp, int bc) { return ((M + bp - 1) / bp) * ((a->K + bc - 1) / bc); };
  if (a->K <= 64) return blocks(256, 64) >= 384 ? 3 : 7;
  if (blocks(128, 128) >= 384) return 0;
  return 6;
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
  drn::launch(kern, dim3(tiles_p * tiles_c), dim3(256), LDS, stream, *a);
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

DRN_API int drn_conv_fwd(DrnConvFwdArgs* a, hipStream_t s);

#define DRN_GLDS_NCFG 38

// Whether the LDS-DMA kernel family supports this convolution.
DRN_API int drn_conv_glds_ok(const DrnConvFwdArgs* a) {
  if (a->C == 4)  // packed stem (stem.hip): tap pairs of 4 channels, two filter rows per stage
    return a->dil == 1 && a->S % 2 == 0 && a->S * a->C <= 32 && a->in_scale == nullptr && a->bn_x == nullptr &&
           a->residual == nullptr;
  if (a->C == 8 || a->C == 16)  // row-staged narrow conv (stem, CIFAR stage 1)
    return a->dil == 1 && a->S * a->C <= 64 && (a->in_scale == nullptr || a->relu_in != 0);
  return a->C % 32 == 0 && a->dil == 1 && (a->in_scale == nullptr || (a->C <= 4096 && a->relu_in != 0));
}

// Dispatch on a->cfg; zero = >= 16 bytes of device zeros (the LDS-DMA loader's padding source).
// A consumer-side BN finalize (in_fin) runs only on the LDS-DMA path; on the register-staged
// kernel the finalize is a separate launch ahead of the conv (drn_bn_finalize semantics).
DRN_API int drn_conv_fwd2(DrnConvFwdArgs* a, const void* zero, hipStream_t s) {
  if ((a->C % 8) != 0 && a->C != 4) return (int)hipErrorInvalidValue;
  if ((a->K % 8) != 0) return (int)hipErrorInvalidValue;
  if (a->C == 4 && (!drn_conv_glds_ok(a) || zero == nullptr || a->cfg == 100 || a->cfg >= DRN_GLDS_NCFG))
    return (int)hipErrorInvalidValue;  // the packed stem exists on the one-tile LDS-DMA path only
  if (a->fin_cnt != nullptr && (a->stats == nullptr || a->K > 64 * 64)) return (int)hipErrorInvalidValue;
  if (a->in_fin.stats != nullptr &&
      (a->in_scale == nullptr || a->in_fin.C != a->C || a->in_fin.G < 1 || a->in_fin.G > DRN_BN_FIN_GMAX))
    return (int)hipErrorInvalidValue;
  if ((a->ksplit > 1 || a->sk_blocks > 0) &&
      (a->cfg < 0 || a->cfg >= DRN_GLDS_NCFG || !drn_conv_glds_ok(a) || zero == nullptr))
    return (int)hipErrorInvalidValue;  // split-K: explicit split-capable LDS-DMA configurations only
  if (a->cfg >= DRN_NK_CFG0 && a->cfg < DRN_NK_CFG0 + DRN_NK_NCFG) return drn::launch_conv_nk(a->cfg - DRN_NK_CFG0, a, s);
  if (a->cfg >= DRN_GLDS_NCFG && a->cfg != 100) return (int)hipErrorInvalidValue;
  if (drn_conv_glds_ok(a) && zero != nullptr && a->cfg != 100)
    return drn::launch_glds_cfg(a->cfg >= 0 ? a->cfg : drn::glds_default_cfg(a), a, zero, s);
  if (a->in_fin.stats != nullptr) {
    if (a->in_fin.publish) {  // non-publishing consumers read the already published parameters
      const int rc = drn_bn_fin_fwd_launch(&a->in_fin, s);
      if (rc) return rc;
    }
    DrnConvFwdArgs b = *a;
    b.in_fin.stats = nullptr;
    return drn_conv_fwd(&b, s);
  }
  return drn_conv_fwd(a, s);
}

#ifdef DRN_CONV_TRACE
// diagnostics: per-workgroup timeline buffer for the LDS-DMA conv kernel (nullptr disables)
DRN_API int drn_conv_trace_set(unsigned long long* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(drn::g_conv_trace), &buf, sizeof(buf));
}
#endif

DRN_API int drn_conv_glds_cfg_bp(int cfg) { return drn::glds_cfg_bp(cfg); }
DRN_API int drn_conv_glds_cfg_bc(int cfg) { return drn::glds_cfg_bc(cfg); }
// k depth of a split-capable configuration's stages (0: not split-K / stream-K capable)
DRN_API int drn_conv_glds_cfg_bk(int cfg) { return drn::glds_cfg_bk(cfg); }
// partial slots per tile a stream-K launch of split-capable config cfg with G workgroups needs
// (0: not split-capable, or more workgroups than tile x k-stage units)
DRN_API int drn_conv_sk_slots_cfg(const DrnConvFwdArgs* a, int cfg, int G) {
  const int bk = drn::glds_cfg_bk(cfg);
  if (bk == 0 || (a->R * a->S * a->C) % bk) return 0;
  const int M = a->N * a->P * a->Q;
  const int bp = drn::glds_cfg_bp(cfg), bc = drn::glds_cfg_bc(cfg);
  return drn::sk_slots(((M + bp - 1) / bp) * ((a->K + bc - 1) / bc), (a->R * a->S * a->C) / bk, G);
}
// narrow-output (K = 16 / 32) register-operand kernels: configuration ids DRN_NK_CFG0 + i
DRN_API int drn_conv_nk_num_cfgs() { return DRN_NK_NCFG; }
DRN_API int drn_conv_nk_cfg0() { return DRN_NK_CFG0; }
DRN_API int drn_conv_glds_num_cfgs() { return DRN_GLDS_NCFG; }
DRN_API int drn_conv_glds_default_cfg(const DrnConvFwdArgs* a) { return drn::glds_default_cfg(a); }

DRN_API int drn_conv_fwd(DrnConvFwdArgs* a, hipStream_t s) {
  if ((a->C % 8) != 0 || (a->K % 8) != 0) return (int)hipErrorInvalidValue;
  if (a->fin_cnt != nullptr && (a->stats == nullptr || a->K > 64 * 64)) return (int)hipErrorInvalidValue;
  if (a->dil != 1 && a->dil != 2) return (int)hipErrorInvalidValue;
  const bool pro = a->in_scale != nullptr;
  const bool dil2 = a->dil == 2;
  if (pro) return dil2 ? drn::dispatch_conv_fwd<true, true>(a, s) : drn::dispatch_conv_fwd<true, false>(a, s);
  return dil2 ? drn::dispatch_conv_fwd<false, true>(a, s) : drn::dispatch_conv_fwd<false, false>(a, s);
}
