// conv_halo.hip -- halo-tiled direct convolution for stride-1 R x S (<= 3 x 3) layers on CDNA4.
//
// The implicit-GEMM kernels of conv_fwd.hip stage an im2col B tile per (tap, channel chunk): a
// 3x3 conv moves every input element through the L2 -> LDS path 9 times. A 128 x 128 x 64 tile
// then does 64 FLOP per staged byte, and at the ~70 GB/s a CU draws from L2 the MFMA pipe runs
// at <= ~45 % (measured: the ResNet-50 3x3 layers at 500-650 TF/s, profiles/r4_*).
//
// Here a workgroup owns a SPATIAL output tile -- `th` whole output rows of one image, or `ni`
// whole images when an image is small (14x14, 7x7) -- times BC output channels. Per 64-channel
// input chunk the tile's input HALO ((th + R - 1) x (W + S - 1) pixels per image, zero padded)
// is staged ONCE into LDS by LDS-DMA, and all R*S taps read their B fragments from it at a
// uniform tap offset; only the weights [BC][64] of each (chunk, tap) step stream through a ring
// of D + 1 LDS buffers (D steps in flight). Staged bytes per FLOP drop ~3-5x (3x3 256@14, BC 128:
// 196 FLOP/B), which lifts the L2 bound above the MFMA rate.
//
// Semantics: y = conv(x, w) (+ residual) with the fused epilogue of conv_fwd.hip (next-BN
// statistics, or the fused BN-backward reduction of a data gradient) -- reference
// resnet_model_official.py:80-91 (conv2d_fixed_padding, SAME for stride 1), :153-175 (the
// bottleneck's 3x3). Stride-1 data gradients of 3x3 convs are the same op on the flipped,
// channel-transposed weights, so both directions run here.
//
// Layout: 8 waves = WAVES_P (pixel groups of MJ 16-pixel fragments) x WAVES_C (channel groups of
// MI 16-channel fragments); MFMA v_mfma_f32_16x16x32_bf16, A = weights (rows = output channels),
// B = halo pixels. LDS rows are 128 B (64 channels) with 16-byte slots XOR-swizzled by
// (row >> 1) & 7 (glds_swz<64>, conflict-free ds_read_b128 fragment reads); the swizzle is
// applied on the per-lane SOURCE address of the lane-linear LDS-DMA.
#include "drn_common.h"
#include "drn_conv.h"
#include "drn_conv_epi.h"

namespace drn {

// Host-computed tile geometry (one launch).
struct HaloGeom {
  int32_t ni, th;        // images per tile (whole images when > 1), output rows per tile
  int32_t tpi;           // tiles per image (ni == 1) = P / th
  int32_t hh, hw;        // halo rows per image segment (th + R - 1), halo columns (Q + S - 1)
  int32_t hpx;           // halo pixels of a tile = ni * hh * hw
  int32_t tp;            // output pixels of a tile = ni * th * Q
  int32_t ntp;           // pixel tiles
};

// s_waitcnt vmcnt(n) for a run-time n (0..63): one scalar branch per step
__device__ __forceinline__ void wait_vmcnt_rt(int n) {
  switch (n) {
#define DRN_W(k) \
  case k:        \
    asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); \
    break;
    DRN_W(0) DRN_W(1) DRN_W(2) DRN_W(3) DRN_W(4) DRN_W(5) DRN_W(6) DRN_W(7) DRN_W(8) DRN_W(9) DRN_W(10)
    DRN_W(11) DRN_W(12) DRN_W(13) DRN_W(14) DRN_W(15) DRN_W(16) DRN_W(17) DRN_W(18) DRN_W(19) DRN_W(20)
    DRN_W(21) DRN_W(22) DRN_W(23) DRN_W(24) DRN_W(25) DRN_W(26) DRN_W(27) DRN_W(28) DRN_W(29) DRN_W(30)
#undef DRN_W
    default:
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// MJ pixel fragments per wave; HPW = max halo pieces (8 pixels x 128 B each) per wave
template <int WAVES_P, int MJ, int WAVES_C, int MI, int D, int HPW>
__global__ __launch_bounds__(512) void conv_halo_kernel(DrnConvFwdArgs a, HaloGeom g, const void* __restrict__ zero) {
  constexpr int NW = 8, NT = 512;
  static_assert(WAVES_P * WAVES_C == NW, "8 waves");
  constexpr int BP = WAVES_P * MJ * 16;   // computed pixel columns (>= g.tp)
  constexpr int BC = WAVES_C * MI * 16;   // output channels per tile
  constexpr int WP = MJ * 16, WC = MI * 16;
  constexpr int NWB = D + 1;              // weight ring buffers
  constexpr int GW = BC / 64;             // weight glds pieces per wave per step (BC rows x 128 B / 8 waves)
  static_assert(GW >= 1 && GW * 64 == BC, "BC multiple of 64");
  static_assert(BP % (NT / ((BC > 128 ? 128 : BC) / 8)) == 0, "the epilogue's row groups must tile BP");
  extern __shared__ __attribute__((aligned(1024))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int C = a.C, K = a.K, R = a.R, S = a.S;
  const int RS = R * S;
  const int nchunk = C >> 6;
  const int T = nchunk * RS;              // steps (chunk-major, tap-minor)
  const int M = a.N * a.P * a.Q;
  const int ntc = K / BC;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tcol = bid % ntc, tpix = bid / ntc;
  const int c0 = tcol * BC;
  // spatial tile -> first image / first output row, first output pixel
  int n0, p0;
  if (g.ni > 1) {
    n0 = tpix * g.ni;
    p0 = 0;
  } else {
    n0 = tpix / g.tpi;
    p0 = (tpix - n0 * g.tpi) * g.th;
  }
  const int m0 = (n0 * a.P + p0) * a.Q;
  const int m_end = min(m0 + g.tp, M);

  // LDS: [halo buffer 0][halo buffer 1 (nchunk > 1)][NWB weight buffers][...]
  const int hbytes = ((g.hpx + 7) >> 3) << 10;  // rounded up to whole 8-pixel pieces
  char* const hbuf0 = smem;
  char* const wbuf0 = smem + (nchunk > 1 ? 2 : 1) * hbytes;
  constexpr int WBYTES = BC * 128;

  // ---- halo loader: per-lane source offsets of this wave's pieces (element offset at chunk 0,
  // -1 = outside the image: the zero page) ----
  const int npieces = (g.hpx + 7) >> 3;
  const int my_pieces = npieces > wave ? (npieces - wave + NW - 1) / NW : 0;  // wave-uniform
  int hoff[HPW];
  const int hslot = lane & 7;
#pragma unroll
  for (int i = 0; i < HPW; ++i) {
    const int hp = (i * NW + wave) * 8 + (lane >> 3);
    int off = -1;
    if (i < my_pieces && hp < g.hpx) {
      const int seg = g.hh * g.hw;
      const int img = hp / seg;
      const int rem = hp - img * seg;
      const int ar = rem / g.hw;
      const int bc = rem - ar * g.hw;
      const int n = n0 + img;
      const int h = p0 - a.pad_h + ar;
      const int w = bc - a.pad_w;
      if (n < a.N && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W)
        off = ((n * a.H + h) * a.W + w) * C + ((hslot ^ glds_swz<64>(hp)) << 3);
    }
    hoff[i] = off;
  }
  const bf16_t* __restrict__ xg = reinterpret_cast<const bf16_t*>(a.x);
  auto issue_halo = [&](int chunk, char* hb) {
#pragma unroll
    for (int i = 0; i < HPW; ++i) {
      if (i < my_pieces) {
        const void* src = hoff[i] >= 0 ? (const void*)(xg + hoff[i] + (chunk << 6)) : zero;
        glds16(src, hb + ((i * NW + wave) << 10));
      }
    }
  };
  // ---- weight loader: rows c0 + row of w[K][R][S][C], 64 channels of one (tap, chunk) ----
  const int Ktot = RS * C;
  const bf16_t* __restrict__ wg = reinterpret_cast<const bf16_t*>(a.w);
  uint32_t woff[GW];
#pragma unroll
  for (int i = 0; i < GW; ++i) {
    const int row = (i * NW + wave) * 8 + (lane >> 3);
    woff[i] = (uint32_t)((c0 + row) * Ktot + (((lane & 7) ^ glds_swz<64>(row)) << 3));
  }
  auto issue_w = [&](int step) {
    const int chunk = step / RS, tap = step - chunk * RS;
    const bf16_t* __restrict__ ws = wg + tap * C + (chunk << 6);
    char* wb = wbuf0 + (step % NWB) * WBYTES;
#pragma unroll
    for (int i = 0; i < GW; ++i) glds16(ws + woff[i], wb + ((i * NW + wave) << 10));
  };

  // ---- fragment addressing ----
  const int wp = wave % WAVES_P, wc = wave / WAVES_P;
  const int fr = lane & 15, fk = lane >> 4;
  // B: output pixel o of the tile -> halo pixel of tap (0, 0); padded columns read pixel 0
  int hb0[MJ];
#pragma unroll
  for (int j = 0; j < MJ; ++j) {
    const int o = (wp * MJ + j) * 16 + fr;
    int hp = 0;
    if (o < g.tp) {
      const int per_img = g.th * a.Q;
      const int img = o / per_img;
      const int rem = o - img * per_img;
      const int r = rem / a.Q;
      const int c = rem - r * a.Q;
      hp = (img * g.hh + r) * g.hw + c;
    }
    hb0[j] = hp;
  }
  uint32_t aoff[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int row = wc * WC + i * 16 + fr;  // 16-aligned groups: the swizzle bits are fr's
    aoff[i] = (uint32_t)(row * 128);
  }
  const int aswz = glds_swz<64>(fr);

  f32x4_t acc[MI][MJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < MJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: halo of chunk 0, weights of steps 0 .. D-1 ----
  issue_halo(0, hbuf0);
#pragma unroll
  for (int s = 0; s < D; ++s)
    if (s < T) issue_w(s);

  const uint32_t lds0 = lds_addr(smem);
  for (int s = 0; s < T; ++s) {
    const int chunk = s / RS, tap = s - chunk * RS;
    // loads allowed to stay in flight: the weights of steps s+1 .. s+D-1, plus the halo batch of
    // the next chunk when it was issued after W(s) (at step chunk*RS, s within D-1 steps of it)
    const int ahead = min(D - 1, T - 1 - s);
    int allowed = ahead * GW;
    const int hs = chunk * RS;  // step that issued the halo batch of chunk + 1
    if (chunk + 1 < nchunk && s > hs && s - hs <= D - 1) allowed += my_pieces;  // (R*S >= D: one batch at most)
    wait_vmcnt_rt(allowed);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (tap == 0 && chunk + 1 < nchunk) issue_halo(chunk + 1, hbuf0 + ((chunk + 1) & 1) * hbytes);
    if (s + D < T) issue_w(s + D);
    // tap offset inside the halo
    const int dr = tap / S, ds = tap - dr * S;
    const int toff = dr * g.hw + ds;
    const uint32_t hbase = lds0 + (uint32_t)((chunk & 1) * hbytes);
    const uint32_t wbase = lds0 + (uint32_t)(wbuf0 - smem) + (uint32_t)((s % NWB) * WBYTES);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      const int c16 = kh * 4 + fk;
      bf16x8_t af[MI], bfr[MJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const u32x4_t v = lds_read16(wbase + aoff[i] + (uint32_t)((c16 ^ aswz) << 4));
        af[i] = __builtin_bit_cast(bf16x8_t, v);
      }
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        const int hp = hb0[j] + toff;
        const u32x4_t v = lds_read16(hbase + (uint32_t)(hp << 7) + (uint32_t)((c16 ^ glds_swz<64>(hp)) << 4));
        bfr[j] = __builtin_bit_cast(bf16x8_t, v);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < MJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every fragment read done before the epilogue reuses the LDS
  constexpr int NH = (BP * BC * 4 > 160 * 1024) ? 2 : 1;
  if constexpr (NH == 1) {
    EpiPre<BP, BC, NT, false> epre;
    epi_prefetch<BP, BC, NT, false>(a, m0, c0, m_end, epre);
    conv_epilogue<BP, BC, WP, WC, MI, MJ, NT, false>(a, smem, acc, wp, wc, m0, c0, m_end, epre);
  } else {
    conv_epilogue_sliced<BP, BC, WP, WC, MI, MJ, NT, NH>(a, smem, acc, wp, wc, m0, c0, m_end);
  }
}

// configurations: {WAVES_P, MJ, WAVES_C, MI, D}
//   0: 224 px x 128 ch (28x28 / 14x14 / 7x7 stages), 3 steps in flight
//   1: 256 px x 64 ch (56x56, 64 channels), 3 in flight
//   2: 448 px x 64 ch (56x56, 8 rows per tile)
//   3: 224 px x 256 ch, 2 in flight (LDS)
//   4: 128 px x 128 ch (7x7: 2 images per tile)
//   5: 256 px x 64 ch, every wave all 64 channels of 32 pixels
#define DRN_HALO_CONFIGS(X) \
  X(0, 2, 7, 4, 2, 3)       \
  X(1, 4, 4, 2, 2, 3)       \
  X(2, 4, 7, 2, 2, 3)       \
  X(3, 2, 7, 4, 4, 2)       \
  X(4, 2, 4, 4, 2, 3)       \
  X(5, 8, 2, 1, 4, 3)
#define DRN_HALO_NCFG 6
#define DRN_HALO_HPW 12

// tile geometry for a computed pixel width BP: the largest tile of whole output rows (th | P) or
// whole images that fits BP; 0 if none
static int halo_geom(const DrnConvFwdArgs* a, int BP, HaloGeom* g) {
  const int P = a->P, Q = a->Q;
  g->ni = 1;
  g->th = 0;
  if (P * Q <= BP) {
    g->th = P;
    g->ni = BP / (P * Q);
    if (g->ni > a->N) g->ni = a->N;
  } else {
    for (int th = P; th >= 1; --th)
      if (P % th == 0 && th * Q <= BP) {
        g->th = th;
        break;
      }
  }
  if (g->th == 0) return 0;
  g->tpi = P / g->th;
  g->hh = g->th + a->R - 1;
  g->hw = Q + a->S - 1;
  g->hpx = g->ni * g->hh * g->hw;
  g->tp = g->ni * g->th * Q;
  g->ntp = g->ni > 1 ? (a->N + g->ni - 1) / g->ni : a->N * g->tpi;
  return 1;
}

template <int WAVES_P, int MJ, int WAVES_C, int MI, int D>
static int launch_halo(const DrnConvFwdArgs* a, const void* zero, hipStream_t s) {
  constexpr int BP = WAVES_P * MJ * 16, BC = WAVES_C * MI * 16;
  if (a->K % BC || a->R * a->S < D) return (int)hipErrorInvalidValue;
  HaloGeom g;
  if (!halo_geom(a, BP, &g)) return (int)hipErrorInvalidValue;
  const int npieces = (g.hpx + 7) / 8;
  if ((npieces + 7) / 8 > DRN_HALO_HPW) return (int)hipErrorInvalidValue;
  const int nchunk = a->C / 64;
  const int hbytes = npieces * 1024;
  const int lds_main = (nchunk > 1 ? 2 : 1) * hbytes + (D + 1) * BC * 128;
  constexpr int NH = (BP * BC * 4 > 160 * 1024) ? 2 : 1;
  const int lds_epi = BP * BC * 4 / NH;
  const int lds = lds_main > lds_epi ? lds_main : lds_epi;
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  // the runtime vmcnt switch covers counts up to 30
  if ((D - 1) * (BC / 64) + (npieces + 7) / 8 > 30) return (int)hipErrorInvalidValue;
  auto kern = conv_halo_kernel<WAVES_P, MJ, WAVES_C, MI, D, DRN_HALO_HPW>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr = true;
  }
  const int grid = g.ntp * (a->K / BC);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), lds, s, *a, g, zero);
  return (int)hipGetLastError();
}

}  // namespace drn

// Whether the halo kernel family supports this convolution (stride 1, R, S <= 3 with SAME
// padding, 64-channel chunks, identity output map, plain input: no fused BN prologue).
DRN_API int drn_conv_halo_ok(const DrnConvFwdArgs* a) {
  return a->stride == 1 && a->dil == 1 && a->R <= 3 && a->S <= 3 && a->R >= 1 && a->S >= 1 && a->C % 64 == 0 &&
         a->K % 64 == 0 && a->in_scale == nullptr && a->bnb_x == nullptr && a->out_stride == 0 && a->ksplit <= 1 &&
         a->sk_blocks == 0 && a->fin_cnt == nullptr && a->P == a->H && a->Q == a->W && a->pad_h >= 0 &&
         a->pad_w >= 0 && a->pad_h < a->R && a->pad_w < a->S;
}

DRN_API int drn_conv_halo_num_cfgs() { return DRN_HALO_NCFG; }

DRN_API int drn_conv_halo(int cfg, const DrnConvFwdArgs* a, const void* zero, hipStream_t s) {
  if (!drn_conv_halo_ok(a) || zero == nullptr) return (int)hipErrorInvalidValue;
  switch (cfg) {
#define DRN_X(id, wp, mj, wc, mi, d) \
  case id:                           \
    return drn::launch_halo<wp, mj, wc, mi, d>(a, zero, s);
    DRN_HALO_CONFIGS(DRN_X)
#undef DRN_X
    default:
      return (int)hipErrorInvalidValue;
  }
}
