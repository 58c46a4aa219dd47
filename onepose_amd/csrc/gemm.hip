// fp32 (or bf16-input) MFMA grouped token-GEMM (see gemm.h).
//
// A workgroup (4 or 8 waves) owns a BM x BN output tile.  Its waves form a
// WM x WN x KS grid: each wave owns a 32 x (FN*32) block of v_mfma_f32_32x32x2_f32
// accumulators and one of the KS k-slices of every stage (KS > 1 splits the K loop inside
// the workgroup; the slices are added through LDS in a fixed order at the end).  The tile
// shape trades per-workgroup efficiency (64 x 64: least LDS / L2 traffic per FLOP) against
// filling 256 CUs: the narrow 256-wide q output and the 128-wide [k_h | v_h] KV tiles use
// 32-row tiles (q also splits K in two) to get more workgroups.
//
// Operands are staged through double-buffered LDS images [row][k] of BKS = 32*KS columns
// with a (BKS+4)-float pitch: a ds_read_b128 lane group (16 lanes, 16 distinct rows, same k)
// hits 16 distinct 16-byte bank slots (pitch = 4 mod 64 floats, or 36), so reads are
// conflict free.  Each b128 read feeds four MFMAs: within one group of 8 k-values, lane half
// h carries k = 8*kk + 4*h + j into MFMA j, identically for A and W, so the k-sum is a
// re-ordering of the plain sum.  Global loads run two stages ahead of the MFMAs (register
// stage + LDS stage); loads are branch- and select-free so the compiler waits on exactly the
// older stage.  One barrier per stage.
#include "gemm.h"

#include <cstdlib>
#include <cstring>
#include <type_traits>

// Pins the pipeline's phase order (the compiler's own schedule measured within +-2%,
// DESIGN.md §3d).
#define ONEPOSE_SCHED_BARRIER() __builtin_amdgcn_sched_barrier(0)
// "// @phase N" comments mark a workgroup's prologue / loop / epilogue boundaries; the
// phase probe's generated copy of this file (tools/probe_src.sh) turns them into stamps.

namespace onepose {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

namespace {

// Operand modes (gemm.h): PM_F32 fp32 LDS image + v_mfma_f32_32x32x2_f32; PM_BF16 one bf16
// image (rounded) + v_mfma_f32_32x32x16_bf16; PM_SPLIT3 three bf16 images per operand, the
// exact split x = hi + mid + lo (hi = bf16(x), mid = bf16(x - hi), lo = x - hi - mid: every
// step is exact in fp32 and lo fits bf16's 8 bits), and six bf16 MFMAs per 16-deep group,
// a_i b_j for i + j <= 2 (the dropped a_mid b_lo, a_lo b_mid, a_lo b_lo are <= 2^-23 of |a b|
// together), accumulated in fp32: an fp32-accurate product at 6 x 32 instead of 8 x 64 MFMA
// cycles per 16-deep group.
// Per-wave MFMA operand fragments of one stage: fp32 (v_mfma_f32_32x32x2_f32, a float4 feeds
// four MFMAs over k = 8 kk + 4 h + j) or bf16 (v_mfma_f32_32x32x16_bf16: lane half h holds
// k = 16 kk + 8 h + j, j < 8, from a bf16 LDS image rounded to nearest even when stored).
template <int PM, int KKW, int FN>
struct FragT {
  float4 a[KKW];
  float4 w[KKW][FN];
};
template <int KKW, int FN>
struct FragT<PM_BF16, KKW, FN> {
  bf16x8 a[KKW];
  bf16x8 w[KKW][FN];
};
template <int KKW, int FN>
struct FragT<PM_SPLIT3, KKW, FN> {   // hi / mid / lo pieces
  bf16x8 a[3][KKW];
  bf16x8 w[3][KKW][FN];
};


constexpr int kScoreGroup = 8;   // N-tiles per column group of the score grid

template <int BM_, int BN_, int KS_, int NW_, int BKS_, int WPE_ = 3, int SUB_ = BM_,
          int SUBN_ = BN_>
struct Tile {
  static constexpr int BM = BM_, BN = BN_, KS = KS_, NW = NW_, BKS = BKS_;
  static constexpr int WPE = WPE_;              // amdgpu_waves_per_eu hint
  // SUB < BM: the tile stands in for BM / SUB tiles of SUB rows -- its InstanceNorm partials,
  // finalize tickets (EPI_STATS) and acc0 (PRO_HEADZ) are those of the SUB x BN tile, so the
  // workspace layout and every result bit are the smaller tile's
  static constexpr int SUB = SUB_;
  static constexpr int NSUB = BM / SUB;
  static constexpr int SUBN = SUBN_;   // columns of the stand-in tile (its acc0 layout)
  static constexpr int NT = 64 * NW;            // threads
  static constexpr int WM = BM / 32;            // waves along M
  static constexpr int WN = NW / (WM * KS);     // waves along N
  static constexpr int FN = BN / (32 * WN);     // accumulators per wave
  static constexpr int KKW = BKS / KS / 8;      // 8-deep MFMA groups per wave per stage
  static constexpr int PITCH = BKS + 4;
  static constexpr int KQ = BKS / 4;            // float4 per row per stage
  static constexpr int A4 = BM * KQ / NT;       // float4 of A per thread per stage
  static constexpr int W4 = BN * KQ / NT;
  static constexpr int STAGE = (BM + BN) * PITCH;
  // bf16 modes: each image (one per split piece) is [BM + BN] rows of BKS bf16 (64 or 128 B, no
  // padding), the row's 16-B k-chunks XOR-swizzled by the row (bsw), so that a ds_read_b128
  // lane group (16 rows, one chunk) hits 16 distinct 4-bank groups and a ds_write_b64 group
  // (one or two rows of contiguous lanes) 32 distinct banks: conflict-free both ways, and 20%
  // less LDS than padded rows (64x64 split: 48 KB for two stages, three workgroups per CU).
  static constexpr int STAGEB = (BM + BN) * BKS;   // bf16 elements per image
  static_assert(WM * WN * KS == NW && FN >= 1 && A4 >= 1 && W4 >= 1 && KKW >= 2, "tile shape");
  static_assert(NT % KQ == 0 && BM * KQ % NT == 0 && BN * KQ % NT == 0, "one k-quad per thread");
};

// Element offset of (row, k) in a bf16 image: 16-B chunk k / 8 XOR-swizzled by the row --
// 64-B rows (BKS 32): by (row >> 2) & 3; 128-B rows (BKS 64): by (row >> 1) & 7.  The 16 rows
// of a ds_read_b128 lane group ({0-3, 12-15, 20-27} etc. of lane & 31) then cover 16 distinct
// (row-in-bank-line, chunk) pairs.
template <class T>
__device__ __forceinline__ int bsw(int row, int k) {
  static_assert(T::BKS == 32 || T::BKS == 64, "swizzled bf16 images have 64- or 128-B rows");
  if constexpr (T::BKS == 32) return row * 32 + ((((k >> 3) ^ (row >> 2)) & 3) << 3) + (k & 7);
  else return row * 64 + ((((k >> 3) ^ (row >> 1)) & 7) << 3) + (k & 7);
}

// Stage registers.  WPL: the W operand comes from NPL bf16 planes in HBM (pre-split weights /
// folded message weights, gemm.h GemmProb::Wp): 8 B per plane and k-quad, copied to LDS as is.
template <class T, bool WPL = false, int NPL = 1>
struct Stage {
  float4 a[T::A4];
  float4 w[WPL ? 1 : T::W4];
  uint2 wp[WPL ? T::W4 : 1][NPL];
  float4 mean, rstd;
};

// Per-launch problem fields, selected field by field from the kernel arguments (a
// dynamically indexed kernel-argument struct would be copied to scratch).
struct Ctx {
  const float *a0, *a1, *w0, *w1, *mean, *rstd;
  const uint16_t *wp0, *wp1;   // W planes of the two K ranges (WPL)
  int64_t wpl0, wpl1;          // plane strides (elements)
  const uint16_t *ap0, *ap1;   // A planes of the two K ranges (DMA 2)
  int64_t apl0, apl1;
  int ldap0, ldap1;
  int lda0, lda1, ldw0, ldw1, ksplit, M, N, K;
};

// Rows past M (N) are loaded from the last valid row: they only feed accumulator rows
// (columns) that are never stored, and every reducing epilogue masks them when it stages the
// tile, so they need no zeroing -- a select right behind each load would make the wave wait
// for the load it just issued.
template <int PRO, class T, bool WPL = false, int NPL = 1, bool DOW = true>
__device__ __forceinline__ void load_stage(const Ctx& c, int m0, int n0, int k0,
                                           Stage<T, WPL, NPL>& s) {
  const int t = threadIdx.x;
  const int kq = (t % T::KQ) * 4;
  const bool first = k0 < c.ksplit;
  const float* A = first ? c.a0 : c.a1;
  const int lda = first ? c.lda0 : c.lda1;
  const int ldw = first ? c.ldw0 : c.ldw1;
  const int kk = first ? (k0 + kq) : (k0 - c.ksplit + kq);
  if (PRO == PRO_NORM_RELU) {
    s.mean = *reinterpret_cast<const float4*>(c.mean + k0 + kq);
    s.rstd = *reinterpret_cast<const float4*>(c.rstd + k0 + kq);
  }
#pragma unroll
  for (int i = 0; i < T::A4; ++i) {
    const int m = min(m0 + (t + T::NT * i) / T::KQ, c.M - 1);
    s.a[i] = *reinterpret_cast<const float4*>(A + (int64_t)m * lda + kk);
  }
  if constexpr (!DOW) {
    (void)ldw;
  } else if constexpr (WPL) {
    const uint16_t* W = first ? c.wp0 : c.wp1;
    const int64_t pl = first ? c.wpl0 : c.wpl1;
#pragma unroll
    for (int i = 0; i < T::W4; ++i) {
      const int o = min(n0 + (t + T::NT * i) / T::KQ, c.N - 1);
#pragma unroll
      for (int q = 0; q < NPL; ++q)
        s.wp[i][q] = *reinterpret_cast<const uint2*>(W + q * pl + (int64_t)o * ldw + kk);
    }
  } else {
    const float* W = first ? c.w0 : c.w1;
#pragma unroll
    for (int i = 0; i < T::W4; ++i) {
      const int o = min(n0 + (t + T::NT * i) / T::KQ, c.N - 1);
      s.w[i] = *reinterpret_cast<const float4*>(W + (int64_t)o * ldw + kk);
    }
  }
}

// W planes of one stage (k0) -> the W rows of the bf16 images at `base` by global_load_lds:
// 16 B per lane, one 1-KB piece = 16 rows of 64 B per wave-instruction (the wave-uniform LDS
// base + 16 x lane: rows of 4 chunks, lane l -> row l / 4, slot l % 4), the slot holding the
// chunk bsw's swizzle puts there (the source address is permuted, the destination is linear).
template <class T, int NPL>
__device__ __forceinline__ void dma_w_stage(const Ctx& c, int n0, int k0, float* base) {
  static_assert(T::BKS == 32 && T::BN % 16 == 0 && (NPL * T::BN / 16) % T::NW == 0, "W pieces");
  constexpr int PIECES = NPL * T::BN / 16, PPW = PIECES / T::NW;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool first = k0 < c.ksplit;
  const uint16_t* W = first ? c.wp0 : c.wp1;
  const int64_t pl = first ? c.wpl0 : c.wpl1;
  const int ldw = first ? c.ldw0 : c.ldw1;
  const int kk = first ? k0 : k0 - c.ksplit;
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int p = wave + T::NW * i;
    const int q = p / (T::BN / 16), rb = (p % (T::BN / 16)) * 16;
    const int row = T::BM + rb + (lane >> 2);   // image row
    const int chunk = ((lane & 3) ^ (row >> 2)) & 3;
    const int o = min(n0 + rb + (lane >> 2), c.N - 1);
    const uint16_t* src = W + q * pl + (int64_t)o * ldw + kk + chunk * 8;
    char* dst = reinterpret_cast<char*>(base) + (int64_t)q * T::STAGEB * 2 + (T::BM + rb) * 64;
    __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
  }
}

// One 16-B-per-lane global_load_lds (1 KB per wave at the wave-uniform LDS base `dst` + 16 x lane).
// (A __device__ function: the builtin cannot appear in the loop's lambdas, which the host pass
// also compiles.)
__device__ __forceinline__ void dma16(const void* src, void* dst) {
  __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
}

// fp32 -> the bf16 image(s) of one k-quad at `b16` (element offset `off`, images STAGEB apart):
// PM_BF16 rounded to nearest even; PM_SPLIT3 the exact split hi + mid + lo.
template <class T, int PM>
__device__ __forceinline__ void store_quad_bf16(__bf16* b16, int off, float4 v) {
  if constexpr (PM == PM_BF16) {
    bf16x4 q;
    q[0] = (__bf16)v.x;
    q[1] = (__bf16)v.y;
    q[2] = (__bf16)v.z;
    q[3] = (__bf16)v.w;
    *reinterpret_cast<bf16x4*>(b16 + off) = q;
  } else {
    bf16x4 q0, q1, q2;
    const float x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const __bf16 h = (__bf16)x[c];
      const float r = x[c] - (float)h;
      const __bf16 m = (__bf16)r;
      q0[c] = h;
      q1[c] = m;
      q2[c] = (__bf16)(r - (float)m);
    }
    *reinterpret_cast<bf16x4*>(b16 + off) = q0;
    *reinterpret_cast<bf16x4*>(b16 + off + T::STAGEB) = q1;
    *reinterpret_cast<bf16x4*>(b16 + off + 2 * T::STAGEB) = q2;
  }
}

// Stage registers -> LDS image at `base` ([BM + BN] rows: A then W), applying the prologue;
// fp32 rows of PITCH floats, or swizzled bf16 images (Tile::STAGEB elements each).
template <int PRO, class T, int PM, bool WPL = false, int NPL = 1, bool DOW = true>
__device__ __forceinline__ void store_stage(float* base, Stage<T, WPL, NPL>& s) {
  const int t = threadIdx.x;
  const int kq = (t % T::KQ) * 4;
  __bf16* b16 = reinterpret_cast<__bf16*>(base);
#pragma unroll
  for (int i = 0; i < T::A4; ++i) {
    float4 v = s.a[i];
    if (PRO == PRO_NORM_RELU) {
      v.x = fmaxf((v.x - s.mean.x) * s.rstd.x, 0.f);
      v.y = fmaxf((v.y - s.mean.y) * s.rstd.y, 0.f);
      v.z = fmaxf((v.z - s.mean.z) * s.rstd.z, 0.f);
      v.w = fmaxf((v.w - s.mean.w) * s.rstd.w, 0.f);
    }
    const int row = (t + T::NT * i) / T::KQ;
    if constexpr (PM == PM_F32)
      *reinterpret_cast<float4*>(base + row * T::PITCH + kq) = v;
    else
      store_quad_bf16<T, PM>(b16, bsw<T>(row, kq), v);
  }
#pragma unroll
  for (int i = 0; i < (DOW ? T::W4 : 0); ++i) {
    const int row = T::BM + (t + T::NT * i) / T::KQ;
    if constexpr (WPL) {
      static_assert(PM != PM_F32 && NPL == (PM == PM_SPLIT3 ? 3 : 1), "W planes");
#pragma unroll
      for (int q = 0; q < NPL; ++q)
        *reinterpret_cast<uint2*>(b16 + q * T::STAGEB + bsw<T>(row, kq)) = s.wp[i][q];
    } else if constexpr (PM == PM_F32) {
      *reinterpret_cast<float4*>(base + row * T::PITCH + kq) = s.w[i];
    } else {
      store_quad_bf16<T, PM>(b16, bsw<T>(row, kq), s.w[i]);
    }
  }
}

// DMA: 0 = register-staged loop; 1 = the lean loop, W planes by global_load_lds and A through
// registers; 2 = the lean loop with A from activation planes by global_load_lds as well.
template <int EPI, int PRO, class T, int PM, bool WPL, int DMA = 0>
__device__ __forceinline__ void gemm_body(const GemmArgs& args, StampTick& tk, StampLds* sl,
                                          int vtile = -1) {
  constexpr int BM = T::BM, BN = T::BN, FN = T::FN, PITCH = T::PITCH;
  constexpr bool BF = PM != PM_F32;   // bf16 LDS images and MFMAs
  constexpr int NPL = PM == PM_SPLIT3 ? 3 : 1;   // bf16 images per operand
  constexpr int NPL_OUT = PM == PM_F32 ? 0 : NPL;  // activation planes of a stored output
  constexpr int STAGE = PM == PM_F32 ? T::STAGE : NPL * T::STAGEB / 2;   // floats
  // epilogue staging tile [BM][TP]: rows of BN + 4 (16-B aligned, read back as float4 rows by
  // the row-store pass), or BN + 1 where columns are read across rows (score, QKV)
  constexpr int TP = EPI == EPI_SCORE ? BN + 1 : BN + 4;
  // QKV's [k_h | v_h] tiles are staged transposed, [BN][BM + 4]
  constexpr int QKVL = EPI == EPI_QKV ? BN * (BM + 4) : 0;
  // LDS stage buffers: two (one stage of loads in flight ahead of the MFMAs), three for the bf16
  // DMA-2 loop (two stages in flight: nothing is staged through registers there, and a bf16
  // stage is small -- 12 KB at 64 x 128 -- so the third buffer fits the epilogue's LDS anyway)
  // (the A pieces must deal evenly over the waves: every wave then waits for its own stage)
  // (four and five buffers measured slower: config 5 1644 -> 1619 / 1499 frames/s, config 2
  // bf16 2906 -> 2901 / 2704; the loop is bound by the L2 -> LDS bytes)
  constexpr int NBUF = (DMA == 2 && PM == PM_BF16 && (NPL * BM / (512 / T::BKS)) % T::NW == 0) ? 3 : 2;
  constexpr int LDS0 = NBUF * STAGE > BM * TP ? NBUF * STAGE : BM * TP;
  constexpr int LDSF = LDS0 > QKVL ? LDS0 : QKVL;
  __shared__ __attribute__((aligned(16))) float lds[LDSF];
  __shared__ float zrow[2 * BM];
  __shared__ float part[(EPI == EPI_STATS) ? (T::NT > T::WM * BN ? T::NT : T::WM * BN) * 2 : 1];

  // XCD-aware tile order: blocks are dealt round-robin over the 8 XCDs, so hand each XCD a
  // contiguous run of logical tiles -- the N-tiles of one M-tile then share that XCD's L2.
  // (vtile >= 0: the logical tile given by a caller that loops over tiles -- tools/phase_probe's
  // persistent form; the library's kernels pass none)
  int bid = vtile >= 0 ? vtile : xcd_contiguous(blockIdx.x, gridDim.x);
  const bool second = bid >= args.p[0].tiles;
#define F(x) (second ? args.p[1].x : args.p[0].x)
  if (second) bid -= args.p[0].tiles;
  const int mtiles = F(mtiles), ntiles = F(ntiles);
  const int per_sample = mtiles * ntiles;
  const int b = bid / per_sample;
  const int r = bid - b * per_sample;
  int mt = r / ntiles;
  int nt = r - mt * ntiles;
  if (EPI == EPI_SCORE && ntiles % kScoreGroup == 0) {
    // score grid in column groups of kScoreGroup N-tiles (D3 rows), all M-tiles of a group
    // consecutive: an XCD's contiguous run of logical tiles then covers one group, so each XCD
    // reads all of D2 and its own slice of D3 once, instead of a D2 slice and all of D3 (the
    // D3 re-fetch by every XCD, 4 MB x 8 at config 2).  Per-tile results are unchanged.
    const int g = r / (mtiles * kScoreGroup), rr = r - g * mtiles * kScoreGroup;
    mt = rr / kScoreGroup;
    nt = g * kScoreGroup + (rr - mt * kScoreGroup);
  }
  const int m0 = mt * BM, n0 = nt * BN;
  Ctx c;
  c.a0 = F(A0) + b * F(a0_bs);
  c.a1 = F(A1) + b * F(a1_bs);
  c.w0 = F(W) + b * F(w_bs);
  const float* w1 = F(W1);
  c.ldw0 = F(ldw);
  c.lda0 = F(lda0);
  c.lda1 = F(lda1);
  c.ksplit = F(ksplit);
  c.M = F(M);
  c.N = F(N);
  c.K = F(K);
  // second K range: its own weights, or the same matrix continuing past ksplit
  c.w1 = w1 ? w1 + b * F(w1_bs) : c.w0 + c.ksplit;
  c.ldw1 = w1 ? F(ldw1) : c.ldw0;
  c.mean = F(pro_mean) + b * F(pro_bs);
  c.rstd = F(pro_rstd) + b * F(pro_bs);
  if constexpr (WPL) {   // W planes (range 1: its own planes, or range 0's continuing)
    const uint16_t* wp1 = F(Wp1);
    c.wp0 = F(Wp) + b * F(wp_bs);
    c.wpl0 = F(wpl);
    c.wp1 = wp1 ? wp1 + b * F(wp1_bs) : c.wp0 + c.ksplit;
    c.wpl1 = wp1 ? F(wpl1) : c.wpl0;
  }
  if constexpr (DMA == 2) {   // A planes (range 1: its own planes, or range 0's continuing)
    const uint16_t* ap1 = F(Ap1);
    c.ap0 = F(Ap) + b * F(ap_bs);
    c.apl0 = F(apl);
    c.ldap0 = F(ldap);
    c.ap1 = ap1 ? ap1 + b * F(ap1_bs) : c.ap0 + c.ksplit;
    c.apl1 = ap1 ? F(apl1) : c.apl0;
    c.ldap1 = ap1 ? F(ldap1) : c.ldap0;
  }

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int ks = wave / (T::WM * T::WN);
  const int wm = (wave % (T::WM * T::WN)) / T::WN;
  const int wn = wave % T::WN;

  floatx16 acc[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
  // the epilogue's bias of the wave's columns, loaded ahead of the K loop (loaded where the
  // epilogue starts, it was a global round trip every workgroup waited on there)
  float bias_pre[FN];
  {
    const float* bp = F(bias);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int gn = n0 + wn * FN * 32 + j * 32 + (lane & 31);
      bias_pre[j] =
          (EPI != EPI_SCORE && EPI != EPI_ACC && bp != nullptr && gn < c.N) ? bp[gn] : 0.f;
    }
  }

  // RESID with at most two residual float4 per thread (fp32 MLP conv 2's 64 x 32 tile): the
  // row-store pass's R loads ahead of the K loop too (the same rows and columns it reads there)
  constexpr int RPER = BM * (BN / 4) / T::NT;
  constexpr bool kRPre = EPI == EPI_RESID && RPER <= 4 && (BM * (BN / 4)) % T::NT == 0;
  float4 r_pre[kRPre ? RPER : 1];
  if constexpr (kRPre) {
    const float* R = F(R) + b * F(r_bs);
    const int ldr = F(ldr);
#pragma unroll
    for (int p = 0; p < RPER; ++p) {
      const int idx = t + T::NT * p, r = idx / (BN / 4), cc = (idx % (BN / 4)) * 4;
      const int gm = min(m0 + r, c.M - 1), gn = min(n0 + cc, c.N - 4);
      r_pre[p] = *reinterpret_cast<const float4*>(R + (int64_t)gm * ldr + gn);
    }
  }

  // Main loop, software-pipelined across the per-stage barrier.  Step kt consumes stage kt
  // from registers (fragments read from LDS right after the previous barrier):
  //   issue global loads of stage kt+2 | MFMA kk0 | store stage kt+1 to the other LDS buffer
  //   | MFMA kk1, kk2 | barrier | read stage kt+1's fragments | MFMA kk3 (hides that read)
  // so the matrix pipe is fed through the store / barrier / LDS-read phase of every stage.
  // Global loads run two stages ahead (register stage + LDS stage).
  const int nk = c.K / T::BKS;
  Stage<T, WPL, NPL> s0, s1;
  constexpr int KG = BF ? 16 : 8;                  // k per MFMA group
  constexpr int KKW = T::BKS / T::KS / KG;         // groups per wave per stage
  static_assert(KKW >= 2, "two MFMA groups per stage (pipeline shape)");
  using Frag = FragT<PM, KKW, FN>;
  Frag f0, f1;
  const int kofs = ks * (T::BKS / T::KS) + (lane >> 5) * (KG / 2);
  const int a_off = (wm * 32 + (lane & 31)) * PITCH + kofs;   // fp32 images
  const int w_off = BM * PITCH + (wn * FN * 32 + (lane & 31)) * PITCH + kofs;
  const int a_row = wm * 32 + (lane & 31);                  // bf16 images (bsw)
  const int w_row = BM + wn * FN * 32 + (lane & 31);
  auto read_frag = [&](const float* buf, Frag& f) __attribute__((always_inline)) {
#pragma unroll
    for (int kk = 0; kk < KKW; ++kk) {
      if constexpr (PM == PM_BF16) {
        const __bf16* b16 = reinterpret_cast<const __bf16*>(buf);
        f.a[kk] = *reinterpret_cast<const bf16x8*>(b16 + bsw<T>(a_row, kofs + kk * KG));
#pragma unroll
        for (int j = 0; j < FN; ++j)
          f.w[kk][j] = *reinterpret_cast<const bf16x8*>(b16 + bsw<T>(w_row + j * 32, kofs + kk * KG));
      } else if constexpr (PM == PM_SPLIT3) {
#pragma unroll
        for (int pc = 0; pc < 3; ++pc) {
          const __bf16* b16 = reinterpret_cast<const __bf16*>(buf) + pc * T::STAGEB;
          f.a[pc][kk] = *reinterpret_cast<const bf16x8*>(b16 + bsw<T>(a_row, kofs + kk * KG));
#pragma unroll
          for (int j = 0; j < FN; ++j)
            f.w[pc][kk][j] =
                *reinterpret_cast<const bf16x8*>(b16 + bsw<T>(w_row + j * 32, kofs + kk * KG));
        }
      } else {
        f.a[kk] = *reinterpret_cast<const float4*>(buf + a_off + kk * KG);
#pragma unroll
        for (int j = 0; j < FN; ++j)
          f.w[kk][j] = *reinterpret_cast<const float4*>(buf + w_off + j * 32 * PITCH + kk * KG);
      }
    }
  };
  auto mfma_kk = [&](floatx16 (&tg)[FN], const Frag& f, int kk) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      if constexpr (PM == PM_BF16) {
        tg[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[kk], f.w[kk][j], tg[j], 0, 0, 0);
      } else if constexpr (PM == PM_SPLIT3) {   // smallest terms first
        tg[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[2][kk], f.w[0][kk][j], tg[j], 0, 0, 0);
        tg[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[1][kk], f.w[1][kk][j], tg[j], 0, 0, 0);
        tg[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[0][kk], f.w[2][kk][j], tg[j], 0, 0, 0);
        tg[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[1][kk], f.w[0][kk][j], tg[j], 0, 0, 0);
        tg[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[0][kk], f.w[1][kk][j], tg[j], 0, 0, 0);
        tg[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[0][kk], f.w[0][kk][j], tg[j], 0, 0, 0);
      } else {
        tg[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a[kk].x, f.w[kk][j].x, tg[j], 0, 0, 0);
        tg[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a[kk].y, f.w[kk][j].y, tg[j], 0, 0, 0);
        tg[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a[kk].z, f.w[kk][j].z, tg[j], 0, 0, 0);
        tg[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a[kk].w, f.w[kk][j].w, tg[j], 0, 0, 0);
      }
    }
  };

  // PRO_HEADZ: the phi(q) part of K is 4 heads x 64 (HS = 64 / BKS stages each) after the
  // x part.  Each head accumulates into acc_h; its rows are scaled by Z*Ns and added to acc
  // when the head's stages are done.  Z's dot products phi(q)_row . ksum_h are taken from
  // the staged A tiles (TPR threads per row, ZK-wide k chunks) right after each stage's
  // fragment read.  zrow is double-buffered by head parity (one head per stage at BKS 64
  // leaves no barrier between one head's fold and the next head's Z).
  constexpr int HS = 64 / T::BKS;
  constexpr int TPR = T::NT / BM, ZK = T::BKS / TPR;
  static_assert(PRO != PRO_HEADZ || (HS >= 1 && T::BKS * HS == 64 && T::NT % BM == 0 &&
                                     ZK % 8 == 0 && ZK * TPR == T::BKS && 64 % TPR == 0),
                "HEADZ tiling");
  const int xs = c.ksplit / T::BKS;
  floatx16 acc_h[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc_h[j][i] = 0.f;
  // one running dot per 8-wide chunk: the head's Z is ((c0 + c1) + (c2 + c3)) over the four
  // chunks of each 32-deep stage whatever the threads per row (TPR 4: one chunk per thread and
  // a two-step butterfly; TPR 2: two chunks added, then one step)
  constexpr int ZC = ZK >= 8 ? ZK / 8 : 1;   // (tiles without HEADZ: unused)
  static_assert(PRO != PRO_HEADZ || (T::BKS == 32 ? ZK / 8 * TPR == 4 : TPR == 4),
                "Z's chunk tree (32-deep stages: four chunks per row)");
  float zp[ZC];
#pragma unroll
  for (int cc = 0; cc < ZC; ++cc) zp[cc] = 0.f;
  const int zr = t / TPR, zq = t % TPR;
  __shared__ float zks[(PRO == PRO_HEADZ) ? 256 : 1];   // sum phi(k) of the source
  if (PRO == PRO_HEADZ)
    for (int i = t; i < 256; i += T::NT) zks[i] = F(ksum)[b * F(ksum_bs) + i];   // 1st barrier
  const float zns = F(ns);
  auto zdot = [&](const float* buf, int sg) __attribute__((always_inline)) {
    if (PRO == PRO_HEADZ && sg >= xs && sg < nk) {
#pragma unroll
      for (int cc = 0; cc < ZK / 8; ++cc) {
        const int k8 = zq * ZK + cc * 8;
        const float* kp = zks + (sg * T::BKS - c.ksplit) + k8;   // LDS
        float4 a0, a1;
        if constexpr (PM == PM_BF16) {   // the phi(q) the bf16 MFMAs see
          const bf16x8 q = *reinterpret_cast<const bf16x8*>(
              reinterpret_cast<const __bf16*>(buf) + bsw<T>(zr, k8));
          a0 = make_float4((float)q[0], (float)q[1], (float)q[2], (float)q[3]);
          a1 = make_float4((float)q[4], (float)q[5], (float)q[6], (float)q[7]);
        } else if constexpr (PM == PM_SPLIT3) {   // hi + mid + lo = the fp32 value, exactly
          const __bf16* b16 = reinterpret_cast<const __bf16*>(buf) + bsw<T>(zr, k8);
          const bf16x8 q0 = *reinterpret_cast<const bf16x8*>(b16);
          const bf16x8 q1 = *reinterpret_cast<const bf16x8*>(b16 + T::STAGEB);
          const bf16x8 q2 = *reinterpret_cast<const bf16x8*>(b16 + 2 * T::STAGEB);
          float x[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] = ((float)q0[e] + (float)q1[e]) + (float)q2[e];
          a0 = make_float4(x[0], x[1], x[2], x[3]);
          a1 = make_float4(x[4], x[5], x[6], x[7]);
        } else {
          const float* ap = buf + zr * PITCH + k8;
          a0 = *reinterpret_cast<const float4*>(ap);
          a1 = *reinterpret_cast<const float4*>(ap + 4);
        }
        const float4 k0 = *reinterpret_cast<const float4*>(kp);
        const float4 k1 = *reinterpret_cast<const float4*>(kp + 4);
        zp[cc] = headz_dot8(zp[cc], a0, a1, k0, k1);
      }
    }
  };
  auto zfinal = [&](int par) __attribute__((always_inline)) {   // the head's partials are in zp
    float z = zp[0];
    if constexpr (ZC == 2) z = zp[0] + zp[1];
    if constexpr (ZC == 4) z = (zp[0] + zp[1]) + (zp[2] + zp[3]);
#pragma unroll
    for (int o = 1; o < TPR; o <<= 1) z += __shfl_xor(z, o, 64);
    if (zq == 0) zrow[par * BM + zr] = (1.0f / (z + 1e-6f)) * zns;
#pragma unroll
    for (int cc = 0; cc < ZC; ++cc) zp[cc] = 0.f;
  };
  auto fold = [&](int par) __attribute__((always_inline)) {     // acc += Z*Ns (per row) * acc_h
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
        acc[j][i] = headz_fold(acc[j][i], zrow[par * BM + row], acc_h[j][i]);
        acc_h[j][i] = 0.f;
      }
  };

  // PRO_HEADZ with acc0: the x range's accumulators were computed before (EPI_ACC, the same
  // MFMA sequence); start from them at stage xs (even, so it sits in LDS buffer 0 like stage 0)
  const float* acc0 = PRO == PRO_HEADZ ? F(acc0) : nullptr;
  const int kt0 = acc0 != nullptr ? xs : 0;
  if (acc0 != nullptr && T::NSUB == 1) {
    const float* a0p = acc0 + b * F(acc0_bs) + ((int64_t)(mt * ntiles + nt) * T::NW + wave) * FN * 1024 + lane;
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[j][i] = a0p[j * 1024 + i * 64];
  } else if (acc0 != nullptr) {
    // acc0 as the 64 x SUBN four-wave tile stored it (2 x 2 waves of 32 x SUBN / 2, FNp
    // accumulators each): this wave's 32 rows are sub-tile wm / 2's wave row wm % 2; its
    // 32-column block cb (global column n0 + 32 cb) is that tile's column tile (n0 + 32 cb) /
    // SUBN, wave column cbp / FNp, accumulator cbp % FNp for cbp = its block within that tile
    // (sub-tiles past M hold nothing and are never stored)
    constexpr int SN = T::SUBN, FNP = SN / 64;
    static_assert(T::NSUB == 1 || (T::SUB == 64 && T::KS == 1 && (SN == 64 || SN == 128) &&
                                   (BN % SN == 0 || SN % BN == 0)),
                  "acc0 of 64-row sub-tiles");
    const int st = mt * T::NSUB + wm / 2;
    const int ntp = c.N / SN;   // the stand-in grid's column tiles
    if (st * 64 < c.M) {
      const float* a0b = acc0 + b * F(acc0_bs) + lane;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int gc = n0 + (wn * FN + j) * 32, cbp = (gc % SN) / 32;
        const float* a0p = a0b + ((int64_t)(st * ntp + gc / SN) * 4 + (wm % 2) * 2 + cbp / FNP) *
                                     FNP * 1024 + (cbp % FNP) * 1024;
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[j][i] = a0p[i * 64];
      }
    }
  }
  if constexpr (DMA >= 1) {
    // The lean DMA loop.  A bf16 stage is only 4-12 MFMAs per wave, so the loop is bound by the
    // instructions around them and by load latency, not by the matrix pipe:
    //  - row / piece offsets are computed once (32-bit, added to a wave-uniform base per stage);
    //  - the x range and each phi(q) head run in loops of their own with the accumulator set
    //    fixed (no accumulator copies or per-stage branches on the head state);
    //  - the stage's LDS reads come before the next stages' loads in program order, and the
    //    barrier is a raw s_barrier after lgkmcnt(0): __syncthreads()' fence would drain every
    //    load and DMA in flight (vmcnt(0)) and undo the lookahead.
    // A and W LA = NBUF - 1 stages ahead: one in two LDS buffers, two in three for the bf16
    // DMA-2 loop (A staged through registers with two stages ahead -- two A register sets --
    // measured no faster).  With the MFMAs under the loads (the scheduling barrier in `stage`),
    // a stage's time follows the bytes its workgroup moves.  Same
    // images, fragments and MFMA order as the register-staged loop, so the same bits.
    static_assert(WPL && PM != PM_F32, "DMA loop: bf16 images, W planes");
    // DMA 2: A from its activation planes too -- no VALU rounding / split, no LDS stores of A
    constexpr bool ADMA = DMA == 2;
    static_assert(!ADMA || PRO != PRO_NORM_RELU, "A planes: no prologue transform");
    // a W piece = one 1-KB global_load_lds: RP rows of BKS bf16 (CPR 16-B chunks per row)
    constexpr int CPR = T::BKS / 8, RP = 64 / CPR;
    constexpr int PIECES = NPL * T::BN / RP, PPW = PIECES / T::NW;
    static_assert((T::BKS == 32 || T::BKS == 64) && T::BN % RP == 0 && PIECES % T::NW == 0,
                  "W pieces");
    const int kq = (t % T::KQ) * 4;
    unsigned aoff0[T::A4], aoff1[T::A4];   // bytes from the stage's base, per K range
#pragma unroll
    for (int i = 0; i < T::A4; ++i) {
      const int m = min(m0 + (t + T::NT * i) / T::KQ, c.M - 1);
      aoff0[i] = (unsigned)((m * c.lda0 + kq) * 4);
      aoff1[i] = (unsigned)((m * c.lda1 + kq) * 4);
    }
    unsigned woff0[PPW], woff1[PPW];
    int wdst[PPW];
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int p = wave + T::NW * i;
      const int q = p / (T::BN / RP), rb = (p % (T::BN / RP)) * RP;
      const int row = T::BM + rb + lane / CPR;   // image row; LDS slot lane % CPR holds the
      const int chunk = bsw<T>(row, (lane % CPR) * 8) - row * T::BKS;   // chunk bsw puts there
      const int o = min(n0 + rb + lane / CPR, c.N - 1);
      woff0[i] = (unsigned)((q * c.wpl0 + (int64_t)o * c.ldw0 + chunk) * 2);
      woff1[i] = (unsigned)((q * c.wpl1 + (int64_t)o * c.ldw1 + chunk) * 2);
      wdst[i] = q * T::STAGEB * 2 + (T::BM + rb) * T::BKS * 2;
    }
    // A pieces (DMA 2): NPL planes x BM rows in 1-KB pieces, dealt to the waves in turn (a
    // wave-uniform predicate skips the slots past the last piece)
    constexpr int APIECES = NPL * BM / RP, APPW = (APIECES + T::NW - 1) / T::NW;
    static_assert(!ADMA || BM % RP == 0, "A pieces");
    unsigned apoff0[ADMA ? APPW : 1], apoff1[ADMA ? APPW : 1];
    int adst[ADMA ? APPW : 1];
    if constexpr (ADMA) {
#pragma unroll
      for (int i = 0; i < APPW; ++i) {
        const int p = min(wave + T::NW * i, APIECES - 1);
        const int q = p / (BM / RP), rb = (p % (BM / RP)) * RP;
        const int row = rb + lane / CPR;   // A image row; slot lane % CPR holds bsw's chunk
        const int chunk = bsw<T>(row, (lane % CPR) * 8) - row * T::BKS;
        const int m = min(m0 + row, c.M - 1);
        apoff0[i] = (unsigned)((q * c.apl0 + (int64_t)m * c.ldap0 + chunk) * 2);
        apoff1[i] = (unsigned)((q * c.apl1 + (int64_t)m * c.ldap1 + chunk) * 2);
        adst[i] = q * T::STAGEB * 2 + rb * T::BKS * 2;
      }
    }
    Stage<T, WPL, NPL> sa;
    auto load_a = [&](int k0) __attribute__((always_inline)) {
      const bool first = PRO != PRO_HEADZ || k0 < c.ksplit;   // one K range but for HEADZ
      const char* base =
          reinterpret_cast<const char*>(first ? c.a0 + k0 : c.a1 + (k0 - c.ksplit));
#pragma unroll
      for (int i = 0; i < T::A4; ++i)
        sa.a[i] = *reinterpret_cast<const float4*>(base + (first ? aoff0[i] : aoff1[i]));
      if (PRO == PRO_NORM_RELU) {
        sa.mean = *reinterpret_cast<const float4*>(c.mean + k0 + kq);
        sa.rstd = *reinterpret_cast<const float4*>(c.rstd + k0 + kq);
      }
    };
    auto buf = [&](int st) __attribute__((always_inline)) { return lds + (st % NBUF) * STAGE; };
    // LA stages of loads in flight: stage kt's MFMAs run while stages kt + 1 .. kt + LA load;
    // at the end of stage kt a wave waits only for stage kt + 1's OPS loads (vmcnt counts in
    // order), so with LA = 2 a load has two stages' time to land instead of one
    constexpr int LA = NBUF - 1;
    constexpr int OPS = PPW + (ADMA ? APPW : 0);   // DMA instructions per wave and stage
    static_assert(LA == 1 || (ADMA && APIECES % T::NW == 0 && (LA - 1) * OPS <= 63),
                  "two stages ahead: A by DMA, the same instruction count on every wave");
    auto dma_w = [&](int st) __attribute__((always_inline)) {
      const int k0 = st * T::BKS;
      const bool first = PRO != PRO_HEADZ || k0 < c.ksplit;
      const char* base =
          reinterpret_cast<const char*>(first ? c.wp0 + k0 : c.wp1 + (k0 - c.ksplit));
      char* dst = reinterpret_cast<char*>(buf(st));
#pragma unroll
      for (int i = 0; i < PPW; ++i)
        dma16(base + (first ? woff0[i] : woff1[i]), dst + wdst[i]);
    };
    auto dma_a = [&](int st) __attribute__((always_inline)) {
      const int k0 = st * T::BKS;
      const bool first = PRO != PRO_HEADZ || k0 < c.ksplit;
      const char* base =
          reinterpret_cast<const char*>(first ? c.ap0 + k0 : c.ap1 + (k0 - c.ksplit));
      char* dst = reinterpret_cast<char*>(buf(st));
#pragma unroll
      for (int i = 0; i < APPW; ++i)
        if (APIECES % T::NW == 0 || wave + T::NW * i < APIECES)
          dma16(base + (first ? apoff0[i] : apoff1[i]), dst + adst[i]);
    };
    // the next stage's A: its planes by DMA, or its fp32 values into registers (stored to LDS,
    // rounded / split, once the stage's MFMAs are issued)
    auto next_a = [&](int st) __attribute__((always_inline)) {
      if constexpr (ADMA) dma_a(st);
      else load_a(st * T::BKS);
    };
    auto raw_barrier = [&]() __attribute__((always_inline)) {
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
    next_a(kt0);
    dma_w(kt0);
#pragma unroll
    for (int s = 1; s < LA; ++s)
      if (kt0 + s < nk) {
        next_a(kt0 + s);
        dma_w(kt0 + s);
      }
    tk = stamp_start(args.stamp, sl);
    if (LA >= 2 && kt0 + LA - 1 < nk)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((LA - 1) * OPS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (!ADMA) store_stage<PRO, T, PM, WPL, NPL, false>(buf(kt0), sa);
    raw_barrier();
    // @phase 1
    // one stage: kt's fragments into tg (zd: phi(q) stage, its Z partials; zf >= 0: the head's
    // last stage, its Z rows to zrow[zf])
    auto stage = [&](int kt, floatx16 (&tg)[FN], bool zd, int zf) __attribute__((always_inline)) {
      float* cur = buf(kt);
      read_frag(cur, f0);
      if (zd) zdot(cur, kt);
      const bool more = kt + LA < nk;   // (the buffer stage kt + LA loads into was last read
      if (more) {                       //  in stage kt - 1, before that stage's barrier)
        dma_w(kt + LA);
        next_a(kt + LA);
      }
#pragma unroll
      for (int kk = 0; kk < KKW; ++kk) mfma_kk(tg, f0, kk);
      if (zf >= 0) zfinal(zf);
      // keep the MFMAs above the wait: register-only, the scheduler would otherwise sink all but
      // the first below the inline wait + barrier (measured so: the DMA's latency then runs
      // alone, before the stage's MFMAs, instead of under them)
      ONEPOSE_SCHED_BARRIER();
      if (LA >= 2 && more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((LA - 1) * OPS) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (!ADMA && more) store_stage<PRO, T, PM, WPL, NPL, false>(buf(kt + 1), sa);
      raw_barrier();
    };
    if (PRO != PRO_HEADZ) {
      for (int kt = kt0; kt < nk; ++kt) stage(kt, acc, false, -1);
    } else {
      for (int kt = kt0; kt < xs; ++kt) stage(kt, acc, false, -1);
#pragma unroll 1
      for (int h = 0; h < 4; ++h) {
#pragma unroll 1
        for (int st = 0; st < HS; ++st) stage(xs + h * HS + st, acc_h, true, st == HS - 1 ? (h & 1) : -1);
        fold(h & 1);   // after the stage's barrier: every row's Z is in zrow
      }
    }
    // @phase 2
  } else {
  load_stage<PRO, T, WPL, NPL>(c, m0, n0, kt0 * T::BKS, s0);
  load_stage<PRO, T, WPL, NPL>(c, m0, n0, (kt0 + 1) * T::BKS, s1);
  tk = stamp_start(args.stamp, sl);
  store_stage<PRO, T, PM, WPL, NPL>(lds, s0);
  __syncthreads();
  // @phase 1
  read_frag(lds, f0);
  zdot(lds, kt0);   // the first phi(q) stage's Z partials when the x range is skipped

  auto step = [&](int kt, Stage<T, WPL, NPL>& next, Stage<T, WPL, NPL>& spare, const Frag& cur, Frag& nxt,
                  floatx16 (&tg)[FN]) __attribute__((always_inline)) {
    // unconditional: past the end the last stage is re-read into the spare set and ignored
    load_stage<PRO, T, WPL, NPL>(c, m0, n0, min(kt + 2, nk - 1) * T::BKS, spare);
    mfma_kk(tg, cur, 0);
    ONEPOSE_SCHED_BARRIER();
    float* na = lds + ((kt + 1) & 1) * STAGE;
    store_stage<PRO, T, PM, WPL, NPL>(na, next);                // (unused after the last step)
    ONEPOSE_SCHED_BARRIER();
#pragma unroll
    for (int kk = 1; kk < KKW - 1; ++kk) mfma_kk(tg, cur, kk);
    __syncthreads();
    read_frag(na, nxt);                               // (unused after the last step)
    zdot(na, kt + 1);
    ONEPOSE_SCHED_BARRIER();
    mfma_kk(tg, cur, KKW - 1);
    ONEPOSE_SCHED_BARRIER();
  };
  if (PRO != PRO_HEADZ) {
    for (int kt = 0; kt < nk; kt += 2) {   // nk is even (checked at launch)
      step(kt, s1, s0, f0, f1, acc);
      step(kt + 1, s0, s1, f1, f0, acc);
    }
  } else {
    for (int kt = kt0; kt < xs; kt += 2) {   // x part
      step(kt, s1, s0, f0, f1, acc);
      step(kt + 1, s0, s1, f1, f0, acc);
    }
    if constexpr (HS == 2) {
      for (int kt = xs; kt < nk; kt += 2) {  // one head of phi(q) per two stages
        step(kt, s1, s0, f0, f1, acc_h);
        zfinal(0);                           // visible to every wave after the next barrier
        step(kt + 1, s0, s1, f1, f0, acc_h);
        fold(0);
      }
    } else {
      for (int kt = xs; kt < nk; kt += 2) {  // one head per stage; its Z partials were taken
        zfinal(0);                           // while the previous step read the stage
        step(kt, s1, s0, f0, f1, acc_h);
        fold(0);
        zfinal(1);
        step(kt + 1, s0, s1, f1, f0, acc_h);
        fold(1);
      }
    }
  }
  // @phase 2
  }   // (register-staged loop)
  __syncthreads();   // every wave done with the LDS stages before they are reused below
  // profiling ticket after the K loop: no in-loop wait (vmcnt counts in order) includes the
  // atomic; its value is needed only at the end
  stamp_ticket(args.stamp, tk);

  // ---- k-slice reduction: slices 1..KS-1 add into slice 0 in order (deterministic) ----
  if (T::KS > 1) {
    float* red = lds;   // [KS-1][WM*WN][FN][16][64]
    static_assert((T::KS - 1) * T::WM * T::WN * FN * 16 * 64 <= LDSF, "reduction fits");
    const int blk = wave % (T::WM * T::WN);
    if (ks > 0) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          red[((((ks - 1) * T::WM * T::WN + blk) * FN + j) * 16 + i) * 64 + lane] = acc[j][i];
    }
    __syncthreads();
    if (ks == 0) {
      for (int s = 1; s < T::KS; ++s)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            acc[j][i] += red[((((s - 1) * T::WM * T::WN + blk) * FN + j) * 16 + i) * 64 + lane];
    }
    __syncthreads();
  }

  // ---- epilogue (waves of slice 0 own the accumulators) ----
  const int M = c.M, N = c.N;
  const float* biasp = F(bias);
  float* Y = F(Y) + b * F(y_bs);
  const int ldy = F(ldy);
  float* tile = lds;   // [BM][TP] staging
  constexpr bool kStage = EPI == EPI_STATS || EPI == EPI_SCORE;
  // BIAS / STATS / RESID: the tile is staged and stored by rows of float4 (1 KB per wave
  // instruction) instead of 4-B stores in the accumulator layout (2 rows x 128 B each): the
  // store-issue-bound tail of the epilogue is 4x shorter; RESID reads R the same way.
  constexpr bool kRowStore =
      EPI == EPI_BIAS || EPI == EPI_STATS || EPI == EPI_RESID || EPI == EPI_BIAS_L2;

  if (EPI == EPI_ACC) {   // raw accumulators in register order (a later PRO_HEADZ's acc0)
    if (ks == 0) {
      float* yp = Y + ((int64_t)(mt * ntiles + nt) * T::NW + wave) * FN * 1024 + lane;
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) yp[j * 1024 + i * 64] = acc[j][i];
    }
    return;
  }
  const int rows = min(BM, M - m0);
  if constexpr (EPI == EPI_QKV) {
    // 128-column tiles of [q (256) | k_0 v_0 | .. | k_3 v_3].  q tiles: phi(q) = elu(q) + 1,
    // stored by float4 rows.  [k_h | v_h] tiles: phi(k) and v / vdiv staged transposed,
    // [column][even rows | odd rows], so that KV_h = phi(k)^T v's MFMAs (MFMA m takes rows 2m,
    // 2m + 1 from lane halves 0, 1) read their operands as float4 runs of one column, and the
    // phi(k) column sums run down the column in row order: the same sums, in the same order, as
    // a row-major staging.
    // (a stand-in tile, SUB = 64 < BM, writes its 64-row sub-tiles' partials: the same chunks,
    // sums and bits as the 64-row tile; four waves per sub-tile)
    static_assert(BN == 128 && T::NW == 4 * T::NSUB && T::KS == 1 && (T::NSUB == 1 || T::SUB == 64),
                  "QKV tile is [k_h | v_h]");
    constexpr int PT = BM + 4;
    const bool q_tile = n0 < 256;
    constexpr int HALF = BM / 2;
    float* tileT = lds;                 // [BN][PT]: even rows at [0, HALF), odd at [HALF, BM)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = wn * FN * 32 + j * 32 + (lane & 31);
      const float bias = bias_pre[j];   // (n0 + col < N = 768 on every QKV tile)
      // v / vdiv: for a power-of-two source length the product with its reciprocal is the
      // same number (exact scaling), without the division's instruction sequence
      const float vdiv = F(vdiv), vrcp = 1.0f / vdiv;
      const bool vpow2 = __builtin_amdgcn_frexp_mant(vdiv) == 0.5f;
      float yv[16];
      auto fill = [&](auto f) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int gm = m0 + wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
          yv[i] = gm < M ? f(acc[j][i] + bias) : 0.f;
        }
      };
      // (the column kind is uniform over the wave's 32-column accumulator block)
      if (q_tile || col < 64)
        fill([&](float y) { return elu1(y) + 1.0f; });   // phi(q), phi(k)
      else if (vpow2)
        fill([&](float y) { return y * vrcp; });          // v / vdiv
      else
        fill([&](float y) { return y / vdiv; });
      if (q_tile) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          tile[(wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5)) * TP + col] = yv[i];
      } else {
        // rows wm 32 + 8 a + 4 h + {0..3}: two even (j = 0, 2) and two odd (j = 1, 3) rows,
        // consecutive within their halves
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          const int e = col * PT + wm * 16 + 4 * a + 2 * (lane >> 5);
          *reinterpret_cast<float2*>(tileT + e) = make_float2(yv[4 * a], yv[4 * a + 2]);
          *reinterpret_cast<float2*>(tileT + e + HALF) = make_float2(yv[4 * a + 1], yv[4 * a + 3]);
        }
      }
    }
    __syncthreads();
    if (q_tile) {
      constexpr int C4 = BN / 4, PER = BM * C4 / T::NT;
      uint16_t* yp = F(Yp);   // phi(q)'s activation planes (bf16 modes), the next A operand
      if (yp != nullptr) yp += b * F(yp_bs);
      const int64_t ypl = F(ypl);
#pragma unroll
      for (int p = 0; p < PER; ++p) {
        const int idx = t + T::NT * p, r = idx / C4, cc = (idx % C4) * 4;
        if (m0 + r < M) {
          const float4 v = *reinterpret_cast<const float4*>(tile + r * TP + cc);
          *reinterpret_cast<float4*>(Y + (int64_t)(m0 + r) * ldy + n0 + cc) = v;
          if (NPL_OUT > 0 && yp != nullptr)
            store_planes4(yp + (int64_t)(m0 + r) * ldy + n0 + cc, ypl, NPL_OUT, v);
        }
      }
      return;
    }
    const int h = (n0 - 256) / 128;
    constexpr int SH = HALF / T::NSUB;   // a sub-tile's rows per half
    const int mtiles_s = T::NSUB == 1 ? mtiles : (M + 63) / 64;
    if (t < 64 * T::NSUB && (t / 64) * (BM / T::NSUB) < rows) {
      // sum phi(k) over the (sub-)tile's rows, in row order (invalid rows hold 0)
      const int sb = t / 64, tc = t % 64;
      const float* cp = tileT + tc * PT + sb * SH;
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < SH; q += 4) {
        const float4 ev = *reinterpret_cast<const float4*>(cp + q);
        const float4 od = *reinterpret_cast<const float4*>(cp + HALF + q);
        s += ev.x;
        s += od.x;
        s += ev.y;
        s += od.y;
        s += ev.z;
        s += od.z;
        s += ev.w;
        s += od.w;
      }
      F(kspart)[((int64_t)b * mtiles_s + mt * T::NSUB + sb) * 256 + h * 64 + tc] = s;
    }
    const int sbw = wave / 4, wv = wave % 4;   // the wave's sub-tile
    if (sbw * (BM / T::NSUB) >= rows) return;   // (a sub-tile past M: no chunk)
    const int wd = wv >> 1, wq = wv & 1;
    floatx16 kv;
#pragma unroll
    for (int i = 0; i < 16; ++i) kv[i] = 0.f;
    const float* ka = tileT + (wd * 32 + (lane & 31)) * PT + HALF * (lane >> 5) + sbw * SH;
    const float* vb = tileT + (64 + wq * 32 + (lane & 31)) * PT + HALF * (lane >> 5) + sbw * SH;
#pragma unroll
    for (int q = 0; q < SH; q += 4) {   // MFMAs m = q .. q + 3: rows 2m + lane half
      const float4 a4 = *reinterpret_cast<const float4*>(ka + q);
      const float4 b4 = *reinterpret_cast<const float4*>(vb + q);
      kv = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, b4.x, kv, 0, 0, 0);
      kv = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, b4.y, kv, 0, 0, 0);
      kv = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, b4.z, kv, 0, 0, 0);
      kv = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, b4.w, kv, 0, 0, 0);
    }
    float* out = F(kvpart) + (((int64_t)b * mtiles_s + mt * T::NSUB + sbw) * 4 + h) * 4096;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int d = wd * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
      out[d * 64 + wq * 32 + (lane & 31)] = kv[i];
    }
    return;
  }
  if (ks == 0) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = wn * FN * 32 + j * 32 + (lane & 31);
      const int gn = n0 + col;
      const bool col_ok = gn < N;
      const float bias = bias_pre[j];   // (0 past N, for SCORE, or without a bias)
      float yv[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
        const int gm = m0 + row;
        float y;
        if (EPI == EPI_SCORE) {
          y = acc[j][i] / F(scale);
        } else {
          y = acc[j][i] + bias;
        }
        yv[i] = (gm < M) ? y : 0.f;
        if (kStage || kRowStore) tile[row * TP + col] = yv[i];
      }
      if (EPI == EPI_STATS) {
        // the column's (mean, M2) over this wave's 32 rows, from the registers: each lane's 16
        // rows, then the lane pair (lane, lane ^ 32) added in the same order on both lanes
        const int cw = max(min(rows - wm * 32, 32), 0);   // valid rows of the wave's block
        float su = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) su += yv[i];          // invalid rows hold 0
        const float so = __shfl_xor(su, 32, 64);
        const float ssum = (lane < 32) ? su + so : so + su;
        const float wmean = cw ? ssum / (float)cw : 0.f;
        float m2 = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int row = wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
          const float d = yv[i] - wmean;
          m2 += (row < rows) ? d * d : 0.f;
        }
        const float mo = __shfl_xor(m2, 32, 64);
        if (lane < 32) {
          part[(wm * BN + col) * 2] = wmean;
          part[(wm * BN + col) * 2 + 1] = m2 + mo;
        }
      }
    }
  }
  if (!kStage && !kRowStore) return;
  __syncthreads();
  // @phase 4
  // the row-store pass (STATS: issued behind its ticket's round trip, below)
  uint16_t* yp = EPI == EPI_RESID ? F(Yp) : nullptr;   // RESID: the output's planes
  if (yp != nullptr) yp += b * F(yp_bs);
  const int64_t ypl = F(ypl);
  auto row_store = [&]() __attribute__((always_inline)) {
    constexpr int C4 = BN / 4, PER = BM * C4 / T::NT;   // float4 per row, per thread
    static_assert(BM * C4 % T::NT == 0, "row-store pass");
    float4 rv[EPI == EPI_RESID ? PER : 1];
    if constexpr (kRPre) {
#pragma unroll
      for (int p = 0; p < PER; ++p) rv[p] = r_pre[p];
    } else if (EPI == EPI_RESID) {   // all residual loads issued before the first store
      const float* R = F(R) + b * F(r_bs);
      const int ldr = F(ldr);
#pragma unroll
      for (int p = 0; p < PER; ++p) {
        const int idx = t + T::NT * p, r = idx / C4, cc = (idx % C4) * 4;
        const int gm = min(m0 + r, M - 1), gn = min(n0 + cc, N - 4);
        rv[p] = *reinterpret_cast<const float4*>(R + (int64_t)gm * ldr + gn);
      }
    }
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int idx = t + T::NT * p, r = idx / C4, cc = (idx % C4) * 4;
      const int gm = m0 + r, gn = n0 + cc;
      if (gm < M && gn < N) {   // N % 4 == 0 (checked at launch)
        float4 v = *reinterpret_cast<const float4*>(tile + r * TP + cc);
        if (EPI == EPI_RESID) {   // R + (acc + bias), as the reference adds
          v.x = rv[p].x + v.x;
          v.y = rv[p].y + v.y;
          v.z = rv[p].z + v.z;
          v.w = rv[p].w + v.w;
        }
        *reinterpret_cast<float4*>(Y + (int64_t)gm * ldy + gn) = v;
        if (EPI == EPI_RESID && NPL_OUT > 0 && yp != nullptr)
          store_planes4(yp + (int64_t)gm * ldy + gn, ypl, NPL_OUT, v);
      }
    }
  };
  if constexpr (EPI == EPI_BIAS || EPI == EPI_RESID) {
    row_store();
    return;
  }
  if constexpr (EPI == EPI_BIAS_L2) {
    // F.normalize(y, p=2, dim=channels) (GATs_SuperGlue.py:245-246) on the staged rows: one wave
    // per row, lane l holding channels 4l..4l+3 -- the arithmetic of l2norm_kernel (the squares
    // of a lane's four channels, then the wave butterfly, max(sqrt, 1e-12), four divisions), so
    // the normalised rows are the bits the separate kernel wrote
    static_assert(EPI != EPI_BIAS_L2 || BN == 256, "whole rows");
    for (int r = wave; r < rows; r += T::NW) {
      float4 v = *reinterpret_cast<const float4*>(tile + r * TP + lane * 4);
      const float ss = wave_sum(v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w);
      const float n = fmaxf(sqrtf(ss), 1e-12f);
      v.x /= n;
      v.y /= n;
      v.z /= n;
      v.w /= n;
      *reinterpret_cast<float4*>(Y + (int64_t)(m0 + r) * ldy + lane * 4) = v;
    }
    return;
  }

  if (EPI == EPI_STATS) {
    // per column and SUB-row sub-tile: its wave-row blocks' (mean, M2 about the block mean)
    // (staged in `part` before the barrier above), Chan-merged in order.  SUB = BM but for the
    // tiles that stand in for several 64-row tiles (Tile::SUB): their partials, tickets and
    // merges are those tiles', sub-tile by sub-tile.
    constexpr int SUB = T::SUB, NSUB = T::NSUB, RG = 32, NRG = SUB / RG;
    static_assert(EPI != EPI_STATS || (T::KS == 1 && T::WN * T::WM == T::NW && NSUB * BN <= T::NT &&
                                       BM % SUB == 0 && SUB % RG == 0),
                  "stats tile");
    const int mtiles_s = NSUB == 1 ? mtiles : (M + SUB - 1) / SUB;
    const int tc = t % BN, ts = t / BN;   // merging thread: column, sub-tile
    const int mt_s = mt * NSUB + ts;
    if (t < NSUB * BN && n0 + tc < N && ts * SUB < rows) {
      float n = 0.f, mean = 0.f, M2 = 0.f;
      for (int g = ts * NRG; g < ts * NRG + NRG; ++g) {
        const float nb = (float)max(min(g * RG + RG, rows) - g * RG, 0);
        if (nb == 0.f) continue;
        const float mb = part[(g * BN + tc) * 2], m2b = part[(g * BN + tc) * 2 + 1];
        in_merge_block(n, mean, M2, nb, mb, m2b);
      }
      float* st_out = F(stats) + ((int64_t)b * mtiles_s + mt_s) * 2 * N;
      if (F(st_cnt) != nullptr) {   // handed to this launch's last tile: write-through (sc1)
        __hip_atomic_store(st_out + n0 + tc, mean, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(st_out + N + n0 + tc, M2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        st_out[n0 + tc] = mean;
        st_out[N + n0 + tc] = M2;
      }
    }
    // InstanceNorm finalize in-launch (replaces a separate reduction launch): every M-tile of
    // this (sample, column block) takes a ticket after its write-through (sc1) partial stores
    // have drained; the one drawing mtiles - 1 reads all mtiles partials with sc1 loads and
    // reduces them in tile order, so the result does not depend on which tile arrives last.
    // Every store and load of the handed-off partials is sc1, so neither an agent-scope
    // release (it would write back the XCD's L2, this tile's Y in it) nor an acquire (an L1
    // invalidate, ~1.7 us) is needed.  The counters are zeroed by the forward's first kernel.
    unsigned* tickets = F(st_cnt);
    if (tickets == nullptr) {
      row_store();
    } else {
      // Two-level finalize.  Every store and load of the handed-off partials is sc1
      // (write-through / L2), so neither an agent-scope release (it would write back the XCD's
      // L2, this tile's Y in it) nor an acquire (an L1 invalidate, ~1.7 us) is needed.
      //  1. each M-tile takes a ticket on its group (kStatsGroup consecutive M-tiles) after its
      //     partial stores drained; the group's last tile merges the group's partials in tile
      //     order (shifted by the group's first mean) into st_grp -- while the other groups'
      //     tiles still compute;
      //  2. that merger takes a ticket on the column block; the last one merges the groups in
      //     group order (shifted by group 0's mean) into mean / rstd.
      // Deterministic: neither result depends on which tile or group arrives last.  (A tile of
      // several sub-tiles takes one ticket per sub-tile, and may close two groups.)
      static_assert(EPI != EPI_STATS || T::NT >= BN, "finalize threads");
      const int G = stats_group_size(mtiles_s);
      const int ngroups = (mtiles_s + G - 1) / G;
      unsigned* cb = tickets + (int64_t)b * F(st_cnt_bs);   // [ntiles] then [ntiles][ngroups]
      double* gp = F(st_grp) + (int64_t)b * ngroups * 2 * N;
      const int col = min(n0 + t, N - 1);
      if (t < NSUB * BN) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // storing waves drain
      __syncthreads();   // partial stores drained; `part` no longer read
      // @phase 5
      int* last = reinterpret_cast<int*>(part);   // [NSUB] group closed by sub-tile s, then [NSUB]
      unsigned ticket = 0u;
      const bool tk_thread = t % BN == 0 && ts < NSUB && ts * SUB < rows;
      if (tk_thread)
        ticket = __hip_atomic_fetch_add(cb + ntiles + nt * ngroups + mt_s / G, 1u,
                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      row_store();   // the tile's Y rows, while the tickets are in flight
      if (t % BN == 0 && ts < NSUB) {
        const int gt0 = (mt_s / G) * G, gsz = min(G, mtiles_s - gt0);
        last[ts] = tk_thread && ticket == (unsigned)(gsz - 1) ? 1 : 0;
      }
      __syncthreads();
      // @phase 6
      for (int s = 0; s < NSUB; ++s) {
        if (!last[s]) continue;
        const int g1 = (mt * NSUB + s) / G, gt0 = g1 * G, gsz = min(G, mtiles_s - gt0);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // (no instruction: keeps the
                                                                 // loads below the ticket)
        if (t < BN) {
          const float* sp = F(stats) + (int64_t)b * mtiles_s * 2 * N + col;
          auto ld = [&](int ti, int half) __attribute__((always_inline)) {
            return __hip_atomic_load(sp + (int64_t)ti * 2 * N + half * N, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
          };
          const double c = (double)ld(gt0, 0);
          double s1 = 0.0, s2 = 0.0, ng = 0.0;
          constexpr int UD = 16;   // tiles' partials in flight per thread
          for (int u0 = 0; u0 < gsz; u0 += UD) {
            float mv[UD], qv[UD];
#pragma unroll
            for (int u = 0; u < UD; ++u) {
              const int ti = gt0 + min(u0 + u, gsz - 1);
              mv[u] = ld(ti, 0);
              qv[u] = ld(ti, 1);
            }
#pragma unroll
            for (int u = 0; u < UD; ++u) {
              if (u0 + u < gsz)
                in_merge_tile(s1, s2, ng, (double)min(SUB, M - (gt0 + u0 + u) * SUB), mv[u], qv[u], c);
            }
          }
          if (n0 + t < N) {
            __hip_atomic_store(gp + (int64_t)g1 * 2 * N + n0 + t, in_group_mean(c, s1, ng),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(gp + (int64_t)g1 * 2 * N + N + n0 + t, in_group_m2(s1, s2, ng),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        if (t == 0) {
          const unsigned t2 = __hip_atomic_fetch_add(cb + nt, 1u, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
          last[NSUB] = t2 == (unsigned)(ngroups - 1) ? 1 : 0;
        }
        __syncthreads();
        if (last[NSUB] && t < BN && n0 + t < N) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          const double* g2 = gp + n0 + t;
          auto ld2 = [&](int g, int half) __attribute__((always_inline)) {
            return __hip_atomic_load(g2 + (int64_t)g * 2 * N + half * N, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
          };
          const double c = ld2(0, 0);
          double S1 = 0.0, S2 = 0.0;
          constexpr int GD = kStatsMaxGroups;   // every group's partials in flight at once
          for (int q0 = 0; q0 < ngroups; q0 += GD) {
            double mg[GD], m2g[GD];
#pragma unroll
            for (int u = 0; u < GD; ++u) {
              const int g = min(q0 + u, ngroups - 1);
              mg[u] = ld2(g, 0);
              m2g[u] = ld2(g, 1);
            }
#pragma unroll
            for (int u = 0; u < GD; ++u) {
              const int g = q0 + u;
              if (g < ngroups)
                in_merge_group(S1, S2, (double)min(G * SUB, M - g * G * SUB), mg[u], m2g[u], c);
            }
          }
          const double n = (double)M;
          F(st_mean)[(int64_t)b * N + n0 + t] = in_final_mean(c, S1, n);
          F(st_rstd)[(int64_t)b * N + n0 + t] = in_final_rstd(S1, S2, n);
        }
      }
    }
  }
  if (EPI == EPI_SCORE) {
    // Per-tile softmax partials, (max, sum exp) of every row over the tile's columns and of
    // every column over its rows.  Four threads per row (then per column) take 16 entries
    // each; the quarters are combined by lane butterflies ((q0 + q1) + (q2 + q3), fixed
    // order).  Reads of the staged tile are bank-conflict free both ways (pitch BN + 1).
    static_assert(EPI != EPI_SCORE || (T::NT >= 4 * BM && T::NT >= 4 * BN && BM % 16 == 0 &&
                                       BN % 16 == 0 && BM <= 128 && BN <= 128), "score tile");
    const int cols = min(BN, N - n0);
    // S from the staged tile by rows, four consecutive columns per thread (one 16-B store per
    // thread and row instead of a 4-B store per accumulator element: the same values)
    {
      constexpr int C4 = BN / 4, PER = BM * C4 / T::NT;
      static_assert(EPI != EPI_SCORE || BM * C4 % T::NT == 0, "score row pass");
      const bool vec = (ldy & 3) == 0 && (n0 & 3) == 0;
#pragma unroll
      for (int p = 0; p < PER; ++p) {
        const int idx = t + T::NT * p, r = idx / C4, cc = (idx % C4) * 4;
        const int gm = m0 + r, gn = n0 + cc;
        if (gm >= M) continue;
        const float* tr = tile + r * TP + cc;   // (pitch BN + 1: scalar reads)
        float* yr = Y + (int64_t)gm * ldy + gn;
        if (vec && gn + 3 < N) {
          *reinterpret_cast<float4*>(yr) = make_float4(tr[0], tr[1], tr[2], tr[3]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (gn + e < N) yr[e] = tr[e];
        }
      }
    }
    const int line = t >> 2, qtr = t & 3;
    // quarters of a row (column) of BN (BM) entries: 16 or 32 each
    const int lo_r = qtr * (BN / 4), lo_c = qtr * (BM / 4);
    // (all LEN staged entries loaded at once -- indices past `count` are still inside the staged
    // tile -- and kept in registers for the exp pass: the same max and the same left-to-right
    // sum over i < count as a loop to count, without a dependent LDS round trip per entry, which
    // made the partials ~60% of the epilogue: 15.8k of its 25.7k cycles, profiles/r03/phase/)
    auto partial = [&](const float* base, int stride, int count, int lo, auto len_c)
        __attribute__((always_inline)) {
      constexpr int LEN = decltype(len_c)::value;
      float v[LEN];
#pragma unroll
      for (int i = 0; i < LEN; ++i) v[i] = base[(lo + i) * stride];
      float mx = -INFINITY;
#pragma unroll
      for (int i = 0; i < LEN; ++i)
        if (lo + i < count) mx = fmaxf(mx, v[i]);
      mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < LEN; ++i)
        if (lo + i < count) s += expf(v[i] - mx);
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      return make_float2(mx, s);
    };
    if (line < BM) {   // row `line` over this tile's columns
      const float2 r = partial(tile + line * TP, 1, cols, lo_r, std::integral_constant<int, BN / 4>());
      if (qtr == 0 && line < rows) {
        float* o = F(rowstat) + (((int64_t)b * M + m0 + line) * ntiles + nt) * 2;
        o[0] = r.x;
        o[1] = r.y;
      }
    }
    if (line < BN) {   // column `line` over this tile's rows
      const float2 r = partial(tile + line, TP, rows, lo_c, std::integral_constant<int, BM / 4>());
      if (qtr == 0 && line < cols) {
        float* o = F(colstat) + (((int64_t)b * mtiles + mt) * N + n0 + line) * 2;
        o[0] = r.x;
        o[1] = r.y;
      }
    }
  }
#undef F
}

template <int EPI, int PRO, class T, int PM, bool WPL, int DMA>
__global__ __launch_bounds__(T::NT) __attribute__((amdgpu_waves_per_eu(T::WPE)))
void gemm_kernel(GemmArgs args) {
  __shared__ StampLds sl;
  StampTick tk{0ull, 0ull};
  gemm_body<EPI, PRO, T, PM, WPL, DMA>(args, tk, &sl);
  stamp_end(args.stamp, tk, &sl);
}

using T64x64 = Tile<64, 64, 1, 4, 32>;
using T32x128 = Tile<32, 128, 1, 4, 32>;
using T64x32K2 = Tile<64, 32, 2, 4, 64>;
using T64x128 = Tile<64, 128, 1, 4, 32>;
using T128x128 = Tile<128, 128, 1, 4, 32>;
using T128x64W8 = Tile<128, 64, 1, 8, 32>;
using T32x64W2 = Tile<32, 64, 1, 2, 32>;
using T32x256W8 = Tile<32, 256, 1, 8, 64, 1>;
using T128x128W8S = Tile<128, 128, 1, 8, 32, 2, 64, 64>;   // split MLP conv 1 for the 64 x 64 tile


template <int EPI, int PRO, class T, int PM, bool WPL = false, int DMA = 0>
void launch_one(GemmArgs& args, int grid, hipStream_t stream) {
  hipLaunchKernelGGL((gemm_kernel<EPI, PRO, T, PM, WPL, DMA>), dim3(grid), dim3(T::NT), 0, stream,
                     args);
}

// DMA 2 is instantiated only for the combinations that use it (gemm_launch checks the rest):
// the attention layers' QKV and MLP conv 1 in the bf16 modes
template <int EPI, int PRO, class T, int PM>
void launch_adma(GemmArgs& args, int grid, hipStream_t stream) {
  if constexpr (PRO != PRO_NORM_RELU && (EPI == EPI_QKV || EPI == EPI_STATS))
    launch_one<EPI, PRO, T, PM, true, 2>(args, grid, stream);
}

struct TileDims {
  int bm, bn, bks;
};
TileDims tile_dims(int tile) {
  switch (tile) {
    case TILE_64x64: return {64, 64, 32};
    case TILE_32x128: return {32, 128, 32};
    case TILE_64x32K2: return {64, 32, 64};
    case TILE_64x128: return {64, 128, 32};
    case TILE_128x128: return {128, 128, 32};
    case TILE_128x64W8: return {128, 64, 32};
    case TILE_32x64W2: return {32, 64, 32};
    case TILE_32x256W8: return {32, 256, 64};
    case TILE_128x128W8: return {128, 128, 32};

    default: return {0, 0, 0};
  }
}

}  // namespace

int gemm_tile_rows(int tile) { return tile_dims(tile).bm; }

static_assert(gemm_tile_bm(TILE_64x64) == 64 && gemm_tile_bn(TILE_64x64) == 64 &&
                  gemm_tile_bm(TILE_32x128) == 32 && gemm_tile_bn(TILE_32x128) == 128 &&
                  gemm_tile_bm(TILE_64x32K2) == 64 && gemm_tile_bn(TILE_64x32K2) == 32 &&
                  gemm_tile_bm(TILE_64x128) == 64 && gemm_tile_bn(TILE_64x128) == 128 &&
                  gemm_tile_bm(TILE_128x128) == 128 && gemm_tile_bn(TILE_128x128) == 128 &&
                  gemm_tile_bm(TILE_128x64W8) == 128 && gemm_tile_bn(TILE_128x64W8) == 64 &&
                  gemm_tile_bm(TILE_32x64W2) == 32 && gemm_tile_bn(TILE_32x64W2) == 64 &&
                  gemm_tile_bm(TILE_32x256W8) == 32 && gemm_tile_bn(TILE_32x256W8) == 256 &&
                  gemm_tile_bm(TILE_128x128W8) == 128 && gemm_tile_bn(TILE_128x128W8) == 128,
              "gemm.h tile shapes must match tile_dims");

GemmProb gemm_prob(const float* A, int lda, const float* W, int ldw, const float* bias,
                   float* Y, int ldy, int M, int N, int K, int batch) {
  GemmProb g;
  memset(&g, 0, sizeof(g));
  g.A0 = A;
  g.lda0 = lda;
  g.a0_bs = (int64_t)M * lda;
  g.ksplit = K;
  g.W = W;
  g.ldw = ldw;
  g.bias = bias;
  g.Y = Y;
  g.ldy = ldy;
  g.y_bs = (int64_t)M * ldy;
  g.M = M;
  g.N = N;
  g.K = K;
  g.batch = batch;
  g.scale = 1.f;
  g.vdiv = 1.f;
  g.ns = 1.f;
  return g;
}

int gemm_launch(int epi, int pro, int tile, GemmArgs& args, hipStream_t stream, int kind,
                int pm) {
  const TileDims td = tile_dims(tile);
  OP_REQUIRE(td.bm > 0, "gemm: unknown tile %d", tile);
  int grid = 0;
  for (int i = 0; i < 2; ++i) {
    GemmProb& P = args.p[i];
    if (i >= args.nprob) {
      P.tiles = 0;
      continue;
    }
    OP_REQUIRE(P.M > 0 && P.N > 0, "gemm: empty problem");
    OP_REQUIRE(P.K % (2 * td.bks) == 0, "gemm: K=%d not a multiple of %d", P.K, 2 * td.bks);
    OP_REQUIRE(P.ksplit % td.bks == 0, "gemm: ksplit=%d", P.ksplit);
    OP_REQUIRE(P.lda0 % 4 == 0 && P.ldw % 4 == 0, "gemm: unaligned leading dimension");
    OP_REQUIRE(epi != EPI_QKV || (td.bn == 128 && P.N == 768), "gemm: QKV tiling");
    const int srows = gemm_tile_stat_rows(tile);
    OP_REQUIRE(epi != EPI_STATS || P.st_cnt == nullptr ||
                   (P.st_grp != nullptr &&
                    P.st_cnt_bs >= ceil_div(P.N, td.bn) * (1 + stats_groups(P.M, srows))),
               "gemm: STATS finalize needs group partials and %d counters per sample",
               ceil_div(P.N, td.bn) * (1 + stats_groups(P.M, srows)));
    OP_REQUIRE(tile != TILE_128x128W8 || (epi == EPI_STATS && pro == PRO_HEADZ && pm == PM_SPLIT3 &&
                                          P.N == 512 && P.ksplit == 256) ||
                   (epi == EPI_QKV && pm == PM_F32),
               "gemm: the 128 x 128 eight-wave tile is the split mode's MLP conv 1 and fp32 QKV's");
    OP_REQUIRE(epi != EPI_BIAS_L2 || (td.bn == 256 && P.N == 256 && P.ldy % 4 == 0),
               "gemm: BIAS_L2 tiles hold whole 256-column rows");
    OP_REQUIRE((epi != EPI_BIAS && epi != EPI_STATS && epi != EPI_RESID) ||
                   (P.N % 4 == 0 && P.ldy % 4 == 0 && (epi != EPI_RESID || P.ldr % 4 == 0)),
               "gemm: row-stored epilogues need N, ldy (and ldr) multiples of 4");
    OP_REQUIRE(pro != PRO_HEADZ || (P.ksplit % 64 == 0 && P.K - P.ksplit == 256 &&
                                    (td.bks == 32 || td.bks == 64) && P.ksum != nullptr),
               "gemm: HEADZ needs 4 heads x 64 after ksplit");
    P.mtiles = ceil_div(P.M, td.bm);
    P.ntiles = ceil_div(P.N, td.bn);
    P.tiles = P.mtiles * P.ntiles * P.batch;
    grid += P.tiles;
  }
  if (grid == 0) return ONEPOSE_OK;
  // W from bf16 planes (every problem of the launch, or none)
  const bool wpl = args.p[0].Wp != nullptr;
  for (int i = 0; i < args.nprob; ++i) {
    const GemmProb& P = args.p[i];
    OP_REQUIRE((P.Wp != nullptr) == wpl, "gemm: W planes on some problems only");
    OP_REQUIRE(!wpl || (pm != PM_F32 && P.ldw % 4 == 0 &&
                        (P.W1 == nullptr) == (P.Wp1 == nullptr)),
               "gemm: W planes need a bf16 mode, 32-deep stages and planes for both K ranges");
  }
  args.stamp = nullptr;
  // split mode: W planes stream into LDS by global_load_lds (the lean DMA loop; the
  // register-staged split loop needs 160+ VGPRs and spills).  bf16 mode: the DMA loop for the
  // 64 x 128 tiles (QKV, MLP conv 1), the register-staged loop for 64 x 64 (MLP conv 2, whose
  // two MFMAs per wave and stage leave a DMA loop nothing to hide behind).
  const bool dma =
      pm == PM_SPLIT3 || (pm == PM_BF16 && tile == TILE_64x128);
  // A from activation planes (every problem of the launch, or none): the DMA loop's DMA-2 form
  const bool adma = args.p[0].Ap != nullptr;
  const bool yplanes = args.p[0].Yp != nullptr;
  for (int i = 0; i < args.nprob; ++i) {
    const GemmProb& P = args.p[i];
    OP_REQUIRE((P.Ap != nullptr) == adma && (P.Yp != nullptr) == yplanes,
               "gemm: activation planes on some problems only");
    OP_REQUIRE(!adma || ((P.A1 == nullptr) == (P.Ap1 == nullptr) && P.ldap % 8 == 0 &&
                         (P.Ap1 == nullptr || P.ldap1 % 8 == 0)),
               "gemm: A planes need planes for both K ranges and 16-B aligned rows");
  }
  OP_REQUIRE(!adma || (dma && wpl && pro != PRO_NORM_RELU && (epi == EPI_QKV || epi == EPI_STATS)),
             "gemm: A planes: QKV / MLP conv 1 on the DMA loop (bf16 modes, W planes)");
  OP_REQUIRE(!yplanes || (pm != PM_F32 && (epi == EPI_RESID || epi == EPI_QKV)),
             "gemm: output planes are written by RESID / QKV launches in the bf16 modes");
#define CASE(E, PR, TI, T, PMV, WP)                                      \
  if (epi == E && pro == PR && tile == TI && pm == PMV && wpl == WP) {  \
    prof_pre(kind, stream);                                              \
    args.stamp = prof_stamp_slot(kind);                                  \
    if constexpr (WP) {                                                  \
      if (adma) launch_adma<E, PR, T, PMV>(args, grid, stream);          \
      else if (dma) launch_one<E, PR, T, PMV, WP, 1>(args, grid, stream); \
      else launch_one<E, PR, T, PMV, WP, 0>(args, grid, stream);         \
    } else {                                                             \
      launch_one<E, PR, T, PMV, WP, 0>(args, grid, stream);              \
    }                                                                    \
    prof_post(kind, stream);                                             \
    OP_LAUNCHED();                                                       \
    return ONEPOSE_OK;                                                   \
  }
  CASE(EPI_QKV, PRO_PLAIN, TILE_32x128, T32x128, PM_F32, false)
  CASE(EPI_QKV, PRO_PLAIN, TILE_64x128, T64x128, PM_F32, false)
  CASE(EPI_QKV, PRO_PLAIN, TILE_128x128W8, T128x128W8S, PM_F32, false)
  CASE(EPI_QKV, PRO_PLAIN, TILE_128x128, T128x128, PM_F32, false)
  CASE(EPI_STATS, PRO_HEADZ, TILE_64x64, T64x64, PM_F32, false)
  CASE(EPI_RESID, PRO_NORM_RELU, TILE_64x64, T64x64, PM_F32, false)
  CASE(EPI_RESID, PRO_NORM_RELU, TILE_64x32K2, T64x32K2, PM_F32, false)
  CASE(EPI_SCORE, PRO_PLAIN, TILE_64x64, T64x64, PM_F32, false)
  CASE(EPI_SCORE, PRO_PLAIN, TILE_128x64W8, T128x64W8, PM_F32, false)
  CASE(EPI_BIAS, PRO_PLAIN, TILE_64x64, T64x64, PM_F32, false)
  CASE(EPI_BIAS_L2, PRO_PLAIN, TILE_32x256W8, T32x256W8, PM_F32, false)
  CASE(EPI_ACC, PRO_PLAIN, TILE_64x64, T64x64, PM_F32, false)
  // attention-layer GEMMs in the bf16 modes: W from the packed bf16 planes (weights rounded /
  // split on the host, Mf by the KV fold), A rounded / split as the stage is stored
  CASE(EPI_ACC, PRO_PLAIN, TILE_64x64, T64x64, PM_BF16, true)
  CASE(EPI_ACC, PRO_PLAIN, TILE_64x64, T64x64, PM_SPLIT3, true)
  CASE(EPI_QKV, PRO_PLAIN, TILE_32x128, T32x128, PM_BF16, true)
  CASE(EPI_STATS, PRO_HEADZ, TILE_64x64, T64x64, PM_BF16, true)
  CASE(EPI_RESID, PRO_NORM_RELU, TILE_64x64, T64x64, PM_BF16, true)
  CASE(EPI_QKV, PRO_PLAIN, TILE_64x128, T64x128, PM_BF16, true)
  CASE(EPI_STATS, PRO_HEADZ, TILE_64x128, T64x128, PM_BF16, true)
  CASE(EPI_RESID, PRO_NORM_RELU, TILE_64x128, T64x128, PM_BF16, true)
  CASE(EPI_ACC, PRO_PLAIN, TILE_64x128, T64x128, PM_BF16, true)
  CASE(EPI_RESID, PRO_NORM_RELU, TILE_32x64W2, T32x64W2, PM_SPLIT3, true)
  CASE(EPI_QKV, PRO_PLAIN, TILE_32x128, T32x128, PM_SPLIT3, true)
  CASE(EPI_STATS, PRO_HEADZ, TILE_64x64, T64x64, PM_SPLIT3, true)
  CASE(EPI_STATS, PRO_HEADZ, TILE_128x128W8, T128x128W8S, PM_SPLIT3, true)
  CASE(EPI_QKV, PRO_PLAIN, TILE_64x128, T64x128, PM_SPLIT3, true)
  CASE(EPI_RESID, PRO_NORM_RELU, TILE_64x64, T64x64, PM_SPLIT3, true)
  // final projection and score GEMM in the split mode (activations as W: VALU split)
  CASE(EPI_SCORE, PRO_PLAIN, TILE_64x64, T64x64, PM_SPLIT3, false)
  CASE(EPI_BIAS, PRO_PLAIN, TILE_64x64, T64x64, PM_SPLIT3, false)
#undef CASE
  set_error("gemm: unsupported epilogue/prologue/tile/mode/planes %d/%d/%d/%d/%d", epi, pro, tile,
            pm, (int)wpl);
  return ONEPOSE_ERR_INVALID;
}

}  // namespace onepose
