// Grouped token-GEMM on gfx950 f32-input MFMA (v_mfma_f32_32x32x2_f32: exact f32 products,
// f32 accumulation, 157 TF/s dense peak).
//
//   Y[b][m][o] = epilogue( sum_k prologue(A)[b][m][k] * W[o][k] + bias[o] )
//
// Activations are token-major ([tokens][channels], a token's channels contiguous), so a
// 1x1 Conv1d of the reference (x [C,N] -> W x + b) is this GEMM with the reference weight
// [O][C] used as is.  A and W may each be split along K at `ksplit` into two sources (the
// MLP's cat[x, message] input and its folded weights).  One launch runs up to two problems
// (the 2D-query side and the 3D side of a layer) and every batch sample of each; tiles never
// straddle samples, so per-sample reductions stay per sample.
#pragma once

#include "common.h"

namespace onepose {

enum GemmEpi {
  EPI_BIAS = 0,    // y = acc + bias
  EPI_QKV = 1,     // 128-col tiles of [q (256) | k_0 v_0 | .. | k_3 v_3] (768 outputs):
                   //   q tiles store phi(q) = elu(q)+1; [k_h | v_h] tiles reduce phi(k), v/vdiv
                   //   to the tile's KV_h = phi(k)^T v and sum phi(k) partials (no store)
  EPI_STATS = 2,   // y = acc + bias, plus per-tile (mean, M2) of every column  (InstanceNorm)
  EPI_RESID = 3,   // y = R + (acc + bias)                                     (desc += delta)
  EPI_SCORE = 4,   // y = acc / scale, plus per-tile row/col (max, sum exp)     (dual softmax)
  EPI_ACC = 5,     // the raw accumulators in register order, Y[b][tile][wave][FN][16][64]
                   //   (tile = mt * ntiles + nt): a PRO_HEADZ launch's acc0
  EPI_BIAS_L2 = 6, // y = (acc + bias) / max(|row|_2, 1e-12): the final projection with
                   //   F.normalize fused (tiles hold whole 256-column rows)
};
enum GemmPro {
  PRO_PLAIN = 0,
  PRO_NORM_RELU = 1,  // a = max((a - mean[k]) * rstd[k], 0)                    (norm + ReLU)
  PRO_HEADZ = 2,      // K range [ksplit, K) = 4 heads x 64 of phi(q): each head's partial
                      //   sum is scaled per row by Z*Ns = ns / (phi(q)_h . ksum_h + 1e-6)
                      //   (linear attention's normaliser, computed from the staged tiles)
};

struct GemmProb {
  const float* A0;     // [batch][M][lda0]; columns [0, ksplit)
  const float* A1;     // [batch][M][lda1]; columns [ksplit, K) (concat), may be null
  int64_t a0_bs, a1_bs;
  int lda0, lda1, ksplit;
  const float* W;      // [N][ldw] (out-major) for k < ksplit; w_bs per sample (0 = shared)
  int64_t w_bs;
  int ldw;
  const float* W1;     // [N][ldw1] for k >= ksplit (null: W continues)
  int64_t w1_bs;
  int ldw1;
  // bf16 modes: W (and W1) as bf16 planes instead -- one (PM_BF16: round to nearest even) or
  // three (PM_SPLIT3: the exact split hi, mid, lo), each [N][ldw] (resp. [N][ldw1]), `wpl`
  // elements apart, wp_bs per sample; copied to LDS as is (no conversion).  Set on every
  // problem of a launch or on none; Wp1 set exactly when W1 is.
  const uint16_t* Wp;
  int64_t wp_bs, wpl;
  const uint16_t* Wp1;
  int64_t wp1_bs, wpl1;
  // bf16 modes: A (and A1) as activation planes (common.h store_planes4: the producer's exact
  // split, NPL planes [M][ldap] per sample, apl elements apart, ap_bs per sample (0 = shared)),
  // moved to LDS by global_load_lds like Wp -- the DMA loop then stages nothing through
  // registers.  Set on every problem of a launch or on none; Ap1 set exactly when A1 is; not
  // with PRO_NORM_RELU (its A is transformed per stage).  The LDS images, and so every result
  // bit, equal the register-staged rounding / split of A.
  const uint16_t* Ap;
  int64_t ap_bs, apl;
  int ldap;
  const uint16_t* Ap1;
  int64_t ap1_bs, apl1;
  int ldap1;
  const float* bias;   // [N] or null
  float* Y;            // [batch][M][ldy]
  int64_t y_bs;
  int ldy;
  // bf16 modes: the stored output's activation planes as well (EPI_RESID: y; EPI_QKV: the
  // phi(q) tiles), NPL planes [M][ldy] per sample (yp_bs), ypl apart; null = fp32 only.
  uint16_t* Yp;
  int64_t yp_bs, ypl;
  const float* R;      // residual, [batch][M][ldr]
  int64_t r_bs;
  int ldr;
  const float* pro_mean;   // [batch][K] (PRO_NORM_RELU)
  const float* pro_rstd;
  int64_t pro_bs;
  float* stats;        // EPI_STATS: [batch][mtiles][2][N]  (mtiles = ceil(M / tile rows))
  unsigned* st_cnt;    // EPI_STATS: arrival counters, zero before the launch, st_cnt_bs per
                       //   sample: [ntiles] column-block counters, then [ntiles][ngroups] group
                       //   counters; null = partials only.  Two levels (gemm.hip): the last
                       //   M-tile of each group (stats_group_size) merges the group into
                       //   st_grp, the last group merger the groups into st_mean / st_rstd
  int st_cnt_bs;
  double* st_grp;      // EPI_STATS with st_cnt: [batch][ngroups][2][N] group (mean, M2)
  float* st_mean;
  float* st_rstd;
  float* rowstat;      // EPI_SCORE: [batch][M][ntiles][2]
  float* colstat;      // EPI_SCORE: [batch][mtiles][N][2] (tile-major: a tile's columns
                       //   contiguous, so a reader's lanes over columns load 8 B each, coalesced)
  float* kvpart;       // EPI_QKV: [batch][mtiles][4][64][64]
  float* kspart;       // EPI_QKV: [batch][mtiles][256]
  const float* ksum;   // PRO_HEADZ: [batch][256] sum phi(k) of the attention source
  int64_t ksum_bs;
  const float* acc0;   // PRO_HEADZ: the accumulators after the K range [0, ksplit), as an
  int64_t acc0_bs;     //   EPI_ACC launch of the same tile over that range stored them (the same
                       //   MFMA sequence, so the same bits); that range is then skipped.  Null:
                       //   start from zero.
  float scale;         // EPI_SCORE divisor (scale_factor)
  float vdiv;          // EPI_QKV: v divisor (source length)
  float ns;            // PRO_HEADZ: source length (v_length)
  int M, N, K, batch;
  int mtiles, ntiles, tiles;   // filled by gemm_launch
};

struct GemmArgs {
  GemmProb p[2];
  int nprob;
  StampAcc* stamp;   // device-stamp profiling accumulator (set by gemm_launch) or null
};

// Operand modes (gemm.hip): exact fp32 MFMA, bf16 (rounded), fp32 by exact 3-way bf16 split.
enum GemmPm { PM_F32 = 0, PM_BF16 = 1, PM_SPLIT3 = 2 };

// Tile configurations: BM x BN output tile, K split into KS slices inside the workgroup.
enum GemmTile {
  TILE_64x64 = 0,   // mlp1 (STATS + HEADZ), mlp2 (RESID + NORM), score, final
  TILE_32x128 = 1,  // qkv (QKV: one head's [k_h | v_h] or two q heads per tile)
  TILE_64x32K2 = 2, // mlp2 fp32 (RESID + NORM): 64 x 32 outputs, K split over two wave pairs
                    //   (N = 256 gives 2x the 64x64 tile count: 640 tiles at config 2)
  TILE_64x128 = 3,  // qkv fp32 at large batches: 2 accumulators per wave, 64-row KV chunks
  TILE_128x128 = 4, // qkv fp32 at larger batches: 4 accumulators per wave, 128-row KV chunks
  TILE_32x64W2 = 6,  // mlp2 in the split mode: 32 x 64 outputs on 2 waves (N = 256: 640 tiles
                     //   at config 2, where 64 x 64 gives 320 for 256 CUs)
  TILE_128x64W8 = 5, // score: 128 x 64 outputs on 8 waves of 32 x 32 (K = 256 is short: half
                     //   the operand loads per FLOP of 64 x 64)
  TILE_32x256W8 = 8, // final projection + L2 normalisation (EPI_BIAS_L2): whole rows on 8 waves
                     //   of 32 x 32 (two per SIMD), 64-deep stages
  // (9: a 256 x 128 eight-wave bf16 MLP conv 1 tile, measured slower; removed, tag r05-lab)
  TILE_128x128W8 = 10, // split-mode MLP conv 1 (STATS + HEADZ, DMA 2): 128 x 128 on 8 waves of
                       //   32 x 64, standing in for 64 x 64 tiles the same way (acc0 included)
};
// Output tile shape of each configuration, usable in constant expressions (the workspace
// plan sizes per-tile partials and counters from these; tile_dims in gemm.hip agrees).
constexpr int gemm_tile_bm(int t) {
  return (t == TILE_32x128 || t == TILE_32x64W2 || t == TILE_32x256W8) ? 32
         : (t == TILE_128x128 || t == TILE_128x64W8) ? 128
         : t == TILE_128x128W8                       ? 128
                                                     : 64;
}
// rows per EPI_STATS partial (and per acc0 tile): the tile's, or its stand-in tile's
constexpr int gemm_tile_stat_rows(int t) {
  return t == TILE_128x128W8 ? 64 : gemm_tile_bm(t);
}
constexpr int gemm_tile_bn(int t) {
  return (t == TILE_32x128 || t == TILE_64x128 || t == TILE_128x128 || t == TILE_128x128W8)
             ? 128
         : t == TILE_64x32K2                                        ? 32
         : t == TILE_32x256W8                                       ? 256
                                                                    : 64;
}
// (STATS + HEADZ also compile for 64x32 / 2 waves and for 64x64 / 8 waves with K split in
// two and 64-deep stages, one head per stage; both measured slower than 64x64 for mlp1 in the
// two-stream frame: DESIGN.md section 3.)

// Supported (epilogue, prologue, tile) combinations: QKV/32x128, STATS+HEADZ/64x64,
// RESID+NORM/64x64 and /64x32K2 (fp32), SCORE/64x64, BIAS/64x64.  K must be a multiple of twice the tile's stage
// depth (32 * KS).
// pm = PM_BF16: operands rounded to bf16 as the stage is stored, v_mfma_f32_32x32x16_bf16 with
// fp32 accumulation (QKV, STATS+HEADZ, RESID+NORM 64x64 only: the attention-layer GEMMs).
// pm = PM_SPLIT3: every operand split exactly into three bf16 pieces, six bf16 MFMAs per
// 16-deep group (fp32-accurate; all 64x64 and 32x128 combinations).
int gemm_launch(int epi, int pro, int tile, GemmArgs& args, hipStream_t stream, int kind,
                int pm = PM_F32);
// Rows per M-tile of a configuration (the chunk size of the STATS / KVPART partials).
int gemm_tile_rows(int tile);

// InstanceNorm finalize: M-tiles per first-level group (at least kStatsGroup, and at most
// kStatsMaxGroups groups: batched launches with many tiles per CU keep few mergers), and the
// groups a STATS launch over M rows with `rows`-row tiles has per sample and column block.
constexpr int kStatsGroup = 8, kStatsMaxGroups = 8;
__host__ __device__ inline int stats_group_size(int mtiles) {
  const int g = (mtiles + kStatsMaxGroups - 1) / kStatsMaxGroups;
  return g > kStatsGroup ? g : kStatsGroup;
}
inline int stats_groups(int M, int rows) {
  const int mtiles = (M + rows - 1) / rows, g = stats_group_size(mtiles);
  return (mtiles + g - 1) / g;
}

// PRO_HEADZ arithmetic, shared by every MLP conv 1 kernel variant (tools/experiments/gemm_bal.hip
// at tag r05-lab too) for the same reason as the merges below: one stage's 8-term piece of phi(q)_row . ksum_h (products rounded, summed left to
// right) added to the running dot, and the head fold acc + Z*Ns * acc_h as one fma.
__device__ __forceinline__ float headz_dot8(float zp, float4 a0, float4 a1, float4 k0, float4 k1) {
#pragma clang fp contract(off)
  return zp + (a0.x * k0.x + a0.y * k0.y + a0.z * k0.z + a0.w * k0.w + a1.x * k1.x +
               a1.y * k1.y + a1.z * k1.z + a1.w * k1.w);
}
__device__ __forceinline__ float headz_fold(float acc, float z, float acc_h) {
  return fmaf(z, acc_h, acc);
}

// InstanceNorm merges of MLP conv 1's in-launch finalize, shared by gemm.hip's tiles (and the
// experimental kernels at tag r05-lab) so that all round every operation alike: each statement exactly as written
// (contraction off -- left to itself the compiler fused some of these in one kernel and not in
// the other), with fma() where the merge takes one.
// (count, mean, M2) of a 32-row block into the running column statistics (Chan et al.)
__device__ __forceinline__ void in_merge_block(float& n, float& mean, float& M2, float nb, float mb,
                                               float m2b) {
#pragma clang fp contract(off)
  const float nn = n + nb, delta = mb - mean;
  mean += delta * (nb / nn);
  M2 += m2b + delta * delta * (n * nb / nn);
  n = nn;
}
// one M-tile's (mean mv, M2 qv) of nb rows into a group's shifted sums (shift c)
__device__ __forceinline__ void in_merge_tile(double& s1, double& s2, double& ng, double nb, float mv,
                                              float qv, double c) {
#pragma clang fp contract(off)
  const double d = (double)mv - c;
  s1 = fma(nb, d, s1);
  s2 = s2 + fma(nb * d, d, (double)qv);
  ng = ng + nb;
}
// one group's (mean mg, M2 m2g) of ngr rows into the column's shifted sums (shift c)
__device__ __forceinline__ void in_merge_group(double& S1, double& S2, double ngr, double mg,
                                               double m2g, double c) {
#pragma clang fp contract(off)
  const double d = mg - c;
  S1 = fma(ngr, d, S1);
  S2 = S2 + fma(ngr * d, d, m2g);
}
__device__ __forceinline__ double in_group_mean(double c, double s1, double ng) {
#pragma clang fp contract(off)
  return c + s1 / ng;
}
__device__ __forceinline__ double in_group_m2(double s1, double s2, double ng) {
#pragma clang fp contract(off)
  return s2 - s1 * s1 / ng;
}
__device__ __forceinline__ float in_final_mean(double c, double S1, double n) {
#pragma clang fp contract(off)
  return (float)(c + S1 / n);
}
__device__ __forceinline__ float in_final_rstd(double S1, double S2, double n) {
#pragma clang fp contract(off)
  return (float)(1.0 / sqrt((S2 - S1 * S1 / n) / n + 1e-5));
}

// Zero-initialised problem with the common fields set.
GemmProb gemm_prob(const float* A, int lda, const float* W, int ldw, const float* bias,
                   float* Y, int ldy, int M, int N, int K, int batch);

}  // namespace onepose
