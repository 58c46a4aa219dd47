// Tile-balanced fp32 MLP conv 1 (gemm.h: EPI_STATS + PRO_HEADZ, N = K = 512, ksplit 256) for
// launches with few 64 x 64 tiles per CU -- the B = 1 frame of config 2.
//
// Why: the 64 x 64 kernel's 640 tiles at config 2 put 3 workgroups on half the
// CUs and 2 on the rest, and its loop is bound by the matrix pipe of the SIMDs with 3 waves, so
// the launch takes the 3-tile time (plus every tile's prologue / epilogue, all at once).  Here
// the work is dealt in 64-row x 32-column *strips* (1280 at config 2), a contiguous run of
// strips per workgroup with equal MFMA work per workgroup (a strip whose x range is cached,
// acc0, counts half), one 8-wave workgroup per CU, and every strip spread over all four SIMDs:
// wave w owns rows 16 (w % 4) .. + 16 and the 16-column half w / 4 of every strip of its
// workgroup (waves w and w + 4 share a SIMD), on v_mfma_f32_16x16x4_f32.  So every SIMD of
// every CU carries the same MFMA work, and a workgroup's operands are shared by all its strips
// (one A stage per 64-row M-tile, one W stage per strip).
//
// Bits: every output is the same fmaf chain as gemm.hip's 64 x 64 tile (the 16x16x4 MFMA pair
// of an 8-deep k group takes k in the order 0, 4, 1, 5 | 2, 6, 3, 7, the 32x32x2 sequence's
// order: tools/mfma_order.hip), the Z * Ns head fold, the bias, the InstanceNorm (mean, M2)
// partials of the 32-row wave blocks and their Chan merge per 64-row M-tile and the two-level
// in-launch finalize are restated operation for operation, so the launch writes the bits the
// 64 x 64 kernel writes (tools/bitcmp.py).  The finalize counters are per 32-column block
// (kBalNS of them per sample, gemm.h st_cnt).
#include "gemm.h"

#include <algorithm>
#include <cstring>

namespace onepose {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));
#define ONEPOSE_BAL_SCHED_BARRIER() __builtin_amdgcn_sched_barrier(0)

constexpr int kBalS = 5;          // strips per workgroup, at most (host-checked)
constexpr int kBalNT = 512;       // 8 waves, two per SIMD
constexpr int kBalRG = 2;         // 64-row M-tiles (row groups) per workgroup, at most
constexpr int kBalRowF = 32;      // floats per LDS row: one 32-deep stage, no padding
// (W rows for an even number of strips: the last W slot of an odd strip count writes a copy of
// its last strip into the next strip's rows)
constexpr int kBalARows = kBalRG * 64, kBalRows = kBalARows + (kBalS + 1) / 2 * 2 * 32;
constexpr int kBalStage = kBalRows * kBalRowF;   // 10240 floats = 40 KB per stage buffer
constexpr int kBalTP = 36;        // epilogue tile pitch: 32 columns + 4
constexpr int kBalNS = 16;        // 32-column strips of N = 512
constexpr int kBalK = 512, kBalKs = 256, kBalStages = kBalK / 32, kBalXs = kBalKs / 32;
static_assert(kBalS * 64 * kBalTP <= 2 * kBalStage, "epilogue tile fits the stage buffers");
static_assert(kBalS <= 8, "one wave per strip in the finalize");

// Position of k (0..31 of a stage) in an LDS row: in 8-deep group kk, MFMA a gives lane group g
// k = 8 kk + {0, 4, 1, 5}[g] and MFMA b k = 8 kk + {2, 6, 3, 7}[g], so lane group g's values for
// the stage are 8 consecutive floats at 8 g: [kk0 a, kk0 b, kk1 a, kk1 b | kk2 a, ..., kk3 b].
// The 16-B chunk c of row r lives at chunk c ^ bal_sw(r): conflict-free ds_read_b128 for the
// fragment pattern (16 rows x one chunk per lane group).
__device__ __forceinline__ int bal_sw(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 2); }
__device__ __forceinline__ int bal_off(int r, int pos) {
  return r * kBalRowF + ((((pos >> 2) ^ bal_sw(r)) & 7) << 2) + (pos & 3);
}

// the first strip whose cost starts at or after T (strips of problem 0 cost c0, then problem 1's
// cost c1; cost = MFMA stages: 2 for a full K range, 1 when the x range comes from acc0)
__host__ __device__ inline int bal_first_strip(int64_t T, int64_t S0, int c0, int c1) {
  if (T <= S0 * c0) return (int)((T + c0 - 1) / c0);
  return (int)(S0 + (T - S0 * c0 + c1 - 1) / c1);
}

struct BalShared {
  float zrow[2][kBalRG][64];                        // Z * Ns per row, by head parity
  __attribute__((aligned(16))) float zks[kBalRG][256];   // sum phi(k) of each row group's source
};

// The workgroup's NS strips (NS = its strip count, a template parameter so that every strip
// loop is unrolled and branch-free); MIX: some strips' x range comes from acc0 (cross-attention
// 1 of a cached forward), so the x-range MFMAs skip those strips.
template <int NS, bool MIX>
__device__ __forceinline__ void bal_body(const GemmArgs& args, int64_t i0, int64_t S0, float* lds,
                                         BalShared& sh, StampLds* sl) {
#define PF(q, x) ((q) ? args.p[1].x : args.p[0].x)
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  // ---- the strips (wave-uniform) and their row groups (one or two 64-row M-tiles) ----
  int s_rg[NS], s_cs[NS], s_k0[NS], s_q[NS], s_b[NS], s_mt[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int i = (int)i0 + s;   // (strip counts are far below 2^31: host-checked grid)
    const int q = i >= (int)S0 ? 1 : 0;
    const int j = i - (q ? (int)S0 : 0);
    const int per = PF(q, mtiles) * kBalNS;
    const int b = j / per, r = j - b * per;
    s_q[s] = q;
    s_b[s] = b;
    s_mt[s] = r / kBalNS;
    s_cs[s] = r - s_mt[s] * kBalNS;
    s_k0[s] = MIX && PF(q, acc0) != nullptr ? kBalXs : 0;
    s_rg[s] = (q == s_q[0] && b == s_b[0] && s_mt[s] == s_mt[0]) ? 0 : 1;
  }
  // row group 1: the last strip's M-tile if it differs from the first's, else row group 0 again
  // (its loads then repeat row group 0's rows and nothing reads them)
  const int rq[kBalRG] = {s_q[0], s_q[NS - 1]}, rb[kBalRG] = {s_b[0], s_b[NS - 1]};
  const int rmt[kBalRG] = {s_mt[0], s_mt[NS - 1]};
  const bool two = s_rg[NS - 1] != 0;
  int kt0 = kBalXs;
#pragma unroll
  for (int s = 0; s < NS; ++s) kt0 = min(kt0, s_k0[s]);
  const float* rg_a0[kBalRG];
  const float* rg_a1[kBalRG];
  int rg_M[kBalRG], rg_m0[kBalRG];
#pragma unroll
  for (int rg = 0; rg < kBalRG; ++rg) {
    const int q = rq[rg], b = rb[rg];
    rg_a0[rg] = PF(q, A0) + b * PF(q, a0_bs);
    rg_a1[rg] = PF(q, A1) + b * PF(q, a1_bs);
    rg_M[rg] = PF(q, M);
    rg_m0[rg] = rmt[rg] * 64;
    const float* ks = PF(q, ksum) + b * PF(q, ksum_bs);
    if (t < 256) sh.zks[rg][t] = ks[t];
  }

  // ---- this thread's global-load slots (branch-free: every slot loads every stage) ----
  const int lrow = t >> 3, lq = t & 7;             // A: row 0..63 of each row group, k quad
  const int wrow = (t & 255) >> 3, whi = t >> 8;   // W slot i: strip 2 i + whi, its row 0..31
  const float* a_p0[kBalRG];
  const float* a_p1[kBalRG];
#pragma unroll
  for (int rg = 0; rg < kBalRG; ++rg) {
    const int m = min(rg_m0[rg] + lrow, rg_M[rg] - 1);
    a_p0[rg] = rg_a0[rg] + (int64_t)m * PF(rq[rg], lda0) + lq * 4;
    a_p1[rg] = rg_a1[rg] + (int64_t)m * PF(rq[rg], lda1) + lq * 4;
  }
  constexpr int SL = (NS + 1) / 2;   // W slots
  const float* w_p0[SL];
  const float* w_p1[SL];
#pragma unroll
  for (int i = 0; i < SL; ++i) {
    // the slot's strip (an odd NS's last slot repeats strip NS - 1 in its upper half)
    const int sa = 2 * i, sb = min(2 * i + 1, NS - 1);
    const int q = whi ? s_q[sb] : s_q[sa], b = whi ? s_b[sb] : s_b[sa];
    const int cs = whi ? s_cs[sb] : s_cs[sa];
    const int o = cs * 32 + wrow;
    const float* w0 = PF(q, W) + b * PF(q, w_bs);
    const bool w1own = PF(q, W1) != nullptr;
    const float* w1 = w1own ? PF(q, W1) + b * PF(q, w1_bs) : w0 + PF(q, ksplit);
    w_p0[i] = w0 + (int64_t)o * PF(q, ldw) + lq * 4;
    w_p1[i] = w1 + (int64_t)o * (w1own ? PF(q, ldw1) : PF(q, ldw)) + lq * 4;
  }
  // LDS positions of a stage quad's two float2 halves (bal_off): (x, z) and (y, w)
  const int pos_xz = 8 * (lq & 1) + 2 * (lq >> 1), pos_yw = 16 + pos_xz;
  // (row offsets that are multiples of 16 leave bal_sw unchanged: the slots' LDS offsets are the
  // first slot's plus compile-time row offsets)
  const int st_a0 = bal_off(lrow, pos_xz), st_a1 = bal_off(lrow, pos_yw);
  const int st_w0 = bal_off(kBalARows + whi * 32 + wrow, pos_xz);
  const int st_w1 = bal_off(kBalARows + whi * 32 + wrow, pos_yw);

  // ---- fragments: wave w, rows 16 (w % 4) + lane % 16 of each strip's row group, columns
  // 16 (w / 4) + lane % 16 of each strip; lane group lane / 16 reads its chunk pair ----
  const int rbase = 16 * (wave & 3), cbh = wave >> 2, lg = lane >> 4, r16 = lane & 15;
  const int fa0 = bal_off(rbase + r16, 8 * lg), fa1 = bal_off(rbase + r16, 8 * lg + 4);
  const int fw0 = bal_off(kBalARows + 16 * cbh + r16, 8 * lg);
  const int fw1 = bal_off(kBalARows + 16 * cbh + r16, 8 * lg + 4);

  floatx4 acc[NS], acc_h[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      acc[s][v] = 0.f;
      acc_h[s][v] = 0.f;
    }
  // strips whose x range is cached start from the 64 x 64 kernel's EPI_ACC accumulators (the
  // same MFMA chain): element (R, Cc) of 64 x 64 tile (mt, nt) is at ((mt ntiles + nt) 4 +
  // wave') 1024 + i' 64 + lane' with wave' = (R / 32) 2 + Cc / 32, r = R % 32,
  // i' = (r & 3) + 4 (r >> 3), lane' = 32 ((r >> 2) & 1) + Cc % 32
  if constexpr (MIX) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (s_k0[s] > 0) {
        const int q = s_q[s];
        const float* a0p = PF(q, acc0) + s_b[s] * PF(q, acc0_bs);
        const int nt = s_cs[s] >> 1, Cc = (s_cs[s] & 1) * 32 + 16 * cbh + r16;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int R = rbase + 4 * lg + v, r = R & 31;
          const int wv = (R >> 5) * 2 + (Cc >> 5);
          const int ip = (r & 3) + 4 * (r >> 3), lp = 32 * ((r >> 2) & 1) + (Cc & 31);
          acc[s][v] = a0p[((int64_t)(s_mt[s] * 8 + nt) * 4 + wv) * 1024 + ip * 64 + lp];
        }
      }
    }
  }

  // ---- stage registers: two sets, two stages of loads in flight ----
  struct Regs {
    float4 a[kBalRG];
    float4 w[SL];
  };
  Regs r0, r1;
  auto load = [&](int kt, Regs& R) __attribute__((always_inline)) {
    const bool hd = kt >= kBalXs;
    const int k0 = (hd ? kt - kBalXs : kt) * 32;
#pragma unroll
    for (int rg = 0; rg < kBalRG; ++rg)
      R.a[rg] = *reinterpret_cast<const float4*>((hd ? a_p1[rg] : a_p0[rg]) + k0);
#pragma unroll
    for (int i = 0; i < SL; ++i)
      R.w[i] = *reinterpret_cast<const float4*>((hd ? w_p1[i] : w_p0[i]) + k0);
  };
  auto store = [&](float* buf, const Regs& R) __attribute__((always_inline)) {
#pragma unroll
    for (int rg = 0; rg < kBalRG; ++rg) {
      float* b0 = buf + rg * 64 * kBalRowF;
      b0[st_a0] = R.a[rg].x;
      b0[st_a0 + 1] = R.a[rg].z;
      b0[st_a1] = R.a[rg].y;
      b0[st_a1 + 1] = R.a[rg].w;
    }
#pragma unroll
    for (int i = 0; i < SL; ++i) {
      float* b0 = buf + i * 64 * kBalRowF;
      b0[st_w0] = R.w[i].x;
      b0[st_w0 + 1] = R.w[i].z;
      b0[st_w1] = R.w[i].y;
      b0[st_w1 + 1] = R.w[i].w;
    }
  };

  // ---- PRO_HEADZ: Z of every row of each head from the staged phi(q) (gemm.hip's zdot: four
  // threads per row, thread zq summing k = 8 zq .. 8 zq + 7 of each stage, the same expression)
  const int zrg = t >> 8, zr = (t & 255) >> 2, zq = t & 3;
  float zp = 0.f;
  const float zns = PF(zrg ? rq[1] : rq[0], ns);
  auto zdot = [&](const float* buf, int kt) __attribute__((always_inline)) {
    const int r = zrg * 64 + zr;
    const float2 p0 = *reinterpret_cast<const float2*>(buf + bal_off(r, 2 * zq));        // k 0, 2
    const float2 p1 = *reinterpret_cast<const float2*>(buf + bal_off(r, 16 + 2 * zq));   // k 1, 3
    const float2 p2 = *reinterpret_cast<const float2*>(buf + bal_off(r, 8 + 2 * zq));    // k 4, 6
    const float2 p3 = *reinterpret_cast<const float2*>(buf + bal_off(r, 24 + 2 * zq));   // k 5, 7
    const float4 a0 = make_float4(p0.x, p1.x, p0.y, p1.y);
    const float4 a1 = make_float4(p2.x, p3.x, p2.y, p3.y);
    const float* kp = &sh.zks[zrg][(kt - kBalXs) * 32 + zq * 8];
    const float4 k0 = *reinterpret_cast<const float4*>(kp);
    const float4 k1 = *reinterpret_cast<const float4*>(kp + 4);
    zp = headz_dot8(zp, a0, a1, k0, k1);
  };
  auto zfinal = [&](int par) __attribute__((always_inline)) {
#pragma unroll
    for (int o = 1; o < 4; o <<= 1) zp += __shfl_xor(zp, o, 64);
    if (zq == 0 && (zrg == 0 || two)) sh.zrow[par][zrg][zr] = (1.0f / (zp + 1e-6f)) * zns;
    zp = 0.f;
  };
  auto fold = [&](int par) __attribute__((always_inline)) {   // acc += Z*Ns (per row) * acc_h
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        acc[s][v] = headz_fold(acc[s][v], sh.zrow[par][s_rg[s]][rbase + 4 * lg + v], acc_h[s][v]);
        acc_h[s][v] = 0.f;
      }
  };
  // fragments of one half stage (k groups 2h, 2h + 1) of every strip, and its MFMAs: part 0 the
  // first k group (.x, .y: MFMA pair a, b), part 1 the second (.z, .w); x range: the strips
  // not from acc0.  Per accumulator the k order is the 32x32x2 chain's.
  // (A fragments once per row group -- a strip takes its row group's by a select -- W per strip)
  struct Frag {
    float4 a[kBalRG], w[NS];
  };
  auto read_half = [&](const float* buf, int h, Frag& F) __attribute__((always_inline)) {
#pragma unroll
    for (int rg = 0; rg < kBalRG; ++rg)
      F.a[rg] = *reinterpret_cast<const float4*>(buf + rg * 64 * kBalRowF + (h ? fa1 : fa0));
#pragma unroll
    for (int s = 0; s < NS; ++s)
      F.w[s] = *reinterpret_cast<const float4*>(buf + s * 32 * kBalRowF + (h ? fw1 : fw0));
  };
  auto mfma_part = [&](const Frag& F, floatx4 (&tg)[NS], bool xr, int part)
      __attribute__((always_inline)) {
#ifdef BAL_PROBE_NOMFMA
    return;
#endif
    // (the pair's two MFMAs of a strip are dependent: issue the first of every strip, then the
    // second, so consecutive MFMAs are independent)
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if (!MIX || !xr || s_k0[s] == 0) {
        const float4 a = s_rg[s] ? F.a[1] : F.a[0];
        tg[s] = __builtin_amdgcn_mfma_f32_16x16x4f32(part ? a.z : a.x, part ? F.w[s].z : F.w[s].x,
                                                      tg[s], 0, 0, 0);
      }
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if (!MIX || !xr || s_k0[s] == 0) {
        const float4 a = s_rg[s] ? F.a[1] : F.a[0];
        tg[s] = __builtin_amdgcn_mfma_f32_16x16x4f32(part ? a.w : a.y, part ? F.w[s].w : F.w[s].y,
                                                      tg[s], 0, 0, 0);
      }
  };

  // ---- main loop, software-pipelined across the stage barrier: stage kt is in LDS buffer
  // kt & 1 and its first half's fragments in F0 when step kt starts; then
  //   global loads of stage kt + 2 | read half 1 -> F1 | MFMAs of F0 | store stage kt + 1 to
  //   the other buffer | MFMAs of F1's first group | barrier | read stage kt + 1's half 0 -> F0
  //   | MFMAs of F1's second group (hiding that read)
  // so the matrix pipe is fed across the store / barrier / read phases.  Stage kt + 2's global
  // loads (register set kt & 1) have two stages to land. ----
  StampTick tk = stamp_start(args.stamp, sl);
#ifdef BAL_PROBE_SETUPONLY
  if (fa0 == -1 && acc[0][0] == 1.f) PF(0, Y)[threadIdx.x] = 0.f;
  return;
#endif
  load(kt0, r0);
  load(kt0 + 1, r1);
  store(lds + (kt0 & 1) * kBalStage, r0);
  __syncthreads();   // (also publishes zks)
  Frag F0, F1;
  read_half(lds + (kt0 & 1) * kBalStage, 0, F0);
  auto step = [&](int kt, Regs& cur, Regs& nxt, floatx4 (&tg)[NS]) __attribute__((always_inline)) {
    // (kt < kBalXs: the x range into acc; kt >= kBalXs: one phi(q) head per two stages into acc_h)
    const float* buf = lds + (kt & 1) * kBalStage;
    float* nbuf = lds + ((kt + 1) & 1) * kBalStage;
    const bool xr = kt < kBalXs, more = kt + 1 < kBalStages;
    const bool head_end = !xr && ((kt - kBalXs) & 1) == 1;
#ifndef BAL_PROBE_NOLOAD
    if (kt + 2 < kBalStages) load(kt + 2, cur);
#endif
    read_half(buf, 1, F1);
    if (!xr) zdot(buf, kt);
    mfma_part(F0, tg, xr, 0);
    mfma_part(F0, tg, xr, 1);
    ONEPOSE_BAL_SCHED_BARRIER();
#ifndef BAL_PROBE_NOSTORE
    if (more) store(nbuf, nxt);
#endif
    ONEPOSE_BAL_SCHED_BARRIER();
    mfma_part(F1, tg, xr, 0);
    if (head_end) zfinal(((kt - kBalXs) >> 1) & 1);
    __syncthreads();
    if (more) read_half(nbuf, 0, F0);
    ONEPOSE_BAL_SCHED_BARRIER();
    mfma_part(F1, tg, xr, 1);
    if (head_end) fold(((kt - kBalXs) >> 1) & 1);   // every row's Z is in zrow now
  };
  for (int kt = kt0; kt < kBalXs; kt += 2) {   // kt0 is 0 or kBalXs: even
    step(kt, r0, r1, acc);
    step(kt + 1, r1, r0, acc);
  }
#pragma unroll 1
  for (int kt = kBalXs; kt < kBalStages; kt += 2) {
    step(kt, r0, r1, acc_h);
    step(kt + 1, r1, r0, acc_h);
  }
  stamp_ticket(args.stamp, tk);
#ifdef BAL_PROBE_NOEPI
  if (acc[0][0] == 12345.f) PF(0, Y)[threadIdx.x] = acc[NS - 1][1] + acc_h[0][2];   // (keep acc)
  return;
#endif

  // ---- epilogue: y = acc + bias staged per strip [64][kBalTP] (invalid rows hold 0) ----
  float* tile = lds;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int q = s_q[s], rg = s_rg[s];
    const int col = s_cs[s] * 32 + 16 * cbh + r16;
    const float* bp = PF(q, bias);
    const float bias = bp != nullptr ? bp[col] : 0.f;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int row = rbase + 4 * lg + v;
      const float y = acc[s][v] + bias;
      tile[(s * 64 + row) * kBalTP + 16 * cbh + r16] = rg_m0[rg] + row < rg_M[rg] ? y : 0.f;
    }
  }
  __syncthreads();
#ifdef BAL_PROBE_EPI_TILE
  return;
#endif

  // InstanceNorm (mean, M2) partials of strip `wave`'s 32 columns over its M-tile: per 32-row
  // block the sums gemm.hip takes from a wave's registers (a lane's 16 rows in register order,
  // then the lane pair), then the two blocks' merge; written through (sc1) for the finalize
  const int ws = wave;   // the strip this wave finalizes (ws < NS)
  const bool fin = ws < NS && lane < 32;
  unsigned ticket = 0u;
  int f_q = 0, f_b = 0, f_mt = 0, f_cs = 0;
#pragma unroll
  for (int s = 0; s < NS; ++s)
    if (s == ws) {
      f_q = s_q[s];
      f_b = s_b[s];
      f_mt = s_mt[s];
      f_cs = s_cs[s];
    }
  const int f_M = PF(f_q, M), f_N = PF(f_q, N), f_mtiles = PF(f_q, mtiles);
  const int f_rows = min(64, f_M - f_mt * 64);
  unsigned* f_cnt = PF(f_q, st_cnt);
  if (ws < NS) {
    if (fin) {
      const float* tc = tile + ws * 64 * kBalTP + lane;
      float n = 0.f, mean = 0.f, M2 = 0.f;
      for (int wm = 0; wm < 2; ++wm) {
        const int cw = max(min(f_rows - wm * 32, 32), 0);
        float su[2], m2h[2];
        float yv[2][16];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          float s_ = 0.f;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            yv[hh][i] = tc[(wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh) * kBalTP];
            s_ += yv[hh][i];
          }
          su[hh] = s_;
        }
        const float ssum = su[0] + su[1];
        const float wmean = cw ? ssum / (float)cw : 0.f;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          float m2 = 0.f;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int row = wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
            const float d = yv[hh][i] - wmean;
            m2 += (row < f_rows) ? d * d : 0.f;
          }
          m2h[hh] = m2;
        }
        const float nb = (float)max(min(wm * 32 + 32, f_rows) - wm * 32, 0);
        if (nb == 0.f) continue;
        in_merge_block(n, mean, M2, nb, wmean, m2h[0] + m2h[1]);
      }
      float* st_out = PF(f_q, stats) + ((int64_t)f_b * f_mtiles + f_mt) * 2 * f_N + f_cs * 32 + lane;
      __hip_atomic_store(st_out, mean, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(st_out + f_N, M2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's partial stores drained
#ifdef BAL_PROBE_EPI_NOFIN
    if (false) {
#else
    if (lane == 0) {
#endif
      const int G1 = stats_group_size(f_mtiles);
      const int ngroups = (f_mtiles + G1 - 1) / G1;
      unsigned* cb = f_cnt + (int64_t)f_b * PF(f_q, st_cnt_bs);
      ticket = __hip_atomic_fetch_add(cb + kBalNS + f_cs * ngroups + f_mt / G1, 1u,
                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }

  // the strips' Y rows (float4 rows of the staged tiles) while the tickets are in flight
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int rg = s_rg[s], q = s_q[s];
    const int r = t >> 3, c4 = (t & 7) * 4;
    if (rg_m0[rg] + r < rg_M[rg]) {
      const float4 v = *reinterpret_cast<const float4*>(tile + (s * 64 + r) * kBalTP + c4);
      float* Y = PF(q, Y) + s_b[s] * PF(q, y_bs);
      *reinterpret_cast<float4*>(Y + (int64_t)(rg_m0[rg] + r) * PF(q, ldy) + s_cs[s] * 32 + c4) = v;
    }
  }

  // two-level finalize (gemm.hip's, per 32-column block): the group's last M-tile merges the
  // group's partials, the last group merger the groups -> mean, rstd
#ifdef BAL_PROBE_EPI_NOFIN
  if (false) {
#else
  if (ws < NS) {
#endif
    const int G1 = stats_group_size(f_mtiles);
    const int ngroups = (f_mtiles + G1 - 1) / G1, g1 = f_mt / G1;
    const int gt0 = g1 * G1, gsz = min(G1, f_mtiles - gt0);
    const int M = f_M, N = f_N;
    ticket = __shfl(ticket, 0, 64);
    if (ticket == (unsigned)(gsz - 1)) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      unsigned* cb = f_cnt + (int64_t)f_b * PF(f_q, st_cnt_bs);
      double* gp = PF(f_q, st_grp) + (int64_t)f_b * ngroups * 2 * N;
      const int col = f_cs * 32 + lane;
      if (fin) {
        const float* sp = PF(f_q, stats) + (int64_t)f_b * f_mtiles * 2 * N + col;
        auto ld = [&](int ti, int half) __attribute__((always_inline)) {
          return __hip_atomic_load(sp + (int64_t)ti * 2 * N + half * N, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        };
        const double c = (double)ld(gt0, 0);
        double s1 = 0.0, s2 = 0.0, ng = 0.0;
        constexpr int UD = 16;
        for (int u0 = 0; u0 < gsz; u0 += UD) {
          float mv[UD], qv[UD];
#pragma unroll
          for (int u = 0; u < UD; ++u) {
            const int ti = gt0 + min(u0 + u, gsz - 1);
            mv[u] = ld(ti, 0);
            qv[u] = ld(ti, 1);
          }
#pragma unroll
          for (int u = 0; u < UD; ++u)
            if (u0 + u < gsz)
              in_merge_tile(s1, s2, ng, (double)min(64, M - (gt0 + u0 + u) * 64), mv[u], qv[u], c);
        }
        __hip_atomic_store(gp + (int64_t)g1 * 2 * N + col, in_group_mean(c, s1, ng),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(gp + (int64_t)g1 * 2 * N + N + col, in_group_m2(s1, s2, ng),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      unsigned t2 = 0u;
      if (lane == 0)
        t2 = __hip_atomic_fetch_add(cb + f_cs, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      t2 = __shfl(t2, 0, 64);
      if (t2 == (unsigned)(ngroups - 1) && fin) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const double* g2 = gp + col;
        auto ld2 = [&](int gi, int half) __attribute__((always_inline)) {
          return __hip_atomic_load(g2 + (int64_t)gi * 2 * N + half * N, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        };
        const double c = ld2(0, 0);
        double S1 = 0.0, S2 = 0.0;
        constexpr int GD = kStatsMaxGroups;
        for (int q0 = 0; q0 < ngroups; q0 += GD) {
          double mg[GD], m2g[GD];
#pragma unroll
          for (int u = 0; u < GD; ++u) {
            const int gi = min(q0 + u, ngroups - 1);
            mg[u] = ld2(gi, 0);
            m2g[u] = ld2(gi, 1);
          }
#pragma unroll
          for (int u = 0; u < GD; ++u) {
            const int gi = q0 + u;
            if (gi < ngroups)
              in_merge_group(S1, S2, (double)min(G1 * 64, M - gi * G1 * 64), mg[u], m2g[u], c);
          }
        }
        const double n = (double)M;
        PF(f_q, st_mean)[(int64_t)f_b * N + col] = in_final_mean(c, S1, n);
        PF(f_q, st_rstd)[(int64_t)f_b * N + col] = in_final_rstd(S1, S2, n);
      }
    }
  }
  stamp_end(args.stamp, tk, sl);
#undef PF
}

template <bool MIX>
__global__ __launch_bounds__(kBalNT) __attribute__((amdgpu_waves_per_eu(2)))
void gemm_mlp1_bal_kernel(GemmArgs args) {
  __shared__ __attribute__((aligned(16))) float lds[2 * kBalStage];
  __shared__ BalShared sh;
  __shared__ StampLds sl;
  const int G = gridDim.x;
  const int g = xcd_contiguous(blockIdx.x, G);   // an XCD's workgroups hold adjacent strips
  const int64_t S0 = (int64_t)args.p[0].batch * args.p[0].mtiles * kBalNS;
  const int64_t S1 = args.nprob > 1 ? (int64_t)args.p[1].batch * args.p[1].mtiles * kBalNS : 0;
  const int c0 = args.p[0].acc0 != nullptr ? 1 : 2;
  const int c1 = (args.nprob > 1 && args.p[1].acc0 != nullptr) ? 1 : 2;
  const int64_t C = S0 * c0 + S1 * c1;
  const int i0 = bal_first_strip(C * g / G, S0, c0, c1);
  const int ns = bal_first_strip(C * (g + 1) / G, S0, c0, c1) - i0;
  switch (ns) {   // (host-checked: 1 <= ns <= kBalS)
    case 1: bal_body<1, MIX>(args, i0, S0, lds, sh, &sl); break;
    case 2: bal_body<2, MIX>(args, i0, S0, lds, sh, &sl); break;
    case 3: bal_body<3, MIX>(args, i0, S0, lds, sh, &sl); break;
    case 4: bal_body<4, MIX>(args, i0, S0, lds, sh, &sl); break;
    case 5: bal_body<5, MIX>(args, i0, S0, lds, sh, &sl); break;
    default: bal_body<5, MIX>(args, i0, S0, lds, sh, &sl); break;
  }
}

int g_num_cus = 0;

}  // namespace

bool g_bal_disable = false;   // (tools/bal_probe.hip: the 64 x 64 kernel for comparison)

int gemm_bal_counters_per_sample(int M) {
  return kBalNS * (1 + stats_groups(M, 64));
}

// Launch MLP conv 1 on the balanced kernel when it applies (fp32, N = K = 512, ksplit 256,
// in-launch finalize, at most kBalS strips per workgroup); returns false (nothing launched) to
// leave the launch to the 64 x 64 kernel.
bool gemm_bal_try(GemmArgs& args, hipStream_t stream, int kind, int* rc) {
  *rc = ONEPOSE_OK;
  if (g_bal_disable || args.nprob < 1 || args.nprob > 2) return false;
  int64_t S[2] = {0, 0};
  int c[2] = {2, 2};
  for (int i = 0; i < args.nprob; ++i) {
    const GemmProb& P = args.p[i];
    if (P.N != 512 || P.K != kBalK || P.ksplit != kBalKs || P.A1 == nullptr || P.st_cnt == nullptr ||
        P.st_grp == nullptr || P.ksum == nullptr || P.Wp != nullptr || P.Ap != nullptr ||
        P.lda0 % 4 || P.lda1 % 4 || P.ldw % 4 || (P.W1 != nullptr && P.ldw1 % 4) || P.ldy % 4 ||
        P.st_cnt_bs < gemm_bal_counters_per_sample(P.M))
      return false;
    S[i] = (int64_t)P.batch * ceil_div(P.M, 64) * kBalNS;
    c[i] = P.acc0 != nullptr ? 1 : 2;
  }
  if (g_num_cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    g_num_cus = n;
  }
  // only where the 64 x 64 tiles leave CUs unevenly loaded: at most 3 tiles per CU
  const int64_t tiles64 = (S[0] + S[1]) / 2;
  if (tiles64 > 3 * (int64_t)g_num_cus) return false;
  const int64_t C = S[0] * c[0] + S[1] * c[1];
  const int G = (int)std::min<int64_t>(g_num_cus, S[0] + S[1]);
  for (int gg = 0; gg < G; ++gg) {
    const int a = bal_first_strip(C * gg / G, S[0], c[0], c[1]);
    const int b = bal_first_strip(C * (gg + 1) / G, S[0], c[0], c[1]);
    if (b - a > kBalS || b - a < 1) return false;
#ifdef ONEPOSE_BAL_MIN2   // (diagnostic build)
    if (b - a < 2) return false;
#endif
  }
  for (int i = 0; i < args.nprob; ++i) {
    GemmProb& P = args.p[i];
    P.mtiles = ceil_div(P.M, 64);
    P.ntiles = 8;
    P.tiles = P.mtiles * P.ntiles * P.batch;
  }
  if (args.nprob == 1) memset(&args.p[1], 0, sizeof(GemmProb));   // never read: S1 = 0
  prof_pre(kind, stream);
  args.stamp = prof_stamp_slot(kind);
  if (c[0] == 1 || c[1] == 1)
    hipLaunchKernelGGL(gemm_mlp1_bal_kernel<true>, dim3(G), dim3(kBalNT), 0, stream, args);
  else
    hipLaunchKernelGGL(gemm_mlp1_bal_kernel<false>, dim3(G), dim3(kBalNT), 0, stream, args);
  prof_post(kind, stream);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("gemm_bal: launch failed: %s", hipGetErrorString(e));
    *rc = ONEPOSE_ERR_HIP;
  }
  return true;
}

}  // namespace onepose
