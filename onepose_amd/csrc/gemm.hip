// fp32 MFMA grouped token-GEMM (see gemm.h).
//
// Tile: 64 tokens x BN outputs x 32-deep K step, 256 threads = 4 waves in a 2x2 grid; each
// wave owns 32 x BN/2 outputs = BN/64 accumulators of v_mfma_f32_32x32x2_f32.  Operands are
// staged through double-buffered LDS images [row][k] with a 36-float row pitch: a
// ds_read_b128 lane group (16 lanes, 16 distinct rows, same k) covers 16 distinct 16-byte
// slots of the 64-bank row -- conflict free (9*i mod 16 is a permutation).  Each b128 read
// feeds four MFMAs: within one group of 8 k-values, lane half h carries k = 8*kk + 4*h + j
// into MFMA j, identically for A and W, so the k-sum is unchanged (a re-ordering of it).
// The next K step's global loads are issued before the MFMAs and are only consumed (prologue
// transform + LDS store) after them, so the loads overlap the matrix work; one barrier per
// K step.
#include "gemm.h"

#include <cstring>

namespace onepose {

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int BM = kGemmBM, BK = kGemmBK;
constexpr int PITCH = BK + 4;   // 36 floats

template <int BN>
struct Stage {
  float4 a[2];
  float4 w[BN / 32];
  float4 mean, rstd;
};

// Per-launch problem fields, selected field by field from the kernel arguments (a
// dynamically indexed kernel-argument struct would be copied to scratch).
struct Ctx {
  const float *a0, *a1, *w0, *w1, *mean, *rstd;
  int lda0, lda1, ldw0, ldw1, ksplit, M, N, K;
};

template <int PRO, int BN>
__device__ __forceinline__ void load_stage(const Ctx& c, int m0, int n0, int k0, Stage<BN>& s) {
  const int t = threadIdx.x;
  const int kq = (t & 7) * 4;
  const bool first = k0 < c.ksplit;
  const float* A = first ? c.a0 : c.a1;
  const int lda = first ? c.lda0 : c.lda1;
  const float* W = first ? c.w0 : c.w1;
  const int ldw = first ? c.ldw0 : c.ldw1;
  const int kk = first ? (k0 + kq) : (k0 - c.ksplit + kq);
  if (PRO == PRO_NORM_RELU) {
    s.mean = *reinterpret_cast<const float4*>(c.mean + k0 + kq);
    s.rstd = *reinterpret_cast<const float4*>(c.rstd + k0 + kq);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + (t >> 3) + 32 * i;
    s.a[i] = (m < c.M) ? *reinterpret_cast<const float4*>(A + (int64_t)m * lda + kk)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int i = 0; i < BN / 32; ++i) {
    const int o = n0 + (t >> 3) + 32 * i;
    s.w[i] = (o < c.N) ? *reinterpret_cast<const float4*>(W + (int64_t)o * ldw + kk)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

template <int PRO, int BN>
__device__ __forceinline__ void store_stage(float* lds_a, float* lds_w, Stage<BN>& s, int m0,
                                            int M) {
  const int t = threadIdx.x;
  const int kq = (t & 7) * 4;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (t >> 3) + 32 * i;
    float4 v = s.a[i];
    if (PRO == PRO_NORM_RELU) {
      if (m0 + row < M) {
        v.x = fmaxf((v.x - s.mean.x) * s.rstd.x, 0.f);
        v.y = fmaxf((v.y - s.mean.y) * s.rstd.y, 0.f);
        v.z = fmaxf((v.z - s.mean.z) * s.rstd.z, 0.f);
        v.w = fmaxf((v.w - s.mean.w) * s.rstd.w, 0.f);
      }
    }
    *reinterpret_cast<float4*>(lds_a + row * PITCH + kq) = v;
  }
#pragma unroll
  for (int i = 0; i < BN / 32; ++i) {
    const int row = (t >> 3) + 32 * i;
    *reinterpret_cast<float4*>(lds_w + row * PITCH + kq) = s.w[i];
  }
}

template <int EPI, int PRO, int BN>
__device__ __forceinline__ void gemm_body(const GemmArgs& args) {
  constexpr int FN = BN / 64;           // accumulators per wave
  constexpr int STAGE = (BM + BN) * PITCH;
  __shared__ __attribute__((aligned(16))) float lds[2 * STAGE];
  __shared__ float zrow[BM];
  __shared__ float zrow_stats[(EPI == EPI_STATS) ? 512 : 1];

  // XCD-aware tile order: blocks are dealt round-robin over the 8 XCDs, so hand each XCD a
  // contiguous run of logical tiles -- the N-tiles of one M-tile then share that XCD's L2
  // (A is fetched once per XCD instead of once per N-tile).
  int bid = xcd_contiguous(blockIdx.x, gridDim.x);
  const bool second = bid >= args.p[0].tiles;
#define F(x) (second ? args.p[1].x : args.p[0].x)
  if (second) bid -= args.p[0].tiles;
  const int mtiles = F(mtiles), ntiles = F(ntiles);
  const int per_sample = mtiles * ntiles;
  const int b = bid / per_sample;
  const int r = bid - b * per_sample;
  const int mt = r / ntiles;
  const int nt = r - mt * ntiles;
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

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  floatx16 acc[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;

  // Prefetch distance 2: while the MFMAs consume K step kt from LDS, step kt+1 sits in
  // registers (loaded one step earlier) and step kt+2's loads are in flight, so each global
  // load has two MFMA phases to land (a lone 64x64 tile per CU has no other waves to hide
  // the latency behind).
  const int nk = c.K / BK;
  Stage<BN> s0, s1;
  load_stage<PRO, BN>(c, m0, n0, 0, s0);
  if (nk > 1) load_stage<PRO, BN>(c, m0, n0, BK, s1);
  store_stage<PRO, BN>(lds, lds + BM * PITCH, s0, m0, c.M);
  __syncthreads();

  auto step = [&](int kt, Stage<BN>& next, Stage<BN>& spare) __attribute__((always_inline)) {
    const float* la = lds + (kt & 1) * STAGE;
    const float* lw = la + BM * PITCH;
    if (kt + 2 < nk) load_stage<PRO, BN>(c, m0, n0, (kt + 2) * BK, spare);
    const float* pa = la + (wm * 32 + (lane & 31)) * PITCH + (lane >> 5) * 4;
    const float* pw = lw + (wn * (BN / 2) + (lane & 31)) * PITCH + (lane >> 5) * 4;
#pragma unroll
    for (int kk = 0; kk < BK / 8; ++kk) {
      const float4 a = *reinterpret_cast<const float4*>(pa + kk * 8);
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const float4 w = *reinterpret_cast<const float4*>(pw + j * 32 * PITCH + kk * 8);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, w.x, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, w.y, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, w.z, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, w.w, acc[j], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) {
      float* na = lds + ((kt + 1) & 1) * STAGE;
      store_stage<PRO, BN>(na, na + BM * PITCH, next, m0, c.M);
    }
    __syncthreads();
  };
  for (int kt = 0; kt < nk; kt += 2) {
    step(kt, s1, s0);
    if (kt + 1 < nk) step(kt + 1, s0, s1);
  }

  // ---- epilogue ----
  const int M = c.M, N = c.N;
  const float* biasp = F(bias);
  float* Y = F(Y) + b * F(y_bs);
  const int ldy = F(ldy);
  float* tile = lds;   // [64][BN+1] staging for the reducing epilogues
  constexpr int TP = BN + 1;
  constexpr bool kStage =
      EPI == EPI_STATS || EPI == EPI_SCORE || EPI == EPI_KVPART || EPI == EPI_QZ;

  float res[FN][16];
  if (EPI == EPI_RESID) {   // all residual loads issued before the first store
    const float* R = F(R) + b * F(r_bs);
    const int ldr = F(ldr);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int gn = n0 + wn * (BN / 2) + j * 32 + (lane & 31);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int gm = m0 + wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
        res[j][i] = (gm < M && gn < N) ? R[(int64_t)gm * ldr + gn] : 0.f;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int col = wn * (BN / 2) + j * 32 + (lane & 31);
    const int gn = n0 + col;
    const bool col_ok = gn < N;
    const float bias = (EPI != EPI_SCORE && biasp != nullptr && col_ok) ? biasp[gn] : 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
      const int gm = m0 + row;
      float y;
      if (EPI == EPI_SCORE) {
        y = acc[j][i] / F(scale);
      } else {
        y = acc[j][i] + bias;
        if (EPI == EPI_QZ) y = elu1(y) + 1.0f;
        if (EPI == EPI_KVPART) y = (col < 64) ? (elu1(y) + 1.0f) : (y / F(vdiv));
      }
      if (EPI == EPI_BIAS || EPI == EPI_STATS || EPI == EPI_SCORE || EPI == EPI_RESID) {
        if (gm < M && col_ok) {
          if (EPI == EPI_RESID) y = res[j][i] + y;
          Y[(int64_t)gm * ldy + gn] = y;
        }
      }
      if (kStage) tile[row * TP + col] = (gm < M) ? y : 0.f;
    }
  }
  if (!kStage) return;
  __syncthreads();
  const int t = threadIdx.x;
  const int rows = min(BM, M - m0);

  if (EPI == EPI_STATS) {
    // per column: 4 row groups of 16 -> (sum, M2 about the group mean), Chan-merged in order
    float* part = reinterpret_cast<float*>(zrow_stats);
    const int col = t & 63, rg = t >> 6;
    const int r0 = rg * 16, r1 = min(r0 + 16, rows);
    const int cnt = max(r1 - r0, 0);
    float s = 0.f;
    for (int rr = r0; rr < r1; ++rr) s += tile[rr * TP + col];
    const float gmean = cnt ? s / (float)cnt : 0.f;
    float m2 = 0.f;
    for (int rr = r0; rr < r1; ++rr) {
      const float d = tile[rr * TP + col] - gmean;
      m2 += d * d;
    }
    part[(rg * 64 + col) * 2] = gmean;
    part[(rg * 64 + col) * 2 + 1] = m2;
    __syncthreads();
    if (t < 64 && n0 + t < N) {
      float n = 0.f, mean = 0.f, M2 = 0.f;
      for (int g = 0; g < 4; ++g) {
        const float nb = (float)max(min(g * 16 + 16, rows) - g * 16, 0);
        if (nb == 0.f) continue;
        const float mb = part[(g * 64 + t) * 2], m2b = part[(g * 64 + t) * 2 + 1];
        const float nn = n + nb, delta = mb - mean;
        mean += delta * (nb / nn);
        M2 += m2b + delta * delta * (n * nb / nn);
        n = nn;
      }
      float* st_out = F(stats) + ((int64_t)b * mtiles + mt) * 2 * N;
      st_out[n0 + t] = mean;
      st_out[N + n0 + t] = M2;
    }
  }
  if (EPI == EPI_SCORE) {
    const int cols = min(BN, N - n0);
    if (t < BM) {
      if (t < rows) {   // row partial over this tile's columns
        float mx = -INFINITY;
        for (int cc = 0; cc < cols; ++cc) mx = fmaxf(mx, tile[t * TP + cc]);
        float s = 0.f;
        for (int cc = 0; cc < cols; ++cc) s += expf(tile[t * TP + cc] - mx);
        float* o = F(rowstat) + (((int64_t)b * M + m0 + t) * ntiles + nt) * 2;
        o[0] = mx;
        o[1] = s;
      }
    } else if (t < BM + BN) {
      const int cc = t - BM;
      if (cc < cols) {   // column partial over this tile's rows
        float mx = -INFINITY;
        for (int rr = 0; rr < rows; ++rr) mx = fmaxf(mx, tile[rr * TP + cc]);
        float s = 0.f;
        for (int rr = 0; rr < rows; ++rr) s += expf(tile[rr * TP + cc] - mx);
        float* o = F(colstat) + (((int64_t)b * N + n0 + cc) * mtiles + mt) * 2;
        o[0] = mx;
        o[1] = s;
      }
    }
  }
  if (EPI == EPI_QZ) {
    // Z[row] = 1 / (phi(q)_row . ksum_h + 1e-6), h = the head this 64-column tile holds
    {
      const float* ks = F(ksum) + b * F(ksum_bs) + n0;
      const int row = t >> 2, q = t & 3;   // 4 lanes per row, 16 channels each
      float s = 0.f;
#pragma unroll
      for (int cc = 0; cc < 16; ++cc) s += tile[row * TP + q * 16 + cc] * ks[q * 16 + cc];
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      if (q == 0) zrow[row] = 1.0f / (s + 1e-6f);
    }
    __syncthreads();
    const float ns = F(ns);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = (t >> 4) + 16 * (i & 3);
      const int cc = (t & 15) + 16 * (i >> 2);
      const int gm = m0 + row;
      if (gm < M) Y[(int64_t)gm * ldy + n0 + cc] = tile[row * TP + cc] * zrow[row] * ns;
    }
  }
  if (EPI == EPI_KVPART) {
    // KV_h[d][q] = sum_rows phi(k)[row][d] * v[row][q]   (columns 0..63 | 64..127 of the tile)
    const int h = n0 / 128;
    if (t < 64) {
      float s = 0.f;
      for (int rr = 0; rr < rows; ++rr) s += tile[rr * TP + t];
      F(kspart)[((int64_t)b * mtiles + mt) * 256 + h * 64 + t] = s;
    }
    const int wd = wave >> 1, wq = wave & 1;
    floatx16 kv;
#pragma unroll
    for (int i = 0; i < 16; ++i) kv[i] = 0.f;
    const float* ka = tile + wd * 32 + (lane & 31);
    const float* vb = tile + 64 + wq * 32 + (lane & 31);
#pragma unroll 8
    for (int k = 0; k < BM; k += 2) {
      const int rr = (k + (lane >> 5)) * TP;
      kv = __builtin_amdgcn_mfma_f32_32x32x2f32(ka[rr], vb[rr], kv, 0, 0, 0);
    }
    float* out = F(kvpart) + (((int64_t)b * mtiles + mt) * 4 + h) * 4096;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int d = wd * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
      out[d * 64 + wq * 32 + (lane & 31)] = kv[i];
    }
  }
#undef F
}

template <int EPI, int PRO, int BN>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmArgs args) {
  stamp_begin(args.stamp);
  gemm_body<EPI, PRO, BN>(args);
  stamp_end(args.stamp);
}

template <int EPI, int PRO, int BN>
void launch_one(GemmArgs& args, int grid, hipStream_t stream) {
  hipLaunchKernelGGL((gemm_f32_kernel<EPI, PRO, BN>), dim3(grid), dim3(256), 0, stream, args);
}

}  // namespace

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

int gemm_launch(int epi, int pro, int bn, GemmArgs& args, hipStream_t stream, int kind) {
  int grid = 0;
  for (int i = 0; i < 2; ++i) {
    GemmProb& P = args.p[i];
    if (i >= args.nprob) {
      P.tiles = 0;
      continue;
    }
    OP_REQUIRE(P.K % kGemmBK == 0, "gemm: K=%d not a multiple of %d", P.K, kGemmBK);
    OP_REQUIRE(P.ksplit % kGemmBK == 0, "gemm: ksplit=%d", P.ksplit);
    OP_REQUIRE(P.lda0 % 4 == 0 && P.ldw % 4 == 0, "gemm: unaligned leading dimension");
    OP_REQUIRE(epi != EPI_KVPART || (bn == 128 && P.N % 128 == 0), "gemm: KVPART tiling");
    OP_REQUIRE(epi != EPI_QZ || (bn == 64 && P.N % 64 == 0), "gemm: QZ tiling");
    P.mtiles = ceil_div(P.M, kGemmBM);
    P.ntiles = ceil_div(P.N, bn);
    P.tiles = P.mtiles * P.ntiles * P.batch;
    grid += P.tiles;
  }
  if (grid == 0) return ONEPOSE_OK;
  args.stamp = nullptr;
#define CASE(E, PR, BN_)                          \
  if (epi == E && pro == PR && bn == BN_) {       \
    prof_pre(kind, stream);                       \
    args.stamp = prof_stamp_slot(kind);           \
    launch_one<E, PR, BN_>(args, grid, stream);   \
    prof_post(kind, stream);                      \
    OP_LAUNCHED();                                \
    return ONEPOSE_OK;                            \
  }
  CASE(EPI_BIAS, PRO_PLAIN, 64)
  CASE(EPI_KVPART, PRO_PLAIN, 128)
  CASE(EPI_QZ, PRO_PLAIN, 64)
  CASE(EPI_STATS, PRO_PLAIN, 64)
  CASE(EPI_RESID, PRO_NORM_RELU, 64)
  CASE(EPI_SCORE, PRO_PLAIN, 64)
#undef CASE
  set_error("gemm: unsupported epilogue/prologue/bn %d/%d/%d", epi, pro, bn);
  return ONEPOSE_ERR_INVALID;
}

}  // namespace onepose
