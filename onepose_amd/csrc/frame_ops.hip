// Per-frame glue around the matcher, all on the device so a frame never round-trips
// through the host:
//   * SuperPoint descriptor sampling (superpoint.py:95-113)
//   * correspondence selection + PnP input conversion (inference.py:147-152,
//     eval_utils.py:22-26)
//   * cm/deg pose error (eval_utils.py:45-63, cmd_evaluator.py:11-31)
#include "common.h"

namespace onepose {

// Bilinear grid_sample (zero padding) at keypoints, then L2 normalise over channels.  The
// float32 operation order of the reference is kept (kp - s/2 + 0.5, / [(w*s - s/2 - 0.5),
// ...], *2 - 1, grid_sampler_compute_source_index, nw/ne/sw/se weights).  One wave per
// keypoint, 4 channels per lane.
__global__ __launch_bounds__(256) void sample_descriptors_kernel(
    const float* __restrict__ kpts, const float* __restrict__ dense, int batch, int n, int c,
    int h, int w, int s, int align_corners, float* __restrict__ out) {
#pragma clang fp contract(off)
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (gw >= batch * n) return;
  const int b = gw / n, k = gw - b * n;
  const float hs = (float)s / 2.0f;
  float x = kpts[((int64_t)b * n + k) * 2 + 0];
  float y = kpts[((int64_t)b * n + k) * 2 + 1];
  x = (x - hs) + 0.5f;
  y = (y - hs) + 0.5f;
  const float dx = (float)((double)w * s - s / 2.0 - 0.5);
  const float dy = (float)((double)h * s - s / 2.0 - 0.5);
  x = x / dx;
  y = y / dy;
  x = x * 2.0f - 1.0f;
  y = y * 2.0f - 1.0f;
  float ix, iy;
  if (align_corners) {
    ix = ((x + 1.0f) / 2.0f) * (float)(w - 1);
    iy = ((y + 1.0f) / 2.0f) * (float)(h - 1);
  } else {
    ix = ((x + 1.0f) * (float)w - 1.0f) / 2.0f;
    iy = ((y + 1.0f) * (float)h - 1.0f) / 2.0f;
  }
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  const int x0 = (int)fx0, y0 = (int)fy0, x1 = x0 + 1, y1 = y0 + 1;
  const float wnw = ((float)x1 - ix) * ((float)y1 - iy);
  const float wne = (ix - (float)x0) * ((float)y1 - iy);
  const float wsw = ((float)x1 - ix) * (iy - (float)y0);
  const float wse = (ix - (float)x0) * (iy - (float)y0);
  const bool vnw = x0 >= 0 && x0 < w && y0 >= 0 && y0 < h;
  const bool vne = x1 >= 0 && x1 < w && y0 >= 0 && y0 < h;
  const bool vsw = x0 >= 0 && x0 < w && y1 >= 0 && y1 < h;
  const bool vse = x1 >= 0 && x1 < w && y1 >= 0 && y1 < h;
  const float* d = dense + (int64_t)b * c * h * w;
  const int64_t plane = (int64_t)h * w;
  float v[8];
  float ss = 0.f;
  const int per = (c + 63) / 64;
  for (int i = 0; i < per && i < 8; ++i) {
    const int ch = lane + 64 * i;
    float acc = 0.f;
    if (ch < c) {
      const float* p = d + ch * plane;
      if (vnw) acc += p[y0 * w + x0] * wnw;
      if (vne) acc += p[y0 * w + x1] * wne;
      if (vsw) acc += p[y1 * w + x0] * wsw;
      if (vse) acc += p[y1 * w + x1] * wse;
    }
    v[i] = acc;
    ss += acc * acc;
  }
  ss = wave_sum(ss);
  const float nrm = fmaxf(sqrtf(ss), 1e-12f);
  float* o = out + (int64_t)b * c * n;
  for (int i = 0; i < per && i < 8; ++i) {
    const int ch = lane + 64 * i;
    if (ch < c) o[(int64_t)ch * n + k] = v[i] / nrm;
  }
}

// Compact the valid matches of each frame in ascending 2D-index order (numpy boolean
// indexing order), converting to the float32 points solvePnPRansac works on:
// pts3d = float32(float64(kpt3d) * scale).  One workgroup per frame, block-wide scan.
__global__ __launch_bounds__(1024) void select_kernel(const int64_t* __restrict__ matches0,
                                                      const float* __restrict__ kp2,
                                                      int64_t kp2_bs,
                                                      const float* __restrict__ kp3,
                                                      int64_t kp3_bs, int n1, int n3,
                                                      double scale, float* __restrict__ p2,
                                                      float* __restrict__ p3,
                                                      int* __restrict__ counts) {
  __shared__ int wave_tot[16];
  __shared__ int base_s;
  const int b = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t* m = matches0 + (int64_t)b * n1;
  const float* k2 = kp2 + b * kp2_bs;
  const float* k3 = kp3 + b * kp3_bs;
  float* o2 = p2 + (int64_t)b * n1 * 2;
  float* o3 = p3 + (int64_t)b * n1 * 3;
  if (t == 0) base_s = 0;
  __syncthreads();
  for (int start = 0; start < n1; start += 1024) {
    const int i = start + t;
    int64_t j = (i < n1) ? m[i] : -1;
    const bool valid = j > -1 && j < n3;
    const unsigned long long bal = __ballot(valid);
    const int before = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wave_tot[wave] = __popcll(bal);
    __syncthreads();
    int off = base_s;
    for (int w2 = 0; w2 < wave; ++w2) off += wave_tot[w2];
    if (valid) {
      const int pos = off + before;
      o2[pos * 2 + 0] = k2[(int64_t)i * 2 + 0];
      o2[pos * 2 + 1] = k2[(int64_t)i * 2 + 1];
      o3[pos * 3 + 0] = (float)((double)k3[j * 3 + 0] * scale);
      o3[pos * 3 + 1] = (float)((double)k3[j * 3 + 1] * scale);
      o3[pos * 3 + 2] = (float)((double)k3[j * 3 + 2] * scale);
    }
    __syncthreads();
    if (t == 0) {
      int tot = 0;
      for (int w2 = 0; w2 < 16; ++w2) tot += wave_tot[w2];
      base_s += tot;
    }
    __syncthreads();
  }
  if (t == 0) counts[b] = base_s;
}

// query_pose_error / Evaluator (pose_error_one, common.h), one thread per frame.
__global__ void pose_error_kernel(const double* __restrict__ pred, const double* __restrict__ gt,
                                  int64_t gt_bs, int batch, double* rerr, double* terr,
                                  uint8_t* cmd) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  pose_error_one(pred + (int64_t)b * 12, gt + b * gt_bs, rerr + b, terr + b, cmd + b * 3);
}

}  // namespace onepose

using namespace onepose;

extern "C" {

int onepose_sample_descriptors(const float* keypoints, const float* dense, int batch, int n,
                               int c, int h, int w, int s, int align_corners, float* out,
                               void* stream) {
  clear_error();
  OP_REQUIRE(keypoints && dense && out, "sample_descriptors: null pointer");
  OP_REQUIRE(batch >= 1 && n >= 0 && c >= 1 && c <= 512 && h >= 1 && w >= 1 && s >= 1,
             "sample_descriptors: bad shape b=%d n=%d c=%d h=%d w=%d s=%d", batch, n, c, h, w, s);
  if (n == 0) return ONEPOSE_OK;
  const int waves = batch * n;
  OP_LAUNCH(K_SAMPLE, static_cast<hipStream_t>(stream), sample_descriptors_kernel, dim3(ceil_div(waves, 4)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), keypoints, dense, batch, n, c, h, w, s,
                     align_corners, out);
  return ONEPOSE_OK;
}

int onepose_select_correspondences(const int64_t* matches0, const float* kpts2d,
                                   int64_t kpts2d_bstride, const float* kpts3d,
                                   int64_t kpts3d_bstride, int batch, int n1, int n3,
                                   double scale3d, float* pts2d, float* pts3d, int* counts,
                                   void* stream) {
  clear_error();
  OP_REQUIRE(matches0 && kpts2d && kpts3d && pts2d && pts3d && counts, "select: null pointer");
  OP_REQUIRE(batch >= 1 && n1 >= 1 && n3 >= 1, "select: bad shape");
  OP_LAUNCH(K_SELECT, static_cast<hipStream_t>(stream), select_kernel, dim3(batch), dim3(1024), 0, static_cast<hipStream_t>(stream),
                     matches0, kpts2d, kpts2d_bstride, kpts3d, kpts3d_bstride, n1, n3, scale3d,
                     pts2d, pts3d, counts);
  return ONEPOSE_OK;
}

int onepose_pose_errors(const double* pose_pred, const double* pose_gt, int64_t gt_bstride,
                        int batch, double* R_err_deg, double* t_err_cm, uint8_t* cmd,
                        void* stream) {
  clear_error();
  OP_REQUIRE(pose_pred && pose_gt && R_err_deg && t_err_cm && cmd, "pose_errors: null pointer");
  OP_REQUIRE(batch >= 1, "pose_errors: batch=%d", batch);
  OP_LAUNCH(K_POSE_ERR, static_cast<hipStream_t>(stream), pose_error_kernel, dim3(ceil_div(batch, 64)), dim3(64), 0,
                     static_cast<hipStream_t>(stream), pose_pred, pose_gt, gt_bstride, batch,
                     R_err_deg, t_err_cm, cmd);
  return ONEPOSE_OK;
}

}  // extern "C"
