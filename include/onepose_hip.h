/*
 * onepose_hip.h -- C-ABI of libonepose_hip.so, the MI355X (gfx950) engine for OnePose's
 * GATsSPG 2D-3D matching + RANSAC-EPnP hot path.
 *
 * Plain pointers and sizes only.  Conventions:
 *   - every buffer belongs to the caller; the launch entry points never allocate or free
 *     device memory and never synchronise, so they are hipGraph-capturable (the measurement
 *     hooks onepose_profile_* are the exception: they own their timing buffers);
 *   - "device" pointers are HIP device memory (e.g. torch tensors' data_ptr()),
 *     "host" pointers are ordinary CPU memory;
 *   - `stream` is a hipStream_t passed as void* (NULL = the default stream);
 *   - every function returns ONEPOSE_OK (0) or an error code, with a thread-local message
 *     in onepose_last_error(); no C++ exception crosses the ABI.
 *
 * The reference (huanghaoran111/OnePose @ /root/reference) has no FFI of its own: its hot
 * path is PyTorch + OpenCV called from Python.  Each entry point below names the
 * reference interface it replaces; INTEGRATION.md shows the ctypes binding
 * (onepose_amd/_lib.py) that a maintainer would drop in.
 */
#ifndef ONEPOSE_HIP_H
#define ONEPOSE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  ONEPOSE_OK = 0,
  ONEPOSE_ERR_INVALID = 1,      /* bad argument / shape                                  */
  ONEPOSE_ERR_HIP = 2,          /* a HIP runtime call failed                            */
  ONEPOSE_ERR_UNSUPPORTED = 3,  /* valid in the reference, not supported by this build  */
  ONEPOSE_ERR_WORKSPACE = 4     /* workspace too small                                  */
};

/* Matcher arithmetic (onepose_match_ex / onepose_match_prepared_ex). */
enum {
  ONEPOSE_PREC_FP32 = 0,        /* every contraction on fp32-input MFMA: the reference's
                                   numerics up to summation order (bit-exact indices)   */
  ONEPOSE_PREC_BF16_ATTN = 1,   /* the attention layers' GEMMs (q/k/v projection, merge+MLP)
                                   take bf16-rounded operands on v_mfma_f32_32x32x16_bf16
                                   with fp32 accumulation (BASELINE config 5); GAT, final
                                   projection, scores and dual softmax stay fp32       */
  ONEPOSE_PREC_FP32_SPLIT = 2   /* every GEMM in fp32 by an exact 3-way bf16 split of both
                                   operands (x = hi + mid + lo) and the six bf16 MFMA
                                   products a_i b_j with i + j <= 2, fp32 accumulation:
                                   fp32-accurate (the dropped terms are < 2^-22 |a b|)  */
};

/* Descriptor element types of the _dt entry points (ABI 4).  The reference upcasts every
 * descriptor input with .float() (GATs_SuperGlue.py:219-221); an fp16 input is converted as it
 * is loaded, so the results are those of the fp32 path on the upcast inputs, bit for bit, and
 * the inputs (the object's leaves above all) take half the bytes in HBM. */
enum { ONEPOSE_DT_F32 = 0, ONEPOSE_DT_F16 = 1 };

/* Thread-local description of the last error ("" when none). */
const char* onepose_last_error(void);
/* ABI version, bumped on any signature change or new entry point (4: the per-precision
 * workspace and object-cache size queries; 5: the object cache's device-side header and
 * onepose_device_errors; 6: onepose_match_cached_stages). */
int onepose_abi_version(void);
/* (ABI 5) The library's sticky device-side error bits (ONEPOSE_DEVERR_*), set by kernels that
 * cannot return a status: *bits receives them, and `clear` != 0 resets them.  Synchronises with
 * the device (a host query; never call it inside a graph capture). */
enum {
  ONEPOSE_DEVERR_STALE_CACHE = 1   /* a cached forward found its object cache's header not the
                                    * one onepose_object_prepare wrote there (the memory was
                                    * freed and reused); that forward reported no match */
};
int onepose_device_errors(int clear, unsigned* bits);

/* ------------------------------------------------------------------------------------ *
 * GATsSPG matcher  --  replaces GATsSuperGlue.forward
 *   (src/models/GATsSPG_architectures/GATs_SuperGlue.py:203-278, reached from
 *    LitModelGATsSPG.forward, src/models/GATsSPG_lightning_model.py:36-37, and
 *    inference.py:146)
 * ------------------------------------------------------------------------------------ */

/* Number of weight tensors the packer consumes, and the reference state-dict key of
 * tensor i (e.g. "gnn.layers.1.attn.proj.0.weight").  The unused kenc_2d / kenc_3d /
 * bin_score entries (never read by forward, GATs_SuperGlue.py:172-201) are not listed. */
int onepose_matcher_num_tensors(void);
const char* onepose_matcher_tensor_name(int i);
/* Element count tensor i must have. */
int64_t onepose_matcher_tensor_numel(int i);

/* Bytes of the packed weight panel. */
size_t onepose_matcher_packed_bytes(void);

/* Pack the float32 host tensors (in onepose_matcher_tensor_name order) into the
 * device-ready panel `packed_host` (onepose_matcher_packed_bytes() bytes, host memory).
 * Packing permutes the q/k/v projections to head-major channel order, folds the GAT
 * attention vectors through W (h.(W a) == (h W).a, GATs.py:68-69,113-115) and lays the
 * matrices out as [out][in].  Upload the panel to the device once; it is read-only. */
int onepose_matcher_pack(const float* const* tensors, int n_tensors, void* packed_host);

/* Workspace bytes onepose_match needs for this shape.  with_conf=0 adds room for the
 * score matrix that would otherwise live in `conf`. */
size_t onepose_match_workspace_bytes(int batch, int n1, int n3, int num_leaf, int with_conf);
/* (ABI 4) The same for one precision: fp32 needs no bf16 activation planes, so its workspace
 * is smaller (the query above is the largest over precisions and stays valid for all).  A
 * match call checks `workspace_bytes` against its own precision's need. */
size_t onepose_match_workspace_bytes_ex(int batch, int n1, int n3, int num_leaf, int with_conf,
                                        int precision);

/* One matcher forward over `batch` frames.
 *   desc2d  [batch, 256, n1]        descriptors2d_query  (device, fp32)
 *   desc3d  [batch, 256, n3]        descriptors3d_db     (device; bstride may be 0)
 *   leaves  [batch, 256, n3*L]      descriptors2d_db     (device; bstride may be 0)
 *   outputs matches0 [batch, n1] int64, matches1 [batch, n3] int64,
 *           mscores0 [batch, n1] fp32, mscores1 [batch, n3] fp32,
 *           conf [batch, n1, n3] fp32 or NULL (conf_matrix).
 * Batch strides are in elements.  n1, n3 >= 1 (the empty-input branch of
 * GATs_SuperGlue.py:223-231 is handled by the caller).  1 <= num_leaf <= 16. */
int onepose_match(const void* packed_weights,
                  const float* desc2d, int64_t desc2d_bstride,
                  const float* desc3d, int64_t desc3d_bstride,
                  const float* leaves, int64_t leaves_bstride,
                  int batch, int n1, int n3, int num_leaf,
                  float scale_factor, float match_threshold,
                  int64_t* matches0, int64_t* matches1,
                  float* mscores0, float* mscores1, float* conf,
                  void* workspace, size_t workspace_bytes, void* stream);

/* Per-object leaf preparation.  The GAT layers read the leaves point-major
 * ([n3][num_leaf][256]: one 3D point's leaves contiguous) -- onepose_match transposes its
 * reference-layout input into the workspace on every call; a caller that keeps one object
 * resident across frames (inference.py:89-90 uploads it per frame) can transpose once with
 * onepose_prepare_leaves and call onepose_match_prepared.
 *   leaves [batch, 256, n3*L] (bstride elements)  ->  out [batch, n3*L, 256]
 * onepose_match_prepared takes the same arguments as onepose_match with the prepared leaves
 * (prepared_bstride elements per sample, 0 = shared) and the same workspace size. */
size_t onepose_leaves_prepared_bytes(int batch, int n3, int num_leaf);
int onepose_prepare_leaves(const float* leaves, int64_t leaves_bstride, int batch, int n3,
                           int num_leaf, float* out, void* stream);
/* (ABI 4) leaves of `dtype` (ONEPOSE_DT_*); the prepared copy is fp32. */
int onepose_prepare_leaves_dt(const void* leaves, int dtype, int64_t leaves_bstride, int batch,
                              int n3, int num_leaf, float* out, void* stream);
/* The same two calls with a precision mode (ONEPOSE_PREC_*); the plain forms are
 * ONEPOSE_PREC_FP32. */
int onepose_match_ex(const void* packed_weights,
                     const float* desc2d, int64_t desc2d_bstride,
                     const float* desc3d, int64_t desc3d_bstride,
                     const float* leaves, int64_t leaves_bstride,
                     int batch, int n1, int n3, int num_leaf,
                     float scale_factor, float match_threshold, int precision,
                     int64_t* matches0, int64_t* matches1,
                     float* mscores0, float* mscores1, float* conf,
                     void* workspace, size_t workspace_bytes, void* stream);
/* (ABI 4) onepose_match_ex with desc2d, desc3d and leaves of `desc_dtype` (ONEPOSE_DT_*). */
int onepose_match_dt(const void* packed_weights,
                     const void* desc2d, int64_t desc2d_bstride,
                     const void* desc3d, int64_t desc3d_bstride,
                     const void* leaves, int64_t leaves_bstride, int desc_dtype,
                     int batch, int n1, int n3, int num_leaf,
                     float scale_factor, float match_threshold, int precision,
                     int64_t* matches0, int64_t* matches1,
                     float* mscores0, float* mscores1, float* conf,
                     void* workspace, size_t workspace_bytes, void* stream);
int onepose_match_prepared_ex(const void* packed_weights,
                              const float* desc2d, int64_t desc2d_bstride,
                              const float* desc3d, int64_t desc3d_bstride,
                              const float* leaves_prepared, int64_t prepared_bstride,
                              int batch, int n1, int n3, int num_leaf,
                              float scale_factor, float match_threshold, int precision,
                              int64_t* matches0, int64_t* matches1,
                              float* mscores0, float* mscores1, float* conf,
                              void* workspace, size_t workspace_bytes, void* stream);
int onepose_match_prepared(const void* packed_weights,
                           const float* desc2d, int64_t desc2d_bstride,
                           const float* desc3d, int64_t desc3d_bstride,
                           const float* leaves_prepared, int64_t prepared_bstride,
                           int batch, int n1, int n3, int num_leaf,
                           float scale_factor, float match_threshold,
                           int64_t* matches0, int64_t* matches1,
                           float* mscores0, float* mscores1, float* conf,
                           void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------ *
 * Per-object cache (SURVEY.md §8b ops_object_prepare, §8f rank 2).  Two parts of the forward
 * depend on the object alone: GAT layer 0 (GATs.py:62-123, the 3D descriptors and their
 * leaves) and the 3D half of self-attention 1 (GATs_SuperGlue.py:67-85 -- the 3D side attends
 * only to itself there).  onepose_object_prepare runs them once per object and leaves the
 * 3D state entering layer 2 in `cache` ([n3][256] fp32), followed by the leaf logits
 * leaf_j . (W a)_lo of GAT layers 1-3 ([3][n3][16] fp32; GATs.py:113, constant per object since
 * the leaves never change, GATs_SuperGlue.py:70-72) and by cross-attention 1's frame-
 * independent 3D half (layer 2, GATs_SuperGlue.py:74-78: the 3D side's phi(q), sum phi(k), the
 * 2D side's folded message weights and the W1a x half of its MLP conv 1) --
 * onepose_object_cache_bytes in all (an opaque layout); onepose_match_cached then runs every
 * frame from there.
 *
 * `flags` (ONEPOSE_OBJ_*) fix the cache's layout and contents at prepare time; pass the same
 * value to onepose_object_cache_bytes and onepose_match_cached.  With ONEPOSE_OBJ_GAT_TABLES and
 * num_leaf <= 8 the cache also holds prefix tables of GAT layers 1-3 (the leaves sorted by
 * logit, exp-weighted prefix and suffix sums: [3][n3][2 num_leaf][256] fp32 plus [3][n3][16]
 * sorted logits, i.e. 6 KB x num_leaf + 192 B per 3D point: 202 MB at n3 = 4096, L = 8), and a
 * cached frame's GAT layers 1-3 read two table rows per 3D point instead of its L leaves; they
 * then differ from computing the layers from the leaves in rounding only.  Without it (flags
 * 0; the tables are never built for num_leaf > 8) the results are bit-identical to
 * onepose_match_prepared_ex's on the same object (the same kernels and tiles produce the cached
 * state), provided the cache was prepared with the same `precision`.  Without tables the cache
 * is 4 KB + 192 B per 3D point (17.6 MB at n3 = 4096) plus a 0.75 MB fixed part.
 *   desc3d:          [256][n3] reference layout (descriptors3d_db of one object)
 *   leaves_prepared: [n3*L][256] point-major (onepose_prepare_leaves of the object)
 * The cache is shared by every sample of a batch (one object per call); it is read-only for
 * onepose_match_cached, so any number of streams may use one cache concurrently.
 *
 * The library records, per cache address, the (n3, num_leaf, precision, flags) that
 * onepose_object_prepare built it with (host-side; nothing is read back from the device).
 * onepose_match_cached returns ONEPOSE_ERR_INVALID for a cache it has no record of, or whose
 * record differs from its own arguments: the layout depends on n3, num_leaf and flags, and
 * the folded Mf weights are fp32 for ONEPOSE_PREC_FP32 and bf16 planes for the other
 * precisions, so a mismatched call would read the wrong bytes. A copy of a cache at another
 * address is therefore refused; prepare it there instead. onepose_object_release forgets a
 * cache's record (call it before the memory is freed, if the allocator may hand the address
 * to another cache that is not prepared again); a new onepose_object_prepare at the same
 * address replaces the record. onepose_object_cache_bytes returns 0 for flags that prepare
 * would refuse.
 * (ABI 5) The record cannot see memory that was freed and handed to something else at the
 * same address without onepose_object_release.  So the prepare also writes a 64-B header at
 * the end of the cache (its n3, num_leaf, precision, flags and a generation the record keeps),
 * and onepose_match_cached's first kernel compares it with the record on the device: a
 * mismatch makes that forward report no match (matches -1, scores 0) and sets
 * ONEPOSE_DEVERR_STALE_CACHE (onepose_device_errors) -- without a host synchronisation, so
 * graph-captured forwards keep the check.
 * ------------------------------------------------------------------------------------ */
enum {
  ONEPOSE_OBJ_GAT_TABLES = 1    /* build / use the GAT prefix tables (num_leaf <= 8)          */
};
size_t onepose_object_cache_bytes(int n3, int num_leaf, int flags);
/* (ABI 4) The cache bytes for one precision: the bf16 activation planes of the cached phi(q)
 * (1.5 KB per point) only in the bf16 modes.  A cache sized by this query must be prepared and
 * matched with that precision; onepose_object_cache_bytes fits every precision. */
size_t onepose_object_cache_bytes_ex(int n3, int num_leaf, int flags, int precision);
size_t onepose_object_prepare_workspace_bytes(int n3, int num_leaf);
int onepose_object_prepare(const void* packed_weights, const float* desc3d,
                           const float* leaves_prepared, int n3, int num_leaf, int precision,
                           int flags, float* cache, void* workspace, size_t workspace_bytes,
                           void* stream);
/* (ABI 4) desc3d [256, n3] of `desc_dtype` (ONEPOSE_DT_*). */
int onepose_object_prepare_dt(const void* packed_weights, const void* desc3d, int desc_dtype,
                              const float* leaves_prepared, int n3, int num_leaf, int precision,
                              int flags, float* cache, void* workspace, size_t workspace_bytes,
                              void* stream);
void onepose_object_release(const float* cache);
/* Workspace: onepose_match_workspace_bytes(batch, n1, n3, num_leaf, conf != NULL). */
int onepose_match_cached(const void* packed_weights,
                         const float* desc2d, int64_t desc2d_bstride,
                         const float* object_cache,
                         const float* leaves_prepared, int64_t prepared_bstride,
                         int batch, int n1, int n3, int num_leaf,
                         float scale_factor, float match_threshold, int precision,
                         int object_flags,
                         int64_t* matches0, int64_t* matches1,
                         float* mscores0, float* mscores1, float* conf,
                         void* workspace, size_t workspace_bytes, void* stream);
/* (ABI 4) desc2d [batch, 256, n1] of `desc_dtype` (ONEPOSE_DT_*). */
int onepose_match_cached_dt(const void* packed_weights,
                            const void* desc2d, int desc_dtype, int64_t desc2d_bstride,
                            const float* object_cache,
                            const float* leaves_prepared, int64_t prepared_bstride,
                            int batch, int n1, int n3, int num_leaf,
                            float scale_factor, float match_threshold, int precision,
                            int object_flags,
                            int64_t* matches0, int64_t* matches1,
                            float* mscores0, float* mscores1, float* conf,
                            void* workspace, size_t workspace_bytes, void* stream);
/* (ABI 6) onepose_match_cached_dt as a range of its stages, for a caller that pipelines frames
 * through buffer slots (one workspace per slot) and wants stages off the matcher's launch
 * chain.  The forward's stages, in order:
 *   ONEPOSE_STAGE_INPUTS        its first kernel: desc2d into the workspace's token-major layout,
 *                               the workspace's arrival counters zeroed, the object cache's
 *                               header checked;
 *   ONEPOSE_STAGE_LAYER0 + i    GNN layer i, i = 0..11 of ['GATs', 'self', 'cross'] x 4
 *                               (GATs_SuperGlue.py:184-191; the cached object supplies GAT 0 and
 *                               the 3D half of self-attention 1);
 *   ONEPOSE_STAGE_FINAL         the final projection (+ L2 normalisation) of both sides;
 *   ONEPOSE_STAGE_SCORE         the score GEMM (S and its softmax partials in the workspace, or
 *                               S in `conf`);
 *   ONEPOSE_STAGE_WINNERS       the dual softmax's winners and the mutual check (matches /
 *                               scores, and conf when requested).
 * onepose_match_cached_stages runs stages first_stage..last_stage.  Consecutive ranges of one
 * forward, run in order with the same arguments (on one stream or ordered by events), give the
 * bits of one onepose_match_cached_dt call (the range INPUTS..WINNERS); nothing else may use
 * the workspace in between.  So the input stage may run as soon as the workspace's previous
 * forward has finished -- e.g. on the stream of that forward's pose stage -- and the last
 * stages on the pose stream of their own frame. */
enum { ONEPOSE_STAGE_INPUTS = 0, ONEPOSE_STAGE_LAYER0 = 1, ONEPOSE_STAGE_FINAL = 13,
       ONEPOSE_STAGE_SCORE = 14, ONEPOSE_STAGE_WINNERS = 15 };
int onepose_match_cached_stages(const void* packed_weights,
                                const void* desc2d, int desc_dtype, int64_t desc2d_bstride,
                                const float* object_cache,
                                const float* leaves_prepared, int64_t prepared_bstride,
                                int batch, int n1, int n3, int num_leaf,
                                float scale_factor, float match_threshold, int precision,
                                int object_flags,
                                int64_t* matches0, int64_t* matches1,
                                float* mscores0, float* mscores1, float* conf,
                                void* workspace, size_t workspace_bytes, int first_stage,
                                int last_stage, void* stream);

/* ------------------------------------------------------------------------------------ *
 * N3-sharded single frame (SURVEY.md §8e optional / §8f rank 4): one frame's 3D points split
 * over `world` ranks (one process per GPU), rank r holding points [start_r, start_r + count_r)
 * with start_r = floor(n3_total * r / world) (onepose_shard_range).  Every rank holds the
 * whole 2D side.  Per attention layer the 3D side's KV / sum phi(k) and its InstanceNorm
 * (n, mean, M2) cross ranks; after the score GEMM the row softmax statistics, the row winners
 * and the column winners do -- each as an all-gather of one fixed-size block per rank,
 * merged in rank order on the device.  The caller supplies the exchange buffers (send: one
 * block of xchg_bytes, recv: world blocks) and a callback that, for `bytes_per_rank` <=
 * xchg_bytes, makes recv hold every rank's first `bytes_per_rank` bytes of send (rank-major,
 * block stride = bytes_per_rank) ordered on `stream` (an RCCL all-gather enqueued there, or a
 * synchronous exchange); it returns 0 on success.
 * Inputs: desc2d [batch,256,n1]; desc3d_shard [batch,256,count_r]; the shard's leaves
 * prepared point-major (onepose_prepare_leaves on the shard).  Outputs on every rank, for the
 * whole frame: matches0 / mscores0 [batch,n1], matches1 / mscores1 [batch,n3_total] (indices
 * global); conf_shard [batch,n1,count_r] optional.
 * ------------------------------------------------------------------------------------ */
typedef int (*onepose_allgather_fn)(size_t bytes_per_rank, void* stream, void* user);
void onepose_shard_range(int n3_total, int world, int rank, int* start, int* count);
size_t onepose_match_sharded_xchg_bytes(int batch, int n1, int n3_total, int world);
size_t onepose_match_sharded_workspace_bytes(int batch, int n1, int n3_total, int world, int rank,
                                             int num_leaf, int with_conf);
int onepose_match_sharded(const void* packed_weights,
                          const float* desc2d, int64_t desc2d_bstride,
                          const float* desc3d_shard, int64_t desc3d_bstride,
                          const float* leaves_shard_prepared, int64_t prepared_bstride,
                          int batch, int n1, int n3_total, int num_leaf, int world, int rank,
                          float scale_factor, float match_threshold, int precision,
                          void* xchg_send, void* xchg_recv, size_t xchg_bytes,
                          onepose_allgather_fn allgather, void* user,
                          int64_t* matches0, int64_t* matches1,
                          float* mscores0, float* mscores1, float* conf_shard,
                          void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------ *
 * SuperPoint descriptor sampling  --  replaces sample_descriptors
 *   (src/models/extractors/SuperPoint/superpoint.py:95-113)
 * keypoints [batch, n, 2] (x, y) pixels, dense [batch, c, h, w] -> out [batch, c, n],
 * bilinear, zero padding, L2-normalised over c.  align_corners mirrors the reference's
 * torch-version switch (superpoint.py:108).  All device pointers.
 * ------------------------------------------------------------------------------------ */
int onepose_sample_descriptors(const float* keypoints, const float* dense,
                               int batch, int n, int c, int h, int w, int s,
                               int align_corners, float* out, void* stream);

/* ------------------------------------------------------------------------------------ *
 * Correspondence selection  --  replaces the host-side masking of inference.py:147-152
 *   (valid = matches > -1; mkpts2d = kpts2d[valid]; mkpts3d = kpts3d[matches[valid]])
 * plus the float64 scaling + float32 conversion solvePnPRansac applies to its inputs
 *   (eval_utils.py:22-26).
 * matches0 [batch, n1] int64, kpts2d [batch, n1, 2] fp32, kpts3d [batch, n3, 3] fp32
 * (kpts3d bstride may be 0) -> pts2d [batch, n1, 2], pts3d [batch, n1, 3] fp32 compacted
 * in ascending 2D index order, counts [batch] int32.  All device pointers.
 * ------------------------------------------------------------------------------------ */
int onepose_select_correspondences(const int64_t* matches0, const float* kpts2d,
                                   int64_t kpts2d_bstride, const float* kpts3d,
                                   int64_t kpts3d_bstride, int batch, int n1, int n3,
                                   double scale3d, float* pts2d, float* pts3d, int* counts,
                                   void* stream);

/* ------------------------------------------------------------------------------------ *
 * Batched RANSAC-EPnP  --  replaces ransac_PnP (src/utils/eval_utils.py:18-42), i.e.
 *   cv2.solvePnPRansac(pts3d*scale, pts2d, K, 0, reprojectionError, iterationsCount,
 *                      flags=SOLVEPNP_EPNP) + Rodrigues + tvec/scale,
 * restated after OpenCV 4.4's solvePnPRansac / RANSACPointSetRegistrator / epnp
 * (same cv::RNG stream, same subset rule, same adaptive iteration count, final EPnP refit
 * on the inliers).  One frame per batch entry; frames are independent.
 *   pts2d [batch, max_points, 2], pts3d [batch, max_points, 3] fp32 (already scaled),
 *   counts [batch] int32, K [batch, 9] fp64 row-major (K_bstride may be 0).
 * Outputs: pose34 [batch, 12] fp64 row-major [R | t/scale], inlier_mask
 * [batch, max_points] uint8, n_inliers [batch] int32, status [batch] int32:
 *   0 = solved; 1 = fewer than 4 points (reference: cv2.error -> identity pose, no inliers);
 *   2 = RANSAC found no model (identity pose, no inliers);
 * Exactly 4 points follow solvePnPRansac's P3P branch: the P3P kernel (Gao) decides model / no
 * model (status 2), the pose is the EPnP refit over all four.
 * All device pointers.
 * ------------------------------------------------------------------------------------ */
size_t onepose_pnp_workspace_bytes(int batch, int max_points, int max_iters);
int onepose_pnp_ransac(const float* pts2d, const float* pts3d, const int* counts,
                       int max_points, const double* K, int64_t K_bstride, int batch,
                       double scale, float reproj_error, int max_iters, double confidence,
                       double* pose34, uint8_t* inlier_mask, int* n_inliers, int* status,
                       void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------ *
 * cm/deg pose error  --  replaces query_pose_error (src/utils/eval_utils.py:45-63) and
 * Evaluator.cm_degree_*_metric (src/evaluators/cmd_evaluator.py:11-31).
 * pose_pred [batch, 12], pose_gt [batch, 12] fp64 row-major 3x4 (gt bstride may be 0)
 * -> R_err_deg [batch], t_err_cm [batch] fp64, cmd [batch, 3] uint8 for 1/3/5 cm-deg.
 * ------------------------------------------------------------------------------------ */
int onepose_pose_errors(const double* pose_pred, const double* pose_gt, int64_t gt_bstride,
                        int batch, double* R_err_deg, double* t_err_cm, uint8_t* cmd,
                        void* stream);

/* ------------------------------------------------------------------------------------ *
 * The whole per-frame pose stage in two launches  --  inference.py:147-160 (mkpts selection,
 * ransac_PnP, evaluator.evaluate): onepose_select_correspondences fused into the RANSAC
 * kernel (which compacts the matches straight into its LDS copy of the points) and
 * onepose_pose_errors fused into the refit kernel.  Same results as the three calls, with
 * max_points = n1 (pts2d [batch, n1, 2], pts3d [batch, n1, 3], inlier_mask [batch, n1]).
 * scale multiplies kpts3d (select) and divides the translation (ransac_PnP), as inference.py
 * uses one scale for both.  pose_gt null: no error outputs (R_err_deg / t_err_cm / cmd may
 * be null).  Workspace: onepose_pnp_workspace_bytes(batch, n1, max_iters).
 * ------------------------------------------------------------------------------------ */
int onepose_pose_stage(const int64_t* matches0, const float* kpts2d, int64_t kpts2d_bstride,
                       const float* kpts3d, int64_t kpts3d_bstride, int batch, int n1, int n3,
                       double scale, const double* K, int64_t K_bstride, float reproj_error,
                       int max_iters, double confidence, const double* pose_gt,
                       int64_t gt_bstride, float* pts2d, float* pts3d, int* counts,
                       double* pose34, uint8_t* inlier_mask, int* n_inliers, int* status,
                       double* R_err_deg, double* t_err_cm, uint8_t* cmd, void* workspace,
                       size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------ *
 * SuperPoint keypoint detector + descriptor -- replaces SuperPoint.forward
 * (src/models/extractors/SuperPoint/superpoint.py:170-224; the model extract_features.py:
 * 27-40 builds, nms_radius 3, keypoint_threshold 0.005, remove_borders 4, max_keypoints
 * 4096 there).  Weights: the 24 tensors conv1a.weight, conv1a.bias, ... convDb.bias in
 * onepose_superpoint_tensor_name order, torch layouts ([cout][cin][k][k], [cout]), packed
 * host-side into onepose_superpoint_packed_bytes() bytes (then copied to the device).
 * image [batch][h][w] fp32 in [0,1] (h, w multiples of 8).  Outputs, per sample b:
 *   keypoints [batch][max_keypoints][2] (x, y), scores [batch][max_keypoints],
 *   descriptors [batch][256][max_keypoints], counts [batch] -- the first counts[b] entries
 *   are the reference's keypoints in its order (raster order when at most max_keypoints
 *   survive NMS + threshold + borders, torch.topk's descending order otherwise); the rest
 *   are zero.  score_map [batch][h][w] and dense_desc [batch][h/8][w/8][256] (normalised)
 *   are optional (may be null).  nms_radius <= 8; max_keypoints in [1, 16384], or >= h*w
 * (the reference's -1: every pixel, no top-k).
 * ------------------------------------------------------------------------------------ */
int onepose_superpoint_num_tensors(void);
const char* onepose_superpoint_tensor_name(int i);
size_t onepose_superpoint_packed_bytes(void);
int onepose_superpoint_pack(const float* const* tensors, int n_tensors, void* packed_host);
size_t onepose_superpoint_workspace_bytes(int batch, int h, int w);
int onepose_superpoint(const void* packed, const float* image, int batch, int h, int w,
                       int nms_radius, float keypoint_threshold, int remove_borders,
                       int max_keypoints, int align_corners, float* keypoints, float* scores,
                       float* descriptors, int* counts, float* score_map, float* dense_desc,
                       void* workspace, size_t workspace_bytes, void* stream);
/* The detector's tail alone -- simple_nms, threshold, remove_borders, top_k_keypoints, the
 * (y,x)->(x,y) flip and sample_descriptors (superpoint.py:47-113, 181-243) -- from a score
 * map [batch][h][w] (softmax + pixel shuffle, before NMS) and a normalised dense descriptor
 * map [batch][h/8][w/8][256].  Outputs and limits as onepose_superpoint. */
size_t onepose_superpoint_detect_workspace_bytes(int batch, int h, int w);
int onepose_superpoint_detect(const float* score_map, const float* dense_desc, int batch, int h,
                              int w, int nms_radius, float keypoint_threshold, int remove_borders,
                              int max_keypoints, int align_corners, float* keypoints,
                              float* scores, float* descriptors, int* counts, void* workspace,
                              size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------ *
 * Measurement hook (bench.py's roofline).  While enabled, every launch whose kernel kind
 * is in `kind_mask` (bit k = kind k, names from onepose_profile_kind_name) is bracketed by
 * two HIP events recorded on the launch's own stream.  Host-side state, not for use during
 * graph capture.  _end synchronises and returns, per bracketed launch, its kind and the
 * elapsed milliseconds between its two events.
 * ------------------------------------------------------------------------------------ */
int onepose_profile_begin(uint64_t kind_mask, int capacity);
/* Device-stamp variant, usable inside captured HIP graphs (event brackets are not).  While
 * enabled, each launch of a masked kind that supports stamps (the token GEMMs: kv/q/mlp1/
 * mlp2/final/score) is timed by its own workgroups on the device's constant-rate clock
 * (s_memrealtime): first workgroup start to last workgroup end; the last workgroup adds the
 * duration to a per-kind total and re-arms the slot, so graph replays and repeated launches
 * all accumulate.  Each launch (or captured graph node) draws its own accumulator from a
 * per-kind pool of 256, so launches of one kind may run concurrently.  A graph
 * captured while enabled carries the accumulator address and keeps timing when replayed;
 * calling _begin_device again re-zeroes the accumulators (same addresses).
 * _end_device synchronises the device and returns, per kind k < n_kinds, the number of
 * launches timed and their total milliseconds. */
int onepose_profile_begin_device(uint64_t kind_mask);
int onepose_profile_end_device(int64_t* launches, double* total_ms, int n_kinds);
int onepose_profile_end(int* kinds, float* ms, int capacity, int* count);
const char* onepose_profile_kind_name(int kind);

#ifdef __cplusplus
}
#endif
#endif /* ONEPOSE_HIP_H */
