/* semtsdf_det — detection helpers of the Mask R-CNN producer.
 *
 * The producer (slam-maskrcnn_amd/semtsdf/maskrcnn.py) runs the reference detector's inference graph
 * (Mask_RCNN/mrcnn/model.py MaskRCNN.build, mode "inference") in PyTorch-ROCm; the greedy
 * non-maximum suppression it needs twice per frame (ProposalLayer, model.py:282-334; the per-class
 * NMS of refine_detections_graph, model.py:736-750) is this library's HIP kernel pair.  Separate from
 * libsemtsdf.so: the fusion library's code (and its build key) does not change with the detector.
 *
 * All pointers are device pointers; every call is asynchronous on `stream` (a hipStream_t, NULL: the
 * null stream); int status as in semtsdf.h (0 ok, SEMTSDF_DET_ERR_INVALID on bad arguments). */
#ifndef SEMTSDF_DET_H
#define SEMTSDF_DET_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SEMTSDF_DET_ABI_VERSION 2
#define SEMTSDF_DET_ERR_INVALID 1
#define SEMTSDF_DET_ERR_HIP 2
#define SEMTSDF_DET_MAX_BOXES 16384

int semtsdf_det_abi_version(void);

/* Bytes of device workspace semtsdf_det_nms needs for n boxes. */
size_t semtsdf_det_nms_workspace(int n);

/* Greedy non-maximum suppression of boxes already sorted by descending score, the rule of
 * tf.image.non_max_suppression and of mrcnn/utils.py:116-150 non_max_suppression: box i is kept
 * when no kept box before it overlaps it with IoU > iou_threshold (IoU of (y1, x1, y2, x2) boxes
 * with areas (y2 - y1)(x2 - x1)); at most max_out boxes are kept.
 *   boxes:  [n][4] f32 (y1, x1, y2, x2), sorted by descending score, 0 <= n <= SEMTSDF_DET_MAX_BOXES
 *   keep:   [max_out] int32, the kept indices in order; entries past *count are set to -1
 *   count:  one int32, the number kept
 *   work:   semtsdf_det_nms_workspace(n) bytes */
int semtsdf_det_nms(const float* boxes, int n, float iou_threshold, int max_out, int32_t* keep, int32_t* count,
                    void* work, void* stream);

/* PyramidROIAlign of mrcnn/model.py:374-452 (ABI 2): rois [n][4] f32 (y1, x1, y2, x2) normalised to the
 * image, each sampled on its own level lvl[r] in 2..5 (the caller's level rule, model.py:406-413), at
 * tf.image.crop_and_resize's pool x pool positions y = y1 (H - 1) + i (y2 - y1) (H - 1) / (pool - 1),
 * bilinearly in f32, 0 outside the map (extrapolation value 0).
 *   feats:  the four levels P2..P5, each [C][H[k]][W[k]] contiguous (batch 1, NCHW) in dtype
 *   dtype:  0 fp16, 1 bf16 (the maps' and the output's element type)
 *   out:    [n][C][pool][pool] in dtype */
int semtsdf_det_roi_align(const void* const feats[4], const int H[4], const int W[4], int C, const float* rois,
                          const int32_t* lvl, int n, int pool, int dtype, void* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif
