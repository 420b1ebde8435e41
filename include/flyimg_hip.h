/*
 * flyimg_hip.h -- C-ABI of libflyimg_hip.so, the MI355X (gfx950) image hot
 * path of flyimg.  Plain C: pointers, sizes and PODs only.
 *
 * What each entry point replaces in the reference (v1o/flyimg):
 *
 *   fi_plan / fi_process_batch / fi_process_batch_device
 *       replace ImageProcessor::processNewImage -> generateCommand ->
 *       Processor::execute("convert ...") (src/Core/Processor/
 *       ImageProcessor.php:49-57, :66-110; Processor.php:44-62): the resize
 *       operator (-thumbnail/-resize, :264-272) with its geometry
 *       (generateCropSize :138-148 / generateSimpleSize :154-162),
 *       -gravity/-extent (c_1), -colorspace Gray (clsp_Gray, :88),
 *       -rotate (forwarded option, :303-315), and -- when FI_SMARTCROP is set --
 *       SmartCropProcessor::smartCrop (SmartCropProcessor.php:21-36: the
 *       python3 smartcrop.py exec plus the "convert -crop" exec).
 *   fi_smartcrop / fi_smartcrop_ex
 *       replace SmartCrop().crop(...) of python/smartcrop.py:137-191 (the
 *       ctypes path of the drop-in smartcrop CLI, smartcrop.py:341-377).
 *
 * Error convention (Processor.php:53-59 throws ExecFailedException on a
 * non-zero exit): every call returns FI_OK (0) or a negative FI_E* code and
 * fi_last_error() returns the thread-local message of the last failure.
 * The PHP FFI shim maps a non-zero return to ExecFailedException; the Python
 * shim maps FI_ENOCROP to ValueError (smartcrop.py:227-228) and the rest to
 * RuntimeError.
 *
 * Ownership: host buffers are caller-owned; device memory, pinned staging and
 * tap tables are owned by the fi_ctx.  Threading: calls on one fi_ctx are
 * serialised by an internal mutex.  One fi_ctx per process per GPU (one
 * process per GPU; torch.distributed-style launch).
 */
#ifndef FLYIMG_HIP_H
#define FLYIMG_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FI_ABI_VERSION 2  /* 2: forwarded convolution operators (unsharp/sharpen/blur fields) */

/* ---- status codes ---------------------------------------------------- */
#define FI_OK 0
#define FI_EINVAL (-1)       /* bad argument / geometry                     */
#define FI_ENOCROP (-2)      /* smartcrop.py crops(): ValueError (:227-228) */
#define FI_ENOMEM (-3)       /* host or device allocation failed            */
#define FI_EDEVICE (-4)      /* HIP runtime / kernel error                  */
#define FI_EUNSUPPORTED (-5) /* operator not implemented on this path       */
#define FI_ECAPACITY (-6)    /* dst_capacity too small (see fi_plan)        */

/* ---- per-image operator flags (mirror the convert argv) --------------- */
#define FI_OP_THUMBNAIL (1u << 0)      /* -thumbnail (default, ImageProcessor.php:269)   */
#define FI_OP_RESIZE (1u << 1)         /* -resize (rz_1)                                  */
#define FI_GEOM_FILL (1u << 2)         /* '^' geometry flag (generateCropSize :143)       */
#define FI_GEOM_SHRINK_ONLY (1u << 3)  /* '>' geometry flag (generateSimpleSize :159)     */
#define FI_OP_EXTENT (1u << 4)         /* -gravity G -extent WxH (c_1, :144-145)          */
#define FI_OP_GRAY (1u << 5)           /* -colorspace Gray (clsp_Gray, :88)               */
#define FI_OP_MONOCHROME (1u << 6)     /* -monochrome (mnchr_1, :90-92); implies Gray      */
#define FI_OP_ROTATE (1u << 7)         /* -rotate <deg>, multiples of 90 (r_90, :306)     */
#define FI_OP_SMARTCROP (1u << 8)      /* compute smartcrop.py's box on the result (smc_1) */
#define FI_OP_SMARTCROP_APPLY (1u << 9) /* and crop to it (SmartCropProcessor.php:30-34)   */
/* forwarded convolutions (ImageProcessor.php:303-315), after -rotate, in this order: */
#define FI_OP_UNSHARP (1u << 10)       /* -unsharp RxS+gain+threshold (unsh_)               */
#define FI_OP_SHARPEN (1u << 11)       /* -sharpen RxS (sh_)                                */
#define FI_OP_BLUR (1u << 12)          /* -blur RxS (blr_)                                  */
/* The source is an IM PseudoClass image (palette PNG/GIF, 8-bit gray PNG,
 * 1-component JPEG -- IM's readers give them a colormap): ResizeImage's
 * default filter is then Mitchell, not Lanczos (resize.c). */
#define FI_SRC_PSEUDOCLASS (1u << 13)

/* ImageMagick GravityType values used by -gravity (parameters.yml:99). */
#define FI_GRAVITY_NORTHWEST 1
#define FI_GRAVITY_NORTH 2
#define FI_GRAVITY_NORTHEAST 3
#define FI_GRAVITY_WEST 4
#define FI_GRAVITY_CENTER 5
#define FI_GRAVITY_EAST 6
#define FI_GRAVITY_SOUTHWEST 7
#define FI_GRAVITY_SOUTH 8
#define FI_GRAVITY_SOUTHEAST 9

/* One image of a batch.  Caller fills the inputs; the library fills the
 * "filled by library" fields.  For fi_process_batch the pointers are host
 * pointers; for fi_process_batch_device they are device pointers. */
typedef struct fi_image {
  const uint8_t *src;      /* HWC RGB8, or RGBA8 (straight alpha)             */
  int32_t src_w, src_h;    /* pixels                                          */
  int32_t src_stride;      /* bytes per row                                   */
  int32_t src_channels;    /* 3, or 4: an IM matte image (PNG with alpha) --   *
                            * Mitchell, alpha-weighted passes (resize.c), out *
                            * RGBA8 or gray+alpha (2); no smartcrop / mono    */
  int32_t target_w;        /* geometry W (0 = absent, getDimensions :240-259) */
  int32_t target_h;        /* geometry H (0 = absent)                         */
  uint32_t flags;          /* FI_OP_* | FI_GEOM_*                             */
  int32_t gravity;         /* FI_GRAVITY_*, 0 = Center                        */
  int32_t rotate;          /* degrees for FI_OP_ROTATE (multiple of 90)       */
  int32_t smartcrop_w;     /* smartcrop.py --width  (0 = 100, CLI default)    */
  int32_t smartcrop_h;     /* smartcrop.py --height (0 = 100)                 */
  uint8_t *dst;            /* output pixels, HWC, out_stride bytes per row    */
  int64_t dst_capacity;    /* bytes available at dst                          */
  /* ---- filled by library ---- */
  int32_t out_w, out_h, out_channels, out_stride;
  int32_t crop_x, crop_y, crop_w, crop_h; /* smartcrop top_crop (smartcrop.py:184-190 rescaled) */
  double crop_score;                      /* top_crop["score"]["total"]           */
  int32_t status;                         /* FI_OK or FI_E* for this image        */
  int32_t n_candidates;                   /* crops re-scored exactly (diagnostic) */
  /* ---- inputs of the forwarded convolutions (ABI 2), IM ParseGeometry values ---- */
  double unsharp[4];       /* radius, sigma (1), gain (1), threshold (0.05) -- FI_OP_UNSHARP */
  double sharpen[2];       /* radius, sigma (1)                             -- FI_OP_SHARPEN */
  double blur[2];          /* radius, sigma (1)                             -- FI_OP_BLUR    */
} fi_image;

/* SmartCrop.__init__ keyword arguments (python/smartcrop.py:41-77). */
typedef struct fi_smartcrop_params {
  double detail_weight;             /* 0.2  */
  double edge_radius;               /* 0.4  */
  double edge_weight;               /* -10  */
  double outside_importance;        /* -0.5 */
  int32_t rule_of_thirds;           /* 1    */
  double saturation_bias;           /* 0.2  */
  double saturation_brightness_max; /* 0.9  */
  double saturation_brightness_min; /* 0.05 */
  double saturation_threshold;      /* 0.4  */
  double saturation_weight;         /* 0.3  */
  int32_t score_down_sample;        /* 1 (only 1 is supported)  */
  double skin_bias;                 /* 0.01 */
  double skin_brightness_max;       /* 1    */
  double skin_brightness_min;       /* 0.2  */
  double skin_color[3];             /* 0.78, 0.57, 0.44 */
  double skin_threshold;            /* 0.8  */
  double skin_weight;               /* 1.8  */
} fi_smartcrop_params;

/* SmartCrop.crop() keyword arguments (smartcrop.py:137-147). */
typedef struct fi_smartcrop_options {
  int32_t prescale;   /* 1 */
  double max_scale;   /* 1 */
  double min_scale;   /* 0.9 */
  double scale_step;  /* 0.1 */
  int32_t step;       /* 8 */
  int32_t exact_all;  /* 1 = score every crop with the reference's sequential sum */
} fi_smartcrop_options;

/* One entry of result["crops"] (smartcrop.py:184-190, score :300-338). */
typedef struct fi_crop_score {
  int32_t x, y, width, height;      /* rescaled ints (crop() :184-190)                  */
  double fx, fy, fw, fh;            /* analysed-image geometry before rescale           */
  double detail, saturation, skin, total; /* exact when `exact` != 0                   */
  int32_t exact;                    /* 1: sequential reference sum; 0: fast-pass value */
  int32_t pad;
} fi_crop_score;

typedef struct fi_ctx fi_ctx;

int32_t fi_abi_version(void);
const char *fi_last_error(void);

/* Devices and contexts. device = HIP ordinal (one process per GPU). */
int fi_device_count(int32_t *count);
int fi_create(fi_ctx **out, int32_t device);
void fi_destroy(fi_ctx *ctx);

/* Geometry only (no pixel work, no GPU): fills out_w/out_h/out_channels/
 * out_stride for each image; status per image.  Returns FI_OK if all ok. */
int fi_plan(fi_image *imgs, int32_t n);
/* Per-image algorithmic HBM bytes of the hot path (SURVEY.md 8(d)/(e)
 * B_img = R_touched * W_in * C_in + out_w * out_h * out_c + 16 when
 * FI_OP_SMARTCROP), R_touched = source rows with a non-zero vertical tap
 * after the ThumbnailImage sample step.  The multi-GPU sharder balances
 * these (greedy LPT).  bytes[i] = -1 for an image that does not plan. */
int fi_plan_bytes(const fi_image *imgs, int32_t n, int64_t *bytes);

/* Face-blur pixelation (FaceDetectProcessor::blurFaces,
 * FaceDetectProcessor.php:58-74): for each box (x, y, w, h) in order -- the
 * facedetect output lines "x y w h" -- the effect of
 *   mogrify -gravity NorthWest -region WxH+X+Y -scale 10% -scale 1000% <img>
 * on an 8-bit HWC image (channels 1 or 3), in place.  FI_EINVAL for a box
 * outside the image or whose 10% scale is empty (IM: NegativeOrZeroImageSize);
 * boxes before it are applied.  Host buffer (synchronous) and device-resident
 * forms (img on ctx's device, stream-ordered after earlier batches). */
int fi_pixelate_regions(fi_ctx *ctx, uint8_t *img, int32_t w, int32_t h, int32_t stride, int32_t channels,
                        const int32_t *boxes, int32_t nboxes);
int fi_pixelate_regions_device(fi_ctx *ctx, uint8_t *img, int32_t w, int32_t h, int32_t stride, int32_t channels,
                               const int32_t *boxes, int32_t nboxes);

/* Host buffers: H2D -> kernels -> D2H.  Synchronous. */
int fi_process_batch(fi_ctx *ctx, fi_image *imgs, int32_t n);
/* Asynchronous form of fi_process_batch: sources are staged to the device
 * and the batch is queued; outputs and records are final after fi_wait.
 * Three batches can be in flight (the next one's staging and upload overlap the
 * earlier ones' kernels).  Sources and outputs in pinned memory
 * (fi_host_alloc) are copied by DMA directly; pageable ones go through the
 * library's pinned staging.  imgs and the buffers must stay valid until
 * fi_wait returns for this batch. */
int fi_submit_batch(fi_ctx *ctx, fi_image *imgs, int32_t n);
/* Pinned host memory for decode targets and outputs of fi_submit_batch. */
void *fi_host_alloc(fi_ctx *ctx, size_t bytes);
int fi_host_free(fi_ctx *ctx, void *p);
/* Device-resident buffers (src/dst are device pointers on ctx's device).
 * Synchronous; the timed kernels are recorded in fi_kernel_stats. */
int fi_process_batch_device(fi_ctx *ctx, fi_image *imgs, int32_t n);
/* Asynchronous form of fi_process_batch_device for pipelined serving: plans,
 * uploads and launches the batch, then returns; `imgs` must stay valid until
 * fi_wait().  Batch k+1 is planned and uploaded on the host while batch k runs
 * on the GPU (three pinned staging slots; a fourth submit waits for the
 * oldest batch).  Streams: the resample, smartcrop and -monochrome /
 * convolution kernels of every batch run on the context's main stream in
 * submission order; the FI_OP_SMARTCROP_APPLY crop of batch k runs on a
 * second stream beside batch k+1's resample (one small workgroup per CU; with
 * FI_SC_CX=3 the whole smartcrop stage of an eligible batch does), and batch
 * k's records and outputs are final once that apply is done (fi_wait covers it).
 * Ordering across the two streams is kept for the caller: a later batch whose
 * sources overlap an earlier batch's dst, and the device-ordered entry points
 * (fi_pixelate_regions_device, fi_jpeg_decode_device, fi_fill_synthetic) wait
 * for the applies still running.  The dst buffers of two in-flight batches
 * must not overlap (sources may be shared).
 * fi_wait(ctx, keep) finalizes submitted batches in order -- fills their
 * result fields -- until at most `keep` remain in flight (0 = drain all) and
 * returns the first error.  fi_query(ctx, &running) returns, without
 * blocking, how many submitted batches are still running on the GPU. */
int fi_submit_batch_device(fi_ctx *ctx, fi_image *imgs, int32_t n);
int fi_wait(fi_ctx *ctx, int32_t keep);
int fi_query(fi_ctx *ctx, int32_t *running);

/* smartcrop.py SmartCrop().crop(rgb, target_w, target_h) on host RGB8.
 * out_xywh = top_crop x, y, width, height; *out_score = its total. */
void fi_smartcrop_default_params(fi_smartcrop_params *p);
void fi_smartcrop_default_options(fi_smartcrop_options *o);
int fi_smartcrop(fi_ctx *ctx, const uint8_t *rgb, int32_t w, int32_t h, int32_t stride,
                 int32_t target_w, int32_t target_h, const fi_smartcrop_params *params,
                 int32_t out_xywh[4], double *out_score);
/* Full result: every crop, top index, analysed maps (skin, edge, sat HWC) and
 * the prescaled image (both analyse_w*analyse_h*3 bytes, may be NULL). */
int fi_smartcrop_ex(fi_ctx *ctx, const uint8_t *rgb, int32_t w, int32_t h, int32_t stride,
                    int32_t target_w, int32_t target_h, const fi_smartcrop_params *params,
                    const fi_smartcrop_options *opts, fi_crop_score *crops, int32_t crops_cap,
                    int32_t *n_crops, int32_t *top_index, int32_t analyse_wh[2],
                    double *prescale, uint8_t *prescaled_out, uint8_t *maps_out,
                    int64_t out_cap);

/* Device memory and synthetic inputs (device-resident batches / benchmarks). */
int fi_device_malloc(fi_ctx *ctx, void **ptr, uint64_t bytes);
int fi_device_free(fi_ctx *ctx, void *ptr);
int fi_memcpy_h2d(fi_ctx *ctx, void *dst, const void *src, uint64_t bytes);
int fi_memcpy_d2h(fi_ctx *ctx, void *dst, const void *src, uint64_t bytes);
/* Seeded synthetic RGB8 image (flyimg_amd/synth.py bit for bit). */
int fi_fill_synthetic(fi_ctx *ctx, uint8_t *dev, int32_t w, int32_t h, int32_t stride,
                      uint32_t seed);

/* Stage timing (HIP event ranges on the launch streams).  enable: 0 off, 1
 * every stage ("batch", "resize", "sc_prep", "sc_score", "crop_apply", "mono",
 * "conv", "h2d_src", "d2h_out"), 2 the resample stage only (each event range
 * adds a few microseconds between dependent kernels).  fi_kernel_stats also
 * reports host timings ("host_*", "host_total") and per-path image counters
 * ("path_vr", "path_vm", "path_hv", "path_generic_v", "path_generic_h",
 * "path_copy", "sc_path_fd", "sc_path_fz", "sc_path_cx"; "vr_fork": batches
 * whose later k_rs_vr launches ran on the forked stream).  bytes = algorithmic bytes
 * accounted to that stage. */
int fi_set_timing(fi_ctx *ctx, int32_t enable);
int fi_reset_stats(fi_ctx *ctx);
int fi_kernel_stats(fi_ctx *ctx, const char *name, double *total_ms, int64_t *launches,
                    double *bytes);

/* Multi-GPU: the one exchange step is the gather of per-image result
 * records to rank 0 over RCCL (xGMI).  The 128-byte unique id is created by
 * rank 0 and distributed out of band. */
typedef struct fi_record {
  int32_t image, status, out_w, out_h;
  int32_t crop_x, crop_y, crop_w, crop_h;
} fi_record;
int fi_rccl_get_unique_id(uint8_t id[128]);
int fi_rccl_init(fi_ctx *ctx, int32_t rank, int32_t world, const uint8_t id[128]);
/* Every rank sends `count` records (same count on every rank); rank 0
 * receives world*count records in rank order.  The gather runs on a stream
 * of its own (no dependency on the batch streams: the records are host data
 * once fi_wait has filled them).  fi_rccl_gather_start enqueues it and
 * returns (send is copied before it returns; recv is written by the matching
 * fi_rccl_gather_finish, which waits); one gather is in flight at a time (a
 * second start finishes the first).  fi_rccl_gather_records = start +
 * finish.  Every rank issues the same sequence of gathers. */
int fi_rccl_gather_start(fi_ctx *ctx, const fi_record *send, int32_t count, fi_record *recv);
int fi_rccl_gather_finish(fi_ctx *ctx);
int fi_rccl_gather_records(fi_ctx *ctx, const fi_record *send, int32_t count, fi_record *recv);

/* Test hook (not a reference interface): the -monochrome kernels on a
 * caller-supplied Q16 gray image (host buffers), w x h row-major, rotated by
 * rot (0/90/180/270) into out (0/255 bytes).  Lets the parity tests feed the
 * oracle's or_im_monochrome the identical input. */
/* Test hook (not a reference interface): the forwarded convolution kernels
 * (FI_OP_UNSHARP/SHARPEN/BLUR bits 0/1/2 of `ops`, conv = the fi_image
 * unsharp[4], sharpen[2], blur[2] values) on a rotated Q16 HWC image
 * (ch 1 or 3) -> 8-bit out (w * ch bytes per row), so tests can run the
 * oracle's or_im_convolve_ops on the identical input. */
int fi_debug_convolve(fi_ctx *ctx, const uint16_t *q16, int32_t w, int32_t h, int32_t ch, const double conv[8],
                      uint32_t ops, uint8_t *out);
int fi_debug_monochrome(fi_ctx *ctx, const uint16_t *gray, int32_t w, int32_t h, int32_t rot, uint8_t *out,
                        int32_t out_stride);
/* GPU JPEG decode: the decode step of ImageProcessor's `convert` (IM reads
 * the source with libjpeg; ImageProcessor.php:66-110) moved onto the device,
 * bit-exact with libjpeg-turbo's default decompression (islow IDCT, fancy
 * upsampling, YCbCr->RGB).  Baseline / extended sequential Huffman 8-bit
 * streams with one scan: gray, or YCbCr with 4:4:4, 4:2:2 or 4:2:0 chroma.
 * fi_jpeg_info (host only): dimensions and output channels (1 gray, 3 RGB),
 * FI_EUNSUPPORTED for streams to decode on the host (progressive, CMYK, ...).
 * fi_jpeg_decode_device: decodes n streams (host memory) into caller device
 * buffers dst[i] (HWC rows of dst_stride[i] bytes; out_channels 0 = the
 * source's, 3 = RGB for every source, gray replicated) and waits; status[i]
 * per image; returns the first failing status (the others are decoded). */
int fi_jpeg_info(const uint8_t *data, size_t len, int32_t *w, int32_t *h, int32_t *channels);
int fi_jpeg_decode_device(fi_ctx *ctx, const uint8_t *const *data, const size_t *len, int32_t n,
                          uint8_t *const *dst, const int64_t *dst_stride, int32_t out_channels,
                          int32_t *status);

/* Test hook (not a reference interface): the skin / saturation table k_sc_fz
 * reads (2^24 entries, index (r << 16) | (g << 8) | b, value skin | sat << 8)
 * built for `params` (NULL: defaults) and copied to out, so a test can compare
 * every colour with the oracle's detect_skin / detect_saturation. */
int fi_debug_skinsat(fi_ctx *ctx, const fi_smartcrop_params *params, uint16_t *out);

/* Test hook (not a reference interface): the batch planner alone, on the
 * host -- no device: the image pointers are planned, never dereferenced --
 * over `iters` passes of the n images; ms[0..6] += per-stage host
 * milliseconds (images, smartcrop, workspace, vm + vr tiles, of which vr, hv
 * tiles, blob).  One host-only context persists across calls (its caches, as
 * a serving context's): (NULL, 0, ...) drops it, (NULL, 1, ...) clears its
 * statistics, (NULL, 2, 0, ms) reads the resample plan's counters since:
 * ms[0] images planned onto k_rs_vr, ms[1] vertical-first images, ms[2]
 * k_rs_vr launches. */
int fi_debug_host_plan(const fi_image *imgs, int32_t n, int32_t iters, double *ms);

#ifdef __cplusplus
}
#endif
#endif /* FLYIMG_HIP_H */
