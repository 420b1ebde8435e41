/* Preprocessor-free subset of include/flyimg_hip.h for PHP FFI::cdef()
 * (PHP's FFI parser takes no #include/#define).  Keep in sync with the
 * header: tests/test_abi_cpu.py checks every declaration here against it. */
typedef struct fi_image {
  const uint8_t *src;
  int32_t src_w, src_h, src_stride, src_channels;
  int32_t target_w, target_h;
  uint32_t flags;
  int32_t gravity, rotate;
  int32_t smartcrop_w, smartcrop_h;
  uint8_t *dst;
  int64_t dst_capacity;
  int32_t out_w, out_h, out_channels, out_stride;
  int32_t crop_x, crop_y, crop_w, crop_h;
  double crop_score;
  int32_t status, n_candidates;
  double unsharp[4];
  double sharpen[2];
  double blur[2];
} fi_image;
typedef struct fi_smartcrop_params {
  double detail_weight;
  double edge_radius;
  double edge_weight;
  double outside_importance;
  int32_t rule_of_thirds;
  double saturation_bias;
  double saturation_brightness_max;
  double saturation_brightness_min;
  double saturation_threshold;
  double saturation_weight;
  int32_t score_down_sample;
  double skin_bias;
  double skin_brightness_max;
  double skin_brightness_min;
  double skin_color[3];
  double skin_threshold;
  double skin_weight;
} fi_smartcrop_params;
typedef struct fi_ctx fi_ctx;
int32_t fi_abi_version(void);
const char *fi_last_error(void);
int fi_create(fi_ctx **out, int32_t device);
void fi_destroy(fi_ctx *ctx);
int fi_plan(fi_image *imgs, int32_t n);
int fi_pixelate_regions(fi_ctx *ctx, uint8_t *img, int32_t w, int32_t h, int32_t stride, int32_t channels,
                        const int32_t *boxes, int32_t nboxes);
int fi_process_batch(fi_ctx *ctx, fi_image *imgs, int32_t n);
void fi_smartcrop_default_params(fi_smartcrop_params *p);
int fi_smartcrop(fi_ctx *ctx, const uint8_t *rgb, int32_t w, int32_t h, int32_t stride,
                 int32_t target_w, int32_t target_h, const fi_smartcrop_params *params,
                 int32_t out_xywh[4], double *out_score);
