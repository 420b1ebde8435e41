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
typedef struct fi_ctx fi_ctx;
int32_t fi_abi_version(void);
const char *fi_last_error(void);
int fi_create(fi_ctx **out, int32_t device);
void fi_destroy(fi_ctx *ctx);
int fi_plan(fi_image *imgs, int32_t n);
int fi_pixelate_regions(fi_ctx *ctx, uint8_t *img, int32_t w, int32_t h, int32_t stride, int32_t channels,
                        const int32_t *boxes, int32_t nboxes);
int fi_process_batch(fi_ctx *ctx, fi_image *imgs, int32_t n);
