// fi_api.cpp -- the C-ABI runtime of libflyimg_hip.so (include/flyimg_hip.h).
//
// One fi_ctx per process per GPU.  A batch call:
//   1. plans every image on the host (fi_plan.cpp): ImageMagick geometry,
//      merged tap tables, Pillow prescale tables, smartcrop crop windows and
//      importance tables -- deduplicated per geometry and cached across calls;
//   2. packs descriptors + tables into ONE pinned blob and uploads it with
//      one hipMemcpyAsync;
//   3. launches the kernels of each stage once for the whole batch (per-image
//      descriptors, flat tile index -> image by prefix search);
//   4. reads back the per-image result records.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <array>
#include <cstdlib>
#include <cmath>
#include <map>
#include <unordered_map>
#include <queue>
#include <set>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "fi_internal.h"
#include "fi_plan.h"

namespace fi {
// kernels (fi_kernels.hip)
__global__ void k_rs_v_u8(const ResizeDesc *, const int32_t *, int, const int32_t *, const float *);
__global__ void k_rs_h_final(const ResizeDesc *, const int32_t *, int, const int32_t *, const float *);
__global__ void k_rs_h_u8(const ResizeDesc *, const int32_t *, int, const int32_t *, const float *);
__global__ void k_rs_v_final(const ResizeDesc *, const int32_t *, int, const int32_t *, const float *);
__global__ void k_rs_copy(const ResizeDesc *, const int32_t *, int);
__global__ void k_sc_reduce(const ScDesc *, const int32_t *, int);
__global__ void k_sc_hpass(const ScDesc *, const int32_t *, int, const int32_t *);
__global__ void k_sc_vpass(const ScDesc *, const int32_t *, int, const int32_t *);
__global__ void k_sc_maps(const ScDesc *, const int32_t *, int, const ScParamsDev);
// per-image smartcrop kernels (fi_smartcrop.hip)
int launch_sc_h(hipStream_t s, const ScDesc *descs, int n, int chunks, int lds, const int32_t *ai);
int launch_sc_v(hipStream_t s, const ScDesc *descs, int n, int chunks, int lds, const int32_t *ai,
                const ScParamsDev &P);
int launch_sc_vq(hipStream_t s, const ScDesc *descs, int n, int chunks, int lds, const int32_t *ai,
                 const ScParamsDev &P);
int launch_sc_fz(hipStream_t s, const ScDesc *descs, int n, int lds, const int32_t *ai, const ScParamsDev &P,
                 const uint16_t *skinsat);
int launch_sc_fd(hipStream_t s, const ScDesc *descs, int n, int lds, const int32_t *ai, const ScParamsDev &P,
                 const uint16_t *skinsat);
int launch_sc_hx(hipStream_t s, int ks, int nch, const ScDesc *descs, const int32_t *tiles, int ntiles,
                 const int32_t *ai);
int launch_sc_vx(hipStream_t s, int kv, int nch, const ScDesc *descs, const int32_t *tiles, int ntiles,
                 const int32_t *ai, const ScParamsDev &P, const uint16_t *skinsat);
int launch_sc_skinsat(hipStream_t s, uint16_t *table, const ScParamsDev &P);
int jpeg_info(const uint8_t *data, size_t len, int *w, int *h, int *c);
int jpeg_decode_batch(hipStream_t st, const uint8_t *const *data, const size_t *len, int n, uint8_t *const *dst,
                      const int64_t *dst_stride, int out_channels, int32_t *status,
                      void *(*alloc)(void *, int, size_t), void *actx, std::string *err);
int launch_sc_score(hipStream_t s, int mode, const ScDesc *descs, int n, size_t lds, const DevCrop *crops,
                    const double *ad, CropScore *scores, ScResult *results, const ScParamsDev &P, const int32_t *ai);
int launch_sc_score3(hipStream_t s, const ScDesc *descs, int n, size_t lds, const DevCrop *crops, const ScGroup *groups,
                     const double *ad, CropScore *scores, ScResult *results, const ScParamsDev &P, const int32_t *ai);
int launch_crop_apply(hipStream_t s, const ApplyDesc *descs, int n, const DevCrop *crops, const ScResult *results,
                      int persistent_wgs);
__global__ void k_synth(uint8_t *, int, int, int64_t, uint32_t);
// tiled horizontal-first pass 1 (fi_kernels.hip)
constexpr int kHTileRows = 16;  // fi_kernels.hip kHTRows
size_t rs_h_tile_lds(int pitch, int taps);
int launch_conv(hipStream_t s, int mode, const ConvStep *steps, const int32_t *prefix, int n, int tiles,
                const double *ad);
int launch_rs4(hipStream_t s, int mode, const ResizeDesc *d1, const int32_t *p1, int n1, int tiles1,
               const ResizeDesc *d2, const int32_t *p2, int n2, int tiles2, const int32_t *ai, const double *ad);
int launch_rs_h_tile(hipStream_t s, const ResizeDesc *descs, const int32_t *prefix, int n, int tiles,
                     const int32_t *ai, const float *af, int pitch, int taps);
// -monochrome (fi_mono.hip)
size_t mono_lds_bytes();
int launch_mono(hipStream_t s, const MonoDesc *descs, int n, const double *wts);
// streaming exact-integer MFMA resample (fi_vm.hip)
size_t vm_lds_bytes(int vpitch, int nocb, int ks, bool q16);
int vm_read_stamps(uint64_t *out, int slots);
int launch_vm(hipStream_t s, const VDesc *descs, const MStrip *strips, const VTile *tiles, int ntiles,
              const int32_t *ai, size_t lds);
// its persistent block-major form (fi_vr.hip)
VrLayout vr_lds_layout(int vpitch, bool q16, int pbuf);
int launch_vr(hipStream_t s, const VDesc *descs, const MStrip *strips, const VrTile *tiles, int ntiles,
              const int32_t *wginfo, int G, const int32_t *ai, VrLayout L);
int vr_read_stamps(uint64_t *out, int slots);
// streaming exact-integer MFMA resample, horizontal first (fi_hv.hip)
size_t hv_lds_bytes(int pp, int nocb);
int launch_hv(hipStream_t s, const HvDesc *descs, const HvStripD *strips, const HvTile *tiles, int ntiles,
              const int32_t *ai, size_t lds);
// face-blur pixelation (fi_pixelate.hip)
int launch_pix(hipStream_t s, int mode, const PixPass &P, const int32_t *ai, const double *ad);
}  // namespace fi

using namespace fi;

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
static thread_local std::string g_err;
static int set_err(int code, const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess)                                                                      \
      return set_err(FI_EDEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                     __LINE__);                                                                \
  } while (0)

// ---------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------
struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
};
struct Stat {
  double ms = 0;
  int64_t launches = 0;
  double bytes = 0;
};
struct TimedRange {
  std::string name;
  hipEvent_t a, b;
  double bytes;
};

// A host-buffer batch (fi_submit_batch / fi_process_batch): the caller's
// records, the device-side records run_batch fills, and where each output
// goes -- straight into a pinned caller dst, or through the slot's pinned
// staging (pageable dst) with one memcpy at fi_wait.
struct HostIo {
  fi_image *user = nullptr;
  std::vector<fi_image> dev;
  std::vector<size_t> dev_dst_off;  // per image: its device dst in the slot's hio buffer
  std::vector<int64_t> pin_off;     // per image: offset in the slot's pinned staging, -1 = dst is pinned
};
// One in-flight batch (fi_submit_batch[_device]): what fi_wait needs to fill
// the caller's fi_image records once the stream has drained.
struct PendingBatch {
  fi_image *imgs = nullptr;
  int n = 0;
  int slot = 0;
  double t_start = 0;
  std::vector<int> status, sc_of;
  std::vector<std::string> errs;
  std::vector<int> sstatus;
  std::vector<std::string> serrs;
  std::vector<int32_t> crop0;   // per smartcrop item: first crop of its list
  std::vector<fi::DevCrop> crops;
  size_t nres = 0;              // ScResult records in the slot's pinned readback
  bool any_apply = false;
  std::vector<TimedRange> timers;  // this batch's HIP-event ranges
  std::shared_ptr<HostIo> host;    // host-buffer batches only
};
// Pinned host staging of one in-flight batch: the upload blob and the result
// readback.  Two slots: batch k+1 is planned and uploaded while batch k runs.
struct Slot {
  void *blob = nullptr;
  size_t blob_cap = 0;
  void *res = nullptr;
  size_t res_cap = 0;
  hipEvent_t done = nullptr;  // recorded after the batch's last readback (rb_stream for host outputs, else the batch stream)
  hipEvent_t rs_done = nullptr;  // resample stage of the batch done (main stream)
  hipEvent_t up_done = nullptr;  // the batch's sources / blob uploaded (up_stream)
  hipEvent_t sc_end = nullptr;   // the batch's last kernel done (on its tail stream)
  hipEvent_t sc_done = nullptr;  // the batch's smartcrop stage done (sc_stream; the crop apply waits for it)
  hipStream_t tail = nullptr;    // the stream of the batch's last kernel (sc_stream, or ap_stream with the apply)
  uintptr_t ap_lo = 0, ap_hi = 0;  // bytes its overlapped crop apply writes (empty: none pending)
  bool busy = false;
  // device buffers of the in-flight batch: the uploaded blob (descriptors) and
  // the workspace (intermediates, smartcrop scratch, scores, results).  Per
  // slot, because batch k+1's upload and resample run while batch k's
  // smartcrop stage still reads its own.
  DevBuf arena, work;
  // host-buffer batches: device copies of the sources / outputs, and the pinned
  // staging of pageable sources and outputs
  DevBuf hio;
  void *hpin = nullptr;
  size_t hpin_cap = 0;
};
// three batches in flight: with the smartcrop stage beside the next resample,
// batch k's stage finishes after batch k+1's resample, and batch k+2's must
// already be queued behind it (two slots serialise the host on batch k)
constexpr int kSlots = 3;
// hash of the planner's cache keys (tuples / pairs of ints, doubles' bits and
// pointers): the per-image lookups of a mixed batch run in O(1) (a std::map
// over thousands of tables cost ~1 us per lookup in cache misses)
struct KeyHash {
  template <class T>
  static void mix(size_t &h, const T &v) {
    h ^= std::hash<T>()(v) + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
  }
  template <class... A>
  size_t operator()(const std::tuple<A...> &t) const {
    size_t h = 0;
    std::apply([&](const auto &...x) { (mix(h, x), ...); }, t);
    return h;
  }
  template <class A, class B>
  size_t operator()(const std::pair<A, B> &p) const {
    size_t h = 0;
    mix(h, p.first);
    mix(h, p.second);
    return h;
  }
  template <class T>
  size_t operator()(T *p) const {
    size_t h = 0;
    mix(h, (uintptr_t)p);
    return h;
  }
};
template <class K, class V>
using HashMap = std::unordered_map<K, V, KeyHash>;
struct fi_ctx {
  int device = 0;
  Slot slots[kSlots];
  int next_slot = 0;
  std::vector<PendingBatch> inflight;  // submission order
  hipStream_t stream = nullptr;     // upload, resample, mono
  hipStream_t sc_stream = nullptr;  // smartcrop stage + crop apply of a batch (waits for its resample)
  // copies off the kernel streams: batch k+1's uploads run during batch k's
  // kernels, batch k's readback during batch k+1's (the main stream waits for
  // up_done, the readback for sc_end; one slot's buffers per batch)
  hipStream_t up_stream = nullptr, rb_stream = nullptr;
  // the crop apply of batch k beside batch k+1's resample (one workgroup per
  // CU, no LDS: it fits next to k_rs_vr's); FI_APPLY_OVERLAP=0: on sc_stream
  hipStream_t ap_stream = nullptr;
  bool apply_overlap = true;
  // a batch with two or more k_rs_vr launches (mixed strip widths) runs the
  // second and later ones on rs2_stream, forked from and joined back into
  // `stream` inside the resize stage, so each persistent launch's tail (its
  // unevenly loaded workgroups finishing) is filled by the other's workgroups
  // instead of idling the CUs it frees; FI_VR_FORK=0: all on `stream`
  hipStream_t rs2_stream = nullptr;
  hipEvent_t rs_fork = nullptr, rs_join = nullptr;
  bool vr_fork = true;
  // recorded on ap_stream after every overlapped apply: entry points that
  // launch on `stream` and may touch a batch's dst (face-blur, JPEG decode,
  // synthetic fill, a later batch whose sources are an earlier batch's
  // outputs) wait for it (order_after_apply), so the stream order the header
  // promises holds across the two streams
  hipEvent_t ap_tail = nullptr;
  bool ap_pending = false;
  // RCCL record gather: its own stream (no dependency on the batch streams),
  // pinned staging, at most one gather in flight (fi_rccl_gather_start / _finish)
  hipStream_t gx_stream = nullptr;
  hipEvent_t gx_done = nullptr;
  void *gx_pin = nullptr;
  size_t gx_pin_cap = 0;
  bool gx_pending = false;
  fi_record *gx_recv = nullptr;  // caller's receive buffer of the gather in flight (rank 0)
  size_t gx_recv_bytes = 0;
  std::mutex mu;
  DevBuf arena, work, io;
  DevBuf gather;  // RCCL record gather staging
  DevBuf pix;     // face-blur pixelation: lists + 10% scratch
  void *pinned = nullptr;
  size_t pinned_cap = 0;
  bool timing = false;
  std::map<std::string, Stat> stats;
  std::vector<hipEvent_t> event_pool;
  std::vector<TimedRange> pending;
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
  // caches (host planning is deterministic, keyed by geometry)
  HashMap<std::tuple<int, uint64_t, int, int, int, int, int, int>, AxisTable> axis_cache;
  HashMap<std::tuple<int, int, int, int, uint64_t>, ScPlan> sc_cache;
  std::map<std::tuple<uint64_t, uint64_t, int, int, uint64_t>, std::vector<double>> imp_cache;
  bool fast_rs = true;  // FI_FORCE_GENERIC=1: the generic two-pass resample (and smartcrop) kernels only
  bool vr_rs = true;     // images with block-major tables take the persistent k_rs_vr (FI_VR_RS=0: k_rs_vm)
  int vr_nl = 0;         // k_rs_vr loader waves forced (FI_VR_NL=2 / 4; 0: by geometry)
  bool vr_split = true;  // k_rs_vr: one-block strips in a launch of their own (FI_VR_SPLIT=0: one launch)
  bool vr_narrow = true;
  bool up_hostsync = true;  // device batches' blob upload waited for on the host (FI_UP_SYNC=0: by the main stream)  // 48-px strips where 64-px ones would have four blocks (FI_VR_NARROW=0: off)
  int vr_pbuf = 0;       // k_rs_vr plane buffers forced (FI_VR_PBUF=1 / 2; 0: by ring room)
  int vr_max_classes = 1 << 30;  // batches with more vertical tables stay on k_rs_vm (FI_VR_MAX_CLASSES)
  bool vm_lpt = true;      // k_rs_vm tiles: LPT images -> XCDs, longest tiles first (FI_VM_LPT=0: round robin)
  int res_align = 16;      // row pitch alignment of the resized image kept for smartcrop apply (FI_RES_ALIGN)
  bool timing_resize_only = false;  // fi_set_timing(2): stage timing events around the resample only
  int n_cu = 256;        // compute units (k_rs_vr: one persistent workgroup per CU)
  bool sc_fz = true;        // FI_DISABLE_SC_FZ=1: k_sc_hmfma + k_sc_vq instead of the fused k_sc_fz
  bool sc_fd = true;        // FI_SC_FD=0: k_sc_fz instead of its LDS-DMA form k_sc_fd
  // k_sc_hx + k_sc_vx (no LDS, <= 64 VGPRs; gray sources, two-k-step
  // vertical windows): FI_SC_CX=0 never; 1 (default) for the gray images none
  // of k_sc_fd / k_sc_fz takes (cfg5's 400 -> 111, which otherwise
  // runs k_sc_hmfma + k_sc_vmaps); 2 for every image it fits; 3 the same, and a
  // batch whose smartcrop images all take them runs the stage on ap_stream
  // beside the next batch's resample (measured a loss on cfg2: DESIGN.md §3.2)
  int sc_cx = 1;
  bool sc_mf = true;        // FI_SC_MFMA=0: k_sc_score2 (f64 VALU fast pass) instead of k_sc_score3
  DevBuf skinsat;           // k_sc_skinsat table: 2^24 colours x u16, built for skinsat_key's parameters
  DevBuf jpeg[3];           // GPU JPEG decode: upload (compressed data + tables), -, coefficients + planes
  void *jpeg_host = nullptr;  // its pinned staging
  size_t jpeg_host_cap = 0;
  std::string skinsat_key;
  HashMap<const AxisTable *, VmV> vmv_cache;   // ok iff nblk > 0
  HashMap<const AxisTable *, VrV> vrv_cache;   // ok iff nblk > 0
  HashMap<std::pair<const AxisTable *, bool>, MfmaH> vmh_cache; // strips of <= kVmMaxNx px; ok iff !strips.empty()
  HashMap<const AxisTable *, HvV> hvv_cache;  // ok iff nblk > 0
  HashMap<const AxisTable *, HvH> hvh_cache;  // ok iff !strips.empty()
  bool sc_prep = true;  // FI_DISABLE_SC_PREP=1 forces the generic per-row smartcrop kernels
  // Device-resident table heaps: every per-geometry table (tap tables, MFMA
  // fragments, Pillow coefficients, importance tables) is uploaded once and
  // stays at a fixed offset; a batch uploads only the tables it adds.  The
  // heaps are append-only between resets, and a reset only ever happens
  // between batches: work queued earlier on the (in-order) stream has read
  // its tables before any later copy overwrites them.
  struct Heap {
    void *p = nullptr;
    size_t cap = 0, used = 0;  // elements
  };
  Heap heap_i, heap_f, heap_d;  // int32 / float / double
  // absolute heap offsets of placed tables, keyed by the cached host object
  struct ScTabs {
    int32_t hb = 0, hk = 0, hkT = 0, vb = 0, vk = 0;
    int32_t hmB = 0, hmC = 0, hmS0 = 0, vqA = 0, vqC = 0, vqK0 = 0;
    int32_t cxA = -1, cxK0 = -1;
  };
  HashMap<const AxisTable *, DevAxis> axis_at;
  HashMap<const AxisTable *, int32_t> axis_wd_at;  // f64 weights (RGBA path) in heap_d
  HashMap<const ScPlan *, ScTabs> sc_at;
  std::map<std::pair<const std::vector<double> *, int>, std::pair<int32_t, double>> imp_at;
  std::map<std::pair<const std::vector<double> *, int>, std::pair<int32_t, double>> imp2_at;  // importance - oi
  // k_sc_score3 B fragments: (table, nx, nslot, step) -> heap offset + the table's digit sums / q
  std::map<std::tuple<const std::vector<double> *, int, int, int>, std::pair<int32_t, ScoreBTab>> sgb_at;
  HashMap<const VmV *, std::array<int32_t, 8>> vv_at;
  HashMap<const VrV *, std::array<int32_t, 4>> vr_at;    // rows, bmeta, w128, frag
  // horizontal tables placed: the strips' device descriptors (heap offsets
  // resolved) and the k_rs_vm LDS of their widest strip, kept with the
  // placement so a batch copies them contiguously instead of re-deriving them
  // from the (cold) MfmaH per batch
  struct MhPlaced {
    int32_t hwsum = 0, hwsum2 = 0;
    size_t lds8 = 0, lds16 = 0;  // k_rs_vm LDS with an 8-bit / Q16 output tile
    std::vector<MStrip> strips;
  };
  HashMap<const MfmaH *, MhPlaced> mh_at;
  HashMap<const HvV *, std::array<int32_t, 3>> hvv_at;   // k0ks, frag, wsum
  HashMap<const HvH *, std::array<int32_t, 3>> hvh_at;   // w128, frag, s0
  int32_t mono_wts_at = -1;
  bool heap_retry = false;
  bool host_only = false;  // fi_debug_host_plan: planner only, no device (no allocation, no stream)
};

static void sync_streams(fi_ctx *c) {
  if (c->host_only) return;
  (void)hipStreamSynchronize(c->stream);
  if (c->sc_stream != c->stream) (void)hipStreamSynchronize(c->sc_stream);
  if (c->up_stream) (void)hipStreamSynchronize(c->up_stream);
  if (c->rb_stream) (void)hipStreamSynchronize(c->rb_stream);
  if (c->ap_stream) (void)hipStreamSynchronize(c->ap_stream);
  if (c->rs2_stream) (void)hipStreamSynchronize(c->rs2_stream);
  if (c->gx_stream) (void)hipStreamSynchronize(c->gx_stream);
}
// Work about to run on c->stream that may read or write an earlier batch's
// dst waits for the crop applies still running beside it on ap_stream.
static int order_after_apply(fi_ctx *c) {
  if (!c->ap_pending) return FI_OK;
  if (hipStreamWaitEvent(c->stream, c->ap_tail, 0) != hipSuccess) return FI_EDEVICE;
  c->ap_pending = false;
  for (Slot &s : c->slots) s.ap_lo = s.ap_hi = 0;
  return FI_OK;
}
static int ensure(fi_ctx *c, DevBuf *b, size_t bytes) {
  if (b->cap >= bytes) return FI_OK;
  sync_streams(c);  // in-flight batches may still read it
  if (b->p) (void)hipFree(b->p);
  b->p = nullptr;
  b->cap = 0;
  size_t cap = std::max(bytes + bytes / 4, (size_t)1 << 20);
  if (hipMalloc(&b->p, cap) != hipSuccess) {
    b->p = nullptr;
    return set_err(FI_ENOMEM, "hipMalloc(%zu) failed on device %d", cap, c->device);
  }
  b->cap = cap;
  return FI_OK;
}
static int ensure_pinned_buf(void **p, size_t *cap_io, size_t bytes) {
  if (*cap_io >= bytes) return FI_OK;
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  *cap_io = 0;
  size_t cap = std::max(bytes + bytes / 4, (size_t)1 << 16);
  if (hipHostMalloc(p, cap, hipHostMallocDefault) != hipSuccess) {
    *p = nullptr;
    return set_err(FI_ENOMEM, "hipHostMalloc(%zu) failed", cap);
  }
  *cap_io = cap;
  return FI_OK;
}
static int ensure_pinned(fi_ctx *c, size_t bytes) {
  if (c->pinned_cap >= bytes) return FI_OK;
  if (c->pinned) (void)hipHostFree(c->pinned);
  c->pinned = nullptr;
  c->pinned_cap = 0;
  size_t cap = std::max(bytes + bytes / 4, (size_t)1 << 20);
  if (hipHostMalloc(&c->pinned, cap, hipHostMallocDefault) != hipSuccess)
    return set_err(FI_ENOMEM, "hipHostMalloc(%zu) failed", cap);
  c->pinned_cap = cap;
  return FI_OK;
}

static hipEvent_t get_event(fi_ctx *c) {
  if (!c->event_pool.empty()) {
    hipEvent_t e = c->event_pool.back();
    c->event_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  (void)hipEventCreate(&e);
  return e;
}
struct Timer {  // HIP-event range: starts on stream sa, ends on stream sb
  fi_ctx *c;
  TimedRange r;
  bool on;
  hipStream_t sb;
  Timer(fi_ctx *c_, const char *name, double bytes) : Timer(c_, name, bytes, c_->stream, c_->stream) {}
  Timer(fi_ctx *c_, const char *name, double bytes, hipStream_t sa, hipStream_t sb_)
      : c(c_), on(c_->timing && (!c_->timing_resize_only || strcmp(name, "resize") == 0)), sb(sb_) {
    if (!on) return;
    r.name = name;
    r.bytes = bytes;
    r.a = get_event(c);
    r.b = get_event(c);
    (void)hipEventRecord(r.a, sa);
  }
  ~Timer() {
    if (!on) return;
    (void)hipEventRecord(r.b, sb);
    c->pending.push_back(r);
  }
};
static void collect_ranges(fi_ctx *c, std::vector<TimedRange> &ranges) {
  for (auto &r : ranges) {
    float ms = 0;
    (void)hipEventSynchronize(r.b);
    (void)hipEventElapsedTime(&ms, r.a, r.b);
    Stat &s = c->stats[r.name];
    s.ms += ms;
    s.launches += 1;
    s.bytes += r.bytes;
    c->event_pool.push_back(r.a);
    c->event_pool.push_back(r.b);
  }
  ranges.clear();
}
static void collect_timers(fi_ctx *c) { collect_ranges(c, c->pending); }

// ---------------------------------------------------------------------------
// upload blob
// ---------------------------------------------------------------------------
struct Blob {
  std::vector<uint8_t> b;
  size_t add(const void *p, size_t n, size_t align = 256) {
    size_t off = (b.size() + align - 1) / align * align;
    b.resize(off + n);
    if (n) memcpy(b.data() + off, p, n);
    return off;
  }
  template <class T>
  size_t addv(const std::vector<T> &v) {
    return add(v.data(), v.size() * sizeof(T));
  }
};
struct Work {  // workspace sub-allocator (device offsets)
  size_t size = 0;
  size_t take(size_t n, size_t align = 256) {
    size_t off = (size + align - 1) / align * align;
    size = off + n;
    return off;
  }
};

static uint64_t dbits(double d) {
  uint64_t u;
  memcpy(&u, &d, 8);
  return u;
}

static ScParamsDev to_dev(const fi_smartcrop_params &p) {
  ScParamsDev d{};
  d.detail_weight = p.detail_weight;
  d.edge_radius = p.edge_radius;
  d.edge_weight = p.edge_weight;
  d.outside_importance = p.outside_importance;
  d.saturation_bias = p.saturation_bias;
  d.saturation_brightness_max = p.saturation_brightness_max;
  d.saturation_brightness_min = p.saturation_brightness_min;
  d.saturation_threshold = p.saturation_threshold;
  d.saturation_weight = p.saturation_weight;
  d.skin_bias = p.skin_bias;
  d.skin_brightness_max = p.skin_brightness_max;
  d.skin_brightness_min = p.skin_brightness_min;
  for (int i = 0; i < 3; i++) d.skin_color[i] = p.skin_color[i];
  d.skin_threshold = p.skin_threshold;
  d.skin_weight = p.skin_weight;
  d.rule_of_thirds = p.rule_of_thirds;
  return d;
}
static uint64_t params_hash(const fi_smartcrop_params &p) {
  const uint8_t *b = reinterpret_cast<const uint8_t *>(&p);
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < sizeof p; i++) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}

// ---------------------------------------------------------------------------
// batch executor
// ---------------------------------------------------------------------------
struct ScItem {       // one smartcrop job
  const uint8_t *img;  // device
  int64_t stride;
  int W, H, C;
  int tw, th;
  int result;          // index into results
  fi_smartcrop_options opt;
  bool padded = false; // every row readable to fd_rp(W) bytes (library-owned buffers)
};

struct Exec {
  fi_ctx *c;
  Blob blob;
  Work work;
  // tables this batch adds to the device heaps (uploaded behind the heaps'
  // used marks bi / bf / bd, which are multiples of 16 elements)
  std::vector<int32_t> ai;
  std::vector<float> af;
  std::vector<double> ad;
  int64_t bi = 0, bf = 0, bd = 0;
  int32_t oi() const { return (int32_t)(bi + (int64_t)ai.size()); }
  int32_t of() const { return (int32_t)(bf + (int64_t)af.size()); }
  int32_t od() const { return (int32_t)(bd + (int64_t)ad.size()); }
  fi_smartcrop_params params;
};

// ---- device table heaps (fi_ctx::Heap) ------------------------------------
constexpr size_t kHeapI = (size_t)1 << 30, kHeapF = (size_t)128 << 20, kHeapD = (size_t)128 << 20;  // elements
constexpr size_t kAxisCacheMax = 8192, kScCacheMax = 4096, kImpCacheMax = 1024;

static void heap_reset(fi_ctx *c) {
  // work queued on either stream may still read tables the next batch overwrites
  sync_streams(c);
  c->heap_i.used = c->heap_f.used = c->heap_d.used = 0;
  c->axis_at.clear();
  c->axis_wd_at.clear();
  c->sc_at.clear();
  c->imp_at.clear();
  c->imp2_at.clear();
  c->sgb_at.clear();
  c->vv_at.clear();
  c->vr_at.clear();
  c->mh_at.clear();
  c->hvv_at.clear();
  c->hvh_at.clear();
  c->mono_wts_at = -1;
}
// Before a batch places anything: evict oversized host caches (only here, so
// no cached object a batch holds a pointer to is ever freed under it; the
// heap placements keyed by those objects go with them), reset heaps past
// three-quarters full, and hand the batch the heaps' used marks.
static int heap_prepare(fi_ctx *c, Exec &E) {
  if (c->axis_cache.size() > kAxisCacheMax || c->sc_cache.size() > kScCacheMax ||
      c->imp_cache.size() > kImpCacheMax) {
    c->axis_cache.clear();
    c->vmv_cache.clear();
    c->vrv_cache.clear();
    c->vmh_cache.clear();
    c->hvv_cache.clear();
    c->hvh_cache.clear();
    c->sc_cache.clear();
    c->imp_cache.clear();
    heap_reset(c);
  }
  struct H {
    fi_ctx::Heap *h;
    size_t cap, esz;
  } hs[3] = {{&c->heap_i, kHeapI, 4}, {&c->heap_f, kHeapF, 4}, {&c->heap_d, kHeapD, 8}};
  for (auto &x : hs) {
    if (c->host_only) {  // planner timing: offsets only, nothing is written through the heaps
      x.h->cap = x.cap;
      continue;
    }
    if (!x.h->p) {
      if (hipMalloc(&x.h->p, x.cap * x.esz) != hipSuccess) {
        x.h->p = nullptr;
        return set_err(FI_ENOMEM, "hipMalloc(%zu) of the table heap failed on device %d", x.cap * x.esz,
                       c->device);
      }
      x.h->cap = x.cap;
      x.h->used = 0;
    }
  }
  if (c->heap_i.used > c->heap_i.cap / 4 * 3 || c->heap_f.used > c->heap_f.cap / 4 * 3 ||
      c->heap_d.used > c->heap_d.cap / 4 * 3)
    heap_reset(c);
  E.bi = (int64_t)c->heap_i.used;
  E.bf = (int64_t)c->heap_f.used;
  E.bd = (int64_t)c->heap_d.used;
  return FI_OK;
}
static bool heap_fits(const fi_ctx *c, const Exec &E) {
  return (size_t)E.bi + E.ai.size() <= c->heap_i.cap && (size_t)E.bf + E.af.size() <= c->heap_f.cap &&
         (size_t)E.bd + E.ad.size() <= c->heap_d.cap;
}
// Enqueue the copies of the batch's new tables (already uploaded in the blob
// at ab + *_off) behind the heaps' used marks; advance the marks (16-element
// aligned, so 16-byte aligned fragment tables stay aligned).
static int heap_commit(fi_ctx *c, Exec &E, const uint8_t *ab, size_t ai_off, size_t af_off, size_t ad_off) {
  static const bool heap_debug = getenv("FI_HEAP_DEBUG") != nullptr;
  if (heap_debug)
    fprintf(stderr, "heap: ai %zu af %zu ad %zu\n", E.ai.size(), E.af.size(), E.ad.size());
  if (!E.ai.empty())
    HIP_TRY(hipMemcpyAsync((int32_t *)c->heap_i.p + E.bi, ab + ai_off, E.ai.size() * 4, hipMemcpyDeviceToDevice,
                           c->stream));
  if (!E.af.empty())
    HIP_TRY(hipMemcpyAsync((float *)c->heap_f.p + E.bf, ab + af_off, E.af.size() * 4, hipMemcpyDeviceToDevice,
                           c->stream));
  if (!E.ad.empty())
    HIP_TRY(hipMemcpyAsync((double *)c->heap_d.p + E.bd, ab + ad_off, E.ad.size() * 8, hipMemcpyDeviceToDevice,
                           c->stream));
  c->heap_i.used = ((size_t)E.bi + E.ai.size() + 15) / 16 * 16;
  c->heap_f.used = ((size_t)E.bf + E.af.size() + 15) / 16 * 16;
  c->heap_d.used = ((size_t)E.bd + E.ad.size() + 15) / 16 * 16;
  if (c->timing) c->stats["heap_upload"].bytes += (double)(E.ai.size() * 4 + E.af.size() * 4 + E.ad.size() * 8);
  return FI_OK;
}


static const AxisTable *add_axis(fi_ctx *c, Exec &E, int filter, double factor, int in_sampled, int out_size,
                                 int o0, int o1, bool sample, int in_src, DevAxis *out,
                                 HashMap<const AxisTable *, DevAxis> &placed) {
  auto key = std::make_tuple(filter, dbits(factor), in_sampled, out_size, o0, o1, (int)sample, in_src);
  auto it = c->axis_cache.find(key);
  if (it == c->axis_cache.end()) {
    AxisTable t;
    build_axis(filter, factor, in_sampled, out_size, o0, o1, sample, in_src, &t);
    it = c->axis_cache.emplace(key, std::move(t)).first;
  }
  const AxisTable *t = &it->second;
  (void)placed;
  auto pit = c->axis_at.find(t);
  if (pit != c->axis_at.end()) {
    *out = pit->second;
    return t;
  }
  DevAxis d{};
  d.n = (int32_t)t->start.size();
  d.start = E.oi();
  E.ai.insert(E.ai.end(), t->start.begin(), t->start.end());
  d.count = E.oi();
  E.ai.insert(E.ai.end(), t->count.begin(), t->count.end());
  d.woff = E.oi();
  const int32_t wbase = E.of();
  for (int32_t w : t->woff) E.ai.push_back(w + wbase);
  E.af.insert(E.af.end(), t->w.begin(), t->w.end());
  d.maxtaps = t->maxtaps;
  d.src_lo = t->src_lo;
  d.src_hi = t->src_hi;
  d.touched = t->touched;
  d.wbase = wbase;
  d.wd = -1;
  c->axis_at[t] = d;
  *out = d;
  return t;
}


// The f64 weights of an axis (RGBA path), placed in the double heap once.
static void add_axis_f64(fi_ctx *c, Exec &E, const AxisTable *t, DevAxis *d) {
  auto it = c->axis_wd_at.find(t);
  if (it == c->axis_wd_at.end()) {
    const int32_t off = E.od();
    E.ad.insert(E.ad.end(), t->wd.begin(), t->wd.end());
    it = c->axis_wd_at.emplace(t, off).first;
  }
  d->wd = it->second;
}


struct ScLaunchData {
  std::vector<ScDesc> descs;
  std::vector<DevCrop> crops;  // one list per distinct plan, shared by its images
  std::vector<ScGroup> groups; // k_sc_score3 groups, shared like the crops
  int nscores = 0;             // per-image CropScore slots
  std::vector<const ScPlan *> plans;
};

// k_sc_score3 groups of one plan's crops (fi_internal.h ScGroup): per
// importance table, the distinct x origins in chunks of 16 (M rows) times the
// y origins in chunks of kSgSlots (`step` apart: crops() walks a full grid per
// scale).  The plan keeps k_sc_score2 when any condition fails: more than
// kSgMax groups, x origins not 8-B aligned (two ds_read_b64 per fragment),
// windows wider than kSgMaxKs k-steps or of more than 2^17 pixels (int32
// sums of 2^14-bounded products), or planes beyond the LDS.
template <class ImpOf, class Placed>
static void plan_score_groups(fi_ctx *c, Exec &E, const ScPlan &P, int step, const ImpOf &imp_of, ScLaunchData *L,
                              Placed *q) {
  const size_t g0 = L->groups.size();
  std::vector<ScGroup> gs;
  std::vector<std::array<int, 3>> where(P.crops.size(), {-1, -1, -1});
  std::vector<std::pair<uint64_t, uint64_t>> order;
  for (const CropHost &ch : P.crops) {
    const auto k = std::make_pair(dbits(ch.fw), dbits(ch.fh));
    if (std::find(order.begin(), order.end(), k) == order.end()) order.push_back(k);
  }
  int tail = 0;
  for (const auto &k : order) {
    const auto &t = imp_of.at(k);
    const std::vector<double> *tab = std::get<0>(t);
    const int nx = std::get<1>(t), ny = std::get<2>(t);
    if ((int64_t)nx * ny >= (1 << 17)) return;
    std::vector<int> xs, ys;
    for (const CropHost &ch : P.crops)
      if (std::make_pair(dbits(ch.fw), dbits(ch.fh)) == k) {
        xs.push_back(ch.x0);
        ys.push_back(ch.y0);
      }
    std::sort(xs.begin(), xs.end());
    xs.erase(std::unique(xs.begin(), xs.end()), xs.end());
    std::sort(ys.begin(), ys.end());
    ys.erase(std::unique(ys.begin(), ys.end()), ys.end());
    for (size_t i = 1; i < ys.size(); i++)
      if (ys[i] - ys[i - 1] != step) return;
    for (int x : xs)
      if (x % 8) return;
    for (size_t xa = 0; xa < xs.size(); xa += 16)
      for (size_t ya = 0; ya < ys.size(); ya += kSgSlots) {
        const int nm = (int)std::min<size_t>(16, xs.size() - xa), nslot = (int)std::min<size_t>(kSgSlots, ys.size() - ya);
        const auto bk = std::make_tuple(tab, nx, nslot, step);
        auto bt = c->sgb_at.find(bk);
        if (bt == c->sgb_at.end()) {
          ScoreBTab b;
          sc_score_btab(*tab, nx, ny, E.params.outside_importance, nslot, step, &b);
          int32_t off = -1;
          if (b.ok) {
            while (E.ai.size() % 4) E.ai.push_back(0);  // 16-B aligned fragments
            off = E.oi();
            E.ai.insert(E.ai.end(), b.frag.begin(), b.frag.end());
          }
          b.frag.clear();
          bt = c->sgb_at.emplace(bk, std::make_pair(off, std::move(b))).first;
        }
        const ScoreBTab &b = bt->second.second;
        if (!b.ok) return;
        ScGroup g{};
        g.bfrag = bt->second.first;
        g.nrows = b.nrows;
        g.ks = b.ks;
        g.ybase = ys[ya];
        g.nm = nm;
        g.nslot = nslot;
        g.q = b.q;
        g.step = step;
        for (int m = 0; m < 16; m++) g.x0[m] = xs[xa + std::min(m, nm - 1)];
        for (int i = 0; i < kSgDigits; i++) g.S[i] = b.S[i];
        tail = std::max(tail, g.x0[nm - 1] + 64 * g.ks);
        for (size_t ci = 0; ci < P.crops.size(); ci++) {
          const CropHost &ch = P.crops[ci];
          if (std::make_pair(dbits(ch.fw), dbits(ch.fh)) != k) continue;
          const auto xi = std::find(xs.begin() + xa, xs.begin() + xa + nm, ch.x0);
          const int yi = (ch.y0 - ys[ya]) / step;
          if (xi == xs.begin() + xa + nm || ch.y0 < ys[ya] || yi >= nslot) continue;
          where[ci] = {(int)gs.size(), (int)(xi - (xs.begin() + xa)), yi};
        }
        gs.push_back(g);
      }
  }
  if (gs.empty() || (int)gs.size() > kSgMax) return;
  // LDS: the seven planes (rows of sg_pitch(aw) bytes) and what the last row's
  // widest fragment reads past them; the maps (exact re-score) and the
  // cross-wave sums reuse the same space
  const int pitch = sg_pitch(P.aw);
  const int64_t lds = std::max<int64_t>({(int64_t)kSgPlanes * P.ah * pitch + std::max(0, tail - pitch) + 16,
                                         (int64_t)P.aw * P.ah * 4, (int64_t)gs.size() * kSgPlanes * 1024});
  if (lds > kScore3Lds) return;
  for (size_t ci = 0; ci < P.crops.size(); ci++) {
    if (where[ci][0] < 0) return;
    DevCrop &dc = L->crops[q->crop0 + ci];
    dc.sg = where[ci][0];
    dc.sm = where[ci][1];
    dc.sj = where[ci][2];
  }
  q->sg0 = (int32_t)g0;
  q->nsg = (int32_t)gs.size();
  q->sg_lds = (int32_t)((lds + 15) & ~15);
  L->groups.insert(L->groups.end(), gs.begin(), gs.end());
}

// Plan the smartcrop stage of `items` into E (descriptors, crops, tables,
// workspace).  Per-item status in status[].  Images sharing a plan (same
// geometry) share its tables and crop list; `want_pre` keeps the prescaled
// image in the workspace (fi_smartcrop_ex).
static void plan_smartcrop(fi_ctx *c, Exec &E, const std::vector<ScItem> &items, ScLaunchData *L,
                           std::vector<int> *status, std::vector<std::string> *errs, bool want_pre) {
  const uint64_t ph = params_hash(E.params);
  // the fast pass's error bound assumes non-negative per-pixel terms
  const bool fast_ok = E.params.skin_bias >= 0 && E.params.saturation_bias >= 0;
  struct Placed {  // per batch: the plan's crop list in this batch's crop array
    int32_t crop0 = 0, ncrops = 0;
    int32_t sg0 = 0, nsg = 0, sg_lds = 0;  // k_sc_score3 groups (nsg = 0: k_sc_score2)
  };
  std::map<const ScPlan *, Placed> placed;
  for (size_t k = 0; k < items.size(); k++) {
    const ScItem &it = items[k];
    const fi_smartcrop_options &o = it.opt;
    uint64_t okey = dbits(o.max_scale) ^ (dbits(o.min_scale) * 3) ^ (dbits(o.scale_step) * 7) ^
                    ((uint64_t)o.step << 40) ^ ((uint64_t)o.prescale << 56);
    auto key = std::make_tuple(it.W, it.H, it.tw, it.th, okey);
    auto pit = c->sc_cache.find(key);
    if (pit == c->sc_cache.end()) {
      ScPlan p;
      plan_sc(it.W, it.H, it.tw, it.th, o, &p);
      pit = c->sc_cache.emplace(key, std::move(p)).first;
    }
    const ScPlan &P = pit->second;
    L->plans.push_back(&P);
    ScDesc d{};
    d.result = it.result;
    if (P.status != FI_OK) {
      (*status)[k] = P.status;
      (*errs)[k] = P.err;
      L->descs.push_back(d);
      continue;
    }
    auto pp = placed.find(&P);
    if (pp == placed.end()) {
      Placed q;
      auto tp = c->sc_at.find(&P);
      if (tp == c->sc_at.end()) {
        fi_ctx::ScTabs t;
        if (P.thumb) {
          t.hb = E.oi();
          E.ai.insert(E.ai.end(), P.hb.begin(), P.hb.end());
          t.hk = E.oi();
          E.ai.insert(E.ai.end(), P.hk.begin(), P.hk.end());
          t.hkT = E.oi();
          E.ai.insert(E.ai.end(), P.hkT.begin(), P.hkT.end());
          t.vb = E.oi();
          E.ai.insert(E.ai.end(), P.vb.begin(), P.vb.end());
          t.vk = E.oi();
          E.ai.insert(E.ai.end(), P.vk.begin(), P.vk.end());
          if (P.hm_ok) {
            while (E.ai.size() % 4) E.ai.push_back(0);  // 16-B aligned fragments
            t.hmB = E.oi();
            E.ai.insert(E.ai.end(), P.hmB.begin(), P.hmB.end());
            t.hmC = E.oi();
            E.ai.insert(E.ai.end(), P.hmC.begin(), P.hmC.end());
            t.hmS0 = E.oi();
            E.ai.insert(E.ai.end(), P.hmS0.begin(), P.hmS0.end());
          }
          if (P.vq_ok) {
            while (E.ai.size() % 4) E.ai.push_back(0);  // 16-B aligned fragments
            t.vqA = E.oi();
            E.ai.insert(E.ai.end(), P.vqA.begin(), P.vqA.end());
            t.vqK0 = E.oi();
            E.ai.insert(E.ai.end(), P.vqK0.begin(), P.vqK0.end());
          }
          if (P.vq_ok || P.cx_ok) {
            t.vqC = E.oi();
            E.ai.insert(E.ai.end(), P.vqC.begin(), P.vqC.end());
          }
          if (P.cx_ok) {
            while (E.ai.size() % 4) E.ai.push_back(0);  // 16-B aligned fragments
            t.cxA = E.oi();
            E.ai.insert(E.ai.end(), P.cxA.begin(), P.cxA.end());
            t.cxK0 = E.oi();
            E.ai.insert(E.ai.end(), P.cxK0.begin(), P.cxK0.end());
          }
        }
        tp = c->sc_at.emplace(&P, t).first;
      }
      // crops + importance tables (one table per distinct window size)
      std::map<std::pair<uint64_t, uint64_t>, std::pair<int, int>> sizes;
      for (const CropHost &ch : P.crops) {
        auto &e = sizes[{dbits(ch.fw), dbits(ch.fh)}];
        e.first = std::max(e.first, ch.nin_x);
        e.second = std::max(e.second, ch.nin_y);
      }
      std::map<std::pair<uint64_t, uint64_t>, std::tuple<int32_t, int32_t, double>> tab_of;
      std::map<std::pair<uint64_t, uint64_t>, std::pair<int32_t, double>> tab2_of;  // importance - oi
      std::map<std::pair<uint64_t, uint64_t>, std::tuple<const std::vector<double> *, int, int>> imp_of;
      for (auto &sz : sizes) {
        double fw, fh;
        memcpy(&fw, &sz.first.first, 8);
        memcpy(&fh, &sz.first.second, 8);
        const int nx = std::max(sz.second.first, 1), ny = std::max(sz.second.second, 1);
        auto ikey = std::make_tuple(sz.first.first, sz.first.second, nx, ny, ph);
        auto iit = c->imp_cache.find(ikey);
        if (iit == c->imp_cache.end()) {
          std::vector<double> t;
          sc_importance_table(E.params, fw, fh, nx, ny, &t);
          iit = c->imp_cache.emplace(ikey, std::move(t)).first;
        }
        auto pk = std::make_pair(&iit->second, nx);
        auto ip = c->imp_at.find(pk);
        if (ip == c->imp_at.end()) {
          double imax = 0;
          for (double v : iit->second) imax = std::max(imax, std::fabs(v));
          const int32_t off = E.od();
          E.ad.insert(E.ad.end(), iit->second.begin(), iit->second.end());
          ip = c->imp_at.emplace(pk, std::make_pair(off, imax)).first;
        }
        tab_of[sz.first] = std::make_tuple(ip->second.first, nx, ip->second.second);
        // the fast pass weighs inside pixels by fl(importance - oi): the outside
        // ones then need no pass (k_sc_score2)
        auto i2 = c->imp2_at.find(pk);
        if (i2 == c->imp2_at.end()) {
          double imax2 = 0;
          const int32_t off = E.od();
          const int nx2 = (nx + 63) / 64 * 64;  // rows padded with zeros: k_sc_score2's idle lanes weigh 0
          for (int y = 0; y < ny; y++) {
            for (int x = 0; x < nx; x++) {
              const double w = iit->second[(size_t)y * nx + x] - E.params.outside_importance;
              imax2 = std::max(imax2, std::fabs(w));
              E.ad.push_back(w);
            }
            E.ad.insert(E.ad.end(), (size_t)(nx2 - nx), 0.0);
          }
          i2 = c->imp2_at.emplace(pk, std::make_pair(off, imax2)).first;
        }
        tab2_of[sz.first] = i2->second;
        imp_of[sz.first] = std::make_tuple(&iit->second, nx, ny);
      }
      q.crop0 = (int32_t)L->crops.size();
      q.ncrops = (int32_t)P.crops.size();
      for (const CropHost &ch : P.crops) {
        DevCrop dc{};
        dc.fx = ch.fx;
        dc.fy = ch.fy;
        dc.fw = ch.fw;
        dc.fh = ch.fh;
        dc.x0 = ch.x0;
        dc.y0 = ch.y0;
        dc.nin_x = ch.nin_x;
        dc.nin_y = ch.nin_y;
        const auto &t = tab_of[{dbits(ch.fw), dbits(ch.fh)}];
        dc.table = std::get<0>(t);
        dc.table_w = std::get<1>(t);
        dc.imax = std::get<2>(t);
        dc.table2 = tab2_of[{dbits(ch.fw), dbits(ch.fh)}].first;
        dc.table2_w = (dc.table_w + 63) / 64 * 64;
        dc.imax2 = tab2_of[{dbits(ch.fw), dbits(ch.fh)}].second;
        dc.rx = ch.rx;
        dc.ry = ch.ry;
        dc.rw = ch.rw;
        dc.rh = ch.rh;
        dc.sg = dc.sm = dc.sj = -1;
        L->crops.push_back(dc);
      }
      if (fast_ok) plan_score_groups(c, E, P, o.step, imp_of, L, &q);
      pp = placed.emplace(&P, q).first;
    }
    const Placed &q = pp->second;
    const fi_ctx::ScTabs &T = c->sc_at.at(&P);
    // the per-image kernels (k_sc_fz; k_sc_hmfma + k_sc_vq, or k_sc_vmaps when the
    // vertical window exceeds one MFMA block), else the generic per-row kernels
    const bool prep = c->sc_prep && P.prep_ok && P.hm_ok;
    d.img = it.img;
    d.stride = it.stride;
    d.W = it.W;
    d.H = it.H;
    d.C = it.C;
    d.fx = P.fx;
    d.fy = P.fy;
    d.rw = P.rw;
    d.rh = P.rh;
    d.need_h = P.need_h;
    d.need_v = P.need_v;
    d.aw = P.aw;
    d.ah = P.ah;
    d.ybox_first = P.ybox_first;
    d.hrows = P.hrows;
    d.ksh = P.ksh;
    d.ksv = P.ksv;
    d.hb = T.hb;
    d.hk = T.hk;
    d.hkT = T.hkT;
    d.vb = T.vb;
    d.vk = T.vk;
    d.prep = prep ? 1 : 0;
    d.hm = prep ? 1 : 0;
    d.hm_rows = P.hm_rows;
    d.hm_ks = P.hm_ks;
    d.hm_pitch = P.hm_pitch;
    d.hm_nb = P.hm_nb;
    d.hmB = T.hmB;
    d.hmC = T.hmC;
    d.hmS0 = T.hmS0;
    d.vq = prep && P.vq_ok ? 1 : 0;
    d.fz = d.vq && P.fz_ok && c->sc_fz ? 1 : 0;
    d.fd = d.fz && c->sc_fd && it.C == 3 && it.stride % 16 == 0 && (it.padded || (it.W * 3) % 16 == 0) &&
                   P.hm_nb <= kFdCWaves &&
                   fd_lds(it.W, P.hm_pitch, P.aw, P.ah) <= kFdMaxLds
               ? 1
               : 0;
    d.vqA = T.vqA;
    d.vqC = T.vqC;
    d.vqK0 = T.vqK0;
    // k_sc_hx + k_sc_vx: their tables, the horizontal ones at <= 2 k-steps, rows
    // readable to the 16-B rounded row bytes (3 or 1 channels; the source's own
    // alignment is checked at launch)
    const int rowb = it.C == 3 ? fd_rp(it.W) : (it.W + 15) / 16 * 16;
    d.cx = prep && c->sc_cx > 0 && P.cx_ok && T.cxA >= 0 && P.fx == 1 && P.fy == 1 &&
                   (it.C == 3 || it.C == 1) && P.hm_ks <= 2 && it.stride % 16 == 0 &&
                   (it.padded || it.W * it.C == rowb)
               ? 1
               : 0;
    d.cx_kv = P.cx_kv;
    d.cx_tp = P.cx_tp;
    d.cxA = T.cxA;
    d.cxK0 = T.cxK0;
    d.prescale = P.prescale;
    d.exact_all = o.exact_all || !fast_ok;
    // workspace (offsets; converted to pointers after allocation)
    auto take = [&](size_t n) { return (uint8_t *)(uintptr_t)(E.work.take(n) + 1); };
    if (P.fx > 1 || P.fy > 1) d.red = take((size_t)P.rw * P.rh * 3);
    if (P.thumb && P.need_h && !d.fz)  // generic kernels: pitch aw*3; k_sc_hmfma: pitch apitch
      d.hbuf = take((size_t)(prep ? (P.aw * 3 + 15) / 16 * 16 : P.aw * 3) * std::max(P.hrows, 1));
    if (P.thumb && (!prep || want_pre)) d.pre = take((size_t)P.aw * P.ah * 3);
    if (d.cx) d.tbuf = take((size_t)P.hm_nb * it.C * 16 * P.cx_tp);
    d.maps = (uint32_t *)take((size_t)P.aw * P.ah * 4);
    d.crop0 = q.crop0;
    d.ncrops = q.ncrops;
    d.sg0 = q.sg0;
    d.ngrp = c->sc_mf ? q.nsg : 0;
    d.sg_lds = q.sg_lds;
    d.score0 = L->nscores;
    L->nscores += q.ncrops;
    L->descs.push_back(d);
  }
}
template <class D>
static void fix_ptr(D *&p, uint8_t *base) {
  if (p) p = reinterpret_cast<D *>(base + ((uintptr_t)p - 1));
}

struct Launch {  // one kernel launch over a subset of descriptors
  size_t desc_off = 0, prefix_off = 0;
  int n = 0, tiles = 0;
};
template <class Desc, class TileFn>
static Launch add_launch(Blob &blob, const std::vector<Desc> &all, const std::vector<int> &members, TileFn tiles) {
  Launch L;
  std::vector<Desc> sub;
  std::vector<int32_t> prefix;
  int32_t acc = 0;
  for (int m : members) {
    const int t = tiles(all[m]);
    if (t <= 0) continue;
    sub.push_back(all[m]);
    prefix.push_back(acc);
    acc += t;
  }
  prefix.push_back(acc);
  L.n = (int)sub.size();
  L.tiles = acc;
  L.desc_off = blob.addv(sub);
  L.prefix_off = blob.addv(prefix);
  return L;
}

// Launch lists of a planned smartcrop stage: the per-image kernels where the
// plan fits them (k_sc_prep, k_sc_score2), the generic per-row kernels
// otherwise.
struct ScLaunches {
  Launch red, hp, vp, maps;        // generic (fi_kernels.hip)
  size_t hm_off = 0, vq_off = 0, vm_off = 0;   // k_sc_hmfma / k_sc_vq / k_sc_vmaps
  int nhm = 0, hm_chunks = 0, hm_lds = 0, nvm = 0, v_chunks = 0, v_lds = 0;
  size_t fz_off = 0, fd_off = 0;  // k_sc_fz, k_sc_fd
  int nfz = 0, fz_lds = 0, nfd = 0, fd_lds = 0;
  // k_sc_hx / k_sc_vx: descriptors, tile lists per variant v = 2 (k-steps - 1) + (channels == 3)
  size_t cx_off = 0, hxt_off[4] = {0, 0, 0, 0}, vxt_off[4] = {0, 0, 0, 0};
  int ncx = 0, hx_tiles[4] = {0, 0, 0, 0}, vx_tiles[4] = {0, 0, 0, 0};
  int nok = 0;  // descriptors planned OK (ncx == nok: the whole stage is co-resident work)
  int nvq = 0, vq_chunks = 0, vq_lds = 0;
  size_t sl_off = 0, sg_off = 0;   // k_sc_score2 with maps in LDS / global
  int nsl = 0, nsg = 0, sl_px = 0;
  size_t s3_off = 0, groups_off = 0;  // k_sc_score3 (exact-integer MFMA fast pass)
  int ns3 = 0, s3_lds = 0;
  size_t crops_off = 0;
};
static void add_sc_launches(fi_ctx *c, Blob &B, const ScLaunchData &SL, const std::vector<int> &sstatus,
                            ScLaunches *X) {
  std::vector<int> sred, shp, svp, smaps;
  std::vector<ScDesc> hm, sl, sg, vq, vm, fz, fd, s3, cx;
  for (size_t k = 0; k < SL.descs.size(); k++) {
    if (sstatus[k] != FI_OK) continue;
    X->nok++;
    const ScDesc &d = SL.descs[k];
    const ScPlan &P = *SL.plans[k];
    if (d.red) sred.push_back((int)k);
    const bool aligned = ((uintptr_t)d.img & 15) == 0;
    const bool fd_ok = d.fz && d.fd && aligned;
    // k_sc_fd where it streams the image (cfg2: 0.353 vs k_sc_hx + k_sc_vx's
    // 0.44 ms per 1024 images), k_sc_fz where it does not, k_sc_hx +
    // k_sc_vx for gray sources in place of the k_sc_hmfma + k_sc_vq /
    // k_sc_vmaps pair (cfg5: 0.137 vs 0.586 ms per 1024 images); RGB keeps the
    // pair (cfg4 sc_prep 20.1 vs 22.6 ms per step with the RGB forms at 128
    // VGPRs and row-segmented tiles; 30.0 when they spilled at 64)
    // (FI_SC_CX=2, 3: first)
    if (d.cx && aligned && (c->sc_cx >= 2 || (d.C == 1 && !(fd_ok || d.fz)))) {
      cx.push_back(d);
    } else if (fd_ok) {
      fd.push_back(d);
      X->fd_lds = std::max(X->fd_lds, fd_lds(d.W, d.hm_pitch, d.aw, d.ah));
    } else if (d.fz) {
      fz.push_back(d);
      X->fz_lds = std::max(X->fz_lds, P.fz_lds);
    } else if (d.prep) {
      if (d.vq) {
        vq.push_back(d);
        X->vq_chunks = std::max(X->vq_chunks, P.vq_chunks);
        X->vq_lds = std::max(X->vq_lds, P.vq_lds);
      } else {
        vm.push_back(d);
        X->v_chunks = std::max(X->v_chunks, P.v_chunks);
        X->v_lds = std::max(X->v_lds, P.v_lds);
      }
      hm.push_back(d);
      X->hm_chunks = std::max(X->hm_chunks, P.hm_chunks);
      X->hm_lds = std::max(X->hm_lds, P.hm_lds);
    } else {
      if (d.hbuf) shp.push_back((int)k);
      if (d.pre) svp.push_back((int)k);
      smaps.push_back((int)k);
    }
    if (d.ngrp > 0) {
      s3.push_back(d);
      X->s3_lds = std::max(X->s3_lds, d.sg_lds);
    } else if ((int64_t)d.aw * d.ah * 4 <= kScoreLdsMaps) {
      sl.push_back(d);
      X->sl_px = std::max(X->sl_px, d.aw * d.ah);
    } else {
      sg.push_back(d);
    }
  }
  X->red = add_launch(B, SL.descs, sred, [](const ScDesc &d) { return d.rh; });
  X->hp = add_launch(B, SL.descs, shp, [](const ScDesc &d) { return d.hrows; });
  X->vp = add_launch(B, SL.descs, svp, [](const ScDesc &d) { return d.ah; });
  X->maps = add_launch(B, SL.descs, smaps, [](const ScDesc &d) { return d.ah; });
  X->hm_off = B.addv(hm);
  X->nhm = (int)hm.size();
  X->vq_off = B.addv(vq);
  X->vm_off = B.addv(vm);
  X->nvm = (int)vm.size();
  X->nvq = (int)vq.size();
  X->fz_off = B.addv(fz);
  X->nfz = (int)fz.size();
  X->fd_off = B.addv(fd);
  X->nfd = (int)fd.size();
  // k_sc_hx tiles (descriptor, first of 4 column blocks, first of kHxRb row blocks), k_sc_vx tiles
  // (descriptor, chunk) four to a workgroup, one list per variant
  X->cx_off = B.addv(cx);
  X->ncx = (int)cx.size();
  for (int v = 0; v < 4; v++) {
    const int ks = v / 2 + 1, nch = (v & 1) ? 3 : 1;
    std::vector<int32_t> ht, vt;
    for (size_t k = 0; k < cx.size(); k++) {
      const ScDesc &d = cx[k];
      if (d.C != nch) continue;
      if (d.hm_ks == ks)
        for (int r = 0; r < d.cx_tp / 16 - 1; r += kHxRb)
          for (int b = 0; b < d.hm_nb; b += 4) {
            ht.push_back((int32_t)k);
            ht.push_back(b);
            ht.push_back(r);
          }
      if (d.cx_kv == ks)
        for (int ch = 0; ch < (d.ah + kVqRows - 1) / kVqRows; ch++) {
          vt.push_back((int32_t)k);
          vt.push_back(ch);
        }
    }
    while (vt.size() % 8) {
      vt.push_back(-1);
      vt.push_back(0);
    }
    X->hxt_off[v] = B.addv(ht);
    X->hx_tiles[v] = (int)(ht.size() / 3);
    X->vxt_off[v] = B.addv(vt);
    X->vx_tiles[v] = (int)(vt.size() / 2);
  }
  c->stats["sc_path_cx"].launches += X->ncx;
  // images per smartcrop prescale kernel (fi_kernel_stats)
  c->stats["sc_path_fd"].launches += X->nfd;
  c->stats["sc_path_fz"].launches += X->nfz;
  X->sl_off = B.addv(sl);
  X->nsl = (int)sl.size();
  X->sg_off = B.addv(sg);
  X->nsg = (int)sg.size();
  X->s3_off = B.addv(s3);
  X->ns3 = (int)s3.size();
  c->stats["sc_score_mfma"].launches += X->ns3;  // images per score kernel (fi_kernel_stats)
  c->stats["sc_score_valu"].launches += X->nsl + X->nsg;
  X->groups_off = B.addv(SL.groups);
  X->crops_off = B.addv(SL.crops);
}
static int enqueue_sc(fi_ctx *c, hipStream_t st, uint8_t *ab, const ScLaunches &X, const int32_t *ai,
                      const double *ad, CropScore *scores, ScResult *results, const ScParamsDev &PD) {
  auto desc = [&](const Launch &L) { return (const ScDesc *)(ab + L.desc_off); };
  auto pre = [&](const Launch &L) { return (const int32_t *)(ab + L.prefix_off); };
  // the skin / saturation table of this parameter set (k_sc_fz<true>), built
  // on the stream that reads it, so batches queued before a parameter change
  // have read the old table first
  const uint16_t *skinsat = nullptr;
  if (X.nfz > 0 || X.nfd > 0 || X.ncx > 0) {
    const std::string key(reinterpret_cast<const char *>(&PD), offsetof(ScParamsDev, pad));
    if (!c->skinsat.p || c->skinsat_key != key) {
      const int rc = ensure(c, &c->skinsat, (size_t)2 << 24);
      if (rc != FI_OK) return rc;
      // readers of the old table may still run on the other stream
      if (c->ap_pending && st == c->stream && order_after_apply(c) != FI_OK) return FI_EDEVICE;
      launch_sc_skinsat(st, (uint16_t *)c->skinsat.p, PD);
      c->skinsat_key = key;
    }
    skinsat = (const uint16_t *)c->skinsat.p;
  }
  {
    Timer t(c, "sc_prep", 0, st, st);
    if (X.red.tiles)
      hipLaunchKernelGGL(k_sc_reduce, dim3(X.red.tiles), dim3(256), 0, st, desc(X.red), pre(X.red), X.red.n);
    if (launch_sc_h(st, (const ScDesc *)(ab + X.hm_off), X.nhm, X.hm_chunks, X.hm_lds, ai) != 0 ||
        launch_sc_vq(st, (const ScDesc *)(ab + X.vq_off), X.nvq, X.vq_chunks, X.vq_lds, ai, PD) != 0 ||
        launch_sc_v(st, (const ScDesc *)(ab + X.vm_off), X.nvm, X.v_chunks, X.v_lds, ai, PD) != 0 ||
        launch_sc_fz(st, (const ScDesc *)(ab + X.fz_off), X.nfz, X.fz_lds, ai, PD, skinsat) != 0 ||
        launch_sc_fd(st, (const ScDesc *)(ab + X.fd_off), X.nfd, X.fd_lds, ai, PD, skinsat) != 0)
      return set_err(FI_EDEVICE, "smartcrop prescale launch rejected (LDS %d/%d/%d/%d)", X.hm_lds, X.vq_lds,
                     X.fz_lds, X.fd_lds);
    for (int v = 0; v < 4; v++) {
      const ScDesc *cd = (const ScDesc *)(ab + X.cx_off);
      if (launch_sc_hx(st, v / 2 + 1, (v & 1) ? 3 : 1, cd, (const int32_t *)(ab + X.hxt_off[v]), X.hx_tiles[v],
                       ai) != 0)
        return set_err(FI_EDEVICE, "k_sc_hx launch rejected");
    }
    for (int v = 0; v < 4; v++) {
      const ScDesc *cd = (const ScDesc *)(ab + X.cx_off);
      if (launch_sc_vx(st, v / 2 + 1, (v & 1) ? 3 : 1, cd, (const int32_t *)(ab + X.vxt_off[v]), X.vx_tiles[v],
                       ai, PD, skinsat) != 0)
        return set_err(FI_EDEVICE, "k_sc_vx launch rejected");
    }
    if (X.hp.tiles)
      hipLaunchKernelGGL(k_sc_hpass, dim3(X.hp.tiles), dim3(256), 0, st, desc(X.hp), pre(X.hp), X.hp.n, ai);
    if (X.vp.tiles)
      hipLaunchKernelGGL(k_sc_vpass, dim3(X.vp.tiles), dim3(256), 0, st, desc(X.vp), pre(X.vp), X.vp.n, ai);
    if (X.maps.tiles)
      hipLaunchKernelGGL(k_sc_maps, dim3(X.maps.tiles), dim3(256), 0, st, desc(X.maps), pre(X.maps),
                         X.maps.n, PD);
  }
  {
    Timer t(c, "sc_score", 0, st, st);
    const DevCrop *crops = (const DevCrop *)(ab + X.crops_off);
    if (launch_sc_score(st, 1, (const ScDesc *)(ab + X.sl_off), X.nsl, (size_t)X.sl_px * 4, crops, ad, scores,
                        results, PD, ai) != 0)
      return set_err(FI_EDEVICE, "k_sc_score2 launch rejected (%d px)", X.sl_px);
    (void)launch_sc_score(st, 0, (const ScDesc *)(ab + X.sg_off), X.nsg, 0, crops, ad, scores, results, PD, ai);
    if (launch_sc_score3(st, (const ScDesc *)(ab + X.s3_off), X.ns3, (size_t)X.s3_lds, crops,
                         (const ScGroup *)(ab + X.groups_off), ad, scores, results, PD, ai) != 0)
      return set_err(FI_EDEVICE, "k_sc_score3 launch rejected (%d B LDS)", X.s3_lds);
  }
  HIP_TRY(hipGetLastError());
  return FI_OK;
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static void host_stat(fi_ctx *c, const char *name, double ms) {
  if (!c->timing) return;
  Stat &s = c->stats[name];
  s.ms += ms;
  s.launches += 1;
}

// ---------------------------------------------------------------------------
// batch pipeline.  run_batch strings the units together:
//   plan_image (per image: geometry, descriptor, resample path + tables)
//   -> plan_batch_sc (smartcrop stage) -> resolve_workspace (device pointers,
//   -monochrome / convolution steps, crop apply) -> build_vm_tiles (k_rs_vr /
//   k_rs_vm) / build_hv_tiles -> pack_batch (one blob) -> launch_batch
//   -> queue_readback (pinned result records, the in-flight list).
// ---------------------------------------------------------------------------
struct MonoItem {
  int img;
  size_t g_off, st_off;
};
struct ConvItem {
  int img;
  size_t a_off, b_off;
};
// Everything a batch plans before it is packed and uploaded.
struct BatchPlan {
  fi_image *imgs = nullptr;
  int n = 0;
  std::vector<ImPlan> plans;
  std::vector<int> status;
  std::vector<std::string> errs;
  std::vector<ResizeDesc> rd;  // resample descriptors of the images that plan
  std::vector<int> rd_of;      // image -> rd index (-1: the image failed)
  std::vector<ScItem> sitems;  // smartcrop jobs
  std::vector<int> sc_of;      // image -> sitems index (-1: none)
  HashMap<const AxisTable *, DevAxis> placed;
  // resample path members (indices into rd) and their tables
  std::vector<int> vm_img;
  std::vector<const VmV *> vm_v;
  std::vector<const MfmaH *> vm_h;
  std::vector<const AxisTable *> vm_vt;  // their vertical axes (k_rs_vr tables)
  std::vector<int> hv_img;
  std::vector<const HvV *> hv_v;
  std::vector<const HvH *> hv_h;
  std::vector<int32_t> hv_W;  // source widths
  int h_tile_pitch = 0;  // k_rs_h_tile: max staged row bytes over the mode-2 images
  int h_tile_taps = 0;   // k_rs_h_tile: max horizontal window over the mode-2 images
  std::vector<size_t> res_off;    // per image: resized buffer in the workspace (smartcrop apply)
  std::vector<int64_t> res_stride;  // per image: the row pitch of out_of (out_stride, or padded in the workspace)
  std::vector<uint8_t *> out_of;  // per image: the final 8-bit output (dst, or the workspace +1-tagged)
  std::vector<MonoItem> mono;
  std::vector<ConvItem> conv_items;
  double resize_bytes = 0;
  // smartcrop stage
  ScLaunchData SL;
  std::vector<int> sstatus;
  std::vector<std::string> serrs;
  size_t results_off = 0, scores_off = 0, outwh_off = 0;
  // resolved against the slot's workspace
  std::vector<MonoDesc> mdesc_mono;
  std::vector<ConvStep> cst[6];  // U-H, U-V+combine, S-2D, B-H, B-V, to8
  std::vector<ApplyDesc> apply;
  // tiles
  std::vector<VDesc> vdescs;
  std::vector<MStrip> vstrips;
  std::vector<VTile> vtiles;
  // k_rs_vr: persistent block-major tiles, per-workgroup {phases, stream rows}, LDS layout
  // (one or more launches: their tiles and per-workgroup info back to back)
  struct VrLaunch {
    int32_t tile0, ntiles, info0, G, images;
    VrLayout L;
  };
  std::vector<VrTile> vrtiles;
  std::vector<int32_t> vr_info;
  std::vector<VrLaunch> vrl;
  size_t vm_lds = 0;
  std::vector<HvDesc> hdescs;
  std::vector<HvStripD> hstrips;
  std::vector<HvTile> htiles;
  size_t hv_lds = 0;
};
// Blob offsets and launch lists of a packed batch.
struct Packed {
  size_t all_rd_off = 0, vdesc_off = 0, vstrip_off = 0, vtile_off = 0, apply_off = 0, mono_off = 0;
  size_t vrtile_off = 0, vrinfo_off = 0;
  size_t hdesc_off = 0, hstrip_off = 0, htile_off = 0;
  size_t ai_off = 0, af_off = 0, ad_off = 0, mono_wts = 0;
  Launch L0, L1a, L2a, L2b, Q0, Q1a, Q2a, Q2b, CL[6];
  bool h_tiled = false;
  ScLaunches SX;
};

// The k_rs_vm column strips of a horizontal table: <= kVmMaxNx output px,
// narrower when the strip's horizontal fragments would not leave room for two
// workgroups per CU (nullptr: no strip width fits).
static const MfmaH *vm_strips(fi_ctx *c, const AxisTable *ht, bool q16) {
  auto hit = c->vmh_cache.find({ht, q16});
  if (hit == c->vmh_cache.end()) {
    MfmaH m;
    const int first_nx = kVmMaxNx;
    for (int mx : {first_nx, 48, 32}) {
      if (!build_mfma_h(*ht, &m, mx)) {
        m = MfmaH();
        break;
      }
      bool fits = true, wide = false;
      for (const MfmaStrip &st : m.strips) {
        fits = fits && vm_lds_bytes(st.vpitch, st.nocb, st.ks, q16) <= kVmMaxLds;
        wide = wide || st.nocb > 3;
      }
      // strips of four 16-px blocks (factors below ~2.7) at 48 px instead, so
      // k_rs_vr (<= 3 blocks a strip) takes the image (FI_VR_NARROW=0: keep 64)
      if (fits && wide && c->vr_narrow && c->vr_rs && mx == first_nx) {
        MfmaH n;
        bool nfits = build_mfma_h(*ht, &n, 48);
        for (const MfmaStrip &st : n.strips) nfits = nfits && vm_lds_bytes(st.vpitch, st.nocb, st.ks, q16) <= kVmMaxLds;
        if (nfits && !n.strips.empty()) m = std::move(n);
      }
      if (fits) break;
      m = MfmaH();
    }
    hit = c->vmh_cache.emplace(std::make_pair(ht, q16), std::move(m)).first;
  }
  return hit->second.strips.empty() ? nullptr : &hit->second;
}

// Choose the resample kernel of one image (d.mode) and add its tables:
//   5  k_rs_vr / k_rs_vm: RGB, vertical first, 16-byte aligned rows (the
//      default; build_vm_tiles picks the kernel);
//   6  k_rs_hv: RGB, horizontal first, contiguous taps, 16-byte aligned rows;
//   1 / 2  the generic two-pass kernels, vertical / horizontal first (RGBA,
//      convolution inputs, unaligned sources, tables that do not fit).
// Returns the algorithmic source bytes the path reads.
static int64_t plan_resample(fi_ctx *c, Exec &E, BatchPlan &Bp, const ImPlan &P, const fi_image &im,
                             ResizeDesc &d) {
  const AxisTable *vt = add_axis(c, E, P.filter, P.yf, P.sh, P.th, P.ey0, P.ey0 + P.eh, P.sample, P.H, &d.v, Bp.placed);
  const AxisTable *ht = add_axis(c, E, P.filter, P.xf, P.sw, P.tw, P.ex0, P.ex0 + P.ew, P.sample, P.W, &d.h, Bp.placed);
  const bool rgb = P.C == 3;
  const bool fast_ok = rgb && !P.conv;  // the streaming kernels write 8-bit only
  if (!rgb) {
    // matte (RGBA) images: the alpha-weighted f64 generic passes (k_rs4_*)
    add_axis_f64(c, E, vt, &d.v);
    add_axis_f64(c, E, ht, &d.h);
  }
  const bool aligned16 = ((uintptr_t)im.src % 16) == 0 && (im.src_stride % 16) == 0;
  const int64_t strip_bytes = (int64_t)vt->touched * (d.h.src_hi - d.h.src_lo) * 3;
  const bool vfirst_fast = fast_ok && !P.hfirst && c->fast_rs && aligned16;
  if (vfirst_fast) {
    auto vit = c->vmv_cache.find(vt);
    if (vit == c->vmv_cache.end()) {
      VmV m;
      if (!build_vm_v(*vt, &m)) m = VmV();
      vit = c->vmv_cache.emplace(vt, std::move(m)).first;
    }
    // the Q16 output tile (gray / rotation) needs more LDS than the 8-bit one
    const MfmaH *hh = vm_strips(c, ht, P.gray || P.rot != 0);
    if (vit->second.nblk > 0 && hh) {
      d.mode = 5;  // streaming exact-integer MFMA, vertical first
      Bp.vm_img.push_back((int)Bp.rd.size());
      Bp.vm_v.push_back(&vit->second);
      Bp.vm_h.push_back(hh);
      Bp.vm_vt.push_back(vt);
      return strip_bytes;
    }
  }
  // horizontal first: contiguous tap ranges (no sample pre-step), 16-byte aligned rows
  if (fast_ok && P.hfirst && !P.sample && c->fast_rs && aligned16) {
    auto vit = c->hvv_cache.find(vt);
    if (vit == c->hvv_cache.end()) {
      HvV m;
      if (!build_hv_v(*vt, &m)) m = HvV();
      vit = c->hvv_cache.emplace(vt, std::move(m)).first;
    }
    auto hit = c->hvh_cache.find(ht);
    if (hit == c->hvh_cache.end()) {
      HvH m;
      if (!build_hv_h(*ht, &m)) m = HvH();
      for (const HvStrip &st : m.strips)
        if (hv_lds_bytes(st.pp, st.nocb) > kVmMaxLds) m = HvH();
      hit = c->hvh_cache.emplace(ht, std::move(m)).first;
    }
    if (vit->second.nblk > 0 && !hit->second.strips.empty()) {
      d.mode = 6;  // streaming exact-integer MFMA, horizontal first
      Bp.hv_img.push_back((int)Bp.rd.size());
      Bp.hv_v.push_back(&vit->second);
      Bp.hv_h.push_back(&hit->second);
      Bp.hv_W.push_back(P.W);
      int64_t cols = 0;
      for (const HvStrip &st : hit->second.strips) cols += std::min(st.pp, P.W - st.px0);
      return (int64_t)vit->second.nrows * cols * 3;
    }
  }
  if (!rgb && !P.hfirst) {
    d.mode = 1;  // RGBA: mid = [eh][source columns src_lo..src_hi) x 4 Q16
    d.mid_c0 = d.h.src_lo;
    d.mid_cols = d.h.src_hi - d.h.src_lo;
    d.mid_rows = P.eh;
    d.mid_stride = 4 * (int64_t)d.mid_cols;
  } else if (!rgb) {
    d.mode = 2;  // RGBA: mid = [source rows src_lo..src_hi][ew] x 4 Q16
    d.mid_r0 = d.v.src_lo;
    d.mid_rows = d.v.src_hi - d.v.src_lo;
    d.mid_cols = P.ew;
    d.mid_stride = 4 * (int64_t)P.ew;
  } else if (!P.hfirst) {
    d.mode = 1;
    const int64_t b_lo = (int64_t)3 * d.h.src_lo / 8 * 8;
    const int64_t b_hi = std::min<int64_t>((int64_t)3 * P.W, ((int64_t)3 * d.h.src_hi + 7) / 8 * 8);
    d.mid_c0 = (int32_t)b_lo;
    d.mid_cols = (int32_t)(b_hi - b_lo);
    d.mid_rows = P.eh;
    d.mid_stride = (d.mid_cols + 7) / 8 * 8;
  } else {
    d.mode = 2;
    d.mid_r0 = d.v.src_lo;
    d.mid_rows = d.v.src_hi - d.v.src_lo;
    d.mid_cols = P.ew;
    d.mid_stride = (3 * P.ew + 7) / 8 * 8;
    // k_rs_h_tile LDS row pitch: the source bytes of a 256-column chunk's windows
    for (int x0 = 0; x0 < P.ew; x0 += 256) {
      const int x1 = std::min(P.ew, x0 + 256);
      const int lo = ht->start[x0], hi = ht->start[x1 - 1] + ht->count[x1 - 1];
      Bp.h_tile_pitch = std::max(Bp.h_tile_pitch, (3 * (hi - lo) + 8 + 15) / 16 * 16);
      Bp.h_tile_taps = std::max(Bp.h_tile_taps, (int)d.h.maxtaps);
    }
  }
  d.mid = (uint16_t *)(uintptr_t)(E.work.take((size_t)d.mid_stride * d.mid_rows * 2) + 1);
  return (int64_t)vt->touched * (d.h.src_hi - d.h.src_lo) * P.C;
}

// Plan image i: geometry (plan_im), output record, the resample descriptor
// and its destination (dst, the apply / -monochrome / convolution workspace),
// and its smartcrop job.  Failures go to the image's status.
static void plan_image(fi_ctx *c, Exec &E, BatchPlan &Bp, int i) {
  fi_image &im = Bp.imgs[i];
  ImPlan &P = Bp.plans[i];
  const int rc = plan_im(im, &P);
  if (rc != FI_OK) {
    Bp.status[i] = rc;
    Bp.errs[i] = P.err;
    return;
  }
  if (!im.src) {
    Bp.status[i] = FI_EINVAL;
    Bp.errs[i] = "src is NULL";
    return;
  }
  const bool smc = (im.flags & FI_OP_SMARTCROP) != 0;
  const bool apply = smc && (im.flags & FI_OP_SMARTCROP_APPLY);
  im.out_w = P.out_w;
  im.out_h = P.out_h;
  im.out_channels = P.out_c;
  im.out_stride = P.out_w * P.out_c;
  const int64_t need = (int64_t)im.out_stride * im.out_h;
  if (!im.dst || im.dst_capacity < need) {
    Bp.status[i] = FI_ECAPACITY;
    Bp.errs[i] = "dst NULL or dst_capacity < out_stride*out_h";
    return;
  }
  ResizeDesc d{};
  d.src = im.src;
  d.src_stride = im.src_stride;
  d.C = P.C;
  d.ew = P.ew;
  d.eh = P.eh;
  d.ex0 = P.ex0;
  d.ey0 = P.ey0;
  d.gray = P.gray;
  d.rot = P.rot;
  d.out_w = P.out_w;
  d.out_h = P.out_h;
  d.out_c = P.out_c;
  d.dst_stride = im.out_stride;
  Bp.res_stride[i] = im.out_stride;
  if (apply) {
    // the resized image stays in the workspace for smartcrop and the crop
    // apply: rows padded to res_align bytes, so the readers' 16-byte loads
    // are aligned (the -monochrome and convolution outputs keep out_stride)
    if (!P.mono && !P.conv) {
      const int64_t a = c->res_align;
      Bp.res_stride[i] = d.dst_stride = (im.out_stride + a - 1) / a * a;
    }
    Bp.res_off[i] = E.work.take((size_t)(Bp.res_stride[i] * im.out_h));
    d.dst = (uint8_t *)(uintptr_t)(Bp.res_off[i] + 1);  // workspace, resolved later
  } else {
    d.dst = im.dst;
  }
  Bp.out_of[i] = d.dst;
  if (P.mono) {
    // the resample epilogue writes the extent window's Q16 gray, unrotated;
    // fi_mono.hip quantizes it and writes the rotated 0/255 output
    MonoItem m;
    m.img = i;
    m.g_off = E.work.take((size_t)P.ew * P.eh * 2);
    m.st_off = E.work.take(sizeof(MonoState));
    Bp.mono.push_back(m);
    d.dst = (uint8_t *)(uintptr_t)(m.g_off + 1);
    d.dst_stride = (int64_t)P.ew * 2;
    d.gray = 2;
    d.rot = 0;
  }
  if (P.conv) {
    // the epilogue writes the rotated Q16 image; the convolutions ping-pong
    // between two such buffers and the last step writes the 8-bit output
    ConvItem ci;
    ci.img = i;
    const size_t qb = (size_t)P.out_w * P.out_h * P.out_c * 2;
    ci.a_off = E.work.take(qb);
    ci.b_off = E.work.take(qb);
    Bp.conv_items.push_back(ci);
    d.dst = (uint8_t *)(uintptr_t)(ci.a_off + 1);
    d.dst_stride = (int64_t)P.out_w * P.out_c * 2;
    d.q16out = 1;
  }
  int64_t src_bytes;
  if (!P.resize) {
    d.mode = 0;
    src_bytes = (int64_t)P.ew * P.eh * P.C;
  } else {
    src_bytes = plan_resample(c, E, Bp, P, im, d);
  }
  Bp.resize_bytes += (double)src_bytes + (double)need;
  static const char *kPath[7] = {"path_copy", "path_generic_v", "path_generic_h", "path_none", "path_none",
                                 "path_vm", "path_hv"};
  c->stats[kPath[d.mode]].launches += 1;  // images per resample path (fi_kernel_stats)
  Bp.rd_of[i] = (int)Bp.rd.size();
  Bp.rd.push_back(d);
  if (smc) {
    ScItem it{};
    it.img = nullptr;  // the resized image: resolved with the workspace
    it.stride = Bp.res_stride[i];
    it.W = P.out_w;
    it.H = P.out_h;
    it.C = P.out_c;
    it.tw = im.smartcrop_w > 0 ? im.smartcrop_w : 100;
    it.th = im.smartcrop_h > 0 ? im.smartcrop_h : 100;
    it.result = (int)Bp.sitems.size();
    it.padded = apply && Bp.res_stride[i] % 16 == 0;  // workspace rows at a 16-B rounded pitch
    fi_smartcrop_default_options(&it.opt);
    Bp.sc_of[i] = (int)Bp.sitems.size();
    Bp.sitems.push_back(it);
  }
}

// The smartcrop stage of the batch: input = each image's resized output.
static void plan_batch_sc(fi_ctx *c, Exec &E, BatchPlan &Bp) {
  Bp.sstatus.assign(Bp.sitems.size(), FI_OK);
  Bp.serrs.assign(Bp.sitems.size(), std::string());
  for (int i = 0; i < Bp.n; i++)
    if (Bp.sc_of[i] >= 0) Bp.sitems[Bp.sc_of[i]].img = Bp.out_of[i];  // may be +1-tagged workspace
  plan_smartcrop(c, E, Bp.sitems, &Bp.SL, &Bp.sstatus, &Bp.serrs, false);
  Bp.results_off = E.work.take(sizeof(ScResult) * std::max<size_t>(Bp.sitems.size(), 1));
  Bp.scores_off = E.work.take(sizeof(CropScore) * std::max(Bp.SL.nscores, 1));
  Bp.outwh_off = E.work.take(sizeof(int32_t) * 2 * std::max(Bp.n, 1));
}

// Resolve the +1-tagged workspace offsets against the slot's workspace wb and
// build what needs device pointers: -monochrome descriptors, the forwarded
// convolution steps (per image in IM's order: unsharp, sharpen, blur; one
// launch per stage), the smartcrop descriptors' buffers and crop apply.
static void resolve_workspace(Exec &E, BatchPlan &Bp, uint8_t *wb) {
  fi_image *imgs = Bp.imgs;
  for (int i = 0; i < Bp.n; i++) {
    if (Bp.rd_of[i] < 0) continue;
    ResizeDesc &d = Bp.rd[Bp.rd_of[i]];
    if (d.mid) fix_ptr(d.mid, wb);
    const bool apply = (imgs[i].flags & FI_OP_SMARTCROP) && (imgs[i].flags & FI_OP_SMARTCROP_APPLY);
    if (apply) fix_ptr(Bp.out_of[i], wb);
    if (d.gray == 2 || d.q16out)
      fix_ptr(d.dst, wb);
    else
      d.dst = Bp.out_of[i];
  }
  for (const MonoItem &m : Bp.mono) {
    const ResizeDesc &d = Bp.rd[Bp.rd_of[m.img]];
    MonoDesc md{};
    md.g = (const uint16_t *)(wb + m.g_off);
    md.w = d.ew;
    md.h = d.eh;
    md.rot = Bp.plans[m.img].rot;
    md.dst = Bp.out_of[m.img];
    md.dst_stride = imgs[m.img].out_stride;
    md.st = (MonoState *)(wb + m.st_off);
    Bp.mdesc_mono.push_back(md);
  }
  for (const ConvItem &ci : Bp.conv_items) {
    const ImPlan &P = Bp.plans[ci.img];
    uint16_t *A = (uint16_t *)(wb + ci.a_off), *Bf = (uint16_t *)(wb + ci.b_off);
    uint16_t *cur = A, *oth = Bf;
    ConvStep base{};
    base.W = P.out_w;
    base.H = P.out_h;
    base.C = P.out_c;
    std::vector<double> kk;
    auto table = [&](const std::vector<double> &v) {
      const int32_t off = E.od();
      E.ad.insert(E.ad.end(), v.begin(), v.end());
      return off;
    };
    if (P.conv & 1) {
      const int w = im_blur_kernel(P.cv[0], P.cv[1], &kk);
      ConvStep h = base, v = base;
      h.k = v.k = table(kk);
      h.kw = w, h.kh = 1, h.in = cur, h.out = oth;
      v.kw = 1, v.kh = w, v.in = oth, v.orig = cur, v.out = cur;
      v.gain = P.cv[2];
      v.thr = 65535.0 * P.cv[3];
      Bp.cst[0].push_back(h);
      Bp.cst[1].push_back(v);
    }
    if (P.conv & 2) {
      const int w = im_sharpen_kernel(P.cv[4], P.cv[5], &kk);
      ConvStep t = base;
      t.k = table(kk);
      t.kw = t.kh = w, t.in = cur, t.out = oth;
      Bp.cst[2].push_back(t);
      std::swap(cur, oth);
    }
    if (P.conv & 4) {
      const int w = im_blur_kernel(P.cv[6], P.cv[7], &kk);
      ConvStep h = base, v = base;
      h.k = v.k = table(kk);
      h.kw = w, h.kh = 1, h.in = cur, h.out = oth;
      v.kw = 1, v.kh = w, v.in = oth, v.out = cur;
      Bp.cst[3].push_back(h);
      Bp.cst[4].push_back(v);
    }
    ConvStep f = base;
    f.in = cur;
    f.dst8 = Bp.out_of[ci.img];
    f.dst_stride = imgs[ci.img].out_stride;
    Bp.cst[5].push_back(f);
  }
  for (ScDesc &d : Bp.SL.descs) {
    fix_ptr(d.red, wb);
    fix_ptr(d.hbuf, wb);
    fix_ptr(d.tbuf, wb);
    fix_ptr(d.pre, wb);
    fix_ptr(d.maps, wb);
  }
  for (int i = 0; i < Bp.n; i++)
    if (Bp.sc_of[i] >= 0) Bp.SL.descs[Bp.sc_of[i]].img = Bp.out_of[i];
  for (int i = 0; i < Bp.n; i++) {
    if (Bp.rd_of[i] < 0 || Bp.sc_of[i] < 0) continue;
    if (!(imgs[i].flags & FI_OP_SMARTCROP_APPLY)) continue;
    if (Bp.sstatus[Bp.sc_of[i]] != FI_OK) continue;
    const ResizeDesc &d = Bp.rd[Bp.rd_of[i]];
    ApplyDesc a{};
    a.src = Bp.out_of[i];
    a.src_stride = Bp.res_stride[i];
    a.W = d.out_w;
    a.H = d.out_h;
    a.C = d.out_c;
    a.result = Bp.sc_of[i];
    a.crop0 = Bp.SL.descs[Bp.sc_of[i]].crop0;
    a.dst = imgs[i].dst;
    a.out_wh = (int32_t *)(wb + Bp.outwh_off + 8 * (size_t)i);
    Bp.apply.push_back(a);
  }
}


// k_rs_vr: images (their k_rs_vm VDesc, strips) with block-major tables.
struct VrWork {
  int32_t img, first_strip, nstrips;
  const VrV *V;
  int32_t hwsum2, hsh;  // the horizontal two-limb tables (fi_plan.h MfmaH::wsum2 / shift2)
};
// k_rs_vr workgroups: tiles (image, strip, band of blocks) in the XCD-aware
// order of k_rs_vm, dealt round-robin to one persistent workgroup per CU; the
// tiles of a workgroup form its row stream.  False (nothing launched) when the
// ring does not fit LDS or a stream needs more rows resident than the ring has.
static bool build_vr_tiles(fi_ctx *c, Exec &E, BatchPlan &Bp, const std::vector<VrWork> &work) {
  auto align4 = [&]() {
    while (E.ai.size() % 4) E.ai.push_back(0);
  };
  auto put = [&](const std::vector<int32_t> &v) {
    const int32_t o = E.oi();
    E.ai.insert(E.ai.end(), v.begin(), v.end());
    return o;
  };
  int vpitch = 0;
  bool q16 = false;
  int64_t nst = 0;
  for (const VrWork &w : work) {
    for (int st = 0; st < w.nstrips; st++) vpitch = std::max(vpitch, Bp.vstrips[w.first_strip + st].vpitch);
    const VDesc &d = Bp.vdescs[w.img];
    q16 = q16 || d.gray || d.rot != 0;
    nst += w.nstrips;
  }
  VrLayout L = vr_lds_layout(vpitch, q16, 1);
  if (L.R <= 0) return false;
  // loader waves: 4 when every strip has one 16-px output block (3 items: one
  // per H wave).  Measured (round 5): cfg5 resize 8.45 -> 7.83 ms; cfg2 (two
  // blocks a strip, two items per H wave) neutral, cfg3 1 % slower, so they
  // keep 2.  FI_VR_NL=2 / 4 forces (4 only where it is valid: <= 2 blocks a
  // strip)
  {
    int max_nocb = 0;
    for (const VrWork &w : work)
      for (int st = 0; st < w.nstrips; st++) max_nocb = std::max(max_nocb, Bp.vstrips[w.first_strip + st].nocb);
    const int want = c->vr_nl ? c->vr_nl : (max_nocb <= 1 ? 4 : 2);
    L.nl = (want == 4 && max_nocb <= 2) ? 4 : 2;
  }
  // per image: a VDesc with the block-major tables
  std::vector<int32_t> desc_of(work.size());
  for (size_t k = 0; k < work.size(); k++) {
    const VrV &V = *work[k].V;
    auto vp = c->vr_at.find(&V);
    if (vp == c->vr_at.end()) {
      std::array<int32_t, 4> o;
      o[0] = put(V.rows);
      E.ai.insert(E.ai.end(), 32, 0);
      if (V.rstep == 0 && !V.rows.empty()) {
        // the uneven list again, as each k_rs_vr loader wave walks it (for 2
        // and for 4 loader waves): class rho = k mod C, entry j = the pair
        // (rows[C j + rho], rows[C j + rho + 1]), so a wave's own pairs (C = 2 NL
        // apart) are consecutive ints
        const int n = (int)V.rows.size(), J4 = vr_pair_cls_len(n, 4), J8 = vr_pair_cls_len(n, 8);
        std::vector<int32_t> pc(8 * (size_t)J4 + 16 * (size_t)J8);
        for (int C : {4, 8}) {
          const int J = C == 4 ? J4 : J8;
          for (int k = 0; k < C * J; k++) {  // the pair starting at list row k (fi_internal.h vr_pair_off)
            const size_t o = (size_t)(vr_pair_off(n, k, C) - (n + 32));
            pc[o] = V.rows[std::min(k, n - 1)];
            pc[o + 1] = V.rows[std::min(k + 1, n - 1)];
          }
        }
        put(pc);
      }
      align4();
      o[1] = put(V.bmeta);
      o[2] = put(V.w128);
      align4();
      o[3] = put(V.frag);
      vp = c->vr_at.emplace(&V, o).first;
    }
    VDesc m = Bp.vdescs[work[k].img];
    m.rows = vp->second[0];
    m.nrows = (int32_t)V.rows.size();
    m.row0 = V.row0;
    m.rstep = V.rstep;
    m.pmeta = vp->second[1];
    m.w128 = vp->second[2];
    m.frag = vp->second[3];
    m.nblk = V.nblk;
    m.vsh = V.shift;
    m.hsh = work[k].hsh;
    m.hwsum = work[k].hwsum2;
    desc_of[k] = (int32_t)Bp.vdescs.size();
    Bp.vdescs.push_back(m);
  }
  // per (tables, band): glen, the rows the band needs resident at once inside
  // it, Rend(b0) - kbase and K0(b1 - 1) - kbase (the seams between tiles)
  struct Span {
    int32_t glen, inner, head, tail;
  };
  HashMap<std::tuple<const VrV *, int, int>, Span> spans;
  std::tuple<const VrV *, int, int> last_key{nullptr, -1, -1};
  const Span *last_sp = nullptr;
  auto span_of = [&](const VrV &V, int b0, int b1) -> const Span & {
    const auto key = std::make_tuple(&V, b0, b1);
    if (last_sp && key == last_key) return *last_sp;  // consecutive images mostly share tables
    last_key = key;
    auto it = spans.find(key);
    if (it != spans.end()) return *(last_sp = &it->second);
    const int32_t *bm = V.bmeta.data();
    const int kbase = bm[4 * b0];
    Span sp{};
    sp.glen = (bm[4 * (b1 - 1) + 2] - kbase + 15) / 16 * 16;
    sp.head = bm[4 * b0 + 2] - kbase;
    sp.tail = bm[4 * (b1 - 1)] - kbase;
    sp.inner = sp.head;
    for (int b = b0; b + 1 < b1; b++) sp.inner = std::max(sp.inner, bm[4 * (b + 1) + 2] - bm[4 * b]);
    last_sp = &spans.emplace(key, sp).first->second;
    return *last_sp;
  };
  // tiles (image, strip, band of blocks), costed as the rows they stream plus
  // a per-phase overhead of 16 rows
  struct TC {
    VrTile t;
    int64_t cost;
    const Span *sp;
  };
  std::vector<TC> all;
  all.reserve((size_t)nst);
  // tiles of one (image, band) share a cost: groups [first, first + n) of `all`
  struct Grp {
    int64_t cost;
    int32_t first, n;
  };
  std::vector<Grp> grps;
  grps.reserve(work.size());
  std::vector<int64_t> img_cost(work.size(), 0);
  for (size_t k = 0; k < work.size(); k++) {
    const VrWork &w = work[k];
    const int nblk = w.V->nblk;
    int bands = nst > 0 ? (int)((2048 + nst - 1) / nst) : 1;
    bands = std::max(1, std::min(bands, nblk));
    for (int bnd = 0; bnd < bands; bnd++) {
      const int b0 = (int)((int64_t)nblk * bnd / bands), b1 = (int)((int64_t)nblk * (bnd + 1) / bands);
      if (b1 <= b0) continue;
      const Span &sp = span_of(*w.V, b0, b1);
      if (sp.inner > L.R) {
        if (getenv("FI_VR_DEBUG")) fprintf(stderr, "vr reject: inner %d > R %d\n", sp.inner, L.R);
        return false;
      }
      const int64_t cost = sp.glen + 16 * (b1 - b0);
      grps.push_back(Grp{cost, (int32_t)all.size(), w.nstrips});
      for (int st = 0; st < w.nstrips; st++)
        all.push_back(TC{VrTile{desc_of[k], w.first_strip + st, b0, b1, 0, 0, 0, (int32_t)k}, cost, &sp});
      img_cost[k] += cost * w.nstrips;
    }
  }
  const int ntiles = (int)all.size();
  if (ntiles == 0) return false;
  VrLayout L1{};
  {
    // two Q16 plane buffers (by block parity: the V waves never wait for the H
    // waves' reads) cost the ring 32 rows; taken when the smaller ring still
    // holds every block's and its successor's rows with max(32, half a block
    // step) to spare.  Measured (round 5): cfg2 (33 spare) 1.99 -> 1.93 ms;
    // cfg3 (19) and cfg5 (3) slower.  FI_VR_PBUF=1 / 2 forces (2 where it fits)
    int inner = 0, step = 0;
    for (const auto &kv : spans) inner = std::max(inner, kv.second.inner);
    for (const VrWork &w : work) {
      const int32_t *bm = w.V->bmeta.data();
      for (int b = 0; b + 1 < w.V->nblk; b++) step = std::max(step, bm[4 * (b + 1)] - bm[4 * b]);
    }
    const VrLayout L2 = vr_lds_layout(vpitch, q16, 2);
    const int want = c->vr_pbuf ? c->vr_pbuf : (L2.R - inner >= std::max(32, step / 2) ? 2 : 1);
    L1 = L;
    if (want == 2 && L2.R >= inner) {
      L = L2;
      L.nl = L1.nl;
    }
  }
  int G = std::min(ntiles, c->n_cu);
  if (G > 8) G -= G % 8;
  // workgroup g runs on XCD g % 8; with fewer than 4 images per XCD (small
  // batches, the serving shape) the tiles spread over every workgroup instead
  const int nx = G >= 8 && work.size() >= 32 ? 8 : 1;
  // images -> XCDs by LPT on their cost (an image's strips share halo columns
  // in that XCD's L2), then each XCD's tiles -> its workgroups by LPT
  std::vector<int> order(work.size());
  for (size_t k = 0; k < work.size(); k++) order[k] = (int)k;
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return img_cost[x] > img_cost[y]; });
  std::vector<int> xcd_of(work.size(), 0);
  {
    std::vector<int64_t> load(nx, 0);
    for (int k : order) {
      const int x = (int)(std::min_element(load.begin(), load.end()) - load.begin());
      xcd_of[k] = x;
      load[x] += img_cost[k];
    }
  }
  // equal costs (a uniform batch) keep the list order: no sort needed; else
  // LPT over the tiles longest first, sorting the (image, band) groups (the
  // tiles of a group cost the same) rather than the tiles
  bool uniform = true;
  for (const Grp &gp : grps) uniform = uniform && gp.cost == grps[0].cost;
  std::vector<const TC *> order_t;
  order_t.reserve(all.size());
  if (uniform) {
    for (const TC &tc : all) order_t.push_back(&tc);
  } else {
    std::stable_sort(grps.begin(), grps.end(), [](const Grp &x, const Grp &y) { return x.cost > y.cost; });
    for (const Grp &gp : grps)
      for (int i = 0; i < gp.n; i++) order_t.push_back(&all[gp.first + i]);
  }
  std::vector<std::vector<const TC *>> per(G);
  for (auto &v : per) v.reserve(ntiles / G + 8);
  if (uniform) {
    // equal costs: LPT is a round robin over each XCD's workgroups
    std::vector<int> next(nx, 0);
    const int per_x = G / nx;
    for (const TC *tc : order_t) {
      const int x = xcd_of[tc->t.pad];
      per[x + nx * (next[x]++ % per_x)].push_back(tc);
    }
  } else {
    // longest first, dealt boustrophedon over each XCD's workgroups (0 .. n-1,
    // n-1 .. 0, ...): O(1) per tile and, over ~80 sorted tiles per
    // workgroup, within a tile of LPT's balance (an LPT heap per tile cost
    // ~1 ms of host planning per cfg4 batch)
    std::vector<int> next(nx, 0);
    const int per_x = G / nx;
    for (const TC *tc : order_t) {
      const int x = xcd_of[tc->t.pad];
      const int i = next[x]++, r = i % per_x;
      per[x + nx * (((i / per_x) & 1) ? per_x - 1 - r : r)].push_back(tc);
    }
  }
  // the streams: workgroup g walks tiles [t0(g), t1(g)); every phase's rows
  // [K0, Rend) and the next phase's must be resident together
  std::vector<VrTile> tiles;
  std::vector<int32_t> info;
  auto streams = [&](int R) -> bool {
    tiles.clear();
    tiles.reserve(ntiles);
    info.assign(4 * (size_t)G, 0);
    for (int g = 0; g < G; g++) {
      int64_t gpos = 0, prev_tail = -1;
      info[4 * g + 2] = (int32_t)tiles.size();
      for (const TC *tc : per[g]) {
        VrTile T = tc->t;
        const VrV &V = *work[T.pad].V;
        const Span &sp = *tc->sp;
        T.kbase = V.bmeta[4 * T.b0];
        T.glen = sp.glen;
        T.g0 = (int32_t)gpos;
        // the seam: this tile's first block's rows and the previous tile's last
        // block's window resident together
        if (prev_tail >= 0 && T.g0 + sp.head - prev_tail > R) return false;
        prev_tail = T.g0 + sp.tail;
        info[4 * g] += T.b1 - T.b0;
        gpos += T.glen;
        if (gpos >= ((int64_t)1 << 30)) return false;
        T.pad = 0;
        tiles.push_back(T);
      }
      info[4 * g + 1] = (int32_t)gpos;
      info[4 * g + 3] = (int32_t)tiles.size();
    }
    return true;
  };
  if (!streams(L.R)) {
    if (L.pbuf != 2) {
      if (getenv("FI_VR_DEBUG")) fprintf(stderr, "vr reject: seam, R %d\n", L.R);
      return false;
    }
    L = L1;  // a seam needs the bigger ring
    if (!streams(L.R)) {
      if (getenv("FI_VR_DEBUG")) fprintf(stderr, "vr reject: seam, R %d (one plane buffer)\n", L.R);
      return false;
    }
  }
  static const bool vr_debug = getenv("FI_VR_DEBUG") != nullptr;
  if (vr_debug) {
    int inner = 0, rpb = 0, nocb = 0;
    for (const auto &kv : spans) inner = std::max(inner, kv.second.inner);
    for (const VrWork &w : work) {
      const int32_t *bm = w.V->bmeta.data();
      for (int b = 0; b + 1 < w.V->nblk; b++) rpb = std::max(rpb, bm[4 * (b + 1)] - bm[4 * b]);
      for (int st = 0; st < w.nstrips; st++) nocb = std::max(nocb, Bp.vstrips[w.first_strip + st].nocb);
    }
    int hist[4] = {0, 0, 0, 0};
    for (const VrTile &t : tiles) hist[std::min(3, Bp.vstrips[t.strip].nocb)]++;
    fprintf(stderr, "vr: R %d pbuf %d nl %d vpitch %d inner %d K0 step max %d nocb %d (tiles by nocb %d %d %d) tiles %d G %d\n",
            L.R, L.pbuf, L.nl, vpitch, inner, rpb, nocb, hist[1], hist[2], hist[3], ntiles, G);
  }
  Bp.vrl.push_back(BatchPlan::VrLaunch{(int32_t)Bp.vrtiles.size(), (int32_t)tiles.size(), (int32_t)Bp.vr_info.size(),
                                        G, (int32_t)work.size(), L});
  Bp.vrtiles.insert(Bp.vrtiles.end(), tiles.begin(), tiles.end());
  Bp.vr_info.insert(Bp.vr_info.end(), info.begin(), info.end());
  return true;
}

// k_rs_vm workgroups: (image, strip, band of blocks); the tables of a geometry
// are placed in the heap once.
static void build_vm_tiles(fi_ctx *c, Exec &E, BatchPlan &Bp) {
  auto align4 = [&]() {
    while (E.ai.size() % 4) E.ai.push_back(0);
  };
  auto put = [&](const std::vector<int32_t> &v) {
    const int32_t o = E.oi();
    E.ai.insert(E.ai.end(), v.begin(), v.end());
    return o;
  };
  HashMap<const MfmaH *, std::array<int32_t, 5>> hplaced;  // first strip, hwsum, hwsum2, LDS (8-bit / Q16 tile)
  struct Work1 {
    int32_t img, first_strip, nstrips;
    const VmV *V;
    const AxisTable *vt;
    int32_t hwsum2, hsh;
  };
  std::vector<Work1> work;
  const int nv = (int)Bp.vm_img.size();
  work.reserve(nv);
  Bp.vdescs.reserve(2 * (size_t)nv);  // + the k_rs_vr descriptors
  for (int q = 0; q < nv; q++) {
    const ResizeDesc &d = Bp.rd[Bp.vm_img[q]];
    const VmV &V = *Bp.vm_v[q];
    const MfmaH &H = *Bp.vm_h[q];
    auto vp = c->vv_at.find(&V);
    if (vp == c->vv_at.end()) {
      std::array<int32_t, 8> o;
      std::vector<int32_t> meta;
      for (size_t k = 0; k < V.plo.size(); k++) {
        meta.push_back(V.plo[k]);
        meta.push_back(V.pn[k]);
        meta.push_back(V.pblk[k]);
        meta.push_back(V.plast[k]);
      }
      align4();
      o[7] = put(meta);
      o[0] = put(V.rows);
      o[1] = put(V.plo);
      o[2] = put(V.pn);
      o[3] = put(V.pblk);
      o[4] = put(V.plast);
      align4();
      o[5] = put(V.w128);
      align4();
      o[6] = put(V.frag);
      vp = c->vv_at.emplace(&V, o).first;
    }
    auto hp = hplaced.find(&H);
    if (hp == hplaced.end()) {
      const int32_t first = (int32_t)Bp.vstrips.size();
      auto ht = c->mh_at.find(&H);
      if (ht == c->mh_at.end()) {
        fi_ctx::MhPlaced pl;
        pl.hwsum = put(H.wsum);
        align4();
        const int32_t frag = put(H.frag);
        const int32_t s0 = put(H.s0);
        align4();  // 16-byte aligned LUT rows (k_rs_vr's LDS-DMA)
        const int32_t lut = put(H.lut);
        align4();
        const int32_t frag2 = put(H.frag2);
        pl.hwsum2 = put(H.wsum2);
        pl.strips.reserve(H.strips.size());
        for (const MfmaStrip &st : H.strips) {
          MStrip m{};
          m.x0 = st.x0;
          m.x1 = st.x1;
          m.b0 = st.b0;
          m.nbytes = st.nbytes;
          m.c_lo = st.c_lo;
          m.ncols = st.ncols;
          m.pitch = st.pitch;
          m.nocb = st.nocb;
          m.ks = st.ks;
          m.lut_px0 = st.lut_px0;
          m.lut_n = st.lut_n;
          m.frag = frag + (int32_t)st.frag;
          m.s0 = s0 + (int32_t)st.s0;
          m.lut = lut + (int32_t)st.lut;
          m.vpitch = st.vpitch;
          m.frag2 = frag2 + (int32_t)st.frag2;
          pl.strips.push_back(m);
          // the workgroup's LDS layout follows its strip and tile kind
          pl.lds8 = std::max(pl.lds8, vm_lds_bytes(st.vpitch, st.nocb, st.ks, false));
          pl.lds16 = std::max(pl.lds16, vm_lds_bytes(st.vpitch, st.nocb, st.ks, true));
        }
        ht = c->mh_at.emplace(&H, std::move(pl)).first;
      }
      const fi_ctx::MhPlaced &pl = ht->second;
      Bp.vstrips.insert(Bp.vstrips.end(), pl.strips.begin(), pl.strips.end());
      hp = hplaced.emplace(&H, std::array<int32_t, 5>{first, pl.hwsum, pl.hwsum2, (int32_t)pl.lds8, (int32_t)pl.lds16})
               .first;
    }
    Bp.vm_lds = std::max(Bp.vm_lds, (size_t)hp->second[(d.gray || d.rot != 0) ? 4 : 3]);
    VDesc m{};
    m.src = d.src;
    m.src_stride = d.src_stride;
    m.dst = d.dst;
    m.dst_stride = d.dst_stride;
    m.ew = d.ew;
    m.eh = d.eh;
    m.rot = d.rot;
    m.gray = d.gray;
    m.rows = vp->second[0];
    m.nrows = (int32_t)V.rows.size();
    m.row0 = V.row0;
    m.rstep = V.rstep;
    m.plo = vp->second[1];
    m.pn = vp->second[2];
    m.pblk = vp->second[3];
    m.plast = vp->second[4];
    m.w128 = vp->second[5];
    m.frag = vp->second[6];
    m.pmeta = vp->second[7];
    m.hwsum = hp->second[1];
    m.nblk = V.nblk;
    work.push_back({(int32_t)Bp.vdescs.size(), hp->second[0], (int32_t)H.strips.size(), &V, Bp.vm_vt[q], hp->second[2],
                    H.shift2});
    Bp.vdescs.push_back(m);
  }
  // k_rs_vr (default; FI_VR_RS=0 turns it off): the images whose vertical axis has block-major
  // tables (fi_plan.h VrV) run on the persistent block-major kernel
  Bp.vrl.clear();
  Bp.vrtiles.clear();
  Bp.vr_info.clear();
  const double t_vr0 = now_ms();
  if (c->vr_rs) {
    std::vector<Work1> rest;
    std::vector<VrWork> vr;
    std::vector<Work1> vr_w;  // the Work1 of each vr entry (back to k_rs_vm if its launch cannot be built)
    for (const Work1 &w : work) {
      auto it = c->vrv_cache.find(w.vt);
      if (it == c->vrv_cache.end()) {
        VrV m;
        if (!build_vr_v(*w.vt, &m)) m = VrV();
        it = c->vrv_cache.emplace(w.vt, std::move(m)).first;
      }
      const VrV &V = it->second;
      const int64_t gap = V.maxgap;  // the DMA's per-lane row offset
      bool narrow = true;  // five H waves take two horizontal items each: <= 3 16-px blocks per strip
      for (int st = 0; st < w.nstrips; st++) narrow = narrow && Bp.vstrips[w.first_strip + st].nocb <= 3;
      if (V.nblk > 0 && w.hsh > 0 && narrow && gap * Bp.vdescs[w.img].src_stride < ((int64_t)1 << 31)) {
        vr.push_back({w.img, w.first_strip, w.nstrips, &V, w.hwsum2, w.hsh});
        vr_w.push_back(w);
      } else {
        rest.push_back(w);
      }
    }
    // mixed geometries (cfg4's 384 size classes x five ops) were slower on
    // k_rs_vr than on k_rs_vm in round 4 (432 vs 385 ms), hence a class cap
    // (FI_VR_MAX_CLASSES); since round 5 (4 loader waves for one-block strips,
    // their own launch) k_rs_vr takes them: cfg4 resize 363 -> 329 ms per step
    // a table's first / last (+ pad) / widest block windows and its
    // widest two consecutive blocks' rows (build_vr_tiles' `inner`)
    HashMap<const VrV *, std::array<int, 4>> wmax_of;
    std::vector<const VrV *> classes;
    classes.reserve(vr.size());
    for (const VrWork &w : vr) classes.push_back(w.V);
    std::sort(classes.begin(), classes.end());
    const int nclasses = (int)(std::unique(classes.begin(), classes.end()) - classes.begin());
    if (!vr.empty() && nclasses <= c->vr_max_classes) {
      // two launches when the batch mixes strips of one 16-px output block
      // (4 loader waves) with wider ones (2) and both halves fill the chip
      std::vector<int> grp(vr.size(), 0);
      int64_t nst[2] = {0, 0};
      for (size_t k = 0; k < vr.size(); k++) {
        int mx = 0;
        for (int st = 0; st < vr[k].nstrips; st++) mx = std::max(mx, Bp.vstrips[vr[k].first_strip + st].nocb);
        grp[k] = mx <= 1 ? 0 : 1;
        nst[grp[k]] += vr[k].nstrips;
      }
      const bool split = c->vr_split && nst[0] >= 2 * c->n_cu && nst[1] >= 2 * c->n_cu;
      for (int g = 0; g < (split ? 2 : 1); g++) {
        std::vector<VrWork> part;
        std::vector<Work1> part_w;
        for (size_t k = 0; k < vr.size(); k++)
          if (!split || grp[k] == g) {
            part.push_back(vr[k]);
            part_w.push_back(vr_w[k]);
          }
        // consecutive tiles of a workgroup's stream hold the last block window
        // of one and the first of the next in the ring together (the seam,
        // build_vr_tiles), and one failing seam sends the whole launch to
        // k_rs_vm.  Images leave (largest windows first) until the largest
        // first window plus the largest last window fit the ring, so the rest
        // chain in any order: whole-image tiles (>= 2048 strips: one band) by
        // their edge blocks' windows, banded ones by their widest window
        {
          int vpitch = 0;
          bool q16 = false;
          int64_t nstp = 0;
          for (const VrWork &w : part) {
            for (int st = 0; st < w.nstrips; st++) vpitch = std::max(vpitch, Bp.vstrips[w.first_strip + st].vpitch);
            q16 = q16 || Bp.vdescs[w.img].gray || Bp.vdescs[w.img].rot != 0;
            nstp += w.nstrips;
          }
          const int R = vr_lds_layout(vpitch, q16, 1).R;
          const bool whole = nstp >= 2048;
          std::vector<std::array<int, 3>> hl(part.size());  // head, last window, index
          for (size_t k = 0; k < part.size(); k++) {
            const VrV &V = *part[k].V;
            auto wm = wmax_of.find(&V);
            if (wm == wmax_of.end()) {
              const int32_t *bm = V.bmeta.data();
              const int nb = V.nblk;
              int w = 0, inner = bm[2] - bm[0];
              for (int b = 0; b < nb; b++) w = std::max(w, bm[4 * b + 2] - bm[4 * b]);
              for (int b = 0; b + 1 < nb; b++) inner = std::max(inner, bm[4 * (b + 1) + 2] - bm[4 * b]);
              const int glen = (bm[4 * (nb - 1) + 2] - bm[0] + 15) / 16 * 16;
              wm = wmax_of
                       .emplace(&V, std::array<int, 4>{bm[2] - bm[0], glen - (bm[4 * (nb - 1)] - bm[0]), w, inner})
                       .first;
            }
            const auto &a = wm->second;
            // a tile's first window is its first block's, its last one (K0s are
            // multiples of 16) its last block's rounded up to 16 rows
            hl[k] = whole ? std::array<int, 3>{a[0], a[1], (int)k} : std::array<int, 3>{a[2], (a[2] + 15) / 16 * 16, (int)k};
            if (a[3] > R) hl[k] = {R + 1, R + 1, (int)k};  // a block pair alone exceeds the ring: always out
          }
          std::sort(hl.begin(), hl.end(), [](const std::array<int, 3> &x, const std::array<int, 3> &y) {
            return std::max(x[0], x[1]) > std::max(y[0], y[1]);
          });
          // the fewest leading (largest) images to drop: suffix maxima of both windows
          std::vector<int> sh(hl.size() + 1, 0), sl(hl.size() + 1, 0);
          for (size_t k = hl.size(); k-- > 0;) {
            sh[k] = std::max(sh[k + 1], hl[k][0]);
            sl[k] = std::max(sl[k + 1], hl[k][1]);
          }
          size_t drop = 0;
          while (drop < hl.size() && sh[drop] + sl[drop] > R) drop++;
          if (drop > 0) {
            std::vector<char> out(part.size(), 0);
            for (size_t k = 0; k < drop; k++) out[hl[k][2]] = 1;
            std::vector<VrWork> keep;
            std::vector<Work1> keep_w;
            for (size_t k = 0; k < part.size(); k++) {
              if (out[k]) {
                rest.push_back(part_w[k]);
              } else {
                keep.push_back(part[k]);
                keep_w.push_back(part_w[k]);
              }
            }
            part.swap(keep);
            part_w.swap(keep_w);
          }
        }
        if (!part.empty() && !build_vr_tiles(c, E, Bp, part)) rest.insert(rest.end(), part_w.begin(), part_w.end());
      }
      work.swap(rest);
    }
  }
  host_stat(c, "host_plan_vr", now_ms() - t_vr0);
  // bands of blocks only when the batch is too small to fill the chip
  int64_t nst = 0;
  for (const Work1 &w : work) nst += w.nstrips;
  // XCD-aware order: the strips of one image go to one XCD queue (blockIdx % 8 under
  // round-robin dispatch) back to back, so the halo columns they share hit that L2
  // With c->vm_lpt (mixed batches: cfg4) the images go to the XCD queues by
  // LPT on their pieces and each queue runs its longest tiles first, so the
  // launch does not end on one 24 MP image's strips.
  std::vector<std::vector<VTile>> q8(8);
  std::vector<std::vector<VTile>> img_tiles(work.size());
  std::vector<int64_t> img_cost(work.size(), 0);
  for (size_t k = 0; k < work.size(); k++) {
    const Work1 &w = work[k];
    const VmV &V = *w.V;
    int bands = nst > 0 ? (int)((2048 + nst - 1) / nst) : 1;
    bands = std::max(1, std::min(bands, V.nblk));
    std::vector<int> first_piece(V.nblk + 1, (int)V.plo.size());
    for (int p = (int)V.plo.size() - 1; p >= 0; p--) first_piece[V.pblk[p]] = p;
    for (int bnd = 0; bnd < bands; bnd++) {
      const int b0 = (int)((int64_t)V.nblk * bnd / bands), b1 = (int)((int64_t)V.nblk * (bnd + 1) / bands);
      if (b1 <= b0) continue;
      const int p0 = first_piece[b0 > 0 ? b0 - 1 : 0];
      const int p1 = first_piece[b1];
      for (int st = 0; st < w.nstrips; st++) {
        img_tiles[k].push_back(VTile{w.img, w.first_strip + st, p0, p1, b0, 0});
        img_cost[k] += p1 - p0 + 1;
      }
    }
  }
  if (c->vm_lpt && work.size() > 1) {
    std::vector<int> order(work.size());
    for (size_t k = 0; k < work.size(); k++) order[k] = (int)k;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return img_cost[x] > img_cost[y]; });
    int64_t load[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k : order) {
      const int x = (int)(std::min_element(load, load + 8) - load);
      load[x] += img_cost[k];
      q8[x].insert(q8[x].end(), img_tiles[k].begin(), img_tiles[k].end());
    }
    for (auto &q : q8)
      std::stable_sort(q.begin(), q.end(), [](const VTile &x, const VTile &y) { return x.p1 - x.p0 > y.p1 - y.p0; });
  } else {
    for (size_t k = 0; k < work.size(); k++) q8[k % 8].insert(q8[k % 8].end(), img_tiles[k].begin(), img_tiles[k].end());
  }
  size_t mx = 0;
  for (auto &q : q8) mx = std::max(mx, q.size());
  for (size_t i = 0; i < mx; i++)
    for (int x = 0; x < 8; x++)
      if (i < q8[x].size()) Bp.vtiles.push_back(q8[x][i]);
}

// k_rs_hv workgroups: (image, strip, band of output blocks); bands only when
// the horizontal-first images alone would not fill the chip (each band
// re-produces the intermediate rows of its first block's window).
static void build_hv_tiles(fi_ctx *c, Exec &E, BatchPlan &Bp) {
  auto align4 = [&]() {
    while (E.ai.size() % 4) E.ai.push_back(0);
  };
  auto put = [&](const std::vector<int32_t> &v) {
    const int32_t o = E.oi();
    E.ai.insert(E.ai.end(), v.begin(), v.end());
    return o;
  };
  HashMap<const HvH *, int32_t> splaced;  // first strip in Bp.hstrips
  struct Work1 {
    int32_t img, first_strip, nstrips, nblk, nrows;
  };
  std::vector<Work1> work;
  for (size_t q = 0; q < Bp.hv_img.size(); q++) {
    const ResizeDesc &d = Bp.rd[Bp.hv_img[q]];
    const HvV &V = *Bp.hv_v[q];
    const HvH &H = *Bp.hv_h[q];
    auto vp = c->hvv_at.find(&V);
    if (vp == c->hvv_at.end()) {
      std::array<int32_t, 3> o;
      o[0] = put(V.k0ks);
      align4();
      o[1] = put(V.frag);
      o[2] = put(V.wsum);
      vp = c->hvv_at.emplace(&V, o).first;
    }
    auto hp = c->hvh_at.find(&H);
    if (hp == c->hvh_at.end()) {
      std::array<int32_t, 3> o;
      o[0] = put(H.w128);
      align4();
      o[1] = put(H.frag);
      o[2] = put(H.s0);
      hp = c->hvh_at.emplace(&H, o).first;
    }
    auto sp = splaced.find(&H);
    if (sp == splaced.end()) {
      const int32_t first = (int32_t)Bp.hstrips.size();
      for (const HvStrip &st : H.strips) {
        HvStripD m{};
        m.x0 = st.x0;
        m.x1 = st.x1;
        m.px0 = st.px0;
        m.pp = st.pp;
        m.nocb = st.nocb;
        m.frag = hp->second[1] + (int32_t)st.frag;
        m.s0 = hp->second[2] + (int32_t)st.s0;
        Bp.hstrips.push_back(m);
        Bp.hv_lds = std::max(Bp.hv_lds, hv_lds_bytes(st.pp, st.nocb));
      }
      sp = splaced.emplace(&H, first).first;
    }
    HvDesc m{};
    m.src = d.src;
    m.src_stride = d.src_stride;
    m.dst = d.dst;
    m.dst_stride = d.dst_stride;
    m.ew = d.ew;
    m.eh = d.eh;
    m.rot = d.rot;
    m.gray = d.gray;
    m.row0 = V.row0;
    m.nrows = V.nrows;
    m.nblk = V.nblk;
    m.vk = vp->second[0];
    m.vfrag = vp->second[1];
    m.vws = vp->second[2];
    m.hw128 = hp->second[0];
    m.W = Bp.hv_W[q];
    work.push_back({(int32_t)Bp.hdescs.size(), sp->second, (int32_t)H.strips.size(), V.nblk, V.nrows});
    Bp.hdescs.push_back(m);
  }
  int64_t nst = 0;
  for (const Work1 &w : work) nst += w.nstrips;
  // XCD-aware order, as build_vm_tiles (with c->vm_lpt: images by LPT on their
  // source rows x strips, each queue's tiles longest first)
  std::vector<std::vector<HvTile>> q8(8);
  std::vector<std::vector<HvTile>> img_tiles(work.size());
  std::vector<int64_t> img_cost(work.size(), 0);
  auto tile_cost = [&](const Work1 &w, const HvTile &t) { return (int64_t)(t.b1 - t.b0) * w.nrows / std::max(w.nblk, 1) + 16; };
  for (size_t k = 0; k < work.size(); k++) {
    const Work1 &w = work[k];
    constexpr int64_t target = 8192;  // workgroups the bands aim for
    int bands = nst > 0 ? (int)((target + nst - 1) / nst) : 1;
    bands = std::max(1, std::min(bands, w.nblk / 6));
    for (int bnd = 0; bnd < bands; bnd++) {
      const int b0 = (int)((int64_t)w.nblk * bnd / bands), b1 = (int)((int64_t)w.nblk * (bnd + 1) / bands);
      if (b1 <= b0) continue;
      for (int st = 0; st < w.nstrips; st++) {
        img_tiles[k].push_back(HvTile{w.img, w.first_strip + st, b0, b1});
        img_cost[k] += tile_cost(w, img_tiles[k].back());
      }
    }
  }
  if (c->vm_lpt && work.size() > 1) {
    std::vector<int> order(work.size());
    for (size_t k = 0; k < work.size(); k++) order[k] = (int)k;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return img_cost[x] > img_cost[y]; });
    std::vector<std::vector<std::pair<int64_t, HvTile>>> qc(8);
    int64_t load[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k : order) {
      const int x = (int)(std::min_element(load, load + 8) - load);
      load[x] += img_cost[k];
      for (const HvTile &t : img_tiles[k]) qc[x].push_back({tile_cost(work[k], t), t});
    }
    for (int x = 0; x < 8; x++) {
      std::stable_sort(qc[x].begin(), qc[x].end(), [](const auto &a, const auto &b) { return a.first > b.first; });
      for (const auto &e : qc[x]) q8[x].push_back(e.second);
    }
  } else {
    for (size_t k = 0; k < work.size(); k++) q8[k % 8].insert(q8[k % 8].end(), img_tiles[k].begin(), img_tiles[k].end());
  }
  size_t mx = 0;
  for (auto &q : q8) mx = std::max(mx, q.size());
  for (size_t i = 0; i < mx; i++)
    for (int x = 0; x < 8; x++)
      if (i < q8[x].size()) Bp.htiles.push_back(q8[x][i]);
}

// Pack descriptors, tiles, launch lists and the batch's new heap tables into
// the upload blob E.blob.
static void pack_batch(fi_ctx *c, Exec &E, BatchPlan &Bp, Packed &K) {
  Blob &B = E.blob;
  // one allocation for the whole blob (no regrowth copies of megabytes of tiles)
  auto bytes = [](const auto &v) { return v.size() * sizeof(v[0]) + 256; };
  B.b.reserve(B.b.size() + bytes(Bp.rd) + bytes(Bp.vdescs) + bytes(Bp.vstrips) + bytes(Bp.vtiles) +
              bytes(Bp.vrtiles) + bytes(Bp.vr_info) + bytes(Bp.hdescs) + bytes(Bp.hstrips) + bytes(Bp.htiles) +
              bytes(Bp.apply) + bytes(E.ai) + bytes(E.af) + bytes(E.ad) + 32 * sizeof(int32_t) * Bp.rd.size() +
              ((size_t)1 << 20));
  std::vector<int> m0, m1, m2, q0, q1, q2;  // q*: RGBA (matte) images of modes 0 / 1 / 2
  for (size_t k = 0; k < Bp.rd.size(); k++) {
    if (Bp.rd[k].mode >= 3) continue;
    if (Bp.rd[k].C == 4)
      (Bp.rd[k].mode == 0 ? q0 : Bp.rd[k].mode == 1 ? q1 : q2).push_back((int)k);
    else
      (Bp.rd[k].mode == 0 ? m0 : Bp.rd[k].mode == 1 ? m1 : m2).push_back((int)k);
  }
  K.all_rd_off = B.addv(Bp.rd);
  K.vdesc_off = B.addv(Bp.vdescs);
  K.vstrip_off = B.addv(Bp.vstrips);
  K.vtile_off = B.addv(Bp.vtiles);
  K.vrtile_off = B.addv(Bp.vrtiles);
  K.vrinfo_off = B.addv(Bp.vr_info);
  K.hdesc_off = B.addv(Bp.hdescs);
  K.hstrip_off = B.addv(Bp.hstrips);
  K.htile_off = B.addv(Bp.htiles);
  auto eh_tiles = [](const ResizeDesc &d) { return d.eh; };
  auto mid_tiles = [](const ResizeDesc &d) { return d.mid_rows; };
  K.L0 = add_launch(B, Bp.rd, m0, eh_tiles);
  K.L1a = add_launch(B, Bp.rd, m1, eh_tiles);
  K.h_tiled = rs_h_tile_lds(Bp.h_tile_pitch, Bp.h_tile_taps) <= 64 * 1024;
  K.L2a = K.h_tiled ? add_launch(B, Bp.rd, m2, [](const ResizeDesc &d) {
    return ((d.mid_rows + kHTileRows - 1) / kHTileRows) * ((d.ew + 255) / 256);
  }) : add_launch(B, Bp.rd, m2, mid_tiles);
  K.L2b = add_launch(B, Bp.rd, m2, eh_tiles);
  K.Q0 = add_launch(B, Bp.rd, q0, eh_tiles);
  K.Q1a = add_launch(B, Bp.rd, q1, eh_tiles);
  K.Q2a = add_launch(B, Bp.rd, q2, mid_tiles);
  K.Q2b = add_launch(B, Bp.rd, q2, eh_tiles);
  add_sc_launches(c, B, Bp.SL, Bp.sstatus, &K.SX);
  K.apply_off = B.addv(Bp.apply);
  K.mono_off = B.addv(Bp.mdesc_mono);
  for (int k = 0; k < 6; k++) {
    std::vector<int> all(Bp.cst[k].size());
    for (size_t j = 0; j < all.size(); j++) all[j] = (int)j;
    K.CL[k] = add_launch(B, Bp.cst[k], all, [](const ConvStep &st) { return st.H; });
  }
  if (!Bp.mono.empty() && c->mono_wts_at >= 0) K.mono_wts = (size_t)c->mono_wts_at;
  if (!Bp.mono.empty() && c->mono_wts_at < 0) {
    // the Riemersma error-queue weights (quantize.c), computed with libm at run
    // time exactly as oracle/fi_oracle.c does
    K.mono_wts = (size_t)E.od();
    c->mono_wts_at = (int32_t)K.mono_wts;
    volatile double qr1 = 65535.0 + 1.0, span = 16 - 1.0;
    const double step = exp(log((double)qr1) / (double)span);
    double weight = 1.0, wts[16];
    for (int k = 0; k < 16; k++) {
      wts[16 - k - 1] = 1.0 / weight;
      weight *= step;
    }
    E.ad.insert(E.ad.end(), wts, wts + 16);
  }
  K.ai_off = B.addv(E.ai);
  K.af_off = B.addv(E.af);
  K.ad_off = B.addv(E.ad);
}

// Enqueue the batch: resample, convolutions, -monochrome and the smartcrop
// stage on the main stream (sc_stream is the same stream); the crop apply on
// ap_stream behind this batch's smartcrop stage, so it runs beside the next
// batch's resample (FI_APPLY_OVERLAP=0: on the main stream).  ap_tail marks
// the last apply for the entry points that must not run before it
// (order_after_apply).
static int launch_batch(fi_ctx *c, const Exec &E, const BatchPlan &Bp, const Packed &K, uint8_t *ab, uint8_t *wb,
                        Slot &S) {
  S.tail = c->sc_stream;
  S.ap_lo = S.ap_hi = 0;
  const int32_t *ai = (const int32_t *)c->heap_i.p;
  const float *af = (const float *)c->heap_f.p;
  const double *ad = (const double *)c->heap_d.p;
  const ScParamsDev PD = to_dev(E.params);
  auto desc_p = [&](const Launch &L) { return ab + L.desc_off; };
  auto pre_p = [&](const Launch &L) { return (const int32_t *)(ab + L.prefix_off); };
  Timer tb(c, "batch", 0, c->stream, c->sc_stream);
  {
    Timer t(c, "resize", Bp.resize_bytes);
    if (K.L0.tiles)
      hipLaunchKernelGGL(k_rs_copy, dim3(K.L0.tiles), dim3(256), 0, c->stream, (const ResizeDesc *)desc_p(K.L0),
                         pre_p(K.L0), K.L0.n);
    const bool fork = c->vr_fork && c->rs2_stream && Bp.vrl.size() >= 2;
    if (fork) {
      if (!c->rs_fork) HIP_TRY(hipEventCreateWithFlags(&c->rs_fork, hipEventDisableTiming));
      if (!c->rs_join) HIP_TRY(hipEventCreateWithFlags(&c->rs_join, hipEventDisableTiming));
      HIP_TRY(hipEventRecord(c->rs_fork, c->stream));
      HIP_TRY(hipStreamWaitEvent(c->rs2_stream, c->rs_fork, 0));
      c->stats["vr_fork"].launches += 1;
    }
    // the join, at the end of the resize scope (before its timer's end event)
    // and on every early error return, so no forked launch outlives the stage
    struct Join {
      fi_ctx *c;
      bool on;
      ~Join() {
        if (!on) return;
        if (hipEventRecord(c->rs_join, c->rs2_stream) != hipSuccess ||
            hipStreamWaitEvent(c->stream, c->rs_join, 0) != hipSuccess)
          (void)hipStreamSynchronize(c->rs2_stream);
      }
    } join{c, fork};
    for (const BatchPlan::VrLaunch &V : Bp.vrl) {
      hipStream_t vs = fork && &V != &Bp.vrl[0] ? c->rs2_stream : c->stream;
      const int vrc = launch_vr(vs, (const VDesc *)(ab + K.vdesc_off), (const MStrip *)(ab + K.vstrip_off),
                                (const VrTile *)(ab + K.vrtile_off) + V.tile0, V.ntiles,
                                (const int32_t *)(ab + K.vrinfo_off) + V.info0, V.G, ai, V.L);
      if (vrc < 0) return set_err(FI_EDEVICE, "block-major MFMA resample launch rejected (LDS %d)", V.L.total);
      if (vrc == 1) c->stats["vr_ablation"].launches += 1;  // FI_VR_VARIANT ablation: wrong pixels
      c->stats["path_vr"].launches += V.images;
      c->stats["path_vm"].launches -= V.images;
    }
    if (!Bp.vtiles.empty() &&
               launch_vm(c->stream, (const VDesc *)(ab + K.vdesc_off), (const MStrip *)(ab + K.vstrip_off),
                         (const VTile *)(ab + K.vtile_off), (int)Bp.vtiles.size(), ai, Bp.vm_lds) != 0)
      return set_err(FI_EDEVICE, "streaming MFMA resample launch rejected (LDS %zu)", Bp.vm_lds);
    // (k_rs_hv on a stream of its own beside k_rs_vm was measured: cfg4 102.1
    // vs 102.5 ms/step -- k_rs_vm's LDS leaves no CU room to overlap into)
    if (!Bp.htiles.empty() &&
        launch_hv(c->stream, (const HvDesc *)(ab + K.hdesc_off), (const HvStripD *)(ab + K.hstrip_off),
                  (const HvTile *)(ab + K.htile_off), (int)Bp.htiles.size(), ai, Bp.hv_lds) != 0)
      return set_err(FI_EDEVICE, "horizontal-first MFMA resample launch rejected (LDS %zu)", Bp.hv_lds);
    if (K.Q0.tiles || K.Q1a.tiles || K.Q2a.tiles) {
      const ResizeDesc *dq0 = (const ResizeDesc *)desc_p(K.Q0), *dq1 = (const ResizeDesc *)desc_p(K.Q1a),
                       *dq2a = (const ResizeDesc *)desc_p(K.Q2a), *dq2b = (const ResizeDesc *)desc_p(K.Q2b);
      launch_rs4(c->stream, 0, dq0, pre_p(K.Q0), K.Q0.n, K.Q0.tiles, nullptr, nullptr, 0, 0, ai, ad);
      launch_rs4(c->stream, 1, dq1, pre_p(K.Q1a), K.Q1a.n, K.Q1a.tiles, dq1, pre_p(K.Q1a), K.Q1a.n, K.Q1a.tiles, ai,
                 ad);
      launch_rs4(c->stream, 2, dq2a, pre_p(K.Q2a), K.Q2a.n, K.Q2a.tiles, dq2b, pre_p(K.Q2b), K.Q2b.n, K.Q2b.tiles,
                 ai, ad);
    }
    if (K.L1a.tiles) {
      hipLaunchKernelGGL(k_rs_v_u8, dim3(K.L1a.tiles), dim3(256), 0, c->stream, (const ResizeDesc *)desc_p(K.L1a),
                         pre_p(K.L1a), K.L1a.n, ai, af);
      hipLaunchKernelGGL(k_rs_h_final, dim3(K.L1a.tiles), dim3(256), 0, c->stream,
                         (const ResizeDesc *)desc_p(K.L1a), pre_p(K.L1a), K.L1a.n, ai, af);
    }
    if (K.L2a.tiles) {
      if (K.h_tiled)
        launch_rs_h_tile(c->stream, (const ResizeDesc *)desc_p(K.L2a), pre_p(K.L2a), K.L2a.n, K.L2a.tiles, ai, af,
                         Bp.h_tile_pitch, Bp.h_tile_taps);
      else
        hipLaunchKernelGGL(k_rs_h_u8, dim3(K.L2a.tiles), dim3(256), 0, c->stream, (const ResizeDesc *)desc_p(K.L2a),
                           pre_p(K.L2a), K.L2a.n, ai, af);
      hipLaunchKernelGGL(k_rs_v_final, dim3(K.L2b.tiles), dim3(256), 0, c->stream,
                         (const ResizeDesc *)desc_p(K.L2b), pre_p(K.L2b), K.L2b.n, ai, af);
    }
  }
  if (!Bp.conv_items.empty()) {
    Timer t(c, "conv", 0);
    static const int kMode[6] = {0, 2, 3, 0, 1, 4};
    for (int k = 0; k < 6; k++)
      launch_conv(c->stream, kMode[k], (const ConvStep *)desc_p(K.CL[k]), pre_p(K.CL[k]), K.CL[k].n, K.CL[k].tiles,
                  ad);
  }
  if (!Bp.mono.empty()) {
    Timer t(c, "mono", 0);
    (void)launch_mono(c->stream, (const MonoDesc *)(ab + K.mono_off), (int)Bp.mono.size(), ad + K.mono_wts);
  }
  HIP_TRY(hipGetLastError());
  // a smartcrop stage made only of co-resident kernels (k_sc_hx / k_sc_vx, the
  // score, the apply) runs on ap_stream behind this batch's resample, beside
  // the next batch's
  const bool beside = c->sc_cx == 3 && c->apply_overlap && c->ap_stream && K.SX.ncx > 0 && K.SX.ncx == K.SX.nok;
  hipStream_t scs = c->sc_stream;
  if (c->sc_stream != c->stream || beside) {
    if (beside) scs = c->ap_stream;
    if (!S.rs_done) HIP_TRY(hipEventCreateWithFlags(&S.rs_done, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(S.rs_done, c->stream));
    HIP_TRY(hipStreamWaitEvent(scs, S.rs_done, 0));
  }
  if (K.SX.nsl + K.SX.nsg + K.SX.ns3 > 0) {
    const int rc = enqueue_sc(c, scs, ab, K.SX, ai, ad, (CropScore *)(wb + Bp.scores_off),
                              (ScResult *)(wb + Bp.results_off), PD);
    if (rc) return rc;
    if (beside) {
      S.tail = scs;
      tb.sb = scs;
    }
    if (!Bp.apply.empty()) {
      hipStream_t as = scs;
      int pw = 0;
      if (beside) {
        pw = c->n_cu;
      } else if (c->apply_overlap && c->ap_stream) {
        if (!S.sc_done) HIP_TRY(hipEventCreateWithFlags(&S.sc_done, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(S.sc_done, c->sc_stream));
        HIP_TRY(hipStreamWaitEvent(c->ap_stream, S.sc_done, 0));
        as = c->ap_stream;
        pw = c->n_cu;
        S.tail = as;
        tb.sb = as;  // the batch range ends with its apply
      }
      {
        Timer t(c, "crop_apply", 0, as, as);
        (void)launch_crop_apply(as, (const ApplyDesc *)(ab + K.apply_off), (int)Bp.apply.size(),
                                (const DevCrop *)(ab + K.SX.crops_off), (const ScResult *)(wb + Bp.results_off), pw);
      }
      if (as == c->ap_stream) {
        if (!c->ap_tail) HIP_TRY(hipEventCreateWithFlags(&c->ap_tail, hipEventDisableTiming));
        // (as in the overlapped apply; the smartcrop kernels beside it write only the slot's workspace)
        HIP_TRY(hipEventRecord(c->ap_tail, as));
        c->ap_pending = true;
        // the bytes this apply writes (a crop is at most the resized image)
        S.ap_lo = UINTPTR_MAX;
        S.ap_hi = 0;
        for (const ApplyDesc &a : Bp.apply) {
          S.ap_lo = std::min(S.ap_lo, (uintptr_t)a.dst);
          S.ap_hi = std::max(S.ap_hi, (uintptr_t)a.dst + (uintptr_t)a.W * a.H * a.C);
        }
      }
    } else if (beside) {
      if (!c->ap_tail) HIP_TRY(hipEventCreateWithFlags(&c->ap_tail, hipEventDisableTiming));
      HIP_TRY(hipEventRecord(c->ap_tail, scs));
      c->ap_pending = true;
    }
    HIP_TRY(hipGetLastError());
  }
  return FI_OK;
}

// Per-image result records into the slot's pinned readback; the batch joins
// the in-flight list (finalize_front fills the caller's records).
static int queue_readback(fi_ctx *c, BatchPlan &Bp, int slot, uint8_t *wb, double t_start,
                          std::shared_ptr<HostIo> host) {
  Slot &S = c->slots[slot];
  // device outputs: the few result bytes go back on the batch's own stream
  // (a cross-stream event costs the next batch's first kernel ~20-30 us of
  // idle GPU, measured in round 5's kernel trace); host outputs (image bytes)
  // on the readback stream, so the next batch's kernels overlap their copies
  hipStream_t tail = S.tail ? S.tail : c->sc_stream;
  hipStream_t rs = host ? c->rb_stream : tail;
  if (rs != tail) {
    if (!S.sc_end) HIP_TRY(hipEventCreateWithFlags(&S.sc_end, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(S.sc_end, tail));
    HIP_TRY(hipStreamWaitEvent(rs, S.sc_end, 0));
  }
  if (host) {
    // outputs to the host, behind the batch's last kernel on sc_stream: the
    // planned (pre-apply) bytes cover the applied crop, which is never larger
    double obytes = 0;
    for (int i = 0; i < Bp.n; i++)
      if (Bp.status[i] == FI_OK && host->user[i].dst) obytes += (double)Bp.imgs[i].out_stride * Bp.imgs[i].out_h;
    Timer t(c, "d2h_out", obytes, rs, rs);
    for (int i = 0; i < Bp.n; i++) {
      const fi_image &d = Bp.imgs[i];
      if (Bp.status[i] != FI_OK || !host->user[i].dst) continue;
      const size_t bytes = (size_t)d.out_stride * d.out_h;
      uint8_t *to = host->pin_off[i] < 0 ? host->user[i].dst : (uint8_t *)S.hpin + host->pin_off[i];
      HIP_TRY(hipMemcpyAsync(to, (uint8_t *)S.hio.p + host->dev_dst_off[i], bytes, hipMemcpyDeviceToHost,
                             rs));
    }
  }
  uint8_t *rp = (uint8_t *)S.res;
  const size_t res_bytes = sizeof(ScResult) * Bp.sitems.size();
  const size_t outwh_bytes = sizeof(int32_t) * 2 * (size_t)Bp.n;
  if (!Bp.sitems.empty())
    HIP_TRY(hipMemcpyAsync(rp, wb + Bp.results_off, res_bytes, hipMemcpyDeviceToHost, rs));
  if (!Bp.apply.empty())
    HIP_TRY(hipMemcpyAsync(rp + res_bytes, wb + Bp.outwh_off, outwh_bytes, hipMemcpyDeviceToHost, rs));
  if (!S.done) HIP_TRY(hipEventCreateWithFlags(&S.done, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(S.done, rs));
  S.busy = true;
  c->next_slot = (slot + 1) % kSlots;
  PendingBatch pb;
  pb.imgs = Bp.imgs;
  pb.n = Bp.n;
  pb.slot = slot;
  pb.t_start = t_start;
  pb.status = std::move(Bp.status);
  pb.errs = std::move(Bp.errs);
  pb.sc_of = std::move(Bp.sc_of);
  pb.sstatus = std::move(Bp.sstatus);
  pb.serrs = std::move(Bp.serrs);
  pb.crop0.resize(Bp.SL.descs.size());
  for (size_t k = 0; k < Bp.SL.descs.size(); k++) pb.crop0[k] = Bp.SL.descs[k].crop0;
  pb.crops = std::move(Bp.SL.crops);
  pb.nres = Bp.sitems.size();
  pb.any_apply = !Bp.apply.empty();
  pb.timers.swap(c->pending);  // waited for when this batch is finalized
  pb.host = std::move(host);
  c->inflight.push_back(std::move(pb));
  return FI_OK;
}

static int drain(fi_ctx *c);
static int wait_slot(fi_ctx *c, int slot);
static int run_batch(fi_ctx *c, fi_image *imgs, int32_t n, bool async, std::shared_ptr<HostIo> host = nullptr) {
  const double t_start = now_ms();
  Exec E;
  E.c = c;
  fi_smartcrop_default_params(&E.params);
  int rc = heap_prepare(c, E);
  if (rc) return rc;
  BatchPlan Bp;
  Bp.imgs = imgs;
  Bp.n = n;
  Bp.plans.resize(n);
  Bp.status.assign(n, FI_OK);
  Bp.errs.resize(n);
  Bp.rd_of.assign(n, -1);
  Bp.sc_of.assign(n, -1);
  Bp.res_off.assign(n, 0);
  Bp.res_stride.assign(n, 0);
  Bp.out_of.assign(n, nullptr);
  for (int i = 0; i < n; i++) plan_image(c, E, Bp, i);
  const double t_images = now_ms();
  plan_batch_sc(c, E, Bp);
  // the batch's slot: pinned staging + device blob/workspace (the batch that
  // used it last must be done before anything here is overwritten)
  const int slot = c->next_slot;
  rc = wait_slot(c, slot);
  if (rc) return rc;
  Slot &S = c->slots[slot];
  rc = ensure(c, &S.work, E.work.size + 256);
  if (rc) return rc;
  uint8_t *wb = (uint8_t *)S.work.p;
  resolve_workspace(E, Bp, wb);
  const double t_sc = now_ms();
  const double t_tiles0 = now_ms();
  build_vm_tiles(c, E, Bp);
  const double t_tiles1 = now_ms();
  build_hv_tiles(c, E, Bp);
  const double t_tiles = now_ms();
  host_stat(c, "host_plan_hv", t_tiles - t_tiles1);
  Packed K;
  pack_batch(c, E, Bp, K);
  if (!heap_fits(c, E)) {
    // the batch's new tables overflow the heaps: start them empty and plan again
    if (c->heap_retry) return set_err(FI_ENOMEM, "batch tables exceed the device table heap");
    heap_reset(c);
    c->heap_retry = true;
    const int rrc = run_batch(c, imgs, n, async, host);
    c->heap_retry = false;
    return rrc;
  }
  // ---- upload (pinned slot: the previous batch may still be running)
  const Blob &B = E.blob;
  rc = ensure(c, &S.arena, B.b.size() + 256);
  if (rc) return rc;
  rc = ensure_pinned_buf(&S.blob, &S.blob_cap, B.b.size() + 256);
  if (rc) return rc;
  rc = ensure_pinned_buf(&S.res, &S.res_cap, sizeof(ScResult) * Bp.sitems.size() + sizeof(int32_t) * 2 * (size_t)n + 64);
  if (rc) return rc;
  memcpy(S.blob, B.b.data(), B.b.size());
  HIP_TRY(hipMemcpyAsync(S.arena.p, S.blob, B.b.size(), hipMemcpyHostToDevice, c->up_stream));
  if (!S.up_done) HIP_TRY(hipEventCreateWithFlags(&S.up_done, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(S.up_done, c->up_stream));
  // device-resident batches: the upload stream carries only this small blob,
  // and the host runs batches ahead of the GPU, so it waits for the copy
  // itself rather than putting a wait packet between the previous batch's
  // score and this batch's resample (measured: that gap 18 -> 11 us per cfg2
  // step); host-buffer batches upload their sources on that stream too
  if (c->up_hostsync && !host)
    HIP_TRY(hipEventSynchronize(S.up_done));
  else
    HIP_TRY(hipStreamWaitEvent(c->stream, S.up_done, 0));
  const double t_planned = now_ms();
  host_stat(c, "host_plan", t_planned - t_start);
  host_stat(c, "host_plan_images", t_images - t_start);
  host_stat(c, "host_plan_sc", t_sc - t_images);
  host_stat(c, "host_plan_tiles", t_tiles - t_sc);
  host_stat(c, "host_plan_vmtiles", t_tiles - t_tiles0);
  host_stat(c, "host_plan_blob", t_planned - t_tiles);
  if (c->timing) c->stats["host_plan"].bytes += (double)B.b.size();
  uint8_t *ab = (uint8_t *)S.arena.p;
  // a source that an earlier batch's overlapped crop apply is still writing
  // (a chained request: this batch resizes that batch's output): the resample
  // waits for the applies (bounding ranges: a false hit only costs the overlap)
  for (const Slot &o : c->slots) {
    if (&o == &S || o.ap_hi <= o.ap_lo) continue;
    bool hit = false;
    for (int i = 0; i < n && !hit; i++) {
      const fi_image &im = imgs[i];
      if (!im.src || im.src_h <= 0 || im.src_stride <= 0) continue;
      const uintptr_t s0 = (uintptr_t)im.src, s1 = s0 + (uintptr_t)im.src_stride * (uintptr_t)im.src_h;
      hit = s0 < o.ap_hi && o.ap_lo < s1;
    }
    if (hit && order_after_apply(c) != FI_OK) return set_err(FI_EDEVICE, "hipStreamWaitEvent failed");
  }
  rc = heap_commit(c, E, ab, K.ai_off, K.af_off, K.ad_off);
  if (rc) return rc;
  rc = launch_batch(c, E, Bp, K, ab, wb, S);
  if (rc) return rc;
  rc = queue_readback(c, Bp, slot, wb, t_start, host);
  if (rc) return rc;
  host_stat(c, "host_launch", now_ms() - t_planned);
  if (async) return FI_OK;
  return drain(c);
}

// Wait for the oldest in-flight batch and fill its fi_image records.
static int finalize_front(fi_ctx *c) {
  PendingBatch pb = std::move(c->inflight.front());
  c->inflight.erase(c->inflight.begin());
  Slot &S = c->slots[pb.slot];
  const double t_wait = now_ms();
  HIP_TRY(hipEventSynchronize(S.done));
  S.busy = false;
  S.ap_lo = S.ap_hi = 0;  // its apply is done (S.done follows it on the tail stream)
  if (c->inflight.empty()) c->ap_pending = false;
  collect_ranges(c, pb.timers);
  const double t_done = now_ms();
  host_stat(c, "host_wait", t_done - t_wait);
  const ScResult *res = (const ScResult *)S.res;
  const int32_t *outwh = (const int32_t *)((const uint8_t *)S.res + sizeof(ScResult) * pb.nres);
  int first_bad = FI_OK;
  std::string first_err;
  for (int i = 0; i < pb.n; i++) {
    fi_image &im = pb.imgs[i];
    im.n_candidates = 0;
    if (pb.status[i] == FI_OK && pb.sc_of[i] >= 0) {
      const int k = pb.sc_of[i];
      if (pb.sstatus[k] != FI_OK) {
        pb.status[i] = pb.sstatus[k];
        pb.errs[i] = pb.serrs[k];
      } else {
        const ScResult &r = res[k];
        if (r.top < 0) {
          pb.status[i] = FI_EUNSUPPORTED;
          pb.errs[i] = "smartcrop: too many crop windows for the scoring kernel";
        } else {
          const DevCrop &dc = pb.crops[pb.crop0[k] + r.top];
          im.crop_x = dc.rx;
          im.crop_y = dc.ry;
          im.crop_w = dc.rw;
          im.crop_h = dc.rh;
          im.crop_score = r.total;
          im.n_candidates = r.n_candidates;
          if ((im.flags & FI_OP_SMARTCROP_APPLY) && pb.any_apply) {
            im.out_w = outwh[2 * i];
            im.out_h = outwh[2 * i + 1];
            im.out_stride = im.out_w * im.out_channels;
          }
        }
      }
    }
    im.status = pb.status[i];
    if (pb.status[i] != FI_OK && first_bad == FI_OK) {
      first_bad = pb.status[i];
      first_err = "image " + std::to_string(i) + ": " + pb.errs[i];
    }
    if (pb.host) {  // host-buffer batch: the caller's record, and its staged output
      fi_image &o = pb.host->user[i];
      o.out_w = im.out_w;
      o.out_h = im.out_h;
      o.out_channels = im.out_channels;
      o.out_stride = im.out_stride;
      o.crop_x = im.crop_x;
      o.crop_y = im.crop_y;
      o.crop_w = im.crop_w;
      o.crop_h = im.crop_h;
      o.crop_score = im.crop_score;
      o.status = im.status;
      o.n_candidates = im.n_candidates;
      if (im.status == FI_OK && o.dst && pb.host->pin_off[i] >= 0)
        memcpy(o.dst, (const uint8_t *)S.hpin + pb.host->pin_off[i], (size_t)im.out_stride * im.out_h);
    }
  }
  host_stat(c, "host_total", now_ms() - pb.t_start);
  if (first_bad != FI_OK) return set_err(first_bad, "%s", first_err.c_str());
  return FI_OK;
}
// Finalize every in-flight batch (in order); returns the first error.
static int drain(fi_ctx *c) {
  int first = FI_OK;
  while (!c->inflight.empty()) {
    const int rc = finalize_front(c);
    if (rc != FI_OK && first == FI_OK) first = rc;
  }
  if (first != FI_OK) return first;  // message of the first failure is in g_err... of the last
  return FI_OK;
}
static int wait_slot(fi_ctx *c, int slot) {
  int first = FI_OK;
  while (c->slots[slot].busy && !c->inflight.empty()) {
    const int rc = finalize_front(c);
    if (rc != FI_OK && first == FI_OK) first = rc;
  }
  return first;
}

// ---------------------------------------------------------------------------
// smartcrop-only path (fi_smartcrop / fi_smartcrop_ex)
// ---------------------------------------------------------------------------
static int run_smartcrop(fi_ctx *c, const uint8_t *d_img, int W, int H, int64_t stride, int C, int tw, int th,
                         const fi_smartcrop_params &params, const fi_smartcrop_options &opt,
                         std::vector<CropScore> *scores, ScResult *result, ScPlan *plan_out,
                         std::vector<uint8_t> *prescaled, std::vector<uint8_t> *maps) {
  Exec E;
  E.c = c;
  E.params = params;
  {
    const int hrc = heap_prepare(c, E);
    if (hrc) return hrc;
  }
  std::vector<ScItem> items(1);
  items[0].img = d_img;
  items[0].stride = stride;
  items[0].W = W;
  items[0].H = H;
  items[0].C = C;
  items[0].tw = tw;
  items[0].th = th;
  items[0].result = 0;
  items[0].opt = opt;
  items[0].padded = true;  // the caller (fi_smartcrop_ex) staged it at a 16-B rounded pitch, + 256 B
  ScLaunchData SL;
  std::vector<int> st(1, FI_OK);
  std::vector<std::string> errs(1);
  plan_smartcrop(c, E, items, &SL, &st, &errs, prescaled != nullptr);
  if (st[0] != FI_OK) return set_err(st[0], "%s", errs[0].c_str());
  *plan_out = *SL.plans[0];
  const size_t results_off = E.work.take(sizeof(ScResult));
  const size_t scores_off = E.work.take(sizeof(CropScore) * std::max(SL.nscores, 1));
  int rc = ensure(c, &c->work, E.work.size + 256);
  if (rc) return rc;
  uint8_t *wb = (uint8_t *)c->work.p;
  ScDesc &d = SL.descs[0];
  fix_ptr(d.red, wb);
  fix_ptr(d.hbuf, wb);
  fix_ptr(d.tbuf, wb);
  fix_ptr(d.pre, wb);
  fix_ptr(d.maps, wb);
  Blob &B = E.blob;
  ScLaunches SX;
  add_sc_launches(c, B, SL, st, &SX);
  const size_t ai_off = B.addv(E.ai), af_off = B.addv(E.af), ad_off = B.addv(E.ad);
  if (!heap_fits(c, E)) return set_err(FI_ENOMEM, "smartcrop tables exceed the device table heap");
  rc = ensure(c, &c->arena, B.b.size() + 256);
  if (rc) return rc;
  rc = ensure_pinned(c, B.b.size() + 256);
  if (rc) return rc;
  memcpy(c->pinned, B.b.data(), B.b.size());
  HIP_TRY(hipMemcpyAsync(c->arena.p, c->pinned, B.b.size(), hipMemcpyHostToDevice, c->stream));
  uint8_t *ab = (uint8_t *)c->arena.p;
  rc = heap_commit(c, E, ab, ai_off, af_off, ad_off);
  if (rc) return rc;
  rc = enqueue_sc(c, c->stream, ab, SX, (const int32_t *)c->heap_i.p, (const double *)c->heap_d.p,
                  (CropScore *)(wb + scores_off), (ScResult *)(wb + results_off), to_dev(params));
  if (rc) return rc;
  scores->resize(SL.nscores);
  HIP_TRY(hipMemcpyAsync(scores->data(), wb + scores_off, sizeof(CropScore) * SL.nscores, hipMemcpyDeviceToHost,
                         c->stream));
  HIP_TRY(hipMemcpyAsync(result, wb + results_off, sizeof(ScResult), hipMemcpyDeviceToHost, c->stream));
  const size_t na = (size_t)d.aw * d.ah;
  if (prescaled) {
    prescaled->resize(na * 3);
    if (d.pre) {
      HIP_TRY(hipMemcpyAsync(prescaled->data(), d.pre, na * 3, hipMemcpyDeviceToHost, c->stream));
    } else {
      // no prescale: the analysed image is the input (C may be 1)
      std::vector<uint8_t> tmp((size_t)stride * H);
      HIP_TRY(hipMemcpyAsync(tmp.data(), d_img, tmp.size(), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++)
          for (int k = 0; k < 3; k++) (*prescaled)[((size_t)y * W + x) * 3 + k] = tmp[(size_t)y * stride + x * C + (C == 3 ? k : 0)];
    }
  }
  std::vector<uint32_t> pm;
  if (maps) {
    pm.resize(na);
    HIP_TRY(hipMemcpyAsync(pm.data(), d.maps, na * 4, hipMemcpyDeviceToHost, c->stream));
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  collect_timers(c);
  if (maps) {
    maps->resize(na * 3);
    for (size_t i = 0; i < na; i++) {
      (*maps)[i * 3 + 0] = pm[i] & 255;
      (*maps)[i * 3 + 1] = (pm[i] >> 8) & 255;
      (*maps)[i * 3 + 2] = (pm[i] >> 16) & 255;
    }
  }
  if (result->top < 0) return set_err(FI_EUNSUPPORTED, "smartcrop: scoring kernel rejected the crop count");
  return FI_OK;
}

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
// face-blur pixelation (fi_pixelate.hip): per box, the crop's 10% ScaleImage
// into a Q16 scratch, then its 1000% ScaleImage onto the image at (X, Y).
static int pixelate_device(fi_ctx *c, uint8_t *img, int w, int h, int64_t stride, int C, const int32_t *boxes,
                           int nboxes) {
  if (!img || w <= 0 || h <= 0 || (C != 1 && C != 3) || stride < (int64_t)w * C || nboxes < 0 ||
      (nboxes > 0 && !boxes))
    return set_err(FI_EINVAL, "bad pixelate arguments");
  std::vector<int32_t> ti;
  std::vector<double> td;
  struct Box {
    PixPass down, up;
  };
  std::vector<Box> plan;
  size_t scratch = 0;
  int first_bad = -1;
  std::string why;
  auto put = [&](const ScaleList &L, int32_t *off, int32_t *idx, int32_t *wt) {
    *off = (int32_t)ti.size();
    ti.insert(ti.end(), L.off.begin(), L.off.end());
    *idx = (int32_t)ti.size();
    ti.insert(ti.end(), L.idx.begin(), L.idx.end());
    *wt = (int32_t)td.size();
    td.insert(td.end(), L.w.begin(), L.w.end());
  };
  for (int b = 0; b < nboxes; b++) {
    const int bx = boxes[4 * b], by = boxes[4 * b + 1], bw = boxes[4 * b + 2], bh = boxes[4 * b + 3];
    if (bw <= 0 || bh <= 0 || bx < 0 || by < 0 || bx >= w || by >= h) {
      first_bad = b;
      why = "geometry does not contain image";
      break;
    }
    const int rw = std::min(bw, w - bx), rh = std::min(bh, h - by);  // CropImage clip
    const int dw = im_percent_size(rw, 10.0), dh = im_percent_size(rh, 10.0);
    if (dw <= 0 || dh <= 0) {
      first_bad = b;
      why = "NegativeOrZeroImageSize (the 10% scale is empty)";
      break;
    }
    const int uw = im_percent_size(dw, 1000.0), uh = im_percent_size(dh, 1000.0);
    Box B{};
    ScaleList L;
    im_scale_rows(rh, dh, &L);
    put(L, &B.down.yoff, &B.down.yidx, &B.down.yw);
    im_scale_cols(rw, dw, &L);
    put(L, &B.down.xoff, &B.down.xidx, &B.down.xw);
    im_scale_rows(dh, uh, &L);
    put(L, &B.up.yoff, &B.up.yidx, &B.up.yw);
    im_scale_cols(dw, uw, &L);
    put(L, &B.up.xoff, &B.up.xidx, &B.up.xw);
    B.down.src8 = img + (int64_t)by * stride + (int64_t)bx * C;
    B.down.sstride = stride;
    B.down.iw = rw;
    B.down.ih = rh;
    B.down.ow = dw;
    B.down.oh = dh;
    B.down.C = C;
    B.down.dst16 = (uint16_t *)(uintptr_t)(scratch + 1);  // tagged: resolved after upload
    B.up.src16 = B.down.dst16;
    B.up.iw = dw;
    B.up.ih = dh;
    B.up.ow = uw;
    B.up.oh = uh;
    B.up.C = C;
    B.up.dst8 = img + (int64_t)by * stride + (int64_t)bx * C;
    B.up.dstride = stride;
    B.up.clip_w = w - bx;  // composite at (X, Y), clipped to the canvas
    B.up.clip_h = h - by;
    scratch += ((size_t)dw * dh * C * 2 + 255) / 256 * 256;
    plan.push_back(B);
  }
  const size_t ti_bytes = ti.size() * 4, td_off = (ti_bytes + 255) / 256 * 256;
  const size_t sc_off = (td_off + td.size() * 8 + 255) / 256 * 256;
  int rc = ensure(c, &c->pix, sc_off + scratch + 256);
  if (rc) return rc;
  uint8_t *pb = (uint8_t *)c->pix.p;
  rc = ensure_pinned(c, sc_off);
  if (rc) return rc;
  memcpy(c->pinned, ti.data(), ti_bytes);
  memcpy((uint8_t *)c->pinned + td_off, td.data(), td.size() * 8);
  if (sc_off) HIP_TRY(hipMemcpyAsync(pb, c->pinned, sc_off, hipMemcpyHostToDevice, c->stream));
  const int32_t *ai = (const int32_t *)pb;
  const double *ad = (const double *)(pb + td_off);
  for (Box &B : plan) {
    fix_ptr(B.down.dst16, pb + sc_off);
    B.up.src16 = B.down.dst16;
    launch_pix(c->stream, 0, B.down, ai, ad);
    launch_pix(c->stream, 1, B.up, ai, ad);
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));  // the pinned lists are reused by the next call
  if (first_bad >= 0) return set_err(FI_EINVAL, "pixelate box %d: %s", first_bad, why.c_str());
  return FI_OK;
}

// ---------------------------------------------------------------------------
extern "C" {

int32_t fi_abi_version(void) { return FI_ABI_VERSION; }
// profiling only (not in the public header): k_rs_vm MODE 9 phase sums, 8 u64 per workgroup
int fi_debug_vm_stamps(fi_ctx *c, uint64_t *out, int32_t slots) {
  if (!c || !out) return FI_EINVAL;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return vm_read_stamps(out, slots) == 0 ? FI_OK : FI_EDEVICE;
}
int fi_debug_vr_stamps(fi_ctx *c, uint64_t *out, int32_t slots) {
  if (!c || !out) return FI_EINVAL;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return vr_read_stamps(out, slots) == 0 ? FI_OK : FI_EDEVICE;
}
// GPU JPEG decode (fi_jpeg.hip): the decode half of the host codec pipeline
// (ImageProcessor's `convert` reads the source with libjpeg) on the device
int fi_jpeg_info(const uint8_t *data, size_t len, int32_t *w, int32_t *h, int32_t *channels) {
  if (!data || !w || !h || !channels) return set_err(FI_EINVAL, "bad arguments");
  int W = 0, H = 0, C = 0;
  const int rc = jpeg_info(data, len, &W, &H, &C);
  if (rc) return set_err(rc, rc == FI_EUNSUPPORTED ? "JPEG stream the GPU decoder does not handle" : "malformed JPEG");
  *w = W;
  *h = H;
  *channels = C;
  return FI_OK;
}
static void *jpeg_alloc(void *actx, int which, size_t bytes) {
  fi_ctx *c = static_cast<fi_ctx *>(actx);
  if (which == 3)  // pinned host staging (the previous call has synchronised)
    return ensure_pinned_buf(&c->jpeg_host, &c->jpeg_host_cap, bytes) == FI_OK ? c->jpeg_host : nullptr;
  return ensure(c, &c->jpeg[which], bytes) == FI_OK ? c->jpeg[which].p : nullptr;
}
int fi_jpeg_decode_device(fi_ctx *c, const uint8_t *const *data, const size_t *len, int32_t n, uint8_t *const *dst,
                          const int64_t *dst_stride, int32_t out_channels, int32_t *status) {
  if (!c || n < 0 || (n > 0 && (!data || !len || !dst || !dst_stride || !status)) ||
      (out_channels != 0 && out_channels != 3))
    return set_err(FI_EINVAL, "bad arguments");
  if (n == 0) return FI_OK;
  HIP_TRY(hipSetDevice(c->device));
  std::lock_guard<std::mutex> lk(c->mu);
  if (order_after_apply(c) != FI_OK) return set_err(FI_EDEVICE, "hipStreamWaitEvent failed");
  std::string err;
  const int rc = jpeg_decode_batch(c->stream, data, len, n, dst, dst_stride, out_channels, status, jpeg_alloc, c, &err);
  if (rc) return set_err(rc, "%s", err.c_str());
  for (int i = 0; i < n; i++)  // the others are decoded; the caller decodes these on the host
    if (status[i])
      return set_err(status[i], "image %d: %s", i,
                     status[i] == FI_EUNSUPPORTED ? "JPEG stream the GPU decoder does not handle" : "malformed JPEG");
  return FI_OK;
}
// Test hook: the skin / saturation table of k_sc_fz<true> / k_sc_fd for `params`,
// returned in r-major colour order (the device table is in sc_colour_key order)
int fi_debug_skinsat(fi_ctx *c, const fi_smartcrop_params *params, uint16_t *out) {
  if (!c || !out) return set_err(FI_EINVAL, "bad arguments");
  fi_smartcrop_params p;
  if (params)
    p = *params;
  else
    fi_smartcrop_default_params(&p);
  HIP_TRY(hipSetDevice(c->device));
  sync_streams(c);  // batches in flight may read the table
  const int rc = ensure(c, &c->skinsat, (size_t)2 << 24);
  if (rc != FI_OK) return rc;
  const ScParamsDev PD = to_dev(p);
  launch_sc_skinsat(c->stream, (uint16_t *)c->skinsat.p, PD);
  c->skinsat_key.clear();  // built on c->stream, not the smartcrop stream: rebuilt before the next use
  HIP_TRY(hipGetLastError());
  std::vector<uint16_t> z((size_t)1 << 24);
  HIP_TRY(hipMemcpyAsync(z.data(), c->skinsat.p, (size_t)2 << 24, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (uint32_t k = 0; k < (1u << 24); k++) out[k] = z[sc_colour_key(k >> 16, (k >> 8) & 255, k & 255)];  // r-major
  return FI_OK;
}
// Test hook: the -monochrome kernels (fi_mono.hip) on a caller-supplied Q16
// gray image (host buffers), so the parity tests can feed the oracle the
// identical input; out is w x h (rot 0/180) or h x w (rot 90/270), 8-bit.
int fi_debug_monochrome(fi_ctx *c, const uint16_t *gray, int32_t w, int32_t h, int32_t rot, uint8_t *out,
                        int32_t out_stride) {
  if (!c || !gray || !out || w <= 0 || h <= 0) return set_err(FI_EINVAL, "bad arguments");
  if (rot != 0 && rot != 90 && rot != 180 && rot != 270) return set_err(FI_EINVAL, "rot must be 0/90/180/270");
  const int ow = (rot == 90 || rot == 270) ? h : w, oh = (rot == 90 || rot == 270) ? w : h;
  if (out_stride < ow) return set_err(FI_EINVAL, "out_stride too small");
  HIP_TRY(hipSetDevice(c->device));
  const size_t gbytes = (size_t)w * h * 2, obytes = (size_t)out_stride * oh;
  const size_t o_st = (gbytes + 255) / 256 * 256, o_desc = o_st + (sizeof(MonoState) + 255) / 256 * 256,
               o_w = o_desc + 256, o_out = o_w + 256, total = o_out + obytes;
  uint8_t *d = nullptr;
  HIP_TRY(hipMalloc(&d, total));
  MonoDesc md{};
  md.g = (const uint16_t *)d;
  md.w = w;
  md.h = h;
  md.rot = rot;
  md.dst = d + o_out;
  md.dst_stride = out_stride;
  md.st = (MonoState *)(d + o_st);
  volatile double qr1 = 65535.0 + 1.0, span = 16 - 1.0;
  const double step = exp(log((double)qr1) / (double)span);
  double weight = 1.0, wts[16];
  for (int k = 0; k < 16; k++) {
    wts[16 - k - 1] = 1.0 / weight;
    weight *= step;
  }
  int rc = FI_OK;
  if (hipMemcpy(d, gray, gbytes, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(d + o_desc, &md, sizeof(md), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(d + o_w, wts, sizeof(wts), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(d + o_out, 0, obytes) != hipSuccess) {
    rc = set_err(FI_EDEVICE, "fi_debug_monochrome: upload failed");
  } else {
    launch_mono(c->stream, (const MonoDesc *)(d + o_desc), 1, (const double *)(d + o_w));
    if (hipStreamSynchronize(c->stream) != hipSuccess || hipGetLastError() != hipSuccess ||
        hipMemcpy(out, d + o_out, obytes, hipMemcpyDeviceToHost) != hipSuccess)
      rc = set_err(FI_EDEVICE, "fi_debug_monochrome: kernel failed");
  }
  (void)hipFree(d);
  return rc;
}

int fi_debug_convolve(fi_ctx *c, const uint16_t *q16, int32_t w, int32_t h, int32_t ch, const double conv[8],
                      uint32_t ops, uint8_t *out) {
  if (!c || !q16 || !conv || !out || w <= 0 || h <= 0 || (ch != 1 && ch != 3) || (ops & ~7u))
    return set_err(FI_EINVAL, "bad arguments");
  HIP_TRY(hipSetDevice(c->device));
  std::vector<double> tab, kk;
  std::vector<ConvStep> st[6];
  const size_t qb = (size_t)w * h * ch * 2;
  const size_t o_b = (qb + 255) / 256 * 256, o_out = 2 * o_b, o_tab = o_out + (qb / 2 + 255) / 256 * 256;
  // host side of the steps (device pointers patched below), as run_batch builds them
  ConvStep base{};
  base.W = w;
  base.H = h;
  base.C = ch;
  int cur = 0;  // 0 = buffer A, 1 = B
  struct Pend {
    int stage, in, out, orig;
    ConvStep s;
  };
  std::vector<Pend> pend;
  auto tbl = [&](const std::vector<double> &v) {
    const int32_t off = (int32_t)tab.size();
    tab.insert(tab.end(), v.begin(), v.end());
    return off;
  };
  if (ops & 1) {
    const int kw = im_blur_kernel(conv[0], conv[1], &kk);
    if (kw < 0) return set_err(FI_EUNSUPPORTED, "unsharp kernel too wide");
    ConvStep a = base, b = base;
    a.k = b.k = tbl(kk);
    a.kw = kw, a.kh = 1;
    b.kw = 1, b.kh = kw, b.gain = conv[2], b.thr = 65535.0 * conv[3];
    pend.push_back({0, cur, 1 - cur, -1, a});
    pend.push_back({1, 1 - cur, cur, cur, b});
  }
  if (ops & 2) {
    const int kw = im_sharpen_kernel(conv[4], conv[5], &kk);
    if (kw < 0) return set_err(FI_EUNSUPPORTED, "sharpen kernel too wide");
    ConvStep a = base;
    a.k = tbl(kk);
    a.kw = a.kh = kw;
    pend.push_back({2, cur, 1 - cur, -1, a});
    cur = 1 - cur;
  }
  if (ops & 4) {
    const int kw = im_blur_kernel(conv[6], conv[7], &kk);
    if (kw < 0) return set_err(FI_EUNSUPPORTED, "blur kernel too wide");
    ConvStep a = base, b = base;
    a.k = b.k = tbl(kk);
    a.kw = kw, a.kh = 1;
    b.kw = 1, b.kh = kw;
    pend.push_back({3, cur, 1 - cur, -1, a});
    pend.push_back({4, 1 - cur, cur, -1, b});
  }
  pend.push_back({5, cur, -1, -1, base});
  const size_t o_desc = o_tab + (tab.size() * 8 + 255) / 256 * 256, o_pre = o_desc + pend.size() * 256;
  const size_t total = o_pre + 256;
  uint8_t *d = nullptr;
  HIP_TRY(hipMalloc(&d, total));
  uint16_t *buf[2] = {(uint16_t *)d, (uint16_t *)(d + o_b)};
  int rc = FI_OK;
  const int32_t pre[2] = {0, h};
  if (hipMemcpy(d, q16, qb, hipMemcpyHostToDevice) != hipSuccess ||
      (!tab.empty() && hipMemcpy(d + o_tab, tab.data(), tab.size() * 8, hipMemcpyHostToDevice) != hipSuccess) ||
      hipMemcpy(d + o_pre, pre, sizeof(pre), hipMemcpyHostToDevice) != hipSuccess)
    rc = set_err(FI_EDEVICE, "fi_debug_convolve: upload failed");
  static const int kMode[6] = {0, 2, 3, 0, 1, 4};
  for (size_t j = 0; rc == FI_OK && j < pend.size(); j++) {
    ConvStep s = pend[j].s;
    s.in = buf[pend[j].in];
    s.out = pend[j].out >= 0 ? buf[pend[j].out] : nullptr;
    s.orig = pend[j].orig >= 0 ? buf[pend[j].orig] : nullptr;
    s.dst8 = d + o_out;
    s.dst_stride = (int64_t)w * ch;
    uint8_t *dd = d + o_desc + 256 * j;
    if (hipMemcpy(dd, &s, sizeof(s), hipMemcpyHostToDevice) != hipSuccess) {
      rc = set_err(FI_EDEVICE, "fi_debug_convolve: upload failed");
      break;
    }
    launch_conv(c->stream, kMode[pend[j].stage], (const ConvStep *)dd, (const int32_t *)(d + o_pre), 1, h,
                (const double *)(d + o_tab));
  }
  if (rc == FI_OK && (hipStreamSynchronize(c->stream) != hipSuccess || hipGetLastError() != hipSuccess ||
                      hipMemcpy(out, d + o_out, (size_t)w * h * ch, hipMemcpyDeviceToHost) != hipSuccess))
    rc = set_err(FI_EDEVICE, "fi_debug_convolve: kernel failed");
  (void)hipFree(d);
  return rc;
}

const char *fi_last_error(void) { return g_err.c_str(); }

int fi_device_count(int32_t *count) {
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  *count = n;
  return FI_OK;
}

int fi_create(fi_ctx **out, int32_t device) {
  if (!out) return set_err(FI_EINVAL, "out is NULL");
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return set_err(FI_EINVAL, "device %d out of range (%d visible)", device, n);
  HIP_TRY(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return set_err(FI_EDEVICE, "device %d is %s; libflyimg_hip.so is built for gfx950 only", device, prop.gcnArchName);
  fi_ctx *c = new fi_ctx();
  c->device = device;
  // Kernel selection is by geometry and LDS fit; three switches keep the
  // fallbacks testable on geometries that would not reach them otherwise:
  //   FI_FORCE_GENERIC=1   the generic two-pass resample and per-row smartcrop kernels
  //   FI_VR_RS=0           k_rs_vm instead of k_rs_vr (vertical-first)
  //   FI_VR_NL=2|4, FI_VR_PBUF=1|2  k_rs_vr's loader waves / plane buffers (where valid)
  //   FI_DISABLE_SC_FZ=1   k_sc_hmfma + k_sc_vq instead of the fused k_sc_fz
  if (const char *e = getenv("FI_FORCE_GENERIC")) c->fast_rs = c->sc_prep = !(e[0] == '1');
  if (const char *e = getenv("FI_VR_RS")) c->vr_rs = e[0] == '1';
  if (const char *e = getenv("FI_VR_NL")) c->vr_nl = atoi(e);
  if (const char *e = getenv("FI_VR_SPLIT")) c->vr_split = e[0] == '1';
  if (const char *e = getenv("FI_VR_NARROW")) c->vr_narrow = e[0] == '1';
  if (const char *e = getenv("FI_UP_SYNC")) c->up_hostsync = e[0] == '1';
  if (const char *e = getenv("FI_VR_PBUF")) c->vr_pbuf = atoi(e);
  if (const char *e = getenv("FI_DISABLE_SC_FZ")) c->sc_fz = !(e[0] == '1');
  if (const char *e = getenv("FI_SC_FD")) c->sc_fd = e[0] == '1';
  if (const char *e = getenv("FI_SC_CX")) c->sc_cx = atoi(e);
  if (const char *e = getenv("FI_SC_MFMA")) c->sc_mf = e[0] == '1';
  if (const char *e = getenv("FI_VR_MAX_CLASSES")) c->vr_max_classes = atoi(e);
  if (const char *e = getenv("FI_VM_LPT")) c->vm_lpt = e[0] == '1';
  if (const char *e = getenv("FI_RES_ALIGN")) c->res_align = std::max(1, atoi(e));
  c->n_cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  // (the smartcrop stage on a stream of its own beside the next batch's
  // resample was measured in round 2: the resample fills every CU, so the
  // overlap only stretched both -- one stream)
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return set_err(FI_EDEVICE, "hipStreamCreate failed");
  }
  c->sc_stream = c->stream;
  if (const char *e = getenv("FI_APPLY_OVERLAP")) c->apply_overlap = e[0] == '1';
  if (const char *e = getenv("FI_VR_FORK")) c->vr_fork = e[0] == '1';
  // ap_stream at the higher priority: its score / apply take the CUs the
  // resample frees before the next resample's workgroups do
  int prio_lo = 0, prio_hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  if (hipStreamCreateWithFlags(&c->up_stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->rb_stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithPriority(&c->ap_stream, hipStreamNonBlocking, prio_hi) != hipSuccess ||
      hipStreamCreateWithFlags(&c->rs2_stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->gx_stream, hipStreamNonBlocking) != hipSuccess) {
    fi_destroy(c);
    return set_err(FI_EDEVICE, "hipStreamCreate failed");
  }
  *out = c;
  return FI_OK;
}

void fi_destroy(fi_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)drain(c);
  sync_streams(c);
  if (c->comm) ncclCommDestroy(c->comm);
  for (DevBuf *b : {&c->arena, &c->work, &c->io, &c->gather, &c->pix, &c->skinsat, &c->jpeg[0], &c->jpeg[1],
                    &c->jpeg[2]})
    if (b->p) (void)hipFree(b->p);
  if (c->pinned) (void)hipHostFree(c->pinned);
  if (c->jpeg_host) (void)hipHostFree(c->jpeg_host);
  for (Slot &sl : c->slots) {
    if (sl.blob) (void)hipHostFree(sl.blob);
    if (sl.res) (void)hipHostFree(sl.res);
    if (sl.hpin) (void)hipHostFree(sl.hpin);
    if (sl.done) (void)hipEventDestroy(sl.done);
    if (sl.rs_done) (void)hipEventDestroy(sl.rs_done);
    if (sl.up_done) (void)hipEventDestroy(sl.up_done);
    if (sl.sc_end) (void)hipEventDestroy(sl.sc_end);
    if (sl.sc_done) (void)hipEventDestroy(sl.sc_done);
    for (DevBuf *b : {&sl.arena, &sl.work, &sl.hio})
      if (b->p) (void)hipFree(b->p);
  }
  for (auto e : c->event_pool) (void)hipEventDestroy(e);
  (void)hipStreamDestroy(c->stream);
  if (c->sc_stream != c->stream) (void)hipStreamDestroy(c->sc_stream);
  if (c->up_stream) (void)hipStreamDestroy(c->up_stream);
  if (c->rb_stream) (void)hipStreamDestroy(c->rb_stream);
  if (c->ap_stream) (void)hipStreamDestroy(c->ap_stream);
  if (c->rs2_stream) (void)hipStreamDestroy(c->rs2_stream);
  if (c->gx_stream) (void)hipStreamDestroy(c->gx_stream);
  if (c->rs_fork) (void)hipEventDestroy(c->rs_fork);
  if (c->rs_join) (void)hipEventDestroy(c->rs_join);
  if (c->ap_tail) (void)hipEventDestroy(c->ap_tail);
  if (c->gx_done) (void)hipEventDestroy(c->gx_done);
  if (c->gx_pin) (void)hipHostFree(c->gx_pin);
  delete c;
}

int fi_plan(fi_image *imgs, int32_t n) {
  if (n < 0 || (n > 0 && !imgs)) return set_err(FI_EINVAL, "bad image array");
  int first = FI_OK;
  for (int i = 0; i < n; i++) {
    ImPlan p;
    const int rc = plan_im(imgs[i], &p);
    imgs[i].status = rc;
    if (rc == FI_OK) {
      imgs[i].out_w = p.out_w;
      imgs[i].out_h = p.out_h;
      imgs[i].out_channels = p.out_c;
      imgs[i].out_stride = p.out_w * p.out_c;
    } else if (first == FI_OK) {
      first = set_err(rc, "image %d: %s", i, p.err.c_str());
    }
  }
  return first;
}

int fi_pixelate_regions_device(fi_ctx *c, uint8_t *img, int32_t w, int32_t h, int32_t stride, int32_t channels,
                               const int32_t *boxes, int32_t nboxes) {
  if (!c) return set_err(FI_EINVAL, "bad arguments");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  // stream-ordered after earlier batches, including their crop applies on ap_stream
  if (order_after_apply(c) != FI_OK) return set_err(FI_EDEVICE, "hipStreamWaitEvent failed");
  return pixelate_device(c, img, w, h, stride, channels, boxes, nboxes);
}

int fi_pixelate_regions(fi_ctx *c, uint8_t *img, int32_t w, int32_t h, int32_t stride, int32_t channels,
                        const int32_t *boxes, int32_t nboxes) {
  if (!c || !img || w <= 0 || h <= 0 || (channels != 1 && channels != 3) || stride < w * channels)
    return set_err(FI_EINVAL, "bad arguments");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  {
    const int rc0 = drain(c);  // the io buffer may be read by in-flight batches
    if (rc0) return rc0;
  }
  const int64_t pitch = (int64_t)w * channels;
  int rc = ensure(c, &c->io, (size_t)pitch * h + 256);
  if (rc) return rc;
  uint8_t *d = (uint8_t *)c->io.p;
  HIP_TRY(hipMemcpy2DAsync(d, pitch, img, stride, pitch, h, hipMemcpyHostToDevice, c->stream));
  rc = pixelate_device(c, d, w, h, pitch, channels, boxes, nboxes);
  // boxes before a rejected one are applied (each face is its own mogrify run)
  HIP_TRY(hipMemcpy2DAsync(img, stride, d, pitch, pitch, h, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return rc;
}

int fi_plan_bytes(const fi_image *imgs, int32_t n, int64_t *bytes) {
  if (n < 0 || (n > 0 && (!imgs || !bytes))) return set_err(FI_EINVAL, "bad arguments");
  int first = FI_OK;
  for (int i = 0; i < n; i++) {
    ImPlan p;
    const int rc = plan_im(imgs[i], &p);
    if (rc != FI_OK) {
      bytes[i] = -1;
      if (first == FI_OK) first = set_err(rc, "image %d: %s", i, p.err.c_str());
      continue;
    }
    int64_t rows = p.eh;  // no resample: the extent window's rows are copied
    if (p.resize) {
      AxisTable t;
      build_axis(p.filter, p.yf, p.sh, p.th, p.ey0, p.ey0 + p.eh, p.sample, p.H, &t);
      rows = t.touched;
    }
    bytes[i] = rows * (int64_t)p.W * p.C + (int64_t)p.out_w * p.out_h * p.out_c +
               ((imgs[i].flags & FI_OP_SMARTCROP) ? 16 : 0);
  }
  return first;
}

// Test hook (host only, needs no GPU): run_batch's planner -- plan_image,
// plan_batch_sc, resolve_workspace, build_vm_tiles (with the k_rs_vr tiles),
// build_hv_tiles, pack_batch -- over `imgs` `iters` times on one host-only
// context (device pointers are planned, never dereferenced; caches and heap
// offsets persist across iterations as across a serving run's batches).
// ms[0..6] += images, smartcrop, workspace, vm + vr tiles, of which vr, hv
// tiles, blob (milliseconds, summed over the iterations).
int fi_debug_host_plan(const fi_image *imgs, int32_t n, int32_t iters, double *ms) {
  static fi_ctx *c = nullptr;  // one host-only context across calls (its caches, as a serving context's)
  if (!imgs && n == 0) {       // (NULL, 0, ...): drop it
    if (c && getenv("FI_PLAN_PROF"))
      for (const auto &kv : c->stats) fprintf(stderr, "%s %.1f ms (%lld)\n", kv.first.c_str(), kv.second.ms, (long long)kv.second.launches);
    delete c;
    c = nullptr;
    return FI_OK;
  }
  if (!imgs && n == 1) {  // (NULL, 1, ...): reset the stage stats (after a warm-up pass)
    if (c) c->stats.clear();
    return FI_OK;
  }
  if (!imgs && n == 2) {  // (NULL, 2, 0, ms): the resample plan's counters
    if (!ms) return set_err(FI_EINVAL, "ms is NULL");
    ms[0] = ms[1] = ms[2] = 0;
    if (c) {
      ms[0] = (double)c->stats["plan_path_vr"].launches;
      ms[1] = (double)c->stats["plan_vertical_first"].launches;
      ms[2] = (double)c->stats["plan_vr_launches"].launches;
    }
    return FI_OK;
  }
  if (!imgs || n <= 0 || iters <= 0 || !ms) return set_err(FI_EINVAL, "bad arguments");
  if (!c) {
    c = new fi_ctx();
    c->host_only = true;
    c->timing = true;
    if (const char *e = getenv("FI_VR_RS")) c->vr_rs = e[0] == '1';
  }
  std::vector<fi_image> v(imgs, imgs + n);
  uint8_t *wb = reinterpret_cast<uint8_t *>((uintptr_t)1 << 40);  // a stand-in workspace base
  int rc = FI_OK;
  for (int it = 0; it < iters && rc == FI_OK; it++) {
    const double t0 = now_ms();
    Exec E;
    E.c = c;
    fi_smartcrop_default_params(&E.params);
    rc = heap_prepare(c, E);
    if (rc) break;
    BatchPlan Bp;
    Bp.imgs = v.data();
    Bp.n = n;
    Bp.plans.resize(n);
    Bp.status.assign(n, FI_OK);
    Bp.errs.resize(n);
    Bp.rd_of.assign(n, -1);
    Bp.sc_of.assign(n, -1);
    Bp.res_off.assign(n, 0);
    Bp.res_stride.assign(n, 0);
    Bp.out_of.assign(n, nullptr);
    for (int i = 0; i < n; i++) plan_image(c, E, Bp, i);
    const double t1 = now_ms();
    plan_batch_sc(c, E, Bp);
    const double t2 = now_ms();
    resolve_workspace(E, Bp, wb);
    const double t3 = now_ms();
    const double vr0 = c->stats["host_plan_vr"].ms;
    build_vm_tiles(c, E, Bp);
    const double t4 = now_ms();
    build_hv_tiles(c, E, Bp);
    const double t5 = now_ms();
    // images per resample kernel (FI_PLAN_PROF lists them; (NULL, 2, ...) reads them)
    int nvr = 0;
    for (const BatchPlan::VrLaunch &V : Bp.vrl) nvr += V.images;
    c->stats["plan_path_vr"].launches += nvr;
    // (build_vr_tiles appends a second descriptor for each of its images)
    c->stats["plan_vertical_first"].launches += (int64_t)Bp.vdescs.size() - nvr;
    c->stats["plan_vr_launches"].launches += (int64_t)Bp.vrl.size();
    Packed K;
    pack_batch(c, E, Bp, K);
    const double t6 = now_ms();
    if (!heap_fits(c, E)) heap_reset(c);
    else {
      c->heap_i.used = (size_t)E.bi + (E.ai.size() + 15) / 16 * 16;
      c->heap_f.used = (size_t)E.bf + (E.af.size() + 15) / 16 * 16;
      c->heap_d.used = (size_t)E.bd + (E.ad.size() + 15) / 16 * 16;
    }
    ms[0] += t1 - t0;
    ms[1] += t2 - t1;
    ms[2] += t3 - t2;
    ms[3] += t4 - t3;
    ms[4] += c->stats["host_plan_vr"].ms - vr0;
    ms[5] += t5 - t4;
    ms[6] += t6 - t5;
  }
  return rc;
}

int fi_process_batch_device(fi_ctx *c, fi_image *imgs, int32_t n) {
  if (!c || n < 0 || (n > 0 && !imgs)) return set_err(FI_EINVAL, "bad arguments");
  if (n == 0) return FI_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  return run_batch(c, imgs, n, false);
}

int fi_submit_batch_device(fi_ctx *c, fi_image *imgs, int32_t n) {
  if (!c || n < 0 || (n > 0 && !imgs)) return set_err(FI_EINVAL, "bad arguments");
  if (n == 0) return FI_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  return run_batch(c, imgs, n, true);
}

int fi_wait(fi_ctx *c, int32_t keep) {
  if (!c || keep < 0) return set_err(FI_EINVAL, "bad arguments");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  int first = FI_OK;
  while ((int32_t)c->inflight.size() > keep) {
    const int rc = finalize_front(c);
    if (rc != FI_OK && first == FI_OK) first = rc;
  }
  return first;
}

// Host-buffer batch, asynchronous: sources into the batch slot's device
// buffer (pinned sources DMA directly; pageable ones through the slot's pinned
// staging), run_batch, outputs back behind the batch (queue_readback).  The
// slot's previous batch is finalized first, so two host batches are in flight.
static bool host_pinned(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // clear the sticky "invalid value" of a pageable pointer
    return false;
  }
  return a.type == hipMemoryTypeHost;
}
static int submit_host(fi_ctx *c, fi_image *imgs, int32_t n) {
  const int slot = c->next_slot;
  {
    const int rc0 = wait_slot(c, slot);  // per-image failures of that batch stay in its records
    if (rc0 == FI_EDEVICE) return rc0;
  }
  Slot &S = c->slots[slot];
  auto host = std::make_shared<HostIo>();
  host->user = imgs;
  host->dev.assign(imgs, imgs + n);
  host->dev_dst_off.assign(n, 0);
  host->pin_off.assign(n, -1);
  std::vector<size_t> soff(n, 0);
  std::vector<int64_t> spin(n, -1);  // pageable source: offset of its packed rows in the staging
  std::vector<uint8_t> src_pinned(n, 0);
  size_t total = 0, pin_total = 0;
  for (int i = 0; i < n; i++) {
    const fi_image &im = imgs[i];
    const int C = im.src_channels == 4 ? 4 : 3;
    const int64_t sstride = ((int64_t)im.src_w * C + 15) / 16 * 16;
    soff[i] = total;
    total += (size_t)std::max<int64_t>(sstride * im.src_h, 0);
    total = (total + 255) / 256 * 256;
    host->dev_dst_off[i] = total;
    total += (size_t)std::max<int64_t>(im.dst_capacity, 0);
    total = (total + 255) / 256 * 256;
    host->dev[i].src_stride = (int32_t)sstride;
    const bool ok = im.src && im.src_w > 0 && im.src_h > 0 && (im.src_channels == 3 || im.src_channels == 4) &&
                    im.src_stride >= im.src_w * im.src_channels;
    if (ok && !(src_pinned[i] = host_pinned(im.src))) {
      spin[i] = (int64_t)pin_total;
      pin_total += ((size_t)im.src_w * im.src_channels * im.src_h + 255) / 256 * 256;
    }
    if (im.dst && im.dst_capacity > 0 && !host_pinned(im.dst)) {
      host->pin_off[i] = (int64_t)pin_total;
      pin_total += ((size_t)im.dst_capacity + 255) / 256 * 256;
    }
  }
  int rc = ensure(c, &S.hio, total + 256);
  if (rc) return rc;
  rc = ensure_pinned_buf(&S.hpin, &S.hpin_cap, pin_total + 256);
  if (rc) return rc;
  uint8_t *io = (uint8_t *)S.hio.p;
  double sbytes = 0;
  for (int i = 0; i < n; i++)
    if (imgs[i].src && imgs[i].src_w > 0 && imgs[i].src_h > 0)
      sbytes += (double)imgs[i].src_w * imgs[i].src_channels * imgs[i].src_h;
  {
  const double t_pack = now_ms();
  Timer t(c, "h2d_src", sbytes, c->up_stream, c->up_stream);
  for (int i = 0; i < n; i++) {
    const fi_image &im = imgs[i];
    fi_image &d = host->dev[i];
    const int C = im.src_channels;
    const bool ok = im.src && im.src_w > 0 && im.src_h > 0 && (C == 3 || C == 4) && im.src_stride >= im.src_w * C;
    d.dst = im.dst ? io + host->dev_dst_off[i] : nullptr;
    if (!ok) {
      d.src = nullptr;
      continue;
    }
    const size_t row = (size_t)im.src_w * C;
    const uint8_t *from = im.src;
    int64_t from_stride = im.src_stride;
    if (!src_pinned[i]) {  // pageable: pack the rows into the pinned staging first
      uint8_t *pin = (uint8_t *)S.hpin + spin[i];
      for (int y = 0; y < im.src_h; y++) memcpy(pin + (size_t)y * row, im.src + (int64_t)y * im.src_stride, row);
      from = pin;
      from_stride = (int64_t)row;
    }
    HIP_TRY(hipMemcpy2DAsync(io + soff[i], d.src_stride, from, from_stride, row, im.src_h, hipMemcpyHostToDevice,
                             c->up_stream));
    d.src = io + soff[i];
  }
  host_stat(c, "host_src_stage", now_ms() - t_pack);  // pageable rows packed into pinned staging + copy issue
  }
  return run_batch(c, host->dev.data(), n, true, host);
}

int fi_submit_batch(fi_ctx *c, fi_image *imgs, int32_t n) {
  if (!c || n < 0 || (n > 0 && !imgs)) return set_err(FI_EINVAL, "bad arguments");
  if (n == 0) return FI_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  return submit_host(c, imgs, n);
}

int fi_process_batch(fi_ctx *c, fi_image *imgs, int32_t n) {
  if (!c || n < 0 || (n > 0 && !imgs)) return set_err(FI_EINVAL, "bad arguments");
  if (n == 0) return FI_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  {
    const int rc0 = drain(c);  // synchronous call: earlier batches complete first
    if (rc0 == FI_EDEVICE) return rc0;
  }
  const int rc = submit_host(c, imgs, n);
  const int rd = drain(c);
  return rc != FI_OK ? rc : rd;
}

void *fi_host_alloc(fi_ctx *c, size_t bytes) {
  if (!c || bytes == 0) return nullptr;
  void *p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
    set_err(FI_ENOMEM, "hipHostMalloc(%zu) failed", bytes);
    return nullptr;
  }
  return p;
}

int fi_host_free(fi_ctx *c, void *p) {
  if (!c) return set_err(FI_EINVAL, "bad arguments");
  if (p) HIP_TRY(hipHostFree(p));
  return FI_OK;
}

void fi_smartcrop_default_params(fi_smartcrop_params *p) {
  memset(p, 0, sizeof *p);
  p->detail_weight = 0.2;
  p->edge_radius = 0.4;
  p->edge_weight = -10;
  p->outside_importance = -0.5;
  p->rule_of_thirds = 1;
  p->saturation_bias = 0.2;
  p->saturation_brightness_max = 0.9;
  p->saturation_brightness_min = 0.05;
  p->saturation_threshold = 0.4;
  p->saturation_weight = 0.3;
  p->score_down_sample = 1;
  p->skin_bias = 0.01;
  p->skin_brightness_max = 1;
  p->skin_brightness_min = 0.2;
  p->skin_color[0] = 0.78;
  p->skin_color[1] = 0.57;
  p->skin_color[2] = 0.44;
  p->skin_threshold = 0.8;
  p->skin_weight = 1.8;
}
void fi_smartcrop_default_options(fi_smartcrop_options *o) {
  memset(o, 0, sizeof *o);
  o->prescale = 1;
  o->max_scale = 1;
  o->min_scale = 0.9;
  o->scale_step = 0.1;
  o->step = 8;
  o->exact_all = 0;
}

int fi_smartcrop_ex(fi_ctx *c, const uint8_t *rgb, int32_t w, int32_t h, int32_t stride, int32_t tw, int32_t th,
                    const fi_smartcrop_params *params, const fi_smartcrop_options *opts, fi_crop_score *crops,
                    int32_t crops_cap, int32_t *n_crops, int32_t *top_index, int32_t analyse_wh[2], double *prescale,
                    uint8_t *prescaled_out, uint8_t *maps_out, int64_t out_cap) {
  if (!c || !rgb || w <= 0 || h <= 0 || stride < 3 * w) return set_err(FI_EINVAL, "bad image arguments");
  fi_smartcrop_params P;
  fi_smartcrop_default_params(&P);
  if (params) P = *params;
  if (P.score_down_sample != 1) return set_err(FI_EUNSUPPORTED, "score_down_sample != 1 is not supported");
  fi_smartcrop_options O;
  fi_smartcrop_default_options(&O);
  if (opts) O = *opts;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  int rc = drain(c);  // io / pinned staging are shared with in-flight batches
  if (rc) return rc;
  const int64_t dstride = ((int64_t)w * 3 + 15) / 16 * 16;
  rc = ensure(c, &c->io, (size_t)dstride * h + 256);
  if (rc) return rc;
  HIP_TRY(hipMemcpy2DAsync(c->io.p, dstride, rgb, stride, (size_t)w * 3, h, hipMemcpyHostToDevice, c->stream));
  std::vector<CropScore> scores;
  ScResult res{};
  ScPlan plan;
  std::vector<uint8_t> pre, maps;
  rc = run_smartcrop(c, (const uint8_t *)c->io.p, w, h, dstride, 3, tw, th, P, O, &scores, &res, &plan,
                     prescaled_out ? &pre : nullptr, maps_out ? &maps : nullptr);
  if (rc) return rc;
  const int nc = (int)plan.crops.size();
  if (n_crops) *n_crops = nc;
  if (top_index) *top_index = res.top;
  if (analyse_wh) {
    analyse_wh[0] = plan.aw;
    analyse_wh[1] = plan.ah;
  }
  if (prescale) *prescale = plan.prescale;
  if (crops) {
    for (int k = 0; k < nc && k < crops_cap; k++) {
      const CropHost &ch = plan.crops[k];
      fi_crop_score &o = crops[k];
      o.x = ch.rx;
      o.y = ch.ry;
      o.width = ch.rw;
      o.height = ch.rh;
      o.fx = ch.fx;
      o.fy = ch.fy;
      o.fw = ch.fw;
      o.fh = ch.fh;
      o.detail = scores[k].detail;
      o.saturation = scores[k].saturation;
      o.skin = scores[k].skin;
      o.total = scores[k].total;
      o.exact = scores[k].exact;
      o.pad = 0;
    }
  }
  const size_t na = (size_t)plan.aw * plan.ah * 3;
  if (prescaled_out) {
    if ((int64_t)na > out_cap) return set_err(FI_ECAPACITY, "out_cap < analyse_w*analyse_h*3");
    memcpy(prescaled_out, pre.data(), na);
  }
  if (maps_out) {
    if ((int64_t)na > out_cap) return set_err(FI_ECAPACITY, "out_cap < analyse_w*analyse_h*3");
    memcpy(maps_out, maps.data(), na);
  }
  return FI_OK;
}

int fi_smartcrop(fi_ctx *c, const uint8_t *rgb, int32_t w, int32_t h, int32_t stride, int32_t tw, int32_t th,
                 const fi_smartcrop_params *params, int32_t out_xywh[4], double *out_score) {
  int32_t n = 0, top = -1;
  int32_t awh[2];
  double pre;
  // crops are needed to decode the top index
  std::vector<fi_crop_score> crops(1);
  {
    // first call with a small buffer just to learn the crop count is wasteful;
    // the planner is cheap, so plan here directly
    fi_smartcrop_options O;
    fi_smartcrop_default_options(&O);
    ScPlan p;
    if (plan_sc(w, h, tw, th, O, &p) != FI_OK) return set_err(p.status, "%s", p.err.c_str());
    crops.resize(p.crops.size());
  }
  int rc = fi_smartcrop_ex(c, rgb, w, h, stride, tw, th, params, nullptr, crops.data(), (int32_t)crops.size(), &n,
                           &top, awh, &pre, nullptr, nullptr, 0);
  if (rc) return rc;
  if (top < 0 || top >= n) return set_err(FI_EDEVICE, "smartcrop: no top crop");
  out_xywh[0] = crops[top].x;
  out_xywh[1] = crops[top].y;
  out_xywh[2] = crops[top].width;
  out_xywh[3] = crops[top].height;
  if (out_score) *out_score = crops[top].total;
  return FI_OK;
}

int fi_device_malloc(fi_ctx *c, void **ptr, uint64_t bytes) {
  if (!c || !ptr) return set_err(FI_EINVAL, "bad arguments");
  HIP_TRY(hipSetDevice(c->device));
  if (hipMalloc(ptr, bytes) != hipSuccess) return set_err(FI_ENOMEM, "hipMalloc(%llu) failed", (unsigned long long)bytes);
  return FI_OK;
}
int fi_device_free(fi_ctx *c, void *ptr) {
  if (!c) return set_err(FI_EINVAL, "bad arguments");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipFree(ptr));
  return FI_OK;
}
int fi_memcpy_h2d(fi_ctx *c, void *dst, const void *src, uint64_t bytes) {
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return FI_OK;
}
int fi_memcpy_d2h(fi_ctx *c, void *dst, const void *src, uint64_t bytes) {
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return FI_OK;
}
int fi_fill_synthetic(fi_ctx *c, uint8_t *dev, int32_t w, int32_t h, int32_t stride, uint32_t seed) {
  if (!c || !dev || w <= 0 || h <= 0 || stride < 3 * w) return set_err(FI_EINVAL, "bad arguments");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  if (order_after_apply(c) != FI_OK) return set_err(FI_EDEVICE, "hipStreamWaitEvent failed");
  const int64_t n = (int64_t)w * h;
  hipLaunchKernelGGL(k_synth, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, dev, w, h, (int64_t)stride,
                     seed);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));
  return FI_OK;
}

int fi_set_timing(fi_ctx *c, int32_t enable) {
  if (!c) return set_err(FI_EINVAL, "ctx is NULL");
  c->timing = enable != 0;
  c->timing_resize_only = enable == 2;
  return FI_OK;
}
int fi_reset_stats(fi_ctx *c) {
  if (!c) return set_err(FI_EINVAL, "ctx is NULL");
  c->stats.clear();
  return FI_OK;
}
int fi_kernel_stats(fi_ctx *c, const char *name, double *total_ms, int64_t *launches, double *bytes) {
  if (!c || !name) return set_err(FI_EINVAL, "bad arguments");
  auto it = c->stats.find(name);
  const Stat s = it == c->stats.end() ? Stat{} : it->second;
  if (total_ms) *total_ms = s.ms;
  if (launches) *launches = s.launches;
  if (bytes) *bytes = s.bytes;
  return FI_OK;
}

int fi_rccl_get_unique_id(uint8_t id[128]) {
  ncclUniqueId u;
  const ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) return set_err(FI_EDEVICE, "ncclGetUniqueId: %s", ncclGetErrorString(r));
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  memcpy(id, &u, 128);
  return FI_OK;
}
int fi_rccl_init(fi_ctx *c, int32_t rank, int32_t world, const uint8_t id[128]) {
  if (!c || rank < 0 || world < 1 || rank >= world) return set_err(FI_EINVAL, "bad rank/world");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  ncclUniqueId u;
  memcpy(&u, id, 128);
  const ncclResult_t r = ncclCommInitRank(&c->comm, world, u, rank);
  if (r != ncclSuccess) return set_err(FI_EDEVICE, "ncclCommInitRank: %s", ncclGetErrorString(r));
  c->rank = rank;
  c->world = world;
  return FI_OK;
}
// The record gather runs on gx_stream, a stream of its own: the records are on
// the host once fi_wait has filled them, so nothing orders the gather after
// the batch streams, and a gather started while the next batch runs returns
// at once (fi_rccl_gather_start); fi_rccl_gather_finish waits for it.  Send
// and receive go through the context's pinned staging, so the caller's
// buffers are plain host memory.
static int gather_finish(fi_ctx *c) {
  if (!c->gx_pending) return FI_OK;
  c->gx_pending = false;
  HIP_TRY(hipEventSynchronize(c->gx_done));
  if (c->gx_recv && c->gx_recv_bytes)
    memcpy(c->gx_recv, (const uint8_t *)c->gx_pin + c->gx_pin_cap / 2, c->gx_recv_bytes);
  c->gx_recv = nullptr;
  c->gx_recv_bytes = 0;
  return FI_OK;
}
static int gather_start(fi_ctx *c, const fi_record *send, int32_t count, fi_record *recv) {
  int rc = gather_finish(c);  // one gather in flight: its staging is reused
  if (rc) return rc;
  const size_t bytes = sizeof(fi_record) * (size_t)count;
  const size_t rbytes = c->rank == 0 ? bytes * (size_t)c->world : 0;
  const size_t total = bytes * (1 + (c->rank == 0 ? c->world : 0));
  if (c->gather.cap < total + 256) {  // its own buffer: batches never read it (no stream drain to grow it)
    if (c->gx_stream) HIP_TRY(hipStreamSynchronize(c->gx_stream));
    if (c->gather.p) HIP_TRY(hipFree(c->gather.p));
    c->gather.p = nullptr;
    c->gather.cap = 0;
    const size_t cap = std::max(total + total / 4 + 256, (size_t)1 << 16);
    if (hipMalloc(&c->gather.p, cap) != hipSuccess) {
      c->gather.p = nullptr;
      return set_err(FI_ENOMEM, "hipMalloc(%zu) for the record gather failed", cap);
    }
    c->gather.cap = cap;
  }
  // pinned staging: send in the first half, receive in the second
  const size_t half = std::max(bytes, rbytes);
  if (c->gx_pin_cap < 2 * half + 64) {
    if (c->gx_pin) HIP_TRY(hipHostFree(c->gx_pin));
    c->gx_pin = nullptr;
    c->gx_pin_cap = 0;
    const size_t cap = 2 * std::max(half + half / 4, (size_t)4096);
    if (hipHostMalloc(&c->gx_pin, cap, hipHostMallocDefault) != hipSuccess) {
      c->gx_pin = nullptr;
      return set_err(FI_ENOMEM, "hipHostMalloc(%zu) for the record gather failed", cap);
    }
    c->gx_pin_cap = cap;
  }
  if (!c->gx_done) HIP_TRY(hipEventCreateWithFlags(&c->gx_done, hipEventDisableTiming));
  uint8_t *pin_s = (uint8_t *)c->gx_pin, *pin_r = pin_s + c->gx_pin_cap / 2;
  hipStream_t st = c->gx_stream;
  uint8_t *sb = (uint8_t *)c->gather.p, *rb = sb + bytes;  // device: send, then world x count receive
  if (c->rank == 0) {
    if (bytes) memcpy(pin_r, send, bytes);  // rank 0's own records: no device round trip
  } else if (bytes) {
    memcpy(pin_s, send, bytes);
    HIP_TRY(hipMemcpyAsync(sb, pin_s, bytes, hipMemcpyHostToDevice, st));
  }
  // nothing between ncclGroupStart and ncclGroupEnd may return early: the
  // group is always closed, then the first error is reported
  ncclResult_t r = ncclGroupStart();
  if (r != ncclSuccess) return set_err(FI_EDEVICE, "ncclGroupStart: %s", ncclGetErrorString(r));
  if (c->rank == 0) {
    for (int p = 1; p < c->world && r == ncclSuccess; p++)
      r = ncclRecv(rb + bytes * p, bytes, ncclUint8, p, c->comm, st);
  } else {
    r = ncclSend(sb, bytes, ncclUint8, 0, c->comm, st);
  }
  const ncclResult_t re = ncclGroupEnd();
  if (r != ncclSuccess || re != ncclSuccess)
    return set_err(FI_EDEVICE, "RCCL gather: %s", ncclGetErrorString(r != ncclSuccess ? r : re));
  if (c->rank == 0 && recv && rbytes > bytes)
    HIP_TRY(hipMemcpyAsync(pin_r + bytes, rb + bytes, rbytes - bytes, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipEventRecord(c->gx_done, st));
  c->gx_pending = true;
  c->gx_recv = c->rank == 0 ? recv : nullptr;
  c->gx_recv_bytes = c->rank == 0 && recv ? rbytes : 0;
  return FI_OK;
}
int fi_rccl_gather_start(fi_ctx *c, const fi_record *send, int32_t count, fi_record *recv) {
  if (!c || !c->comm || count < 0 || (count > 0 && !send)) return set_err(FI_EINVAL, "RCCL not initialised");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  return gather_start(c, send, count, recv);
}
int fi_rccl_gather_finish(fi_ctx *c) {
  if (!c) return set_err(FI_EINVAL, "ctx is NULL");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  return gather_finish(c);
}
int fi_rccl_gather_records(fi_ctx *c, const fi_record *send, int32_t count, fi_record *recv) {
  if (!c || !c->comm || count < 0 || (count > 0 && !send)) return set_err(FI_EINVAL, "RCCL not initialised");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  const int rc = gather_start(c, send, count, recv);
  return rc ? rc : gather_finish(c);
}
int fi_query(fi_ctx *c, int32_t *running) {
  if (!c || !running) return set_err(FI_EINVAL, "bad arguments");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  int n = 0;
  for (const PendingBatch &pb : c->inflight) {
    const hipError_t e = hipEventQuery(c->slots[pb.slot].done);
    if (e == hipErrorNotReady) {
      n++;
    } else if (e != hipSuccess) {
      return set_err(FI_EDEVICE, "hipEventQuery: %s", hipGetErrorString(e));
    }
  }
  *running = n;
  return FI_OK;
}

}  // extern "C"
