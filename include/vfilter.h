/*
 * vfilter.h — C ABI of libvfilter_hip.so, the MI355X (gfx950) frame-filter backend.
 *
 * This library replaces the per-frame filter of kylemcdonald/distributed-video-filter:
 *
 *     inverted = cv2.bitwise_not(frame)            # inverter.py:41
 *
 * called once per frame from Worker.start()         # worker.py:57 -> inverter.py:29-46
 *
 * The reference is pure Python; its "FFI" for this path is the Python call into
 * OpenCV.  The build's Python side binds these entry points with ctypes
 * (distributed-video-filter_amd/vfilter/_lib.py); INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - every entry point is extern "C", never throws, and returns an int status:
 *     VF_OK (0) on success, a negative VF_E_* code on failure;
 *   - the failing hipError_t and a human-readable message are kept per context
 *     (vf_last_error) and per thread for calls made without a context;
 *   - buffers are plain pointers and byte counts; any alignment and any byte count
 *     (including 0 and counts that are not a multiple of 16) are accepted;
 *   - HIP streams cross the boundary as `void*` (a hipStream_t; NULL = the null stream),
 *     so no HIP or torch type appears in a signature;
 *   - a context is bound to one device and is not thread-safe: one per worker process
 *     (the reference runs one filter per process, worker.py:5-28).
 *
 * Semantics of the filter (OpenCV `bitwise_not`, inverter.py:41): dst[i] = ~src[i] for
 * every byte of a C-contiguous uint8 H x W x 3 frame.  The operation is channel-order
 * agnostic (BGR vs RGB irrelevant) and shape agnostic, so a batch of frames packed back
 * to back is filtered as one byte range.
 */
#ifndef VFILTER_H
#define VFILTER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VF_ABI_VERSION 3

/* status codes */
#define VF_OK           0
#define VF_E_INVALID   -1  /* bad argument (NULL pointer, negative count, size > capacity) */
#define VF_E_HIP       -2  /* a HIP runtime call failed; see vf_last_error / vf_last_hip_error */
#define VF_E_NOMEM     -3  /* host or device allocation failed */
#define VF_E_NODEVICE  -4  /* no usable gfx950 device / bad device ordinal */
#define VF_E_JPEG      -5  /* malformed, truncated or unsupported JPEG stream */

typedef struct vf_ctx vf_ctx;

/* ---- library / context ------------------------------------------------------------ */

/* ABI version of the loaded library (VF_ABI_VERSION).  Makes no HIP call. */
int vf_get_abi_version(void);

/* Static string for a VF_* status code.  Makes no HIP call. */
const char *vf_status_string(int status);

/* Number of visible HIP devices (0 when there is no GPU; never fails for that). */
int vf_device_count(int *out_count);

/* PCI address of HIP device `device` ("dddd:bb:dd.f", from hipDeviceGetPCIBusId) in `buf`
 * (`len` >= 13 bytes).  The host side reads the device's NUMA node from sysfs with it and
 * places that GPU worker's shared-memory frame ring on the node (the reference's workers keep
 * no host buffers of their own: frames arrive in pyzmq messages, worker.py:50-51). */
int vf_device_pci_bus_id(int device, char *buf, int len);

/* Create a context on `device`.  Allocates the pinned host staging ring and device slot
 * buffers used by the host->host entry points (VF_SLOTS slots, default 4, each of
 * min(`max_frame_bytes` x `max_batch`, 16 MiB) bytes; VF_SLOT_BYTES overrides, clamped to
 * [1 MiB, 64 MiB]) and two HIP streams (H2D + kernel, D2H: one SDMA engine per direction).
 * Replaces the per-process filter state of InverterWorker.__init__ (inverter.py:10-20). */
int vf_create(int device, size_t max_frame_bytes, int max_batch, vf_ctx **out);

/* Destroy a context (NULL is allowed).  Synchronises its streams first. */
int vf_destroy(vf_ctx *ctx);

/* Last error message of `ctx`, or of the calling thread when ctx is NULL.  Never NULL.
 * Every failing call also records its message for the calling thread, so a caller that
 * shares one context between threads (JPEG calls lease separate codecs) should read
 * vf_last_error(NULL) on the thread that saw the failure. */
const char *vf_last_error(const vf_ctx *ctx);

/* Last hipError_t recorded by `ctx` (0 if none), or by the calling thread when ctx is NULL. */
int vf_last_hip_error(const vf_ctx *ctx);

/* Device ordinal of the context. */
int vf_ctx_device(const vf_ctx *ctx, int *out_device);

/* ---- host -> host filtering (synchronous) ------------------------------------------- */

/* Invert `nbytes` bytes of host memory: dst[i] = ~src[i].
 * Replaces `cv2.bitwise_not(frame)` (inverter.py:41) for one frame.  `src` and `dst` may
 * be pageable or pinned, any alignment; they must not partially overlap (src == dst is
 * allowed).  Returns when dst is complete.  Paths: when both ranges lie inside page-locked
 * memory noted by vf_alloc_host / vf_host_register, ONE kernel launch reads src and writes
 * dst over PCIe in place (zero-copy: no HBM staging; 48.5 GB/s each way at 1080p x 32, the
 * same as two SDMA copies at once); otherwise H2D || kernel || D2H run pipelined over the
 * context's staging slots (other page-locked memory is DMA'd directly, pageable memory is
 * staged).  VF_ZEROCOPY=0 in the environment at vf_create turns the zero-copy path off. */
int vf_invert_host(vf_ctx *ctx, const uint8_t *src, uint8_t *dst, size_t nbytes);

/* Invert a batch of `n` frames of `frame_bytes` each, packed back to back in `src`;
 * results packed the same way in `dst`.  Replaces the per-frame loop
 * worker.py:35-57 -> inverter.py:41 for a batch.  Same rules as vf_invert_host. */
int vf_invert_batch_host(vf_ctx *ctx, const uint8_t *src, uint8_t *dst,
                         size_t frame_bytes, int n);

/* Invert `n` separately allocated frames (srcs[i] -> dsts[i], nbytes[i] bytes each; sizes
 * may differ, e.g. a mixed 480p/1080p/4K batch).  Frames in page-locked, device-mapped
 * memory are inverted by one launch per 64 frames, all at once (zero-copy); others are
 * gathered into the staging slots, filtered with one launch per slot and scattered back, so
 * small frames are not paid for one launch each.  Frames are independent: one frame's
 * destination must not overlap another frame's source or destination (a frame's own src and
 * dst may be equal).  Replaces worker.py:50-57 + inverter.py:29-46 for a batch of raw
 * frames. */
int vf_invert_frames_host(vf_ctx *ctx, const uint8_t *const *srcs, uint8_t *const *dsts,
                          const size_t *nbytes, int n);

/* ---- host -> host, asynchronous ------------------------------------------------------ */

/* Queue the filter for `n` frames (srcs[i] -> dsts[i], nbytes[i] each) and return at once
 * with a ticket (> 0); the asynchronous form of vf_invert_frames_host (worker.py:57).  The
 * context's engine thread streams queued batches through its slot ring back to back, so a
 * worker can receive its next batch while this one moves.  The caller keeps every buffer
 * alive and untouched until vf_wait(ticket) returns.  Page-locked buffers (vf_alloc_host,
 * vf_host_register, e.g. a shared-memory frame ring) are inverted in place over PCIe by one
 * launch per 64 frames on the context's zero-copy stream; pageable ones are staged through
 * the slot ring.  Tickets of the two paths may complete in either order. */
int vf_invert_frames_async(vf_ctx *ctx, const uint8_t *const *srcs, uint8_t *const *dsts,
                           const size_t *nbytes, int n, uint64_t *ticket);

/* Block until submission `ticket` has completed (its last D2H landed) and return its status.
 * *gpu_ms (may be NULL) gets its device time from first H2D to last D2H (-1 if unknown).
 * Also sets what vf_elapsed_ms / vf_last_timeline report. */
int vf_wait(vf_ctx *ctx, uint64_t ticket, float *gpu_ms);

/* *done = 1 if submission `ticket` has completed, else 0 (never blocks). */
int vf_query(vf_ctx *ctx, uint64_t ticket, int *done);

/* ---- device-resident filtering (asynchronous) -------------------------------------- */

/* Enqueue the invert kernel on `stream` over device memory: ddst[i] = ~dsrc[i].
 * Returns after the launch (does not synchronise).  Kernel-only path used by benchmarks
 * and by callers that keep frames resident in HBM. */
int vf_invert_device(vf_ctx *ctx, const void *dsrc, void *ddst, size_t nbytes, void *stream);

/* Enqueue one launch over `n` device frames given by device-memory descriptor arrays
 * (dsrcs/ddsts/nbytes are themselves arrays in DEVICE memory, n entries each).  For
 * HBM-resident frame pools whose frames are not contiguous. */
int vf_invert_device_frames(vf_ctx *ctx, const void *const *dsrcs, void *const *ddsts,
                            const size_t *nbytes, int n, size_t total_bytes, void *stream);

/* ---- memory helpers --------------------------------------------------------------- */

int vf_alloc_device(vf_ctx *ctx, size_t nbytes, void **out);
int vf_free_device(vf_ctx *ctx, void *p);
/* page-locked host memory (DMA-able without staging) */
int vf_alloc_host(vf_ctx *ctx, size_t nbytes, void **out);
int vf_free_host(vf_ctx *ctx, void *p);
/* page-lock an existing host range (e.g. a shared-memory frame ring) in place */
int vf_host_register(vf_ctx *ctx, void *p, size_t nbytes);
int vf_host_unregister(vf_ctx *ctx, void *p);
/* asynchronous copies on `stream` (synchronous w.r.t. the host if the host side is pageable) */
int vf_upload(vf_ctx *ctx, void *ddst, const void *hsrc, size_t nbytes, void *stream);
int vf_download(vf_ctx *ctx, void *hdst, const void *dsrc, size_t nbytes, void *stream);
int vf_memset_device(vf_ctx *ctx, void *d, int value, size_t nbytes, void *stream);
/* wait for `stream` (NULL = every stream of the context and the device) */
int vf_sync(vf_ctx *ctx, void *stream);

/* ---- timing ----------------------------------------------------------------------- */

/* Sum of kernel durations (ms, hipEvents) of the last host->host call on ctx. */
int vf_elapsed_ms(const vf_ctx *ctx, float *out_ms);

/* Per-chunk GPU timeline of the last host->host call (for Perfetto spans, the GPU side of
 * the reference's trace export, distributor.py:63-171).  For chunk i < min(n, max_chunks):
 * out4[4i..4i+3] = {H2D start, kernel start, kernel end, D2H end} in ms after the call's
 * start event, chunk_bytes[i] = its size (either array may be NULL).  *n_chunks = n.
 * A zero-copy call reports one record {0, 0, t, t}: one launch moved every byte. */
int vf_last_timeline(const vf_ctx *ctx, float *out4, size_t *chunk_bytes, int max_chunks,
                     int *n_chunks);

/* Benchmark loop over HBM-resident buffers: for step s in [0, steps) launch the invert
 * kernel from srcs[s % nbuf] to dsts[s % nbuf] (`nbytes` each, host arrays of device
 * pointers) back to back on `stream`, then synchronise.  A hipEvent pair brackets the whole
 * sequence; its duration (ms) goes to *region_ms (may be NULL).  If per_launch_ms is not
 * NULL, an extra event pair is recorded around every launch and each launch's duration goes
 * to per_launch_ms[s] (the pairs add a few microseconds of gap per launch).  The region pair
 * belongs to the context and is created by its first call (so a timed call only records,
 * launches and synchronises): calls on one context must not overlap. */
int vf_bench_device_ring(vf_ctx *ctx, void *const *srcs, void *const *dsts, int nbuf,
                         size_t nbytes, int steps, void *stream, float *per_launch_ms,
                         float *region_ms);


/* ---- JPEG: the reference's default mode (use_jpeg=True) ------------------------------
 *
 * With use_jpeg=True (the default, inverter.py:10) every frame travels as a JPEG made by
 * PyTurboJPEG (webcam_app.py:110), and the worker runs
 *     frame = self.jpeg.decode(frame_bytes)     # inverter.py:32
 *     inverted = cv2.bitwise_not(frame)         # inverter.py:41
 *     return self.jpeg.encode(inverted)         # inverter.py:44
 * with PyTurboJPEG's defaults (quality 85, TJSAMP_422, TJPF_BGR, flags 0).  These entry
 * points replace those TurboJPEG calls (tjDecompressHeader3 / tjDecompress2 / tjCompress2)
 * with a gfx950 baseline-JPEG codec whose integer arithmetic is libjpeg-turbo's: outputs are
 * bit-exact with libjpeg-turbo.  Constants below are TurboJPEG's (turbojpeg.h).
 * Supported: 8-bit baseline / extended-sequential Huffman JPEG, 1 or 3 components, one
 * interleaved scan, any Huffman tables, with or without restart intervals (DRI / RSTn)
 * (decode); TJSAMP_444/422/420/GRAY/440 (encode).
 * Anything else returns VF_E_JPEG with a message. */
#define VF_TJPF_RGB 0
#define VF_TJPF_BGR 1
#define VF_TJSAMP_444 0
#define VF_TJSAMP_422 1
#define VF_TJSAMP_420 2
#define VF_TJSAMP_GRAY 3
#define VF_TJSAMP_440 4
#define VF_TJFLAG_FASTUPSAMPLE 256   /* replicate chroma instead of fancy upsampling */
#define VF_TJFLAG_FASTDCT 2048       /* "ifast" forward DCT (else the accurate "islow") */
#define VF_TJFLAG_ACCURATEDCT 4096   /* accepted; islow is the default */

/* Header of one JPEG, no GPU work (replaces TurboJPEG.decode_header).  *subsamp = TJSAMP_*
 * (-1 if none matches), *colorspace = TJCS_YCbCr (1) or TJCS_GRAY (2). */
int vf_jpeg_header(const uint8_t *jpeg, size_t size, int *width, int *height, int *subsamp,
                   int *colorspace);

/* Decoder frame-size limit of the context: a JPEG whose SOF claims more than max_pixels
 * (width x height) is refused with VF_E_JPEG before anything is sized from it, as is any side
 * above 65500 (libjpeg's JPEG_MAX_DIMENSION, jdinput.c initial_setup).  0 restores the
 * default, 8192 x 8192.  The frames a worker decodes come off the network
 * (inverter.py:31-32): without a limit, a few hundred bytes of header could ask the codec for
 * tens of GB.  Replaces no reference call (libjpeg-turbo applies only the per-side limit). */
int vf_jpeg_set_max_pixels(vf_ctx *ctx, uint64_t max_pixels);

/* Worst-case size of a vf_jpeg_encode output (tjBufSize); 0 for bad arguments. */
size_t vf_jpeg_buffer_size(int width, int height, int subsamp);

/* Encode n images (inverter.py:44, webcam_app.py:110): imgs[i] is an interleaved 8-bit
 * heights[i] x widths[i] x 3 image in pixel_format; outs[i] receives the JPEG (caps[i]
 * bytes available), sizes[i] its length.  One batched pass on the GPU. */
int vf_jpeg_encode(vf_ctx *ctx, const uint8_t *const *imgs, const int *widths, const int *heights,
                   int n, int pixel_format, int quality, int subsamp, int flags,
                   uint8_t *const *outs, const size_t *caps, size_t *sizes);

/* Decode n JPEGs (inverter.py:32, webcam_app.py:140) into interleaved 8-bit pixels
 * (outs[i] holds width x height x 3 bytes, caps[i] available). */
int vf_jpeg_decode(vf_ctx *ctx, const uint8_t *const *jpegs, const size_t *jpeg_sizes, int n,
                   int pixel_format, int flags, uint8_t *const *outs, const size_t *caps);

/* The whole default-mode filter for n frames on the GPU: decode -> bitwise_not -> encode
 * (inverter.py:32 -> :41 -> :44) with no host round trip of the pixels.  outs[i] receives
 * the inverted JPEG (caps[i] bytes available), sizes[i] its length. */
int vf_jpeg_invert(vf_ctx *ctx, const uint8_t *const *jpegs, const size_t *jpeg_sizes, int n,
                   int quality, int subsamp, int flags, uint8_t *const *outs, const size_t *caps,
                   size_t *sizes);

/* vf_jpeg_invert in three steps, so one host thread keeps batches in flight (the worker loop
 * of worker.py:35-76 receiving batch k+1 while batch k is on the GPU) instead of blocking per
 * batch:
 *   vf_jpeg_invert_submit  parses and stages the batch and queues all of its GPU work; returns
 *                          a ticket without waiting for the GPU.  The inputs are copied: the
 *                          caller may reuse them at once.  Each in-flight batch holds one of the
 *                          context's codecs (at most 8 in flight; never blocks);
 *   vf_jpeg_invert_query   *done = 1 once the batch's results have landed in host memory;
 *   vf_jpeg_invert_wait    blocks until then; *total = bytes of the packed outputs (frames
 *                          back to back, 64-B aligned).  A failed batch ends here (ticket gone);
 *   vf_jpeg_invert_fetch   copies the packed outputs to `out` (cap >= total; frame i is
 *                          sizes[i] bytes at offsets[i]) and ends the batch.  out == NULL ends
 *                          it without copying.  VF_E_INVALID with cap too small keeps it.
 * Same results as vf_jpeg_invert, bit for bit. */
int vf_jpeg_invert_submit(vf_ctx *ctx, const uint8_t *const *jpegs, const size_t *jpeg_sizes, int n,
                          int quality, int subsamp, int flags, uint64_t *ticket);
int vf_jpeg_invert_query(vf_ctx *ctx, uint64_t ticket, int *done);
int vf_jpeg_invert_wait(vf_ctx *ctx, uint64_t ticket, size_t *total);
int vf_jpeg_invert_fetch(vf_ctx *ctx, uint64_t ticket, uint8_t *out, size_t cap, size_t *sizes,
                         size_t *offsets);

/* After vf_jpeg_invert_wait: frame i's inverted JPEG straight into outs[i] when outs[i] is not
 * NULL and the JPEG fits caps[i] (e.g. the output half of the frame's shared-memory ring slot),
 * so the caller needs no packed buffer and no second copy.  sizes[i] = frame i's size either
 * way; *placed = how many frames were copied.  The batch stays open: release it with
 * vf_jpeg_invert_fetch(ctx, ticket, NULL, 0, NULL, NULL), or fetch the frames that did not
 * fit with a packed buffer first. */
int vf_jpeg_invert_scatter(vf_ctx *ctx, uint64_t ticket, uint8_t *const *outs, const size_t *caps,
                           size_t *sizes, int *placed);

/* Benchmark: the GPU part of vf_jpeg_invert (inputs already in HBM) run `iters` times; *ms =
 * mean wall ms per iteration; stage_ms (may be NULL, 8 floats) = mean ms of unstuff, Huffman
 * sync, Huffman write, DC+IDCT, colour+invert, FDCT+Huffman encode, byte stuffing, and the
 * mean number of sync passes. */
int vf_jpeg_bench_invert(vf_ctx *ctx, const uint8_t *const *jpegs, const size_t *jpeg_sizes, int n,
                         int quality, int subsamp, int flags, int iters, float *ms, float *stage_ms);

#ifdef __cplusplus
}
#endif

#endif /* VFILTER_H */
