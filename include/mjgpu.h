/*
 * mjgpu.h -- C-ABI of libmjgpu.so, the MI355X (gfx950) MJPEG segment encoder.
 *
 * Drop-in boundary.  The reference (Rouji/ffmpeg_distributed) has no FFI: its hot
 * path is the per-segment worker process built at ffmpeg_distributed.py:131-138
 *     nice -n10 ionice -c3 ffmpeg -f matroska -i pipe: <remote_args> -f matroska pipe:
 * and launched/supervised at ffmpeg_distributed.py:139-141 (FFMPEGProc.run,
 * ffmpeg_distributed.py:59-91).  For the north-star profile
 *     [-vf scale=W:H:flags=bicubic] -c:v mjpeg -q:v N -dct int -huffman default -bitexact
 * this library replaces the arithmetic that worker runs (swscale bicubic + tv->pc
 * range conversion, jfdctint + quantiser + default-table Huffman + 0xFF stuffing)
 * and the Python host code in ffmpeg_distributed_amd/ (worker.py, dispatcher.py)
 * replaces the process around it with the same stdin/stdout/stderr/exit-code
 * contract.  Plain C types only; no torch types cross this boundary.
 *
 * Threading: one mjg_ctx per (device, caller thread); a ctx owns its HIP stream,
 * device buffers and filter tables.  Calls on different contexts may run
 * concurrently.  The library never writes to stdout (stdout is the data stream).
 * Every call returns MJG_OK (0) or a negative MJG_E_* code; mjg_last_error()
 * returns a thread-local description of the last failure.
 */
#ifndef MJGPU_H
#define MJGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MJG_OK 0
#define MJG_E_INVALID (-1)     /* bad argument / unsupported geometry */
#define MJG_E_HIP (-2)         /* HIP runtime error (no device, launch failure ...) */
#define MJG_E_NOMEM (-3)       /* device or pinned-host allocation failed */
#define MJG_E_CAPACITY (-4)    /* caller buffer too small */
#define MJG_E_STATE (-5)       /* call out of order (e.g. fetch before submit) */

/* mjg_config.flags */
#define MJG_F_TIMING 1u        /* record HIP events around every kernel launch */
#define MJG_F_DEBUG_COEFS 2u   /* keep quantized coefficients of every block (tests) */
#define MJG_F_SWS_NO_BITEXACT 4u /* swscale filter tables without SWS_BITEXACT */
#define MJG_F_COM_ITU601 8u    /* add COM "CS=ITU601" (FFmpeg builds whose CLI hands the encoder
                                  yuv420p+full-range instead of yuvj420p; mjpegenc_common.c
                                  jpeg_put_comments) */
#define MJG_F_HUFFMAN_OPTIMAL 16u /* -huffman optimal (FFmpeg's default): per-frame Huffman tables
                                  from the frame's symbol counts (mjpegenc_huffman.c); the
                                  header's DHT then differs per frame */
#define MJG_F_RST 32u          /* slice-threaded bitstream (-slices N / -thread_type slice): DRI =
                                  MCUs per row, every MCU row its own entropy-coded segment
                                  (DC predictors reset, 1-bit padded, RST0..7 between rows;
                                  mpegvideo_enc.c encode_thread rtp_mode + mjpegenc.c
                                  ff_mjpeg_encode_stuffing).  Implies -huffman default, as
                                  FFmpeg forces; MJG_F_RST | MJG_F_HUFFMAN_OPTIMAL is invalid */

/* mjg_config.chroma_format */
#define MJG_CHROMA_420 0       /* yuv(j)420p: MCU 16x16, Y 2x2 Cb 1x1 Cr 1x1 */
#define MJG_CHROMA_422 1       /* yuv(j)422p: MCU 16x16, Y 2x2 Cb 1x2 Cr 1x2 */
#define MJG_CHROMA_444 2       /* yuv(j)444p: MCU 8x16, every component 1x2 (ff_mjpeg_init_hvsample) */

#define MJG_F_TIMING_DETAIL 64u /* MJG_F_TIMING plus events around every tail kernel (scan, 0xFF
                                  count, write: MJG_K_SCAN_BITS .. MJG_K_WRITE); each event adds
                                  ~10 us of GPU idle between those short kernels */
#define MJG_F_MERGE 1024u      /* opt-in library-side merging: single-segment device submits are held
                                  and launched two at a time (see mjg_submit; the caller keeps each
                                  submit's frames valid until its own mjg_sync).  Without it every
                                  mjg_submit is a launch of its own, launched inside the call */

/* Kernel ids for mjg_kernel_times() */
#define MJG_K_SCALE 0          /* bicubic hscale + range + vscale (per plane) */
#define MJG_K_ENCODE 1         /* load + FDCT + quant + Huffman -> chunk bits */
#define MJG_K_SCAN_BITS 2      /* per-frame exclusive scan of chunk bit lengths      */
#define MJG_K_COUNT_FF 3       /* realign chunk bits, pad, count 0xFF per chunk group */
#define MJG_K_SCAN_FF 4        /* per-frame scan of 0xFF counts -> frame sizes, offsets */
#define MJG_K_WRITE 5          /* header + stuffed scan + EOI into packed output     */
#define MJG_K_HUFF 6           /* -huffman optimal: symbol-count pass + table build   */
#define MJG_K_TAIL 7           /* MJG_K_SCAN_BITS .. MJG_K_WRITE as one interval (MJG_F_TIMING) */
#define MJG_NUM_KERNELS 8

typedef struct mjg_config {
  int32_t src_w, src_h;      /* decoded frame size (packed I420: Y, then U, then V)    */
  int32_t dst_w, dst_h;      /* encoded size; == src when remote_args has no -vf scale */
  int32_t in_full_range;     /* 1: yuvj420p input; 0: yuv420p (tv) -> tv->pc as swscale */
  int32_t qscale;            /* effective mpegvideo qscale, 2..31 (see -q:v mapping)   */
  int32_t sar_num, sar_den;  /* JFIF APP0 density; 0/0 omits APP0 (unknown SAR)        */
  int32_t max_batch;         /* most frames one mjg_submit() may carry                 */
  uint32_t flags;            /* MJG_F_*                                                */
  int32_t chroma_format;     /* MJG_CHROMA_*; frames are packed planar Y, Cb, Cr       */
} mjg_config;

typedef struct mjg_ctx mjg_ctx;

/* Library version (major*10000 + minor*100 + patch). */
int mjg_version(void);
/* Thread-local text of the last error (never NULL). */
const char *mjg_last_error(void);
/* Number of visible HIP devices, or a negative MJG_E_* code. */
int mjg_device_count(void);
/* NUMA node of `device` (its PCI function's numa_node in sysfs), -1 when the platform does
 * not say, or a negative MJG_E_* code.  The worker binds its reader threads to that node. */
int mjg_device_numa_node(int device);

/* Create a context on `device`: validates cfg, builds quant/Huffman/filter tables,
 * allocates device buffers for cfg->max_batch frames.  Replaces one
 * `ffmpeg ... <remote_args>` worker's codec/scaler initialisation
 * (ffmpeg_distributed.py:131-138). */
int mjg_open(int device, const mjg_config *cfg, mjg_ctx **out);
void mjg_close(mjg_ctx *ctx);

/* Bytes of one packed planar input frame (src_w x src_h in cfg->chroma_format). */
size_t mjg_frame_bytes(const mjg_ctx *ctx);
/* The per-config JPEG header (SOI .. SOS) every frame starts with.  With
 * MJG_F_HUFFMAN_OPTIMAL each frame carries its own DHT; this returns the header with the
 * default tables (same layout, different DHT contents). */
int mjg_header(const mjg_ctx *ctx, uint8_t *out, size_t cap, size_t *len);

/* Encode `nframes` (<= max_batch) packed I420 frames, asynchronously: H2D, scale and
 * k_encode on a launch slot's stream, the scan/stuff/write tail on the ctx's tail stream
 * after the launch's k_encode.  mjg_queue_depth() launches may be queued (each has its own
 * output and scratch buffers and its own stream): the next one's k_encode runs beside the
 * previous one's drain and tail.  src_is_device = 0: `frames` is host memory (copied H2D
 * through the slot's staging buffer; pinned memory from mjg_host_alloc() makes this
 * asynchronous), a launch of its own; src_is_device = 1: `frames` is device memory on ctx's
 * device, read in place.  Without MJG_F_MERGE every submit is launched (stream-ordered) inside
 * this call.  With MJG_F_MERGE (opt-in; MJG_MERGE=1 in the environment turns it off again) a
 * device submit is held and launched together with the next device submit, as one segment
 * list (mjg_submit_segments' kernels), or alone when the caller syncs it; each submit stays a
 * job of its own for mjg_sync / mjg_fetch with exactly the bytes of an unmerged launch.  A held
 * submit's kernels read its frames after this call returns, so with MJG_F_MERGE the frames must
 * stay valid and unchanged until the job is synced (stream order on the caller's side does not
 * protect them).  Up to mjg_ctx_queue_depth(ctx) device submits may be pending; MJG_E_STATE
 * past that (or when no launch slot is free for a host submit).
 * Replaces the per-segment encode the reference runs at ffmpeg_distributed.py:139-141. */
int mjg_submit(mjg_ctx *ctx, const uint8_t *frames, int nframes, int src_is_device);
/* Several segments in one submit: segment k's seg_nframes[k] packed I420 frames at device
 * pointer seg_frames[k] (on ctx's device), nsegs in 1..mjg_max_segments(), the total within
 * max_batch.  One launch of each kernel (k_scale, k_encode, the tail) covers all
 * of them, so the launch's ramp and drain are paid once; the output is the frames in segment
 * order, exactly the bytes of one mjg_submit per segment.  The resident encoder / a GPU worker
 * with several segments queued on one GPU (ffmpeg_distributed.py:139-141 once per segment)
 * hands them over together. */
int mjg_submit_segments(mjg_ctx *ctx, const uint8_t *const *seg_frames, const int *seg_nframes, int nsegs);
/* Most segments one mjg_submit_segments() may carry (4). */
int mjg_max_segments(void);
/* Wait for the oldest pending submit (with none pending: report the last synced one again;
 * a held one is launched first).
 * frame_sizes (may be NULL) receives its nframes JPEG sizes; *total (may be NULL) the packed
 * total.  Grows the output buffer and re-runs the final kernel if the packed output
 * exceeded its capacity. */
int mjg_sync(mjg_ctx *ctx, uint64_t *frame_sizes, uint64_t *total);
/* Copy the packed JPEGs of the last synced submit (frame after frame) to host memory; syncs
 * the oldest queued submit first when mjg_sync was not called since the last mjg_submit.
 * Page-locked `out` (from mjg_host_alloc) receives them by one DMA; pageable memory through
 * the context's page-locked buffer (mjg_fetch_host) and one host copy. */
int mjg_fetch(mjg_ctx *ctx, uint8_t *out, size_t cap);
/* The same bytes without the copy into caller memory: *data points at the context's
 * page-locked copy (DMA'd from the device), *len its size; valid until the next
 * mjg_fetch / mjg_fetch_host or mjg_close. */
int mjg_fetch_host(mjg_ctx *ctx, const uint8_t **data, size_t *len);
/* Device pointers of the packed output and of the per-frame byte offsets (nframes+1
 * entries, valid after mjg_sync). */
int mjg_output_device(mjg_ctx *ctx, const uint8_t **data, const uint64_t **offsets);
/* The hipStream_t the next submit launches H2D, scale and k_encode on (for event timing by
 * the caller; the tail kernels run on another stream ordered after k_encode).  Consecutive
 * submits rotate over mjg_queue_depth() such streams. */
void *mjg_stream(mjg_ctx *ctx);
/* How many launches may be queued before one must be synced (2): the depth for host submits
 * and mjg_submit_segments, which each take a launch of their own. */
int mjg_queue_depth(void);
/* How many single-segment device submits (mjg_submit, src_is_device = 1) ctx holds pending
 * before one must be synced: with MJG_F_MERGE mjg_queue_depth() launches of up to two merged
 * submits each (4), else mjg_queue_depth(). */
int mjg_ctx_queue_depth(const mjg_ctx *ctx);

/* Pinned host memory for mjg_submit / mjg_fetch. */
int mjg_host_alloc(size_t bytes, void **ptr);
int mjg_host_free(void *ptr);

/* Average device time (ms) per launch of each kernel (MJG_K_*) since the last reset,
 * and the number of submits it was averaged over.  Needs MJG_F_TIMING. */
int mjg_kernel_times(mjg_ctx *ctx, double *ms /* [MJG_NUM_KERNELS] */, int *launches, int reset);

/* Device-free helpers (no HIP call; usable on a host without a GPU). */
/* The per-config JPEG header (SOI .. SOS) for cfg (dst_w/dst_h/qscale/sar/chroma_format and the
 * MJG_F_COM_ITU601 / MJG_F_RST flags are read). */
int mjg_build_header(const mjg_config *cfg, uint8_t *out, size_t cap, size_t *len);
/* swscale bicubic filter table the scale stage applies: one = 1<<14 (horizontal) or 1<<12
 * (vertical); align = 4 / 2 (x86 swscale); pos = swscale local position (128 = centred).
 * coeff receives dst_len*taps int16, pos_out dst_len int32; query taps with coeff == NULL. */
int mjg_sws_filter(int src_len, int dst_len, int one, int align, int bitexact, int src_pos,
                   int dst_pos, int16_t *coeff, size_t coeff_cap, int32_t *pos_out, int *taps);

/* Test hooks (tests/ only). */
/* Quantized coefficients (natural order) of frame `frame` of the last submit, blocks
 * in coding order (4:2:0: Y0 Y1 Y2 Y3 Cb Cr per MCU).  Needs MJG_F_DEBUG_COEFS. */
int mjg_debug_coefs(mjg_ctx *ctx, int frame, int16_t *out, size_t nblocks);
/* The full-range encoder-input planes (after scale/range stage) of frame `frame`,
 * packed planar at dst size.  Only for a scaling config. */
int mjg_debug_planes(mjg_ctx *ctx, int frame, uint8_t *out, size_t cap);
/* Filter tables the context generated: plane 0 = luma, 1 = chroma; dir 0 = horizontal,
 * 1 = vertical.  taps/len may be queried with coeff == NULL. */
int mjg_debug_filter(mjg_ctx *ctx, int plane, int dir, int16_t *coeff, int32_t *pos,
                     int *taps, int *len);
/* -huffman optimal's table builder (k_huff_build) on given symbol counts, on GPU `device`:
 * hist[f][544] (AC luma 0-255, AC chroma 256-511, DC luma 512-527, DC chroma 528-543) for
 * nframes frames -> dht[f][t][272] (BITS[1..16] then HUFFVAL; t: 0 DC luma, 1 DC chroma,
 * 2 AC luma, 3 AC chroma) and nval[f][t] (HUFFVAL entries).  Replaces the table build of
 * ff_mjpeg_encode_huffman_close (libavcodec/mjpegenc_huffman.c); tests compare it with the oracle. */
int mjg_debug_huff_build(int device, const uint32_t *hist, int nframes, uint8_t *dht, uint32_t *nval);

#ifdef __cplusplus
}
#endif
#endif /* MJGPU_H */
