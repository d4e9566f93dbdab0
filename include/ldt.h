/*
 * ldt.h — C-ABI of libldt.so, the MI355X (gfx950) batch-decode path that
 * replaces lance-distributed-training's per-row PIL/torchvision transform.
 *
 * Drop-in boundary (reference = /root/reference, pure Python):
 *   - to_tensor_fn  decode_tensor_image(batch, **kwargs)   lance_iterable.py:38-50
 *       (registered at LanceDataset(..., to_tensor_fn=...) lance_iterable.py:53-59)
 *   - collate_fn    collate_fn(batch_of_dicts)             lance_map_style.py:21-44
 *       (registered at get_safe_loader(..., collate_fn=...) lance_map_style.py:60-69)
 *   - samplers      ShardedBatchSampler / ShardedFragmentSampler(pad=True)
 *                                                          lance_iterable.py:61-69
 * The reference has no FFI of its own (it is Python over pylance/Pillow); the
 * Python host package ldt_amd binds these symbols with ctypes, exactly as a
 * maintainer would (INTEGRATION.md shows the stub). No torch types cross this
 * boundary: plain pointers, sizes and an opaque hipStream_t passed as void*.
 *
 * Conventions
 *   - Every function returns an int status (LDT_OK == 0, negative = error);
 *     no C++ exception crosses the ABI. ldt_last_error() gives a message.
 *   - Host input pointers are borrowed for the duration of the call only: the
 *     call copies what it needs into the context's pinned staging ring before
 *     returning. Output device pointers are owned by the caller (torch).
 *   - Work is enqueued on `stream` (torch's current stream); results are
 *     stream-ordered. One context per (process, device); a context is not
 *     thread-safe.
 */
#ifndef LDT_H
#define LDT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (return values) ---- */
#define LDT_OK 0
#define LDT_ERR_ARG -1        /* bad argument                                  */
#define LDT_ERR_HIP -2        /* a HIP runtime call failed                     */
#define LDT_ERR_NOMEM -3      /* host/device allocation failed                 */
#define LDT_ERR_IMAGE -4      /* >= 1 image failed: see per_image_status       */

/* ---- per-image status codes (per_image_status[i]) ---- */
#define LDT_IMG_OK 0
#define LDT_IMG_NOT_JPEG 1    /* no SOI / malformed marker segments            */
#define LDT_IMG_UNSUPPORTED 2 /* arithmetic, lossless, 12-bit, CMYK, multi-scan sequential, or a progressive file libjpeg would block-smooth */
#define LDT_IMG_CORRUPT 3     /* entropy data truncated or restart markers wrong */
#define LDT_IMG_TOO_LARGE 4   /* dimension beyond LDT_MAX_DIM                  */
#define LDT_IMG_NULL 5        /* null cell                                     */

#define LDT_MAX_DIM 8192      /* max width/height of a decoded image           */

/* ---- options (ldt_set_option) ---- */
#define LDT_OPT_SYNC_STATUS 1 /* 1 (default): decode calls wait for the stream and
                                 report device-side per-image errors before
                                 returning; 0: asynchronous, errors are read
                                 later with ldt_fetch_status()                  */
#define LDT_OPT_HUFF_MODE 2   /* 0 auto (default) and 2: the parallel
                                 self-synchronising decoder, one workgroup per
                                 image (the serial one for images with > 256
                                 restart segments); 1: serial per segment      */
#define LDT_OPT_SUBSEQ_BITS 3 /* minimum subsequence length of the parallel
                                 decoder: 64..8192 bits, multiple of 32
                                 (default 256); each image uses the smallest
                                 S >= this that fits its slots in 1024 lanes   */
#define LDT_OPT_PROFILE 4     /* 1: record HIP events around every stage on the
                                 caller's stream (read with ldt_stage_times)    */
#define LDT_OPT_RESIZE_IMPL 5 /* 0 auto (default): one wave per band
                                 (k_resize4), the streaming workgroup kernel for
                                 sources wider than 1120 px, 4:2:0 sources
                                 <= 512 px wide with the fancy upsampling on
                                 packed 16-bit pairs (k_resize4<5>); 1: the
                                 same with 32-bit upsampling (k_resize4<0>,
                                 round 3's default, cross-check); 2: the
                                 streaming kernel for all (cross-check)        */
#define LDT_OPT_SYNC_WARM 7   /* parallel decoder phase 1 starts this % of S
                                 before each range (0..200, default 0)         */
#define LDT_OPT_COPY_THREADS 8 /* threads of the context's host copy pool that
                                 move a batch's cells into the pinned slot while
                                 the calling thread walks the headers (0..31;
                                 -1 = default: the cgroup CPU quota divided by
                                 LOCAL_WORLD_SIZE, minus 2, at most 6)         */
#define LDT_OPT_HOST_TIMING 9 /* 1: accumulate host phase times of every
                                 decode call (read with ldt_host_times)        */
#define LDT_OPT_RESIZE_WAVES_PCT 10 /* resize bands per batch as % of one full
                                 wave of resize waves on the device (10..1000,
                                 default 100); more bands fill the pipeline's
                                 CU gaps, fewer keep the kernel efficient      */
#define LDT_OPT_DEBUG_COUNTERS 16 /* 1: the decoders count their phases (cycle
                                 stamps, rounds, symbols) into the plan blob,
                                 read with ldt_debug_counters; 0 (default): no
                                 counters (their atomics cost kernel time)     */
#define LDT_OPT_HUFF_WINDOW 17 /* cap in bytes on the parallel Huffman decoder's
                                 LDS stream window (-1, the default: what the
                                 CU's LDS leaves; 0: every stream read from
                                 global memory, destuffed by k_destuff_*) --
                                 a study knob                  */
#define LDT_OPT_RESIZE_WG_WAVES 15 /* waves (one band each) per k_resize4
                                 workgroup for JPEG sources: 0 default (4),
                                 1, 2 or 4 (tuning knob: 4 keeps 12 waves
                                 per CU at 512 px)           */
#define LDT_OPT_FUSED_DESTUFF 11 /* 1 (default): the parallel Huffman decoder
                                 destuffs the scan bytes of an image whose
                                 stream fits its LDS window itself; 0: every
                                 image through the k_destuff_* kernels
                                 (cross-check)                                  */
#define LDT_OPT_COPY_MODE 12  /* 0 (default): a host batch's cells go to HBM in
                                 one DMA on a per-device copy stream, which
                                 `stream` waits for (the transfer overlaps the
                                 kernels of earlier batches); 1: the DMA on
                                 `stream` itself                              */
#define LDT_OPT_COPY_BIND 13  /* 2 (default): copy-pool threads placed on
                                 physical cores local to the GPU's NUMA node,
                                 spread over its L3 domains, the block of
                                 cores chosen by LOCAL_RANK, each thread free
                                 to run on any CPU of its core's L3 domain;
                                 1: each thread pinned to its core; 0: unbound */
#define LDT_OPT_COPY_NT 14    /* 1 (default): the copy pool writes the pinned slot with
                                 non-temporal stores (AVX2, default); 0: memcpy */

/* ---- stages reported by ldt_stage_times ---- */
#define LDT_STAGE_H2D 0       /* cell + plan copies into HBM                   */
#define LDT_STAGE_DESTUFF 1   /* coefficient clear + k_destuff                 */
#define LDT_STAGE_HUFFMAN 2   /* k_huff_*                                      */
#define LDT_STAGE_IDCT 3      /* k_idct                                        */
#define LDT_STAGE_RESIZE 4    /* k_resize (fused upsample/colour/resize/store) */
#define LDT_NUM_STAGES 5

typedef struct ldt_ctx ldt_ctx;

/* Normalize(mean, std) applied after ToTensor (lance_iterable.py:31). */
typedef struct {
  float mean[3];
  float std[3];
} ldt_norm;

/* Create a decode context on HIP device `device`. max_batch_bytes / max_n are
 * initial workspace hints (buffers grow on demand). Returns NULL on failure. */
ldt_ctx *ldt_create(int device, size_t max_batch_bytes, int max_n);
void ldt_destroy(ldt_ctx *ctx);
const char *ldt_last_error(ldt_ctx *ctx);
int ldt_set_option(ldt_ctx *ctx, int option, int64_t value);
/* The hipStream_t a host batch's cells go to HBM on under LDT_OPT_COPY_MODE 0
 * (NULL, the default: a per-device copy stream the library creates). The
 * stream must outlive the context's use of it; the decode stream waits for
 * the DMA with an event, and the DMA waits for the slot's previous readers. */
int ldt_set_copy_stream(ldt_ctx *ctx, void *stream);
/* Library version string, e.g. "ldt 0.1.0 gfx950". */
const char *ldt_version(void);

/* decode_tensor_image / collate_fn core, Arrow `binary` column (int32 offsets).
 *   data, offsets      : the Arrow array's data and offsets buffers (host);
 *   arr_offset         : Array.offset (slices share buffers), in rows;
 *   n                  : rows;
 *   validity           : Arrow validity bitmap or NULL (a null cell -> LDT_IMG_NULL);
 *   labels             : int64 label buffer (host) or NULL, label_offset in rows;
 *   out_img_dev        : float32 [n, 3, 224, 224] contiguous, device;
 *   out_lbl_dev        : int64 [n], device (ignored when labels == NULL);
 *   norm_or_null       : NULL = ToTensor only, else Normalize(mean, std) fused;
 *   stream             : hipStream_t (void*), 0 = null stream;
 *   per_image_status   : int32 [n] host, written with LDT_IMG_* codes.
 * Replaces lance_iterable.py:41-49 (to_pylist + PIL open/convert + Resize +
 * ToTensor + stack) and lance_map_style.py:34-44. */
int ldt_decode_batch(ldt_ctx *ctx, const uint8_t *data, const int32_t *offsets,
                     int64_t arr_offset, int64_t n, const uint8_t *validity,
                     const int64_t *labels, int64_t label_offset, float *out_img_dev,
                     int64_t *out_lbl_dev, const ldt_norm *norm_or_null, void *stream,
                     int32_t *per_image_status);

/* Same, Arrow `large_binary` column (int64 offsets). */
int ldt_decode_batch_large(ldt_ctx *ctx, const uint8_t *data, const int64_t *offsets,
                           int64_t arr_offset, int64_t n, const uint8_t *validity,
                           const int64_t *labels, int64_t label_offset, float *out_img_dev,
                           int64_t *out_lbl_dev, const ldt_norm *norm_or_null, void *stream,
                           int32_t *per_image_status);

/* Device-resident input (bench / pre-staged loaders): the JPEG cells already
 * live in HBM at data_dev (same layout as the host copy data_host, which is
 * read only for the marker headers). offsets are int64, host, absolute byte
 * offsets of each cell in both buffers (n+1 entries). Labels as above. */
int ldt_decode_batch_resident(ldt_ctx *ctx, const uint8_t *data_host, const uint8_t *data_dev,
                              const int64_t *offsets, int64_t n, const int64_t *labels,
                              float *out_img_dev, int64_t *out_lbl_dev,
                              const ldt_norm *norm_or_null, void *stream,
                              int32_t *per_image_status);

/* Zero-copy host input. ldt_register_host page-locks [ptr, ptr+len) in place
 * (hipHostRegister) for every context of the process: a later ldt_decode_batch
 * whose cells lie inside a registered range copies them to HBM by DMA straight
 * from those pages, without the memcpy into the context's pinned ring. Meant
 * for a memory-mapped Arrow IPC / Lance fragment registered once (the
 * dataset's `image` data buffer), replacing the per-batch copy SURVEY.md
 * §8f row 1 names. The range must stay mapped until ldt_unregister_host(ptr),
 * which waits for the device first. Returns LDT_OK or LDT_ERR_* (a range the
 * driver cannot lock stays on the copying path). */
int ldt_register_host(ldt_ctx *ctx, const void *ptr, size_t len);
int ldt_unregister_host(ldt_ctx *ctx, const void *ptr);

/* Wait for the last decode on `stream` and merge device-side per-image errors
 * into per_image_status[n] (for LDT_OPT_SYNC_STATUS = 0). */
int ldt_fetch_status(ldt_ctx *ctx, void *stream, int32_t *per_image_status, int64_t n);

/* Tickets (LDT_OPT_SYNC_STATUS = 0): every decode call that enqueues work gets
 * the next ticket of its context (1, 2, ...; ldt_last_ticket returns the most
 * recent one, 0 before any). A context holds the device-side status of its
 * last two calls: ldt_fetch_status_ticket waits only for that call's batch
 * (not for newer work on the stream) and merges its errors as above; a ticket
 * older than the last two returns LDT_ERR_ARG. This lets a pipeline check a
 * batch two uses of the context later, long after it completed, instead of
 * synchronising on the batch just before it. Replaces the per-batch status
 * check of lance_iterable.py:42 (PIL raising in the loop) without a stall. */
int64_t ldt_last_ticket(ldt_ctx *ctx);
int ldt_fetch_status_ticket(ldt_ctx *ctx, int64_t ticket, int32_t *per_image_status, int64_t n);

/* Profiling (LDT_OPT_PROFILE = 1): waits for every recorded stage event and
 * adds the elapsed milliseconds of each stage since the last reset into
 * ms_out[stage] and the number of timed launches into count_out[stage]
 * (arrays of LDT_NUM_STAGES). reset != 0 clears the accumulators after reading. */
int ldt_stage_times(ldt_ctx *ctx, double *ms_out, int64_t *count_out, int reset);

/* Host phase times (LDT_OPT_HOST_TIMING = 1), microseconds summed over the
 * timed calls since the last reset, into us_out[LDT_NUM_HOST_PHASES]:
 * pinned slot + copy start, header walk (overlaps the cell copy), plan blob,
 * cell copy join + H2D enqueue, kernel launches, status; then two copy-pool
 * diagnostics that overlap those: the pool's wake-up (copy start to the first
 * chunk a pool thread took) and the copy's span (start to last chunk done);
 * *calls_out = calls. */
#define LDT_NUM_HOST_PHASES 8
int ldt_host_times(ldt_ctx *ctx, double *us_out, int64_t *calls_out, int reset);

/* The context's host copy placement as a JSON object (NUL-terminated, into
 * buf[len]): copy_threads, copy_cpus, gpu_numa (the GPU's NUMA node from
 * sysfs), quota_cpus (cgroup), local_rank / local_world (torchrun's
 * LOCAL_RANK / LOCAL_WORLD_SIZE), l3_domains, candidate_cores, and the
 * copy_bind / copy_nt / copy_mode options, local_cpulist (the GPU's local
 * CPUs from sysfs, "" if unknown). Creates the pool if needed. */
int ldt_host_info(ldt_ctx *ctx, char *buf, size_t len);

/* Diagnostics (LDT_OPT_DEBUG_COUNTERS = 1): waits for `stream`, then copies the
 * parallel Huffman decoder's 16 int32 counters of the last batch into out16,
 * summed over its images: [1] images, [2] convergence rounds (sum), [3] rounds
 * (max), [4] memo adoptions, [5] write-pass symbols (sum over lanes), [6] the
 * symbols of each wave's slowest lane (sum), [8] setup, [9] phase 1, [10]
 * rounds, [11] block-count scan, [12] write pass (10 ns ticks), [13] needy
 * slots and [14] the waves they ran on (summed over rounds); [0], [7], [15]
 * unused. LDT_ERR_ARG when no batch was decoded with the option on. */
int ldt_debug_counters(ldt_ctx *ctx, int32_t *out16, void *stream);

/* Config 5: raw uint8 HWC cells (no JPEG) -> Resize(224,224) [+Normalize] ->
 * float32 [n,3,224,224]. `hwc` is a device pointer when hwc_is_device != 0,
 * else host (copied through the pinned ring). Cell i starts at
 * hwc + i * cell_stride bytes and is h*w*3 bytes. */
int ldt_resize_raw(ldt_ctx *ctx, const uint8_t *hwc, int hwc_is_device, int64_t n, int h, int w,
                   int64_t cell_stride, float *out_img_dev, const ldt_norm *norm_or_null,
                   void *stream);

/* ShardedBatchSampler index computation (README.md:257-271), on device.
 * Writes the rank's batch row ranges as int64 pairs [start, end) into
 * out_ranges_dev (capacity pairs) and the pair count into *out_count_dev.
 * Batch k = [k*B, min(k*B+B, num_rows)), rank r gets k = r, r+W, ... */
int ldt_shard_ranges(ldt_ctx *ctx, int64_t num_rows, int64_t batch_size, int rank,
                     int world_size, int64_t *out_ranges_dev, int64_t capacity,
                     int64_t *out_count_dev, void *stream);

/* ShardedFragmentSampler index computation (README.md:140-155), on device.
 * fragment_rows_dev: int64 [nfrag] rows per fragment (dataset order).
 * Writes records of 5 int64 {fragment, start, end, global_start, is_pad} for
 * the rank's batches (fragments r, r+W, ...; batches never cross fragments)
 * into out_dev (capacity records), and the record count into *out_count_dev.
 * pad_to < 0: no padding. pad_to >= 0: pad the rank's list to pad_to records
 * (the max-over-ranks count agreed by all_reduce(MAX)) with this build's rule:
 * cycle the rank's own batches; a rank with no rows cycles the global batch
 * list from index `rank`. *out_local_count_dev receives the unpadded count. */
int ldt_shard_fragments(ldt_ctx *ctx, const int64_t *fragment_rows_dev, int nfrag,
                        int64_t batch_size, int rank, int world_size, int64_t pad_to,
                        int64_t *out_dev, int64_t capacity, int64_t *out_count_dev,
                        int64_t *out_local_count_dev, void *stream);

/* torch.utils.data.DistributedSampler index computation, on device — the
 * map-style loader's sampler (lance_map_style.py:58 -> torch 2.10
 * torch/utils/data/distributed.py:94-103 (num_samples) and :107-141 (__iter__)).
 * Writes the rank's num_samples indices (int64) into out_dev (capacity
 * entries) and num_samples into *num_samples_out (host, may be NULL):
 *   perm = torch.randperm(dataset_len, generator=manual_seed(seed)) when
 *   shuffle != 0 (bit-exact: MT19937 seeded with the low 32 bits of the 64-bit
 *   torch seed, forward Fisher-Yates), else the identity; padded by wrapping
 *   (drop_last == 0) or truncated; then every num_replicas-th from rank.
 * `seed` is the sampler's seed + epoch as torch's uint64 seed (two's complement
 * for negative values). dataset_len must be < 2^32/20 (torch draws 64-bit
 * numbers beyond that). */
int ldt_distributed_indices(ldt_ctx *ctx, int64_t dataset_len, int num_replicas, int rank,
                            int shuffle, uint64_t seed, int drop_last, int64_t *out_dev,
                            int64_t capacity, int64_t *num_samples_out, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* LDT_H */
