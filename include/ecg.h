/*
 * ecg.h -- MI355X-native Reed-Solomon erasure-coding engine for DAOS EC
 * objects: the core C-ABI.
 *
 * Plain C, host pointers / device pointers / sizes only (no HIP, no torch
 * types).  Streams are opaque `void *` (a hipStream_t; NULL = the context's
 * own stream).  Every function returns 0 or a negative DAOS errno
 * (ref:src/include/daos_errno.h); ecg_strerror() gives the detail of the last
 * failure on the calling thread.  All entry points are thread-safe.
 *
 * What this replaces: the arithmetic boundary of DAOS's EC
 * object class -- ISA-L ec_encode_data / ec_encode_data_update / xor_gen as
 * called from ref:src/object/cli_ec.c:540,571,2641,
 * ref:src/object/srv_ec_aggregate.c:693,1092,1099,1136 -- batched over stripes
 * and executed by hand-written gfx950 kernels on device-resident cells.
 * The ISA-L-signature drop-in is ecg_isal.h; the DAOS codec surface
 * (obj_ec_codec_*, obj_ec_encode_buf, recovery codec) is ecg_daos.h.
 *
 * Arithmetic is GF(2^8) with polynomial 0x11d and generator 2, bit-exact with
 * ISA-L's ec_encode_data_base (and therefore with every ISA-L SIMD path).
 */
#ifndef ECG_H
#define ECG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Negative DAOS errno values (ref:src/include/daos_errno.h). */
#define ECG_DER_INVAL		1003
#define ECG_DER_NOMEM		1009
#define ECG_DER_NOSYS		1010	/* no gfx950 device / HIP runtime */
#define ECG_DER_IO		2001	/* HIP runtime or kernel failure */
#define ECG_DER_REC2BIG		2013
#define ECG_DER_DATA_LOSS	2026	/* more erasures than parity cells */

/* Limits (ref:src/object/obj_ec.h:16-20, ref:src/object/obj_class.c:587-601). */
#define ECG_MAX_K		64
#define ECG_MAX_P		8

/* Parity row pitch.  Client-layout parity [p][S][C] runs fastest with its p
 * rows one buffer at a pitch of S*C + ECG_PARITY_ROW_PAD: rows a large power
 * of two apart, or separately allocated rows the allocator happens to place
 * at such distances, alias in HBM (measured, profiles/r05/: EC_4P2 1 MiB x
 * 1024 encode with the rows as two hipMalloc allocations 0.91 of the padded
 * rate, EC_8P2 x 512 with the unpadded pitch 0.96).  The library's own
 * staging pads its parity rows this way; callers choose their own layout. */
#define ECG_PARITY_ROW_PAD	4096

/* Flags for ecg_matmul */
#define ECG_F_ACCUMULATE	0x1u	/* dst ^= product (else dst = product) */

typedef struct ecg_ctx ecg_ctx_t;

/* ---- context / device ---------------------------------------------------- */
/* Number of usable (gfx950) HIP devices; 0 when none.  Never fails. */
int ecg_device_count(void);
/* Binds a context to `device` (index into the visible HIP devices).
 * -ECG_DER_NOSYS when the device is absent or not gfx950: the batched device
 * API has no CPU fallback (the drop-in surfaces route host cells to the CPU
 * path themselves, ecg_set_dropin_crossover). */
int ecg_ctx_create(int device, ecg_ctx_t **ctx);
void ecg_ctx_destroy(ecg_ctx_t *ctx);
int ecg_ctx_device(const ecg_ctx_t *ctx);
/* 1 when the context's device served misaligned dword loads and stores at
 * creation (the unaligned access mode ROCm enables on gfx9+): destinations
 * off a dword boundary then run on the vector lanes; 0 when it did not (or
 * ECG_UNALIGNED=0 was set): such launches run the byte kernels, same
 * results, ~8x slower.  The probe assumes a misaligned access is served (or
 * rounded), not trapped: on a device configured to FAULT on misaligned
 * accesses, set ECG_UNALIGNED=0 before creating a context. */
int ecg_ctx_unaligned_ok(ecg_ctx_t *ctx);
/* PCI bus id ("0000:c1:00.0") of a visible device: tells ranks or shards
 * that landed on the same physical GPU apart. */
int ecg_device_pci_bus_id(int device, char *buf, int len);
/* NUMA node of a PCI device ("0000:23:00.0", any case) from sysfs
 * (/sys/bus/pci/devices/<bdf>/numa_node), and of a HIP device; -1 when
 * unknown.  ecg_multi workers run on their device's node and queue staging
 * is allocated there; $ECG_NUMA=0 turns that off. */
int ecg_pci_numa_node(const char *pci_bus_id);
int ecg_device_numa_node(int device);
/* The context's default stream (used when a call passes stream == NULL). */
void *ecg_ctx_stream(ecg_ctx_t *ctx);
const char *ecg_strerror(void);
/* Name of the kernel the last ecg_* compute call on this thread launched. */
const char *ecg_last_kernel(void);
/* Identity of this build: "src_sha256=<16 hex>;hipcc=<version>;arch=gfx950",
 * the hash over every source, header and build file of the library
 * (daos_amd/csrc/Makefile HASHED), fixed at build time. */
const char *ecg_build_info(void);

/* ---- field and matrices (host; setup only) ------------------------------- */
unsigned char ecg_gf_mul(unsigned char a, unsigned char b);
unsigned char ecg_gf_inv(unsigned char a);
/* (k+p) x k Cauchy1 encode matrix: identity rows then 1/(i ^ j), the matrix
 * DAOS builds per EC class (ref:src/object/obj_class.c:611-617). */
int ecg_gen_cauchy1(int k, int p, unsigned char *en_matrix);
/* n x n inverse over GF(2^8); `in` is destroyed; -ECG_DER_INVAL if singular. */
int ecg_invert_matrix(unsigned char *in, unsigned char *out, int n);
/* DAOS recovery codec (ref:src/object/cli_ec.c:2152-2250): for LOGICAL error
 * indices err_list[nerrs] (cells 0..k-1 data, k..k+p-1 parity) produce the
 * decode rows (nerrs x k, in err_list order), dec_idx[k] (the surviving cells
 * they consume) and *reused_encode (1 when all p parity cells and no data
 * cell are lost: rows are then the encode parity rows and dec_idx = 0..k-1,
 * ref:src/object/cli_ec.c:2205-2210).  -ECG_DER_DATA_LOSS when nerrs > p. */
int ecg_recov_matrix(int k, int p, const unsigned char *en_matrix,
		     const uint32_t *err_list, int nerrs, unsigned char *de_rows,
		     uint32_t *dec_idx, int *reused_encode);

/* ---- device-resident batched codec (the hot path) ----------------------- */
/*
 * dst cell r of stripe s  (^)=  XOR_{j<k} coef[r*k + j] * (src cell j of s)
 * for every byte i < cell_bytes and every stripe s < nstripes, where
 *   src cell j of s = src + s*src_stripe_stride + src_cell_off[j]
 *   dst cell r of s = dst + s*dst_stripe_stride + dst_cell_off[r]
 * All pointers are device pointers.  k <= 64, rows <= 8 (larger k is split
 * into accumulating launches).  Any alignment: 16-byte aligned cells run
 * 16-byte lanes, dword-aligned sources dword lanes, sources at any byte
 * funnel-shifted dword lanes; outputs at any byte are stored as misaligned
 * dwords by the same lanes.
 * Asynchronous on `stream`.
 */
int ecg_matmul(ecg_ctx_t *ctx, int k, int rows, const unsigned char *coef,
	       uint64_t cell_bytes, uint32_t nstripes,
	       const void *src, const int64_t *src_cell_off, int64_t src_stripe_stride,
	       void *dst, const int64_t *dst_cell_off, int64_t dst_stripe_stride,
	       unsigned flags, void *stream);

/* Full-stripe encode with the Cauchy1 matrix (ISA-L ec_encode_data with the
 * DAOS codec tables).  Data cell j of stripe s at
 *   data + s*data_stripe_stride + j*cell_bytes,
 * parity cell r of stripe s at
 *   parity + r*parity_cell_stride + s*parity_stripe_stride.
 * Client write layout (ref:src/object/cli_ec.c:75-97,638-640): data [S][k][C],
 * parity [p][S][C] => data_stripe_stride = k*C, parity_cell_stride = S*C,
 * parity_stripe_stride = C.  Recovery layout [S][k+p][C] => parity = data +
 * k*C, parity_cell_stride = C, both stripe strides (k+p)*C. */
int ecg_encode(ecg_ctx_t *ctx, int k, int p, uint64_t cell_bytes, uint32_t nstripes,
	       const void *data, int64_t data_stripe_stride,
	       void *parity, int64_t parity_cell_stride, int64_t parity_stripe_stride,
	       void *stream);

/* In-place degraded-read / rebuild recovery over stripes laid out
 * [S][k+p][cell_bytes] in logical cell order, stripe s at
 * stripes + s*stripe_stride (obj_ec_recov_data, ref:src/object/cli_ec.c:
 * 2814-2885).  Erased cells (logical indices) are regenerated from the first
 * k survivors.  Decode matrices are cached per (k, p, err_list). */
int ecg_recover(ecg_ctx_t *ctx, int k, int p, uint64_t cell_bytes, uint32_t nstripes,
		void *stripes, int64_t stripe_stride,
		const uint32_t *err_list, int nerrs, void *stream);

/* Aggregation delta parity update (xor_gen + ec_encode_data_update fused,
 * ref:src/object/srv_ec_aggregate.c:1062-1105), batched over stripes:
 *   parity[r] ^= XOR_u coef[r][cell_idx[u]] * (old[u] ^ new[u])
 * for the nupd updated data cells of each stripe.  Cell u of stripe s:
 *   old_cells + s*old_stripe_stride + u*cell_bytes (same for new_cells);
 * parity cell r of stripe s: parity + r*parity_cell_stride + s*parity_stripe_stride. */
int ecg_update(ecg_ctx_t *ctx, int k, int p, uint64_t cell_bytes, uint32_t nstripes,
	       int nupd, const uint32_t *cell_idx,
	       const void *old_cells, const void *new_cells, int64_t upd_stripe_stride,
	       void *parity, int64_t parity_cell_stride, int64_t parity_stripe_stride,
	       void *stream);

/* ---- host-resident pipeline (PCIe-inclusive) ---------------------------- */
/* One stripe, ISA-L ec_encode_data calling convention: pointers src[k],
 * dst[rows] (any alignment), `len` bytes each;
 * dst[r] (^)= XOR_j coef[r*k+j] * src[j], on ctx's GPU.  Host cells go
 * through per-thread pinned staging; device cells (src[0] hipMalloc'd: then
 * every cell must lie inside a device allocation, else -ECG_DER_INVAL) run
 * in place on one of the context's ECG_DROPIN_STREAMS (4) drop-in streams,
 * and the call waits only for its own launch.  Synchronous.  k may exceed
 * ECG_MAX_K (xor_gen: accumulating launches). */
int ecg_matmul_host(ecg_ctx_t *ctx, int len, int k, int rows, const unsigned char *coef,
		    unsigned char *const *src, unsigned char *const *dst, unsigned flags);
/* ---- CPU product and drop-in routing (host memory) ----------------------
 * The same product on the calling CPU thread (host pointers only; no device
 * needed): vgf2p8affineqb with AVX-512 or AVX2 GFNI, vpshufb nibble tables
 * with AVX2, byte tables otherwise (widest the CPU has; ecg_cpu_set_isa /
 * $ECG_CPU_ISA choose a narrower one: "avx512-gfni", "avx2-gfni", "avx2",
 * "scalar", "auto").  k <= ECG_MAX_K + 256, rows <= 256.  Synchronous. */
int ecg_cpu_matmul(int len, int k, int rows, const unsigned char *coef,
		   unsigned char *const *src, unsigned char *const *dst, unsigned flags);
const char *ecg_cpu_isa(void);
int ecg_cpu_set_isa(const char *isa);
/* Where the drop-in surfaces (ecg_isal.h data-plane calls, and the
 * synchronous one-stripe calls of ecg_daos.h) run a call: device cells on
 * the GPU; host cells on the CPU when len * (k + rows) is below this
 * crossover (bytes), when the process has no usable gfx950 device, or with
 * $ECG_FORCE_CPU=1; otherwise on the GPU through pinned staging.  Default:
 * the measured crossover, $ECG_DROPIN_CROSSOVER overrides;
 * 0 = host cells always on the GPU, UINT64_MAX = never. */
int ecg_set_dropin_crossover(uint64_t bytes);
uint64_t ecg_dropin_crossover(void);

/* Encode host-resident stripes (data [S][k][C], parity [p][S][C] in host
 * memory; pinned memory from ecg_host_alloc is fastest) by streaming chunks
 * of `chunk_stripes` through device staging on 3 rotating streams
 * (H2D / kernel / D2H overlap); 0 = about 32 MiB of input cells per chunk.
 * Synchronous. */
int ecg_encode_host(ecg_ctx_t *ctx, int k, int p, uint64_t cell_bytes, uint32_t nstripes,
		    const void *data, void *parity, uint32_t chunk_stripes);
/* Same for recovery over host [S][k+p][C] stripes: only survivors travel
 * H2D, only regenerated cells travel D2H.  Synchronous. */
int ecg_recover_host(ecg_ctx_t *ctx, int k, int p, uint64_t cell_bytes, uint32_t nstripes,
		     void *stripes, const uint32_t *err_list, int nerrs,
		     uint32_t chunk_stripes);

/* ---- batching facade for one-stripe callers ------------------------------
 * Every reference caller issues ONE stripe per codec call (client write
 * ref:src/object/cli_ec.c:627-659, rebuild ref:src/object/srv_obj_migrate.c:
 * 1116-1177, aggregation ULTs on the offload xstream ref:src/object/
 * srv_ec_aggregate.c:701-734).  An ecg_queue accepts such requests from any
 * number of threads, coalesces compatible ones (same op, k, p, cell size and
 * erasure set) into one device batch, and completes each request through its
 * callback -- the place DAOS sets its ABT_eventual (srv_ec_aggregate.c:696).
 * Host buffers must stay valid until the callback runs.  Callbacks run on the
 * queue's completion threads and must not block on the queue.
 * Cells may be host memory or device memory of one of the queue's devices.
 * Host cells go where the ISA-L drop-in would send them: below its crossover
 * (ecg_set_dropin_crossover; with a GFNI CPU, every size) the queue's
 * completion threads compute them in place on the CPU path -- such a batch
 * closes while a completion thread is free if it is the queue's only work or
 * holds a request per free thread, so a lone request does not wait
 * max_wait_us -- else they are staged through the queue's pinned slots (PCIe
 * both ways).  Device cells (k <= 16): such requests batch into one
 * pointer-table launch on the cells in place (updates: one ecg_update_ptrs
 * call), and a batch launches as soon as the device has fewer than 2 of the
 * queue's batches in flight -- a lone request does not wait either.  A request's cells are all host memory or all
 * memory of one device (-ECG_DER_INVAL naming the odd cell otherwise). */
typedef struct ecg_queue ecg_queue_t;
typedef void (*ecg_done_cb_t)(void *arg, int rc);

typedef struct ecg_queue_attr {
	uint32_t max_batch;	/* stripes per device batch (default 256) */
	uint32_t max_wait_us;	/* longest a request waits for company (default 50) */
	uint64_t max_cell_bytes; /* staging sized for this cell size (default 1 MiB) */
} ecg_queue_attr_t;

/* attr may be NULL for defaults.  ctx NULL (or $ECG_FORCE_CPU=1): the CPU
 * executor -- the same requests, batching and callbacks with no device, the
 * products computed on the queue's completion threads by the CPU path
 * straight from the callers' cells, nothing staged (host cells only; a
 * GPU-less process can use the facade). */
int ecg_queue_create(ecg_ctx_t *ctx, const ecg_queue_attr_t *attr, ecg_queue_t **q);
/* Drains outstanding requests (their callbacks run) then frees the queue. */
void ecg_queue_destroy(ecg_queue_t *q);
/* Encode one stripe: data[k] -> parity[p] (cell_bytes each; host, or device
 * memory of one of the queue's devices). */
int ecg_queue_encode(ecg_queue_t *q, int k, int p, uint64_t cell_bytes,
		     unsigned char *const *data, unsigned char *const *parity,
		     ecg_done_cb_t cb, void *arg);
/* Recover one stripe in place: `stripe` is [k+p][cell_bytes] in logical cell
 * order (host, or device memory of one of the queue's devices); err_list
 * holds the erased logical cells. */
int ecg_queue_recover(ecg_queue_t *q, int k, int p, uint64_t cell_bytes, unsigned char *stripe,
		      const uint32_t *err_list, int nerrs, ecg_done_cb_t cb, void *arg);
/* Aggregation delta update of one stripe's parity (agg_update_parity:
 * xor_gen(old, new -> diff) then ec_encode_data_update(vec_i), ref:src/object/
 * srv_ec_aggregate.c:1086-1102):  parity[r] ^= coef[r][vec_i] * (old ^ new)
 * for the p parity cells (updated in place when the callback runs).  Requests
 * of one (k, p, cell size) batch together whatever their vec_i.  k <= 16.
 * Host cells: on the CPU path the deltas are computed and XORed into the
 * parity on the completion threads; staged, old ^ new crosses PCIe and the
 * deltas are XORed in on the host.
 * Device cells: ecg_update_ptrs batches in place -- requests naming the same
 * parity cells fold into one pass, and the update batches of one device run
 * in order, so concurrent updates of one stripe never lose a delta; a batch
 * ecg_update_ptrs refuses (an old / new cell overlapping a parity cell of
 * the batch) runs its requests one by one, each with its own result.  An
 * old / new cell that is another pending request's parity is read before or
 * after that request's delta, whichever ran first. */
int ecg_queue_update(ecg_queue_t *q, int k, int p, uint64_t cell_bytes, int vec_i,
		     const unsigned char *old_cell, const unsigned char *new_cell,
		     unsigned char *const *parity, ecg_done_cb_t cb, void *arg);
/* Block until every request submitted before the call has completed. */
int ecg_queue_flush(ecg_queue_t *q);
/* Counters: requests completed, device batches launched. */
int ecg_queue_stats(ecg_queue_t *q, uint64_t *requests, uint64_t *batches);

/* ---- memory / streams / timing plumbing --------------------------------- */
int ecg_dev_alloc(ecg_ctx_t *ctx, size_t bytes, void **ptr);
int ecg_dev_free(ecg_ctx_t *ctx, void *ptr);
int ecg_host_alloc(ecg_ctx_t *ctx, size_t bytes, void **ptr);	/* pinned */
int ecg_host_free(ecg_ctx_t *ctx, void *ptr);
/* kind: 0 H2D, 1 D2H, 2 D2D, 3 default (runtime infers). Async on stream. */
int ecg_memcpy(ecg_ctx_t *ctx, void *dst, const void *src, size_t bytes, int kind, void *stream);
int ecg_memset(ecg_ctx_t *ctx, void *dst, int value, size_t bytes, void *stream);
int ecg_stream_create(ecg_ctx_t *ctx, void **stream);
int ecg_stream_destroy(ecg_ctx_t *ctx, void *stream);
int ecg_stream_sync(ecg_ctx_t *ctx, void *stream);
int ecg_event_create(ecg_ctx_t *ctx, void **event);
int ecg_event_destroy(ecg_ctx_t *ctx, void *event);
int ecg_event_record(ecg_ctx_t *ctx, void *event, void *stream);
int ecg_event_elapsed_ms(ecg_ctx_t *ctx, void *start, void *stop, float *ms);
int ecg_device_sync(ecg_ctx_t *ctx);
/* Streaming kernels (16 B/lane) used to measure the achievable HBM rate:
 * mode 0 copy src->dst, 1 read-only (dst receives 16 B per thread of the
 * launch, <= 8 MiB), 2 write-only (fills dst).  ecg_set_launch's grid_x, when
 * set, caps the block count (default: one 4 x 16 B slice per thread). */
int ecg_dev_copy_kernel(ecg_ctx_t *ctx, void *dst, const void *src, size_t bytes, int mode,
			void *stream);

/* ---- telemetry ------------------------------------------------------------
 * The engine counts EC full-stripe and partial updates with GURT telemetry
 * (opm_update_ec_full / _partial, ref:src/object/srv_ec.c:21-87); the codec's
 * own counters, per context since creation or the last reset (relaxed
 * atomics: safe from any thread, a snapshot is not one consistent instant):
 *   encode_*   full-stripe products: stripes and user-data bytes (k*C*S)
 *   recover_*  regenerations: stripes and regenerated bytes (nerrs*C*S)
 *   update_*   partial-stripe parity updates: updated cells and their bytes
 *   csum_chunks  checksums computed (standalone and fused)
 *   launches   codec kernel launches (product, fused, checksum)
 *   h2d_bytes / d2h_bytes  cell bytes the host-resident pipelines and the
 *              batching queue moved over PCIe
 * The batching queue counts its batches on the context of the slot that ran
 * them (encode / recover / update rows above, and launches). */
typedef struct ecg_stats {
	uint64_t encode_stripes, encode_bytes;
	uint64_t recover_stripes, recover_bytes;
	uint64_t update_cells, update_bytes;
	uint64_t csum_chunks;
	uint64_t launches;
	uint64_t h2d_bytes, d2h_bytes;
} ecg_stats_t;
/* Copy the counters to *out (may be NULL) and, if reset != 0, zero them. */
int ecg_get_stats(ecg_ctx_t *ctx, ecg_stats_t *out, int reset);

/* ---- launch tuning (benchmarks; 0 = default) ----------------------------
 * variant: 0 auto, 1 runtime-shaped kernel, 2 byte kernel, 3 dword lanes
 * whatever the operands' alignment (misaligned dword accesses served by the
 * hardware's unaligned access mode; A/B only). */
int ecg_set_launch(ecg_ctx_t *ctx, uint32_t grid_x, uint32_t grid_y, uint32_t variant);
/* Block -> (stripe, 4 KiB column) mapping of the product kernel: 0 = 2D
 * grid (columns x stripes, default); 1 = 1D stripe-fastest; 2 = 1D with each
 * XCD streaming its own eighth of the column-fastest items; 3 = as 2,
 * stripe-fastest.  Tuning only; results never depend on it. */
int ecg_set_launch_order(ecg_ctx_t *ctx, uint32_t order);
/* Blocks per CU of the product kernel's 2D grid: 0 = the per-shape default
 * (currently no cap for any shape), 2..16 = that cap, 255 = no cap.  Enforced
 * with unused dynamic LDS.  Tuning only; results never depend on it. */
int ecg_set_wg_per_cu(ecg_ctx_t *ctx, uint32_t wg_per_cu);
/* Launch tuner (on by default; ECG_AUTOTUNE=0 in the environment turns it off
 * for new contexts): the first 23 product launches of each wide shape (k >= 16,
 * > 2048 blocks) in a context run 4 uncapped then 19 at the candidate cap (2
 * blocks per CU), the last 3 of each arm timed with events on the
 * stream of the launch that started the probe (a switch to a cap runs slow for
 * its first ~10-20 launches); once every timing has completed the faster time
 * per block is kept for the shape (the cap only when it wins by > 1.5 %).  A
 * shape is (k, rows, acc/diff, cell bytes, lane granule, layout class:
 * source and destination sharing one stripe stride or not, or a pointer
 * table from ecg_matmul_ptrs / ecg_obj_ec_recx_encode) -- NOT the batch
 * size, so batches of varying size share one probe and one decision.  Skipped
 * when ecg_set_wg_per_cu or ecg_set_launch / _order set a geometry, and on
 * streams under graph capture.  on: 0 off, 1 on, 2 on and forget every
 * decision (and the counters).  Tuning only; results never depend on it. */
int ecg_set_autotune(ecg_ctx_t *ctx, int on);
/* The tuner's state of a shape (k inputs, rows outputs, acc/diff off, the
 * launch's source and destination stripe strides -- encode: k*C and the
 * parity stripe stride; in-place recovery: (k+p)*C both): 1 decided (*cap =
 * the cap, or 255 = none; both arms' median times per block, scaled to a
 * launch of nstripes stripes), 0 still probing or not seen.  nstripes is not part of the shape (it only has to
 * make the launch tunable, > 2048 blocks, to have been probed). */
int ecg_tune_state(ecg_ctx_t *ctx, int k, int rows, uint64_t cell_bytes, uint32_t nstripes, int64_t sstride,
		   int64_t dstride, uint32_t *cap, float *ms_uncapped, float *ms_capped);
/* The tuner's counters since the context was created (or ecg_set_autotune(ctx,
 * 2)): probe cycles started, launches that ran inside a probe, shapes held. */
int ecg_tune_counters(ecg_ctx_t *ctx, uint64_t *probe_cycles, uint64_t *probe_launches, uint32_t *shapes);

/* Pointer-table product: ISA-L's per-stripe pointer arrays
 * (ec_encode_data(len, k, rows, tbls, data[], coding[])) batched over
 * nstripes.  cells[s*(k+rows) + j] is the DEVICE address of input cell j
 * (j < k) or output cell j-k of stripe s; the table itself is a host array
 * (copied before return is not required: it is staged internally).  k <= 16,
 * rows <= 8; any alignment.  A table whose cells sit at fixed offsets from a
 * per-stripe base (cell j of stripe s at cells[j] + s*stride, one stride for
 * the inputs, one for the outputs -- a contiguous client buffer) runs as the
 * strided product (ecg_matmul) with no table upload.  Asynchronous on
 * `stream`. */
int ecg_matmul_ptrs(ecg_ctx_t *ctx, int k, int rows, const unsigned char *coef,
		    uint64_t cell_bytes, uint32_t nstripes, void *const *cells, void *stream);

/* Per-request delta parity updates on DEVICE cells: agg_update_parity's
 * xor_gen(old, new) + ec_encode_data_update(vec_i) of one updated data cell
 * (ref:src/object/srv_ec_aggregate.c:1086-1102), nreq requests in one call:
 *   parity_r ^= coef[r][vec_i[i]] * (old ^ new)        r < p
 * with the codec's Cauchy parity rows.  cells[i*(2+p) + 0] = old cell,
 * + 1 = new cell, + 2 + r = parity cell r of request i (device addresses,
 * cell_bytes each, any alignment).  Requests may name the same parity cells
 * (several cells of one stripe) or overlapping ones: the result is every
 * request applied, as if one after another.  Requests naming the same parity
 * cells are folded into one pass over that parity; the rest run in as few
 * ordered launches as keep every parity byte's read-modify-writes apart.  An
 * old/new cell must not overlap a parity cell of the call; one request's
 * parity cells must not overlap one another (-DER_INVAL).  k <= 16, p <= 8.
 * The table is a host array, staged internally.  Asynchronous on `stream`. */
int ecg_update_ptrs(ecg_ctx_t *ctx, int k, int p, uint64_t cell_bytes, uint32_t nreq,
		    void *const *cells, const uint8_t *vec_i, void *stream);

#ifdef __cplusplus
}
#endif
#endif
