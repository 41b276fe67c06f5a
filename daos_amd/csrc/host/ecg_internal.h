/*
 * ecg_internal.h -- private declarations of the C host layer.
 */
#ifndef ECG_INTERNAL_H
#define ECG_INTERNAL_H

#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <stdint.h>

#include "../../../include/ecg.h"
#include "../ecg_kabi.h"

#define ECG_RCACHE 16	/* recovery-matrix cache entries per context */

struct ecg_rcache_ent {
	int valid;
	int k, p, nerrs;
	uint32_t err_list[ECG_MAX_P];
	unsigned char rows[ECG_MAX_P * ECG_MAX_K];	/* data-first order */
	uint32_t out_idx[ECG_MAX_P];			/* cell each row writes */
	uint32_t dec_idx[ECG_MAX_K];
	uint64_t stamp;
};

/* Host-staging buffers for the PCIe pipeline (per context, 3 slots). */
#define ECG_NSLOT 3
struct ecg_stage {
	size_t dev_bytes;
	void *dev[ECG_NSLOT];
	hipStream_t st[ECG_NSLOT];
	hipEvent_t done[ECG_NSLOT];
};

/* Pointer tables and gathered cells (ecg_ptrs.c): two slots used in turn,
 * each guarded by ctx->lock and the `done` event of the last launch that read
 * it, so a call only waits for the launch before last. */
#ifndef ECG_NSCRATCH
#define ECG_NSCRATCH 2
#endif
struct ecg_scratch_slot {
	void *pin;
	size_t pin_bytes;
	void *dev;
	size_t dev_bytes;
	hipEvent_t done;
	int pending;
};

struct ecg_scratch {
	struct ecg_scratch_slot slot[ECG_NSCRATCH];
	unsigned next;
};

struct ecg_ctx {
	int device;
	hipStream_t stream;
	ecg_launch_cfg_t cfg;
	pthread_mutex_t lock;
	struct ecg_rcache_ent rcache[ECG_RCACHE];
	uint64_t rstamp;
	struct ecg_stage stage;
#define ECG_NCSUM_TBL 4
	void *csum_tbl[ECG_NCSUM_TBL];	/* device CRC tables by hash type (ecg_csum.c) */
	uint32_t csum_blocks;		/* csum grid cap, 0 = kernel default */
	uint32_t fused_cols;		/* fused kernel columns per item, 0 = default */
#define ECG_NSPLIT_CACHE 8
	struct ecg_split_ent {		/* workgroup-per-chunk CRC shifts (ecg_csum.c) */
		int valid, type;
		uint64_t m;
		uint64_t sh[ECG_CSUM_SPLIT_NW];
	} split_cache[ECG_NSPLIT_CACHE];
	unsigned split_next;
#define ECG_NKH_CACHE 8
	struct ecg_kh_ent {		/* fused-kernel item multipliers (ecg_csum.c) */
		int valid, type;
		uint64_t rcs, last;
		uint32_t ncols;
		void *dev;
	} kh_cache[ECG_NKH_CACHE];
	unsigned kh_next;
	struct ecg_scratch scratch;
#define ECG_DROPIN_STREAMS 4
	hipStream_t dpool[ECG_DROPIN_STREAMS];	/* device-cell drop-in calls (ecg_stage.c) */
	int ndpool;
	struct ecg_tuner *tuner;	/* blocks-per-CU cap per shape (ecg_tune.c) */
	ecg_stats_t stats;		/* telemetry (ecg_get_stats), updated with atomics */
};

/* telemetry: add n to one ecg_stats_t field of ctx (any thread) */
#define ECG_STAT_ADD(ctx, field, n) __atomic_fetch_add(&(ctx)->stats.field, (uint64_t)(n), __ATOMIC_RELAXED)

/* errors (thread-local detail string) */
int ecg_fail(int rc, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int ecg_hip_fail(hipError_t e, const char *what);
/* Pinned-host <-> device staging copy of a contiguous range issued as a 2D
 * copy of rows of a multiple of `row` bytes up to 1 MiB (the remainder, if
 * any, as a 1D copy).  Measured under concurrent traffic
 * in the other direction, the 2D path sustains ~97 % of the raw pinned H2D
 * rate where one 1D copy reaches ~84 % (tools/bench_pcie.py,
 * profiles/r01/pcie.json). */
hipError_t ecg_stage_copy(void *dst, const void *src, size_t bytes, size_t row, hipMemcpyKind kind,
			  hipStream_t st);
void ecg_set_last_kernel(const char *name);

/* GF(2^8) tables (ecg_gf.c) */
void ecg_gf_init(void);
extern unsigned char ecg_gf_mul_tbl[256][256];
void ecg_build_ptbl(unsigned char c, ecg_ptbl_t *t);
/* data-first decode rows: out_idx[i] = logical cell written by rows[i] */
int ecg_recov_rows(int k, int p, const unsigned char *en_matrix,
		   const uint32_t *err_list, int nerrs, unsigned char *rows,
		   uint32_t *out_idx, uint32_t *dec_idx, int *reused_encode);

/* pointer tables (ecg_ptrs.c) */
void ecg_scratch_free(ecg_ctx_t *ctx);
/* ecg_update_ptrs with explicit parity rows coef[rows][k]; *nlaunch (may be
 * NULL) = the ordered launches the batch took */
int ecg_update_ptrs_coef(ecg_ctx_t *ctx, int k, int rows, const unsigned char *coef, uint64_t C, uint32_t nreq,
			 void *const *cells, const uint8_t *vec_i, void *stream, uint32_t *nlaunch);
/* next scratch slot with at least these sizes, free of readers (ctx->lock held) */
int ecg_scratch_reserve(ecg_ctx_t *ctx, size_t pin_bytes, size_t dev_bytes,
			struct ecg_scratch_slot **out);
/* The first `bytes` of sc->pin to sc->dev, queued on st (a fetch kernel:
 * ecg_k_launch_fetch); `what` names the table in the error. */
int ecg_table_upload(struct ecg_scratch_slot *sc, size_t bytes, hipStream_t st, const char *what);

/* batched segment copies (ecg_sgl.c).  A fixed list (cap preset, fixed = 1)
 * writes into caller memory and fails instead of growing. */
struct ecg_segs {
	ecg_copy_seg_t *seg;
	size_t n, cap;
	uint64_t tiles;
	int fixed;
};
int ecg_segs_add(struct ecg_segs *v, uint64_t dst, uint64_t src, uint64_t len);
void ecg_segs_fini(struct ecg_segs *v);
/* launch over a device copy of v->seg already queued on st */
int ecg_segs_launch(const struct ecg_segs *v, const void *segs_dev, hipStream_t st);

/* checksums (ecg_csum.c) */
void ecg_csum_ctx_fini(ecg_ctx_t *ctx);
int ecg_csum_fused_params(ecg_ctx_t *ctx, int type, uint64_t chunksize, uint64_t rec_size,
			  uint64_t C, int k, int rows, void *csums, ecg_mmcs_params_t *q);

/* product + chunk checksums of every output cell, cells as extents from
 * record index 0; csums[row_slot[r]][s][chunk] (ecg_core.c) */
int ecg_matmul_csum(ecg_ctx_t *ctx, int k, int rows, const unsigned char *coef, uint64_t C,
		    uint32_t S, const void *src, const int64_t *soff, int64_t sstride, void *dst,
		    const int64_t *doff, int64_t dstride, int type, uint64_t chunksize,
		    uint64_t rec_size, void *csums, const uint32_t *row_slot, void *stream);

/* one-cell product, per-stripe coefficient column sel_dev[s] < ncols
 * (coef rows x ncols), 16-byte aligned operands (ecg_core.c) */
int ecg_matmul_sel(ecg_ctx_t *ctx, int ncols, int rows, const unsigned char *coef, uint64_t C, uint32_t S,
		   const void *src, int64_t sstride, const uint8_t *sel_dev, void *dst, const int64_t *doff,
		   int64_t dstride, void *stream);
/* host pipeline with an explicit parity row pitch (ecg_core.c) */
int ecg_encode_host_rows(ecg_ctx_t *ctx, int k, int p, uint64_t C, uint32_t S, const void *data,
			 void *parity, size_t prow, uint32_t chunk);
/* "0,1,2" / "all" / NULL -> device list (ecg_multi.c); count or -ECG_DER_INVAL */
int ecg_parse_devices(const char *spec, int *dev, int max);

/* roctx ranges (ecg_trace.c): no-ops without the roctx library or with
 * ECG_ROCTX=0 */
void ecg_trace_push(const char *name);
void ecg_trace_pop(void);
int ecg_trace_active(void);

/* launch tuner (ecg_tune.c): product launches of wide shapes measure the
 * blocks-per-CU cap against none and keep the faster */
#define ECG_NTUNE 16
struct ecg_tuner;
int ecg_tune_init(ecg_ctx_t *ctx);
void ecg_tune_fini(ecg_ctx_t *ctx);
int ecg_tune_launch(ecg_ctx_t *ctx, const ecg_mm_params_t *p, hipStream_t st, uint32_t *kid);
/* The device whose memory p is; < 0 for host memory: ECG_PTR_HOST (known to
 * the HIP runtime: pinned, registered, managed) or ECG_PTR_UNKNOWN (plain
 * malloc / mmap) (ecg_stage.c). */
#define ECG_PTR_HOST (-1)
#define ECG_PTR_UNKNOWN (-2)
int ecg_ptr_device(const void *p);
/* ecg_ptr_device through the calling thread's short-lived cache of 2 MiB
 * regions of plain host memory (ecg_dropin.c): near-free for a caller's
 * reused malloc'd buffers */
int ecg_ptr_device_cached(const void *p);
/* The same for any launcher of the product (the pointer-table kernel): `g`
 * its lane granule, `layout` its layout class (ECG_TUNE_LAYOUT_*), `fn(p,
 * cfg, stream, kid, arg)` the launch under a given geometry. */
typedef int (*ecg_mm_launch_fn)(const ecg_mm_params_t *p, const ecg_launch_cfg_t *cfg, void *stream,
				uint32_t *kid, const void *arg);
#define ECG_TUNE_LAYOUT_SEPARATE 0u	/* source and destination stripe strides differ */
#define ECG_TUNE_LAYOUT_INTERLEAVED 1u	/* one stripe stride: in-place recovery */
#define ECG_TUNE_LAYOUT_PTRS 2u		/* per-stripe pointer table */
int ecg_tune_launch_fn(ecg_ctx_t *ctx, const ecg_mm_params_t *p, uint32_t g, uint32_t layout,
		       ecg_mm_launch_fn fn, const void *arg, hipStream_t st, uint32_t *kid);

/* synchronous one-stripe product on ctx's GPU; place = ecg_cells_place's
 * placement of the k + rows cells (NULL: all host memory) (ecg_stage.c) */
int ecg_matmul_host_mem(ecg_ctx_t *ctx, int len, int k, int rows, const unsigned char *coef,
			unsigned char *const *src, unsigned char *const *dst, unsigned flags, const signed char *place);
/* Forget every thread's remembered device ranges (ecg_cells_place): called
 * when the library frees device memory. */
void ecg_place_forget(void);
/* placement of every cell of a one-stripe call: place[i] = device or -1
 * (host); returns the device cells' count (*dev their device) or a negative
 * DER code (cells on two devices, a device cell past its allocation) */
int ecg_cells_place(unsigned char *const *src, int k, unsigned char *const *dst, int rows, uint64_t len,
		    int (*query)(const void *), signed char *place, int *dev);
/* every cell [v[i], v[i] + len) inside one allocation of ctx's device, else
 * -DER_INVAL naming `what` (ecg_stage.c) */
int ecg_cells_on_device(ecg_ctx_t *ctx, unsigned char *const *v, int n, uint64_t len, const char *what);
/* drop-in routing (ecg_dropin.c): device cells -> GPU, host cells -> CPU
 * below the crossover or without a usable device, else GPU.  ctx NULL = the
 * calling thread's default context. */
int ecg_dropin_product(const char *fn, ecg_ctx_t *ctx, int len, int k, int rows, const unsigned char *coef,
		       unsigned char *const *src, unsigned char *const *dst, unsigned flags);
/* 1 when the drop-in may use a GPU in this process */
int ecg_dropin_gpu(void);
/* Host cells of `bytes` (len x (k + rows)) compute on the CPU path: below the
 * drop-in crossover, or $ECG_FORCE_CPU=1 (ecg_dropin.c). */
int ecg_dropin_host_on_cpu(uint64_t bytes);
/* the calling thread's default context; NULL without a usable device */
ecg_ctx_t *ecg_dropin_ctx(void);

/* context helpers (ecg_core.c) */
int ecg_ctx_enter(ecg_ctx_t *ctx);
#ifdef ECG_QUEUE_TIMING
void ecg_ptrs_timing_print(void);	/* diagnostic build: update_ptrs call phases */
#endif

/* NUMA placement (ecg_numa.c); the cpu_set_t helpers need _GNU_SOURCE in the
 * including file */
int ecg_numa_enabled(void);
#ifdef _GNU_SOURCE
#include <sched.h>
int ecg_numa_node_cpus(int node, cpu_set_t *set);
int ecg_numa_bind_thread(int device, cpu_set_t *saved);
void ecg_numa_restore_thread(const cpu_set_t *saved);
#endif
hipStream_t ecg_pick_stream(ecg_ctx_t *ctx, void *stream);

#endif
