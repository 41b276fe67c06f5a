/*
 * ecg_core.c -- context, batched codec entry points and the host-staging
 * (PCIe) pipeline of the MI355X EC engine.  See include/ecg.h.
 *
 * Reference loops these entry points replace (one ISA-L call per stripe on
 * the CPU today):
 *   client encode     obj_ec_recx_encode   ref:src/object/cli_ec.c:593-663
 *   degraded read     obj_ec_recov_data    ref:src/object/cli_ec.c:2814-2885
 *   rebuild parity    migrate_update_parity ref:src/object/srv_obj_migrate.c:1096-1181
 *   aggregation       agg_encode_full_stripe_ult / agg_update_parity
 *                     ref:src/object/srv_ec_aggregate.c:671-697, 1062-1105
 */
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ecg_internal.h"
#include "../../../include/ecg_csum.h"

static __thread char t_err[512];
static __thread const char *t_last_kernel = "";

int ecg_fail(int rc, const char *fmt, ...)
{
	va_list ap;

	va_start(ap, fmt);
	vsnprintf(t_err, sizeof(t_err), fmt, ap);
	va_end(ap);
	return rc;
}

int ecg_hip_fail(hipError_t e, const char *what)
{
	return ecg_fail(-ECG_DER_IO, "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
}

const char *ecg_strerror(void)
{
	return t_err;
}

void ecg_set_last_kernel(const char *name)
{
	t_last_kernel = name;
}

const char *ecg_last_kernel(void)
{
	return t_last_kernel;
}

#define HIPCHK(call)                                                   \
	do {                                                           \
		hipError_t e__ = (call);                               \
		if (e__ != hipSuccess)                                 \
			return ecg_hip_fail(e__, #call);               \
	} while (0)

/* ------------------------------------------------------------------------ */
/* devices / contexts                                                        */
/* ------------------------------------------------------------------------ */
static int is_gfx950(int dev)
{
	hipDeviceProp_t prop;

	if (hipGetDeviceProperties(&prop, dev) != hipSuccess)
		return 0;
	return strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

int ecg_device_count(void)
{
	int n = 0, i, good = 0;

	if (hipGetDeviceCount(&n) != hipSuccess)
		return 0;
	for (i = 0; i < n; i++)
		good += is_gfx950(i);
	return good;
}

int ecg_ctx_create(int device, ecg_ctx_t **out)
{
	ecg_ctx_t *ctx;
	hipError_t e;
	int n = 0;

	if (out == NULL)
		return ecg_fail(-ECG_DER_INVAL, "ctx_create: NULL out");
	*out = NULL;
	e = hipGetDeviceCount(&n);
	if (e != hipSuccess || n == 0)
		return ecg_fail(-ECG_DER_NOSYS, "ctx_create: no HIP device (%s)",
				hipGetErrorString(e));
	if (device < 0 || device >= n)
		return ecg_fail(-ECG_DER_INVAL, "ctx_create: device %d of %d", device, n);
	if (!is_gfx950(device))
		return ecg_fail(-ECG_DER_NOSYS, "ctx_create: device %d is not gfx950", device);
	ctx = calloc(1, sizeof(*ctx));
	if (ctx == NULL)
		return ecg_fail(-ECG_DER_NOMEM, "ctx_create: calloc");
	ctx->device = device;
	pthread_mutex_init(&ctx->lock, NULL);
	ecg_gf_init();
	e = hipSetDevice(device);
	if (e == hipSuccess)
		e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
	if (e != hipSuccess) {
		free(ctx);
		return ecg_hip_fail(e, "ctx_create");
	}
	if (ecg_tune_init(ctx)) {
		(void)hipStreamDestroy(ctx->stream);
		free(ctx);
		return -ECG_DER_NOMEM;
	}
	{
		/* misaligned dword accesses served? (destinations off a dword, partial
		 * columns of unaligned sources); ECG_UNALIGNED=0 forces the byte
		 * kernels for those operands, as a device without them would get */
		const char *env = getenv("ECG_UNALIGNED");
		int ok = 0, rc;

		if (env && env[0] == '0') {
			ok = 0;
		} else if ((rc = ecg_k_unaligned_check((void *)ctx->stream, &ok)) != 0) {
			/* the probe itself failed: byte kernels for misaligned
			 * operands (same bytes, ~8x slower) -- say so */
			(void)hipGetLastError();
			fprintf(stderr, "ecg: device %d: misaligned-access probe failed (%s); misaligned "
				"operands run the byte kernels\n", device, hipGetErrorString((hipError_t)rc));
			ok = 0;
		}
		ctx->cfg.no_unaligned = ok ? 0u : 1u;
	}
	*out = ctx;
	return 0;
}

int ecg_ctx_unaligned_ok(ecg_ctx_t *ctx)
{
	if (ctx == NULL)
		return ecg_fail(-ECG_DER_INVAL, "NULL context");
	return ctx->cfg.no_unaligned ? 0 : 1;
}

static void stage_free(ecg_ctx_t *ctx)
{
	int i;

	for (i = 0; i < ECG_NSLOT; i++) {
		if (ctx->stage.dev[i])
			(void)hipFree(ctx->stage.dev[i]);
		if (ctx->stage.st[i])
			(void)hipStreamDestroy(ctx->stage.st[i]);
		if (ctx->stage.done[i])
			(void)hipEventDestroy(ctx->stage.done[i]);
	}
	memset(&ctx->stage, 0, sizeof(ctx->stage));
}

void ecg_ctx_destroy(ecg_ctx_t *ctx)
{
	if (ctx == NULL)
		return;
	(void)hipSetDevice(ctx->device);
	(void)hipStreamSynchronize(ctx->stream);
	stage_free(ctx);
	ecg_scratch_free(ctx);
	ecg_csum_ctx_fini(ctx);
	ecg_tune_fini(ctx);
	for (int i = 0; i < ctx->ndpool; i++) {
		(void)hipStreamSynchronize(ctx->dpool[i]);
		(void)hipStreamDestroy(ctx->dpool[i]);
	}
	(void)hipStreamDestroy(ctx->stream);
	pthread_mutex_destroy(&ctx->lock);
	free(ctx);
}

int ecg_ctx_device(const ecg_ctx_t *ctx)
{
	return ctx ? ctx->device : -1;
}

int ecg_device_pci_bus_id(int device, char *buf, int len)
{
	hipError_t e;

	if (buf == NULL || len < 13)
		return ecg_fail(-ECG_DER_INVAL, "pci_bus_id: buffer too small");
	e = hipDeviceGetPCIBusId(buf, len, device);
	if (e != hipSuccess)
		return ecg_hip_fail(e, "hipDeviceGetPCIBusId");
	return 0;
}

void *ecg_ctx_stream(ecg_ctx_t *ctx)
{
	return ctx ? (void *)ctx->stream : NULL;
}

int ecg_ctx_enter(ecg_ctx_t *ctx)
{
	hipError_t e;

	if (ctx == NULL)
		return ecg_fail(-ECG_DER_INVAL, "NULL context");
	e = hipSetDevice(ctx->device);
	if (e != hipSuccess)
		return ecg_hip_fail(e, "hipSetDevice");
	return 0;
}

hipStream_t ecg_pick_stream(ecg_ctx_t *ctx, void *stream)
{
	return stream ? (hipStream_t)stream : ctx->stream;
}

int ecg_set_launch(ecg_ctx_t *ctx, uint32_t grid_x, uint32_t grid_y, uint32_t variant)
{
	if (ctx == NULL)
		return ecg_fail(-ECG_DER_INVAL, "NULL context");
	ctx->cfg.grid_x = grid_x;
	ctx->cfg.grid_y = grid_y;
	ctx->cfg.variant = variant;
	return 0;
}

int ecg_set_launch_order(ecg_ctx_t *ctx, uint32_t order)
{
	if (ctx == NULL || order > 3)
		return ecg_fail(-ECG_DER_INVAL, "set_launch_order: bad argument");
	ctx->cfg.order = order;
	return 0;
}

int ecg_get_stats(ecg_ctx_t *ctx, ecg_stats_t *out, int reset)
{
	uint64_t *f, *o;
	size_t i, n = sizeof(ecg_stats_t) / sizeof(uint64_t);

	if (ctx == NULL)
		return ecg_fail(-ECG_DER_INVAL, "get_stats: NULL context");
	f = (uint64_t *)&ctx->stats;
	o = (uint64_t *)out;
	for (i = 0; i < n; i++) {
		const uint64_t v = reset ? __atomic_exchange_n(&f[i], 0, __ATOMIC_RELAXED)
					 : __atomic_load_n(&f[i], __ATOMIC_RELAXED);

		if (o)
			o[i] = v;
	}
	return 0;
}

int ecg_set_wg_per_cu(ecg_ctx_t *ctx, uint32_t wg_per_cu)
{
	if (ctx == NULL || (wg_per_cu > 16 && wg_per_cu != ECG_WG_UNCAPPED))
		return ecg_fail(-ECG_DER_INVAL, "set_wg_per_cu: bad argument");
	ctx->cfg.wg_per_cu = wg_per_cu;
	return 0;
}

/* ------------------------------------------------------------------------ */
/* batched GF matrix x cells                                                 */
/* ------------------------------------------------------------------------ */
static int launch(ecg_ctx_t *ctx, const ecg_mm_params_t *prm, hipStream_t st)
{
	uint32_t kid = 0;
	int e;

	ecg_trace_push("ecg:launch");
	e = ecg_tune_launch(ctx, prm, st, &kid);
	ecg_trace_pop();
	if (e != 0)
		return ecg_hip_fail((hipError_t)e, "kernel launch");
	ECG_STAT_ADD(ctx, launches, 1);
	ecg_set_last_kernel(ecg_k_kernel_name(kid));
	return 0;
}

/*
 * Core product with optional second source (diff mode).  Splits k into
 * groups of ECG_KMAX_K (later groups accumulate) and rows into groups of
 * ECG_KMAX_R.
 */
static int matmul2(ecg_ctx_t *ctx, int k, int rows, const unsigned char *coef,
		   uint64_t C, uint32_t S,
		   const void *src, const int64_t *soff, int64_t sstride,
		   const void *src2, const int64_t *soff2, int64_t sstride2,
		   void *dst, const int64_t *doff, int64_t dstride,
		   unsigned flags, void *stream)
{
	ecg_mm_params_t *prm;
	hipStream_t st;
	int r0, j0, rc;

	if (k < 1 || k > ECG_MAX_K || rows < 1 || rows > 256)
		return ecg_fail(-ECG_DER_INVAL, "matmul: bad k=%d rows=%d", k, rows);
	if (coef == NULL || soff == NULL || doff == NULL || src == NULL || dst == NULL)
		return ecg_fail(-ECG_DER_INVAL, "matmul: NULL argument");
	if (C == 0 || S == 0)
		return 0;
	rc = ecg_ctx_enter(ctx);
	if (rc)
		return rc;
	ecg_gf_init();
	st = ecg_pick_stream(ctx, stream);
	prm = calloc(1, sizeof(*prm));
	if (prm == NULL)
		return ecg_fail(-ECG_DER_NOMEM, "matmul: calloc");

	for (r0 = 0; r0 < rows; r0 += ECG_KMAX_R) {
		int rr = rows - r0 < ECG_KMAX_R ? rows - r0 : ECG_KMAX_R;

		for (j0 = 0; j0 < k; j0 += ECG_KMAX_K) {
			int kk = k - j0 < ECG_KMAX_K ? k - j0 : ECG_KMAX_K;
			int r, j;

			memset(prm, 0, sizeof(*prm));
			prm->src = src;
			prm->src2 = src2;
			prm->dst = dst;
			prm->src_stripe_stride = sstride;
			prm->src2_stripe_stride = sstride2;
			prm->dst_stripe_stride = dstride;
			prm->cell_bytes = C;
			prm->nstripes = S;
			prm->k = (uint32_t)kk;
			prm->rows = (uint32_t)rr;
			prm->accumulate = (flags & ECG_F_ACCUMULATE) || j0 > 0;
			prm->diff = src2 != NULL;
			for (j = 0; j < kk; j++) {
				prm->src_cell_off[j] = soff[j0 + j];
				if (src2)
					prm->src2_cell_off[j] = soff2[j0 + j];
			}
			for (r = 0; r < rr; r++) {
				prm->dst_cell_off[r] = doff[r0 + r];
				for (j = 0; j < kk; j++)
					ecg_build_ptbl(coef[(size_t)(r0 + r) * k + j0 + j],
						       &prm->tbl[r][j]);
			}
			rc = launch(ctx, prm, st);
			if (rc) {
				free(prm);
				return rc;
			}
		}
	}
	free(prm);
	return 0;
}

int ecg_matmul(ecg_ctx_t *ctx, int k, int rows, const unsigned char *coef,
	       uint64_t cell_bytes, uint32_t nstripes,
	       const void *src, const int64_t *src_cell_off, int64_t src_stripe_stride,
	       void *dst, const int64_t *dst_cell_off, int64_t dst_stripe_stride,
	       unsigned flags, void *stream)
{
	return matmul2(ctx, k, rows, coef, cell_bytes, nstripes, src, src_cell_off,
		       src_stripe_stride, NULL, NULL, 0, dst, dst_cell_off, dst_stripe_stride,
		       flags, stream);
}

int ecg_matmul_sel(ecg_ctx_t *ctx, int ncols, int rows, const unsigned char *coef, uint64_t C, uint32_t S,
		   const void *src, int64_t sstride, const uint8_t *sel_dev, void *dst, const int64_t *doff,
		   int64_t dstride, void *stream)
{
	ecg_mm_params_t *prm;
	uint32_t kid = 0;
	int rc, r, j, e;

	if (ncols < 1 || ncols > ECG_KMAX_K || rows < 1 || rows > ECG_KMAX_R || coef == NULL ||
	    src == NULL || sel_dev == NULL || dst == NULL || doff == NULL)
		return ecg_fail(-ECG_DER_INVAL, "matmul_sel: bad arguments");
	if (C == 0 || S == 0)
		return 0;
	rc = ecg_ctx_enter(ctx);
	if (rc)
		return rc;
	ecg_gf_init();
	prm = calloc(1, sizeof(*prm));
	if (prm == NULL)
		return ecg_fail(-ECG_DER_NOMEM, "matmul_sel: calloc");
	prm->src = src;
	prm->dst = dst;
	prm->src_stripe_stride = sstride;
	prm->dst_stripe_stride = dstride;
	prm->cell_bytes = C;
	prm->nstripes = S;
	prm->k = 1;
	prm->rows = (uint32_t)rows;
	for (r = 0; r < rows; r++) {
		prm->dst_cell_off[r] = doff[r];
		for (j = 0; j < ncols; j++)
			ecg_build_ptbl(coef[r * ncols + j], &prm->tbl[r][j]);
	}
	e = ecg_k_launch_matmul_sel(prm, sel_dev, (uint32_t)ncols, (void *)ecg_pick_stream(ctx, stream), &kid);
	free(prm);
	if (e)
		return ecg_hip_fail((hipError_t)e, "matmul_sel launch");
	ECG_STAT_ADD(ctx, launches, 1);
	ecg_set_last_kernel(ecg_k_kernel_name(kid));
	return 0;
}

static int check_kp(int k, int p)
{
	/* DAOS class limits, ref:src/object/obj_class.c:587-601 */
	if (k < 1 || k > ECG_MAX_K || p < 1 || p > ECG_MAX_P)
		return ecg_fail(-ECG_DER_INVAL, "bad k=%d p=%d", k, p);
	return 0;
}

int ecg_encode(ecg_ctx_t *ctx, int k, int p, uint64_t C, uint32_t S,
	       const void *data, int64_t data_stripe_stride,
	       void *parity, int64_t parity_cell_stride, int64_t parity_stripe_stride,
	       void *stream)
{
	unsigned char en[(ECG_MAX_K + ECG_MAX_P) * ECG_MAX_K];
	int64_t soff[ECG_MAX_K], doff[ECG_MAX_P];
	int i, rc;

	rc = check_kp(k, p);
	if (rc)
		return rc;
	ecg_gen_cauchy1(k, p, en);
	for (i = 0; i < k; i++)
		soff[i] = (int64_t)i * (int64_t)C;
	for (i = 0; i < p; i++)
		doff[i] = (int64_t)i * parity_cell_stride;
	ecg_trace_push("ecg:encode");
	rc = ecg_matmul(ctx, k, p, &en[k * k], C, S, data, soff, data_stripe_stride,
			parity, doff, parity_stripe_stride, 0, stream);
	ecg_trace_pop();
	if (rc == 0) {
		ECG_STAT_ADD(ctx, encode_stripes, S);
		ECG_STAT_ADD(ctx, encode_bytes, (uint64_t)k * C * S);
	}
	return rc;
}

/* Recovery rows through the per-context cache (the reference caches its
 * recovery codec while the error list is unchanged, ref:src/object/cli_ec.c:
 * 2183-2185). */
static int recov_lookup(ecg_ctx_t *ctx, int k, int p, const uint32_t *err_list, int nerrs,
			struct ecg_rcache_ent *out)
{
	unsigned char en[(ECG_MAX_K + ECG_MAX_P) * ECG_MAX_K];
	struct ecg_rcache_ent *victim = NULL;
	int i, rc, reused;

	pthread_mutex_lock(&ctx->lock);
	for (i = 0; i < ECG_RCACHE; i++) {
		struct ecg_rcache_ent *e = &ctx->rcache[i];

		if (e->valid && e->k == k && e->p == p && e->nerrs == nerrs &&
		    memcmp(e->err_list, err_list, sizeof(uint32_t) * nerrs) == 0) {
			e->stamp = ++ctx->rstamp;
			*out = *e;
			pthread_mutex_unlock(&ctx->lock);
			return 0;
		}
		if (victim == NULL || !e->valid || (victim->valid && e->stamp < victim->stamp))
			victim = e;
	}
	pthread_mutex_unlock(&ctx->lock);

	memset(out, 0, sizeof(*out));
	ecg_gen_cauchy1(k, p, en);
	rc = ecg_recov_rows(k, p, en, err_list, nerrs, out->rows, out->out_idx, out->dec_idx,
			    &reused);
	if (rc)
		return rc;
	out->valid = 1;
	out->k = k;
	out->p = p;
	out->nerrs = nerrs;
	memcpy(out->err_list, err_list, sizeof(uint32_t) * nerrs);

	pthread_mutex_lock(&ctx->lock);
	out->stamp = ++ctx->rstamp;
	*victim = *out;
	pthread_mutex_unlock(&ctx->lock);
	return 0;
}

static int recover_with(ecg_ctx_t *ctx, const struct ecg_rcache_ent *ent, uint64_t C,
			uint32_t S, void *stripes, int64_t stripe_stride, void *stream)
{
	int64_t soff[ECG_MAX_K], doff[ECG_MAX_P];
	int i;

	for (i = 0; i < ent->k; i++)
		soff[i] = (int64_t)ent->dec_idx[i] * (int64_t)C;
	for (i = 0; i < ent->nerrs; i++)
		doff[i] = (int64_t)ent->out_idx[i] * (int64_t)C;
	i = ecg_matmul(ctx, ent->k, ent->nerrs, ent->rows, C, S, stripes, soff,
		       stripe_stride, stripes, doff, stripe_stride, 0, stream);
	if (i == 0) {
		ECG_STAT_ADD(ctx, recover_stripes, S);
		ECG_STAT_ADD(ctx, recover_bytes, (uint64_t)ent->nerrs * C * S);
	}
	return i;
}

int ecg_recover(ecg_ctx_t *ctx, int k, int p, uint64_t C, uint32_t S,
		void *stripes, int64_t stripe_stride,
		const uint32_t *err_list, int nerrs, void *stream)
{
	struct ecg_rcache_ent ent;
	int rc;

	rc = check_kp(k, p);
	if (rc)
		return rc;
	if (err_list == NULL)
		return ecg_fail(-ECG_DER_INVAL, "recover: NULL err_list");
	if (nerrs > p)
		return ecg_fail(-ECG_DER_DATA_LOSS, "recover: %d erasures > p=%d", nerrs, p);
	if (nerrs <= 0)
		return 0;
	ecg_trace_push("ecg:recover");
	rc = recov_lookup(ctx, k, p, err_list, nerrs, &ent);
	if (rc == 0)
		rc = recover_with(ctx, &ent, C, S, stripes, stripe_stride, stream);
	ecg_trace_pop();
	return rc;
}

/*
 * Product + chunked checksums of every output cell (include/ecg_csum.h).  One
 * fused launch when the shape allows (CRC types, k <= 16, rows <= 8, 16-byte
 * aligned cells, record chunk a multiple of 4 KiB); otherwise the product
 * followed by one ecg_csum_extents launch per output row -- both on the
 * device, the fused path only saves the re-read of the outputs.
 * csums[row_slot[r]][s][chunk].
 */
static int aligned16_ok(const void *src, const int64_t *soff, int k, int64_t sstride,
			const void *dst, const int64_t *doff, int rows, int64_t dstride)
{
	uint64_t bits = (uint64_t)(uintptr_t)src | (uint64_t)(uintptr_t)dst | (uint64_t)sstride |
			(uint64_t)dstride;

	for (int j = 0; j < k; j++)
		bits |= (uint64_t)soff[j];
	for (int r = 0; r < rows; r++)
		bits |= (uint64_t)doff[r];
	return (bits & 15u) == 0;
}

int ecg_matmul_csum(ecg_ctx_t *ctx, int k, int rows, const unsigned char *coef, uint64_t C,
		    uint32_t S, const void *src, const int64_t *soff, int64_t sstride, void *dst,
		    const int64_t *doff, int64_t dstride, int type, uint64_t chunksize,
		    uint64_t rec_size, void *csums, const uint32_t *row_slot, void *stream)
{
	const int cl = ecg_csum_len(type);
	ecg_mmcs_params_t q;
	hipStream_t st;
	uint32_t nch;
	int fused = 0, rc, r;

	if (cl < 0)
		return ecg_fail(-ECG_DER_NOTSUPPORTED, "csum: hash type %d not supported", type);
	if (csums == NULL || rec_size == 0 || chunksize == 0 || C % rec_size)
		return ecg_fail(-ECG_DER_INVAL, "csum: bad chunk/record size or NULL csums");
	if (C == 0 || S == 0)
		return 0;
	rc = ecg_ctx_enter(ctx);
	if (rc)
		return rc;
	ecg_gf_init();
	st = ecg_pick_stream(ctx, stream);
	if (k <= ECG_KMAX_K && rows <= ECG_KMAX_R) {
		fused = ecg_csum_fused_params(ctx, type, chunksize, rec_size, C, k, rows, csums, &q);
		if (fused < 0)
			return fused;
	}
	if (fused) {
		ecg_mm_params_t *prm = calloc(1, sizeof(*prm));
		uint32_t kid = 0;
		int e, j;

		if (prm == NULL)
			return ecg_fail(-ECG_DER_NOMEM, "matmul_csum: calloc");
		prm->src = src;
		prm->dst = dst;
		prm->src_stripe_stride = sstride;
		prm->dst_stripe_stride = dstride;
		prm->cell_bytes = C;
		prm->nstripes = S;
		prm->k = (uint32_t)k;
		prm->rows = (uint32_t)rows;
		for (j = 0; j < k; j++)
			prm->src_cell_off[j] = soff[j];
		for (r = 0; r < rows; r++) {
			prm->dst_cell_off[r] = doff[r];
			q.row_slot[r] = row_slot[r];
			for (j = 0; j < k; j++)
				ecg_build_ptbl(coef[(size_t)r * k + j], &prm->tbl[r][j]);
		}
		/* the workgroup kernel XORs per-wave partials into the checksums */
		if (aligned16_ok(src, soff, k, sstride, dst, doff, rows, dstride)) {
			hipError_t he = hipMemsetAsync(csums, 0, (size_t)rows * S * q.nch * (size_t)cl, st);

			if (he != hipSuccess) {
				free(prm);
				return ecg_hip_fail(he, "csum memset");
			}
		}
		e = ecg_k_launch_matmul_csum(prm, &q, &ctx->cfg, (void *)st, &kid);
		free(prm);
		if (e == 0) {
			ECG_STAT_ADD(ctx, launches, 1);
			ECG_STAT_ADD(ctx, csum_chunks, (uint64_t)rows * S * q.nch);
			ecg_set_last_kernel(ecg_k_kernel_name(kid));
			return 0;
		}
		if (e != 1)
			return ecg_hip_fail((hipError_t)e, "fused kernel launch");
		/* e == 1: operands not 16-byte aligned -> two-pass path */
	}
	rc = matmul2(ctx, k, rows, coef, C, S, src, soff, sstride, NULL, NULL, 0, dst, doff, dstride,
		     0, (void *)st);
	if (rc)
		return rc;
	nch = ecg_csum_chunk_count(chunksize, rec_size, 0, C / rec_size);
	for (r = 0; r < rows; r++) {
		rc = ecg_csum_extents(ctx, type, chunksize, rec_size, 0, C / rec_size,
				      (const uint8_t *)dst + doff[r], dstride, S,
				      (uint8_t *)csums + (uint64_t)row_slot[r] * S * nch * (uint64_t)cl,
				      (void *)st);
		if (rc)
			return rc;
	}
	return 0;
}

int ecg_encode_csum(ecg_ctx_t *ctx, int k, int p, uint64_t C, uint32_t S, const void *data,
		    int64_t data_stripe_stride, void *parity, int64_t parity_cell_stride,
		    int64_t parity_stripe_stride, int type, uint64_t chunksize, uint64_t rec_size,
		    void *csums, void *stream)
{
	unsigned char en[(ECG_MAX_K + ECG_MAX_P) * ECG_MAX_K];
	int64_t soff[ECG_MAX_K], doff[ECG_MAX_P];
	uint32_t slot[ECG_MAX_P];
	int i, rc;

	rc = check_kp(k, p);
	if (rc)
		return rc;
	if (data == NULL || parity == NULL)
		return ecg_fail(-ECG_DER_INVAL, "encode_csum: NULL buffer");
	ecg_gen_cauchy1(k, p, en);
	for (i = 0; i < k; i++)
		soff[i] = (int64_t)i * (int64_t)C;
	for (i = 0; i < p; i++) {
		doff[i] = (int64_t)i * parity_cell_stride;
		slot[i] = (uint32_t)i;
	}
	rc = ecg_matmul_csum(ctx, k, p, &en[k * k], C, S, data, soff, data_stripe_stride, parity, doff,
			     parity_stripe_stride, type, chunksize, rec_size, csums, slot, stream);
	if (rc == 0) {
		ECG_STAT_ADD(ctx, encode_stripes, S);
		ECG_STAT_ADD(ctx, encode_bytes, (uint64_t)k * C * S);
	}
	return rc;
}

int ecg_recover_csum(ecg_ctx_t *ctx, int k, int p, uint64_t C, uint32_t S, void *stripes,
		     int64_t stripe_stride, const uint32_t *err_list, int nerrs, int type,
		     uint64_t chunksize, uint64_t rec_size, void *csums, void *stream)
{
	struct ecg_rcache_ent ent;
	int64_t soff[ECG_MAX_K], doff[ECG_MAX_P];
	uint32_t slot[ECG_MAX_P];
	int i, j, rc;

	rc = check_kp(k, p);
	if (rc)
		return rc;
	if (err_list == NULL || stripes == NULL)
		return ecg_fail(-ECG_DER_INVAL, "recover_csum: NULL argument");
	if (nerrs > p)
		return ecg_fail(-ECG_DER_DATA_LOSS, "recover_csum: %d erasures > p=%d", nerrs, p);
	if (nerrs <= 0)
		return 0;
	rc = recov_lookup(ctx, k, p, err_list, nerrs, &ent);
	if (rc)
		return rc;
	for (i = 0; i < ent.k; i++)
		soff[i] = (int64_t)ent.dec_idx[i] * (int64_t)C;
	for (i = 0; i < ent.nerrs; i++) {
		doff[i] = (int64_t)ent.out_idx[i] * (int64_t)C;
		slot[i] = 0;
		for (j = 0; j < nerrs; j++)	/* checksum rows in err_list order */
			if (err_list[j] == ent.out_idx[i])
				slot[i] = (uint32_t)j;
	}
	rc = ecg_matmul_csum(ctx, ent.k, ent.nerrs, ent.rows, C, S, stripes, soff, stripe_stride,
			     stripes, doff, stripe_stride, type, chunksize, rec_size, csums, slot,
			     stream);
	if (rc == 0) {
		ECG_STAT_ADD(ctx, recover_stripes, S);
		ECG_STAT_ADD(ctx, recover_bytes, (uint64_t)ent.nerrs * C * S);
	}
	return rc;
}

int ecg_update(ecg_ctx_t *ctx, int k, int p, uint64_t C, uint32_t S,
	       int nupd, const uint32_t *cell_idx,
	       const void *old_cells, const void *new_cells, int64_t upd_stripe_stride,
	       void *parity, int64_t parity_cell_stride, int64_t parity_stripe_stride,
	       void *stream)
{
	unsigned char en[(ECG_MAX_K + ECG_MAX_P) * ECG_MAX_K];
	unsigned char coef[ECG_MAX_P * ECG_MAX_K];
	int64_t soff[ECG_MAX_K], doff[ECG_MAX_P];
	int u, r, rc;

	rc = check_kp(k, p);
	if (rc)
		return rc;
	if (nupd < 1 || nupd > k || cell_idx == NULL)
		return ecg_fail(-ECG_DER_INVAL, "update: bad nupd=%d", nupd);
	ecg_gen_cauchy1(k, p, en);
	for (u = 0; u < nupd; u++) {
		if (cell_idx[u] >= (uint32_t)k)
			return ecg_fail(-ECG_DER_INVAL, "update: cell %u >= k", cell_idx[u]);
		soff[u] = (int64_t)u * (int64_t)C;
		for (r = 0; r < p; r++)
			coef[r * nupd + u] = en[(k + r) * k + cell_idx[u]];
	}
	for (r = 0; r < p; r++)
		doff[r] = (int64_t)r * parity_cell_stride;
	ecg_trace_push("ecg:update");
	rc = matmul2(ctx, nupd, p, coef, C, S, old_cells, soff, upd_stripe_stride,
		     new_cells, soff, upd_stripe_stride, parity, doff, parity_stripe_stride,
		     ECG_F_ACCUMULATE, stream);
	ecg_trace_pop();
	if (rc == 0) {
		ECG_STAT_ADD(ctx, update_cells, (uint64_t)nupd * S);
		ECG_STAT_ADD(ctx, update_bytes, (uint64_t)nupd * C * S);
	}
	return rc;
}

/* ------------------------------------------------------------------------ */
/* host-staging pipeline                                                     */
/* ------------------------------------------------------------------------ */
static int stage_reserve(ecg_ctx_t *ctx, size_t bytes)
{
	int i;

	if (ctx->stage.dev_bytes >= bytes)
		return 0;
	stage_free(ctx);
	for (i = 0; i < ECG_NSLOT; i++) {
		HIPCHK(hipMalloc(&ctx->stage.dev[i], bytes));
		HIPCHK(hipStreamCreateWithFlags(&ctx->stage.st[i], hipStreamNonBlocking));
		HIPCHK(hipEventCreateWithFlags(&ctx->stage.done[i], hipEventDisableTiming));
	}
	ctx->stage.dev_bytes = bytes;
	return 0;
}

hipError_t ecg_stage_copy(void *dst, const void *src, size_t bytes, size_t row, hipMemcpyKind kind,
			  hipStream_t st)
{
	hipError_t e = hipSuccess;
	size_t h;

	/* both sides are contiguous, so any row length works: whole rows up to
	 * 1 MiB (short rows made the queue's 32 KiB-cell copies slower) */
	if (row && row < (1u << 20))
		row *= (1u << 20) / row;
	h = row ? bytes / row : 0;

	if (h == 0)
		return bytes ? hipMemcpyAsync(dst, src, bytes, kind, st) : hipSuccess;
	e = hipMemcpy2DAsync(dst, row, src, row, row, h, kind, st);
	if (e == hipSuccess && bytes > h * row)
		e = hipMemcpyAsync((char *)dst + h * row, (const char *)src + h * row, bytes - h * row,
				   kind, st);
	return e;
}

/* H2D copy of an encode_host chunk: 0 (default) one 2D copy of cell rows
 * (ecg_stage_copy), 1 one 1D copy, 3 one strided 2D copy per cell column
 * (ECG_ENC_H2D_PARTS; tools/bench_pcie.py: 52.1 / 45.0 / 50.5 GiB/s EC_8P2) */
static int g_enc_h2d_parts;
static pthread_once_t g_enc_h2d_once = PTHREAD_ONCE_INIT;

static void enc_h2d_init(void)
{
	const char *e = getenv("ECG_ENC_H2D_PARTS");

	g_enc_h2d_parts = e ? atoi(e) : 0;
}

static int enc_h2d_parts(void)
{
	pthread_once(&g_enc_h2d_once, enc_h2d_init);
	return g_enc_h2d_parts;
}

/* Stripes per staging chunk when the caller passes 0: ~32 MiB of input cells
 * per chunk.  Each call ends by draining its last chunk (kernel + D2H) while
 * the H2D link idles, so small chunks keep alternating encode / recovery
 * calls near the link rate: EC_8P2 1 MiB rebuild stream, 64-stripe calls,
 * 16 / 8 / 4 stripes per chunk = 0.91-0.93 / 0.93-0.94 / 0.945 of the raw
 * H2D rate (profiles/r02/host_chunk_sweep/); long single calls are flat from
 * 8 to 32 stripes (profiles/r01/pcie.json). */
static uint32_t host_chunk_default(int k, uint64_t C)
{
	const uint64_t n = (32ull << 20) / ((uint64_t)k * C);

	return n < 1 ? 1 : n > 4096 ? 4096 : (uint32_t)n;
}

/* parity row r of stripe s at parity + r*prow + s*C (prow = S*C for the
 * [p][S][C] layout; a shard of a larger batch passes the batch's row pitch) */
int ecg_encode_host_rows(ecg_ctx_t *ctx, int k, int p, uint64_t C, uint32_t S, const void *data,
			 void *parity, size_t prow, uint32_t chunk)
{
	const unsigned char *hd = data;
	unsigned char *hp = parity;
	const int h2d_mode = enc_h2d_parts();
	uint32_t s0, slot = 0;
	int rc, r;

	rc = check_kp(k, p);
	if (rc)
		return rc;
	if (data == NULL || parity == NULL)
		return ecg_fail(-ECG_DER_INVAL, "encode_host: NULL buffer");
	rc = ecg_ctx_enter(ctx);
	if (rc)
		return rc;
	if (S == 0 || C == 0)
		return 0;
	if (chunk == 0)
		chunk = host_chunk_default(k, C);
	if (chunk > S)
		chunk = S;
	pthread_mutex_lock(&ctx->lock);
	ecg_trace_push("ecg:encode_host");
	/* staged parity rows at a pitch of cs*C + ECG_PARITY_ROW_PAD (include/ecg.h) */
	rc = stage_reserve(ctx, (size_t)chunk * (k + p) * C + (size_t)p * ECG_PARITY_ROW_PAD);
	for (s0 = 0; rc == 0 && s0 < S; s0 += chunk, slot = (slot + 1) % ECG_NSLOT) {
		uint32_t cs = S - s0 < chunk ? S - s0 : chunk;
		unsigned char *dd = ctx->stage.dev[slot];
		unsigned char *dp = dd + (size_t)cs * k * C;
		const size_t dprow = (size_t)cs * C + ECG_PARITY_ROW_PAD;
		hipStream_t st = ctx->stage.st[slot];
		hipError_t e;

		ecg_trace_push("ecg:stage_wait");
		e = hipEventSynchronize(ctx->stage.done[slot]);
		ecg_trace_pop();
		if (e == hipSuccess && h2d_mode == 1) {
			e = hipMemcpyAsync(dd, hd + (size_t)s0 * k * C, (size_t)cs * k * C,
					   hipMemcpyHostToDevice, st);
		} else if (e == hipSuccess && h2d_mode == 3) {
			for (r = 0; e == hipSuccess && r < k; r++)
				e = hipMemcpy2DAsync(dd + (size_t)r * C, (size_t)k * C,
						     hd + (size_t)s0 * k * C + (size_t)r * C, (size_t)k * C, C, cs,
						     hipMemcpyHostToDevice, st);
		} else if (e == hipSuccess) {
			e = ecg_stage_copy(dd, hd + (size_t)s0 * k * C, (size_t)cs * k * C, C,
					   hipMemcpyHostToDevice, st);
		}
		if (e != hipSuccess) {
			rc = ecg_hip_fail(e, "encode_host H2D");
			break;
		}
		rc = ecg_encode(ctx, k, p, C, cs, dd, (int64_t)k * C, dp, (int64_t)dprow, (int64_t)C, st);
		for (r = 0; rc == 0 && r < p; r++) {
			e = ecg_stage_copy(hp + (size_t)r * prow + (size_t)s0 * C, dp + (size_t)r * dprow,
					   (size_t)cs * C, C, hipMemcpyDeviceToHost, st);
			if (e != hipSuccess)
				rc = ecg_hip_fail(e, "encode_host D2H");
		}
		if (rc == 0) {
			e = hipEventRecord(ctx->stage.done[slot], st);
			if (e != hipSuccess)
				rc = ecg_hip_fail(e, "encode_host event");
		}
	}
	for (r = 0; r < ECG_NSLOT; r++)
		if (ctx->stage.st[r])
			(void)hipStreamSynchronize(ctx->stage.st[r]);
	if (rc == 0) {
		ECG_STAT_ADD(ctx, h2d_bytes, (uint64_t)k * C * S);
		ECG_STAT_ADD(ctx, d2h_bytes, (uint64_t)p * C * S);
	}
	ecg_trace_pop();
	pthread_mutex_unlock(&ctx->lock);
	return rc;
}

int ecg_encode_host(ecg_ctx_t *ctx, int k, int p, uint64_t C, uint32_t S,
		    const void *data, void *parity, uint32_t chunk)
{
	return ecg_encode_host_rows(ctx, k, p, C, S, data, parity, (size_t)S * C, chunk);
}

int ecg_recover_host(ecg_ctx_t *ctx, int k, int p, uint64_t C, uint32_t S,
		     void *stripes, const uint32_t *err_list, int nerrs, uint32_t chunk)
{
	struct ecg_rcache_ent ent;
	unsigned char *hs = stripes;
	const size_t sstride = (size_t)(k + p) * C;
	uint32_t s0, slot = 0;
	int rc, i;

	rc = check_kp(k, p);
	if (rc)
		return rc;
	if (err_list == NULL || stripes == NULL)
		return ecg_fail(-ECG_DER_INVAL, "recover_host: NULL argument");
	if (nerrs > p)
		return ecg_fail(-ECG_DER_DATA_LOSS, "recover_host: %d erasures > p=%d", nerrs, p);
	if (nerrs <= 0 || S == 0 || C == 0)
		return 0;
	rc = ecg_ctx_enter(ctx);
	if (rc)
		return rc;
	rc = recov_lookup(ctx, k, p, err_list, nerrs, &ent);
	if (rc)
		return rc;
	if (chunk == 0)
		chunk = host_chunk_default(k, C);
	if (chunk > S)
		chunk = S;
	pthread_mutex_lock(&ctx->lock);
	ecg_trace_push("ecg:recover_host");
	rc = stage_reserve(ctx, (size_t)chunk * sstride);
	for (s0 = 0; rc == 0 && s0 < S; s0 += chunk, slot = (slot + 1) % ECG_NSLOT) {
		uint32_t cs = S - s0 < chunk ? S - s0 : chunk;
		unsigned char *dd = ctx->stage.dev[slot];
		hipStream_t st = ctx->stage.st[slot];
		hipError_t e;

		ecg_trace_push("ecg:stage_wait");
		e = hipEventSynchronize(ctx->stage.done[slot]);
		ecg_trace_pop();

		/* survivors the decode reads: k cells per stripe, one strided 2D
		 * copy per run of consecutive cells */
		for (i = 0; e == hipSuccess && i < k;) {
			int n = 1;

			while (i + n < k && ent.dec_idx[i + n] == ent.dec_idx[i] + (uint32_t)n)
				n++;
			e = hipMemcpy2DAsync(dd + (size_t)ent.dec_idx[i] * C, sstride,
					     hs + (size_t)s0 * sstride + (size_t)ent.dec_idx[i] * C,
					     sstride, (size_t)n * C, cs, hipMemcpyHostToDevice, st);
			i += n;
		}
		if (e != hipSuccess) {
			rc = ecg_hip_fail(e, "recover_host H2D");
			break;
		}
		rc = recover_with(ctx, &ent, C, cs, dd, (int64_t)sstride, st);
		for (i = 0; rc == 0 && i < nerrs;) {
			int n = 1;	/* runs of consecutive erased cells in err_list order */

			while (i + n < nerrs && err_list[i + n] == err_list[i] + (uint32_t)n)
				n++;
			e = hipMemcpy2DAsync(hs + (size_t)s0 * sstride + (size_t)err_list[i] * C,
					     sstride, dd + (size_t)err_list[i] * C, sstride, (size_t)n * C, cs,
					     hipMemcpyDeviceToHost, st);
			if (e != hipSuccess)
				rc = ecg_hip_fail(e, "recover_host D2H");
			i += n;
		}
		if (rc == 0) {
			e = hipEventRecord(ctx->stage.done[slot], st);
			if (e != hipSuccess)
				rc = ecg_hip_fail(e, "recover_host event");
		}
	}
	for (i = 0; i < ECG_NSLOT; i++)
		if (ctx->stage.st[i])
			(void)hipStreamSynchronize(ctx->stage.st[i]);
	if (rc == 0) {
		ECG_STAT_ADD(ctx, h2d_bytes, (uint64_t)k * C * S);
		ECG_STAT_ADD(ctx, d2h_bytes, (uint64_t)nerrs * C * S);
	}
	ecg_trace_pop();
	pthread_mutex_unlock(&ctx->lock);
	return rc;
}

/* ------------------------------------------------------------------------ */
/* plumbing                                                                  */
/* ------------------------------------------------------------------------ */
int ecg_dev_alloc(ecg_ctx_t *ctx, size_t bytes, void **ptr)
{
	int rc = ecg_ctx_enter(ctx);

	if (rc)
		return rc;
	if (ptr == NULL)
		return ecg_fail(-ECG_DER_INVAL, "dev_alloc: NULL ptr");
	{
		hipError_t e = hipMalloc(ptr, bytes ? bytes : 1);

		if (e == hipErrorOutOfMemory)
			return ecg_fail(-ECG_DER_NOMEM, "dev_alloc: %zu bytes", bytes);
		if (e != hipSuccess)
			return ecg_hip_fail(e, "hipMalloc");
	}
	return 0;
}

int ecg_dev_free(ecg_ctx_t *ctx, void *ptr)
{
	int rc = ecg_ctx_enter(ctx);

	if (rc)
		return rc;
	ecg_place_forget();
	HIPCHK(hipFree(ptr));
	return 0;
}

int ecg_host_alloc(ecg_ctx_t *ctx, size_t bytes, void **ptr)
{
	int rc = ecg_ctx_enter(ctx);

	if (rc)
		return rc;
	if (ptr == NULL)
		return ecg_fail(-ECG_DER_INVAL, "host_alloc: NULL ptr");
	HIPCHK(hipHostMalloc(ptr, bytes ? bytes : 1, hipHostMallocDefault));
	return 0;
}

int ecg_host_free(ecg_ctx_t *ctx, void *ptr)
{
	int rc = ecg_ctx_enter(ctx);

	if (rc)
		return rc;
	HIPCHK(hipHostFree(ptr));
	return 0;
}

int ecg_memcpy(ecg_ctx_t *ctx, void *dst, const void *src, size_t bytes, int kind, void *stream)
{
	static const hipMemcpyKind kinds[] = {hipMemcpyHostToDevice, hipMemcpyDeviceToHost,
					      hipMemcpyDeviceToDevice, hipMemcpyDefault};
	int rc = ecg_ctx_enter(ctx);

	if (rc)
		return rc;
	if (kind < 0 || kind > 3)
		return ecg_fail(-ECG_DER_INVAL, "memcpy: kind %d", kind);
	HIPCHK(hipMemcpyAsync(dst, src, bytes, kinds[kind], ecg_pick_stream(ctx, stream)));
	return 0;
}

int ecg_memset(ecg_ctx_t *ctx, void *dst, int value, size_t bytes, void *stream)
{
	int rc = ecg_ctx_enter(ctx);

	if (rc)
		return rc;
	HIPCHK(hipMemsetAsync(dst, value, bytes, ecg_pick_stream(ctx, stream)));
	return 0;
}

int ecg_stream_create(ecg_ctx_t *ctx, void **stream)
{
	int rc = ecg_ctx_enter(ctx);

	if (rc)
		return rc;
	HIPCHK(hipStreamCreateWithFlags((hipStream_t *)stream, hipStreamNonBlocking));
	return 0;
}

int ecg_stream_destroy(ecg_ctx_t *ctx, void *stream)
{
	int rc = ecg_ctx_enter(ctx);

	if (rc)
		return rc;
	HIPCHK(hipStreamDestroy((hipStream_t)stream));
	return 0;
}

int ecg_stream_sync(ecg_ctx_t *ctx, void *stream)
{
	int rc = ecg_ctx_enter(ctx);

	if (rc)
		return rc;
	HIPCHK(hipStreamSynchronize(ecg_pick_stream(ctx, stream)));
	return 0;
}

int ecg_event_create(ecg_ctx_t *ctx, void **event)
{
	int rc = ecg_ctx_enter(ctx);

	if (rc)
		return rc;
	HIPCHK(hipEventCreate((hipEvent_t *)event));
	return 0;
}

int ecg_event_destroy(ecg_ctx_t *ctx, void *event)
{
	int rc = ecg_ctx_enter(ctx);

	if (rc)
		return rc;
	HIPCHK(hipEventDestroy((hipEvent_t)event));
	return 0;
}

int ecg_event_record(ecg_ctx_t *ctx, void *event, void *stream)
{
	int rc = ecg_ctx_enter(ctx);

	if (rc)
		return rc;
	HIPCHK(hipEventRecord((hipEvent_t)event, ecg_pick_stream(ctx, stream)));
	return 0;
}

int ecg_event_elapsed_ms(ecg_ctx_t *ctx, void *start, void *stop, float *ms)
{
	int rc = ecg_ctx_enter(ctx);

	if (rc)
		return rc;
	HIPCHK(hipEventSynchronize((hipEvent_t)stop));
	HIPCHK(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
	return 0;
}

int ecg_device_sync(ecg_ctx_t *ctx)
{
	int rc = ecg_ctx_enter(ctx);

	if (rc)
		return rc;
	HIPCHK(hipDeviceSynchronize());
	return 0;
}

int ecg_dev_copy_kernel(ecg_ctx_t *ctx, void *dst, const void *src, size_t bytes, int mode,
			void *stream)
{
	int rc = ecg_ctx_enter(ctx);
	uint32_t kid = 0;
	int e;

	if (rc)
		return rc;
	if (mode < 0 || mode > 2)
		return ecg_fail(-ECG_DER_INVAL, "copy kernel: mode %d", mode);
	e = ecg_k_launch_copy(src, dst, bytes, mode, (void *)ecg_pick_stream(ctx, stream),
			      ctx->cfg.grid_x, &kid);
	if (e)
		return ecg_hip_fail((hipError_t)e, "copy kernel");
	ecg_set_last_kernel(ecg_k_kernel_name(kid));
	return 0;
}
