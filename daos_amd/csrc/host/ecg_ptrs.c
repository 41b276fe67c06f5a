/*
 * ecg_ptrs.c -- pointer-table products and the scatter-gather encode of the
 * DAOS client (include/ecg.h ecg_matmul_ptrs, include/ecg_daos.h
 * ecg_obj_ec_recx_encode).
 *
 * ISA-L's interface takes one array of cell pointers per stripe
 * (ec_encode_data(len, k, rows, tbls, data[], coding[])); the client's encode
 * loop hands it cells that live wherever the user's scatter-gather list put
 * them (ref:src/object/cli_ec.c:476-546, 593-663).  Here the per-stripe
 * pointer arrays of a whole batch become one device table and one launch of
 * ecg_mm_ptr_kernel.
 *
 * Scratch (per context, ctx->lock): pinned staging + device copy of the
 * pointer table, and device space for cells gathered from several iovs.  The
 * event `done` is recorded after every launch that reads the scratch; the
 * next user waits for it before overwriting, whatever its stream.
 */
#include <stdlib.h>
#include <string.h>

#include "ecg_internal.h"
#include "../../../include/ecg_daos.h"

/* Next scratch slot, grown to size and free of readers (ctx->lock held). */
int ecg_scratch_reserve(ecg_ctx_t *ctx, size_t pin_bytes, size_t dev_bytes,
			   struct ecg_scratch_slot **out)
{
	struct ecg_scratch_slot *sc = &ctx->scratch.slot[ctx->scratch.next];
	hipError_t e;

	ctx->scratch.next = (ctx->scratch.next + 1) % ECG_NSCRATCH;
	if (sc->done == NULL) {
		e = hipEventCreateWithFlags(&sc->done, hipEventDisableTiming);
		if (e != hipSuccess)
			return ecg_hip_fail(e, "scratch event");
	}
	if (sc->pending) {		/* the launch before last still reading it? */
		e = hipEventSynchronize(sc->done);
		if (e != hipSuccess)
			return ecg_hip_fail(e, "scratch wait");
		sc->pending = 0;
	}
	/* grow in whole steps (at least 64 KiB, at least double): a pinned
	 * re-allocation costs ~250 us (hipHostFree + hipHostMalloc), and the
	 * batching queue's tables grow batch by batch (gpurun_out/r6f: 7-8
	 * re-allocations per queue_bench run at 128 KiB cells) */
	if (pin_bytes > sc->pin_bytes && pin_bytes < (16u << 20)) {
		size_t want = sc->pin_bytes * 2 > (64u << 10) ? sc->pin_bytes * 2 : (64u << 10);

		pin_bytes = pin_bytes > want ? pin_bytes : want;
	}
	/* (device scratch also holds gathered cells, which can be GiBs: doubled
	 * only while small) */
	if (dev_bytes > sc->dev_bytes && dev_bytes < (16u << 20)) {
		size_t want = sc->dev_bytes * 2 > (64u << 10) ? sc->dev_bytes * 2 : (64u << 10);

		dev_bytes = dev_bytes > want ? dev_bytes : want;
	}
	if (pin_bytes > sc->pin_bytes) {
		if (sc->pin)
			(void)hipHostFree(sc->pin);
		sc->pin = NULL;
		sc->pin_bytes = 0;
		/* read by the fetch kernel of whichever device the context
		 * drives: mapped for every device */
		e = hipHostMalloc(&sc->pin, pin_bytes, hipHostMallocPortable);
		if (e != hipSuccess)
			return ecg_hip_fail(e, "scratch pinned alloc");
		sc->pin_bytes = pin_bytes;
	}
	if (dev_bytes > sc->dev_bytes) {
		if (sc->dev)
			(void)hipFree(sc->dev);
		sc->dev = NULL;
		sc->dev_bytes = 0;
		e = hipMalloc(&sc->dev, dev_bytes);
		if (e != hipSuccess)
			return ecg_hip_fail(e, "scratch device alloc");
		sc->dev_bytes = dev_bytes;
	}
	*out = sc;
	return 0;
}

int ecg_table_upload(struct ecg_scratch_slot *sc, size_t bytes, hipStream_t st, const char *what)
{
	const size_t words = (bytes + 7) / 8;
	hipError_t e;

	if (words > UINT32_MAX)
		return ecg_fail(-ECG_DER_INVAL, "%s: %zu bytes", what, bytes);
	/* A fetch kernel, not hipMemcpyAsync: a small pinned H2D copy queued
	 * behind running work held the queue's worker 47-185 us per batch
	 * (profiles/r06/queue_unlocked/qt_subphases_before.log), while a launch
	 * returns in ~5 us; one-thread device-update batches ran 111-204 GiB/s
	 * against 39-58 with the copy (qt_fetch_vs_memcpy.log), large encode
	 * batches the same either way. */
	e = (hipError_t)ecg_k_launch_fetch((const uint64_t *)sc->pin, (uint64_t *)sc->dev, (uint32_t)words, st);
	return e == hipSuccess ? 0 : ecg_hip_fail(e, what);
}

void ecg_scratch_free(ecg_ctx_t *ctx)
{
	for (int i = 0; i < ECG_NSCRATCH; i++) {
		struct ecg_scratch_slot *sc = &ctx->scratch.slot[i];

		if (sc->pending && sc->done)
			(void)hipEventSynchronize(sc->done);
		if (sc->pin)
			(void)hipHostFree(sc->pin);
		if (sc->dev)
			(void)hipFree(sc->dev);
		if (sc->done)
			(void)hipEventDestroy(sc->done);
	}
	memset(&ctx->scratch, 0, sizeof(ctx->scratch));
}

/* Lane access of a pointer table (ecg_k_launch_matmul_ptrs): from the OR of
 * the input and of the output cell addresses; 0 (the byte kernel) when the
 * device serves no misaligned dwords and an address is off a dword. */
static int ptr_granule(const uint64_t *tab, uint32_t S, int k, int rows, int no_unaligned)
{
	uint64_t in = 0, out = 0;

	for (uint64_t s = 0; s < S; s++) {
		const uint64_t *t = tab + s * (uint64_t)(k + rows);

		for (int j = 0; j < k; j++)
			in |= t[j];
		for (int r = 0; r < rows; r++)
			out |= t[k + r];
	}
	if (no_unaligned && ((in | out) & 3u))
		return 0;
	/* k = 8 inputs off a 16-byte boundary: 16-byte lanes funnel-shifted out
	 * of dword-aligned loads, as the offset kernel (ecg_kernels.hip) */
	if ((in & 15u) && !no_unaligned && k == 8 && rows >= 1 && rows <= 3)
		return 2;
	if (in & 3u)
		return 1;	/* outputs at any byte: misaligned dword stores */
	return ((in | out) & 15u) == 0 ? 16 : 4;
}

/* A table whose every cell sits at a fixed offset from a per-stripe base --
 * cell j of stripe s at tab[j] + s * stride, one stride for the inputs and
 * one for the outputs -- is the offset kernel's layout: the client's encode
 * over one contiguous iov (data [S][k][C] in place, ref:src/object/cli_ec.c:
 * 510-536) and parity of stripe n at pbufs[m] + n*C (:638-640).  That launch
 * needs no table upload and no dependent address load per block (the
 * pointer-table kernel ran 4-15 % behind it on the same layout, and a
 * 128 KiB-cell call paid ~25 us of table staging; profiles/r04/ptr_ab/). */
static int table_affine(const uint64_t *tab, uint32_t S, int k, int rows, int64_t *soff, int64_t *sstride,
			int64_t *doff, int64_t *dstride)
{
	const uint64_t n = (uint64_t)(k + rows);
	const uint64_t bs = S > 1 ? tab[n] - tab[0] : 0, bd = S > 1 ? tab[n + (uint64_t)k] - tab[k] : 0;

	for (uint64_t s = 1; s < S; s++)
		for (uint64_t j = 0; j < n; j++)
			if (tab[s * n + j] != tab[j] + s * (j < (uint64_t)k ? bs : bd))
				return 0;
	for (int j = 0; j < k; j++)
		soff[j] = (int64_t)(tab[j] - tab[0]);
	for (int r = 0; r < rows; r++)
		doff[r] = (int64_t)(tab[k + r] - tab[k]);
	*sstride = (int64_t)bs;
	*dstride = (int64_t)bd;
	return 1;
}

/* The offset-kernel launch of an affine table (ecg_matmul: lane choice,
 * launch tuner and last-kernel report as for any strided call). */
static int launch_affine(ecg_ctx_t *ctx, const uint64_t *tab, int k, int rows, const unsigned char *coef,
			 uint64_t C, uint32_t S, hipStream_t st, int *done)
{
	int64_t soff[ECG_KMAX_K], doff[ECG_KMAX_R], ss, ds;

	*done = 0;
	if (k > ECG_KMAX_K || rows > ECG_KMAX_R || !table_affine(tab, S, k, rows, soff, &ss, doff, &ds))
		return 0;
	*done = 1;
	return ecg_matmul(ctx, k, rows, coef, C, S, (const void *)(uintptr_t)tab[0], soff, ss,
			  (void *)(uintptr_t)tab[k], doff, ds, 0, (void *)st);
}

struct ptr_launch_arg {
	const uint64_t *cells_dev;
	int granule;
};

static int launch_ptrs(const ecg_mm_params_t *p, const ecg_launch_cfg_t *cfg, void *stream, uint32_t *kid,
		       const void *arg)
{
	const struct ptr_launch_arg *a = arg;

	return ecg_k_launch_matmul_ptrs(p, a->cells_dev, a->granule, cfg, stream, kid);
}

/* Table already in sc->pin (S x (k+rows) entries); copy, launch, record
 * (ctx->lock held).  With `gather`, its segment table follows the pointer
 * table at byte seg_off of the slot (pinned and device alike): both travel in
 * one H2D and the gather copies run before the product. */
static int launch_table(ecg_ctx_t *ctx, struct ecg_scratch_slot *sc, int k, int rows,
			const unsigned char *coef, uint64_t C, uint32_t S, hipStream_t st,
			const struct ecg_segs *gather, size_t seg_off)
{
	const int granule = ptr_granule((const uint64_t *)sc->pin, S, k, rows, (int)ctx->cfg.no_unaligned);
	size_t tbytes = (size_t)S * (size_t)(k + rows) * sizeof(uint64_t);
	ecg_mm_params_t *prm;
	uint32_t kid = 0;
	hipError_t e;
	int r, j, ke, done;

	if (!(gather && gather->n)) {	/* no gather copies: maybe the offset kernel's layout */
		r = launch_affine(ctx, (const uint64_t *)sc->pin, k, rows, coef, C, S, st, &done);
		if (done)
			return r;
	}
	if (gather && gather->n)
		tbytes = seg_off + gather->n * sizeof(ecg_copy_seg_t);
	r = ecg_table_upload(sc, tbytes, st, "pointer table");
	if (r)
		return r;
	if (gather && gather->n) {
		r = ecg_segs_launch(gather, (unsigned char *)sc->dev + seg_off, st);
		if (r)
			return r;
	}
	prm = calloc(1, sizeof(*prm));
	if (prm == NULL)
		return ecg_fail(-ECG_DER_NOMEM, "matmul_ptrs: calloc");
	ecg_gf_init();
	prm->cell_bytes = C;
	prm->nstripes = S;
	prm->k = (uint32_t)k;
	prm->rows = (uint32_t)rows;
	for (r = 0; r < rows; r++)
		for (j = 0; j < k; j++)
			ecg_build_ptbl(coef[(size_t)r * k + j], &prm->tbl[r][j]);
	{
		/* through the launch tuner like the strided product: wide stripes
		 * probe the blocks-per-CU cap per (shape, pointer-table layout) */
		const struct ptr_launch_arg a = {(const uint64_t *)sc->dev, granule};

		ke = ecg_tune_launch_fn(ctx, prm, (uint32_t)granule, ECG_TUNE_LAYOUT_PTRS, launch_ptrs, &a, st, &kid);
	}
	free(prm);
	if (ke != 0)
		return ecg_hip_fail((hipError_t)ke, "pointer-table kernel launch");
	e = hipEventRecord(sc->done, st);
	if (e != hipSuccess)
		return ecg_hip_fail(e, "scratch event record");
	sc->pending = 1;
	ecg_set_last_kernel(ecg_k_kernel_name(kid));
	return 0;
}

int ecg_matmul_ptrs(ecg_ctx_t *ctx, int k, int rows, const unsigned char *coef, uint64_t cell_bytes,
		    uint32_t nstripes, void *const *cells, void *stream)
{
	const size_t n = (size_t)nstripes * (size_t)(k + rows);
	struct ecg_scratch_slot *sc = NULL;
	hipStream_t st;
	int rc;

	if (ctx == NULL || coef == NULL || (nstripes && cells == NULL))
		return ecg_fail(-ECG_DER_INVAL, "matmul_ptrs: NULL argument");
	if (k < 1 || k > ECG_KMAX_K || rows < 1 || rows > ECG_KMAX_R)
		return ecg_fail(-ECG_DER_INVAL, "matmul_ptrs: k=%d rows=%d (max %d x %d)", k, rows,
				ECG_KMAX_K, ECG_KMAX_R);
	if (cell_bytes == 0 || nstripes == 0)
		return 0;
	for (size_t i = 0; i < n; i++) {
		if (cells[i] == NULL)
			return ecg_fail(-ECG_DER_INVAL, "matmul_ptrs: NULL cell %zu", i);
	}
	rc = ecg_ctx_enter(ctx);
	if (rc)
		return rc;
	st = ecg_pick_stream(ctx, stream);
	{
		int done;

		rc = launch_affine(ctx, (const uint64_t *)cells, k, rows, coef, cell_bytes, nstripes, st, &done);
		if (done)
			return rc;
	}
	pthread_mutex_lock(&ctx->lock);
	rc = ecg_scratch_reserve(ctx, n * sizeof(uint64_t), n * sizeof(uint64_t), &sc);
	if (rc == 0) {
		memcpy(sc->pin, cells, n * sizeof(uint64_t));
		rc = launch_table(ctx, sc, k, rows, coef, cell_bytes, nstripes, st, NULL, 0);
	}
	pthread_mutex_unlock(&ctx->lock);
	return rc;
}

/* ---- per-request delta updates on device cells -------------------------- */

/* Diagnostic build only (-DECG_QUEUE_TIMING): where an update_ptrs call's
 * host time goes -- set device, host planning, ctx lock, scratch, H2D
 * enqueue, kernel launches, event -- wall ns summed over calls. */
#ifdef ECG_QUEUE_TIMING
#include <stdio.h>
#include <time.h>
static uint64_t g_upt[8], g_upn;
static uint64_t upt_now(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}
#define UPT(i) (tp[i] = upt_now())
void ecg_ptrs_timing_print(void)
{
	static const char *nm[7] = {"set device", "plan", "lock", "scratch", "h2d", "kernels", "event"};

	if (g_upn == 0)
		return;
	fprintf(stderr, "update_ptrs timing: %llu calls; us per call:", (unsigned long long)g_upn);
	for (int i = 0; i < 7; i++)
		fprintf(stderr, " %s %.1f", nm[i], g_upt[i] / 1e3 / g_upn);
	fprintf(stderr, "\n");
}
#else
#define UPT(i) ((void)0)
#endif

/*
 * agg_update_parity runs, per updated data cell of a stripe, xor_gen(old, new)
 * then ec_encode_data_update(vec_i) into the stripe's parity cells
 * (ref:src/object/srv_ec_aggregate.c:1086-1102).  A batch of such requests
 * becomes launches of ecg_upd_ptr_kernel (kernels/ecg_ptr_kernels.hip):
 *   1. requests naming the same parity cells (the cells of one stripe updated
 *      one by one) fold into one item of up to ECG_UPD_MU pairs, so that
 *      stripe's parity is read and written once;
 *   2. the parity read-modify-writes of one launch must not touch a byte
 *      twice: items of one parity set beyond the first MU pairs go to later
 *      launches, and so does any item whose parity cells overlap another's
 *      (different pointers into one buffer) -- launches on one stream run in
 *      order, XOR commutes, so the result is the requests applied one by one.
 */
struct upd_req {
	uint64_t par[ECG_KMAX_R];	/* the sort key: the parity cells, then the request's index */
	uint32_t idx;
};

static int upd_req_cmp(const void *a, const void *b)
{
	const struct upd_req *x = a, *y = b;

	for (int r = 0; r < ECG_KMAX_R; r++)
		if (x->par[r] != y->par[r])
			return x->par[r] < y->par[r] ? -1 : 1;
	return x->idx < y->idx ? -1 : x->idx > y->idx;
}

struct upd_ival {
	uint64_t lo, hi;
	uint32_t item;
};

static int upd_ival_cmp(const void *a, const void *b)
{
	const struct upd_ival *x = a, *y = b;

	return x->lo < y->lo ? -1 : x->lo > y->lo;
}

struct upd_item {
	uint32_t first, n;	/* sorted requests [first, first + n) */
	uint32_t wave;
	uint32_t set;		/* parity set (group of identical parity pointers) */
};

/* Any two items of different parity sets whose parity bytes overlap?  A
 * request whose own parity cells overlap one another is refused (its rows
 * would race inside one work item), and so is an old or new cell that
 * overlaps any parity cell of the call (a launch would read bytes another
 * work item is rewriting). */
static int upd_sets_overlap(const struct upd_req *rq, const struct upd_item *it, uint32_t nit, int rows,
			    uint64_t C, void *const *cells, uint32_t nreq, int *overlap)
{
	struct upd_ival *v;
	uint64_t hi = 0;
	size_t n = 0;
	int rc = 0;

	*overlap = 0;
	for (uint32_t i = 0; i < nit; i++) {
		const uint64_t *par = rq[it[i].first].par;

		for (int r = 0; r < rows; r++)
			for (int q = 0; q < r; q++)
				if (par[r] < par[q] + C && par[q] < par[r] + C)
					return ecg_fail(-ECG_DER_INVAL,
							"update_ptrs: parity cells %d and %d of one request overlap", q, r);
	}
	v = malloc(sizeof(*v) * (size_t)nit * (size_t)rows);
	if (v == NULL)
		return ecg_fail(-ECG_DER_NOMEM, "update_ptrs: malloc");
	for (uint32_t i = 0; i < nit; i++) {
		if (i && it[i].set == it[i - 1].set)
			continue;		/* one interval list per parity set */
		for (int r = 0; r < rows; r++)
			v[n++] = (struct upd_ival){rq[it[i].first].par[r], rq[it[i].first].par[r] + C, it[i].set};
	}
	qsort(v, n, sizeof(*v), upd_ival_cmp);
	/* a set's own intervals are disjoint (checked above), so an interval
	 * starting below the highest end so far overlaps another set's */
	for (size_t i = 0; i < n; i++) {
		if (i && v[i].lo < hi)
			*overlap = 1;
		if (v[i].hi > hi)
			hi = v[i].hi;
		v[i].hi = hi;		/* from here on: the running maximum of the ends */
	}
	/* an input [a, a + C) meets a parity interval iff, among the intervals
	 * starting below a + C, the highest end exceeds a */
	for (uint32_t i = 0; i < nreq && rc == 0; i++)
		for (uint32_t j = 0; j < 2 && rc == 0; j++) {
			const uint64_t a = (uint64_t)(uintptr_t)cells[(size_t)i * (rows + 2) + j];
			size_t lo = 0, up = n;	/* first interval with lo >= a + C */

			while (lo < up) {
				const size_t mid = (lo + up) / 2;

				if (v[mid].lo < a + C)
					lo = mid + 1;
				else
					up = mid;
			}
			if (lo > 0 && v[lo - 1].hi > a)
				rc = ecg_fail(-ECG_DER_INVAL, "update_ptrs: request %u: the %s cell overlaps a parity cell "
					      "of the call", i, j ? "new" : "old");
		}
	free(v);
	return rc;
}

/* Launch (wave) of every item when parity sets share bytes: greedy colouring
 * in item order over the conflict graph -- two items conflict when any of
 * their parity intervals meet (items of one set always do) -- built by one
 * sweep over every item's intervals sorted by start, so the cost is
 * O(n log n + conflicting pairs), not a pairwise scan. */
static int upd_color(const struct upd_req *rq, struct upd_item *it, uint32_t nit, int rows, uint64_t C,
		     uint32_t *nwave)
{
	const size_t n = (size_t)nit * (size_t)rows;
	struct upd_ival *v = malloc(sizeof(*v) * n);
	uint32_t *deg = calloc((size_t)nit + 1, sizeof(*deg)), *adj = NULL, *used = NULL;
	size_t ne = 0, x, y;
	int rc = 0;

	if (v == NULL || deg == NULL) {
		rc = ecg_fail(-ECG_DER_NOMEM, "update_ptrs: malloc");
		goto out;
	}
	for (uint32_t i = 0; i < nit; i++)
		for (int r = 0; r < rows; r++)
			v[(size_t)i * rows + r] = (struct upd_ival){rq[it[i].first].par[r], rq[it[i].first].par[r] + C, i};
	qsort(v, n, sizeof(*v), upd_ival_cmp);
	/* each meeting pair once, listed under its later item (CSR: count, then fill) */
	for (int pass = 0; pass < 2; pass++) {
		if (pass == 1) {
			for (uint32_t i = 0; i < nit; i++)
				deg[i + 1] += deg[i];	/* deg[i] = start of item i's list */
			adj = malloc(sizeof(*adj) * (ne ? ne : 1));
			if (adj == NULL) {
				rc = ecg_fail(-ECG_DER_NOMEM, "update_ptrs: malloc");
				goto out;
			}
		}
		for (x = 0; x < n; x++)
			for (y = x + 1; y < n && v[y].lo < v[x].hi; y++) {
				const uint32_t a = v[x].item < v[y].item ? v[x].item : v[y].item;
				const uint32_t b = v[x].item ^ v[y].item ^ a;

				if (a == b)
					continue;
				if (pass == 0) {
					deg[b + 1]++;
					ne++;
				} else {
					adj[deg[b]++] = a;
				}
			}
		if (pass == 1)		/* fill advanced each start to the next item's */
			for (uint32_t i = nit; i > 0; i--)
				deg[i] = deg[i - 1];
	}
	deg[0] = 0;
	used = calloc((size_t)nit + 1, sizeof(*used));
	if (used == NULL) {
		rc = ecg_fail(-ECG_DER_NOMEM, "update_ptrs: malloc");
		goto out;
	}
	*nwave = 0;
	for (uint32_t i = 0; i < nit; i++) {
		uint32_t w = 0;

		/* used[w] == i + 1: wave w holds an earlier item meeting item i */
		for (uint32_t e = deg[i]; e < deg[i + 1]; e++)
			if (it[adj[e]].wave <= nit)
				used[it[adj[e]].wave] = i + 1;
		while (used[w] == i + 1)
			w++;
		it[i].wave = w;
		if (w + 1 > *nwave)
			*nwave = w + 1;
	}
out:
	free(v);
	free(deg);
	free(adj);
	free(used);
	return rc;
}

int ecg_update_ptrs_coef(ecg_ctx_t *ctx, int k, int rows, const unsigned char *coef, uint64_t C, uint32_t nreq,
			 void *const *cells, const uint8_t *vec_i, void *stream, uint32_t *nlaunch)
{
	const uint32_t per = (uint32_t)(rows + 2), rec = (uint32_t)ECG_UPD_REC(rows);
	struct upd_req *rq = NULL;
	struct upd_item *it = NULL;
	struct ecg_scratch_slot *sc = NULL;
	ecg_mm_params_t *prm = NULL;
	uint64_t bits = C;
	uint32_t nit = 0, nset = 0, nwave = 0, kid = 0;
	hipStream_t st;
	int rc = 0, overlap = 0, granule;

	if (nlaunch)
		*nlaunch = 0;
	if (ctx == NULL || coef == NULL || (nreq && (cells == NULL || vec_i == NULL)))
		return ecg_fail(-ECG_DER_INVAL, "update_ptrs: NULL argument");
	if (k < 1 || k > ECG_KMAX_K || rows < 1 || rows > ECG_KMAX_R)
		return ecg_fail(-ECG_DER_INVAL, "update_ptrs: k=%d rows=%d (max %d x %d)", k, rows, ECG_KMAX_K,
				ECG_KMAX_R);
	if (C == 0 || nreq == 0)
		return 0;
	for (uint32_t i = 0; i < nreq; i++) {
		if (vec_i[i] >= (uint8_t)k)
			return ecg_fail(-ECG_DER_INVAL, "update_ptrs: request %u: vec_i %u >= k=%d", i, vec_i[i], k);
		for (uint32_t j = 0; j < per; j++) {
			if (cells[(size_t)i * per + j] == NULL)
				return ecg_fail(-ECG_DER_INVAL, "update_ptrs: request %u: NULL cell %u", i, j);
			bits |= (uint64_t)(uintptr_t)cells[(size_t)i * per + j];
		}
	}
#ifdef ECG_QUEUE_TIMING
	uint64_t tp[8];
#endif
	UPT(0);
	rc = ecg_ctx_enter(ctx);
	if (rc)
		return rc;
	UPT(1);
	rq = calloc(nreq, sizeof(*rq));
	it = calloc(nreq, sizeof(*it));
	prm = calloc(1, sizeof(*prm));
	if (rq == NULL || it == NULL || prm == NULL) {
		rc = ecg_fail(-ECG_DER_NOMEM, "update_ptrs: calloc");
		goto out;
	}
	for (uint32_t i = 0; i < nreq; i++) {
		for (int r = 0; r < rows; r++)
			rq[i].par[r] = (uint64_t)(uintptr_t)cells[(size_t)i * per + 2 + r];
		rq[i].idx = i;
	}
	qsort(rq, nreq, sizeof(*rq), upd_req_cmp);
	/* items: runs of one parity set, at most MU pairs each; the j-th item of
	 * a set goes to launch j */
	for (uint32_t i = 0; i < nreq;) {
		uint32_t e = i + 1, lvl = 0;

		while (e < nreq && memcmp(rq[e].par, rq[i].par, sizeof(rq[i].par)) == 0)
			e++;
		for (uint32_t f = i; f < e; f += ECG_UPD_MU, lvl++) {
			it[nit] = (struct upd_item){f, e - f < ECG_UPD_MU ? e - f : ECG_UPD_MU, lvl, nset};
			if (lvl + 1 > nwave)
				nwave = lvl + 1;
			nit++;
		}
		nset++;
		i = e;
	}
	rc = upd_sets_overlap(rq, it, nit, rows, C, cells, nreq, &overlap);
	if (rc)
		goto out;
	if (overlap) {
		/* parity sets that share bytes: each item in the first launch
		 * none of its conflicting items is in */
		rc = upd_color(rq, it, nit, rows, C, &nwave);
		if (rc)
			goto out;
	}
	/* lane access: 16-byte lanes when everything is 16-byte aligned; dword
	 * lanes when C % 4 == 0 and the addresses are dword-aligned or the device
	 * serves misaligned dwords; else one byte per lane */
	if ((bits & 15u) == 0)
		granule = 16;
	else if ((C & 3u) == 0 && ((bits & 3u) == 0 || !ctx->cfg.no_unaligned))
		granule = 4;
	else
		granule = 0;
	ecg_gf_init();
	prm->cell_bytes = C;
	prm->rows = (uint32_t)rows;
	prm->k = 1;
	for (int r = 0; r < rows; r++)
		for (int j = 0; j < k; j++)
			ecg_build_ptbl(coef[(size_t)r * k + j], &prm->tbl[r][j]);
	st = ecg_pick_stream(ctx, stream);
	UPT(2);
	pthread_mutex_lock(&ctx->lock);
	UPT(3);
	rc = ecg_scratch_reserve(ctx, (size_t)nit * rec * sizeof(uint64_t), (size_t)nit * rec * sizeof(uint64_t),
				 &sc);
	UPT(4);
	if (rc == 0) {
		uint64_t *t = sc->pin;
		uint32_t at = 0, w, i;
		hipError_t e;

		/* records launch by launch: launch w is the records [start_w, at) */
		for (w = 0; w < nwave; w++) {
			for (i = 0; i < nit; i++) {
				uint64_t *o = t + (size_t)at * rec, cols = 0;

				if (it[i].wave != w)
					continue;
				memset(o, 0, rec * sizeof(uint64_t));
				for (int r = 0; r < rows; r++)
					o[r] = rq[it[i].first].par[r];
				for (uint32_t m = 0; m < it[i].n; m++) {
					const uint32_t q = rq[it[i].first + m].idx;

					o[rows + 2 * m] = (uint64_t)(uintptr_t)cells[(size_t)q * per];
					o[rows + 2 * m + 1] = (uint64_t)(uintptr_t)cells[(size_t)q * per + 1];
					cols |= (uint64_t)vec_i[q] << (8 * m);
				}
				o[rows + 2 * ECG_UPD_MU] = cols;
				o[rows + 2 * ECG_UPD_MU + 1] = it[i].n;
				at++;
			}
		}
		rc = ecg_table_upload(sc, (size_t)nit * rec * sizeof(uint64_t), st, "update table");
		UPT(5);
		for (w = 0, at = 0; w < nwave && rc == 0; w++) {
			uint32_t cnt = 0;
			int ke;

			for (i = 0; i < nit; i++)
				cnt += it[i].wave == w;
			prm->nstripes = cnt;
			ke = ecg_k_launch_update_ptrs(prm, (const uint64_t *)sc->dev + (size_t)at * rec, (uint32_t)k,
						      granule, (void *)st, &kid);
			if (ke != 0)
				rc = ecg_hip_fail((hipError_t)ke, "update_ptrs kernel launch");
			at += cnt;
		}
		UPT(6);
		if (rc == 0) {
			e = hipEventRecord(sc->done, st);
			if (e != hipSuccess)
				rc = ecg_hip_fail(e, "scratch event record");
			sc->pending = rc == 0;
		}
		UPT(7);
#ifdef ECG_QUEUE_TIMING
		for (int i = 0; i < 7; i++)
			__atomic_add_fetch(&g_upt[i], tp[i + 1] - tp[i], __ATOMIC_RELAXED);
		__atomic_add_fetch(&g_upn, 1, __ATOMIC_RELAXED);
#endif
	}
	pthread_mutex_unlock(&ctx->lock);
	if (rc == 0) {
		ECG_STAT_ADD(ctx, launches, nwave);
		ECG_STAT_ADD(ctx, update_cells, nreq);
		ECG_STAT_ADD(ctx, update_bytes, (uint64_t)nreq * C);
		ecg_set_last_kernel(ecg_k_kernel_name(kid));
		if (nlaunch)
			*nlaunch = nwave;
	}
out:
	free(rq);
	free(it);
	free(prm);
	return rc;
}

int ecg_update_ptrs(ecg_ctx_t *ctx, int k, int p, uint64_t cell_bytes, uint32_t nreq, void *const *cells,
		    const uint8_t *vec_i, void *stream)
{
	unsigned char en[(ECG_MAX_K + ECG_MAX_P) * ECG_MAX_K];

	if (k < 1 || k > ECG_KMAX_K || p < 1 || p > ECG_KMAX_R)
		return ecg_fail(-ECG_DER_INVAL, "update_ptrs: k=%d p=%d (max %d + %d)", k, p, ECG_KMAX_K, ECG_KMAX_R);
	ecg_gen_cauchy1(k, p, en);	/* parity rows: the codec's, ref:src/object/obj_class.c:614 */
	return ecg_update_ptrs_coef(ctx, k, p, &en[k * k], cell_bytes, nreq, cells, vec_i, stream, NULL);
}

/* ---- obj_ec_recx_encode over a device-resident sgl ---------------------- */

struct sgl_cur {
	const ecg_iov_t *iovs;
	uint32_t nr, idx;
	uint64_t off;
};

static uint64_t iov_left(const struct sgl_cur *c)
{
	return c->idx < c->nr ? c->iovs[c->idx].iov_buf_len - c->off : 0;
}

/* daos_sgl_move (ref:src/include/daos/common.h:419-433): landing exactly on
 * an iov's end steps to the next iov.  Returns bytes actually moved. */
static uint64_t sgl_move(struct sgl_cur *c, uint64_t dist)
{
	uint64_t moved = 0;

	while (moved < dist && c->idx < c->nr) {
		uint64_t left = iov_left(c), step = left < dist - moved ? left : dist - moved;

		c->off += step;
		moved += step;
		if (iov_left(c) == 0) {
			c->idx++;
			c->off = 0;
		}
	}
	return moved;
}

/* Walk the recxs over the sgl exactly as obj_ec_recx_encode /
 * obj_ec_stripe_encode do (ref:src/object/cli_ec.c:493-541, 625-660): a data
 * cell wholly inside the current iov is used in place, any other is gathered
 * into gbase (one copy segment per piece, added to `segs`).  tbl == NULL: dry
 * run that only counts the gathered cells and their pieces.  Fills
 * tbl[n*(k+p) + c] with cell addresses. */
static int sgl_walk(const ecg_iov_t *iovs, uint32_t iov_nr, const ecg_ec_recx_t *recxs,
		    uint32_t recx_nr, int k, int p, uint64_t C, unsigned char *const *pbufs,
		    uint64_t *tbl, unsigned char *gbase, struct ecg_segs *segs, uint64_t *ngather,
		    uint64_t *npieces, uint64_t *bits)
{
	struct sgl_cur cur = {iovs, iov_nr, 0, 0};
	uint64_t last_off = 0, n = 0;

	*ngather = 0;
	*npieces = 0;
	for (uint32_t i = 0; i < recx_nr; i++) {
		sgl_move(&cur, recxs[i].byte_off - last_off);		/* :630-633 */
		last_off = recxs[i].byte_off;
		for (uint32_t j = 0; j < recxs[i].stripe_nr; j++, n++) {
			uint64_t *row = tbl ? tbl + n * (uint64_t)(k + p) : NULL;

			for (int c = 0; c < k; c++) {
				if (iov_left(&cur) >= C) {
					if (row)
						row[c] = (uint64_t)(uintptr_t)iovs[cur.idx].iov_buf + cur.off;
					sgl_move(&cur, C);
					continue;
				}
				unsigned char *dst = gbase ? gbase + *ngather * C : NULL;
				uint64_t copied = 0;

				(*ngather)++;
				if (row)
					row[c] = (uint64_t)(uintptr_t)dst;
				while (copied < C) {
					uint64_t left, cp;

					if (cur.idx >= cur.nr)
						return ecg_fail(-ECG_DER_REC2BIG,
								"recx_encode: sgl shorter than the recxs");
					left = iov_left(&cur);
					cp = left < C - copied ? left : C - copied;
					if (cp == 0) {			/* empty iov: next */
						cur.idx++;
						cur.off = 0;
						continue;
					}
					(*npieces)++;
					if (row) {
						int rc = ecg_segs_add(
							segs, (uint64_t)(uintptr_t)(dst + copied),
							(uint64_t)(uintptr_t)iovs[cur.idx].iov_buf + cur.off, cp);
						if (rc)
							return rc;
					}
					copied += sgl_move(&cur, cp);
				}
			}
			if (row) {
				for (int m = 0; m < p; m++)		/* oer_pbufs[m] + n*C, :637-640 */
					row[k + m] = (uint64_t)(uintptr_t)pbufs[m] + n * C;
				for (int c = 0; c < k + p; c++)
					*bits |= row[c];
			}
		}
		last_off += (uint64_t)recxs[i].stripe_nr * (uint64_t)k * C;	/* :655-656 */
	}
	return 0;
}

int ecg_obj_ec_recx_encode(ecg_ctx_t *ctx, uint32_t oc_id, uint64_t cell_bytes,
			   const ecg_iov_t *iovs, uint32_t iov_nr, const ecg_ec_recx_t *recxs,
			   uint32_t recx_nr, unsigned char *const *pbufs, void *stream)
{
	unsigned char en[(ECG_MAX_K + ECG_MAX_P) * ECG_MAX_K];
	struct ecg_scratch_slot *sc = NULL;
	uint64_t S = 0, ngather = 0, npieces = 0, bits = cell_bytes, tbytes, sbytes;
	int k, p, rc;
	uint32_t i;
	hipStream_t st;

	if (ctx == NULL || iovs == NULL || recxs == NULL || pbufs == NULL || cell_bytes == 0)
		return ecg_fail(-ECG_DER_INVAL, "recx_encode: bad arguments");
	rc = ecg_obj_ec_class_kp(oc_id, &k, &p);
	if (rc)
		return rc;
	ecg_gen_cauchy1(k, p, en);	/* the codec's matrix, ref:src/object/obj_class.c:614 */
	if (k > ECG_KMAX_K)
		return ecg_fail(-ECG_DER_INVAL, "recx_encode: k=%d > %d", k, ECG_KMAX_K);
	for (i = 0; i < recx_nr; i++) {
		S += recxs[i].stripe_nr;
		if (i && recxs[i].byte_off < recxs[i - 1].byte_off +
					     (uint64_t)recxs[i - 1].stripe_nr * (uint64_t)k * cell_bytes)
			return ecg_fail(-ECG_DER_INVAL, "recx_encode: recxs overlap or out of order");
	}
	if (S == 0)
		return 0;
	rc = sgl_walk(iovs, iov_nr, recxs, recx_nr, k, p, cell_bytes, pbufs, NULL, NULL, NULL,
		      &ngather, &npieces, &bits);	/* dry run: validate + count gathers */
	if (rc)
		return rc;
	rc = ecg_ctx_enter(ctx);
	if (rc)
		return rc;
	st = ecg_pick_stream(ctx, stream);
	/* slot layout: [pointer table | gather segments | gathered cells (dev)] */
	tbytes = (S * (uint64_t)(k + p) * sizeof(uint64_t) + 255) & ~255ull;
	sbytes = (npieces * sizeof(ecg_copy_seg_t) + 255) & ~255ull;

	pthread_mutex_lock(&ctx->lock);
	rc = ecg_scratch_reserve(ctx, tbytes + sbytes, tbytes + sbytes + ngather * cell_bytes, &sc);
	if (rc == 0) {
		struct ecg_segs segs = {(ecg_copy_seg_t *)((unsigned char *)sc->pin + tbytes), 0, npieces, 0, 1};

		rc = sgl_walk(iovs, iov_nr, recxs, recx_nr, k, p, cell_bytes, pbufs, (uint64_t *)sc->pin,
			      (unsigned char *)sc->dev + tbytes + sbytes, &segs, &ngather, &npieces, &bits);
		if (rc == 0)	/* one H2D of both tables, gather launch, product launch */
			rc = launch_table(ctx, sc, k, p, &en[k * k], cell_bytes, (uint32_t)S, st, &segs, tbytes);
	}
	pthread_mutex_unlock(&ctx->lock);
	return rc;
}
