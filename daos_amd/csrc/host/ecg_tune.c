/*
 * ecg_tune.c -- per-context launch tuner for the product kernel's
 * blocks-per-CU cap.
 *
 * Wide stripes (k = 16) keep k + rows cell streams in flight per block;
 * with every block the registers allow resident, the HBM streams of an
 * EC_16P2 launch run up to ~9 % below what the same launch reaches at 2
 * blocks per CU -- on some boxes.  Round 2 and 3 measured the sign of the
 * effect per box and per timing pattern: back to back the cap
 * won on one box in every allocation trial and lost 4-6 % on another, and no
 * pointer residue predicts it.  The library therefore measures instead of
 * guessing: the first launches of each large wide shape in a context run as
 * two back-to-back blocks -- ECG_TUNE_W0 + ECG_TUNE_T launches uncapped, then
 * ECG_TUNE_W1 + ECG_TUNE_T at the candidate cap, the last ECG_TUNE_T of each
 * timed with HIP events on the launch stream;
 * once the events have completed (queried without blocking on a later launch
 * of the shape) the faster arm is kept for the shape, the cap only when it
 * wins by more than ECG_TUNE_MARGIN.  Results never depend on the choice
 * (tests/test_gpu_tuning.py); only launch geometry does.
 *
 * Not tuned: launches with an explicit ecg_set_wg_per_cu, grids of <= 2048
 * blocks (latency-bound), k <= 4 (every cap loses, profiles/r02/wg_cap),
 * streams under graph capture, and contexts with tuning off
 * (ecg_set_autotune(ctx, 0) or ECG_AUTOTUNE=0 in the environment).
 *
 * Shapes are keyed coarsely (round 4): by (k, rows,
 * acc, diff, cell bytes, lane granule, layout class) where the layout class
 * is "interleaved" (source and destination share one stripe stride: in-place
 * recovery, the recovery-layout encode), "separate" (the client write
 * layout) or "pointer table" (ecg_matmul_ptrs / recx_encode launches of the
 * pointer-table kernel, which come in through ecg_tune_launch_fn with their
 * own launcher).  The batch size is not part of the key: callers whose batches
 * vary (queue flushes, the last batch of a rebuild, per-shard counts) share
 * one decision, and the arms compare the median time PER BLOCK, so a probe
 * stays valid when batch sizes change under it.  A probe runs on the stream
 * of the launch that started it (launches of the shape on other streams run
 * uncapped meanwhile), every event of both arms must have completed with a
 * valid time before a decision (an invalid one restarts the probe, at most
 * twice), and a context starts at most ECG_TUNE_MAX_CYCLES probes.
 */
#include <stdlib.h>
#include <string.h>

#include "ecg_internal.h"

#define ECG_TUNE_W0 1		/* untimed launches at the start of the uncapped arm */
/* ... and of the capped arm: the first ~10-20 launches after a switch to a
 * capped geometry run up to 12 % slow (EC_16P2 at 2 blocks per CU: 0.434 ms,
 * then 0.38, profiles/r03/tuner_check/) -- timing them rejected caps that win
 * in the steady state.  Switching back to uncapped shows no such transient,
 * and a kept cap needs no switch at all. */
#define ECG_TUNE_W1 16
#define ECG_TUNE_T 3		/* timed launches per arm (median) */
#define ECG_TUNE_ARM0 (ECG_TUNE_W0 + ECG_TUNE_T)
#define ECG_TUNE_PROBE (ECG_TUNE_ARM0 + ECG_TUNE_W1 + ECG_TUNE_T)
#define ECG_TUNE_MARGIN 0.015	/* the cap must win by more than 1.5 % */
#define ECG_TUNE_MAX_CYCLES 64	/* probe cycles per context */
#define ECG_TUNE_RESTARTS 2	/* probes restarted after invalid timings */
/* launches of a probing shape from other streams, with the probe's own stream
 * silent meanwhile, after which the probe moves to the stream asking: the
 * stream that started it went idle (its thread exited, its stream was
 * destroyed -- whose handle may even be reused by an unrelated stream) */
#define ECG_TUNE_STALL 64

struct ecg_tune_ent {
	int valid, decided, events, restarts;
	uint32_t k, rows, acc, diff, g, layout;
	uint64_t C;
	hipStream_t stream;	/* the probe's stream */
	uint32_t cand;		/* candidate cap */
	uint32_t choice;	/* decided: the cap, or ECG_WG_UNCAPPED */
	uint32_t n;		/* probing launches so far */
	uint32_t stall;		/* foreign launches since the probe last advanced */
	uint32_t handovers;	/* times the probe moved to another stream */
	uint64_t stamp;
	hipEvent_t ev[2][ECG_TUNE_T][2];
	uint64_t blocks[2][ECG_TUNE_T];	/* blocks of each timed launch */
	float msb[2];		/* decided: median ms per block of each arm */
};

struct ecg_tuner {
	pthread_mutex_t lock;
	int enabled;		/* -1 = not yet read from the environment */
	uint64_t clock;
	uint64_t cycles;	/* probe cycles started */
	uint64_t probe_launches;	/* launches that ran as part of a probe */
	struct ecg_tune_ent ent[ECG_NTUNE];
};

static uint64_t mm_blocks(const ecg_mm_params_t *p)
{
	return ((p->cell_bytes + 4095) / 4096) * (uint64_t)p->nstripes;
}

static uint32_t candidate_cap(const ecg_mm_params_t *p)
{
	if (mm_blocks(p) <= 2048 || p->rows == 0)
		return 0;
	if (p->k >= 16)
		return 2;	/* profiles/r02/wg_cap: k = 16 best at 2 blocks per CU */
	/* k = 8: since its product kernel loads in two phases (round 4) every
	 * cap loses -- 3 blocks per CU +7-10 % (profiles/r04/ec_ab/) */
	return 0;
}

static uint32_t layout_class(const ecg_mm_params_t *p)
{
	return p->src_stripe_stride == p->dst_stripe_stride ? ECG_TUNE_LAYOUT_INTERLEAVED : ECG_TUNE_LAYOUT_SEPARATE;
}

int ecg_tune_init(ecg_ctx_t *ctx)
{
	struct ecg_tuner *t = calloc(1, sizeof(*t));

	if (t == NULL)
		return ecg_fail(-ECG_DER_NOMEM, "tune_init: calloc");
	pthread_mutex_init(&t->lock, NULL);
	t->enabled = -1;
	ctx->tuner = t;
	return 0;
}

static void ent_free(struct ecg_tune_ent *e)
{
	int a, i, j;

	if (e->events)
		for (a = 0; a < 2; a++)
			for (i = 0; i < ECG_TUNE_T; i++)
				for (j = 0; j < 2; j++)
					(void)hipEventDestroy(e->ev[a][i][j]);
	memset(e, 0, sizeof(*e));
}

void ecg_tune_fini(ecg_ctx_t *ctx)
{
	struct ecg_tuner *t = ctx->tuner;
	int i;

	if (t == NULL)
		return;
	for (i = 0; i < ECG_NTUNE; i++)
		ent_free(&t->ent[i]);
	pthread_mutex_destroy(&t->lock);
	free(t);
	ctx->tuner = NULL;
}

static int enabled(struct ecg_tuner *t)
{
	if (t->enabled < 0) {
		const char *s = getenv("ECG_AUTOTUNE");

		t->enabled = !(s && s[0] == '0');
	}
	return t->enabled;
}

int ecg_set_autotune(ecg_ctx_t *ctx, int on)
{
	struct ecg_tuner *t;
	int i;

	if (ctx == NULL || ctx->tuner == NULL)
		return ecg_fail(-ECG_DER_INVAL, "set_autotune: NULL context");
	t = ctx->tuner;
	pthread_mutex_lock(&t->lock);
	t->enabled = on ? 1 : 0;
	if (on < 0 || on > 1) {		/* 2: forget every decision, tuning on */
		for (i = 0; i < ECG_NTUNE; i++)
			ent_free(&t->ent[i]);
		t->cycles = t->probe_launches = 0;
		t->enabled = 1;
	}
	pthread_mutex_unlock(&t->lock);
	return 0;
}

static int same_shape(const struct ecg_tune_ent *e, const ecg_mm_params_t *p, uint32_t g, uint32_t layout)
{
	return e->valid && e->k == p->k && e->rows == p->rows && e->acc == p->accumulate && e->diff == p->diff &&
	       e->C == p->cell_bytes && e->layout == layout && (g == 0 || e->g == g);
}

/* g = 0 matches any lane granule (ecg_tune_state) */
static struct ecg_tune_ent *lookup(struct ecg_tuner *t, const ecg_mm_params_t *p, uint32_t g, uint32_t layout,
				   int create)
{
	struct ecg_tune_ent *old = NULL;
	int i;

	for (i = 0; i < ECG_NTUNE; i++) {
		if (same_shape(&t->ent[i], p, g, layout)) {
			t->ent[i].stamp = ++t->clock;
			return &t->ent[i];
		}
	}
	if (!create || t->cycles >= ECG_TUNE_MAX_CYCLES)
		return NULL;
	/* a free slot, else the least recently used decided shape, else the
	 * least recently used probing one */
	for (i = 0; i < ECG_NTUNE; i++) {
		struct ecg_tune_ent *e = &t->ent[i];

		if (!e->valid) {
			old = e;
			break;
		}
		if (old == NULL || (e->decided && !old->decided) ||
		    (e->decided == old->decided && e->stamp < old->stamp))
			old = e;
	}
	ent_free(old);
	old->valid = 1;
	old->k = p->k;
	old->rows = p->rows;
	old->acc = p->accumulate;
	old->diff = p->diff;
	old->C = p->cell_bytes;
	old->g = g;
	old->layout = layout;
	old->stamp = ++t->clock;
	t->cycles++;
	return old;
}

static float median3(float a, float b, float c)
{
	if (a > b) { float x = a; a = b; b = x; }
	if (b > c) { float x = b; b = c; c = x; }
	return a > b ? a : b;
}

/* every timed event of both arms complete: decide (returns 1); a timing
 * that cannot be read restarts the probe (returns -1, at most
 * ECG_TUNE_RESTARTS times, then uncapped); 0 while events are pending. */
static int try_decide(struct ecg_tune_ent *e)
{
	float per[2][ECG_TUNE_T], ms;
	int a, i, bad = 0;

	for (a = 0; a < 2; a++)
		for (i = 0; i < ECG_TUNE_T; i++)
			if (hipEventQuery(e->ev[a][i][1]) != hipSuccess)
				return 0;
	for (a = 0; a < 2; a++)
		for (i = 0; i < ECG_TUNE_T; i++) {
			if (hipEventElapsedTime(&ms, e->ev[a][i][0], e->ev[a][i][1]) != hipSuccess || !(ms > 0.0f) ||
			    e->blocks[a][i] == 0)
				bad = 1;
			else
				per[a][i] = ms / (float)e->blocks[a][i];
		}
	if (bad) {
		if (e->restarts++ < ECG_TUNE_RESTARTS) {
			e->n = 0;
			return -1;
		}
		e->decided = 1;
		e->choice = ECG_WG_UNCAPPED;
		e->msb[0] = e->msb[1] = 0.0f;
		return 1;
	}
	for (a = 0; a < 2; a++)
		e->msb[a] = median3(per[a][0], per[a][1], per[a][2]);
	e->decided = 1;
	e->choice = ECG_WG_UNCAPPED;
	if (e->msb[1] < e->msb[0] * (1.0f - (float)ECG_TUNE_MARGIN))
		e->choice = e->cand;
	return 1;
}

static int make_events(struct ecg_tune_ent *e)
{
	int a, i, j;

	for (a = 0; a < 2; a++)
		for (i = 0; i < ECG_TUNE_T; i++)
			for (j = 0; j < 2; j++)
				if (hipEventCreate(&e->ev[a][i][j]) != hipSuccess) {
					/* destroy what was made; the shape stays untuned */
					int n = (a * ECG_TUNE_T + i) * 2 + j, m;

					for (m = 0; m < n; m++)
						(void)hipEventDestroy(e->ev[m / (2 * ECG_TUNE_T)][(m / 2) % ECG_TUNE_T][m % 2]);
					return -1;
				}
	e->events = 1;
	return 0;
}

static int launch_offsets(const ecg_mm_params_t *p, const ecg_launch_cfg_t *cfg, void *stream, uint32_t *kid,
			  const void *arg)
{
	(void)arg;
	return ecg_k_launch_matmul(p, cfg, stream, kid);
}

int ecg_tune_launch(ecg_ctx_t *ctx, const ecg_mm_params_t *p, hipStream_t st, uint32_t *kid)
{
	return ecg_tune_launch_fn(ctx, p, ecg_k_align_granule(p), layout_class(p), launch_offsets, NULL, st, kid);
}

int ecg_tune_launch_fn(ecg_ctx_t *ctx, const ecg_mm_params_t *p, uint32_t g, uint32_t layout,
		       ecg_mm_launch_fn fn, const void *arg, hipStream_t st, uint32_t *kid)
{
	struct ecg_tuner *t = ctx->tuner;
	ecg_launch_cfg_t cfg = ctx->cfg;
	struct ecg_tune_ent *e;
	hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
	uint32_t cand;
	int arm, idx, timed = 0, rc;

	cand = candidate_cap(p);
	if (t == NULL || cand == 0 || cfg.wg_per_cu != 0 || cfg.variant != 0 || cfg.order != 0 ||
	    cfg.grid_x != 0 || cfg.grid_y != 0)
		return fn(p, &ctx->cfg, (void *)st, kid, arg);
	if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone)
		return fn(p, &ctx->cfg, (void *)st, kid, arg);

	pthread_mutex_lock(&t->lock);
	if (!enabled(t)) {
		pthread_mutex_unlock(&t->lock);
		return fn(p, &ctx->cfg, (void *)st, kid, arg);
	}
	e = lookup(t, p, g, layout, 1);
	if (e == NULL) {		/* probe budget spent: untuned shapes run uncapped */
		cfg.wg_per_cu = ECG_WG_UNCAPPED;
		pthread_mutex_unlock(&t->lock);
		return fn(p, &cfg, (void *)st, kid, arg);
	}
	if (e->n == 0 && !e->decided) {
		e->stream = st;		/* the probe runs on the stream that starts it */
		e->cand = cand;
	}
	if (!e->decided && e->n >= ECG_TUNE_PROBE)
		(void)try_decide(e);
	if (e->decided) {
		cfg.wg_per_cu = e->choice;
		pthread_mutex_unlock(&t->lock);
		return fn(p, &cfg, (void *)st, kid, arg);
	}
	if (e->n < ECG_TUNE_PROBE && st != e->stream && ++e->stall >= ECG_TUNE_STALL) {
		/* the probe's stream went quiet: start over on this one (events of
		 * the old stream are re-recorded before they are read again) */
		e->stream = st;
		e->n = 0;
		e->stall = 0;
		e->handovers++;
	}
	if (e->n >= ECG_TUNE_PROBE || st != e->stream) {
		/* timings still in flight, or another stream: run uncapped */
		cfg.wg_per_cu = ECG_WG_UNCAPPED;
		pthread_mutex_unlock(&t->lock);
		return fn(p, &cfg, (void *)st, kid, arg);
	}
	if (!e->events && make_events(e)) {
		e->decided = 1;
		e->choice = ECG_WG_UNCAPPED;
		cfg.wg_per_cu = ECG_WG_UNCAPPED;
		pthread_mutex_unlock(&t->lock);
		return fn(p, &cfg, (void *)st, kid, arg);
	}
	/* probing: arm 0 uncapped, arm 1 capped, each W untimed + T timed, back
	 * to back; the lock is held across the timed launch so concurrent callers
	 * of the shape cannot interleave inside an event pair */
	e->stall = 0;
	arm = e->n < ECG_TUNE_ARM0 ? 0 : 1;
	idx = arm ? (int)(e->n - ECG_TUNE_ARM0) - ECG_TUNE_W1 : (int)e->n - ECG_TUNE_W0;
	e->n++;
	t->probe_launches++;
	cfg.wg_per_cu = arm ? e->cand : ECG_WG_UNCAPPED;
	if (idx >= 0) {
		timed = hipEventRecord(e->ev[arm][idx][0], st) == hipSuccess;
		e->blocks[arm][idx] = mm_blocks(p);
	}
	rc = fn(p, &cfg, (void *)st, kid, arg);
	if (timed && (rc != 0 || hipEventRecord(e->ev[arm][idx][1], st) != hipSuccess)) {
		e->decided = 1;		/* give up on this shape: uncapped */
		e->choice = ECG_WG_UNCAPPED;
	}
	pthread_mutex_unlock(&t->lock);
	return rc;
}

int ecg_tune_state(ecg_ctx_t *ctx, int k, int rows, uint64_t cell_bytes, uint32_t nstripes, int64_t sstride,
		   int64_t dstride, uint32_t *cap, float *ms_uncapped, float *ms_capped)
{
	struct ecg_tuner *t;
	struct ecg_tune_ent *e;
	ecg_mm_params_t *p;
	int rc;

	if (ctx == NULL || ctx->tuner == NULL)
		return ecg_fail(-ECG_DER_INVAL, "tune_state: NULL context");
	t = ctx->tuner;
	p = calloc(1, sizeof(*p));
	if (p == NULL)
		return ecg_fail(-ECG_DER_NOMEM, "tune_state: calloc");
	p->k = (uint32_t)k;
	p->rows = (uint32_t)rows;
	p->cell_bytes = cell_bytes;
	p->nstripes = nstripes;
	p->src_stripe_stride = sstride;
	p->dst_stripe_stride = dstride;
	pthread_mutex_lock(&t->lock);
	e = lookup(t, p, 0, layout_class(p), 0);
	if (e && !e->decided && e->n >= ECG_TUNE_PROBE)
		(void)try_decide(e);
	rc = e && e->decided ? 1 : 0;
	if (cap)
		*cap = e && e->decided ? e->choice : 0;
	/* the arms' medians per block, scaled to a launch of nstripes */
	if (ms_uncapped)
		*ms_uncapped = e && e->decided ? e->msb[0] * (float)mm_blocks(p) : 0.0f;
	if (ms_capped)
		*ms_capped = e && e->decided ? e->msb[1] * (float)mm_blocks(p) : 0.0f;
	pthread_mutex_unlock(&t->lock);
	free(p);
	return rc;
}

int ecg_tune_counters(ecg_ctx_t *ctx, uint64_t *probe_cycles, uint64_t *probe_launches, uint32_t *shapes)
{
	struct ecg_tuner *t;
	uint32_t n = 0;
	int i;

	if (ctx == NULL || ctx->tuner == NULL)
		return ecg_fail(-ECG_DER_INVAL, "tune_counters: NULL context");
	t = ctx->tuner;
	pthread_mutex_lock(&t->lock);
	for (i = 0; i < ECG_NTUNE; i++)
		n += t->ent[i].valid != 0;
	if (probe_cycles)
		*probe_cycles = t->cycles;
	if (probe_launches)
		*probe_launches = t->probe_launches;
	if (shapes)
		*shapes = n;
	pthread_mutex_unlock(&t->lock);
	return 0;
}
