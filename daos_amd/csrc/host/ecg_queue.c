/*
 * ecg_queue.c -- batching facade: one-stripe requests from many threads ->
 * batched device launches (see include/ecg.h, "batching facade").
 *
 * Why: every DAOS caller hands the codec one stripe at a time (SURVEY §0.6;
 * ref:src/object/cli_ec.c:627-659, ref:src/object/srv_obj_migrate.c:1116-1177,
 * ref:src/object/srv_ec_aggregate.c:701-734), and a single-stripe GPU call is
 * launch- and PCIe-latency bound.  The queue turns N concurrent
 * one-stripe calls into one device product over N stripes.
 *
 * Structure: nslot pinned staging slots, each owned by one request class
 * (op, k, p, cell size, erasure set) while it fills:
 *   FREE -> FILLING -> READY -> INFLIGHT -> DONE -> FREE
 * A submitter reserves a stripe index in a FILLING slot of its class (or
 * opens a FREE slot), copies its input cells into the slot's pinned staging
 * itself -- so gathers run in parallel on the callers' threads -- and
 * returns.  The worker thread closes a slot when it is full or its oldest
 * request has waited max_wait_us (or a flush is pending), launches
 * H2D(inputs) -> kernel -> D2H(outputs) on the slot's own stream, and polls
 * in-flight slots; when one completes, NFIN completion threads scatter the
 * outputs to the requests' buffers and fire their callbacks.  Slots in
 * different states overlap: one fills while another's H2D, another's kernel
 * and another's D2H run.  Staging layout per slot: inputs [n][k][pitch], outputs
 * [n][rows][pitch] (pitch = cell size rounded to 64 B), so only inputs
 * cross H2D and only outputs cross D2H.
 *
 * Aggregation updates (ecg_queue_update: agg_update_parity's xor_gen +
 * ec_encode_data_update per cell, ref:src/object/srv_ec_aggregate.c:
 * 1086-1102) are a third class per (k, p, cell size): the submitter writes
 * diff = old ^ new into the staging (the xor_gen), the device computes the p
 * parity deltas coef[r][vec_i] * diff with the stripe's own column vec_i
 * (ecg_mm_sel_kernel), and the completion threads XOR the deltas into the
 * caller's parity cells -- parity never crosses PCIe in either direction.
 *
 * Slots are spread round-robin over the contexts of an ecg_multi_t
 * (ecg_queue_create_multi): each slot's staging, stream and launches live on
 * its own device.
 *
 * Device cells (an engine whose bio buffers live in HBM): requests whose cells
 * are memory of one of the queue's devices go to slots of that device that
 * hold no data at all -- only the stripes' cell pointers, ISA-L's data[] /
 * coding[] laid end to end -- and a batch is one pointer-table launch on the
 * cells in place (ecg_matmul_ptrs), no PCIe.  Updates batch the same way into
 * ecg_update_ptrs launches: requests naming the same parity cells (one
 * stripe's cells updated one by one) fold into one pass over that parity, and
 * requests whose parity bytes would meet inside one launch go to ordered
 * launches; the update batches of one device run in order on its one update
 * stream (q->ust), so two batches never read-modify-write one parity byte at
 * once.
 * Such a slot closes as soon as its device has no batch of this queue in
 * flight, so a lone request launches at once and requests arriving while a
 * batch runs form the next one.
 *
 * The worker enqueues a device batch's HIP work with the queue lock released
 * (S_LAUNCHING), so submitters and completion threads never wait out a launch.
 *
 * CPU route (cpuexec slots): host-cell requests go where the ISA-L drop-in
 * would send the same cells -- below its crossover (with a GFNI CPU, every
 * size) the slot, like a device-cell one, holds only the cell addresses, a
 * closed slot goes straight to DONE and the completion threads (one per CPU,
 * 4..16) compute each request in place with ecg_cpu_matmul; above it the
 * staged path above.  Such a slot closes early while a completion thread is
 * free if it is the queue's only work or holds a request per free thread.
 * The CPU executor (ecg_queue_create(NULL, ...), or $ECG_FORCE_CPU=1) is the
 * same with no device at all -- the engine's DSS_XS_OFFLOAD ULT +
 * ABT_eventual pattern this facade replaces
 * (ref:src/object/srv_ec_aggregate.c:701-734, ref:src/engine/ult.c:394-470).
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/prctl.h>
#include <time.h>

#include "../../../include/ecg_multi.h"
#include "ecg_internal.h"

#define OP_ENCODE 0
#define OP_RECOVER 1
#define OP_UPDATE 2
#define NSLOT_MIN 4	/* staging slots for one device; 2 per device beyond */
#define NSLOT_MAX 32
#define NFIN 4		/* completion threads at least: output scatter, callbacks, */
#define NFIN_CPU 16	/* ... and CPU-route products: one per CPU, at most this many */
#define NDSTLOCK 64	/* striped locks serialising update deltas into one parity cell */
#define RES_OPEN (1ull << 31)
#define RES_CNT (RES_OPEN - 1)

/* S_LAUNCHING: the worker is enqueuing the batch's work with the queue lock
 * released (only the worker moves a slot out of it). */
enum slot_state { S_FREE, S_FILLING, S_READY, S_LAUNCHING, S_INFLIGHT, S_DONE };

struct qreq {
	int op, k, p, nerrs;
	uint64_t C;
	unsigned char *dst[ECG_MAX_P];	/* where each output row goes (XORed in for updates) */
	ecg_done_cb_t cb;
	void *arg;
	int rc;				/* this request's own result (a batch split up) */
};

struct qslot {
	ecg_ctx_t *ctx;			/* device this slot's staging and launches live on (NULL: CPU) */
	int ui;				/* update stream of ctx's DEVICE: the first ctxs[] entry on
					 * that device (a multi-device queue may list a device twice) */
	enum slot_state state;
	/* class */
	int op, k, p, nerrs, rows;
	int devcells;			/* cells in device memory of ctx's device: tab, no staging */
	int cpuexec;			/* host cells computed on the completion threads (the CPU
					 * executor, or a device queue's host cells below the
					 * drop-in crossover): tab, no staging */
	uint64_t C, pitch;
	uint32_t err[ECG_MAX_P];
	unsigned char coef[ECG_MAX_P * ECG_MAX_K];
	uint32_t dec_idx[ECG_MAX_K], out_idx[ECG_MAX_P];
	int nin;			/* input cells staged per request (k, or 1 for updates) */
	/* fill state */
	uint32_t cap;
	/* Reservations without the queue lock: res = generation << 32 | RES_OPEN
	 * | requests reserved, CAS-incremented by submitters while the slot is
	 * open (FILLING), its open bit cleared by the worker when it closes the
	 * slot -- which fixes `reserved`.  The generation changes at every
	 * slot_open, so a submitter that checked the class of an earlier
	 * opening cannot reserve in a reopened slot.  `filled` counts requests
	 * whose inputs are in (atomic). */
	uint64_t res;
	uint32_t reserved, filled;
	uint32_t fin_next, fin_done;	/* completion progress (S_DONE) */
	uint64_t t_open_ns;
	struct qreq *reqs;		/* cap entries */
	uint64_t *tab;			/* devcells: cap x (k + rows) cell addresses; updates
					 * cap x (2 + rows): old, new, parity cells */
	uint8_t *uvec;			/* devcells updates: vec_i per request */
	/* staging */
	unsigned char *host;		/* pinned: inputs [cap][k][pitch], (updates: vec_i [cap]),
					 * outputs [cap][rows][pitch] at out_off */
	size_t out_off;
	unsigned char *dev;
	size_t bytes;
	hipStream_t st;
	hipEvent_t done;
	int rc;
#ifdef ECG_QUEUE_TIMING
	uint64_t tm[4];			/* closed, launch start, launch end, completion seen */
#endif
};

struct ecg_queue {
	ecg_ctx_t *ctx;
	int cpu;			/* CPU executor: no device, host cells only */
	int nctx;
	ecg_ctx_t *ctxs[NSLOT_MAX];
	/* device-cell update batches of device ctxs[i] run in order on its one
	 * update stream */
	hipStream_t ust[NSLOT_MAX];
	ecg_queue_attr_t attr;
	size_t slot_bytes;
	pthread_mutex_t lock;
	pthread_cond_t cv_work;		/* worker wakeups */
	pthread_cond_t cv_slot;		/* a slot became FREE or gained room */
	pthread_cond_t cv_done;		/* completions (flush) */
	pthread_cond_t cv_fin;		/* a slot reached S_DONE */
	int nslot;
	uint32_t open_next;		/* where the next FREE-slot search starts */
	struct qslot slot[NSLOT_MAX];
	uint64_t submitted, completed, batches, flush_target;
	int stop, worker_exited;
	pthread_t worker;
	pthread_t fin[NFIN_CPU];
	int nfin;
	int fin_busy;			/* requests the completion threads hold (lock) */
	/* Updates of one stripe submitted back to back (one per updated cell, all
	 * naming the same parity cells) land in one batch or in batches of
	 * different devices, and their completions run on different threads:
	 * the read-modify-write parity ^= delta of two of them must not
	 * interleave.  A lock striped on the destination address serialises
	 * exactly those (XOR commutes, so their order does not matter). */
	pthread_mutex_t dst_lock[NDSTLOCK];
#ifdef ECG_QUEUE_TIMING
	uint64_t tm_sum[5], tm_n;	/* per-batch phase times (ns), requests */
	uint64_t tm_cpu;		/* the worker's thread CPU time inside launches */
#endif
};

/* Diagnostic build only (make EXP_CFLAGS=-DECG_QUEUE_TIMING): where a batch's
 * time goes -- closed -> launch start (inputs landing, worker wake-up),
 * launch (host side), in flight (GPU + completion poll), completion (callbacks,
 * slot freed) -- printed when the queue is destroyed. */
#ifdef ECG_QUEUE_TIMING
#define QT(x) x
#else
#define QT(x)
#endif

/* Cell addresses per request in s->tab (device-cell slots and the CPU
 * executor): k + rows (encode, recovery), or old, new and the rows parity
 * cells (updates). */
static uint32_t qtab_width(const struct qslot *s)
{
	return s->op == OP_UPDATE ? 2u + (uint32_t)s->rows : (uint32_t)(s->k + s->rows);
}

static uint64_t now_ns(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

#ifdef ECG_QUEUE_TIMING
static uint64_t cpu_ns(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

static void queue_timing_add(struct ecg_queue *q, const struct qslot *s)
{
	const uint64_t t = now_ns();

	q->tm_sum[0] += s->tm[1] - s->tm[0];
	q->tm_sum[1] += s->tm[2] - s->tm[1];
	q->tm_sum[2] += s->tm[3] - s->tm[2];
	q->tm_sum[3] += t - s->tm[3];
	q->tm_sum[4] += s->reserved;
	q->tm_n++;
}
#endif

static void abs_deadline(struct timespec *ts, uint64_t wait_ns)
{
	clock_gettime(CLOCK_REALTIME, ts);
	ts->tv_sec += (time_t)(wait_ns / 1000000000ull);
	ts->tv_nsec += (long)(wait_ns % 1000000000ull);
	if (ts->tv_nsec >= 1000000000L) {
		ts->tv_sec++;
		ts->tv_nsec -= 1000000000L;
	}
}

static uint64_t pitch_of(uint64_t C)
{
	return (C + 63) & ~63ull;
}

/* The slot's class is the request's.  dev: the cells' device (device-cell
 * requests), -1 for host cells.  Read without the lock by the reservation
 * fast path: a slot reopened meanwhile fails that path's CAS (generation). */
#define LD(x) __atomic_load_n(&(x), __ATOMIC_RELAXED)
#define ST(x, v) __atomic_store_n(&(x), (v), __ATOMIC_RELAXED)

static int class_matches(const struct qslot *s, int op, int k, int p, uint64_t C,
			 const uint32_t *err, int nerrs, int dev, int cpuexec)
{
	if (LD(s->op) != op || LD(s->k) != k || LD(s->p) != p || LD(s->C) != C || LD(s->nerrs) != nerrs ||
	    LD(s->devcells) != (dev >= 0) || LD(s->cpuexec) != cpuexec || (dev >= 0 && s->ctx->device != dev))
		return 0;
	for (int i = 0; op == OP_RECOVER && i < nerrs; i++)
		if (LD(s->err[i]) != err[i])
			return 0;
	return 1;
}

/* Reserve a request index in an open slot of this class; 0 if it is not
 * open, not this class or full. */
static int slot_try_reserve(struct qslot *s, int op, int k, int p, uint64_t C, const uint32_t *err,
			    int nerrs, int dev, int cpuexec, uint32_t *idx)
{
	uint64_t w = __atomic_load_n(&s->res, __ATOMIC_ACQUIRE);
	const uint64_t gen = w >> 32;

	if (!(w & RES_OPEN) || !class_matches(s, op, k, p, C, err, nerrs, dev, cpuexec))
		return 0;
	/* the class was checked for this opening (generation) only */
	while ((w >> 32) == gen && (w & RES_OPEN) && (uint32_t)(w & RES_CNT) < LD(s->cap)) {
		if (__atomic_compare_exchange_n(&s->res, &w, w + 1, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
			*idx = (uint32_t)(w & RES_CNT);
			return 1;
		}
	}
	return 0;
}

static uint32_t res_count(const struct qslot *s)
{
	return (uint32_t)(__atomic_load_n(&s->res, __ATOMIC_ACQUIRE) & RES_CNT);
}

/* FILLING -> READY (lock held): no reservation after this one. */
static void slot_close(struct qslot *s)
{
	const uint64_t w = __atomic_fetch_and(&s->res, ~RES_OPEN, __ATOMIC_SEQ_CST);

	s->reserved = (uint32_t)(w & RES_CNT);
	s->state = S_READY;
	QT(s->tm[0] = now_ns());
}

/* Assign a FREE slot to a class: decode rows for recovery, capacity from the
 * slot's staging bytes. */
static int slot_open(struct ecg_queue *q, struct qslot *s, int op, int k, int p, uint64_t C,
		     const uint32_t *err, int nerrs, int dev, int cpuexec)
{
	unsigned char en[(ECG_MAX_K + ECG_MAX_P) * ECG_MAX_K];
	uint64_t per;
	int j, reused, rc;

	/* the class fields are read without the lock by slot_try_reserve
	 * (relaxed atomics; the generation in `res` decides) */
	ST(s->op, op);
	ST(s->k, k);
	ST(s->p, p);
	ST(s->C, C);
	s->pitch = pitch_of(C);
	ST(s->nerrs, nerrs);
	ecg_gen_cauchy1(k, p, en);
	if (op == OP_ENCODE || op == OP_UPDATE) {
		s->rows = p;
		memcpy(s->coef, &en[k * k], (size_t)p * k);
		for (j = 0; j < k; j++)
			s->dec_idx[j] = (uint32_t)j;
		for (j = 0; j < p; j++)
			s->out_idx[j] = (uint32_t)(k + j);
	} else {
		for (j = 0; j < nerrs; j++)
			ST(s->err[j], err[j]);
		rc = ecg_recov_rows(k, p, en, err, nerrs, s->coef, s->out_idx, s->dec_idx, &reused);
		if (rc)
			return rc;
		s->rows = nerrs;
	}
	s->nin = op == OP_UPDATE ? 1 : k;	/* staged input cells per request */
	ST(s->devcells, dev >= 0);
	ST(s->cpuexec, cpuexec);
	/* an update request also stages its vec_i byte (+64 B of alignment slack) */
	per = s->pitch * (uint64_t)(s->nin + s->rows) + (op == OP_UPDATE ? 1 : 0);
	/* device cells stage nothing: only the pointer table bounds a batch */
	{
		uint32_t cap = dev >= 0 || cpuexec ? q->attr.max_batch : (uint32_t)((q->slot_bytes - 64) / per);

		ST(s->cap, cap > q->attr.max_batch ? q->attr.max_batch : cap);
	}
	if (s->cap == 0)
		return ecg_fail(-ECG_DER_REC2BIG, "queue: one stripe (%llu B) exceeds a slot",
				(unsigned long long)per);
	s->out_off = (size_t)s->pitch * s->nin * s->cap;
	if (op == OP_UPDATE)
		s->out_off += ((size_t)s->cap + 63) & ~(size_t)63;
	s->reserved = 0;
	__atomic_store_n(&s->filled, 0u, __ATOMIC_RELAXED);
	s->rc = 0;
	s->t_open_ns = now_ns();
	s->state = S_FILLING;
	/* the class above is published with the open bit.  `res` is read
	 * atomically: a submitter that loaded the last generation's word may
	 * still be running its (failing) compare-exchange on it -- the C driver's
	 * ThreadSanitizer run flagged the plain read here */
	__atomic_store_n(&s->res, ((__atomic_load_n(&s->res, __ATOMIC_RELAXED) >> 32) + 1) << 32 | RES_OPEN,
			 __ATOMIC_RELEASE);
	return 0;
}

/* Device-cell batches of this queue queued or running on one device at once:
 * a second one hides the first's completion poll and the next launch
 * (profiles/r05/queue_dev/). */
/* How often the worker polls batches in flight on a device (ns). */
#ifndef ECG_QUEUE_POLL_NS
#define ECG_QUEUE_POLL_NS 20000ull
#endif

#ifndef ECG_QUEUE_DEV_DEPTH
#define ECG_QUEUE_DEV_DEPTH 2
#endif

/* ctx's device has ECG_QUEUE_DEV_DEPTH device-cell batches of this queue
 * queued or running (host-cell batches, PCIe-bound, do not count). */
static int device_busy(const struct ecg_queue *q, const ecg_ctx_t *ctx)
{
	int n = 0;

	for (int i = 0; i < q->nslot; i++) {
		const struct qslot *s = &q->slot[i];

		if (s->ctx == ctx && s->devcells &&
		    (s->state == S_INFLIGHT || s->state == S_READY || s->state == S_LAUNCHING))
			n++;
	}
	return n >= ECG_QUEUE_DEV_DEPTH;
}

/* Close a CPU-route batch now?  Only while a completion thread is free (no
 * request of a DONE slot waits to be claimed and fewer are held than there
 * are threads), and then when the batch is the queue's only work -- a lone
 * request does not wait max_wait_us for company -- or holds at least one
 * request per free thread.  Closing every request alone instead would tie up
 * the few slots with one request each (lock held). */
static int cpu_close_now(const struct ecg_queue *q, const struct qslot *self, uint32_t n)
{
	int free = q->nfin - q->fin_busy, alone = 1;

	for (int i = 0; i < q->nslot; i++) {
		const struct qslot *o = &q->slot[i];

		if (o->state == S_DONE)
			free -= (int)(o->reserved - o->fin_next);
		if (o != self && o->state != S_FREE && !(o->state == S_FILLING && res_count(o) == 0))
			alone = 0;
	}
	return free > 0 && (alone || n >= (uint32_t)free);
}

static void close_due_slots(struct ecg_queue *q, uint64_t t, int force)
{
	for (int i = 0; i < q->nslot; i++) {
		struct qslot *s = &q->slot[i];

		uint32_t n;

		if (s->state != S_FILLING || (n = res_count(s)) == 0)
			continue;
		if (force || n >= s->cap || t >= s->t_open_ns + (uint64_t)q->attr.max_wait_us * 1000ull ||
		    (s->devcells && !device_busy(q, s->ctx)) || (s->cpuexec && cpu_close_now(q, s, n)))
			slot_close(s);
	}
}

/* READY and fully copied in: launch H2D -> product -> D2H.  The CPU
 * executor's slots go straight to DONE (lock held); a device slot is
 * S_LAUNCHING and the lock is NOT held -- the HIP calls enqueuing its work
 * take tens of microseconds, which submitters and completion threads need
 * not wait out -- and the worker marks it INFLIGHT afterwards. */
static void launch_slot(struct ecg_queue *q, struct qslot *s)
{
	const uint32_t n = s->reserved;
	const uint64_t in_stride = s->pitch * (uint64_t)s->nin;
	const uint64_t out_stride = s->pitch * (uint64_t)s->rows;
	const size_t sel_off = (size_t)in_stride * s->cap;	/* updates: vec_i bytes */
	unsigned char *dout = s->dev + s->out_off;
	int64_t soff[ECG_MAX_K], doff[ECG_MAX_P];
	hipError_t e;
	int j, rc;

	if (s->cpuexec) {
		/* the completion threads compute each request from its cells
		 * (finish_req) */
		s->rc = 0;
		s->fin_next = 0;
		s->fin_done = 0;
		s->state = S_DONE;
		QT(s->tm[3] = now_ns());
		q->batches++;
		pthread_cond_broadcast(&q->cv_fin);
		return;
	}
	ecg_trace_push("ecg:queue_batch");
	e = hipSetDevice(s->ctx->device);
	if (s->devcells) {
		/* the cells in place: one pointer-table launch (its table upload
		 * and kernel on the slot's stream), nothing crosses back */
		/* updates run on the device's one update stream, after the previous
		 * update batch: one parity cell's read-modify-writes never overlap
		 * across batches */
		hipStream_t st = s->op == OP_UPDATE ? q->ust[s->ui] : s->st;

		rc = e == hipSuccess ? 0 : ecg_hip_fail(e, "queue set device");
		if (rc == 0 && s->op == OP_UPDATE) {
			rc = ecg_update_ptrs_coef(s->ctx, s->k, s->rows, s->coef, s->C, n, (void *const *)s->tab,
						  s->uvec, st, NULL);
			/* refused as a batch (some request's old / new cell overlaps a
			 * parity cell of the batch): the requests one after another on
			 * the update stream, each with its own result -- the order
			 * they would have run in one by one */
			for (uint32_t i = 0; rc == -ECG_DER_INVAL && n > 1 && i < n; i++)
				s->reqs[i].rc = ecg_update_ptrs_coef(s->ctx, s->k, s->rows, s->coef, s->C, 1,
								     (void *const *)s->tab + (size_t)i * (2 + s->rows),
								     &s->uvec[i], st, NULL);
			if (rc == -ECG_DER_INVAL && n > 1)
				rc = 0;
		} else if (rc == 0)
			rc = ecg_matmul_ptrs(s->ctx, s->k, s->rows, s->coef, s->C, n, (void *const *)s->tab, st);
		if (rc == 0) {
			e = hipEventRecord(s->done, st);
			if (e != hipSuccess)
				rc = ecg_hip_fail(e, "queue batch event");
		}
		if (rc == 0 && s->op == OP_UPDATE) {
			;	/* counted by ecg_update_ptrs_coef */
		} else if (rc == 0 && s->op == OP_ENCODE) {
			ECG_STAT_ADD(s->ctx, encode_stripes, n);
			ECG_STAT_ADD(s->ctx, encode_bytes, (uint64_t)s->k * s->C * n);
		} else if (rc == 0) {
			ECG_STAT_ADD(s->ctx, recover_stripes, n);
			ECG_STAT_ADD(s->ctx, recover_bytes, (uint64_t)s->rows * s->C * n);
		}
		s->rc = rc;
		ecg_trace_pop();
		return;
	}
	for (j = 0; j < s->k; j++)
		soff[j] = (int64_t)(j * s->pitch);
	for (j = 0; j < s->rows; j++)
		doff[j] = (int64_t)(j * s->pitch);
	if (e == hipSuccess)
		e = ecg_stage_copy(s->dev, s->host, (size_t)in_stride * n, (size_t)s->pitch,
				   hipMemcpyHostToDevice, s->st);
	if (e == hipSuccess && s->op == OP_UPDATE)
		e = hipMemcpyAsync(s->dev + sel_off, s->host + sel_off, n, hipMemcpyHostToDevice, s->st);
	rc = e == hipSuccess ? 0 : ecg_hip_fail(e, "queue H2D");
	if (rc == 0 && s->op == OP_UPDATE)
		rc = ecg_matmul_sel(s->ctx, s->k, s->rows, s->coef, s->C, n, s->dev, (int64_t)in_stride,
				    s->dev + sel_off, dout, doff, (int64_t)out_stride, s->st);
	else if (rc == 0)
		rc = ecg_matmul(s->ctx, s->k, s->rows, s->coef, s->C, n, s->dev, soff, (int64_t)in_stride,
				dout, doff, (int64_t)out_stride, 0, s->st);
	if (rc == 0) {
		e = ecg_stage_copy(s->host + s->out_off, dout, (size_t)out_stride * n,
				   (size_t)s->pitch, hipMemcpyDeviceToHost, s->st);
		if (e == hipSuccess)
			e = hipEventRecord(s->done, s->st);
		if (e != hipSuccess)
			rc = ecg_hip_fail(e, "queue D2H");
	}
	if (rc == 0) {	/* the queue's work in the device's counters */
		ECG_STAT_ADD(s->ctx, h2d_bytes, (uint64_t)s->nin * s->C * n);
		ECG_STAT_ADD(s->ctx, d2h_bytes, (uint64_t)s->rows * s->C * n);
		if (s->op == OP_ENCODE) {
			ECG_STAT_ADD(s->ctx, encode_stripes, n);
			ECG_STAT_ADD(s->ctx, encode_bytes, (uint64_t)s->k * s->C * n);
		} else if (s->op == OP_RECOVER) {
			ECG_STAT_ADD(s->ctx, recover_stripes, n);
			ECG_STAT_ADD(s->ctx, recover_bytes, (uint64_t)s->rows * s->C * n);
		} else {
			ECG_STAT_ADD(s->ctx, update_cells, n);
			ECG_STAT_ADD(s->ctx, update_bytes, (uint64_t)s->C * n);
		}
	}
	s->rc = rc;
	ecg_trace_pop();
}

/* One request's outputs back to its buffers, then its callback (lock NOT
 * held). */
/* dst ^= src (n bytes, any alignment) */
static void xor_into(unsigned char *dst, const unsigned char *a, const unsigned char *b, uint64_t n)
{
	uint64_t i = 0;

	for (; i + 8 <= n; i += 8) {
		uint64_t x, y;

		memcpy(&x, a + i, 8);
		memcpy(&y, b + i, 8);
		x ^= y;
		memcpy(dst + i, &x, 8);
	}
	for (; i < n; i++)
		dst[i] = a[i] ^ b[i];
}

/* Striped locks over the ADDRESS RANGE of a parity cell: the address space
 * is cut into 64 KiB regions, each region hashed to one of NDSTLOCK locks.
 * parity ^= delta runs region by region under that region's lock, so two
 * updates whose parity bytes overlap -- through the same cell pointer or
 * through different pointers into one buffer -- serialise on every region
 * they share (XOR commutes: the order does not matter, only that each
 * read-modify-write of a byte is whole).  One lock is held at a time: no
 * lock ordering to get wrong. */
#define DST_REGION_SHIFT 16

static pthread_mutex_t *region_lock(struct ecg_queue *q, uint64_t region)
{
	uint64_t a = region;

	a ^= a >> 17;
	a *= 0x9E3779B97F4A7C15ull;
	return &q->dst_lock[a >> 58];	/* top 6 bits: NDSTLOCK = 64 */
}

static void xor_into_locked(struct ecg_queue *q, unsigned char *dst, const unsigned char *delta, uint64_t n)
{
	uint64_t a = (uint64_t)(uintptr_t)dst;
	const uint64_t end = a + n;

	while (a < end) {
		uint64_t next = ((a >> DST_REGION_SHIFT) + 1) << DST_REGION_SHIFT;
		pthread_mutex_t *l = region_lock(q, a >> DST_REGION_SHIFT);
		unsigned char *d = (unsigned char *)(uintptr_t)a;

		if (next > end)
			next = end;
		pthread_mutex_lock(l);
		xor_into(d, d, delta + (a - (uint64_t)(uintptr_t)dst), next - a);
		pthread_mutex_unlock(l);
		a = next;
	}
}

/* A completion thread's scratch: the CPU executor's update deltas. */
struct fin_scratch {
	unsigned char *p;
	size_t n;
};

/* Columns per CPU-executor product: an update's deltas (rows x this) stay in
 * the thread's cache until XORed into the parity, and any cell size fits the
 * kernels' int length. */
#define CPU_CHUNK (256u << 10)

/* CPU executor: request i's product straight from the caller's cells (the
 * request holds only their addresses, s->tab, as the device-cell path does:
 * the callers keep them valid until the callback) -- encode and recovery into
 * the request's output cells, an update's p deltas coef[r][vec_i] * (old ^
 * new) into the thread's scratch, then XORed into the parity under the region
 * locks like the staged path's.  Returns 0 or a negative DER code. */
static int cpu_product(struct ecg_queue *q, struct qslot *s, uint32_t i, struct fin_scratch *fs)
{
	const uint64_t *t = s->tab + (size_t)i * (uint64_t)qtab_width(s);
	const int upd = s->op == OP_UPDATE, nin = upd ? 2 : s->k;
	unsigned char *src[ECG_MAX_K], *dst[ECG_MAX_P];
	unsigned char col[2 * ECG_MAX_P];
	const unsigned char *coef = s->coef;
	int rc = 0;

	if (upd) {
		const size_t need = (size_t)CPU_CHUNK * s->rows;

		if (fs->n < need) {
			unsigned char *np = realloc(fs->p, need);

			if (np == NULL)
				return ecg_fail(-ECG_DER_NOMEM, "queue: update scratch");
			fs->p = np;
			fs->n = need;
		}
		/* parity delta r = c * old ^ c * new, c = coef[r][vec_i]: one
		 * product of the two cells, no diff buffer */
		for (int r = 0; r < s->rows; r++)
			col[2 * r] = col[2 * r + 1] = s->coef[(size_t)r * s->k + s->uvec[i]];
		coef = col;
	}
	for (uint64_t off = 0; off < s->C && rc == 0; off += CPU_CHUNK) {
		const uint64_t n = s->C - off < CPU_CHUNK ? s->C - off : CPU_CHUNK;

		for (int j = 0; j < nin; j++)
			src[j] = (unsigned char *)(uintptr_t)t[j] + off;
		for (int r = 0; r < s->rows; r++)
			dst[r] = upd ? fs->p + (size_t)r * CPU_CHUNK : (unsigned char *)(uintptr_t)t[s->k + r] + off;
		rc = ecg_cpu_matmul((int)n, nin, s->rows, coef, src, dst, 0);
		for (int r = 0; upd && rc == 0 && r < s->rows; r++)
			xor_into_locked(q, (unsigned char *)(uintptr_t)t[2 + r] + off, dst[r], n);
	}
	return rc;
}

static void finish_req(struct ecg_queue *q, struct qslot *s, uint32_t i, struct fin_scratch *fs)
{
	struct qreq *r = &s->reqs[i];
	int rc = s->rc;

	ecg_trace_push("ecg:queue_complete");
	if (s->cpuexec) {
		rc = cpu_product(q, s, i, fs);
	} else if (s->devcells) {
		if (rc == 0)			/* written in place by the launch */
			rc = r->rc;
	} else if (s->rc == 0) {		/* the staged outputs of request i */
		const unsigned char *out = s->host + s->out_off + i * s->pitch * (uint64_t)s->rows;

		for (int j = 0; j < s->rows; j++) {
			if (s->op == OP_UPDATE)	/* parity ^= coef[r][vec_i] * diff */
				xor_into_locked(q, r->dst[j], out + j * s->pitch, s->C);
			else
				memcpy(r->dst[j], out + j * s->pitch, s->C);
		}
	}
	ecg_trace_pop();
	if (r->cb)
		r->cb(r->arg, rc);
}

/* Completion threads: claim requests of S_DONE slots -- one at a time for
 * host cells, so the host-side scatter of a batch runs on NFIN threads; a
 * whole batch at once for device cells, which have only callbacks to run --
 * and the last one frees the slot. */
static void *fin_main(void *argp)
{
	struct ecg_queue *q = argp;
	struct fin_scratch fs = {NULL, 0};

	pthread_mutex_lock(&q->lock);
	for (;;) {
		struct qslot *s = NULL;
		uint32_t i, n;

		for (int j = 0; j < q->nslot && s == NULL; j++)
			if (q->slot[j].state == S_DONE && q->slot[j].fin_next < q->slot[j].reserved)
				s = &q->slot[j];
		if (s == NULL) {
			if (q->stop && q->worker_exited)
				break;
			pthread_cond_wait(&q->cv_fin, &q->lock);
			continue;
		}
		i = s->fin_next;
		n = s->devcells ? s->reserved - i : 1;
		s->fin_next += n;
		q->fin_busy += (int)n;
		pthread_mutex_unlock(&q->lock);
		for (uint32_t x = 0; x < n; x++)
			finish_req(q, s, i + x, &fs);
		pthread_mutex_lock(&q->lock);
		q->fin_busy -= (int)n;
		for (int j = 0; s->cpuexec && j < q->nslot; j++)	/* a free thread: a waiting */
			if (q->slot[j].state == S_FILLING && q->slot[j].cpuexec &&	/* CPU batch may close */
			    res_count(&q->slot[j]) > 0) {
				pthread_cond_signal(&q->cv_work);
				break;
			}
		if ((s->fin_done += n) == s->reserved) {
			q->completed += s->reserved;
			QT(queue_timing_add(q, s));
			s->state = S_FREE;
			pthread_cond_broadcast(&q->cv_slot);
			pthread_cond_broadcast(&q->cv_done);
			pthread_cond_signal(&q->cv_work);
		}
	}
	pthread_mutex_unlock(&q->lock);
	free(fs.p);
	return NULL;
}

static void *worker_main(void *argp)
{
	struct ecg_queue *q = argp;

	/* the in-flight polls below wait 20 us: without this the kernel's
	 * default 50 us timer slack would stretch every one of them */
	(void)prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
	pthread_mutex_lock(&q->lock);
	for (;;) {
		int busy = 0, idle = 1;
		uint64_t t = now_ns(), next = UINT64_MAX;

		close_due_slots(q, t, q->stop || q->completed < q->flush_target);
		for (int i = 0; i < q->nslot; i++) {
			struct qslot *s = &q->slot[i];

			if (s->state == S_READY && __atomic_load_n(&s->filled, __ATOMIC_SEQ_CST) == s->reserved) {
				QT(s->tm[1] = now_ns());
				QT(q->tm_cpu -= cpu_ns());
				if (s->cpuexec) {
					launch_slot(q, s);
				} else {
					s->state = S_LAUNCHING;
					pthread_mutex_unlock(&q->lock);
					launch_slot(q, s);
					pthread_mutex_lock(&q->lock);
					s->state = S_INFLIGHT;
					q->batches++;
				}
				QT(q->tm_cpu += cpu_ns());
				QT(s->tm[2] = now_ns());
				idle = 0;
			}
		}
		for (int i = 0; i < q->nslot; i++) {
			struct qslot *s = &q->slot[i];

			if (s->state == S_INFLIGHT) {
				hipError_t e = hipEventQuery(s->done);

				if (e == hipErrorNotReady) {
					busy = 1;
					continue;
				}
				if (e != hipSuccess && s->rc == 0)
					s->rc = ecg_hip_fail(e, "queue batch");
				s->fin_next = 0;
				s->fin_done = 0;
				s->state = S_DONE;
				QT(s->tm[3] = now_ns());
				pthread_cond_broadcast(&q->cv_fin);
				idle = 0;
			} else if (s->state == S_FILLING && res_count(s) > 0) {
				uint64_t dl = s->t_open_ns + (uint64_t)q->attr.max_wait_us * 1000ull;

				if (dl < next)
					next = dl;
			} else if (s->state == S_READY) {
				busy = 1;	/* waiting for a submitter's copy to land */
			}
		}
		if (!idle)
			continue;
		if (q->stop) {
			int live = 0;

			for (int i = 0; i < q->nslot; i++)
				live += q->slot[i].state != S_FREE;
			if (!live)
				break;
		}
		{
			struct timespec ts;
			uint64_t wait = busy ? ECG_QUEUE_POLL_NS : 100000000ull;	/* poll in-flight work */

			if (next != UINT64_MAX)
				wait = next > t ? (next - t < wait ? next - t : wait) : 0;
			if (wait) {
				abs_deadline(&ts, wait);
				pthread_cond_timedwait(&q->cv_work, &q->lock, &ts);
			}
		}
	}
	q->worker_exited = 1;
	pthread_cond_broadcast(&q->cv_fin);
	pthread_mutex_unlock(&q->lock);
	return NULL;
}

static void slot_free(struct qslot *s)
{
	if (s->ctx == NULL) {		/* CPU executor: plain memory, nothing on a device */
		free(s->host);
		free(s->reqs);
		free(s->tab);
		free(s->uvec);
		return;
	}
	(void)hipSetDevice(s->ctx->device);
	if (s->host)
		(void)hipHostFree(s->host);
	if (s->dev)
		(void)hipFree(s->dev);
	if (s->st)
		(void)hipStreamDestroy(s->st);
	if (s->done)
		(void)hipEventDestroy(s->done);
	free(s->reqs);
	free(s->tab);
	free(s->uvec);
}

/* Completion threads of the CPU executor: they compute the products, so one
 * per CPU the process may run on, NFIN .. NFIN_CPU. */
static int cpu_workers(void)
{
	cpu_set_t set;
	int n = NFIN;

	if (sched_getaffinity(0, sizeof(set), &set) == 0)
		n = CPU_COUNT(&set);
	return n < NFIN ? NFIN : n > NFIN_CPU ? NFIN_CPU : n;
}

/* Slots round-robin over ctxs[nctx] (one context = one device); nctx = 0:
 * the CPU executor. */
static int queue_create(ecg_ctx_t *const *ctxs, int nctx, const ecg_queue_attr_t *attr,
			ecg_queue_t **out)
{
	struct ecg_queue *q;
	hipError_t e = hipSuccess;
	int i;

	q = calloc(1, sizeof(*q));
	if (q == NULL)
		return ecg_fail(-ECG_DER_NOMEM, "queue_create: calloc");
	q->cpu = nctx == 0;
	q->ctx = nctx ? ctxs[0] : NULL;
	q->nctx = nctx < NSLOT_MAX ? nctx : NSLOT_MAX;
	for (i = 0; i < q->nctx; i++)
		q->ctxs[i] = ctxs[i];
	q->nslot = nctx <= 1 ? NSLOT_MIN : 2 * nctx;
	if (q->nslot < NSLOT_MIN)
		q->nslot = NSLOT_MIN;
	if (q->nslot > NSLOT_MAX)
		q->nslot = NSLOT_MAX;
	if (attr)
		q->attr = *attr;
	if (q->attr.max_batch == 0)
		q->attr.max_batch = 256;
	if (q->attr.max_wait_us == 0)
		q->attr.max_wait_us = 50;
	if (q->attr.max_cell_bytes == 0)
		q->attr.max_cell_bytes = 1 << 20;
	/* a slot holds max_batch stripes of 8+2 cells of max_cell_bytes, capped
	 * at 128 MiB (bigger classes get proportionally fewer stripes) */
	q->slot_bytes = (size_t)pitch_of(q->attr.max_cell_bytes) * 10u * q->attr.max_batch;
	if (q->slot_bytes > (128u << 20))
		q->slot_bytes = 128u << 20;
	if (q->slot_bytes < (size_t)pitch_of(q->attr.max_cell_bytes) * (ECG_MAX_K + ECG_MAX_P) + 64)
		q->slot_bytes = (size_t)pitch_of(q->attr.max_cell_bytes) * (ECG_MAX_K + ECG_MAX_P) + 64;
	pthread_mutex_init(&q->lock, NULL);
	pthread_cond_init(&q->cv_work, NULL);
	pthread_cond_init(&q->cv_slot, NULL);
	pthread_cond_init(&q->cv_done, NULL);
	pthread_cond_init(&q->cv_fin, NULL);
	for (i = 0; i < NDSTLOCK; i++)
		pthread_mutex_init(&q->dst_lock[i], NULL);
	for (i = 0; i < q->nslot && e == hipSuccess; i++) {
		struct qslot *s = &q->slot[i];

		s->reqs = calloc(q->attr.max_batch, sizeof(*s->reqs));
		/* cell addresses: device cells k <= ECG_KMAX_K (one launch); the CPU
		 * executor any k */
		s->tab = calloc((size_t)q->attr.max_batch * (ECG_MAX_K + ECG_MAX_P), sizeof(*s->tab));
		s->uvec = calloc(q->attr.max_batch, 1);
		if (s->reqs == NULL || s->tab == NULL || s->uvec == NULL) {
			e = hipErrorOutOfMemory;
			break;
		}
		s->bytes = q->slot_bytes;
		if (q->cpu)		/* nothing staged: the completion threads read the cells */
			continue;
		s->ctx = ctxs[i % nctx];
		for (s->ui = 0; ctxs[s->ui]->device != s->ctx->device; s->ui++)
			;
		e = hipSetDevice(s->ctx->device);
		if (e == hipSuccess) {
			/* the slot's pinned staging on its device's NUMA node: the
			 * pages are touched (pinned) by this thread while it runs
			 * there, and NumaUser keeps the runtime from placing them */
			cpu_set_t saved;
			const int node = ecg_numa_bind_thread(s->ctx->device, &saved);

			e = hipHostMalloc((void **)&s->host, s->bytes,
					  hipHostMallocDefault | (node >= 0 ? hipHostMallocNumaUser : 0));
			if (node >= 0)
				ecg_numa_restore_thread(&saved);
		}
		if (e == hipSuccess)
			e = hipMalloc((void **)&s->dev, s->bytes);
		if (e == hipSuccess)
			e = hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking);
		if (e == hipSuccess)
			e = hipEventCreateWithFlags(&s->done, hipEventDisableTiming);
	}
	for (i = 0; i < q->nctx && e == hipSuccess; i++) {
		/* one per device (ust[i] of the first entry naming it; ui above) */
		e = hipSetDevice(q->ctxs[i]->device);
		if (e == hipSuccess)
			e = hipStreamCreateWithFlags(&q->ust[i], hipStreamNonBlocking);
	}
	for (i = 0; i < cpu_workers() && e == hipSuccess; i++) {
		if (pthread_create(&q->fin[i], NULL, fin_main, q) != 0)
			e = hipErrorOutOfMemory;
		else
			q->nfin++;
	}
	if (e == hipSuccess && pthread_create(&q->worker, NULL, worker_main, q) != 0)
		e = hipErrorOutOfMemory;
	if (e != hipSuccess && q->nfin) {
		pthread_mutex_lock(&q->lock);
		q->stop = q->worker_exited = 1;
		pthread_cond_broadcast(&q->cv_fin);
		pthread_mutex_unlock(&q->lock);
		for (i = 0; i < q->nfin; i++)
			pthread_join(q->fin[i], NULL);
	}
	if (e != hipSuccess) {
		for (i = 0; i < q->nslot; i++)
			slot_free(&q->slot[i]);
		const int cpu = q->cpu;

		for (i = 0; i < q->nctx; i++)
			if (q->ust[i])
				(void)hipStreamDestroy(q->ust[i]);
		free(q);
		return cpu ? ecg_fail(-ECG_DER_NOMEM, "queue_create: out of memory or threads")
			   : ecg_hip_fail(e, "queue_create");
	}
	*out = q;
	return 0;
}

int ecg_queue_create(ecg_ctx_t *ctx, const ecg_queue_attr_t *attr, ecg_queue_t **out)
{
	const char *force = getenv("ECG_FORCE_CPU");
	int rc;

	if (out == NULL)
		return ecg_fail(-ECG_DER_INVAL, "queue_create: NULL argument");
	/* no context, or $ECG_FORCE_CPU=1: the CPU executor, no device touched */
	if (ctx == NULL || (force && force[0] == '1'))
		return queue_create(NULL, 0, attr, out);
	rc = ecg_ctx_enter(ctx);
	if (rc)
		return rc;
	return queue_create(&ctx, 1, attr, out);
}

int ecg_queue_create_multi(ecg_multi_t *m, const ecg_queue_attr_t *attr, ecg_queue_t **out)
{
	ecg_ctx_t *ctxs[ECG_MULTI_MAX];
	int i, n = ecg_multi_count(m);

	if (m == NULL || out == NULL || n < 1)
		return ecg_fail(-ECG_DER_INVAL, "queue_create_multi: bad argument");
	for (i = 0; i < n; i++)
		ctxs[i] = ecg_multi_ctx(m, i);
	return queue_create(ctxs, n, attr, out);
}

void ecg_queue_destroy(ecg_queue_t *q)
{
	if (q == NULL)
		return;
	pthread_mutex_lock(&q->lock);
	q->stop = 1;
	pthread_cond_broadcast(&q->cv_work);
	pthread_cond_broadcast(&q->cv_slot);
	pthread_mutex_unlock(&q->lock);
	pthread_join(q->worker, NULL);
	for (int i = 0; i < q->nfin; i++)
		pthread_join(q->fin[i], NULL);
#ifdef ECG_QUEUE_TIMING
	if (q->tm_n)
		fprintf(stderr, "ecg queue timing: %llu batches, %.1f requests each; us per batch: closed->launch %.1f, "
			"launch %.1f, in flight %.1f, completion %.1f\n", (unsigned long long)q->tm_n,
			(double)q->tm_sum[4] / q->tm_n, q->tm_sum[0] / 1e3 / q->tm_n, q->tm_sum[1] / 1e3 / q->tm_n,
			q->tm_sum[2] / 1e3 / q->tm_n, q->tm_sum[3] / 1e3 / q->tm_n);
	if (q->tm_n)
		fprintf(stderr, "ecg queue timing: launch thread CPU %.1f us per batch\n", q->tm_cpu / 1e3 / q->tm_n);
	ecg_ptrs_timing_print();
#endif
	for (int i = 0; i < q->nslot; i++)
		slot_free(&q->slot[i]);
	for (int i = 0; i < q->nctx; i++) {
		(void)hipSetDevice(q->ctxs[i]->device);
		(void)hipStreamDestroy(q->ust[i]);
	}
	pthread_cond_destroy(&q->cv_work);
	pthread_cond_destroy(&q->cv_slot);
	pthread_cond_destroy(&q->cv_done);
	pthread_cond_destroy(&q->cv_fin);
	for (int i = 0; i < NDSTLOCK; i++)
		pthread_mutex_destroy(&q->dst_lock[i]);
	pthread_mutex_destroy(&q->lock);
	free(q);
}

/* Where a request's cells are (ecg_cells_place, through the drop-in's
 * per-thread cache of plain host memory): all host memory -> -1; all memory
 * of one of the queue's devices -> that device (every cell inside one of its
 * allocations, and the shape one pointer-table launch takes); anything else
 * -> -1 with a negative DER code in *rc naming the cell.  A recovery's stripe
 * is one [k+p][cell] range.  The CPU executor takes host memory only (and
 * looks nothing up when the process sees no device at all). */
static int request_device(struct ecg_queue *q, int op, int k, int p, uint64_t C, int rows,
			  unsigned char *const *src, unsigned char *stripe, unsigned char *const *dst, int *rc)
{
	signed char place[ECG_MAX_K + ECG_MAX_P];
	unsigned char *one[1] = {stripe};
	const int nin = op == OP_RECOVER ? 1 : op == OP_UPDATE ? 2 : k;
	const int nout = op == OP_RECOVER ? 0 : p;
	ecg_ctx_t *ctx = NULL;
	int dev = -1, ndev;

	*rc = 0;
	if (q->cpu && !ecg_dropin_gpu())
		return -1;
	ndev = ecg_cells_place(op == OP_RECOVER ? one : src, nin, dst, nout,
			       op == OP_RECOVER ? C * (uint64_t)(k + p) : C, ecg_ptr_device_cached, place, &dev);
	if (ndev <= 0) {
		*rc = ndev < 0 ? ndev : 0;
		return -1;
	}
	if (ndev != nin + nout) {
		for (int i = 0; i < nin + nout; i++)
			if (place[i] < 0) {
				*rc = ecg_fail(-ECG_DER_INVAL, "queue: %s %d is host memory, other cells of the request "
					       "memory of device %d (a request's cells are all host or all device "
					       "memory)", i < nin ? "input" : "parity", i < nin ? i : i - nin, dev);
				break;
			}
		return -1;
	}
	if (q->cpu) {
		*rc = ecg_fail(-ECG_DER_INVAL, "queue: cells are memory of device %d, and this queue runs on the CPU "
			       "(created without a context, or $ECG_FORCE_CPU=1)", dev);
		return -1;
	}
	for (int i = 0; i < q->nctx && ctx == NULL; i++)
		if (q->ctxs[i]->device == dev)
			ctx = q->ctxs[i];
	if (ctx == NULL)
		*rc = ecg_fail(-ECG_DER_INVAL, "queue: cells are memory of device %d, which has no slot in "
			       "this queue", dev);
	else if (k > ECG_KMAX_K || rows > ECG_KMAX_R)
		*rc = ecg_fail(-ECG_DER_INVAL, "queue: device cells need k <= %d and rows <= %d (k=%d rows=%d)",
			       ECG_KMAX_K, ECG_KMAX_R, k, rows);
	return dev;
}

/* Reserve a stripe index in a slot of this class (opening one if needed),
 * copy the inputs in (device cells: their addresses) without the lock, then
 * publish. */
static int submit(struct ecg_queue *q, int op, int k, int p, uint64_t C, const uint32_t *err,
		  int nerrs, unsigned char *const *src, unsigned char *stripe,
		  unsigned char *const *dst, int vec_i, ecg_done_cb_t cb, void *arg)
{
	struct qslot *s = NULL;
	uint32_t idx;
	int i, rc = 0;
	const int rows = op == OP_RECOVER ? nerrs : p;
	const int dev = request_device(q, op, k, p, C, rows, src, stripe, dst, &rc);
	/* host cells where the drop-in would compute them: on the CPU path below
	 * its crossover (with a GFNI CPU always -- one core outruns a PCIe round
	 * trip at every size), so the queue's completion threads
	 * compute them in place instead of staging them over PCIe */
	const int cpuexec = q->cpu ||
			    (dev < 0 && ecg_dropin_host_on_cpu(C * (uint64_t)((op == OP_UPDATE ? 2 : k) + rows)));

	if (rc)
		return rc;
	/* fast path, no lock: an open slot of this class with room */
	for (i = 0; i < q->nslot && s == NULL; i++)
		if (slot_try_reserve(&q->slot[i], op, k, p, C, err, nerrs, dev, cpuexec, &idx))
			s = &q->slot[i];
	if (s == NULL) {
		pthread_mutex_lock(&q->lock);
		while (s == NULL) {
			if (q->stop) {
				pthread_mutex_unlock(&q->lock);
				return ecg_fail(-ECG_DER_INVAL, "queue is being destroyed");
			}
			for (i = 0; i < q->nslot && s == NULL; i++)
				if (q->slot[i].state == S_FILLING &&
				    slot_try_reserve(&q->slot[i], op, k, p, C, err, nerrs, dev, cpuexec, &idx))
					s = &q->slot[i];
			/* open FREE slots from a rotating start: batches spread over
			 * the devices of a multi-device queue */
			for (i = 0; i < q->nslot && s == NULL; i++) {
				struct qslot *f = &q->slot[(q->open_next + (uint32_t)i) % (uint32_t)q->nslot];

				if (f->state == S_FREE && (dev < 0 || f->ctx->device == dev)) {
					rc = slot_open(q, f, op, k, p, C, err, nerrs, dev, cpuexec);
					if (rc) {
						f->state = S_FREE;
						pthread_mutex_unlock(&q->lock);
						return rc;
					}
					q->open_next = (uint32_t)(f - q->slot) + 1;
					if (slot_try_reserve(f, op, k, p, C, err, nerrs, dev, cpuexec, &idx))
						s = f;
				}
			}
			if (s == NULL) {
				pthread_cond_broadcast(&q->cv_work);	/* make the worker drain */
				pthread_cond_wait(&q->cv_slot, &q->lock);
			}
		}
		pthread_mutex_unlock(&q->lock);
	}
	__atomic_add_fetch(&q->submitted, 1, __ATOMIC_RELAXED);

	{
		struct qreq *r = &s->reqs[idx];
		const int addr = s->devcells || s->cpuexec;	/* the request holds addresses */
		unsigned char *in = addr ? NULL : s->host + (size_t)idx * s->pitch * (uint64_t)s->nin;

		r->op = op;
		r->k = k;
		r->p = p;
		r->C = C;
		r->nerrs = nerrs;
		r->cb = cb;
		r->arg = arg;
		r->rc = 0;
		if (addr && op == OP_UPDATE) {	/* old, new, parity: ecg_update_ptrs' row */
			uint64_t *t = s->tab + (size_t)idx * (uint64_t)(2 + s->rows);

			t[0] = (uint64_t)(uintptr_t)src[0];
			t[1] = (uint64_t)(uintptr_t)src[1];
			for (i = 0; i < s->rows; i++)
				t[2 + i] = (uint64_t)(uintptr_t)dst[i];
			s->uvec[idx] = (uint8_t)vec_i;
		} else if (addr) {	/* the stripe's ISA-L pointers, nothing copied */
			uint64_t *t = s->tab + (size_t)idx * (uint64_t)(k + s->rows);

			for (i = 0; i < k; i++)
				t[i] = (uint64_t)(uintptr_t)(op == OP_ENCODE ? src[i]
							     : stripe + (uint64_t)s->dec_idx[i] * C);
			for (i = 0; i < s->rows; i++)
				t[k + i] = (uint64_t)(uintptr_t)(op == OP_ENCODE ? dst[i]
								 : stripe + (uint64_t)s->out_idx[i] * C);
		} else if (op == OP_UPDATE) {	/* the xor_gen: diff = old ^ new */
			xor_into(in, src[0], src[1], C);
			s->host[(size_t)s->pitch * s->nin * s->cap + idx] = (unsigned char)vec_i;
		}
		for (i = 0; !addr && op != OP_UPDATE && i < k; i++) {
			const unsigned char *from = op == OP_ENCODE ? src[i]
					: stripe + (uint64_t)s->dec_idx[i] * C;

			memcpy(in + (uint64_t)i * s->pitch, from, C);
		}
		for (i = 0; i < s->rows; i++)
			r->dst[i] = op != OP_RECOVER ? dst[i] : stripe + (uint64_t)s->out_idx[i] * C;
	}

	/* wake the worker only for what it acts on: a slot's first request (a new
	 * deadline to wait for; for device cells, a batch that may launch at
	 * once), a slot this request filled up, and a closed slot -- whose last
	 * inputs may be the ones landing now.  Store-then-load of two different
	 * words on each side (here `filled` then `res`; slot_close clears `res`'s
	 * open bit, the worker then loads `filled`): only sequentially consistent
	 * operations rule out both sides reading the old values, which would skip
	 * this wake-up (the worker's 20 us poll of READY slots would still catch
	 * it, late).  The slot's fields are read BEFORE `filled` counts this
	 * request: from then on the worker may launch it, the completion threads
	 * free it and another submitter reopen it with a new class (the
	 * ThreadSanitizer run of tests/c queue_cpu_stress caught a read of `cap`
	 * racing with slot_open here).  `res` itself carries the generation: a
	 * reopened slot's open bit means this one's batch has already launched. */
	{
		const uint32_t cap = LD(s->cap);
		const uint32_t n = __atomic_add_fetch(&s->filled, 1u, __ATOMIC_SEQ_CST);

		if (n == 1 || idx + 1 == cap || !(__atomic_load_n(&s->res, __ATOMIC_SEQ_CST) & RES_OPEN)) {
			pthread_mutex_lock(&q->lock);
			pthread_cond_signal(&q->cv_work);
			pthread_mutex_unlock(&q->lock);
		}
	}
	return 0;
}

int ecg_queue_encode(ecg_queue_t *q, int k, int p, uint64_t C, unsigned char *const *data,
		     unsigned char *const *parity, ecg_done_cb_t cb, void *arg)
{
	if (q == NULL || data == NULL || parity == NULL || k < 1 || k > ECG_MAX_K || p < 1 ||
	    p > ECG_MAX_P || C == 0)
		return ecg_fail(-ECG_DER_INVAL, "queue_encode: bad arguments");
	return submit(q, OP_ENCODE, k, p, C, NULL, 0, data, NULL, parity, 0, cb, arg);
}

int ecg_queue_recover(ecg_queue_t *q, int k, int p, uint64_t C, unsigned char *stripe,
		      const uint32_t *err_list, int nerrs, ecg_done_cb_t cb, void *arg)
{
	int i, j;

	if (q == NULL || stripe == NULL || err_list == NULL || k < 1 || k > ECG_MAX_K || p < 1 ||
	    p > ECG_MAX_P || C == 0 || nerrs < 1)
		return ecg_fail(-ECG_DER_INVAL, "queue_recover: bad arguments");
	if (nerrs > p)
		return ecg_fail(-ECG_DER_DATA_LOSS, "queue_recover: %d erasures > p=%d", nerrs, p);
	for (i = 0; i < nerrs; i++) {
		if (err_list[i] >= (uint32_t)(k + p))
			return ecg_fail(-ECG_DER_INVAL, "queue_recover: cell %u", err_list[i]);
		for (j = 0; j < i; j++)
			if (err_list[j] == err_list[i])
				return ecg_fail(-ECG_DER_INVAL, "queue_recover: duplicate cell %u",
						err_list[i]);
	}
	return submit(q, OP_RECOVER, k, p, C, err_list, nerrs, NULL, stripe, NULL, 0, cb, arg);
}

int ecg_queue_update(ecg_queue_t *q, int k, int p, uint64_t C, int vec_i, const unsigned char *old_cell,
		     const unsigned char *new_cell, unsigned char *const *parity, ecg_done_cb_t cb,
		     void *arg)
{
	unsigned char *src[2];

	/* one launch stages the tables of every column: k <= ECG_KMAX_K */
	if (q == NULL || old_cell == NULL || new_cell == NULL || parity == NULL || k < 1 ||
	    k > ECG_KMAX_K || p < 1 || p > ECG_MAX_P || C == 0 || vec_i < 0 || vec_i >= k)
		return ecg_fail(-ECG_DER_INVAL, "queue_update: bad arguments");
	src[0] = (unsigned char *)old_cell;
	src[1] = (unsigned char *)new_cell;
	return submit(q, OP_UPDATE, k, p, C, NULL, 0, src, NULL, parity, vec_i, cb, arg);
}

int ecg_queue_flush(ecg_queue_t *q)
{
	uint64_t target;

	if (q == NULL)
		return ecg_fail(-ECG_DER_INVAL, "queue_flush: NULL queue");
	pthread_mutex_lock(&q->lock);
	target = __atomic_load_n(&q->submitted, __ATOMIC_RELAXED);
	if (q->flush_target < target)
		q->flush_target = target;
	pthread_cond_broadcast(&q->cv_work);
	while (q->completed < target)
		pthread_cond_wait(&q->cv_done, &q->lock);
	pthread_mutex_unlock(&q->lock);
	return 0;
}

int ecg_queue_stats(ecg_queue_t *q, uint64_t *requests, uint64_t *batches)
{
	if (q == NULL)
		return ecg_fail(-ECG_DER_INVAL, "queue_stats: NULL queue");
	pthread_mutex_lock(&q->lock);
	if (requests)
		*requests = q->completed;
	if (batches)
		*batches = q->batches;
	pthread_mutex_unlock(&q->lock);
	return 0;
}
