/*
 * ecg_stage.c -- synchronous host-memory product over pointer arrays: the
 * calling convention of ISA-L ec_encode_data (k source pointers, `rows`
 * destination pointers, arbitrary alignment and length), executed on the GPU
 * through per-thread pinned staging.  Serves the ISA-L drop-in (ecg_isal.c)
 * and obj_ec_encode_buf (ecg_daos.c).  One stripe per call is what every
 * reference caller issues (ref:src/object/cli_ec.c:540, 571, 2641;
 * ref:src/object/srv_ec_aggregate.c:693, 1136), so this path is PCIe- and
 * launch-latency-bound by construction; the batched entry points in ecg.h
 * are the throughput path.
 */
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ecg_internal.h"

struct tstage {
	ecg_ctx_t *ctx;
	int device;
	void *host;
	size_t host_bytes;
	void *dev;
	size_t dev_bytes;
	hipStream_t st;
	hipEvent_t ev;		/* device-cell calls wait on this */
	hipEvent_t ev_in;	/* ... after ordering behind the context stream with this */
	int ev_device;
};

static pthread_key_t g_key;
static pthread_once_t g_key_once = PTHREAD_ONCE_INIT;

/* Staging bytes up to which a call skips the DMA copies and lets the kernel
 * work on the pinned staging in place (env ECG_ZERO_COPY_MAX overrides;
 * tools/bench_dropin.py, profiles/r01/bench_dropin.jsonl). */
static size_t g_zero_copy_max = 4u << 20;

static void tstage_release(struct tstage *t)
{
	if (t->st) {
		(void)hipSetDevice(t->device);
		(void)hipStreamSynchronize(t->st);
		(void)hipStreamDestroy(t->st);
	}
	if (t->host)
		(void)hipHostFree(t->host);
	if (t->dev)
		(void)hipFree(t->dev);
	if (t->ev) {
		(void)hipSetDevice(t->ev_device);
		(void)hipEventDestroy(t->ev);
		(void)hipEventDestroy(t->ev_in);
	}
	memset(t, 0, sizeof(*t));
}

static void tstage_dtor(void *p)
{
	if (p) {
		tstage_release(p);
		free(p);
	}
}

static void key_init(void)
{
	const char *env = getenv("ECG_ZERO_COPY_MAX");

	pthread_key_create(&g_key, tstage_dtor);
	if (env)
		g_zero_copy_max = (size_t)strtoull(env, NULL, 0);
}

static struct tstage *tstage_self(void)
{
	struct tstage *t;

	pthread_once(&g_key_once, key_init);
	t = pthread_getspecific(g_key);
	if (t == NULL) {
		t = calloc(1, sizeof(*t));
		if (t != NULL)
			pthread_setspecific(g_key, t);
	}
	return t;
}

/* The calling thread's completion event on ctx's device (device-cell calls);
 * kept apart from the host staging so alternating host and device cells of
 * different devices does not free either. */
static int tstage_event(ecg_ctx_t *ctx, struct tstage **out)
{
	struct tstage *t = tstage_self();
	hipError_t e;

	if (t == NULL)
		return ecg_fail(-ECG_DER_NOMEM, "stage: calloc");
	if (t->ev && t->ev_device != ctx->device) {
		(void)hipEventDestroy(t->ev);
		(void)hipEventDestroy(t->ev_in);
		t->ev = t->ev_in = NULL;
	}
	if (t->ev == NULL) {
		e = hipEventCreateWithFlags(&t->ev, hipEventDisableTiming);
		if (e == hipSuccess) {
			e = hipEventCreateWithFlags(&t->ev_in, hipEventDisableTiming);
			if (e != hipSuccess)
				(void)hipEventDestroy(t->ev);
		}
		if (e != hipSuccess) {
			t->ev = t->ev_in = NULL;
			return ecg_hip_fail(e, "stage event");
		}
		t->ev_device = ctx->device;
	}
	*out = t;
	return 0;
}

static int tstage_get(ecg_ctx_t *ctx, size_t bytes, struct tstage **out)
{
	struct tstage *t = tstage_self();
	hipError_t e;

	if (t == NULL)
		return ecg_fail(-ECG_DER_NOMEM, "stage: calloc");
	if (t->ctx != ctx || t->device != ctx->device) {
		/* host staging of another context: free it, keep the events */
		hipEvent_t ev = t->ev, ev_in = t->ev_in;
		int ev_device = t->ev_device;

		t->ev = t->ev_in = NULL;
		tstage_release(t);
		t->ev = ev;
		t->ev_in = ev_in;
		t->ev_device = ev_device;
	}
	t->ctx = ctx;
	t->device = ctx->device;
	if (t->st == NULL) {
		e = hipStreamCreateWithFlags(&t->st, hipStreamNonBlocking);
		if (e != hipSuccess)
			return ecg_hip_fail(e, "stage stream");
	}
	if (t->host_bytes < bytes) {
		if (t->host)
			(void)hipHostFree(t->host);
		t->host = NULL;
		t->host_bytes = 0;
		e = hipHostMalloc(&t->host, bytes, hipHostMallocDefault);
		if (e != hipSuccess)
			return ecg_hip_fail(e, "stage pinned alloc");
		t->host_bytes = bytes;
	}
	if (t->dev_bytes < bytes) {
		if (t->dev)
			(void)hipFree(t->dev);
		t->dev = NULL;
		t->dev_bytes = 0;
		e = hipMalloc(&t->dev, bytes);
		if (e != hipSuccess)
			return ecg_hip_fail(e, "stage device alloc");
		t->dev_bytes = bytes;
	}
	*out = t;
	return 0;
}

/* The device whose memory p is (hipMalloc'd), ECG_PTR_HOST for host memory
 * the HIP runtime knows (pinned, registered, managed), ECG_PTR_UNKNOWN for
 * memory it does not (plain malloc / mmap: host memory).  The failed query's
 * error is cleared so a later launch check does not report it. */
int ecg_ptr_device(const void *p)
{
	hipPointerAttribute_t a;

	memset(&a, 0, sizeof(a));
	if (hipPointerGetAttributes(&a, p) != hipSuccess) {
		(void)hipGetLastError();
		return ECG_PTR_UNKNOWN;
	}
	if (a.type == hipMemoryTypeUnregistered)	/* pageable memory the runtime never saw */
		return ECG_PTR_UNKNOWN;
	return a.type == hipMemoryTypeDevice ? a.device : ECG_PTR_HOST;
}

/* Every cell [v[i], v[i] + len) lies inside one allocation of ctx's device:
 * a pointer into host memory, another device or past an allocation's end
 * would make the launch fault the GPU, so it is refused here.  Cells of one
 * buffer (the usual stripe) cost one attribute and one range query in all. */
int ecg_cells_on_device(ecg_ctx_t *ctx, unsigned char *const *v, int n, uint64_t len, const char *what)
{
	struct {
		uintptr_t lo, hi;
	} seen[4];
	int nseen = 0, i, x;

	for (i = 0; i < n; i++) {
		const uintptr_t a = (uintptr_t)v[i], e = a + (uintptr_t)len;
		hipDeviceptr_t base = NULL;
		size_t size = 0;

		for (x = 0; x < nseen; x++)
			if (a >= seen[x].lo && e <= seen[x].hi)
				break;
		if (x < nseen)
			continue;
		if (ecg_ptr_device(v[i]) != ctx->device)
			return ecg_fail(-ECG_DER_INVAL, "matmul_host: %s %d is not memory of device %d "
					"(every cell of a call must be)", what, i, ctx->device);
		if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)v[i]) != hipSuccess) {
			(void)hipGetLastError();
			return ecg_fail(-ECG_DER_INVAL, "matmul_host: %s %d: no device allocation", what, i);
		}
		if (e > (uintptr_t)base + size)
			return ecg_fail(-ECG_DER_INVAL, "matmul_host: %s %d: %llu bytes run past the end of its "
					"allocation", what, i, (unsigned long long)len);
		x = nseen < 4 ? nseen++ : i % 4;
		seen[x].lo = (uintptr_t)base;
		seen[x].hi = (uintptr_t)base + size;
	}
	return 0;
}

/* The device allocations a thread's recent calls found their cells in, each
 * with its range and device: a cell inside one costs no query.  The pointer
 * and range queries serialise on a runtime lock that launches need too -- 16
 * threads posting device-cell requests to a queue kept its worker's launches
 * waiting on it (profiles/r06/queue_dev_update/).  A device range is
 * remembered for 1 ms (ECG_PLACE_CACHE_US; 0 = within one call only, the
 * round-5 behaviour); runtime-known host ranges (pinned, registered, managed)
 * only within the call.  ecg_dev_free clears every thread's ranges.  What the
 * window does not see: an allocation freed by the caller's own hipFree and
 * its addresses reallocated within it -- as pinned host memory the kernel
 * still reaches the cells (they are GPU-mapped), as another device's memory
 * it would not. */
#define PLACE_N 4
static __thread struct {
	uintptr_t lo, hi;
	uint64_t until;
	int dev;
} t_place[PLACE_N];
static __thread unsigned t_place_next;
static __thread uint64_t t_place_gen;
static int64_t g_place_ttl_ns = -1;
static uint64_t g_place_gen;	/* bumped by every device free through the library */

void ecg_place_forget(void)
{
	__atomic_add_fetch(&g_place_gen, 1, __ATOMIC_RELEASE);
}

static uint64_t place_ttl_ns(void)
{
	int64_t t = __atomic_load_n(&g_place_ttl_ns, __ATOMIC_RELAXED);

	if (t < 0) {
		const char *env = getenv("ECG_PLACE_CACHE_US");

		t = env && *env ? (int64_t)strtoll(env, NULL, 10) * 1000 : 1000000;
		if (t < 0)
			t = 0;
		__atomic_store_n(&g_place_ttl_ns, t, __ATOMIC_RELAXED);
	}
	return (uint64_t)t;
}

/* Placement of every cell of a one-stripe call (src[0..k) then dst[0..rows)):
 * place[i] = the device whose allocation holds cell i whole, or -1 for host
 * memory (plain malloc / mmap, pinned, registered, managed: the CPU can
 * address it).  `query` is the placement lookup (ecg_ptr_device, or the
 * drop-in's cached one).  Cells inside a runtime-known range seen by this
 * thread within the cache window (one allocation: the usual stripe, a
 * buffer pool) cost no query.  Returns the number of device cells (*dev =
 * their device), or -DER_INVAL naming the cell for cells on two devices or a
 * device cell running past its allocation. */
int ecg_cells_place(unsigned char *const *src, int k, unsigned char *const *dst, int rows, uint64_t len,
		    int (*query)(const void *), signed char *place, int *dev)
{
	struct timespec ts;
	uint64_t now;
	int ndev = 0, i, x;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	now = (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
	{
		const uint64_t gen = __atomic_load_n(&g_place_gen, __ATOMIC_ACQUIRE);

		if (gen != t_place_gen) {	/* a device free since: start over */
			memset(t_place, 0, sizeof(t_place));
			t_place_gen = gen;
		}
	}
	*dev = -1;
	for (i = 0; i < k + rows; i++) {
		const unsigned char *c = i < k ? src[i] : dst[i - k];
		const uintptr_t a = (uintptr_t)c, e = a + (uintptr_t)len;
		const char *what = i < k ? "source" : "output";
		const int idx = i < k ? i : i - k;
		hipDeviceptr_t base = NULL;
		size_t size = 0;
		int d;

		if (c == NULL)
			return ecg_fail(-ECG_DER_INVAL, "%s %d is NULL", what, idx);
		for (x = 0; x < PLACE_N; x++)
			if (now <= t_place[x].until && a >= t_place[x].lo && e <= t_place[x].hi)
				break;
		if (x < PLACE_N) {
			d = t_place[x].dev;
		} else {
			d = query(c);
			if (d != ECG_PTR_UNKNOWN) {
				/* runtime-known memory: its allocation's range, so the
				 * stripe's other cells in it need no query */
				if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)c) == hipSuccess) {
					if (d >= 0 && e > (uintptr_t)base + size)
						return ecg_fail(-ECG_DER_INVAL, "%s %d: %llu bytes run past the end of its "
								"device allocation", what, idx, (unsigned long long)len);
					x = (int)(t_place_next++ % PLACE_N);
					t_place[x].lo = (uintptr_t)base;
					t_place[x].hi = (uintptr_t)base + size;
					t_place[x].dev = d >= 0 ? d : -1;
					/* host ranges only for this call: a device
					 * allocation reusing their addresses must never
					 * reach the CPU path */
					t_place[x].until = now + (d >= 0 ? place_ttl_ns() : 0);
				} else {
					(void)hipGetLastError();
					if (d >= 0)
						return ecg_fail(-ECG_DER_INVAL, "%s %d: no device allocation", what, idx);
				}
			}
			if (d < 0)
				d = -1;
		}
		place[i] = (signed char)(d < 0 ? -1 : d);
		if (d >= 0) {
			if (*dev >= 0 && *dev != d)
				return ecg_fail(-ECG_DER_INVAL, "%s %d is memory of device %d, an earlier cell of device %d "
						"(one call's cells may span one device and host memory)", what, idx, d,
						*dev);
			*dev = d;
			ndev++;
		}
	}
	return ndev;
}

/* The stream of the calling thread among the context's drop-in pool
 * (created on first use): concurrent synchronous callers spread over up to
 * ECG_DROPIN_STREAMS streams -- the box's hardware queues -- instead of
 * queueing behind each other on one. */
static int pool_stream(ecg_ctx_t *ctx, hipStream_t *out)
{
	static unsigned next_slot;
	static __thread unsigned slot = ~0u;
	hipError_t e = hipSuccess;
	int n;

	if (slot == ~0u)
		slot = __atomic_fetch_add(&next_slot, 1u, __ATOMIC_RELAXED);
	n = __atomic_load_n(&ctx->ndpool, __ATOMIC_ACQUIRE);
	if (n == 0) {
		const char *env = getenv("ECG_DROPIN_STREAMS");
		int want = env ? atoi(env) : ECG_DROPIN_STREAMS, i;

		if (want < 1 || want > ECG_DROPIN_STREAMS)
			want = ECG_DROPIN_STREAMS;
		pthread_mutex_lock(&ctx->lock);
		n = ctx->ndpool;
		for (i = n; i < want && e == hipSuccess; i++) {
			e = hipStreamCreateWithFlags(&ctx->dpool[i], hipStreamNonBlocking);
			if (e == hipSuccess)
				n = i + 1;
		}
		__atomic_store_n(&ctx->ndpool, n, __ATOMIC_RELEASE);
		pthread_mutex_unlock(&ctx->lock);
		if (n == 0)
			return ecg_hip_fail(e, "drop-in stream pool");
	}
	*out = ctx->dpool[slot % (unsigned)n];
	return 0;
}

/* One-stripe product of any k (<= ECG_MAX_K + 256) and rows (<= 256) as
 * launches of at most ECG_MAX_K sources (later source groups accumulate) and
 * 8 rows, so the sliced coefficients stay a 512-byte stack array (a caller
 * may be a user-level thread with a small stack). */
static int launch_split(ecg_ctx_t *ctx, int len, int k, int rows, const unsigned char *coef, const void *sbase,
			const int64_t *soff, void *dbase, const int64_t *doff, unsigned flags, hipStream_t st)
{
	unsigned char cc[ECG_MAX_K * 8];
	int j0, r0, r, rc = 0;

	if (k <= ECG_MAX_K)
		return ecg_matmul(ctx, k, rows, coef, (uint64_t)len, 1, sbase, soff, 0, dbase, doff, 0, flags, st);
	for (j0 = 0; rc == 0 && j0 < k; j0 += ECG_MAX_K) {
		const int kk = k - j0 < ECG_MAX_K ? k - j0 : ECG_MAX_K;
		const unsigned f = flags | (j0 ? ECG_F_ACCUMULATE : 0u);

		for (r0 = 0; rc == 0 && r0 < rows; r0 += 8) {
			const int rr = rows - r0 < 8 ? rows - r0 : 8;

			for (r = 0; r < rr; r++)
				memcpy(&cc[r * kk], &coef[(size_t)(r0 + r) * k + j0], (size_t)kk);
			rc = ecg_matmul(ctx, kk, rr, cc, (uint64_t)len, 1, sbase, soff + j0, 0, dbase, doff + r0, 0,
					f, st);
		}
	}
	return rc;
}

/* The ISA-L data-plane calls with DEVICE cells (an engine whose bio buffers
 * live in HBM keeps its ec_encode_data call sites): strided launches on the
 * cells in place (cell offsets relative to the first source / output; more
 * than ECG_MAX_K sources -- xor_gen -- as accumulating groups), on the
 * caller's pool stream (ordered behind the work queued on the context's own
 * stream), then a wait for an event recorded right after them: the call
 * waits for its own launches and what precedes them on that stream, not for
 * every other thread's drop-in work (ISA-L's calls are synchronous). */
static int matmul_device(ecg_ctx_t *ctx, int len, int k, int rows, const unsigned char *coef,
			 unsigned char *const *src, unsigned char *const *dst, unsigned flags)
{
	int64_t soff[ECG_MAX_K + 256], doff[256];
	struct tstage *t = NULL;
	hipStream_t st = NULL;
	hipError_t e;
	int j, r, rc;

	rc = pool_stream(ctx, &st);
	if (rc == 0)
		rc = tstage_event(ctx, &t);
	if (rc)
		return rc;
	for (j = 0; j < k; j++)
		soff[j] = (int64_t)((uintptr_t)src[j] - (uintptr_t)src[0]);
	for (r = 0; r < rows; r++)
		doff[r] = (int64_t)((uintptr_t)dst[r] - (uintptr_t)dst[0]);
	/* keep the order a caller of the context's own stream relies on (an
	 * ecg_memcpy / ecg_memset there before this call, as when device cells
	 * used that stream): the pool stream waits for what is queued on it now.
	 * An idle context stream -- the drop-in-only engine -- costs one query
	 * (0.07 us) instead of the record + wait (3.2 us, tools/hipcall_cost.hip) */
	e = hipStreamQuery(ctx->stream);
	if (e == hipErrorNotReady) {
		e = hipEventRecord(t->ev_in, ctx->stream);
		if (e == hipSuccess)
			e = hipStreamWaitEvent(st, t->ev_in, 0);
	}
	if (e != hipSuccess)
		return ecg_hip_fail(e, "matmul_host: order behind the context stream");
	rc = launch_split(ctx, len, k, rows, coef, src[0], soff, dst[0], doff, flags, st);
	if (rc)
		return rc;
	e = hipEventRecord(t->ev, st);
	if (e == hipSuccess)
		e = hipEventSynchronize(t->ev);
	return e == hipSuccess ? 0 : ecg_hip_fail(e, "matmul_host: device cells sync");
}

/*
 * dst[r][i] (^)= XOR_j coef[r*k + j] * src[j][i], i < len, on ctx's GPU.
 * place[] (ecg_cells_place, k + rows entries; NULL = every cell host memory)
 * says where each cell is: host cells are staged through pinned memory,
 * device cells (memory of ctx's device, checked by the caller) are used in
 * place -- all of them device cells: launches on the cells alone, no staging.
 * With ECG_F_ACCUMULATE the current bytes of host dst cells travel to the
 * device first (ec_encode_data_update semantics).
 */
int ecg_matmul_host_mem(ecg_ctx_t *ctx, int len, int k, int rows, const unsigned char *coef,
			unsigned char *const *src, unsigned char *const *dst, unsigned flags, const signed char *place)
{
	int64_t soff[ECG_MAX_K + 256], doff[256];
	struct tstage *t = NULL;
	size_t pitch, bytes;
	unsigned char *h, *d;
	hipError_t e;
	int rc, j, r;

	if (len < 0 || k < 1 || k > ECG_MAX_K + 256 || rows < 1 || rows > 256)
		return ecg_fail(-ECG_DER_INVAL, "matmul_host: bad len=%d k=%d rows=%d", len,
				k, rows);
	if (len == 0)
		return 0;
	if (src == NULL || dst == NULL || coef == NULL)
		return ecg_fail(-ECG_DER_INVAL, "matmul_host: NULL argument");
	rc = ecg_ctx_enter(ctx);
	if (rc)
		return rc;
	if (place) {
		int ndev = 0;

		for (j = 0; j < k + rows; j++) {
			if (place[j] >= 0 && place[j] != ctx->device)
				return ecg_fail(-ECG_DER_INVAL, "matmul_host: %s %d is memory of device %d, not of the "
						"context's device %d", j < k ? "source" : "output", j < k ? j : j - k,
						place[j], ctx->device);
			ndev += place[j] >= 0;
		}
		if (ndev == k + rows)
			return matmul_device(ctx, len, k, rows, coef, src, dst, flags);
		if (ndev == 0)
			place = NULL;
	}
	pitch = ((size_t)len + 255) & ~(size_t)255;
	bytes = pitch * (size_t)(k + rows);
	rc = tstage_get(ctx, bytes, &t);
	if (rc)
		return rc;
	h = t->host;
	d = t->dev;
	/* host cells into the staging; device cells (mixed placement) stay put */
	for (j = 0; j < k; j++)
		if (!(place && place[j] >= 0))
			memcpy(h + j * pitch, src[j], (size_t)len);
	for (r = 0; r < rows; r++)
		if ((flags & ECG_F_ACCUMULATE) && !(place && place[k + r] >= 0))
			memcpy(h + (k + r) * pitch, dst[r], (size_t)len);
	if (bytes <= g_zero_copy_max) {
		/* small call: the kernel reads and writes the pinned staging over
		 * PCIe directly -- one launch instead of H2D + launch + D2H */
		void *hd = NULL;

		e = hipHostGetDevicePointer(&hd, h, 0);
		if (e != hipSuccess)
			return ecg_hip_fail(e, "matmul_host device view of staging");
		d = hd;
	} else {
		/* 1D: a lone synchronous call is latency-bound and the 2D copy
		 * path costs more per call (tools/bench_dropin.py: 1 MiB cells
		 * 435 -> 584 us with 2D) */
		e = hipMemcpyAsync(d, h, (flags & ECG_F_ACCUMULATE) ? bytes : pitch * k,
				   hipMemcpyHostToDevice, t->st);
		if (e != hipSuccess)
			return ecg_hip_fail(e, "matmul_host H2D");
	}
	/* cell offsets from the staging base d: a device cell's is its distance
	 * from d (one address space) */
	for (j = 0; j < k; j++)
		soff[j] = place && place[j] >= 0 ? (int64_t)((uintptr_t)src[j] - (uintptr_t)d) : (int64_t)(j * pitch);
	for (r = 0; r < rows; r++)
		doff[r] = place && place[k + r] >= 0 ? (int64_t)((uintptr_t)dst[r] - (uintptr_t)d)
						     : (int64_t)((k + r) * pitch);
	rc = launch_split(ctx, len, k, rows, coef, d, soff, d, doff, flags, t->st);
	if (rc)
		return rc;
	e = hipSuccess;
	if (d == (unsigned char *)t->dev)
		e = hipMemcpyAsync(h + k * pitch, d + k * pitch, pitch * rows, hipMemcpyDeviceToHost,
				   t->st);
	/* the caller is synchronous (ISA-L convention): poll rather than let the
	 * runtime put the thread to sleep and pay its wake-up */
	if (e == hipSuccess)
		while ((e = hipStreamQuery(t->st)) == hipErrorNotReady)
			;
	if (e != hipSuccess)
		return ecg_hip_fail(e, "matmul_host D2H");
	for (r = 0; r < rows; r++)
		if (!(place && place[k + r] >= 0))
			memcpy(dst[r], h + (k + r) * pitch, (size_t)len);
	return 0;
}

int ecg_matmul_host(ecg_ctx_t *ctx, int len, int k, int rows, const unsigned char *coef,
		    unsigned char *const *src, unsigned char *const *dst, unsigned flags)
{
	if (ctx == NULL)
		return ecg_fail(-ECG_DER_INVAL, "NULL context");
	if (len <= 0 || src == NULL || dst == NULL || k < 1 || k > ECG_MAX_K + 256 || rows < 1 || rows > 256)
		return ecg_matmul_host_mem(ctx, len, k, rows, coef, src, dst, flags, NULL);
	{
		signed char place[ECG_MAX_K + 256 + 256];
		int dev, rc = ecg_ctx_enter(ctx);

		if (rc == 0)
			rc = ecg_cells_place(src, k, dst, rows, (uint64_t)len, ecg_ptr_device, place, &dev);
		if (rc < 0)
			return rc;
		return ecg_matmul_host_mem(ctx, len, k, rows, coef, src, dst, flags, rc ? place : NULL);
	}
}
