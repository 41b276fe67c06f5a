/*
 * ecg_dropin.c -- where a synchronous one-stripe product of the drop-in
 * surfaces runs (ISA-L ec_encode_data / ec_encode_data_update / xor_gen in
 * ecg_isal.c; obj_ec_encode_buf, agg_* and singv in ecg_daos.c).
 *
 * The rule ("CPU for small len, GPU via staging above a
 * threshold"):
 *   - every cell device memory (hipMalloc'd)        -> HIP kernels, in place;
 *   - host and device cells mixed (host bio buffers,
 *     parity in HBM)                                  -> HIP kernels, the host
 *                                                       cells through pinned
 *                                                       staging;
 *   - host cells, len * (k + rows) >= crossover       -> HIP kernels through
 *                                                       pinned staging;
 *   - host cells below the crossover, every call in a process without a
 *     usable gfx950 device, and ECG_FORCE_CPU=1       -> the CPU path
 *                                                       (ecg_cpu.c).
 * Placement is decided from EVERY cell (ecg_cells_place), so a device address
 * never reaches the CPU path; cells of two devices in one call, or a device
 * cell past its allocation, fail with the cell named.
 * The default crossover is the measured one for the CPU path in use
 * (crossover_for_isa below, DESIGN.md §7: on the MI355X box one EPYC core with
 * GFNI beats the PCIe round trip of a synchronous call at every size, so with
 * GFNI host cells stay on the CPU; the nibble-table and scalar paths hand
 * large calls to the GPU); ECG_DROPIN_CROSSOVER=<bytes> or
 * ecg_set_dropin_crossover() move it.
 *
 * Contexts: one per device of $ECG_DEVICES ("0,1,2,3" / "all"; default
 * $ECG_DEVICE, else device 0), created on the first call that needs the GPU;
 * calling threads are spread over them round-robin on their first such call,
 * so an engine's xstreams use every listed GPU.  Device cells run on the
 * context of their own device.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ecg_internal.h"

#define DROPIN_MAXDEV 64

/* Measured crossover in bytes of len * (k + rows), by the CPU path the
 * process runs (ecg_cpu_isa(): the one-thread synchronous call on the CPU vs
 * the GPU through pinned staging, EC_4P2 / EC_8P2 / EC_16P2 with 4 KiB - 4 MiB
 * cells on the MI355X box's EPYC 9575F, tools/dropin_bench.c with
 * $ECG_CPU_ISA forcing each variant; DESIGN.md §7, profiles/r06/dropin_isa/):
 *   GFNI (avx512 / avx2)  the CPU ahead at every size: never the GPU
 *   avx2 (nibble tables)  the CPU ahead below 64 MiB (16P2 x 4 MiB = 72 MiB
 *                         ties: 4.10 vs 4.08 ms)
 *   scalar                the GPU ahead from 64 KiB (16P2 x 4 KiB = 72 KiB:
 *                         17.5 vs 27.2 us; 8P2 x 4 KiB = 40 KiB: 17.9 vs 13.9)
 * $ECG_DROPIN_CROSSOVER or ecg_set_dropin_crossover() replace it. */
static uint64_t crossover_for_isa(const char *isa)
{
	if (strstr(isa, "gfni"))
		return UINT64_MAX;
	if (strcmp(isa, "avx2") == 0)
		return 64ull << 20;
	return 64ull << 10;
}

static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static int g_gpu;		/* a gfx950 device is visible */
static int g_force_cpu;		/* ECG_FORCE_CPU=1: host cells never take the GPU */
static uint64_t g_crossover;	/* explicit crossover (g_crossover_set) */
static int g_crossover_set;

static pthread_once_t g_ctx_once = PTHREAD_ONCE_INIT;
static ecg_ctx_t *g_ctx[DROPIN_MAXDEV];
static int g_nctx;
static int g_ctx_rc;
static char g_ctx_err[256];
static unsigned g_next;
static __thread ecg_ctx_t *t_ctx;
static int g_warned;

static void once_init(void)
{
	const char *force = getenv("ECG_FORCE_CPU");
	const char *x = getenv("ECG_DROPIN_CROSSOVER");

	if (x && *x) {
		g_crossover = strtoull(x, NULL, 0);
		g_crossover_set = 1;
	}
	g_force_cpu = force && force[0] == '1';
	g_gpu = ecg_device_count() > 0;
}

static void ctx_init(void)
{
	const char *list = getenv("ECG_DEVICES");
	const char *one = getenv("ECG_DEVICE");
	int dev[DROPIN_MAXDEV], n, i;

	if (list) {
		n = ecg_parse_devices(list, dev, DROPIN_MAXDEV);
	} else {
		dev[0] = one ? atoi(one) : 0;
		n = 1;
	}
	if (n <= 0) {
		g_ctx_rc = n < 0 ? ecg_fail(-ECG_DER_INVAL, "bad ECG_DEVICES '%s'", list)
				 : ecg_fail(-ECG_DER_NOSYS, "ECG_DEVICES names no device");
	}
	for (i = 0; i < n && g_ctx_rc == 0; i++)
		g_ctx_rc = ecg_ctx_create(dev[i], &g_ctx[i]);
	if (g_ctx_rc) {
		snprintf(g_ctx_err, sizeof(g_ctx_err), "%s", ecg_strerror());
		while (i-- > 0)
			if (g_ctx[i]) {
				ecg_ctx_destroy(g_ctx[i]);
				g_ctx[i] = NULL;
			}
		n = 0;
	}
	g_nctx = n;
}

int ecg_dropin_gpu(void)
{
	pthread_once(&g_once, once_init);
	return g_gpu;
}

int ecg_set_dropin_crossover(uint64_t bytes)
{
	pthread_once(&g_once, once_init);
	__atomic_store_n(&g_crossover, bytes, __ATOMIC_RELAXED);
	__atomic_store_n(&g_crossover_set, 1, __ATOMIC_RELEASE);
	return 0;
}

int ecg_dropin_host_on_cpu(uint64_t bytes)
{
	(void)ecg_dropin_gpu();		/* reads the environment once */
	return g_force_cpu || bytes < ecg_dropin_crossover();
}

uint64_t ecg_dropin_crossover(void)
{
	pthread_once(&g_once, once_init);
	/* the default follows the CPU path in use (ecg_cpu_set_isa may narrow it) */
	if (!__atomic_load_n(&g_crossover_set, __ATOMIC_ACQUIRE))
		return crossover_for_isa(ecg_cpu_isa());
	return __atomic_load_n(&g_crossover, __ATOMIC_RELAXED);
}

/* The calling thread's default context (NULL + error text when the devices
 * of $ECG_DEVICES cannot be opened). */
static ecg_ctx_t *thread_ctx(void)
{
	pthread_once(&g_ctx_once, ctx_init);
	if (g_ctx_rc) {
		ecg_fail(g_ctx_rc, "%s", g_ctx_err);
		return NULL;
	}
	if (t_ctx == NULL)
		t_ctx = g_ctx[__atomic_fetch_add(&g_next, 1u, __ATOMIC_RELAXED) % (unsigned)g_nctx];
	return t_ctx;
}

/* The context of device `dev` among the default ones. */
static ecg_ctx_t *device_ctx(const char *fn, int dev)
{
	ecg_ctx_t *c = thread_ctx();
	int i;

	if (c == NULL || ecg_ctx_device(c) == dev)
		return c;
	for (i = 0; i < g_nctx; i++)
		if (ecg_ctx_device(g_ctx[i]) == dev)
			return g_ctx[i];
	ecg_fail(-ECG_DER_INVAL, "%s: cells are memory of device %d, which $ECG_DEVICES does not list "
		 "(add it to ECG_DEVICES)", fn, dev);
	return NULL;
}

/*
 * Where does a call's src[0] live?  The HIP runtime's pointer queries take a
 * process-wide lock: 0.08 us alone, 7.4 us per query with 16 threads asking
 * at once (tools/hipcall_cost.hip, profiles/r05/dropin/), which capped 16
 * threads of 32 KiB host-cell calls at 212 GiB/s against 1417 GiB/s with no
 * query at all (tools/dropin_threads.c).  So each thread remembers, for
 * HOSTC_TTL_NS, the 2 MiB regions in which it found memory the runtime does
 * not know at all (plain malloc / mmap -- DAOS's sgl and bio buffers).  Such
 * a region cannot hold a device allocation: ROCm carves those out of GPU
 * apertures it reserves at initialisation, apart from ordinary mappings; the
 * expiry is a second guard.  Runtime-known host memory (pinned, registered,
 * managed -- which may share an aperture with device allocations) and device
 * answers are never cached.  ECG_DROPIN_HOSTCACHE=0 queries every call.
 */
#define HOSTC_N 8
#define HOSTC_TTL_NS 10000000ull	/* 10 ms */
static __thread struct {
	uintptr_t region;	/* (address >> 21) + 1; 0 = empty */
	uint64_t until;
} t_hostc[HOSTC_N];
static int g_hostc = -1;

static uint64_t coarse_ns(void)
{
	struct timespec t;

	clock_gettime(CLOCK_MONOTONIC_COARSE, &t);
	return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

static int cell_device(const void *p)
{
	const uintptr_t region = ((uintptr_t)p >> 21) + 1;
	const unsigned slot = (unsigned)(region * 0x9E3779B1u) >> 29;	/* top 3 bits: 0..7 */
	uint64_t now;
	int dev;

	if (__atomic_load_n(&g_hostc, __ATOMIC_RELAXED) < 0) {
		const char *env = getenv("ECG_DROPIN_HOSTCACHE");

		__atomic_store_n(&g_hostc, !(env && env[0] == '0'), __ATOMIC_RELAXED);
	}
	if (!__atomic_load_n(&g_hostc, __ATOMIC_RELAXED))
		return ecg_ptr_device(p);
	now = coarse_ns();
	if (t_hostc[slot].region == region && now < t_hostc[slot].until)
		return ECG_PTR_UNKNOWN;
	dev = ecg_ptr_device(p);
	if (dev == ECG_PTR_UNKNOWN) {
		t_hostc[slot].region = region;
		t_hostc[slot].until = now + HOSTC_TTL_NS;
	}
	return dev;
}

int ecg_ptr_device_cached(const void *p)
{
	return cell_device(p);
}

ecg_ctx_t *ecg_dropin_ctx(void)
{
	return ecg_dropin_gpu() && !g_force_cpu ? thread_ctx() : NULL;
}

int ecg_dropin_product(const char *fn, ecg_ctx_t *ctx, int len, int k, int rows, const unsigned char *coef,
		       unsigned char *const *src, unsigned char *const *dst, unsigned flags)
{
	signed char place[ECG_MAX_K + 256 + 256];
	int dev, ndev, rc;

	if (len <= 0 || src == NULL || dst == NULL || k < 1 || k > ECG_MAX_K + 256 || rows < 1 || rows > 256)
		return ecg_cpu_matmul(len, k, rows, coef, src, dst, flags);
	if (!ecg_dropin_gpu())
		return ecg_cpu_matmul(len, k, rows, coef, src, dst, flags);
	/* where every cell is, not only src[0]: a device address must never
	 * reach the CPU path (it would fault there), and a call mixing host and
	 * device cells -- host bio buffers, parity kept in HBM -- runs on that
	 * device with its host cells staged */
	ndev = ecg_cells_place(src, k, dst, rows, (uint64_t)len, cell_device, place, &dev);
	if (ndev < 0)
		return ndev;	/* ecg_strerror() names the cell; the caller names fn */
	if (ndev > 0) {
		/* device cells: only the GPU can touch them */
		if (ctx == NULL || ecg_ctx_device(ctx) != dev)
			ctx = device_ctx(fn, dev);
		if (ctx == NULL)
			return g_ctx_rc ? g_ctx_rc : -ECG_DER_INVAL;
		return ecg_matmul_host_mem(ctx, len, k, rows, coef, src, dst, flags, place);
	}
	if (g_force_cpu || (uint64_t)len * (uint64_t)(k + rows) < ecg_dropin_crossover())
		return ecg_cpu_matmul(len, k, rows, coef, src, dst, flags);
	if (ctx == NULL)
		ctx = thread_ctx();
	if (ctx != NULL) {
		rc = ecg_matmul_host_mem(ctx, len, k, rows, coef, src, dst, flags, NULL);
		if (rc == 0)
			return 0;
	}
	/* host cells: the CPU computes the same bytes, so a GPU that cannot be
	 * used (not openable, a HIP failure) costs speed, never parity */
	if (!__atomic_exchange_n(&g_warned, 1, __ATOMIC_RELAXED))
		fprintf(stderr, "ecg: %s: GPU path unavailable (%s); host cells run on the CPU\n", fn,
			ecg_strerror());
	return ecg_cpu_matmul(len, k, rows, coef, src, dst, flags);
}
