/*
 * ecg_isal.c -- ISA-L-signature exports (see include/ecg_isal.h).
 *
 * Setup functions (matrices, tables) are host code, as in ISA-L.  The
 * data-plane functions run on the MI355X through ecg_matmul_host; there is
 * deliberately no CPU path.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../../include/ecg_isal.h"
#include "ecg_internal.h"

int ecg_matmul_host(ecg_ctx_t *ctx, int len, int k, int rows, const unsigned char *coef,
		    unsigned char *const *src, unsigned char *const *dst, unsigned flags);

/* One context per device of $ECG_DEVICES ("0,1,2,3" / "all"; default
 * $ECG_DEVICE, else device 0).  Calling threads are spread over them
 * round-robin on their first call, so an engine's xstreams calling the
 * synchronous ISA-L API use every listed GPU. */
#define ISAL_MAXDEV 64
static ecg_ctx_t *g_ctx[ISAL_MAXDEV];
static int g_nctx;
static int g_ctx_rc;
static unsigned g_next;
static pthread_once_t g_ctx_once = PTHREAD_ONCE_INIT;
static __thread ecg_ctx_t *t_ctx;

static void default_ctx_init(void)
{
	const char *list = getenv("ECG_DEVICES");
	const char *one = getenv("ECG_DEVICE");
	int dev[ISAL_MAXDEV], n, i;

	if (list) {
		n = ecg_parse_devices(list, dev, ISAL_MAXDEV);
	} else {
		dev[0] = one ? atoi(one) : 0;
		n = 1;
	}
	if (n <= 0) {
		g_ctx_rc = n < 0 ? ecg_fail(-ECG_DER_INVAL, "bad ECG_DEVICES '%s'", list)
				 : ecg_fail(-ECG_DER_NOSYS, "ECG_DEVICES: no device");
		return;
	}
	for (i = 0; i < n && g_ctx_rc == 0; i++)
		g_ctx_rc = ecg_ctx_create(dev[i], &g_ctx[i]);
	g_nctx = i;
}

/* The ISA-L data-plane ABI is `void`: a failure cannot be returned, and
 * silently skipping the parity would corrupt stored objects.  Fail loudly. */
static void die(const char *fn, int rc)
{
	fprintf(stderr, "ecg: %s failed (rc=%d): %s\n", fn, rc, ecg_strerror());
	abort();
}

static ecg_ctx_t *default_ctx(const char *fn)
{
	pthread_once(&g_ctx_once, default_ctx_init);
	if (g_ctx_rc)
		die(fn, g_ctx_rc);
	if (t_ctx == NULL)
		t_ctx = g_ctx[__atomic_fetch_add(&g_next, 1u, __ATOMIC_RELAXED) % (unsigned)g_nctx];
	return t_ctx;
}

/* The context for a call's cells: the thread's for host cells (staged), the
 * one on the cells' own device for device cells (used in place; a device not
 * in $ECG_DEVICES is an error, not a silent peer access). */
static ecg_ctx_t *ctx_for(const char *fn, const void *cell)
{
	ecg_ctx_t *c = default_ctx(fn);
	const int dev = ecg_ptr_device(cell);
	int i;

	if (dev < 0 || ecg_ctx_device(c) == dev)
		return c;
	for (i = 0; i < g_nctx; i++)
		if (ecg_ctx_device(g_ctx[i]) == dev)
			return g_ctx[i];
	fprintf(stderr, "ecg: %s: cells in memory of device %d, which $ECG_DEVICES does not list\n", fn, dev);
	abort();
}

void gf_vect_mul_init(unsigned char c, unsigned char *tbl)
{
	int n;

	ecg_gf_init();
	for (n = 0; n < 16; n++) {
		tbl[n] = ecg_gf_mul_tbl[c][n];
		tbl[16 + n] = ecg_gf_mul_tbl[c][n << 4];
	}
}

void ec_init_tables(int k, int rows, unsigned char *a, unsigned char *gftbls)
{
	int i;

	for (i = 0; i < k * rows; i++)
		gf_vect_mul_init(a[i], gftbls + 32 * i);
}

/* The coefficient of each 32-byte table is its byte 1 (c * 1).  The tables
 * must be ec_init_tables' base/AVX2 layout [c*0..c*15 | c*0x00..c*0xF0]; a
 * libisal ec_init_tables resolved first in the process may emit its GFNI
 * layout instead, and reading that as coefficients would
 * silently corrupt parity -- so check and die instead. */
static unsigned char table_coef(const char *fn, const unsigned char *t)
{
	const unsigned char c = t[1];

	if (t[0] != 0 || t[16] != 0 || t[2] != ecg_gf_mul(c, 2) || t[15] != ecg_gf_mul(c, 15) ||
	    t[17] != ecg_gf_mul(c, 0x10) || t[31] != ecg_gf_mul(c, 0xF0)) {
		fprintf(stderr, "ecg: %s: gftbls are not ec_init_tables' 32-byte layout "
			"(tables from another ISA-L build?)\n", fn);
		abort();
	}
	return c;
}

static void coef_from_tables(const char *fn, int k, int rows, const unsigned char *gftbls,
			     unsigned char *coef)
{
	int i;

	for (i = 0; i < k * rows; i++)
		coef[i] = table_coef(fn, gftbls + 32 * i);
}

void ec_encode_data(int len, int k, int rows, unsigned char *gftbls, unsigned char **data,
		    unsigned char **coding)
{
	unsigned char coef[ECG_MAX_K * 256];
	int rc;

	if (len <= 0 || rows <= 0 || k <= 0)
		return;
	if (k > ECG_MAX_K || rows > 256)
		die("ec_encode_data (k/rows out of range)", -ECG_DER_INVAL);
	coef_from_tables("ec_encode_data", k, rows, gftbls, coef);
	rc = ecg_matmul_host(ctx_for("ec_encode_data", data[0]), len, k, rows, coef, data, coding, 0);
	if (rc)
		die("ec_encode_data", rc);
}

void ec_encode_data_update(int len, int k, int rows, int vec_i, unsigned char *gftbls,
			   unsigned char *data, unsigned char **coding)
{
	unsigned char coef[256];
	unsigned char *src[1];
	int r, rc;

	if (len <= 0 || rows <= 0)
		return;
	if (rows > 256 || vec_i < 0 || vec_i >= k)
		die("ec_encode_data_update (bad arguments)", -ECG_DER_INVAL);
	for (r = 0; r < rows; r++)
		coef[r] = table_coef("ec_encode_data_update", gftbls + 32 * (r * k + vec_i));
	src[0] = data;
	rc = ecg_matmul_host(ctx_for("ec_encode_data_update", data), len, 1, rows, coef, src, coding,
			     ECG_F_ACCUMULATE);
	if (rc)
		die("ec_encode_data_update", rc);
}

unsigned char gf_mul(unsigned char a, unsigned char b)
{
	return ecg_gf_mul(a, b);
}

unsigned char gf_inv(unsigned char a)
{
	return ecg_gf_inv(a);
}

void gf_gen_cauchy1_matrix(unsigned char *a, int m, int k)
{
	(void)ecg_gen_cauchy1(k, m - k, a);
}

/* ISA-L gf_gen_rs_matrix: identity, then rows of consecutive powers of
 * successive generators 1, 2, 4, ... (Vandermonde-like; not used by DAOS). */
void gf_gen_rs_matrix(unsigned char *a, int m, int k)
{
	unsigned char gen = 1;
	int i, j;

	ecg_gf_init();
	memset(a, 0, (size_t)k * m);
	for (i = 0; i < k; i++)
		a[k * i + i] = 1;
	for (i = k; i < m; i++) {
		unsigned char v = 1;

		for (j = 0; j < k; j++) {
			a[k * i + j] = v;
			v = ecg_gf_mul_tbl[v][gen];
		}
		gen = ecg_gf_mul_tbl[gen][2];
	}
}

int gf_invert_matrix(unsigned char *in, unsigned char *out, const int n)
{
	return ecg_invert_matrix(in, out, n) == 0 ? 0 : -1;
}

int xor_gen(int vects, int len, void **array)
{
	unsigned char ones[ECG_MAX_K + 256];
	unsigned char **v = (unsigned char **)array;
	int rc;

	if (vects < 3)
		return 1;
	if (len <= 0)
		return 0;
	if (vects - 1 > ECG_MAX_K + 256)
		return 1;
	memset(ones, 1, sizeof(ones));
	rc = ecg_matmul_host(ctx_for("xor_gen", v[0]), len, vects - 1, 1, ones, v, &v[vects - 1], 0);
	if (rc)
		die("xor_gen", rc);
	return 0;
}
