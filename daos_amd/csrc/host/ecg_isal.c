/*
 * ecg_isal.c -- ISA-L-signature exports (see include/ecg_isal.h).
 *
 * Setup functions (matrices, tables) are host code, as in ISA-L.  The
 * data-plane functions (ec_encode_data, ec_encode_data_update, xor_gen) go
 * through ecg_dropin_product (ecg_dropin.c): device cells run the gfx950
 * kernels in place, host cells run the product's CPU path below the measured
 * crossover and in every process without a usable gfx950 device -- ISA-L's
 * contract is a `void` call that succeeds on any CPU, and libdaos (the
 * client library, ref:src/object/SConscript:19-23) calls ec_encode_data
 * (ref:src/object/cli_ec.c:540) on nodes without a GPU.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../../include/ecg_isal.h"
#include "ecg_internal.h"

/* The ISA-L data-plane ABI is `void`: a failure cannot be returned, and
 * silently skipping the parity would corrupt stored objects.  What is left to
 * fail once host cells always have the CPU path is a call on device cells
 * (the GPU is then the only thing that can reach them) or bad arguments:
 * name the cause and the remedy, then abort. */
static void die(const char *fn, int rc)
{
	fprintf(stderr, "ecg: %s failed (rc=%d): %s\n"
		"ecg: host cells never fail this way (they run on the CPU when no GPU is usable); for "
		"device cells list their device in $ECG_DEVICES and check the HIP runtime (rocminfo), "
		"or pass host buffers\n", fn, rc, ecg_strerror());
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

	const unsigned char *m = ecg_gf_mul_tbl[c];

	if (t[0] != 0 || t[16] != 0 || t[2] != m[2] || t[15] != m[15] || t[17] != m[0x10] ||
	    t[31] != m[0xF0]) {
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

	ecg_gf_init();
	for (i = 0; i < k * rows; i++)
		coef[i] = table_coef(fn, gftbls + 32 * i);
}

void ec_encode_data(int len, int k, int rows, unsigned char *gftbls, unsigned char **data,
		    unsigned char **coding)
{
	unsigned char small[ECG_MAX_K * 8];
	unsigned char *coef = small;
	int rc;

	if (len <= 0 || rows <= 0 || k <= 0)
		return;
	if (k > ECG_MAX_K || rows > 256)
		die("ec_encode_data (k/rows out of range)", -ECG_DER_INVAL);
	/* a user-level thread's stack is small: only rows > 8 take the heap */
	if ((size_t)k * rows > sizeof(small) && (coef = malloc((size_t)k * rows)) == NULL)
		die("ec_encode_data (malloc)", -ECG_DER_NOMEM);
	coef_from_tables("ec_encode_data", k, rows, gftbls, coef);
	rc = ecg_dropin_product("ec_encode_data", NULL, len, k, rows, coef, data, coding, 0);
	if (coef != small)
		free(coef);
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
	ecg_gf_init();
	for (r = 0; r < rows; r++)
		coef[r] = table_coef("ec_encode_data_update", gftbls + 32 * (r * k + vec_i));
	src[0] = data;
	rc = ecg_dropin_product("ec_encode_data_update", NULL, len, 1, rows, coef, src, coding,
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
	rc = ecg_dropin_product("xor_gen", NULL, len, vects - 1, 1, ones, v, &v[vects - 1], 0);
	if (rc)
		die("xor_gen", rc);
	return 0;
}
