/*
 * ecg_gf.c -- GF(2^8) field, encode/decode matrices and perm-table builder.
 *
 * Field: polynomial 0x11d, generator 2 -- the field of ISA-L (v2.31.1,
 * pinned at ref:utils/build.config:8) that DAOS's EC codec runs in.  The full
 * 256x256 product table is built by shift-and-reduce multiplication once
 * (64 KiB); everything here is setup-time host work, never on the data path.
 */
#include <stdlib.h>
#include <string.h>

#include "ecg_internal.h"

unsigned char ecg_gf_mul_tbl[256][256];
static unsigned char g_inv[256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static unsigned char peasant_mul(unsigned a, unsigned b)
{
	unsigned r = 0;

	while (b) {
		if (b & 1)
			r ^= a;
		a <<= 1;
		if (a & 0x100)
			a ^= 0x11d;
		b >>= 1;
	}
	return (unsigned char)r;
}

static void gf_build(void)
{
	unsigned a, b;

	for (a = 0; a < 256; a++)
		for (b = 0; b < 256; b++)
			ecg_gf_mul_tbl[a][b] = peasant_mul(a, b);
	g_inv[0] = 0;
	for (a = 1; a < 256; a++)
		for (b = 1; b < 256; b++)
			if (ecg_gf_mul_tbl[a][b] == 1) {
				g_inv[a] = (unsigned char)b;
				break;
			}
}

void ecg_gf_init(void)
{
	pthread_once(&g_once, gf_build);
}

unsigned char ecg_gf_mul(unsigned char a, unsigned char b)
{
	ecg_gf_init();
	return ecg_gf_mul_tbl[a][b];
}

unsigned char ecg_gf_inv(unsigned char a)
{
	ecg_gf_init();
	return g_inv[a];
}

/* Cauchy1: identity on the first k rows, 1/(i ^ j) on parity rows.
 * Same matrix as ISA-L gf_gen_cauchy1_matrix(a, k+p, k) called at
 * ref:src/object/obj_class.c:614. */
int ecg_gen_cauchy1(int k, int p, unsigned char *en)
{
	int i, j;

	if (k < 1 || p < 0 || k + p > 256 || en == NULL)
		return ecg_fail(-ECG_DER_INVAL, "gen_cauchy1: bad k=%d p=%d", k, p);
	ecg_gf_init();
	memset(en, 0, (size_t)(k + p) * k);
	for (i = 0; i < k; i++)
		en[i * k + i] = 1;
	for (i = k; i < k + p; i++)
		for (j = 0; j < k; j++)
			en[i * k + j] = g_inv[(unsigned char)(i ^ j)];
	return 0;
}

/* Gauss-Jordan inverse over GF(2^8) (ISA-L gf_invert_matrix contract,
 * ref:src/object/cli_ec.c:2223): `in` is consumed, singular -> error. */
int ecg_invert_matrix(unsigned char *in, unsigned char *out, int n)
{
	int c, r, i;

	if (n < 1 || in == NULL || out == NULL)
		return ecg_fail(-ECG_DER_INVAL, "invert_matrix: bad n=%d", n);
	ecg_gf_init();
	memset(out, 0, (size_t)n * n);
	for (i = 0; i < n; i++)
		out[i * n + i] = 1;
	for (c = 0; c < n; c++) {
		int piv = -1;

		for (r = c; r < n; r++)
			if (in[r * n + c]) {
				piv = r;
				break;
			}
		if (piv < 0)
			return ecg_fail(-ECG_DER_INVAL, "invert_matrix: singular");
		if (piv != c) {
			for (i = 0; i < n; i++) {
				unsigned char t = in[c * n + i];

				in[c * n + i] = in[piv * n + i];
				in[piv * n + i] = t;
				t = out[c * n + i];
				out[c * n + i] = out[piv * n + i];
				out[piv * n + i] = t;
			}
		}
		{
			const unsigned char *sc = ecg_gf_mul_tbl[g_inv[in[c * n + c]]];

			for (i = 0; i < n; i++) {
				in[c * n + i] = sc[in[c * n + i]];
				out[c * n + i] = sc[out[c * n + i]];
			}
		}
		for (r = 0; r < n; r++) {
			const unsigned char *f;

			if (r == c || in[r * n + c] == 0)
				continue;
			f = ecg_gf_mul_tbl[in[r * n + c]];
			for (i = 0; i < n; i++) {
				in[r * n + i] ^= f[in[c * n + i]];
				out[r * n + i] ^= f[out[c * n + i]];
			}
		}
	}
	return 0;
}

/*
 * Decode rows for a set of erased LOGICAL cells, following DAOS
 * obj_ec_recov_codec_init (ref:src/object/cli_ec.c:2152-2250):
 *   dec_idx = first k surviving cells, b = en[dec_idx], inv = b^-1,
 *   data cell e  -> row inv[e],  parity cell e -> row en[e] * inv,
 *   all p parity cells lost (and no data) -> plain re-encode (:2205-2210).
 * Rows are produced data-errors-first (out_idx says which cell each row
 * regenerates).  The reference indexes inv with the first er_data_nerrs
 * entries of its insertion-ordered list: a parity cell among them reads a
 * row past the k x k inverse inside its zero-filled (k+p) x k buffer
 * (:1963-1984), so the reference writes that parity cell as all zeros; data
 * cells it always gets right.  Producing rows data-first gives the
 * reference's bytes wherever the reference is right, and the true parity in
 * that one cell -- a deliberate divergence in a cell degraded reads never
 * return (tests/test_oracle.py pins the reference's zeros).
 */
int ecg_recov_rows(int k, int p, const unsigned char *en, const uint32_t *err_list,
		   int nerrs, unsigned char *rows, uint32_t *out_idx, uint32_t *dec_idx,
		   int *reused_encode)
{
	unsigned char b[ECG_MAX_K * ECG_MAX_K], inv[ECG_MAX_K * ECG_MAX_K];
	int in_err[ECG_MAX_K + ECG_MAX_P];
	int i, j, r, n = 0, data_nerrs = 0;

	if (k < 1 || k > ECG_MAX_K || p < 1 || p > ECG_MAX_P)
		return ecg_fail(-ECG_DER_INVAL, "recov: bad k=%d p=%d", k, p);
	if (nerrs > p)
		return ecg_fail(-ECG_DER_DATA_LOSS, "recov: %d erasures > p=%d", nerrs, p);
	if (nerrs < 1)
		return ecg_fail(-ECG_DER_INVAL, "recov: no erasures");
	ecg_gf_init();
	memset(in_err, 0, sizeof(in_err));
	for (i = 0; i < nerrs; i++) {
		if (err_list[i] >= (uint32_t)(k + p))
			return ecg_fail(-ECG_DER_INVAL, "recov: cell %u out of range", err_list[i]);
		if (in_err[err_list[i]])
			return ecg_fail(-ECG_DER_INVAL, "recov: duplicate cell %u", err_list[i]);
		in_err[err_list[i]] = 1;
		if (err_list[i] < (uint32_t)k)
			data_nerrs++;
	}
	*reused_encode = 0;
	if (data_nerrs == 0 && nerrs == p) {
		for (i = 0; i < p; i++) {
			memcpy(&rows[i * k], &en[(k + i) * k], k);
			out_idx[i] = (uint32_t)(k + i);
		}
		for (i = 0; i < k; i++)
			dec_idx[i] = (uint32_t)i;
		*reused_encode = 1;
		return 0;
	}
	for (i = 0, r = 0; i < k; i++, r++) {
		while (in_err[r])
			r++;
		memcpy(&b[i * k], &en[r * k], k);
		dec_idx[i] = (uint32_t)r;
	}
	if (ecg_invert_matrix(b, inv, k) != 0)
		return ecg_fail(-ECG_DER_INVAL, "recov: singular survivor matrix");
	/* data errors first, in list order */
	for (i = 0; i < nerrs; i++) {
		if (err_list[i] >= (uint32_t)k)
			continue;
		memcpy(&rows[n * k], &inv[err_list[i] * k], k);
		out_idx[n++] = err_list[i];
	}
	for (i = 0; i < nerrs; i++) {
		const unsigned char *e;

		if (err_list[i] < (uint32_t)k)
			continue;
		e = &en[err_list[i] * k];
		for (j = 0; j < k; j++) {
			unsigned char s = 0;
			int t;

			for (t = 0; t < k; t++)
				s ^= ecg_gf_mul_tbl[e[t]][inv[t * k + j]];
			rows[n * k + j] = s;
		}
		out_idx[n++] = err_list[i];
	}
	return 0;
}

int ecg_recov_matrix(int k, int p, const unsigned char *en_matrix, const uint32_t *err_list,
		     int nerrs, unsigned char *de_rows, uint32_t *dec_idx, int *reused_encode)
{
	unsigned char rows[ECG_MAX_P * ECG_MAX_K];
	uint32_t out_idx[ECG_MAX_P];
	int rc, i, n;

	if (en_matrix == NULL || err_list == NULL || de_rows == NULL || dec_idx == NULL ||
	    reused_encode == NULL)
		return ecg_fail(-ECG_DER_INVAL, "recov_matrix: NULL argument");
	rc = ecg_recov_rows(k, p, en_matrix, err_list, nerrs, rows, out_idx, dec_idx,
			    reused_encode);
	if (rc)
		return rc;
	/* hand rows back in the caller's err_list order */
	for (i = 0; i < nerrs; i++)
		for (n = 0; n < nerrs; n++)
			if (out_idx[n] == err_list[i])
				memcpy(&de_rows[i * k], &rows[n * k], k);
	return 0;
}

/* Perm tables for one coefficient (see ecg_kabi.h). */
void ecg_build_ptbl(unsigned char c, ecg_ptbl_t *t)
{
	const unsigned char *m = ecg_gf_mul_tbl[c];
	uint32_t lo0 = 0, hi0 = 0, lo1 = 0, hi1 = 0, t2 = 0;
	int i;

	for (i = 0; i < 4; i++) {
		lo0 |= (uint32_t)m[i] << (8 * i);
		hi0 |= (uint32_t)m[i + 4] << (8 * i);
		lo1 |= (uint32_t)m[i << 3] << (8 * i);
		hi1 |= (uint32_t)m[(i + 4) << 3] << (8 * i);
		t2 |= (uint32_t)m[i << 6] << (8 * i);
	}
	t->t0lo = lo0;
	t->t0hi = hi0;
	t->t1lo = lo1;
	t->t1hi = hi1;
	t->t2 = t2;
}
