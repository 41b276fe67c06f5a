/*
 * ec_ref.c -- scalar CPU ORACLE (test infrastructure only; see ec_ref.h).
 *
 * Restates ISA-L v2.31.1 erasure_code/ec_base.c semantics (external, pinned at
 * ref:utils/build.config:8, not present in /root/reference) and the DAOS
 * matrix logic around it.  Each function cites the DAOS call site it serves.
 * Parity unpinned by any reference fixture -- see ec_ref.h header.
 */
#include "ec_ref.h"

#include <stdlib.h>
#include <string.h>

/* --------------------------------------------------------------------------
 * GF(2^8): primitive polynomial x^8+x^4+x^3+x^2+1 (0x11d), generator 2.
 * Log/antilog tables built once (ISA-L ships them precomputed as
 * gff_base / gflog_base; values are identical by construction).
 * ------------------------------------------------------------------------ */
static unsigned char g_exp[256];
static unsigned char g_log[256];
static int g_ready;

static void gf_tables_init(void)
{
	unsigned int x = 1;
	int i;

	if (g_ready)
		return;
	for (i = 0; i < 255; i++) {
		g_exp[i] = (unsigned char)x;
		g_log[x] = (unsigned char)i;
		x <<= 1;
		if (x & 0x100)
			x ^= 0x11d;
	}
	g_exp[255] = g_exp[0];	/* exp[255] == 1, used by gf_inv(1) */
	g_log[0] = 0;		/* never consulted: gf_mul/gf_inv test for zero */
	g_ready = 1;
}

/* ISA-L gf_mul: 0 if either operand is 0, else exp[(log a + log b) mod 255].
 * DAOS use: ref:src/object/cli_ec.c:2239 */
unsigned char ref_gf_mul(unsigned char a, unsigned char b)
{
	int s;

	gf_tables_init();
	if (a == 0 || b == 0)
		return 0;
	s = g_log[a] + g_log[b];
	if (s > 254)
		s -= 255;
	return g_exp[s];
}

/* ISA-L gf_inv: 0 -> 0, else exp[255 - log a]. */
unsigned char ref_gf_inv(unsigned char a)
{
	gf_tables_init();
	if (a == 0)
		return 0;
	return g_exp[255 - g_log[a]];
}

/* ISA-L gf_gen_cauchy1_matrix(a, m, k): identity on the top k rows, then
 * a[i][j] = 1/(i ^ j) for i in [k, m).  DAOS: ref:src/object/obj_class.c:614 */
void ref_gf_gen_cauchy1_matrix(unsigned char *a, int m, int k)
{
	int i, j;

	memset(a, 0, (size_t)m * k);
	for (i = 0; i < k; i++)
		a[(size_t)k * i + i] = 1;
	for (i = k; i < m; i++)
		for (j = 0; j < k; j++)
			a[(size_t)k * i + j] = ref_gf_inv((unsigned char)(i ^ j));
}

/* ISA-L gf_invert_matrix(in, out, n): Gauss-Jordan over GF(2^8); `in` is
 * destroyed; -1 when singular.  The inverse is unique, so the pivot order
 * cannot change the output.  DAOS: ref:src/object/cli_ec.c:2223 */
int ref_gf_invert_matrix(unsigned char *in, unsigned char *out, int n)
{
	int col, r, c;

	memset(out, 0, (size_t)n * n);
	for (r = 0; r < n; r++)
		out[(size_t)r * n + r] = 1;

	for (col = 0; col < n; col++) {
		unsigned char piv_inv;

		if (in[(size_t)col * n + col] == 0) {
			int sw;

			for (sw = col + 1; sw < n; sw++)
				if (in[(size_t)sw * n + col] != 0)
					break;
			if (sw == n)
				return -1;
			for (c = 0; c < n; c++) {
				unsigned char t;

				t = in[(size_t)col * n + c];
				in[(size_t)col * n + c] = in[(size_t)sw * n + c];
				in[(size_t)sw * n + c] = t;
				t = out[(size_t)col * n + c];
				out[(size_t)col * n + c] = out[(size_t)sw * n + c];
				out[(size_t)sw * n + c] = t;
			}
		}
		piv_inv = ref_gf_inv(in[(size_t)col * n + col]);
		for (c = 0; c < n; c++) {
			in[(size_t)col * n + c] = ref_gf_mul(in[(size_t)col * n + c], piv_inv);
			out[(size_t)col * n + c] = ref_gf_mul(out[(size_t)col * n + c], piv_inv);
		}
		for (r = 0; r < n; r++) {
			unsigned char f;

			if (r == col)
				continue;
			f = in[(size_t)r * n + col];
			if (f == 0)
				continue;
			for (c = 0; c < n; c++) {
				in[(size_t)r * n + c] ^= ref_gf_mul(f, in[(size_t)col * n + c]);
				out[(size_t)r * n + c] ^= ref_gf_mul(f, out[(size_t)col * n + c]);
			}
		}
	}
	return 0;
}

/* ISA-L gf_vect_mul_init(c, tbl): tbl[0..15] = c*{0..15},
 * tbl[16..31] = c*{0x00,0x10,...,0xf0}.  ec_init_tables applies it to every
 * coefficient of the rows x k matrix, row-major, 32 B each.
 * DAOS: ref:src/object/obj_class.c:616-617, ref:src/object/cli_ec.c:2246-2247 */
void ref_ec_init_tables(int k, int rows, const unsigned char *a, unsigned char *gftbls)
{
	int i, n;

	for (i = 0; i < k * rows; i++) {
		unsigned char c = a[i];

		for (n = 0; n < 16; n++) {
			gftbls[32 * i + n] = ref_gf_mul(c, (unsigned char)n);
			gftbls[32 * i + 16 + n] = ref_gf_mul(c, (unsigned char)(n << 4));
		}
	}
}

/* ISA-L ec_encode_data_base: coding[l][i] = XOR_j gf_mul(data[j][i], c[l][j])
 * where c[l][j] = gftbls[32*(l*k+j) + 1] (entry "c*1" of the nibble table).
 * DAOS: ref:src/object/cli_ec.c:540,571,2641; srv_ec_aggregate.c:693,1136 */
void ref_ec_encode_data(int len, int k, int rows, const unsigned char *gftbls,
			unsigned char **data, unsigned char **coding)
{
	int l, i, j;

	for (l = 0; l < rows; l++) {
		for (i = 0; i < len; i++) {
			unsigned char s = 0;

			for (j = 0; j < k; j++)
				s ^= ref_gf_mul(data[j][i], gftbls[32 * (l * k + j) + 1]);
			coding[l][i] = s;
		}
	}
}

/* ISA-L ec_encode_data_update_base: coding[l][i] ^= gf_mul(data[i], c[l][vec_i]).
 * DAOS: ref:src/object/srv_ec_aggregate.c:1099-1101 */
void ref_ec_encode_data_update(int len, int k, int rows, int vec_i,
			       const unsigned char *gftbls, const unsigned char *data,
			       unsigned char **coding)
{
	int l, i;

	for (l = 0; l < rows; l++) {
		unsigned char c = gftbls[32 * (l * k + vec_i) + 1];

		for (i = 0; i < len; i++)
			coding[l][i] ^= ref_gf_mul(data[i], c);
	}
}

/* ISA-L xor_gen(vects, len, array): array[vects-1] = XOR of array[0..vects-2].
 * The SIMD ISA-L versions reject fewer than two sources (returns non-zero).
 * DAOS: ref:src/object/srv_ec_aggregate.c:1089-1092 (vects = 3). */
int ref_xor_gen(int vects, int len, void **array)
{
	unsigned char **v = (unsigned char **)array;
	int i, j;

	if (vects < 3)
		return 1;
	for (i = 0; i < len; i++) {
		unsigned char x = v[0][i];

		for (j = 1; j < vects - 1; j++)
			x ^= v[j][i];
		v[vects - 1][i] = x;
	}
	return 0;
}

/* DAOS obj_ec_recov_codec_init (ref:src/object/cli_ec.c:2152-2250),
 * restated with logical indices.  Faithful to the reference, including:
 *  - nerrs > p -> -DER_DATA_LOSS (:2169-2174)
 *  - all p parity lost and no data lost -> reuse encode tables (:2205-2210)
 *  - b = rows of the first k surviving logical cells (:2213-2220)
 *  - data-error rows taken from inv for the first er_data_nerrs entries of
 *    err_list (:2226-2231) -- the reference assumes data errors come first;
 *    callers that pass parity errors first get what the reference gets.
 *    The inverse lives in a buffer of roundup((k+p)*k, 8) bytes from a
 *    zeroing D_ALLOC (obj_ec_recov_codec_alloc, :1963-1984; D_ALLOC ->
 *    d_calloc, ref:src/include/gurt/common.h:143-146,308) of which
 *    gf_invert_matrix writes only the k x k head (:2223), so a parity cell
 *    listed among the first er_data_nerrs entries reads an all-zero row of
 *    it and the reference writes an all-zero cell there.  Restated exactly:
 *    the inverse here is the same zeroed (k+p) x k buffer.
 *  - parity-error rows = enc[e] * inv (:2233-2243) */
int ref_obj_ec_recov_codec_init(int k, int p, const unsigned char *en_matrix,
				const uint32_t *err_list, int nerrs,
				unsigned char *de_matrix, uint32_t *dec_idx,
				uint32_t *out_err_list, unsigned char *gftbls,
				int *reused_encode)
{
	unsigned char *b, *inv;
	int in_err[64 + 8];
	int data_nerrs = 0;
	int i, j, r, e;

	*reused_encode = 0;
	if (nerrs > p)
		return -REF_DER_DATA_LOSS;
	memset(in_err, 0, sizeof(in_err));
	for (i = 0; i < nerrs; i++) {
		out_err_list[i] = err_list[i];
		in_err[err_list[i]] = 1;
		if ((int)err_list[i] < k)
			data_nerrs++;
	}
	if (data_nerrs == 0 && nerrs == p) {
		ref_ec_init_tables(k, p, &en_matrix[k * k], gftbls);
		*reused_encode = 1;
		return 0;
	}

	b = malloc((size_t)k * k);
	inv = calloc((size_t)(k + p), (size_t)k);	/* rows k.. stay zero, as in the reference */
	if (b == NULL || inv == NULL) {
		free(b);
		free(inv);
		return -REF_DER_NOMEM;
	}
	for (i = 0, r = 0; i < k; i++, r++) {
		while (in_err[r])
			r++;
		memcpy(&b[(size_t)k * i], &en_matrix[(size_t)k * r], k);
		dec_idx[i] = (uint32_t)r;
	}
	if (ref_gf_invert_matrix(b, inv, k) != 0) {
		free(b);
		free(inv);
		return -REF_DER_INVAL;	/* unreachable for Cauchy matrices */
	}
	for (i = 0; i < data_nerrs; i++)
		memcpy(&de_matrix[(size_t)k * i], &inv[(size_t)k * err_list[i]], k);
	for (e = data_nerrs; e < nerrs; e++) {
		for (i = 0; i < k; i++) {
			unsigned char s = 0;

			for (j = 0; j < k; j++)
				s ^= ref_gf_mul(inv[(size_t)j * k + i],
						en_matrix[(size_t)k * err_list[e] + j]);
			de_matrix[(size_t)k * e + i] = s;
		}
	}
	ref_ec_init_tables(k, nerrs, de_matrix, gftbls);
	free(b);
	free(inv);
	return 0;
}

/* obj_ec_recov_stripe (ref:src/object/cli_ec.c:2626-2643). */
void ref_obj_ec_recov_stripe(int k, int nerrs, const unsigned char *gftbls,
			     const uint32_t *dec_idx, const uint32_t *err_list,
			     unsigned char *stripe, uint64_t cell_sz)
{
	unsigned char *src[64];
	unsigned char *dst[8];
	int i;

	for (i = 0; i < k; i++)
		src[i] = stripe + dec_idx[i] * cell_sz;
	for (i = 0; i < nerrs; i++)
		dst[i] = stripe + err_list[i] * cell_sz;
	ref_ec_encode_data((int)cell_sz, k, nerrs, gftbls, src, dst);
}

/* obj_ec_encode_buf (ref:src/object/cli_ec.c:548-573): data cells are
 * consecutive in `buffer`; parity goes to p_bufs[0..p). */
void ref_obj_ec_encode_buf(int k, int p, const unsigned char *en_matrix,
			   uint64_t cell_bytes, const unsigned char *buffer,
			   unsigned char **p_bufs)
{
	unsigned char tbls[64 * 8 * 32];
	unsigned char *data[64];
	int i;

	ref_ec_init_tables(k, p, &en_matrix[k * k], tbls);
	for (i = 0; i < k; i++)
		data[i] = (unsigned char *)buffer + i * cell_bytes;
	ref_ec_encode_data((int)cell_bytes, k, p, tbls, data, p_bufs);
}

/* Batch encode in the client layout: data [S][k][C] (user sgl order),
 * parity [p][S][C] (oer_pbufs[m] + n*C, ref:src/object/cli_ec.c:638-640). */
void ref_encode_batch(int k, int p, uint64_t C, uint32_t S,
		      const unsigned char *data, unsigned char *parity, int nthreads)
{
	unsigned char en[(64 + 8) * 64];
	unsigned char tbls[64 * 8 * 32];
	long s;

	ref_gf_gen_cauchy1_matrix(en, k + p, k);
	ref_ec_init_tables(k, p, &en[k * k], tbls);
	(void)nthreads;
#pragma omp parallel for schedule(static) if (nthreads > 1) num_threads(nthreads > 1 ? nthreads : 1)
	for (s = 0; s < (long)S; s++) {
		unsigned char *src[64];
		unsigned char *dst[8];
		int i;

		for (i = 0; i < k; i++)
			src[i] = (unsigned char *)data + ((uint64_t)s * k + i) * C;
		for (i = 0; i < p; i++)
			dst[i] = parity + ((uint64_t)i * S + s) * C;
		ref_ec_encode_data((int)C, k, p, tbls, src, dst);
	}
}

void ref_recov_batch(int k, int nerrs, const unsigned char *gftbls,
		     const uint32_t *dec_idx, const uint32_t *err_list,
		     uint64_t C, uint64_t stripe_stride, uint32_t S,
		     unsigned char *stripes, int nthreads)
{
	long s;

	(void)nthreads;
#pragma omp parallel for schedule(static) if (nthreads > 1) num_threads(nthreads > 1 ? nthreads : 1)
	for (s = 0; s < (long)S; s++)
		ref_obj_ec_recov_stripe(k, nerrs, gftbls, dec_idx, err_list,
					stripes + (uint64_t)s * stripe_stride, C);
}

/* agg_diff_preprocess, ref:src/object/srv_ec_aggregate.c:1006-1058, restated
 * with the stripe start already subtracted from the extents. */
void ref_agg_diff_preprocess(unsigned char *diff, uint64_t len, uint64_t rsize,
			     unsigned int cell_idx, const uint64_t *ext_start,
			     const uint64_t *ext_nr, unsigned int n_ext)
{
	uint64_t cell_start = (uint64_t)cell_idx * len;
	uint64_t cell_end = cell_start + len;
	uint64_t hole_off = 0;
	unsigned int i;

	for (i = 0; i < n_ext; i++) {
		uint64_t estart = ext_start[i];
		uint64_t eend = estart + ext_nr[i];
		uint64_t hole_end;

		if (estart >= cell_end)
			break;
		if (eend <= cell_start)
			continue;
		hole_end = cell_start + hole_off;
		if (estart > hole_end)
			memset(diff + hole_off * rsize, 0, (estart - hole_end) * rsize);
		hole_off = eend - cell_start;
	}
	if (hole_off > 0 && hole_off < len)
		memset(diff + hole_off * rsize, 0, (len - hole_off) * rsize);
}

int ref_agg_update_parity(int k, int p, uint64_t len, uint64_t rsize, const uint8_t *bit_map,
			  unsigned int cell_cnt, const unsigned char *obuf,
			  const unsigned char *nbuf, const uint64_t *ext_start,
			  const uint64_t *ext_nr, unsigned int n_ext, unsigned char *parity)
{
	unsigned char en[(64 + 8) * 64], tbls[64 * 8 * 32];
	unsigned char *pb[8];
	uint64_t cb = len * rsize;
	unsigned char *diff = malloc(cb ? cb : 1);
	unsigned int i, j;
	int r;

	if (diff == NULL)
		return -REF_DER_NOMEM;
	ref_gf_gen_cauchy1_matrix(en, k + p, k);
	ref_ec_init_tables(k, p, &en[k * k], tbls);
	for (r = 0; r < p; r++)
		pb[r] = parity + (uint64_t)r * cb;
	for (i = 0, j = 0; i < cell_cnt; i++, j++) {
		void *v[3];

		v[0] = (void *)(obuf + (uint64_t)i * cb);
		v[1] = (void *)(nbuf + (uint64_t)i * cb);
		v[2] = diff;
		ref_xor_gen(3, (int)cb, v);
		while (!(bit_map[j / 8] & (1u << (j % 8))))
			j++;
		ref_agg_diff_preprocess(diff, len, rsize, j, ext_start, ext_nr, n_ext);
		ref_ec_encode_data_update((int)cb, k, p, (int)j, tbls, diff, pb);
	}
	free(diff);
	return 0;
}

uint64_t ref_singv_cell_bytes(uint64_t rec_gsize, int k)
{
	uint64_t c = rec_gsize / (uint64_t)k;

	if (rec_gsize % (uint64_t)k)
		c++;
	return (c + 7) & ~7ull;
}

void ref_singv_encode(int k, int p, uint64_t iod_size, const unsigned char *value,
		      unsigned char **p_bufs)
{
	uint64_t cb = ref_singv_cell_bytes(iod_size, k);
	unsigned char *cells = calloc((size_t)k, cb);
	unsigned char en[(64 + 8) * 64], tbls[64 * 8 * 32];
	unsigned char *data[64];
	int j;

	memcpy(cells, value, iod_size);		/* last cell keeps its zero padding */
	for (j = 0; j < k; j++)
		data[j] = cells + (uint64_t)j * cb;
	ref_gf_gen_cauchy1_matrix(en, k + p, k);
	ref_ec_init_tables(k, p, &en[k * k], tbls);
	ref_ec_encode_data((int)cb, k, p, tbls, data, p_bufs);
	free(cells);
}
