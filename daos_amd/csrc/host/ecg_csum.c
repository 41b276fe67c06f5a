/*
 * ecg_csum.c -- host side of the chunked checksums (include/ecg_csum.h):
 * CRC tables built from the polynomials, per-context device copies, chunk
 * geometry of an extent (ref:src/common/checksum.c:1444-1565), launch.
 */
#include <stdlib.h>
#include <string.h>

#include "ecg_internal.h"
#include "../../../include/ecg_csum.h"

struct crc_def {
	int width;
	int refl;
	uint64_t poly;		/* reflected for refl, MSB-first otherwise */
	uint64_t init, xorout;
};

/* ISA-L crc16_t10dif / crc32_iscsi / crc64_ecma_refl as DAOS calls them
 * (seed 0; crc64 inverts the register on entry and exit). */
static const struct crc_def g_defs[4] = {
	[ECG_HASH_CRC16] = {16, 0, 0x8BB7, 0, 0},
	[ECG_HASH_CRC32] = {32, 1, 0x82F63B78u, 0, 0},
	[ECG_HASH_CRC64] = {64, 1, 0xC96C5795D7870F42ull, ~0ull, ~0ull},
};

/* CRC table kinds are fixed per kernel (ecg_kernels.hip CS_TB,
 * ecg_csum_kernels.hip kind_ok): standalone kernels use the nibble tables
 * (SDWA-addressed, conflict-free; profiles/r03/crc_sq/), their byte-granular
 * variants the 5-bit tables; the fused kernels the byte tables for crc64 and
 * for crc32 at EC_8P2, the 5-bit tables elsewhere (profiles/r02/fused_tables_ab/,
 * profiles/r03/fused_tb3/, fused_tb4/).  The other kinds were A/B builds. */

int ecg_csum_len(int type)
{
	switch (type) {
	case ECG_HASH_CRC16:
		return 2;
	case ECG_HASH_CRC32:
	case ECG_HASH_ADLER32:
		return 4;
	case ECG_HASH_CRC64:
		return 8;
	default:
		return -ECG_DER_NOTSUPPORTED;
	}
}

uint64_t ecg_csum_record_chunksize(uint64_t chunksize, uint64_t rec_size)
{
	if (rec_size == 0 || chunksize == 0)
		return 0;
	if (rec_size > chunksize)
		return rec_size;
	return chunksize / rec_size * rec_size;
}

uint32_t ecg_csum_chunk_count(uint64_t chunksize, uint64_t rec_size, uint64_t rx_idx,
			      uint64_t rx_nr)
{
	const uint64_t rcs = ecg_csum_record_chunksize(chunksize, rec_size);
	uint64_t per, lo, hi_end;

	if (rcs == 0 || rx_nr == 0)
		return 0;
	if (rx_nr == 1)
		return 1;
	per = rcs / rec_size;
	lo = rx_idx / per;
	hi_end = (rx_idx + (rx_nr - 1)) / per;
	return (uint32_t)(hi_end - lo + 1);
}

/* CRC register after one zero byte: c * x^8 mod P */
static uint64_t zero_byte(const struct crc_def *d, uint64_t c)
{
	const uint64_t mask = d->width == 64 ? ~0ull : (1ull << d->width) - 1;

	for (int b = 0; b < 8; b++) {
		if (d->refl)
			c = (c & 1) ? (c >> 1) ^ d->poly : c >> 1;
		else
			c = ((c >> (d->width - 1)) & 1) ? ((c << 1) & mask) ^ d->poly : (c << 1) & mask;
	}
	return c;
}

/* "1" in the register representation */
static uint64_t crc_one(const struct crc_def *d)
{
	return d->refl ? 1ull << (d->width - 1) : 1;
}

/* a * b mod P (same representations as the device mulmod) */
static uint64_t crc_mulmod(const struct crc_def *d, uint64_t a, uint64_t b)
{
	const uint64_t mask = d->width == 64 ? ~0ull : (1ull << d->width) - 1;
	uint64_t p = 0;

	for (int i = d->width - 1; i >= 0; i--) {
		if (d->refl) {
			if ((a >> i) & 1)
				p ^= b;
			b = (b & 1) ? (b >> 1) ^ d->poly : b >> 1;
		} else {
			p = ((p >> (d->width - 1)) & 1) ? ((p << 1) & mask) ^ d->poly : (p << 1) & mask;
			if ((a >> i) & 1)
				p ^= b;
		}
	}
	return p;
}

/* x^(-8z) mod P: x^-1 = (P - 1) / x since P(0) = 1 */
static uint64_t crc_unshift(const struct crc_def *d, uint64_t z)
{
	const uint64_t mask = d->width == 64 ? ~0ull : (1ull << d->width) - 1;
	const uint64_t xinv = d->refl ? (((d->poly << 1) & mask) | 1)
				      : ((1ull << (d->width - 1)) | (d->poly >> 1));
	uint64_t r = crc_one(d), b = xinv;

	for (uint64_t e = 8 * z; e; e >>= 1) {	/* square and multiply */
		if (e & 1)
			r = crc_mulmod(d, r, b);
		b = crc_mulmod(d, b, b);
	}
	return r;
}

/* x^(8n) mod P: "1" moved through n zero bytes, by square and multiply */
static uint64_t crc_xpow8(const struct crc_def *d, uint64_t n)
{
	uint64_t r = crc_one(d), b = zero_byte(d, crc_one(d));

	for (; n; n >>= 1) {
		if (n & 1)
			r = crc_mulmod(d, r, b);
		b = crc_mulmod(d, b, b);
	}
	return r;
}

/* Workgroup-per-chunk CRC: shift of each wave's slice to the end of a chunk
 * of m 1 KiB steps (ecg_kabi.h split_sh), cached per context by (type, m). */
static void split_shifts(ecg_ctx_t *ctx, int type, uint64_t m, uint64_t *sh)
{
	const uint64_t ms = ECG_CSUM_SPLIT_MS(m);
	struct ecg_split_ent *e;

	pthread_mutex_lock(&ctx->lock);
	for (int i = 0; i < ECG_NSPLIT_CACHE; i++) {
		e = &ctx->split_cache[i];
		if (e->valid && e->type == type && e->m == m) {
			memcpy(sh, e->sh, sizeof(e->sh));
			pthread_mutex_unlock(&ctx->lock);
			return;
		}
	}
	e = &ctx->split_cache[ctx->split_next++ % ECG_NSPLIT_CACHE];
	for (int w = 0; w < ECG_CSUM_SPLIT_NW; w++) {
		const uint64_t i0 = w * ms < m ? w * ms : m, i1 = i0 + ms < m ? i0 + ms : m;

		e->sh[w] = crc_xpow8(&g_defs[type], (m - i1) * ECG_CSUM_STRIDE);
	}
	e->type = type;
	e->m = m;
	e->valid = 1;
	memcpy(sh, e->sh, sizeof(e->sh));
	pthread_mutex_unlock(&ctx->lock);
}

/* linear map "shift by n zero bytes" as NB byte tables at t */
static void build_shift(const struct crc_def *d, int n, uint64_t *t)
{
	const int nb = d->width / 8;
	uint64_t basis[64];

	for (int i = 0; i < d->width; i++) {
		uint64_t c = 1ull << i;

		for (int z = 0; z < n; z++)
			c = zero_byte(d, c);
		basis[i] = c;
	}
	for (int j = 0; j < nb; j++)
		for (int v = 0; v < 256; v++) {
			uint64_t c = 0;

			for (int b = 0; b < 8; b++)
				if (v & (1 << b))
					c ^= basis[8 * j + b];
			t[(size_t)j * 256 + v] = c;
		}
}

/* raw CRC (zero register) of len bytes */
static uint64_t crc_raw(const struct crc_def *d, const unsigned char *buf, int len)
{
	const uint64_t mask = d->width == 64 ? ~0ull : (1ull << d->width) - 1;
	uint64_t c = 0;

	for (int i = 0; i < len; i++) {
		c ^= d->refl ? (uint64_t)buf[i] : (uint64_t)buf[i] << (d->width - 8);
		c = zero_byte(d, c) & mask;
	}
	return c;
}

/* 5-bit field tables (ecg_kabi.h p5 / a5): field (dword j, field i) covers
 * bits 32j + 5i .. +4 of the piece or register; entry v = XOR of the basis
 * images of v's set bits.  a5 for a shift of n zero bytes. */
static void build_p5(const struct crc_def *d, uint64_t zeros, uint64_t *p5)
{
	const uint64_t sh = zeros ? crc_xpow8(d, zeros) : 0;
	uint64_t basis[128];
	unsigned char piece[16];

	for (int k = 0; k < 128; k++) {
		memset(piece, 0, sizeof(piece));
		piece[k / 8] = (unsigned char)(1u << (k % 8));
		basis[k] = crc_raw(d, piece, 16);
		if (zeros)	/* the piece followed by `zeros` zero bytes */
			basis[k] = crc_mulmod(d, basis[k], sh);
	}
	for (int f = 0; f < ECG_CSUM_NF5; f++) {
		const int j = f / 7, i = f % 7;

		for (int v = 0; v < 32; v++) {
			uint64_t c = 0;

			for (int t = 0; t < 5; t++)
				if ((v >> t) & 1 && 5 * i + t < 32)
					c ^= basis[32 * j + 5 * i + t];
			p5[(size_t)f * 32 + v] = c;
		}
	}
}

/* nibble tables (ecg_kabi.h q4 / a4): nibble t covers bits 4t..4t+3 of the
 * piece (q4, the piece followed by `zeros` zero bytes) or of the register
 * shifted by n zero bytes (a4) */
static void build_q4(const struct crc_def *d, uint64_t zeros, uint64_t *q4)
{
	const uint64_t sh = zeros ? crc_xpow8(d, zeros) : 0;
	uint64_t basis[128];
	unsigned char piece[16];

	for (int k = 0; k < 128; k++) {
		memset(piece, 0, sizeof(piece));
		piece[k / 8] = (unsigned char)(1u << (k % 8));
		basis[k] = crc_raw(d, piece, 16);
		if (zeros)
			basis[k] = crc_mulmod(d, basis[k], sh);
	}
	for (int t = 0; t < 32; t++)
		for (int v = 0; v < 16; v++) {
			uint64_t c = 0;

			for (int b = 0; b < 4; b++)
				if ((v >> b) & 1)
					c ^= basis[4 * t + b];
			q4[(size_t)t * 16 + v] = c;
		}
}

static void build_a4(const struct crc_def *d, uint64_t n, uint64_t *a4)
{
	const uint64_t sh = crc_xpow8(d, n);

	for (int t = 0; t < d->width / 4; t++)
		for (int v = 0; v < 16; v++) {
			uint64_t c = 0;

			for (int b = 0; b < 4; b++)
				if ((v >> b) & 1)
					c ^= crc_mulmod(d, 1ull << (4 * t + b), sh);
			a4[(size_t)t * 16 + v] = c;
		}
}

static void build_a5(const struct crc_def *d, uint64_t n, uint64_t *a5)
{
	const uint64_t sh = crc_xpow8(d, n);
	const int na = d->width == 16 ? 4 : 7 * d->width / 32;

	for (int f = 0; f < na; f++) {
		const int h = d->width == 16 ? 0 : f / 7, i = d->width == 16 ? f : f % 7;

		for (int v = 0; v < 32; v++) {
			uint64_t c = 0;

			for (int t = 0; t < 5; t++) {
				const int bit = 32 * h + 5 * i + t;

				if ((v >> t) & 1 && 5 * i + t < 32 && bit < d->width)
					c ^= crc_mulmod(d, 1ull << bit, sh);
			}
			a5[(size_t)f * 32 + v] = c;
		}
	}
}

/* Device table image (layout in ecg_kabi.h): sl, sh (1 KiB), k64, sh4k,
 * k256, p2, sh256, p5, a5 (1 KiB, 256 B, 4 KiB); entries of 4 (W <= 32) or
 * 8 (W = 64) bytes. */
static void *build_crc_tables(const struct crc_def *d, size_t *bytes)
{
	const int nb = d->width / 8, es = d->width == 64 ? 8 : 4;
	const size_t n = ECG_CSUM_TBL_ENTRIES(nb);
	uint64_t *t = calloc(n, sizeof(uint64_t));
	unsigned char *img;
	uint64_t c;

	if (t == NULL)
		return NULL;
	/* sl[j][v] (j < NB) and s16[j][v] (j < 16): register after byte v (from
	 * zero) and then j zero bytes */
	for (int v = 0; v < 256; v++) {
		uint64_t c = d->refl ? (uint64_t)v : (uint64_t)v << (d->width - 8);

		c = zero_byte(d, c);
		for (int j = 0; j < 16; j++) {
			if (j < nb)
				t[(size_t)j * 256 + v] = c;
			t[ECG_CSUM_OFF_S16(nb) + (size_t)j * 256 + v] = c;
			c = zero_byte(d, c);
		}
	}
	build_shift(d, ECG_CSUM_STRIDE, t + ECG_CSUM_OFF_SH(nb));
	build_shift(d, ECG_MMCS_STRIDE, t + ECG_CSUM_OFF_SH4K(nb));
	build_shift(d, ECG_CSUM_GSTRIDE, t + ECG_CSUM_OFF_SH256(nb));
	/* k64[lane] = x^(8*16*(63-lane)), k256[t] = x^(8*16*(255-t)) mod P:
	 * "1" moved through that many zero bytes, walking down from the last */
	c = crc_one(d);
	for (int l = 255; l >= 0; l--) {
		if (l >= 192)
			t[ECG_CSUM_OFF_K64(nb) + (l - 192)] = c;
		t[ECG_CSUM_OFF_K256(nb) + l] = c;
		for (int z = 0; z < 16; z++)
			c = zero_byte(d, c);
	}
	/* p2[j] = x^(8*2^j) mod P */
	c = zero_byte(d, crc_one(d));
	for (int j = 0; j < ECG_CSUM_NP2; j++) {
		t[ECG_CSUM_OFF_P2(nb) + j] = c;
		c = crc_mulmod(d, c, c);
	}
	build_p5(d, 0, t + ECG_CSUM_OFF_P5(nb));
	for (int u = 1; u < ECG_CSUM_P5U; u++) {
		build_p5(d, (uint64_t)u * ECG_CSUM_STRIDE,
			 t + ECG_CSUM_OFF_P5X_1K(nb) + (size_t)(u - 1) * ECG_CSUM_NF5 * 32);
		build_p5(d, (uint64_t)u * ECG_CSUM_GSTRIDE,
			 t + ECG_CSUM_OFF_P5X_256(nb) + (size_t)(u - 1) * ECG_CSUM_NF5 * 32);
	}
	for (int u = 1; u < ECG_MMCS_P5U; u++)
		build_p5(d, (uint64_t)u * ECG_MMCS_STRIDE,
			 t + ECG_CSUM_OFF_P5X_4K(nb) + (size_t)(u - 1) * ECG_CSUM_NF5 * 32);
	build_a5(d, (uint64_t)ECG_MMCS_P5U * ECG_MMCS_STRIDE, t + ECG_CSUM_OFF_A5_32K(nb));
	if (d->refl) {
		/* nibl[n][l] = (n << (W - 4)) * x^(8*16*(63-l)); r4[m] = m * x^4 */
		for (int l = 0; l < 64; l++)
			for (int n = 0; n < 16; n++)
				t[ECG_CSUM_OFF_NIBL(nb) + (size_t)n * 64 + l] =
					crc_mulmod(d, (uint64_t)n << (d->width - 4), t[ECG_CSUM_OFF_K64(nb) + l]);
		for (int m = 0; m < 16; m++) {
			uint64_t c = (uint64_t)m;

			for (int b = 0; b < 4; b++)
				c = (c >> 1) ^ (d->poly & (0 - (c & 1)));
			t[ECG_CSUM_OFF_R4(nb) + m] = c;
		}
	}
	build_a5(d, ECG_CSUM_STRIDE, t + ECG_CSUM_OFF_A5_1K(nb));
	build_a5(d, ECG_CSUM_GSTRIDE, t + ECG_CSUM_OFF_A5_256(nb));
	build_a5(d, ECG_MMCS_STRIDE, t + ECG_CSUM_OFF_A5_4K(nb));
	for (int u = 0; u < ECG_CSUM_P5U; u++) {
		build_q4(d, (uint64_t)u * ECG_CSUM_STRIDE, t + ECG_CSUM_OFF_Q4_1K(nb) + (size_t)u * ECG_CSUM_NQ4);
		build_q4(d, (uint64_t)u * ECG_CSUM_GSTRIDE, t + ECG_CSUM_OFF_Q4_256(nb) + (size_t)u * ECG_CSUM_NQ4);
	}
	build_a4(d, (uint64_t)ECG_CSUM_P5U * ECG_CSUM_STRIDE, t + ECG_CSUM_OFF_A4_4K(nb));
	build_a4(d, (uint64_t)ECG_CSUM_P5U * ECG_CSUM_GSTRIDE, t + ECG_CSUM_OFF_A4_1K(nb));
	for (int u = 0; u < ECG_MMCS_P5U; u++)
		build_q4(d, (uint64_t)u * ECG_MMCS_STRIDE, t + ECG_CSUM_OFF_Q4_4K(nb) + (size_t)u * ECG_CSUM_NQ4);
	build_a4(d, (uint64_t)ECG_MMCS_P5U * ECG_MMCS_STRIDE, t + ECG_CSUM_OFF_A4_32K(nb));

	*bytes = n * (size_t)es;
	if (es == 8)
		return t;
	img = malloc(*bytes);
	if (img)
		for (size_t i = 0; i < n; i++) {
			uint32_t w = (uint32_t)t[i];

			memcpy(img + 4 * i, &w, 4);
		}
	free(t);
	return img;
}

/* Device copy of a type's tables, built once per context (ctx->lock). */
static int crc_tables(ecg_ctx_t *ctx, int type, const void **out)
{
	int rc = 0;

	pthread_mutex_lock(&ctx->lock);
	if (ctx->csum_tbl[type] == NULL) {
		size_t bytes = 0;
		void *img = build_crc_tables(&g_defs[type], &bytes), *dev = NULL;
		hipError_t e;

		if (img == NULL) {
			rc = ecg_fail(-ECG_DER_NOMEM, "csum tables");
		} else {
			e = hipMalloc(&dev, bytes);
			if (e == hipSuccess)
				e = hipMemcpy(dev, img, bytes, hipMemcpyHostToDevice);
			if (e != hipSuccess) {
				if (dev)
					(void)hipFree(dev);
				rc = ecg_hip_fail(e, "csum tables");
			} else {
				ctx->csum_tbl[type] = dev;
			}
			free(img);
		}
	}
	*out = ctx->csum_tbl[type];
	pthread_mutex_unlock(&ctx->lock);
	return rc;
}

void ecg_csum_ctx_fini(ecg_ctx_t *ctx)
{
	for (int i = 0; i < ECG_NCSUM_TBL; i++)
		if (ctx->csum_tbl[i]) {
			(void)hipFree(ctx->csum_tbl[i]);
			ctx->csum_tbl[i] = NULL;
		}
	for (int i = 0; i < ECG_NKH_CACHE; i++)
		if (ctx->kh_cache[i].dev) {
			(void)hipFree(ctx->kh_cache[i].dev);
			memset(&ctx->kh_cache[i], 0, sizeof(ctx->kh_cache[i]));
		}
}

/* Columns per fused-kernel work item (a whole chunk when shorter): fewer
 * columns per item walk a chunk with more workgroups in parallel, more
 * amortise the per-item reduction.  Measured A/B in one process on random
 * data (tools/tune12.py, tools/fused_libs.py; profiles/r01/tune12.json,
 * profiles/r02/fused_libs/, profiles/r03/fused_tail/); ecg_set_fused_cols /
 * ECG_FUSED_COLS override. */
static int g_fused_cols_env;
static pthread_once_t g_fused_cols_once = PTHREAD_ONCE_INIT;

static void fused_cols_init(void)
{
	const char *e = getenv("ECG_FUSED_COLS");

	g_fused_cols_env = e ? atoi(e) : 0;
	if (g_fused_cols_env < 0)
		g_fused_cols_env = 0;
}

static uint32_t fused_cols(const ecg_ctx_t *ctx, uint64_t m, int type, int k, int rows)
{
	/* tools/fused_libs.py, profiles/r02/fused_libs/, profiles/r03/fused_tail/:
	 * one output row (a parity shard's rebuild) 4; >= 2 rows: 4 for k >= 8
	 * (EC_8P2 crc32 +8 % vs +18 % at 8; crc64, now that its item tail reads no
	 * HBM, +12.5 % vs +20 %), 8 for k <= 4 (EC_4P2 crc32 +8 % vs +15 % at 4) */
	/* round 3, after the item tail stopped reading HBM: crc32 at EC_8P2 (byte
	 * tables) walks 2 columns best -- +6.0 / +7.3 % vs +9.0 / +9.9 % at 4 on two
	 * boxes; k = 16 and one or three rows keep 4 (profiles/r03/fused_cols/) */
	const uint64_t dflt = type == ECG_HASH_CRC32 && k == 8 && rows == 2 ? 2 : rows == 1 ? 4 : k >= 8 ? 4 : 8;
	const int env = ctx->fused_cols ? (int)ctx->fused_cols
					: (pthread_once(&g_fused_cols_once, fused_cols_init), g_fused_cols_env);

	if (env > 0)
		return (uint32_t)((uint64_t)env < m ? (uint64_t)env : m);
	return (uint32_t)(m < dflt ? m : dflt);
}

/* Device table of the fused kernel's per-item multipliers (ecg_kabi.h
 * ecg_mmcs_params kh): row h < nh of a full chunk of m columns, rows nh + h of
 * the last chunk (m_last columns, z padding bytes):
 *   crc16:      kh[row][t] = x^(8*(16*(255-t) + 4096*(columns after item h))) * x^(-8z)
 *   reflected:  the factor f(row, w) = x^(8*(1024*(3-w) + 4096*(columns after
 *               item h))) * x^(-8z) of wave w as its W bit-products,
 *               kh[row][w][b] = e_b * f(row, w) (e_b: the register with only
 *               bit b set; entries b >= W zero) -- the kernel applies the lane
 *               part from the LDS nibl tables and then f bit-parallel, lane b
 *               contributing kh[row][w][b] when bit b of the wave's sum is set
 * Cached per context by (type, chunk bytes, columns per item, last length). */
static int fused_kh(ecg_ctx_t *ctx, int type, uint64_t rcs, uint64_t last, uint32_t ncols,
		    uint32_t nh, uint32_t nh_last, const void **out)
{
	const struct crc_def *d = &g_defs[type];
	const uint64_t m = rcs / ECG_MMCS_STRIDE;
	const uint64_t m_last = (last + ECG_MMCS_STRIDE - 1) / ECG_MMCS_STRIDE;
	const uint64_t z = m_last * ECG_MMCS_STRIDE - last;
	const size_t es = d->width == 64 ? 8 : 4, nrow = (size_t)nh + nh_last;
	/* entries per row: 4 waves x 64 bit-products, or 256 threads */
	const size_t per = d->refl ? 4 * 64 : 256;
	struct ecg_kh_ent *e;
	uint64_t k256[256];
	unsigned char *img;
	void *dev = NULL;
	hipError_t he;
	int rc = 0;

	pthread_mutex_lock(&ctx->lock);
	for (int i = 0; i < ECG_NKH_CACHE; i++) {
		e = &ctx->kh_cache[i];
		if (e->valid && e->type == type && e->rcs == rcs && e->last == last && e->ncols == ncols) {
			*out = e->dev;
			pthread_mutex_unlock(&ctx->lock);
			return 0;
		}
	}
	img = malloc(nrow * per * es);
	if (img == NULL) {
		pthread_mutex_unlock(&ctx->lock);
		return ecg_fail(-ECG_DER_NOMEM, "fused csum multipliers");
	}
	k256[255] = crc_one(d);
	for (int t = 254; t >= 0; t--)
		k256[t] = crc_mulmod(d, k256[t + 1], crc_xpow8(d, 16));
	for (size_t row = 0; row < nrow; row++) {
		const int lastc = row >= nh;
		const uint64_t h = lastc ? row - nh : row, mc = lastc ? m_last : m;
		const uint64_t end = (h + 1) * ncols < mc ? (h + 1) * ncols : mc;
		uint64_t sh = crc_xpow8(d, (mc - end) * ECG_MMCS_STRIDE);

		if (lastc)
			sh = crc_mulmod(d, sh, crc_unshift(d, z));
		uint64_t f = 0;

		for (size_t t = 0; t < per; t++) {
			uint64_t v;

			if (d->refl) {
				/* wave w's factor (k256[64 w + 63] = x^(8*16*(192-64w)) =
				 * x^(8*1024*(3-w))) times the item's shift, as bit-products */
				const size_t w = t / 64, b = t % 64;

				if (b == 0)
					f = crc_mulmod(d, k256[64 * w + 63], sh);
				v = b < (size_t)d->width ? crc_mulmod(d, (uint64_t)1 << b, f) : 0;
			} else {	/* crc16: thread t's */
				v = crc_mulmod(d, k256[t], sh);
			}
			if (es == 8) {
				memcpy(img + (row * per + t) * 8, &v, 8);
			} else {
				const uint32_t w32 = (uint32_t)v;

				memcpy(img + (row * per + t) * 4, &w32, 4);
			}
		}
	}
	he = hipMalloc(&dev, nrow * per * es);
	if (he == hipSuccess)
		he = hipMemcpy(dev, img, nrow * per * es, hipMemcpyHostToDevice);
	free(img);
	if (he != hipSuccess) {
		if (dev)
			(void)hipFree(dev);
		pthread_mutex_unlock(&ctx->lock);
		return ecg_hip_fail(he, "fused csum multipliers");
	}
	e = &ctx->kh_cache[ctx->kh_next++ % ECG_NKH_CACHE];
	if (e->dev) {
		/* launches queued on any stream may still read the evicted table */
		(void)hipDeviceSynchronize();
		(void)hipFree(e->dev);
	}
	e->valid = 1;
	e->type = type;
	e->rcs = rcs;
	e->last = last;
	e->ncols = ncols;
	e->dev = dev;
	*out = dev;
	pthread_mutex_unlock(&ctx->lock);
	return rc;
}

int ecg_csum_extents(ecg_ctx_t *ctx, int type, uint64_t chunksize, uint64_t rec_size,
		     uint64_t rx_idx, uint64_t rx_nr, const void *buf, int64_t ext_stride,
		     uint32_t n_ext, void *csums, void *stream)
{
	ecg_csum_params_t prm;
	const uint64_t rcs = ecg_csum_record_chunksize(chunksize, rec_size);
	uint64_t per, first_end;
	uint32_t kid = 0;
	int rc, e;

	if (ctx == NULL || (n_ext && rx_nr && (buf == NULL || csums == NULL)) || rcs == 0)
		return ecg_fail(-ECG_DER_INVAL, "csum_extents: bad arguments");
	if (ecg_csum_len(type) < 0)
		return ecg_fail(-ECG_DER_NOTSUPPORTED, "csum_extents: hash type %d not supported",
				type);
	if (rx_nr > UINT64_MAX / rec_size || (rx_nr && rx_nr - 1 > UINT64_MAX - rx_idx))
		return ecg_fail(-ECG_DER_INVAL, "csum_extents: extent overflows");
	if (n_ext == 0 || rx_nr == 0)
		return 0;
	rc = ecg_ctx_enter(ctx);
	if (rc)
		return rc;
	memset(&prm, 0, sizeof(prm));
	if (type != ECG_HASH_ADLER32) {
		rc = crc_tables(ctx, type, &prm.tbl);
		if (rc)
			return rc;
		prm.poly = g_defs[type].poly;
		prm.init = g_defs[type].init;
		prm.xorout = g_defs[type].xorout;
	}
	/* chunk 0 runs from rx_idx to the end of its aligned chunk (clipped);
	 * the rest are whole chunks, the last one clipped
	 * (csum_recx_chunkidx2range, ref:src/common/checksum.c:1489-1565) */
	per = rcs / rec_size;
	first_end = rx_idx - rx_idx % per + (per - 1);
	if (first_end < rx_idx)		/* csum_chunk_align_ceiling overflow guard */
		first_end = UINT64_MAX;
	if (first_end > rx_idx + (rx_nr - 1))
		first_end = rx_idx + (rx_nr - 1);
	prm.src = buf;
	prm.out = csums;
	prm.ext_stride = ext_stride;
	prm.ext_bytes = rx_nr * rec_size;
	prm.first_bytes = (first_end - rx_idx + 1) * rec_size;
	prm.chunk_bytes = rcs;
	prm.n_ext = n_ext;
	prm.nchunks = ecg_csum_chunk_count(chunksize, rec_size, rx_idx, rx_nr);
	prm.type = (uint32_t)type;
	if (type != ECG_HASH_ADLER32) {
		/* a workgroup per chunk when one wave per chunk would leave fewer
		 * than 4 waves per SIMD and each wave still gets >= 2 KiB steps
		 * (tools/bench_csum.py shape_* rows) */
		const uint64_t total = (uint64_t)n_ext * prm.nchunks;
		const uint64_t steps = (rcs / 16 + 63) / 64;
		const int split = total < 4096 && steps >= 2 * ECG_CSUM_SPLIT_NW;
		const uint64_t lens[3] = {
			prm.first_bytes, rcs,
			prm.nchunks >= 2 ? prm.ext_bytes - prm.first_bytes - (uint64_t)(prm.nchunks - 2) * rcs
					 : prm.first_bytes};

		/* short chunks (<= 8 KiB): a 16-lane group each, so the per-lane
		 * final multiply is paid once per >= 8 pieces instead of per 1-2 */
		const int group = !split && steps <= 8;

		prm.variant = split ? 2 : group ? 3 : 1;
		for (int c = 0; split && c < 3; c++) {
			prm.split_m[c] = ECG_CSUM_STEPS(lens[c]);
			split_shifts(ctx, type, prm.split_m[c], prm.split_sh[c]);
		}
	} else {
		prm.variant = 0;	/* adler32: the kernel picks by shape */
	}
	e = ecg_k_launch_csum(&prm, (void *)ecg_pick_stream(ctx, stream), ctx->csum_blocks, &kid);
	if (e != 0)
		return ecg_hip_fail((hipError_t)e, "csum kernel launch");
	ECG_STAT_ADD(ctx, launches, 1);
	ECG_STAT_ADD(ctx, csum_chunks, (uint64_t)prm.n_ext * prm.nchunks);
	ecg_set_last_kernel(ecg_k_kernel_name(kid));
	return 0;
}

int ecg_set_csum_launch(ecg_ctx_t *ctx, uint32_t max_blocks)
{
	if (ctx == NULL)
		return ecg_fail(-ECG_DER_INVAL, "set_csum_launch: NULL context");
	ctx->csum_blocks = max_blocks;
	return 0;
}

int ecg_set_fused_cols(ecg_ctx_t *ctx, uint32_t ncols)
{
	if (ctx == NULL || ncols > 4096)
		return ecg_fail(-ECG_DER_INVAL, "set_fused_cols: bad arguments");
	ctx->fused_cols = ncols;
	return 0;
}

/* Fused product + checksum parameters (ecg_kabi.h) for output cells of C
 * bytes that start on chunk boundaries.  Returns 1 when the fused kernels
 * can take the request, 0 when the caller must run the product and
 * ecg_csum_extents separately, < 0 on error. */
int ecg_csum_fused_params(ecg_ctx_t *ctx, int type, uint64_t chunksize, uint64_t rec_size,
			  uint64_t C, int k, int rows, void *csums, ecg_mmcs_params_t *q)
{
	const uint64_t rcs = ecg_csum_record_chunksize(chunksize, rec_size);
	const struct crc_def *d;
	uint64_t last, m;
	int rc;

	memset(q, 0, sizeof(*q));
	if (type != ECG_HASH_CRC16 && type != ECG_HASH_CRC32 && type != ECG_HASH_CRC64)
		return 0;
	if (rcs == 0 || rcs % ECG_MMCS_STRIDE || C % 16 || C % rec_size)
		return 0;
	/* the kernel XORs partials in with 32-bit (crc16/crc32) or 64-bit atomics */
	if ((uintptr_t)csums % (type == ECG_HASH_CRC64 ? 8u : 4u))
		return 0;
	d = &g_defs[type];
	rc = crc_tables(ctx, type, &q->tbl);
	if (rc)
		return rc;
	q->out = csums;
	q->chunk_bytes = rcs;
	q->nch = (uint32_t)((C + rcs - 1) / rcs);
	q->init = d->init;
	q->xorout = d->xorout;
	q->poly = d->poly;
	q->type = (uint32_t)type;
	last = C - (uint64_t)(q->nch - 1) * rcs;
	m = rcs / ECG_MMCS_STRIDE;
	q->m = (uint32_t)m;
	q->m_last = (uint32_t)((last + ECG_MMCS_STRIDE - 1) / ECG_MMCS_STRIDE);
	q->ncols = fused_cols(ctx, m, type, k, rows);
	/* bound the multiplier table (nh + nh_last rows of 256 entries) for
	 * very long chunks: at most 2048 items per chunk */
	if ((m + q->ncols - 1) / q->ncols > 2048)
		q->ncols = (uint32_t)((m + 2047) / 2048);
	q->nh = (uint32_t)((m + q->ncols - 1) / q->ncols);
	q->nh_last = (q->m_last + q->ncols - 1) / q->ncols;
	if ((uint64_t)(q->nch - 1) * q->nh + q->nh_last > UINT32_MAX)
		return 0;
	q->nitems = (q->nch - 1) * q->nh + q->nh_last;
	/* the workgroup kernel for every shape: since its item tail no longer
	 * reads HBM (round 3) it beats the wave-per-chunk kernel of rounds 1-2
	 * for crc64 at EC_4P2 too (+13 % vs +19 % over the plain encode,
	 * profiles/r03/fused_tail/); the wave kernel was retired in round 4 */
	rc = fused_kh(ctx, type, rcs, last, q->ncols, q->nh, q->nh_last, &q->kh);
	if (rc)
		return rc;
	return 1;
}
