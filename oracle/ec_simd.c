/*
 * ec_simd.c -- SIMD CPU BASELINE for the EC codec (test/bench infrastructure
 * only; see ec_ref.h).  "ISA-L-equivalent restatement": ISA-L v2.31.1 itself
 * is unavailable offline (ref:utils/build.config:8), so this restates the
 * algorithms of its x86 kernels:
 *   - AVX2: per-coefficient 16-entry low/high nibble tables + vpshufb, XOR
 *     accumulation over k sources (gf_vect_dot_prod_avx2 / gf_Nvect_dot_prod).
 *   - GFNI (AVX-512): multiplication by a constant is GF(2)-linear, so every
 *     coefficient becomes an 8x8 bit matrix applied with vgf2p8affineqb (the
 *     ISA-L >=2.31 GFNI path; vgf2p8mulb is unusable: it hard-wires 0x11b).
 * Output bytes are identical to ref_ec_encode_data (checked by tests).
 * Used by bench.py as cpu_baseline kind "port".
 */
#include "ec_ref.h"

#include <immintrin.h>
#include <string.h>

#define MAXK 64
#define MAXR 8

static int g_variant = -1;

int ref_simd_variant(void)
{
	if (g_variant < 0) {
		__builtin_cpu_init();
		if (__builtin_cpu_supports("gfni") && __builtin_cpu_supports("avx512bw"))
			g_variant = 2;
		else if (__builtin_cpu_supports("avx2"))
			g_variant = 1;
		else
			g_variant = 0;
	}
	return g_variant;
}

/* c * 2^j for j = 0..7 -> GF(2) matrix for vgf2p8affineqb.  Output bit i is
 * parity(A.byte[7-i] & x), so A.byte[7-i] bit j = bit i of (c * 2^j). */
static uint64_t gfni_matrix(unsigned char c)
{
	unsigned char col[8];
	uint64_t m = 0;
	int i, j;

	for (j = 0; j < 8; j++)
		col[j] = ref_gf_mul(c, (unsigned char)(1u << j));
	for (i = 0; i < 8; i++) {
		unsigned char row = 0;

		for (j = 0; j < 8; j++)
			if (col[j] & (1u << i))
				row |= (unsigned char)(1u << j);
		m |= (uint64_t)row << (8 * (7 - i));
	}
	return m;
}

__attribute__((target("avx2")))
static void encode_avx2(int len, int k, int rows, const unsigned char *gftbls,
			unsigned char **data, unsigned char **coding)
{
	int i = 0, j, l;

	for (; i + 32 <= len; i += 32) {
		__m256i acc[MAXR];
		const __m256i m0f = _mm256_set1_epi8(0x0f);

		for (l = 0; l < rows; l++)
			acc[l] = _mm256_setzero_si256();
		for (j = 0; j < k; j++) {
			__m256i x = _mm256_loadu_si256((const __m256i *)(data[j] + i));
			__m256i lo = _mm256_and_si256(x, m0f);
			__m256i hi = _mm256_and_si256(_mm256_srli_epi64(x, 4), m0f);

			for (l = 0; l < rows; l++) {
				const unsigned char *t = gftbls + 32 * (l * k + j);
				__m256i tl = _mm256_broadcastsi128_si256(
					_mm_loadu_si128((const __m128i *)t));
				__m256i th = _mm256_broadcastsi128_si256(
					_mm_loadu_si128((const __m128i *)(t + 16)));

				acc[l] = _mm256_xor_si256(acc[l],
					_mm256_xor_si256(_mm256_shuffle_epi8(tl, lo),
							 _mm256_shuffle_epi8(th, hi)));
			}
		}
		for (l = 0; l < rows; l++)
			_mm256_storeu_si256((__m256i *)(coding[l] + i), acc[l]);
	}
	if (i < len) {
		unsigned char *d2[MAXK], *c2[MAXR];

		for (j = 0; j < k; j++)
			d2[j] = data[j] + i;
		for (l = 0; l < rows; l++)
			c2[l] = coding[l] + i;
		ref_ec_encode_data(len - i, k, rows, gftbls, d2, c2);
	}
}

__attribute__((target("avx512f,avx512bw,gfni")))
static void encode_gfni(int len, int k, int rows, const unsigned char *gftbls,
			unsigned char **data, unsigned char **coding)
{
	uint64_t mat[MAXR * MAXK];
	int i = 0, j, l;

	for (l = 0; l < rows; l++)
		for (j = 0; j < k; j++)
			mat[l * k + j] = gfni_matrix(gftbls[32 * (l * k + j) + 1]);

	for (; i + 64 <= len; i += 64) {
		__m512i acc[MAXR];

		for (l = 0; l < rows; l++)
			acc[l] = _mm512_setzero_si512();
		for (j = 0; j < k; j++) {
			__m512i x = _mm512_loadu_si512((const void *)(data[j] + i));

			for (l = 0; l < rows; l++)
				acc[l] = _mm512_xor_si512(acc[l],
					_mm512_gf2p8affine_epi64_epi8(
						x, _mm512_set1_epi64((long long)mat[l * k + j]), 0));
		}
		for (l = 0; l < rows; l++)
			_mm512_storeu_si512((void *)(coding[l] + i), acc[l]);
	}
	if (i < len) {
		unsigned char *d2[MAXK], *c2[MAXR];

		for (j = 0; j < k; j++)
			d2[j] = data[j] + i;
		for (l = 0; l < rows; l++)
			c2[l] = coding[l] + i;
		ref_ec_encode_data(len - i, k, rows, gftbls, d2, c2);
	}
}

void ref_simd_encode_data(int len, int k, int rows, const unsigned char *gftbls,
			  unsigned char **data, unsigned char **coding)
{
	switch (ref_simd_variant()) {
	case 2:
		encode_gfni(len, k, rows, gftbls, data, coding);
		break;
	case 1:
		encode_avx2(len, k, rows, gftbls, data, coding);
		break;
	default:
		ref_ec_encode_data(len, k, rows, gftbls, data, coding);
	}
}

void ref_simd_encode_batch(int k, int p, uint64_t C, uint32_t S,
			   const unsigned char *data, unsigned char *parity, int nthreads)
{
	unsigned char en[(MAXK + MAXR) * MAXK];
	unsigned char tbls[MAXK * MAXR * 32];
	long s;

	ref_gf_gen_cauchy1_matrix(en, k + p, k);
	ref_ec_init_tables(k, p, &en[k * k], tbls);
	(void)ref_simd_variant();
#pragma omp parallel for schedule(static) num_threads(nthreads > 1 ? nthreads : 1)
	for (s = 0; s < (long)S; s++) {
		unsigned char *src[MAXK];
		unsigned char *dst[MAXR];
		int i;

		for (i = 0; i < k; i++)
			src[i] = (unsigned char *)data + ((uint64_t)s * k + i) * C;
		for (i = 0; i < p; i++)
			dst[i] = parity + ((uint64_t)i * S + s) * C;
		ref_simd_encode_data((int)C, k, p, tbls, src, dst);
	}
}

void ref_simd_recov_batch(int k, int nerrs, const unsigned char *gftbls,
			  const uint32_t *dec_idx, const uint32_t *err_list,
			  uint64_t C, uint64_t stripe_stride, uint32_t S,
			  unsigned char *stripes, int nthreads)
{
	long s;

	(void)ref_simd_variant();
#pragma omp parallel for schedule(static) num_threads(nthreads > 1 ? nthreads : 1)
	for (s = 0; s < (long)S; s++) {
		unsigned char *stripe = stripes + (uint64_t)s * stripe_stride;
		unsigned char *src[MAXK];
		unsigned char *dst[MAXR];
		int i;

		for (i = 0; i < k; i++)
			src[i] = stripe + dec_idx[i] * C;
		for (i = 0; i < nerrs; i++)
			dst[i] = stripe + err_list[i] * C;
		ref_simd_encode_data((int)C, k, nerrs, gftbls, src, dst);
	}
}
