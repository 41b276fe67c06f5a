/*
 * ecg_cpu.c -- the product's CPU path for the synchronous one-stripe product
 * on HOST memory (the ISA-L calling convention: k source pointers, `rows`
 * destination pointers, any length and alignment).
 *
 * Why a CPU path exists in a GPU codec: ISA-L's ec_encode_data /
 * ec_encode_data_update / xor_gen are `void`, always-succeeding calls on any
 * CPU, and DAOS calls them from processes that have no GPU at all -- the
 * client library libdaos compiles cli_ec.c (ref:src/object/SConscript:19-23,
 * ec_encode_data at ref:src/object/cli_ec.c:540).  And for a small host-
 * resident call one core finishes before a PCIe round trip has started
 * (DESIGN.md §7).  The drop-in therefore routes host cells here below the
 * measured crossover and in every process without a gfx950 device
 * (ecg_dropin.c); device cells always run the HIP kernels.
 *
 * Arithmetic: multiplication by a constant c in GF(2^8)/0x11d is linear over
 * GF(2), i.e. an 8x8 bit matrix.  With GFNI that matrix is one
 * vgf2p8affineqb per (coefficient, 64 or 32 source bytes); without it the
 * product is split by nibble, c*x = c*(x & 0x0f) ^ c*(x & 0xf0), two 16-entry
 * vpshufb lookups.  Both tables come from the product's own field table
 * (ecg_gf.c), built once per process for all 256 coefficients so a call pays
 * no table setup.  Dispatch picks the widest variant the CPU has (cpuid);
 * ECG_CPU_ISA / ecg_cpu_set_isa force a narrower one (tests).
 *
 * Loop structure: destinations in groups of up to 8 rows, sources in groups of
 * up to 32 (later source groups accumulate), so the per-group matrices stay
 * small enough for a 16 KiB user-level-thread stack; per 64-byte column every
 * source is loaded once and folded into all rows of the group.  AVX-512 tails
 * use masked loads/stores, the AVX2 ones the byte table.
 */
#include <immintrin.h>
#include <stdlib.h>
#include <string.h>

#include "ecg_internal.h"

#define RG 8	/* destination rows per pass */
#define SG 32	/* sources per pass */

static uint64_t g_aff[256];		/* affine matrix of x -> c*x */
static unsigned char g_nib[256][32];	/* c*{0..15} | c*{0x00,0x10..0xf0} */
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

enum { ISA_SCALAR, ISA_AVX2, ISA_AVX2_GFNI, ISA_AVX512_GFNI, ISA_N };
static const char *const g_isa_name[ISA_N] = {"scalar", "avx2", "avx2-gfni", "avx512-gfni"};
static int g_isa_best;			/* widest the CPU supports */
static int g_isa;			/* in use */

/* Output bit i of vgf2p8affineqb is the parity of (matrix byte 7-i & x):
 * byte 7-i therefore holds, in bit j, bit i of c*2^j. */
static uint64_t affine_of(unsigned char c)
{
	uint64_t m = 0;
	int i, j;

	for (j = 0; j < 8; j++) {
		const unsigned v = ecg_gf_mul_tbl[c][1u << j];

		for (i = 0; i < 8; i++)
			m |= (uint64_t)((v >> i) & 1u) << (8 * (7 - i) + j);
	}
	return m;
}

static int isa_parse(const char *s)
{
	int i;

	for (i = 0; i < ISA_N; i++)
		if (strcmp(s, g_isa_name[i]) == 0)
			return i;
	return -1;
}

static void cpu_init(void)
{
	const char *env = getenv("ECG_CPU_ISA");
	int c, i;

	ecg_gf_init();
	for (c = 0; c < 256; c++) {
		g_aff[c] = affine_of((unsigned char)c);
		for (i = 0; i < 16; i++) {
			g_nib[c][i] = ecg_gf_mul_tbl[c][i];
			g_nib[c][16 + i] = ecg_gf_mul_tbl[c][i << 4];
		}
	}
	__builtin_cpu_init();
	g_isa_best = ISA_SCALAR;
	if (__builtin_cpu_supports("avx2"))
		g_isa_best = ISA_AVX2;
	if (g_isa_best == ISA_AVX2 && __builtin_cpu_supports("gfni"))
		g_isa_best = ISA_AVX2_GFNI;
	if (g_isa_best == ISA_AVX2_GFNI && __builtin_cpu_supports("avx512f") &&
	    __builtin_cpu_supports("avx512bw"))
		g_isa_best = ISA_AVX512_GFNI;
	g_isa = g_isa_best;
	if (env && (i = isa_parse(env)) >= 0 && i < g_isa_best)
		g_isa = i;
}

const char *ecg_cpu_isa(void)
{
	pthread_once(&g_once, cpu_init);
	return g_isa_name[__atomic_load_n(&g_isa, __ATOMIC_RELAXED)];
}

int ecg_cpu_set_isa(const char *isa)
{
	int i;

	pthread_once(&g_once, cpu_init);
	if (isa == NULL || strcmp(isa, "auto") == 0) {
		__atomic_store_n(&g_isa, g_isa_best, __ATOMIC_RELAXED);
		return 0;
	}
	i = isa_parse(isa);
	if (i < 0)
		return ecg_fail(-ECG_DER_INVAL, "cpu_set_isa: unknown '%s'", isa);
	if (i > g_isa_best)
		return ecg_fail(-ECG_DER_NOSYS, "cpu_set_isa: this CPU has no %s (best %s)", isa,
				g_isa_name[g_isa_best]);
	__atomic_store_n(&g_isa, i, __ATOMIC_RELAXED);
	return 0;
}

/* One pass: dst[r][i] (^)= XOR_j coef_r,j * src[j][i] for r < nr <= RG,
 * j < ns <= SG, i in [i0, len).  `cf` holds the group's coefficients row by
 * row (nr x ns); acc = fold into the current destination bytes. */
struct pass {
	size_t len;
	int nr, ns, acc, all_one;
	const unsigned char *cf;
	const unsigned char *const *src;
	unsigned char *const *dst;
};

/* Bytes [i0, len) through the field's product table (the scalar variant,
 * and the AVX2 variants' tails): eight bytes of every source at a time,
 * their eight lookups packed into one 64-bit word per row, so a row's bytes
 * are loaded and stored once per word.  Sources and outputs are distinct
 * cells, as in ISA-L. */
static void tail_bytes(const struct pass *q, size_t i0)
{
	const size_t len = q->len;
	int r, j;

	for (r = 0; r < q->nr; r++) {
		unsigned char *d = q->dst[r];
		size_t i = i0;

		for (; i + 8 <= len; i += 8) {
			uint64_t a = 0;

			if (q->acc)
				memcpy(&a, d + i, 8);
			for (j = 0; j < q->ns; j++) {
				const unsigned char *tb = ecg_gf_mul_tbl[q->cf[r * q->ns + j]];
				uint64_t x;

				memcpy(&x, q->src[j] + i, 8);
				a ^= (uint64_t)tb[x & 0xff] | (uint64_t)tb[(x >> 8) & 0xff] << 8 |
				     (uint64_t)tb[(x >> 16) & 0xff] << 16 | (uint64_t)tb[(x >> 24) & 0xff] << 24 |
				     (uint64_t)tb[(x >> 32) & 0xff] << 32 | (uint64_t)tb[(x >> 40) & 0xff] << 40 |
				     (uint64_t)tb[(x >> 48) & 0xff] << 48 | (uint64_t)tb[x >> 56] << 56;
			}
			memcpy(d + i, &a, 8);
		}
		for (; i < len; i++) {
			unsigned char v = q->acc ? d[i] : 0;

			for (j = 0; j < q->ns; j++)
				v ^= ecg_gf_mul_tbl[q->cf[r * q->ns + j]][q->src[j][i]];
			d[i] = v;
		}
	}
}

/* One 64-byte column of the group (masked when mk is partial). */
static inline __attribute__((always_inline, target("avx512f,avx512bw,gfni")))
void col_avx512_gfni(unsigned char *const *d, const unsigned char *const *s, const uint64_t *m, size_t i,
		     __mmask64 mk, int full, const int nr, int ns, int acc, int all_one)
{
	__m512i a[RG];
	int r, j;

	_Pragma("GCC unroll 8") for (r = 0; r < nr; r++)
		a[r] = !acc ? _mm512_setzero_si512() : full ? _mm512_loadu_si512(d[r] + i)
							   : _mm512_maskz_loadu_epi8(mk, d[r] + i);
	for (j = 0; j < ns; j++) {
		const __m512i x = full ? _mm512_loadu_si512(s[j] + i) : _mm512_maskz_loadu_epi8(mk, s[j] + i);

		if (all_one) {
			_Pragma("GCC unroll 8") for (r = 0; r < nr; r++)
				a[r] = _mm512_xor_si512(a[r], x);
		} else {
			_Pragma("GCC unroll 8") for (r = 0; r < nr; r++)
				a[r] = _mm512_xor_si512(a[r], _mm512_gf2p8affine_epi64_epi8(
								x, _mm512_set1_epi64((long long)m[j * RG + r]), 0));
		}
	}
	_Pragma("GCC unroll 8") for (r = 0; r < nr; r++) {
		if (full)
			_mm512_storeu_si512(d[r] + i, a[r]);
		else
			_mm512_mask_storeu_epi8(d[r] + i, mk, a[r]);
	}
}

static inline __attribute__((always_inline, target("avx512f,avx512bw,gfni")))
void pass_avx512_gfni_body(const struct pass *q, const int nr)
{
	uint64_t m[SG * RG];			/* [source][row] */
	const unsigned char *s[SG];
	unsigned char *d[RG];
	const int ns = q->ns, acc = q->acc, all_one = q->all_one;
	const size_t len = q->len, full = len & ~(size_t)63;
	size_t i;
	int r, j;

	for (j = 0; j < ns; j++) {
		s[j] = q->src[j];
		for (r = 0; r < nr; r++)
			m[j * RG + r] = g_aff[q->cf[r * ns + j]];
	}
	for (r = 0; r < nr; r++)
		d[r] = q->dst[r];
	for (i = 0; i < full; i += 64)
		col_avx512_gfni(d, s, m, i, ~(__mmask64)0, 1, nr, ns, acc, all_one);
	if (i < len)
		col_avx512_gfni(d, s, m, i, ((__mmask64)1 << (len - i)) - 1, 0, nr, ns, acc, all_one);
}

static inline __attribute__((always_inline, target("avx2,gfni")))
void pass_avx2_gfni_body(const struct pass *q, const int nr)
{
	uint64_t m[SG * RG];			/* [source][row] */
	const unsigned char *s[SG];
	unsigned char *d[RG];
	__m256i a[RG];
	const int ns = q->ns, acc = q->acc, all_one = q->all_one;
	const size_t len = q->len;
	size_t i;
	int r, j;

	for (j = 0; j < ns; j++) {
		s[j] = q->src[j];
		for (r = 0; r < nr; r++)
			m[j * RG + r] = g_aff[q->cf[r * ns + j]];
	}
	for (r = 0; r < nr; r++)
		d[r] = q->dst[r];
	for (i = 0; i + 32 <= len; i += 32) {
		_Pragma("GCC unroll 8") for (r = 0; r < nr; r++)
			a[r] = acc ? _mm256_loadu_si256((const __m256i *)(d[r] + i)) : _mm256_setzero_si256();
		for (j = 0; j < ns; j++) {
			const __m256i x = _mm256_loadu_si256((const __m256i *)(s[j] + i));

			_Pragma("GCC unroll 8") for (r = 0; r < nr; r++)
				a[r] = _mm256_xor_si256(a[r], all_one ? x : _mm256_gf2p8affine_epi64_epi8(
						x, _mm256_set1_epi64x((long long)m[j * RG + r]), 0));
		}
		_Pragma("GCC unroll 8") for (r = 0; r < nr; r++)
			_mm256_storeu_si256((__m256i *)(d[r] + i), a[r]);
	}
	tail_bytes(q, i);
}

static inline __attribute__((always_inline, target("avx2")))
void pass_avx2_body(const struct pass *q, const int nr)
{
	const __m256i low4 = _mm256_set1_epi8(0x0f);
	const unsigned char *t[SG * RG];	/* [source][row] nibble tables */
	const unsigned char *s[SG];
	unsigned char *d[RG];
	__m256i a[RG];
	const int ns = q->ns, acc = q->acc, all_one = q->all_one;
	const size_t len = q->len;
	size_t i;
	int r, j;

	for (j = 0; j < ns; j++) {
		s[j] = q->src[j];
		for (r = 0; r < nr; r++)
			t[j * RG + r] = g_nib[q->cf[r * ns + j]];
	}
	for (r = 0; r < nr; r++)
		d[r] = q->dst[r];
	for (i = 0; i + 32 <= len; i += 32) {
		_Pragma("GCC unroll 8") for (r = 0; r < nr; r++)
			a[r] = acc ? _mm256_loadu_si256((const __m256i *)(d[r] + i)) : _mm256_setzero_si256();
		for (j = 0; j < ns; j++) {
			const __m256i x = _mm256_loadu_si256((const __m256i *)(s[j] + i));
			const __m256i lo = _mm256_and_si256(x, low4);
			const __m256i hi = _mm256_and_si256(_mm256_srli_epi16(x, 4), low4);

			if (all_one) {
				_Pragma("GCC unroll 8") for (r = 0; r < nr; r++)
					a[r] = _mm256_xor_si256(a[r], x);
				continue;
			}
			_Pragma("GCC unroll 8") for (r = 0; r < nr; r++) {
				const unsigned char *tb = t[j * RG + r];
				const __m256i tl = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)tb));
				const __m256i th = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)(tb + 16)));

				a[r] = _mm256_xor_si256(a[r], _mm256_xor_si256(_mm256_shuffle_epi8(tl, lo),
										_mm256_shuffle_epi8(th, hi)));
			}
		}
		_Pragma("GCC unroll 8") for (r = 0; r < nr; r++)
			_mm256_storeu_si256((__m256i *)(d[r] + i), a[r]);
	}
	tail_bytes(q, i);
}

/* one instance per row count: the accumulators then live in registers */
#define ROW_INSTANCES(name, tgt)                                                              \
	__attribute__((target(tgt))) static void name##_1(const struct pass *q) { name##_body(q, 1); } \
	__attribute__((target(tgt))) static void name##_2(const struct pass *q) { name##_body(q, 2); } \
	__attribute__((target(tgt))) static void name##_3(const struct pass *q) { name##_body(q, 3); } \
	__attribute__((target(tgt))) static void name##_4(const struct pass *q) { name##_body(q, 4); } \
	__attribute__((target(tgt))) static void name##_5(const struct pass *q) { name##_body(q, 5); } \
	__attribute__((target(tgt))) static void name##_6(const struct pass *q) { name##_body(q, 6); } \
	__attribute__((target(tgt))) static void name##_7(const struct pass *q) { name##_body(q, 7); } \
	__attribute__((target(tgt))) static void name##_8(const struct pass *q) { name##_body(q, 8); } \
	static void name(const struct pass *q)                                                \
	{                                                                                     \
		static void (*const f[RG])(const struct pass *) = {                           \
			name##_1, name##_2, name##_3, name##_4, name##_5, name##_6, name##_7, name##_8}; \
		f[q->nr - 1](q);                                                              \
	}

ROW_INSTANCES(pass_avx512_gfni, "avx512f,avx512bw,gfni")
ROW_INSTANCES(pass_avx2_gfni, "avx2,gfni")
ROW_INSTANCES(pass_avx2, "avx2")

static void pass_scalar(const struct pass *q)
{
	tail_bytes(q, 0);
}

int ecg_cpu_matmul(int len, int k, int rows, const unsigned char *coef, unsigned char *const *src,
		   unsigned char *const *dst, unsigned flags)
{
	static void (*const fn[ISA_N])(const struct pass *) = {pass_scalar, pass_avx2, pass_avx2_gfni,
								pass_avx512_gfni};
	unsigned char cf[RG * SG];
	void (*run)(const struct pass *);
	int isa, r0, j0, r, j, all_one = 1;

	if (len < 0 || k < 1 || k > ECG_MAX_K + 256 || rows < 1 || rows > 256)
		return ecg_fail(-ECG_DER_INVAL, "cpu_matmul: bad len=%d k=%d rows=%d", len, k, rows);
	if (len == 0)
		return 0;
	if (src == NULL || dst == NULL || coef == NULL)
		return ecg_fail(-ECG_DER_INVAL, "cpu_matmul: NULL argument");
	pthread_once(&g_once, cpu_init);
	isa = __atomic_load_n(&g_isa, __ATOMIC_RELAXED);
	run = fn[isa];
	for (j = 0; j < k * rows && all_one; j++)
		all_one = coef[j] == 1;
	for (r0 = 0; r0 < rows; r0 += RG) {
		const int nr = rows - r0 < RG ? rows - r0 : RG;

		for (j0 = 0; j0 < k; j0 += SG) {
			const int ns = k - j0 < SG ? k - j0 : SG;
			struct pass q = {
				.len = (size_t)len, .nr = nr, .ns = ns, .all_one = all_one, .cf = cf,
				.src = (const unsigned char *const *)(src + j0), .dst = dst + r0,
				.acc = j0 > 0 || (flags & ECG_F_ACCUMULATE) != 0,
			};

			for (r = 0; r < nr; r++)
				for (j = 0; j < ns; j++)
					cf[r * ns + j] = coef[(size_t)(r0 + r) * k + j0 + j];
			run(&q);
		}
	}
	ecg_set_last_kernel(isa == ISA_AVX512_GFNI ? "cpu:avx512-gfni" : isa == ISA_AVX2_GFNI ? "cpu:avx2-gfni" :
			    isa == ISA_AVX2 ? "cpu:avx2" : "cpu:scalar");
	return 0;
}
