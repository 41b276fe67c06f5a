// ecg_crc_dev.h -- CRC device helpers shared by the checksum kernels
// (ecg_csum_kernels.hip) and the fused product + checksum kernels
// (ecg_kernels.hip).  W-bit register, NB = W/8; tables are the host-built
// image described in ecg_kabi.h.  See ecg_csum_kernels.hip for the scheme.
#ifndef ECG_CRC_DEV_H
#define ECG_CRC_DEV_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../ecg_kabi.h"

namespace ecg_crc {

template <int W> struct reg { using T = uint32_t; };
template <> struct reg<64> { using T = uint64_t; };

// state -> state shifted by a fixed number of zero bytes (byte-wise linear map)
template <int W, typename T>
__device__ __forceinline__ T lin_map(T c, const T *tb)
{
	T r = 0;
#pragma unroll
	for (int j = 0; j < W / 8; j++)
		r ^= tb[j * 256 + (uint32_t)((c >> (8 * j)) & 0xff)];
	return r;
}

// raw CRC (zero register) of one 16-byte piece, slice-by-NB with the register
// folded into each NB-byte word
template <int W, bool REFL, typename T>
__device__ __forceinline__ T piece_crc(const uint32_t d[4], const T *sl)
{
	T c = 0;
	if constexpr (W == 32) {
#pragma unroll
		for (int j = 0; j < 4; j++) {
			const uint32_t x = c ^ d[j];
			c = sl[3 * 256 + (x & 0xff)] ^ sl[2 * 256 + ((x >> 8) & 0xff)] ^
			    sl[1 * 256 + ((x >> 16) & 0xff)] ^ sl[x >> 24];
		}
	} else if constexpr (W == 64) {
#pragma unroll
		for (int h = 0; h < 2; h++) {
			const uint32_t lo = (uint32_t)c ^ d[2 * h], hi = (uint32_t)(c >> 32) ^ d[2 * h + 1];
			c = sl[7 * 256 + (lo & 0xff)] ^ sl[6 * 256 + ((lo >> 8) & 0xff)] ^
			    sl[5 * 256 + ((lo >> 16) & 0xff)] ^ sl[4 * 256 + (lo >> 24)] ^
			    sl[3 * 256 + (hi & 0xff)] ^ sl[2 * 256 + ((hi >> 8) & 0xff)] ^
			    sl[1 * 256 + ((hi >> 16) & 0xff)] ^ sl[hi >> 24];
		}
	} else {
		// crc16/T10-DIF, MSB first: byte pairs (b0, b1) -> x = c ^ (b0 << 8 | b1)
#pragma unroll
		for (int j = 0; j < 4; j++) {
#pragma unroll
			for (int h = 0; h < 2; h++) {
				const uint32_t b0 = (d[j] >> (16 * h)) & 0xff, b1 = (d[j] >> (16 * h + 8)) & 0xff;
				c = sl[256 + (((c >> 8) ^ b0) & 0xff)] ^ sl[((c ^ b1) & 0xff)];
			}
		}
	}
	return c;
}

// raw CRC (zero register) of one 16-byte piece from the s16 tables: 16
// independent lookups (no serial fold through the register)
template <int W, typename T>
__device__ __forceinline__ T piece_crc16(const uint32_t d[4], const T *s16)
{
	T c = 0;
#pragma unroll
	for (int j = 0; j < 4; j++)
#pragma unroll
		for (int b = 0; b < 4; b++)
			c ^= s16[(15 - 4 * j - b) * 256 + ((d[j] >> (8 * b)) & 0xffu)];
	return c;
}

// ---- 5-bit tables (ecg_kabi.h p5 / a5): every lookup hits a 32-entry table,
// so the lanes of a ds_read group never collide on a bank ----
template <int W>
struct f5 {
	static constexpr int NF = ECG_CSUM_NF5;			// fields of a 16-byte piece
	static constexpr int NA = ECG_CSUM_NA5(W / 8);		// fields of the register
	static constexpr int N = (NF + NA) * 32;		// LDS entries: p5 then a5
};

// field i of dword x: bits 5i..5i+4 (i = 6: bits 30-31)
__device__ __forceinline__ uint32_t fld5(uint32_t x, int i)
{
	return i == 6 ? x >> 30 : (x >> (5 * i)) & 31u;
}

// 3-input XOR (one v_bitop3_b32 per 32 bits)
__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c)
{
	return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint64_t x3(uint64_t a, uint64_t b, uint64_t c)
{
	return ((uint64_t)x3((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32)) << 32) |
	       x3((uint32_t)a, (uint32_t)b, (uint32_t)c);
}

// raw CRC (zero register) of one 16-byte piece: 28 lookups
template <int W, typename T>
__device__ __forceinline__ T piece_crc5(const uint32_t d[4], const T *p5)
{
	T c = 0;
#pragma unroll
	for (int j = 0; j < 4; j++)
#pragma unroll
		for (int i = 0; i < 7; i++)
			c ^= p5[(7 * j + i) * 32 + fld5(d[j], i)];
	return c;
}

// raw CRC of one 16-byte piece from the 5-bit tables at q5 + off bytes (off:
// a wave-uniform multiple of the 32-entry table size, e.g. the position
// table of a runtime position).  off is laundered so the compiler cannot
// prove (field & mask) | off disjoint and turn the OR into an add: each
// lookup address is then a shift and one v_and_or_b32, the cost of a fixed
// table's lookup.
template <int W, typename T>
__device__ __forceinline__ T piece_crc5p(const uint32_t d[4], const T *q5, uint32_t off)
{
	constexpr uint32_t ES = sizeof(T) == 8 ? 3 : 2;	// log2 entry bytes
	constexpr uint32_t M = 31u << ES, TS = 32u << ES;
	const char *b = (const char *)q5;
	T c = 0;

	asm volatile("" : "+v"(off));
#pragma unroll
	for (int j = 0; j < 4; j++) {
		const uint32_t x = d[j];
		const char *t = b + 7 * TS * j;
		const T e0 = *(const T *)(t + (((x << ES) & M) | off));
		const T e1 = *(const T *)(t + TS + (((x >> (5 - ES)) & M) | off));
		const T e2 = *(const T *)(t + 2 * TS + (((x >> (10 - ES)) & M) | off));
		const T e3 = *(const T *)(t + 3 * TS + (((x >> (15 - ES)) & M) | off));
		const T e4 = *(const T *)(t + 4 * TS + (((x >> (20 - ES)) & M) | off));
		const T e5 = *(const T *)(t + 5 * TS + (((x >> (25 - ES)) & M) | off));
		const T e6 = *(const T *)(t + 6 * TS + (((x >> (30 - ES)) & (3u << ES)) | off));
		c = x3(c, e0, e1);
		c = x3(c, e2, e3);
		c = x3(c, e4, e5);
		c ^= e6;
	}
	return c;
}

// ---- positional 5-bit tables: a Horner step over U = ECG_CSUM_P5U pieces
// of a lane, q5[u] being p5 followed by u strides of zero bytes, so the
// register is shifted once per U pieces (by U strides) instead of per piece:
// acc' = shift_U(acc) ^ XOR_u q5[U-1-u](piece u).  LDS image: q5[U][NF][32]
// then the a5 table of the U-stride shift.
template <int W, int U_ = ECG_CSUM_P5U>
struct f5u {
	static constexpr int U = U_;
	static constexpr int NF = ECG_CSUM_NF5;
	static constexpr int NA = ECG_CSUM_NA5(W / 8);
	static constexpr int N = (U * NF + NA) * 32;
};

// U pieces d[0..U-1] (in stream order) folded into acc
template <int W, typename T>
__device__ __forceinline__ T horner5u(T acc, const uint32_t (*d)[4], const T *q5)
{
	constexpr int U = f5u<W>::U, NF = ECG_CSUM_NF5;
	const T *a5 = q5 + U * NF * 32;
	T c;

	if constexpr (W == 16) {
		const uint32_t x = (uint32_t)acc;
		c = x3(a5[(x & 31u)], a5[32 + ((x >> 5) & 31u)], a5[64 + ((x >> 10) & 31u)]);
		c ^= a5[96 + ((x >> 15) & 31u)];
	} else {
		c = 0;
#pragma unroll
		for (int h = 0; h < W / 32; h++) {
			const uint32_t x = (uint32_t)((uint64_t)acc >> (32 * h));
			const T *a = a5 + 7 * 32 * h;
			c = x3(c, a[fld5(x, 0)], a[32 + fld5(x, 1)]);
			c = x3(c, a[64 + fld5(x, 2)], a[96 + fld5(x, 3)]);
			c = x3(c, a[128 + fld5(x, 4)], a[160 + fld5(x, 5)]);
			c ^= a[192 + fld5(x, 6)];
		}
	}
#pragma unroll
	for (int u = 0; u < U; u++) {
		const T *p5 = q5 + (U - 1 - u) * NF * 32;
#pragma unroll
		for (int j = 0; j < 4; j++) {
			const uint32_t x = d[u][j];
			const T *t = p5 + 7 * 32 * j;
			c = x3(c, t[fld5(x, 0)], t[32 + fld5(x, 1)]);
			c = x3(c, t[64 + fld5(x, 2)], t[96 + fld5(x, 3)]);
			c = x3(c, t[128 + fld5(x, 4)], t[160 + fld5(x, 5)]);
			c ^= t[192 + fld5(x, 6)];
		}
	}
	return c;
}

// stage q5 (p5 = position 0, positions 1..U-1 at gt + p5x_off) and the
// U-stride a5 (gt + a5_off) into LDS s5[f5u<W, U>::N]
template <int W, int U = ECG_CSUM_P5U, typename T>
__device__ __forceinline__ void stage5u(T *s5, const T *gt, int p5x_off, int a5_off, int nthreads)
{
	constexpr int NB = W / 8, P = ECG_CSUM_NF5 * 32;
	for (int i = threadIdx.x; i < f5u<W, U>::N; i += nthreads)
		s5[i] = i < P ? gt[ECG_CSUM_OFF_P5(NB) + i]
		      : i < U * P ? gt[p5x_off + i - P] : gt[a5_off + i - U * P];
}

// ---- nibble tables (ecg_kabi.h q4 / a4): a 16-byte piece is 32 nibbles, each
// indexing a 16-entry table (conflict-free like the 5-bit tables: 16 entries
// of 4 or 8 bytes sit on distinct banks).  The nibbles are byte-aligned, so a
// lookup's LDS address is ONE SDWA instruction on a byte of a pre-masked word
// (v_lshlrev_b32_sdwa: low nibble << log2(entry bytes); v_and_b32_sdwa: the
// high nibble already shifted into place) and the table's own offset rides in
// the ds_read's immediate offset -- 10 VALU per 8 lookups of a dword, against
// 2 per lookup (shift + and) for 5-bit fields.  The CRC kernels are VALU-issue
// bound (profiles/r03/crc_sq), so this is the count that matters.
template <int B, int ES>
__device__ __forceinline__ uint32_t nib_lo_addr(uint32_t lo)
{
	uint32_t r;
	static_assert(B >= 0 && B < 4 && (ES == 2 || ES == 3), "byte select / entry size");
	if constexpr (B == 0)
		asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"
		    : "=v"(r) : "i"(ES), "v"(lo));
	else if constexpr (B == 1)
		asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
		    : "=v"(r) : "i"(ES), "v"(lo));
	else if constexpr (B == 2)
		asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2"
		    : "=v"(r) : "i"(ES), "v"(lo));
	else
		asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3"
		    : "=v"(r) : "i"(ES), "v"(lo));
	return r;
}

template <int B>
__device__ __forceinline__ uint32_t nib_hi_addr(uint32_t hs, uint32_t mask)
{
	uint32_t r;
	static_assert(B >= 0 && B < 4, "byte select");
	if constexpr (B == 0)
		asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"
		    : "=v"(r) : "s"(mask), "v"(hs));
	else if constexpr (B == 1)
		asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
		    : "=v"(r) : "s"(mask), "v"(hs));
	else if constexpr (B == 2)
		asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2"
		    : "=v"(r) : "s"(mask), "v"(hs));
	else
		asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3"
		    : "=v"(r) : "s"(mask), "v"(hs));
	return r;
}

template <int W, int U_ = ECG_CSUM_P5U>
struct f4u {
	static constexpr int U = U_;
	static constexpr int NF = 32;		// nibbles of a piece
	static constexpr int NA = W / 4;	// nibbles of the register
	static constexpr int N = (U * NF + NA) * 16;
};

// entry of table `tab` (16 entries each) at LDS byte address `a` (an SDWA
// result) from q: the constant part folds into the ds_read offset
template <typename T>
__device__ __forceinline__ T nib_ent(const T *q, int tab, uint32_t a)
{
	return *(const T *)((const char *)(q + 16 * tab) + a);
}

// XOR into c the 8 lookups of dword x (nibbles 8j .. 8j+7 of table group t0)
template <typename T>
__device__ __forceinline__ T nib_dword(T c, uint32_t x, const T *q, int t0, uint32_t hmask)
{
	constexpr int ES = sizeof(T) == 8 ? 3 : 2;
	const uint32_t lo = x & 0x0F0F0F0Fu;
	const uint32_t hs = x >> (4 - ES);
	c = x3(c, nib_ent(q, t0 + 0, nib_lo_addr<0, ES>(lo)), nib_ent(q, t0 + 1, nib_hi_addr<0>(hs, hmask)));
	c = x3(c, nib_ent(q, t0 + 2, nib_lo_addr<1, ES>(lo)), nib_ent(q, t0 + 3, nib_hi_addr<1>(hs, hmask)));
	c = x3(c, nib_ent(q, t0 + 4, nib_lo_addr<2, ES>(lo)), nib_ent(q, t0 + 5, nib_hi_addr<2>(hs, hmask)));
	c = x3(c, nib_ent(q, t0 + 6, nib_lo_addr<3, ES>(lo)), nib_ent(q, t0 + 7, nib_hi_addr<3>(hs, hmask)));
	return c;
}

// high-nibble mask for nib_dword: (x >> (4 - ES)) & mask = high nibble << ES
template <typename T>
__device__ __forceinline__ uint32_t nib_hmask()
{
	return sizeof(T) == 8 ? 0x78u : 0x3Cu;
}

// U pieces d[0..U-1] (in stream order) folded into acc with the nibble
// tables q4 (LDS: q4[U][32][16], then a4[W/4][16] of the U-stride shift)
template <int W, int U, typename T>
__device__ __forceinline__ T horner4u(T acc, const uint32_t (*d)[4], const T *q4, uint32_t hmask)
{
	const T *a4 = q4 + U * 32 * 16;
	T c = 0;

#pragma unroll
	for (int h = 0; h < (W + 31) / 32; h++) {
		const uint32_t x = W == 16 ? (uint32_t)acc & 0xFFFFu : (uint32_t)((uint64_t)acc >> (32 * h));
		if constexpr (W == 16) {	// 4 nibbles: bytes 0, 1 of the low half
			constexpr int ES = sizeof(T) == 8 ? 3 : 2;
			const uint32_t lo = x & 0x0F0Fu, hs = x >> (4 - ES);
			c = x3(c, nib_ent(a4, 0, nib_lo_addr<0, ES>(lo)), nib_ent(a4, 1, nib_hi_addr<0>(hs, hmask)));
			c = x3(c, nib_ent(a4, 2, nib_lo_addr<1, ES>(lo)), nib_ent(a4, 3, nib_hi_addr<1>(hs, hmask)));
		} else {
			c = nib_dword(c, x, a4, 8 * h, hmask);
		}
	}
#pragma unroll
	for (int u = 0; u < U; u++) {
		const T *p4 = q4 + (U - 1 - u) * 32 * 16;
#pragma unroll
		for (int j = 0; j < 4; j++)
			c = nib_dword(c, d[u][j], p4, 8 * j, hmask);
	}
	return c;
}

// stage q4 (positions 0..U-1 at gt + q4_off) and a4 (gt + a4_off) into LDS
template <int W, int U, typename T>
__device__ __forceinline__ void stage4u(T *s4, const T *gt, int q4_off, int a4_off, int nthreads)
{
	constexpr int P = U * 32 * 16;
	for (int i = threadIdx.x; i < f4u<W, U>::N; i += nthreads)
		s4[i] = i < P ? gt[q4_off + i] : gt[a4_off + i - P];
}

// lane value * x^(8*16*(63-lane)) for reflected CRCs, nibble by nibble: the
// per-lane tables nibl[16][64] are read from the table image in HBM/L2 (they
// depend only on the value, so all W/4 loads issue together), the 4-bit
// reduction r4 from LDS -- W/4 steps instead of mulmod's W bit steps
template <int W, typename T>
__device__ __forceinline__ T lane_mul_nib(T x, const T *gnib, const T *r4, uint32_t lane)
{
	T n[W / 4];
#pragma unroll
	for (int i = 0; i < W / 4; i++)
		n[i] = gnib[(((uint32_t)(x >> (4 * i))) & 15u) * 64u + lane];
	T u = 0;
#pragma unroll
	for (int i = 0; i < W / 4; i++)
		u = (u >> 4) ^ r4[(uint32_t)u & 15u] ^ n[i];
	return u;
}

// raw CRC of one 16-byte piece from the s16 byte tables (16 independent
// lookups; table 15 - 4j - b for byte b of dword j), each address ONE SDWA
// instruction (byte << log2(entry bytes)) with the table's offset in the
// ds_read's immediate: 16 + NB*2 VALU per piece for crc32 instead of ~50 with
// shift-and-mask addresses.  Byte tables are bank-conflicted (~3x per
// lookup), so this pays where the LDS has slack -- the fused product +
// checksum kernels, whose VALU carries the GF product too.
template <int W, typename T>
__device__ __forceinline__ T piece_crc16s(const uint32_t d[4], const T *s16)
{
	constexpr int ES = sizeof(T) == 8 ? 3 : 2;
	T c = 0;

#pragma unroll
	for (int j = 0; j < 4; j++) {
		const uint32_t x = d[j];
		c = x3(c, nib_ent(s16, 16 * (15 - 4 * j), nib_lo_addr<0, ES>(x)),
		       nib_ent(s16, 16 * (14 - 4 * j), nib_lo_addr<1, ES>(x)));
		c = x3(c, nib_ent(s16, 16 * (13 - 4 * j), nib_lo_addr<2, ES>(x)),
		       nib_ent(s16, 16 * (12 - 4 * j), nib_lo_addr<3, ES>(x)));
	}
	return c;
}

// raw CRC of one 16-byte piece from one position's nibble tables q4[32][16]
// (32 conflict-free lookups, one SDWA address each; the fused workgroup
// kernel's TB 4: the position selects how many columns follow the piece)
template <typename T>
__device__ __forceinline__ T piece_crc4(const uint32_t d[4], const T *q4)
{
	const uint32_t hmask = nib_hmask<T>();
	T c = 0;

#pragma unroll
	for (int j = 0; j < 4; j++)
		c = nib_dword(c, d[j], q4, 8 * j, hmask);
	return c;
}

// register -> register shifted by the a4 table's fixed number of zero bytes
// (nibble fields, SDWA addresses; a4[16][16], rows >= W/4 unused)
template <int W, typename T>
__device__ __forceinline__ T lin_map4(T acc, const T *a4)
{
	const uint32_t hmask = nib_hmask<T>();
	T c = 0;

#pragma unroll
	for (int h = 0; h < (W + 31) / 32; h++) {
		const uint32_t x = W == 16 ? (uint32_t)acc & 0xFFFFu : (uint32_t)((uint64_t)acc >> (32 * h));
		if constexpr (W == 16) {
			constexpr int ES = sizeof(T) == 8 ? 3 : 2;
			const uint32_t lo = x & 0x0F0Fu, hs = x >> (4 - ES);
			c = x3(c, nib_ent(a4, 0, nib_lo_addr<0, ES>(lo)), nib_ent(a4, 1, nib_hi_addr<0>(hs, hmask)));
			c = x3(c, nib_ent(a4, 2, nib_lo_addr<1, ES>(lo)), nib_ent(a4, 3, nib_hi_addr<1>(hs, hmask)));
		} else {
			c = nib_dword(c, x, a4, 8 * h, hmask);
		}
	}
	return c;
}

// register -> register shifted by the a5 table's fixed number of zero bytes
template <int W, typename T>
__device__ __forceinline__ T lin_map5(T c, const T *a5)
{
	T r;
	if constexpr (W == 16) {
		const uint32_t x = (uint32_t)c;
		r = x3(a5[(x & 31u)], a5[32 + ((x >> 5) & 31u)], a5[64 + ((x >> 10) & 31u)]);
		r ^= a5[96 + ((x >> 15) & 31u)];
	} else {
		r = 0;
#pragma unroll
		for (int h = 0; h < W / 32; h++) {
			const uint32_t x = (uint32_t)((uint64_t)c >> (32 * h));
			const T *a = a5 + 7 * 32 * h;
			r = x3(r, a[fld5(x, 0)], a[32 + fld5(x, 1)]);
			r = x3(r, a[64 + fld5(x, 2)], a[96 + fld5(x, 3)]);
			r = x3(r, a[128 + fld5(x, 4)], a[160 + fld5(x, 5)]);
			r ^= a[192 + fld5(x, 6)];
		}
	}
	return r;
}

// stage p5 and one a5 section (entries at gt + a5_off) into LDS s5[f5<W>::N]
template <int W, typename T>
__device__ __forceinline__ void stage5(T *s5, const T *gt, int a5_off, int nthreads)
{
	constexpr int NB = W / 8;
	for (int i = threadIdx.x; i < f5<W>::N; i += nthreads)
		s5[i] = i < f5<W>::NF * 32 ? gt[ECG_CSUM_OFF_P5(NB) + i] : gt[a5_off + i - f5<W>::NF * 32];
}

template <int W, bool REFL, typename T>
__device__ __forceinline__ T byte_step(T c, uint32_t b, const T *sl)
{
	if constexpr (REFL)
		return (c >> 8) ^ sl[(uint32_t)((c ^ b) & 0xff)];
	else
		return (T)(((c << 8) & 0xffff) ^ sl[(uint32_t)(((c >> 8) ^ b) & 0xff)]);
}

// a * b mod P over GF(2): reflected (bit W-1 = x^0) or MSB-first (bit i = x^i)
template <int W, bool REFL, typename T>
__device__ __forceinline__ T mulmod(T a, T b, T poly)
{
	T p = 0;
	if constexpr (REFL) {
#pragma unroll
		for (int i = W - 1; i >= 0; i--) {
			p ^= b & (T)(0 - ((a >> i) & 1));
			b = (b >> 1) ^ (poly & (T)(0 - (b & 1)));
		}
	} else {
		const T mask = (T)((((uint64_t)1) << W) - 1);
#pragma unroll
		for (int i = W - 1; i >= 0; i--) {
			p = ((p << 1) & mask) ^ (poly & (T)(0 - ((p >> (W - 1)) & 1)));
			p ^= b & (T)(0 - ((a >> i) & 1));
		}
	}
	return p;
}

// a wave-uniform value moved to SGPRs (so arithmetic on it runs on the
// scalar unit)
template <typename T>
__device__ __forceinline__ T uniform(T v)
{
	// (the builtin returns int: cast through uint32_t, or the low half would
	// be sign-extended into the high half)
	if constexpr (sizeof(T) == 8)
		return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
		       (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
	else
		return (T)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
}

// XOR of one 32-bit word over the 64 lanes, as a wave-uniform value: DPP
// steps inside rows (pairs, quads, half-row and row mirrors), row broadcasts
// across rows, lane 63 read into an SGPR -- VALU only, no LDS crossbar
// (ds_bpermute) round trips.  Every lane must be active.
__device__ __forceinline__ uint32_t wave_xor_dpp32(uint32_t x)
{
	x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);	// quad_perm [1,0,3,2]
	x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);	// quad_perm [2,3,0,1]
	x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false);	// row_half_mirror
	x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false);	// row_mirror
	x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);	// row_bcast:15 -> rows 1, 3
	x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);	// row_bcast:31 -> rows 2, 3
	return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

template <typename T>
__device__ __forceinline__ T wave_xor_uniform(T v)
{
	if constexpr (sizeof(T) == 8)
		return ((uint64_t)wave_xor_dpp32((uint32_t)(v >> 32)) << 32) | wave_xor_dpp32((uint32_t)v);
	else
		return (T)wave_xor_dpp32((uint32_t)v);
}

template <typename T>
__device__ __forceinline__ T wave_xor(T v)
{
	if constexpr (sizeof(T) == 8) {
		uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#pragma unroll
		for (int s = 32; s >= 1; s >>= 1) {
			lo ^= __shfl_xor(lo, s);
			hi ^= __shfl_xor(hi, s);
		}
		return ((uint64_t)hi << 32) | lo;
	} else {
#pragma unroll
		for (int s = 32; s >= 1; s >>= 1)
			v ^= __shfl_xor(v, s);
		return v;
	}
}

} // namespace ecg_crc

#endif
