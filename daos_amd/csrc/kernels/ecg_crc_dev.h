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

// register -> register shifted by the a5 table's fixed number of zero bytes
template <int W, typename T>
__device__ __forceinline__ T lin_map5(T c, const T *a5)
{
	T r = 0;
	if constexpr (W == 16) {
		const uint32_t x = (uint32_t)c;
#pragma unroll
		for (int i = 0; i < 4; i++)
			r ^= a5[i * 32 + ((x >> (5 * i)) & 31u)];
	} else {
#pragma unroll
		for (int h = 0; h < W / 32; h++) {
			const uint32_t x = (uint32_t)((uint64_t)c >> (32 * h));
#pragma unroll
			for (int i = 0; i < 7; i++)
				r ^= a5[(7 * h + i) * 32 + fld5(x, i)];
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
