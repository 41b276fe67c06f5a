// ecg_csum_kernels.hip -- chunked checksums of device-resident cells for gfx950.
//
// DAOS checksums every chunk of an extent it writes, including the parity
// cells rebuild regenerates (ref:src/object/srv_obj_migrate.c:1156) and the
// cells recovery rebuilds; the csummer hashes each chunk from a reset state
// (ref:src/common/checksum.c:467-497) with one of crc16 / crc32 / crc64 /
// adler32 (ref:src/common/multihash_isal.c:27-256).  This file computes the
// same values on the device, one wavefront per chunk, so regenerated cells
// never leave HBM to be checksummed.
//
// CRC scheme (W-bit register, NB = W/8 bytes):
//  * lane l takes the 16-byte pieces q = 64*i + l - z of its chunk: every
//    load instruction of the wave reads 1 KiB contiguous (coalesced);
//  * z zero pieces are prepended so every lane has the same piece count m;
//    leading zeros do not change a zero-initialised CRC;
//  * per piece: acc = shift_1KiB(acc) ^ crc(piece)  -- Horner over the
//    lane's pieces, the shift being a byte-wise linear map (NB lookups) and
//    crc(piece) slice-by-NB with the register folded in (16 lookups);
//  * lane l's sum is then multiplied by x^(8*16*(63-l)) mod P (GF(2)
//    polynomial multiply, W steps) and the wave XOR-reduces: the chunk's
//    raw CRC of its 16-byte-aligned part; lane 0 finishes the <16 B tail
//    byte by byte;
//  * a non-zero initial register (crc64: ~0) is XORed into the first NB
//    bytes of the chunk, the standard identity for reflected CRCs.
// Tables live in LDS (crc16 4 KiB, crc32 8 KiB, crc64 32 KiB per block) and
// blocks stride over chunks so each block loads them once.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../ecg_kabi.h"
#include "ecg_crc_dev.h"

namespace {

using namespace ecg_crc;

constexpr int CS_BLOCK = 256;
constexpr int CS_WAVES = CS_BLOCK / 64;
#ifndef ECG_CS_UNROLL
#define ECG_CS_UNROLL 4
#endif
constexpr int CS_UNROLL = ECG_CS_UNROLL;	// pieces in flight per lane
constexpr uint32_t ADLER_MOD = 65521;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool ALIGNED>
__device__ __forceinline__ void load16(const uint8_t *p, uint32_t d[4])
{
	if constexpr (ALIGNED) {
		const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
		d[0] = v.x;
		d[1] = v.y;
		d[2] = v.z;
		d[3] = v.w;
	} else {
#pragma unroll
		for (int j = 0; j < 4; j++)
			d[j] = (uint32_t)p[4 * j] | ((uint32_t)p[4 * j + 1] << 8) |
			       ((uint32_t)p[4 * j + 2] << 16) | ((uint32_t)p[4 * j + 3] << 24);
	}
}

__device__ __forceinline__ void chunk_geom(const ecg_csum_params_t &p, uint64_t g, uint64_t &off,
					   uint64_t &len, const uint8_t *&base)
{
	const uint64_t e = g / p.nchunks, c = g - e * p.nchunks;

	off = c == 0 ? 0 : p.first_bytes + (c - 1) * p.chunk_bytes;
	len = c == 0 ? p.first_bytes : p.chunk_bytes;
	if (off + len > p.ext_bytes)
		len = p.ext_bytes - off;
	base = p.src + (int64_t)e * p.ext_stride + off;
}

// CRC table kinds (ecg_kabi.h): TK_5 conflict-free 5-bit fields, TK_B8 byte
// tables (the A/B variant), TK_4 nibble fields addressed by SDWA byte selects
// (the default: fewest VALU per lookup, and the CRC kernels are VALU-issue
// bound -- profiles/r03/crc_sq)
constexpr int TK_5 = 0, TK_B8 = 1, TK_4 = 2;

// Horner steps of a lane's accumulator over the UN pieces d[0..UN-1] (those
// with i + u < m): byte tables (sl, sh), one step per piece, acc * x^(8 *
// stride) ^ crc(piece); 5-bit / nibble tables (s5 = positional q then a),
// one step per UN = ECG_CSUM_P5U pieces (m is then a multiple of UN).
template <int W, bool REFL, int TK, int UN, typename T>
__device__ __forceinline__ T horner(T acc, const uint32_t (*d)[4], int64_t i, int64_t m, const T *s5,
				    const T *sl, const T *sh)
{
	if constexpr (TK == TK_B8) {
#pragma unroll
		for (int u = 0; u < UN; u++)
			if (i + u < m)
				acc = lin_map<W>(acc, sh) ^ piece_crc<W, REFL>(d[u], sl);
		return acc;
	} else if constexpr (TK == TK_4) {
		static_assert(UN == ECG_CSUM_P5U, "nibble path steps ECG_CSUM_P5U pieces at a time");
		return horner4u<W, UN>(acc, d, s5, nib_hmask<T>());
	} else {
		static_assert(UN == ECG_CSUM_P5U, "5-bit path steps ECG_CSUM_P5U pieces at a time");
		return horner5u<W>(acc, d, s5);
	}
}

// LDS images of one kernel: the positional 5-bit or nibble tables (q, a), or
// the byte tables; UN pieces in flight per lane
template <int W, int TK>
struct crc_lds {
	using T = typename reg<W>::T;
	static constexpr int NB = W / 8;
	static constexpr int N5 = TK == TK_B8 ? 1 : TK == TK_4 ? f4u<W>::N : f5u<W>::N;
	static constexpr int NSL = TK == TK_B8 ? NB * 256 : 1;
	static constexpr int UN = TK == TK_B8 ? CS_UNROLL : ECG_CSUM_P5U;
};

// positional tables of stride `q_off` (5-bit p5x / nibble q4) and the
// U-stride shift into LDS
template <int W, int TK, typename T>
__device__ __forceinline__ void stage_tables(T *s5, T *sl, T *sh, const T *gt, int p5x_off, int a5_off,
					     int q4_off, int a4_off, int nthreads)
{
	constexpr int NB = W / 8;
	if constexpr (TK == TK_B8) {
		for (int i = threadIdx.x; i < NB * 256; i += nthreads) {
			sl[i] = gt[i];
			sh[i] = gt[NB * 256 + i];
		}
	} else if constexpr (TK == TK_4) {
		stage4u<W, ECG_CSUM_P5U>(s5, gt, q4_off, a4_off, nthreads);
	} else {
		stage5u<W>(s5, gt, p5x_off, a5_off, nthreads);
	}
}

// the lane's final shift x^(8*16*(G-1-l)) (G lanes per chunk; klane = its
// k64 entry): reflected CRCs from the nibl tables (W/4 steps), else mulmod
template <int W, bool REFL, typename T>
__device__ __forceinline__ T lane_shift(T acc, T klane, const T *gt, const T *r4, uint32_t nib_lane, T poly)
{
	if constexpr (REFL)
		return lane_mul_nib<W>(acc, gt + ECG_CSUM_OFF_NIBL(W / 8), r4, nib_lane);
	else
		return mulmod<W, REFL>(klane, acc, poly);
}

// lane steps of a chunk of nq pieces, `per` pieces per step
template <int TK>
__device__ __forceinline__ int64_t lane_steps(int64_t nq, int64_t per)
{
	const int64_t m = (nq + per - 1) / per;
	return TK == TK_B8 ? m : (m + ECG_CSUM_P5U - 1) / ECG_CSUM_P5U * ECG_CSUM_P5U;
}

// the U pieces of lane step i (pieces (i+u)*64 + lane - z): `first` masks
// the zero prefix (q < 0) and folds the initial register into piece 0; later
// steps are unconditional (q > 0 for i >= ECG_CSUM_P5U since z < 64 U)
template <int UN, int W, bool ALIGNED, bool FIRST, typename T>
__device__ __forceinline__ void load_step(const uint8_t *base, int64_t i, int64_t stride_pieces, int64_t lane_q0,
					  int64_t m, T init, uint32_t (*d)[4])
{
#pragma unroll
	for (int u = 0; u < UN; u++) {
		const int64_t q = (i + u) * stride_pieces + lane_q0;
		if constexpr (FIRST) {
			if (i + u < m && q >= 0) {
				load16<ALIGNED>(base + 16 * q, d[u]);
				if (q == 0) {	// fold the initial register into the first bytes
					d[u][0] ^= (uint32_t)init;
					if constexpr (W == 64)
						d[u][1] ^= (uint32_t)((uint64_t)init >> 32);
				}
			} else {
				d[u][0] = d[u][1] = d[u][2] = d[u][3] = 0;
			}
		} else {
			load16<ALIGNED>(base + 16 * q, d[u]);
		}
	}
}

// chunk g's geometry with a 32-bit division when the counts allow (the
// 64-bit one expands to ~100 VALU per chunk)
__device__ __forceinline__ void chunk_geom_fast(const ecg_csum_params_t &p, uint64_t g, uint64_t &off,
						uint64_t &len, const uint8_t *&base)
{
	if (((g | p.nchunks) >> 32) == 0) {
		const uint32_t e = (uint32_t)g / p.nchunks, c = (uint32_t)g - e * p.nchunks;

		off = c == 0 ? 0 : p.first_bytes + (uint64_t)(c - 1) * p.chunk_bytes;
		len = c == 0 ? p.first_bytes : p.chunk_bytes;
		if (off + len > p.ext_bytes)
			len = p.ext_bytes - off;
		base = p.src + (int64_t)e * p.ext_stride + off;
	} else {
		chunk_geom(p, g, off, len, base);
	}
}

template <int W, bool REFL, bool ALIGNED, int TK>
__global__ __launch_bounds__(CS_BLOCK) void ecg_crc_kernel(ecg_csum_params_t p)
{
	using T = typename reg<W>::T;
	using L = crc_lds<W, TK>;
	constexpr int NB = W / 8;
	__shared__ T s5[L::N5];
	__shared__ T sl[L::NSL];
	__shared__ T sh[L::NSL];
	__shared__ T r4[REFL ? 16 : 1];
	const T *gt = (const T *)p.tbl;

	stage_tables<W, TK>(s5, sl, sh, gt, ECG_CSUM_OFF_P5X_1K(NB), ECG_CSUM_OFF_A5_4K(NB), ECG_CSUM_OFF_Q4_1K(NB),
			    ECG_CSUM_OFF_A4_4K(NB), CS_BLOCK);
	if (REFL && threadIdx.x < 16)
		r4[threadIdx.x] = gt[ECG_CSUM_OFF_R4(NB) + threadIdx.x];
	const int lane = threadIdx.x & 63;
	const T klane = REFL ? (T)0 : gt[2 * NB * 256 + lane];
	const T poly = (T)p.poly, init = (T)p.init, xorout = (T)p.xorout;
	__syncthreads();

	const uint64_t total = (uint64_t)p.n_ext * p.nchunks;
	const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	for (uint64_t g = (uint64_t)blockIdx.x * CS_WAVES + wv; g < total; g += (uint64_t)gridDim.x * CS_WAVES) {
		uint64_t off, len;
		const uint8_t *base;

		chunk_geom_fast(p, g, off, len, base);
		const int64_t nq = (int64_t)(len / 16);
		const int64_t m = lane_steps<TK>(nq, 64);
		const int64_t z = m * 64 - nq;
		T acc = 0;

		if (m > 0) {
			uint32_t d[L::UN][4];

			load_step<L::UN, W, ALIGNED, true>(base, 0, 64, lane - z, m, init, d);
			acc = horner<W, REFL, TK, L::UN>(acc, d, 0, m, s5, sl, sh);
			for (int64_t i = L::UN; i < m; i += L::UN) {
				load_step<L::UN, W, ALIGNED, TK == TK_B8>(base, i, 64, lane - z, m, init, d);	// byte tables: m need not be a multiple of UN
				acc = horner<W, REFL, TK, L::UN>(acc, d, i, m, s5, sl, sh);
			}
		}
		acc = lane_shift<W, REFL>(acc, klane, gt, r4, (uint32_t)lane, poly);
		acc = wave_xor_uniform(acc);	// DPP, no ds_bpermute
		if (lane == 0) {
			T crc = nq == 0 ? init : acc;

			for (uint64_t b = (uint64_t)nq * 16; b < len; b++)	// tail bytes: sl[0] in memory
				crc = byte_step<W, REFL>(crc, base[b], gt);
			crc ^= xorout;
			if constexpr (W == 16)
				((uint16_t *)p.out)[g] = (uint16_t)crc;
			else
				((T *)p.out)[g] = crc;
		}
	}
}

template <typename T>
__device__ __forceinline__ T shfl_xor_t(T v, int s)
{
	if constexpr (sizeof(T) == 8)
		return ((uint64_t)(uint32_t)__shfl_xor((uint32_t)(v >> 32), s) << 32) |
		       (uint32_t)__shfl_xor((uint32_t)v, s);
	else
		return (T)__shfl_xor((uint32_t)v, s);
}

// Short chunks (<= 8 KiB): with a wave per chunk each lane holds only 1-8
// pieces and the per-lane final multiply (W GF(2) steps) dominates.  Here a
// group of G = ECG_CSUM_GLANES lanes takes a chunk (4 chunks per wave): lane
// l of the group takes pieces q = G*i + l - z, so each load instruction still
// reads 4 x 256 B contiguous, Horner-steps by G*16 bytes (sh256 table), and
// the group reduces with shuffles after multiplying by x^(8*16*(G-1-l)) =
// k64[64 - G + l].  Otherwise as ecg_crc_kernel.
template <int W, bool REFL, int TK>
__global__ __launch_bounds__(CS_BLOCK) void ecg_crc_group_kernel(ecg_csum_params_t p)
{
	using T = typename reg<W>::T;
	using L = crc_lds<W, TK>;
	constexpr int NB = W / 8;
	constexpr int G = ECG_CSUM_GLANES;
	constexpr int GPW = 64 / G;		// chunks per wave
	__shared__ T s5[L::N5];
	__shared__ T sl[L::NSL];
	__shared__ T sh[L::NSL];
	__shared__ T r4[REFL ? 16 : 1];
	const T *gt = (const T *)p.tbl;

	if constexpr (TK == TK_B8) {
		for (int i = threadIdx.x; i < NB * 256; i += CS_BLOCK) {
			sl[i] = gt[i];
			sh[i] = gt[ECG_CSUM_OFF_SH256(NB) + i];
		}
	} else {
		stage_tables<W, TK>(s5, sl, sh, gt, ECG_CSUM_OFF_P5X_256(NB), ECG_CSUM_OFF_A5_1K(NB),
				    ECG_CSUM_OFF_Q4_256(NB), ECG_CSUM_OFF_A4_1K(NB), CS_BLOCK);
	}
	if (REFL && threadIdx.x < 16)
		r4[threadIdx.x] = gt[ECG_CSUM_OFF_R4(NB) + threadIdx.x];
	const int lane = threadIdx.x & 63, gl = lane % G;
	const T klane = gt[ECG_CSUM_OFF_K64(NB) + 64 - G + gl];
	const T poly = (T)p.poly, init = (T)p.init, xorout = (T)p.xorout;
	__syncthreads();

	const uint64_t total = (uint64_t)p.n_ext * p.nchunks;
	const uint64_t waves = (uint64_t)gridDim.x * CS_WAVES;
	// every lane runs the same number of outer iterations (shuffles below
	// need the whole wave): the wave's first chunk decides, idle groups mask
	for (uint64_t g0 = ((uint64_t)blockIdx.x * CS_WAVES + (threadIdx.x >> 6)) * GPW; g0 < total;
	     g0 += waves * GPW) {
		const uint64_t g = g0 + lane / G;
		const bool live = g < total;
		uint64_t off = 0, len = 0;
		const uint8_t *base = p.src;

		if (live)
			chunk_geom_fast(p, g, off, len, base);
		const int64_t nq = (int64_t)(len / 16);
		const int64_t m = lane_steps<TK>(nq, G);
		const int64_t z = m * G - nq;
		T acc = 0;

		for (int64_t i = 0; i < m; i += L::UN) {
			uint32_t d[L::UN][4];

			load_step<L::UN, W, true, true>(base, i, G, gl - z, m, init, d);
			acc = horner<W, REFL, TK, L::UN>(acc, d, i, m, s5, sl, sh);
		}
		acc = lane_shift<W, REFL>(acc, klane, gt, r4, (uint32_t)(64 - G + gl), poly);
#pragma unroll
		for (int s = G / 2; s >= 1; s >>= 1)
			acc ^= shfl_xor_t(acc, s);
		if (live && gl == 0) {
			T crc = nq == 0 ? init : acc;

			for (uint64_t b = (uint64_t)nq * 16; b < len; b++)
				crc = byte_step<W, REFL>(crc, base[b], gt);
			crc ^= xorout;
			if constexpr (W == 16)
				((uint16_t *)p.out)[g] = (uint16_t)crc;
			else
				((T *)p.out)[g] = crc;
		}
	}
}


// Long chunks, few of them (e.g. 1024 chunks of 1 MiB = one wave per SIMD
// with ecg_crc_kernel): one workgroup of NW waves per chunk.  The chunk's
// 1 KiB steps are cut into NW contiguous slices; each wave computes the raw
// CRC of its slice exactly as ecg_crc_kernel does a whole chunk, moves it to
// the end of the chunk's aligned part by multiplying with x^(8 * bytes after
// the slice) mod P -- that power is the product of the p2[j] = x^(8*2^j)
// table entries of its set bits, one bit per lane, multiplied down the wave
// in 6 butterfly steps -- and the waves' values are XORed through LDS (CRC
// is linear: crc(A || B) = crc(A) * x^(8|B|) ^ crc(B) for zero registers).
template <int W, bool REFL, int NW, int TK>
__global__ __launch_bounds__(64 * NW) void ecg_crc_split_kernel(ecg_csum_params_t p)
{
	using T = typename reg<W>::T;
	using L = crc_lds<W, TK>;
	constexpr int NB = W / 8;
	__shared__ T s5[L::N5];
	__shared__ T sl[L::NSL];
	__shared__ T sh[L::NSL];
	__shared__ T part[NW];
	__shared__ T r4[REFL ? 16 : 1];
	const T *gt = (const T *)p.tbl;

	stage_tables<W, TK>(s5, sl, sh, gt, ECG_CSUM_OFF_P5X_1K(NB), ECG_CSUM_OFF_A5_4K(NB), ECG_CSUM_OFF_Q4_1K(NB),
			    ECG_CSUM_OFF_A4_4K(NB), 64 * NW);
	if (REFL && threadIdx.x < 16)
		r4[threadIdx.x] = gt[ECG_CSUM_OFF_R4(NB) + threadIdx.x];
	const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	const T klane = gt[2 * NB * 256 + lane];
	const T one = REFL ? (T)((T)1 << (W - 1)) : (T)1;
	const T p2 = lane < ECG_CSUM_NP2 ? gt[ECG_CSUM_OFF_P2(NB) + lane] : one;
	const T poly = (T)p.poly, init = (T)p.init, xorout = (T)p.xorout;
	__syncthreads();

	const uint64_t total = (uint64_t)p.n_ext * p.nchunks;
	for (uint64_t g = blockIdx.x; g < total; g += gridDim.x) {
		uint64_t off, len;
		const uint8_t *base;

		chunk_geom_fast(p, g, off, len, base);
		static_assert(NW == ECG_CSUM_SPLIT_NW, "host split shifts assume ECG_CSUM_SPLIT_NW slices");
		const int64_t nq = (int64_t)(len / 16);
		const int64_t m = (int64_t)ECG_CSUM_STEPS((uint64_t)len);	// as the host's split_m
		const int64_t z = m * 64 - nq;
		const int64_t ms = (int64_t)ECG_CSUM_SPLIT_MS((uint64_t)m);
		const int64_t i0 = wv * ms < m ? wv * ms : m;
		const int64_t i1 = i0 + ms < m ? i0 + ms : m;
		T acc = 0;

		for (int64_t i = i0; i < i1; i += L::UN) {
			uint32_t d[L::UN][4];

			load_step<L::UN, W, true, true>(base, i, 64, lane - z, i1, init, d);
			acc = horner<W, REFL, TK, L::UN>(acc, d, i, i1, s5, sl, sh);
		}
		acc = lane_shift<W, REFL>(acc, klane, gt, r4, (uint32_t)lane, poly);
		acc = wave_xor_uniform(acc);	// DPP, no ds_bpermute
		// x^(8 * (m - i1) KiB): the host's constant for this chunk length,
		// else the product of p2[j] over the set bits j (one bit per lane)
		T f;
		if (m == (int64_t)p.split_m[0] || m == (int64_t)p.split_m[1] || m == (int64_t)p.split_m[2]) {
			const int c = m == (int64_t)p.split_m[0] ? 0 : m == (int64_t)p.split_m[1] ? 1 : 2;
			f = (T)p.split_sh[c][wv];
		} else {
			const uint64_t after = (uint64_t)(m - i1) * ECG_CSUM_STRIDE;
			f = lane < ECG_CSUM_NP2 && ((after >> lane) & 1) ? p2 : one;
#pragma unroll
			for (int s = 32; s >= 1; s >>= 1)
				f = mulmod<W, REFL>(f, shfl_xor_t(f, s), poly);
		}
		acc = mulmod<W, REFL>(f, acc, poly);
		if (lane == 0)
			part[wv] = acc;
		__syncthreads();
		if (threadIdx.x == 0) {
			T crc = 0;

#pragma unroll
			for (int w = 0; w < NW; w++)
				crc ^= part[w];
			if (nq == 0)
				crc = init;
			for (uint64_t b = (uint64_t)nq * 16; b < len; b++)
				crc = byte_step<W, REFL>(crc, base[b], gt);
			crc ^= xorout;
			if constexpr (W == 16)
				((uint16_t *)p.out)[g] = (uint16_t)crc;
			else
				((T *)p.out)[g] = crc;
		}
		__syncthreads();
	}
}

// adler32 with A = B = 0 at each chunk start (isal_adler32(0, ...)): lanes sum
// bytes and position-weighted bytes of their pieces (v_dot4_u32_u8), the wave
// reduces, A = sum mod 65521, B = L*sum - sum(pos*byte) mod 65521.
template <bool ALIGNED>
__global__ __launch_bounds__(CS_BLOCK) void ecg_adler_kernel(ecg_csum_params_t p)
{
	const int lane = threadIdx.x & 63;
	const uint64_t total = (uint64_t)p.n_ext * p.nchunks;

	for (uint64_t g = (uint64_t)blockIdx.x * CS_WAVES + (threadIdx.x >> 6); g < total;
	     g += (uint64_t)gridDim.x * CS_WAVES) {
		uint64_t off, len;
		const uint8_t *base;

		chunk_geom(p, g, off, len, base);
		const uint64_t nq = len / 16;
		uint64_t s = 0, w = 0;

		for (uint64_t q = lane, it = 0; q < nq; q += 64, it++) {
			uint32_t d[4];
			uint32_t s16 = 0, w16 = 0;

			load16<ALIGNED>(base + 16 * q, d);
#pragma unroll
			for (int j = 0; j < 4; j++) {
				s16 = __builtin_amdgcn_udot4(d[j], 0x01010101u, s16, false);
				// weights 4j .. 4j+3 packed as bytes
				w16 = __builtin_amdgcn_udot4(d[j], 0x03020100u + 0x04040404u * j, w16, false);
			}
			s += s16;
			w += 16 * q * (uint64_t)s16 + w16;
			if ((it & 255) == 255) {
				s %= ADLER_MOD;
				w %= ADLER_MOD;
			}
		}
		s %= ADLER_MOD;
		w %= ADLER_MOD;
		// wave sum (values < 2^17 each: 64 of them fit easily)
#pragma unroll
		for (int sft = 32; sft >= 1; sft >>= 1) {
			s += __shfl_xor(s, sft);
			w += __shfl_xor(w, sft);
		}
		if (lane == 0) {
			for (uint64_t b = nq * 16; b < len; b++) {
				s += base[b];
				w += b * (uint64_t)base[b];
			}
			const uint64_t A = s % ADLER_MOD;
			const uint64_t Bp = ((len % ADLER_MOD) * A) % ADLER_MOD;
			const uint64_t B = (Bp + ADLER_MOD - w % ADLER_MOD) % ADLER_MOD;
			((uint32_t *)p.out)[g] = (uint32_t)((B << 16) | A);
		}
	}
}

// adler32 of long chunks that are few (one wave per chunk would leave the
// CUs idle, e.g. 1024 chunks of 1 MiB): a workgroup of NW waves per chunk.
// The sums use absolute positions within the chunk, so the threads' partial
// sums simply add: thread t takes the 16-byte pieces t, t + 64*NW, ... (every
// load instruction of a wave still reads 1 KiB contiguous), the waves reduce
// with shuffles and combine through LDS.
template <int NW>
__global__ __launch_bounds__(64 * NW) void ecg_adler_split_kernel(ecg_csum_params_t p)
{
	__shared__ uint64_t ps[NW], pw[NW];
	const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	const uint64_t total = (uint64_t)p.n_ext * p.nchunks;

	for (uint64_t g = blockIdx.x; g < total; g += gridDim.x) {
		uint64_t off, len;
		const uint8_t *base;

		chunk_geom(p, g, off, len, base);
		const uint64_t nq = len / 16;
		uint64_t s = 0, w = 0;

		for (uint64_t q = threadIdx.x, it = 0; q < nq; q += 64 * NW, it++) {
			uint32_t d[4];
			uint32_t s16 = 0, w16 = 0;

			load16<true>(base + 16 * q, d);
#pragma unroll
			for (int j = 0; j < 4; j++) {
				s16 = __builtin_amdgcn_udot4(d[j], 0x01010101u, s16, false);
				w16 = __builtin_amdgcn_udot4(d[j], 0x03020100u + 0x04040404u * j, w16, false);
			}
			s += s16;
			w += 16 * q * (uint64_t)s16 + w16;
			if ((it & 255) == 255) {
				s %= ADLER_MOD;
				w %= ADLER_MOD;
			}
		}
		s %= ADLER_MOD;
		w %= ADLER_MOD;
#pragma unroll
		for (int sft = 32; sft >= 1; sft >>= 1) {
			s += __shfl_xor(s, sft);
			w += __shfl_xor(w, sft);
		}
		if (lane == 0) {
			ps[wv] = s;
			pw[wv] = w;
		}
		__syncthreads();
		if (threadIdx.x == 0) {
			s = 0;
			w = 0;
#pragma unroll
			for (int i = 0; i < NW; i++) {
				s += ps[i];
				w += pw[i];
			}
			for (uint64_t b = nq * 16; b < len; b++) {
				s += base[b];
				w += b * (uint64_t)base[b];
			}
			const uint64_t A = s % ADLER_MOD;
			const uint64_t Bp = ((len % ADLER_MOD) * A) % ADLER_MOD;
			const uint64_t B = (Bp + ADLER_MOD - w % ADLER_MOD) % ADLER_MOD;
			((uint32_t *)p.out)[g] = (uint32_t)((B << 16) | A);
		}
		__syncthreads();
	}
}

typedef void (*csum_fn_t)(ecg_csum_params_t);
struct csum_entry {
	uint32_t type;
	bool aligned;
	int tk;			/* CRC table kind (TK_*); adler32: 0 */
	csum_fn_t fn;
	const char *name;
};

const csum_entry g_csum[] = {
	{1, true, TK_4, ecg_crc_kernel<16, false, true, TK_4>, "ecg_crc_kernel<crc16>"},
	{1, false, TK_5, ecg_crc_kernel<16, false, false, TK_5>, "ecg_crc_kernel<crc16,bytes>"},
	{2, true, TK_4, ecg_crc_kernel<32, true, true, TK_4>, "ecg_crc_kernel<crc32>"},
	{2, false, TK_5, ecg_crc_kernel<32, true, false, TK_5>, "ecg_crc_kernel<crc32,bytes>"},
	{3, true, TK_4, ecg_crc_kernel<64, true, true, TK_4>, "ecg_crc_kernel<crc64>"},
	{3, false, TK_5, ecg_crc_kernel<64, true, false, TK_5>, "ecg_crc_kernel<crc64,bytes>"},
	{7, true, 0, ecg_adler_kernel<true>, "ecg_adler_kernel"},
	{7, false, 0, ecg_adler_kernel<false>, "ecg_adler_kernel<bytes>"},
};
constexpr uint32_t N_CSUM = sizeof(g_csum) / sizeof(g_csum[0]);

constexpr int SPLIT_NW = ECG_CSUM_SPLIT_NW;	// waves per chunk in the split kernel
const csum_entry g_split[] = {
	{1, true, TK_4, ecg_crc_split_kernel<16, false, SPLIT_NW, TK_4>, "ecg_crc_split_kernel<crc16>"},
	{2, true, TK_4, ecg_crc_split_kernel<32, true, SPLIT_NW, TK_4>, "ecg_crc_split_kernel<crc32>"},
	{3, true, TK_4, ecg_crc_split_kernel<64, true, SPLIT_NW, TK_4>, "ecg_crc_split_kernel<crc64>"},
	{7, true, 0, ecg_adler_split_kernel<SPLIT_NW>, "ecg_adler_split_kernel"},
};
constexpr uint32_t N_SPLIT = sizeof(g_split) / sizeof(g_split[0]);

const csum_entry g_group[] = {
	{1, true, TK_4, ecg_crc_group_kernel<16, false, TK_4>, "ecg_crc_group_kernel<crc16>"},
	{2, true, TK_4, ecg_crc_group_kernel<32, true, TK_4>, "ecg_crc_group_kernel<crc32>"},
	{3, true, TK_4, ecg_crc_group_kernel<64, true, TK_4>, "ecg_crc_group_kernel<crc64>"},
};
constexpr uint32_t N_GROUP = sizeof(g_group) / sizeof(g_group[0]);

/* one table kind per kernel: the nibble tables for 16-byte aligned extents,
 * the 5-bit tables for the byte-granular kernels (the byte and 5-bit aligned
 * variants of rounds 1-3 were A/B builds, profiles/r03/crc_sq/) */
__host__ inline bool kind_ok(const csum_entry &e, const ecg_csum_params_t *p)
{
	(void)p;
	return e.type == 7 || e.tk == (e.aligned ? TK_4 : TK_5);
}

} // namespace

extern "C" const char *ecg_k_csum_kernel_name(uint32_t id)
{
	if (id >= ECG_KID_CSUM && id < ECG_KID_CSUM + N_CSUM)
		return g_csum[id - ECG_KID_CSUM].name;
	if (id >= ECG_KID_CSUM + N_CSUM && id < ECG_KID_CSUM + N_CSUM + N_SPLIT)
		return g_split[id - ECG_KID_CSUM - N_CSUM].name;
	if (id >= ECG_KID_CSUM + N_CSUM + N_SPLIT && id < ECG_KID_CSUM + N_CSUM + N_SPLIT + N_GROUP)
		return g_group[id - ECG_KID_CSUM - N_CSUM - N_SPLIT].name;
	return "?";
}

extern "C" int ecg_k_launch_csum(const ecg_csum_params_t *p, void *stream, uint32_t max_blocks,
				 uint32_t *kernel_id)
{
	const uint64_t total = (uint64_t)p->n_ext * p->nchunks;
	const bool aligned = (((uint64_t)(uintptr_t)p->src | (uint64_t)p->ext_stride | p->first_bytes |
			       p->chunk_bytes) & 15u) == 0;
	uint64_t blocks = (total + CS_WAVES - 1) / CS_WAVES;

	if (total == 0)
		return (int)hipSuccess;
	if (aligned) {
		// a workgroup per chunk when one wave per chunk would leave fewer
		// than 4 waves per SIMD and every wave still gets >= 2 steps
		// (adler32 too: profiles/r01/bench_csum.json adler32_cs1024K rows)
		const uint64_t steps = (p->chunk_bytes / 16 + 63) / 64;
		const bool split = p->variant == 2 ||
				   (p->variant == 0 && total < 4096 && steps >= 2 * SPLIT_NW);

		for (uint32_t i = 0; split && i < N_SPLIT; i++) {
			if (g_split[i].type != p->type || !kind_ok(g_split[i], p))
				continue;
			uint64_t nb = total;
			const uint64_t cap = max_blocks ? max_blocks : 256 * 8;

			if (nb > cap)
				nb = cap;
			hipLaunchKernelGGL(g_split[i].fn, dim3((uint32_t)nb), dim3(64 * SPLIT_NW), 0,
					   (hipStream_t)stream, *p);
			if (kernel_id)
				*kernel_id = ECG_KID_CSUM + N_CSUM + i;
			return (int)hipGetLastError();
		}
	}
	if (max_blocks == 0)
		max_blocks = 256 * 16;	// 16 blocks per CU, grid-stride beyond
	if (p->type != 7 && aligned && p->variant == 3) {
		const uint32_t per_block = CS_WAVES * (64 / ECG_CSUM_GLANES);
		uint64_t nb = (total + per_block - 1) / per_block;

		if (nb > max_blocks)
			nb = max_blocks;
		for (uint32_t i = 0; i < N_GROUP; i++) {
			if (g_group[i].type != p->type || !kind_ok(g_group[i], p))
				continue;
			hipLaunchKernelGGL(g_group[i].fn, dim3((uint32_t)nb), dim3(CS_BLOCK), 0,
					   (hipStream_t)stream, *p);
			if (kernel_id)
				*kernel_id = ECG_KID_CSUM + N_CSUM + N_SPLIT + i;
			return (int)hipGetLastError();
		}
	}
	if (blocks > max_blocks)
		blocks = max_blocks;
	for (uint32_t i = 0; i < N_CSUM; i++) {
		if (g_csum[i].type == p->type && g_csum[i].aligned == aligned && kind_ok(g_csum[i], p)) {
			hipLaunchKernelGGL(g_csum[i].fn, dim3((uint32_t)blocks), dim3(CS_BLOCK), 0,
					   (hipStream_t)stream, *p);
			if (kernel_id)
				*kernel_id = ECG_KID_CSUM + i;
			return (int)hipGetLastError();
		}
	}
	return (int)hipErrorInvalidValue;
}
