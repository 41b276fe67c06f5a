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
constexpr int CS_UNROLL = 4;		// pieces in flight per lane
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

template <int W, bool REFL, bool ALIGNED>
__global__ __launch_bounds__(CS_BLOCK) void ecg_crc_kernel(ecg_csum_params_t p)
{
	using T = typename reg<W>::T;
	constexpr int NB = W / 8;
	__shared__ T sl[NB * 256];
	__shared__ T sh[NB * 256];
	const T *gt = (const T *)p.tbl;

	for (int i = threadIdx.x; i < NB * 256; i += CS_BLOCK) {
		sl[i] = gt[i];
		sh[i] = gt[NB * 256 + i];
	}
	const int lane = threadIdx.x & 63;
	const T klane = gt[2 * NB * 256 + lane];
	const T poly = (T)p.poly, init = (T)p.init, xorout = (T)p.xorout;
	__syncthreads();

	const uint64_t total = (uint64_t)p.n_ext * p.nchunks;
	for (uint64_t g = (uint64_t)blockIdx.x * CS_WAVES + (threadIdx.x >> 6); g < total;
	     g += (uint64_t)gridDim.x * CS_WAVES) {
		uint64_t off, len;
		const uint8_t *base;

		chunk_geom(p, g, off, len, base);
		const int64_t nq = (int64_t)(len / 16);
		const int64_t m = (nq + 63) / 64;
		const int64_t z = m * 64 - nq;
		T acc = 0;

		for (int64_t i = 0; i < m; i += CS_UNROLL) {
			uint32_t d[CS_UNROLL][4];
#pragma unroll
			for (int u = 0; u < CS_UNROLL; u++) {
				const int64_t q = (i + u) * 64 + lane - z;
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
			}
#pragma unroll
			for (int u = 0; u < CS_UNROLL; u++) {
				if (i + u < m)
					acc = lin_map<W>(acc, sh) ^ piece_crc<W, REFL>(d[u], sl);
			}
		}
		acc = mulmod<W, REFL>(klane, acc, poly);
		acc = wave_xor(acc);
		if (lane == 0) {
			T crc = nq == 0 ? init : acc;

			for (uint64_t b = (uint64_t)nq * 16; b < len; b++)
				crc = byte_step<W, REFL>(crc, base[b], sl);
			crc ^= xorout;
			if constexpr (W == 16)
				((uint16_t *)p.out)[g] = (uint16_t)crc;
			else
				((T *)p.out)[g] = crc;
		}
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

typedef void (*csum_fn_t)(ecg_csum_params_t);
struct csum_entry {
	uint32_t type;
	bool aligned;
	csum_fn_t fn;
	const char *name;
};

const csum_entry g_csum[] = {
	{1, true, ecg_crc_kernel<16, false, true>, "ecg_crc_kernel<crc16>"},
	{1, false, ecg_crc_kernel<16, false, false>, "ecg_crc_kernel<crc16,bytes>"},
	{2, true, ecg_crc_kernel<32, true, true>, "ecg_crc_kernel<crc32>"},
	{2, false, ecg_crc_kernel<32, true, false>, "ecg_crc_kernel<crc32,bytes>"},
	{3, true, ecg_crc_kernel<64, true, true>, "ecg_crc_kernel<crc64>"},
	{3, false, ecg_crc_kernel<64, true, false>, "ecg_crc_kernel<crc64,bytes>"},
	{7, true, ecg_adler_kernel<true>, "ecg_adler_kernel"},
	{7, false, ecg_adler_kernel<false>, "ecg_adler_kernel<bytes>"},
};
constexpr uint32_t N_CSUM = sizeof(g_csum) / sizeof(g_csum[0]);

} // namespace

extern "C" const char *ecg_k_csum_kernel_name(uint32_t id)
{
	return id >= ECG_KID_CSUM && id < ECG_KID_CSUM + N_CSUM ? g_csum[id - ECG_KID_CSUM].name : "?";
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
	if (max_blocks == 0)
		max_blocks = 256 * 16;	// 16 blocks per CU, grid-stride beyond
	if (blocks > max_blocks)
		blocks = max_blocks;
	for (uint32_t i = 0; i < N_CSUM; i++) {
		if (g_csum[i].type == p->type && g_csum[i].aligned == aligned) {
			hipLaunchKernelGGL(g_csum[i].fn, dim3((uint32_t)blocks), dim3(CS_BLOCK), 0,
					   (hipStream_t)stream, *p);
			if (kernel_id)
				*kernel_id = ECG_KID_CSUM + i;
			return (int)hipGetLastError();
		}
	}
	return (int)hipErrorInvalidValue;
}
