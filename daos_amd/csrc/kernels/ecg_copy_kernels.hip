// ecg_copy_kernels.hip -- batched byte-range copies between device buffers
// (gfx950): the stripe gather of the client encode (cells spanning iovs,
// ref:src/object/cli_ec.c:510-536) and the fill-back of recovered records
// into the user's scatter-gather list (obj_ec_recov_fill_back,
// ref:src/object/cli_ec.c:2710-2812).  Both are lists of (dst, src, len)
// segments with arbitrary byte alignment: one launch copies all of them.
//
// Work unit: a 16 KiB tile of one segment's destination (256 lanes x 4 x
// 16 B).  Segment s owns tiles [tile0[s], tile0[s+1]); each wave finds its
// segment by a 64-ary search over the tile0 column.  Inside a segment the
// destination is split into
//   head  -- bytes up to the first 16-byte aligned destination address,
//   body  -- 16-byte aligned destination words,
//   tail  -- the < 16 bytes after the last whole word.
// Body words are written with global_store_dwordx4.  The source of a word
// starts at an arbitrary byte: each lane loads the two aligned 16-byte words
// covering it and funnel-shifts them (v_alignbyte_b32).  An aligned 16-byte
// load that contains at least one byte of the segment stays inside a page the
// segment touches, so the over-read cannot fault.  The source misalignment is
// uniform per segment, so its 4 dword cases are a wave-uniform branch; an
// aligned source takes one load per word.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../ecg_kabi.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CP_BLOCK 256
#define CP_WORDS 4			/* 16-byte words per lane per tile */

__device__ __forceinline__ u32x4 ld16(const uint8_t *p)
{
	return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
}

__device__ __forceinline__ void st16(uint8_t *p, u32x4 v)
{
	__builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
}

// bytes [r, r + 4) of the 8-byte little-endian value hi:lo
__device__ __forceinline__ uint32_t fsh(uint32_t hi, uint32_t lo, uint32_t r)
{
	return __builtin_amdgcn_alignbyte(hi, lo, r);
}

// the 16 bytes starting 4*q + r bytes into the aligned pair a:b
__device__ __forceinline__ u32x4 shift_pair(u32x4 a, u32x4 b, uint32_t q, uint32_t r)
{
	const uint32_t d[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};

	// q is wave-uniform: a scalar branch, registers indexed statically
	switch (q) {
	case 0:
		return (u32x4){fsh(d[1], d[0], r), fsh(d[2], d[1], r), fsh(d[3], d[2], r), fsh(d[4], d[3], r)};
	case 1:
		return (u32x4){fsh(d[2], d[1], r), fsh(d[3], d[2], r), fsh(d[4], d[3], r), fsh(d[5], d[4], r)};
	case 2:
		return (u32x4){fsh(d[3], d[2], r), fsh(d[4], d[3], r), fsh(d[5], d[4], r), fsh(d[6], d[5], r)};
	default:
		return (u32x4){fsh(d[4], d[3], r), fsh(d[5], d[4], r), fsh(d[6], d[5], r), fsh(d[7], d[6], r)};
	}
}

__global__ void __launch_bounds__(CP_BLOCK)
ecg_copy_segs_kernel(const ecg_copy_seg_t *__restrict__ segs, uint32_t nseg)
{
	// This tile's segment: the last s with segs[s].tile0 <= blockIdx.x.  A
	// 64-ary search per wave: each round the lanes probe 64 evenly spaced
	// entries of the bracket and a ballot picks the sub-bracket, so a list
	// of up to 4096 segments costs two dependent loads instead of a binary
	// search's dozen.
	const uint32_t lane = threadIdx.x & 63u;
	uint32_t lo = 0, n = nseg;
	while (n > 1) {
		const uint32_t step = (n + 63u) / 64u;
		const bool in = lane * step < n;
		const bool le = in && segs[lo + lane * step].tile0 <= blockIdx.x;
		const uint32_t c = (uint32_t)__popcll(__ballot(le));	// >= 1: segs[lo] qualifies

		lo += (c - 1u) * step;
		n = n - (c - 1u) * step < step ? n - (c - 1u) * step : step;
	}
	const ecg_copy_seg_t sg = segs[lo];
	const uint64_t t = blockIdx.x - sg.tile0;
	uint8_t *dst = reinterpret_cast<uint8_t *>(sg.dst);
	const uint8_t *src = reinterpret_cast<const uint8_t *>(sg.src);
	const uint64_t len = sg.len;
	uint64_t head = (16u - (sg.dst & 15u)) & 15u;

	if (head > len)
		head = len;
	const uint64_t nw = (len - head) / 16;		// body words
	const uint64_t tail0 = head + nw * 16;

	if (t == 0) {			// head: lanes 0..14, tail: lanes 64..78
		if (threadIdx.x < head)
			dst[threadIdx.x] = src[threadIdx.x];
		else if (threadIdx.x >= 64 && threadIdx.x - 64 < len - tail0)
			dst[tail0 + threadIdx.x - 64] = src[tail0 + threadIdx.x - 64];
	}

	uint8_t *bd = dst + head;
	const uint8_t *bs = src + head;
	const uint32_t sh = (uint32_t)((uintptr_t)bs & 15u);
	const uint64_t w0 = t * (CP_BLOCK * CP_WORDS) + threadIdx.x;

	if (sh == 0) {
		u32x4 v[CP_WORDS];
#pragma unroll
		for (int q = 0; q < CP_WORDS; q++) {
			const uint64_t w = w0 + (uint64_t)q * CP_BLOCK;
			if (w < nw)
				v[q] = ld16(bs + w * 16);
		}
#pragma unroll
		for (int q = 0; q < CP_WORDS; q++) {
			const uint64_t w = w0 + (uint64_t)q * CP_BLOCK;
			if (w < nw)
				st16(bd + w * 16, v[q]);
		}
	} else {
		// Word w needs source bytes bsa + 16w + sh .. + 15: the aligned
		// words at bsa + 16w and bsa + 16w + 16, both holding segment bytes.
		// (Taking the second word from the next lane with a shuffle instead
		// of a second load measured the same: the extra 16 B per lane hits
		// L1, the cost of a misaligned source is the extra line per wave.)
		const uint8_t *bsa = bs - sh;
		const uint32_t dq = sh >> 2, r = sh & 3u;
		u32x4 a[CP_WORDS], b[CP_WORDS];
#pragma unroll
		for (int q = 0; q < CP_WORDS; q++) {
			const uint64_t w = w0 + (uint64_t)q * CP_BLOCK;
			if (w < nw) {
				a[q] = ld16(bsa + w * 16);
				b[q] = ld16(bsa + w * 16 + 16);
			}
		}
#pragma unroll
		for (int q = 0; q < CP_WORDS; q++) {
			const uint64_t w = w0 + (uint64_t)q * CP_BLOCK;
			if (w < nw)
				st16(bd + w * 16, shift_pair(a[q], b[q], dq, r));
		}
	}
}

// Table fetch: one 64-bit word per lane, read from pinned host memory at
// system scope (the CPU wrote it just before the launch; nothing stale may
// come from a cache) and stored to device memory for the launches behind it.
#define FETCH_BLOCK 256

__global__ void __launch_bounds__(FETCH_BLOCK) ecg_fetch_kernel(const uint64_t *__restrict__ src,
								  uint64_t *__restrict__ dst, uint32_t n)
{
	const uint32_t i = blockIdx.x * FETCH_BLOCK + threadIdx.x;

	if (i < n)
		dst[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

extern "C" int ecg_k_launch_fetch(const uint64_t *host_src, uint64_t *dst, uint32_t nwords, void *stream)
{
	if (nwords == 0)
		return (int)hipSuccess;
	if (host_src == nullptr || dst == nullptr)
		return (int)hipErrorInvalidValue;
	hipLaunchKernelGGL(ecg_fetch_kernel, dim3((nwords + FETCH_BLOCK - 1) / FETCH_BLOCK), dim3(FETCH_BLOCK), 0,
			   (hipStream_t)stream, host_src, dst, nwords);
	return (int)hipGetLastError();
}

extern "C" uint64_t ecg_k_copy_tiles(uint64_t dst, uint64_t len)
{
	uint64_t head = (16u - (dst & 15u)) & 15u;

	if (head > len)
		head = len;
	const uint64_t nw = (len - head) / 16;
	const uint64_t tiles = (nw + CP_BLOCK * CP_WORDS - 1) / (CP_BLOCK * CP_WORDS);
	return tiles ? tiles : (len ? 1 : 0);
}

extern "C" int ecg_k_launch_copy_segs(const ecg_copy_seg_t *segs_dev, uint32_t nseg, uint64_t ntiles,
				      void *stream, uint32_t *kernel_id)
{
	if (nseg == 0 || ntiles == 0)
		return (int)hipSuccess;
	if (ntiles > 0x7fffffffull)
		return (int)hipErrorInvalidValue;
	hipLaunchKernelGGL(ecg_copy_segs_kernel, dim3((uint32_t)ntiles), dim3(CP_BLOCK), 0, (hipStream_t)stream,
			   segs_dev, nseg);
	if (kernel_id)
		*kernel_id = ECG_KID_COPY_SEGS;
	return (int)hipGetLastError();
}
