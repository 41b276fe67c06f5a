// ecg_fused_kernels.hip -- the fused GF(2^8) product + chunk checksum kernel
// (include/ecg_csum.h ecg_encode_csum / ecg_recover_csum):
// the regenerated cells are checksummed from registers while they are
// written, instead of a second HBM pass over them (the reference checksums
// rebuilt cells after encoding, ref:src/object/srv_obj_migrate.c:1156).
// The product itself is ecg_mm_dev.h's, exactly as ecg_mm_kernel computes it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../ecg_kabi.h"
#include "ecg_crc_dev.h"
#include "ecg_mm_dev.h"

#ifndef ECG_FUSED_PF64
#define ECG_FUSED_PF64 1	// prefetch in the crc64 fused kernels too
#endif
#ifndef ECG_FUSED_PF_MAXK
#define ECG_FUSED_PF_MAXK 8	// fused kernels: next column's loads in flight for k <= this
#endif
// fused kernels: the waves per SIMD their register budget targets.  crc16 /
// crc32 get the 3-wave budget (<= 168 VGPRs): at a 4-wave budget the register
// allocator spilled EC_8P2's pipelined loop to scratch, at 3 it settles at
// 104 VGPRs -- 4 waves anyway, no spills.  crc64 fits 4 waves without spills.
#ifndef ECG_FUSED_WPE
#define ECG_FUSED_WPE(W) ((W) == 64 ? 4 : 3)
#endif
// fused workgroup kernel: fold each column's outputs into the CRC one column
// later, while the next column's product is computed (independent work the
// scheduler can interleave with the lookup chains).  Bit 0: crc16/crc32,
// bit 1: crc64.  Measured (tools/fused_libs.py, 3 interleaved rounds,
// profiles/r03/defer/): EC_8P2 x 512 crc64 0.906 -> 0.886 ms (encode 0.838),
// crc32 and EC_4P2 unchanged within +-0.5 %.  Timed as back-to-back blocks
// (round 4, tools/ec_ab.py EC_OPS=crc32,crc64, 3 rotated rounds,
// profiles/r04/ec_ab/ec_ab_fused_defer.json, ms): EC_8P2 crc32 0.903 deferred
// vs 0.891 immediate, crc64 0.920 vs 0.912, EC_4P2 x 1024 crc64 1.077 vs
// 1.110 -- so crc32 folds immediately, crc64 one column late.
#ifndef ECG_FUSED_DEFER
#define ECG_FUSED_DEFER 2
#endif

// Work item `it` of the fused kernel -> chunk c, sub-chunk h, its columns
// [col0, col1) and the row of Q.kh its threads multiply by (ecg_kabi.h).
__device__ __forceinline__ void mmcs_item(const ecg_mmcs_params_t &Q, uint32_t it, uint32_t &c, uint32_t &col0,
					  uint32_t &col1, uint32_t &khrow)
{
	c = it / Q.nh;
	const uint32_t h = it - c * Q.nh;
	const bool lastc = c + 1 == Q.nch;
	const uint32_t m = lastc ? Q.m_last : Q.m;

	col0 = h * Q.ncols;
	col1 = col0 + Q.ncols < m ? col0 + Q.ncols : m;
	khrow = (lastc ? Q.nh : 0) + h;
}

// One column of a fused product + checksum item (the workgroup kernel's 4 KiB
// columns, the wave kernel's 1 KiB rows; STRIDE bytes): with PF, first the
// next column's loads into nxt (when `more`), then the product of cur -- the
// sources already in registers -- and its stores, then each output row's
// 16-byte piece folded into the row's CRC.  TB 0: pos = columns to the item
// end mod U selects the positional table; the register is shifted by U
// columns at each group start (pos == U - 1).  `first`: this piece starts
// the chunk, the initial register is folded into it.  `next`: the column the
// prefetch reads (the walk need not be in address order); gshift = false for
// a walk whose positions all fit the U tables (no register shift at all).
// The kernel arguments re-read (scalar loads, K$ hits) where they are used:
// an empty asm on their constant-space address stops the compiler from
// keeping every cell offset of the launch live in SGPRs across a column loop
// (the fused kernels spilled SGPRs into VGPR lanes).
typedef __attribute__((address_space(4))) const ecg_mm_params_t kparams_t;

__device__ __forceinline__ const ecg_mm_params_t &kernarg_fresh()
{
	// the kernel's first argument sits at the start of the kernarg segment
	kparams_t *p = (kparams_t *)__builtin_amdgcn_kernarg_segment_ptr();

	asm volatile("" : "+s"(p));
	return *(const ecg_mm_params_t *)p;
}

// A column's outputs waiting to be folded (ECG_FUSED_DEFER): the fold of
// column i runs after column i+1's product.  The zero state (have = false,
// gshift = false) folds to nothing on a zero register.
template <int RM>
struct mmcs_pend {
	u32x4 v[RM];
	bool have, first, gshift;
	uint32_t pos;
};

// Fold one column's output pieces into the rows' CRC registers: the register
// shift of the table kind, then the piece's lookups (see mmcs_col).  TB 0:
// 5-bit positional tables, the register shifted by U columns at each group
// start; TB 1: byte tables (slice-by-NB) after an a5 shift by one column.
template <int RM, int W, bool REFL, int TB, int U, typename T>
__device__ __forceinline__ void mmcs_fold(const T *s_sl, const T *s_sh, int rows, const u32x4 *outv, bool have,
					  bool first, uint64_t init, uint32_t pos, bool gshift, T *crc)
{
	using F5 = ecg_crc::f5u<W, U>;
	static_assert(TB == 0 || TB == 1, "table kind");
#pragma unroll
	for (int r = 0; r < RM; r++) {
		if (r < rows) {
			if constexpr (TB == 1)
				crc[r] = ecg_crc::lin_map5<W>(crc[r], s_sh);	// a5 of one column
			else if (gshift && pos == F5::U - 1)
				crc[r] = ecg_crc::lin_map5<W>(crc[r], s_sl + F5::U * F5::NF * 32);
			if (have) {
				uint32_t d[4] = {outv[r][0], outv[r][1], outv[r][2], outv[r][3]};
				if (first) {	// initial register
					d[0] ^= (uint32_t)init;
					if constexpr (W == 64)
						d[1] ^= (uint32_t)(init >> 32);
				}
				if constexpr (TB == 1)
					crc[r] ^= ecg_crc::piece_crc<W, REFL>(d, s_sl);
				else
					crc[r] ^= ecg_crc::piece_crc5p<W>(d, s_sl, pos * (uint32_t)(F5::NF * 32 * sizeof(T)));
			}
		}
	}
}

// DF: 0 fold this column now; 1 fold the pending column and leave this one
// pending; 2 leave this one pending (nothing pending yet).
template <int KM, int RM, int W, bool REFL, int TB, bool PF, uint32_t STRIDE, bool FULL, int U, int DF = 0,
	  typename T>
__device__ __forceinline__ void mmcs_col(const ecg_mm_params_t &P0, const u32x4 *s_tbl, const T *s_sl,
					 const T *s_sh, int k, int rows, uint32_t s, uint64_t cbase, uint64_t next,
					 uint32_t lo, bool more, bool first, uint64_t init, uint32_t pos, bool gshift,
					 u32x4 *cur, u32x4 *nxt, T *crc, mmcs_pend<RM> *pd = nullptr)
{
	const ecg_mm_params_t &P = kernarg_fresh();	// == P0 (first kernel argument)
	(void)P0;
	const uint64_t C = P.cell_bytes;
	const bool have = FULL || cbase + lo + 16 <= C;	// C % 16 == 0
	u32x4 outv[RM];
	uint32_t z = 0;

	if constexpr (PF) {
		// no branch around the prefetch: a load that may or may not be
		// issued makes the compiler's waitcnt merge wait for everything
		// (vmcnt(0)) before the product.  Past the item's last column the
		// wave re-reads stripe 0's first column (cache-resident, unused).
		mm_load_any<KM>(P, k, more ? s : 0, more ? next : 0, lo, nxt);
	} else {
		// unconditional (clamped) loads: a load skipped by some lanes would
		// keep cur live across columns and items (zero-filled and spilled)
		mm_load_any<KM>(P, k, s, cbase, lo, cur);
	}
	asm volatile("" : "+v"(z));
	const u32x4 *tb = s_tbl + z;
	// FULL (the column lies inside the cell): no branch, so the pipelined
	// loop of the callers has one path -- a partial-column path that may skip
	// the loads or use other registers for its stores makes the compiler wait
	// for everything (vmcnt(0)) at the loop head
	if constexpr (!FULL && DF != 0) {
#pragma unroll
		for (int r = 0; r < RM; r++)
			outv[r] = (u32x4){0, 0, 0, 0};
	}
	if (FULL || cbase + STRIDE <= C)
		mm_compute<KM, RM, false, true>(P, tb, k, rows, s, cbase, lo, cur, outv);
	else if (have)
		mm_compute<KM, RM, false, true>(P, tb, k, rows, s, cbase, lo, cur, outv);
	if constexpr (DF == 0) {
		mmcs_fold<RM, W, REFL, TB, U>(s_sl, s_sh, rows, outv, have, first, init, pos, gshift, crc);
	} else {
		if constexpr (DF == 1)
			mmcs_fold<RM, W, REFL, TB, U>(s_sl, s_sh, rows, pd->v, pd->have, pd->first, init, pd->pos,
						      pd->gshift, crc);
#pragma unroll
		for (int r = 0; r < RM; r++)
			pd->v[r] = outv[r];
		pd->have = have;
		pd->first = first;
		pd->pos = pos;
		pd->gshift = gshift;
	}
}

// Fused product + checksum of every output cell (ecg_kabi.h, ecg_mmcs_params).
// Block = a stream of (stripe, sub-chunk) items of a few 4 KiB columns each;
// it walks the columns, computing and storing the outputs exactly as
// ecg_mm_kernel does, and folds each thread's 16-byte output piece into a
// per-row Horner CRC (acc = shift_4KiB(acc) ^ crc(piece)).  At the end of an
// item every thread multiplies by its kh entry (moves its pieces to the end
// of the chunk, undoes a ragged last chunk's zero padding), the waves
// XOR-reduce and XOR their values into the zeroed checksum.  Cutting a
// chunk into several items keeps one workgroup from walking a whole 32 KiB+
// chunk serially (tools/tune8.py: ~4 columns per workgroup is best).
// The outputs are never re-read from HBM: the checksum costs LDS lookups on
// p/(k+p) of the traffic instead of a second pass over the regenerated
// cells (ref:src/object/srv_obj_migrate.c:1156 checksums them after encode).
template <int K, int R, int W, bool REFL, int TB>
__global__ void __launch_bounds__(BLOCK, ECG_FUSED_WPE(W))
ecg_mm_csum_kernel(const ecg_mm_params_t P, const ecg_mmcs_params_t Q)
{
	using T = typename ecg_crc::reg<W>::T;
	constexpr int UF = ECG_MMCS_P5U;
	using F5 = ecg_crc::f5u<W, UF>;
	constexpr int NB = W / 8;
	constexpr int KM = K ? K : ECG_KMAX_K;
	constexpr int RM = R ? R : ECG_KMAX_R;
	constexpr bool PF = K != 0 && K <= ECG_FUSED_PF_MAXK && (ECG_FUSED_PF64 || W != 64);	// prefetch: 4*KM more VGPRs
	constexpr bool DEFER = (ECG_FUSED_DEFER & (W == 64 ? 2 : 1)) != 0;	// fold one column late
	constexpr int T2V = (RM + 3) / 4;
	constexpr int PER_J = RM + T2V;
	__shared__ u32x4 s_tbl[KM * PER_J];
	// CRC tables (TB): 0 5-bit (conflict-free, ecg_kabi.h: positional p5 of
	// 0..U-1 columns + a5 shift by U columns, U = ECG_MMCS_P5U); 1 byte
	// tables sl (slice-by-NB, register folded) + the a5 4 KiB shift
	static_assert(TB == 0 || TB == 1, "table kind");
	constexpr int NSL = TB == 0 ? F5::N : NB * 256;
	__shared__ T s_sl[NSL];
	// TB 1: the column shift as 5-bit a5 tables
	__shared__ T s_sh[TB ? ECG_CSUM_NA5(NB) * 32 : 1];
	__shared__ T s_r4[REFL ? 16 : 1];		// reflected: 4-bit reduction of the lane multiply
	__shared__ T s_nibl[REFL ? 16 * 64 : 1];	// reflected: the lane factors' nibble tables
	const int k = K ? K : (int)P.k;
	const int rows = R ? R : (int)P.rows;
	const uint64_t C = P.cell_bytes;
	const uint32_t lo = threadIdx.x * 16u;
	const T *gt = (const T *)Q.tbl;
	const T *kh = (const T *)Q.kh;
	const T poly = (T)Q.poly;

	// Prologue.  The tables are staged in two phases around the first
	// column's HBM loads: every entry this thread stages is loaded into
	// registers (L2 hits), then the workgroup's first item's first column is
	// requested, then the entries are written to LDS -- vmcnt counts in issue
	// order, so the writes wait only for the table loads and the staging and
	// barrier run in the shadow of the first HBM round trip (a workgroup
	// normally owns exactly one item).
	constexpr int P5 = ECG_CSUM_NF5 * 32;
	constexpr int NSH = TB ? ECG_CSUM_NA5(NB) * 32 : 0;
	constexpr int NNB = REFL ? 16 * 64 + 16 : 0;		// nibl, then r4
	constexpr int NST = NSL + NSH + NNB;
	constexpr int QST = (NST + BLOCK - 1) / BLOCK;
	static_assert(KM * RM <= BLOCK, "one product-table entry per thread");
	auto st_src = [&](int i) -> int {		// entry i of the staged image -> index in gt
		if (i < NSL) {
			if constexpr (TB == 0)
				return i < P5 ? ECG_CSUM_OFF_P5(NB) + i
				     : i < UF * P5 ? ECG_CSUM_OFF_P5X_4K(NB) + i - P5 : ECG_CSUM_OFF_A5_32K(NB) + i - UF * P5;
			else
				return i;	// slice-by-NB byte tables at the image start
		}
		i -= NSL;
		if (i < NSH)
			return ECG_CSUM_OFF_A5_4K(NB) + i;
		i -= NSH;
		return i < 16 * 64 ? ECG_CSUM_OFF_NIBL(NB) + i : ECG_CSUM_OFF_R4(NB) + i - 16 * 64;
	};
	auto st_dst = [&](int i) -> T * {
		if (i < NSL)
			return &s_sl[i];
		i -= NSL;
		if (i < NSH)
			return &s_sh[i];
		i -= NSH;
		return i < 16 * 64 ? &s_nibl[i] : &s_r4[i - 16 * 64];
	};
	T sv[QST];
#pragma unroll
	for (int q = 0; q < QST; q++)
		if (q * BLOCK + (int)threadIdx.x < NST)
			sv[q] = gt[st_src(q * BLOCK + (int)threadIdx.x)];
	const int tj = (int)threadIdx.x / RM, tr = (int)threadIdx.x % RM;
	const bool tst = (int)threadIdx.x < KM * RM && tj < k && tr < rows;
	ecg_ptbl_t tv;
	if (tst)
		tv = P.tbl[tr][tj];

	// the first item's first column (unconditional, clamped: a load only
	// some paths issue makes the compiler wait for everything)
	u32x4 xa[KM];
	if constexpr (PF) {
		uint32_t c, i, col1, khrow;

		mmcs_item(Q, blockIdx.x, c, i, col1, khrow);
		const uint64_t c0 = (uint64_t)c * Q.chunk_bytes + (uint64_t)i * CHUNK_BYTES;
		mm_load_any<KM>(P, k, c0 < C ? blockIdx.y : 0u, c0 < C ? c0 : 0u, lo, xa);
	}
#pragma unroll
	for (int q = 0; q < QST; q++)
		if (q * BLOCK + (int)threadIdx.x < NST)
			*st_dst(q * BLOCK + (int)threadIdx.x) = sv[q];
	if (tst) {
		s_tbl[tj * PER_J + tr] = (u32x4){tv.t0lo, tv.t0hi, tv.t1lo, tv.t1hi};
		reinterpret_cast<uint32_t *>(&s_tbl[tj * PER_J + RM])[tr] = tv.t2;
	}
	__syncthreads();

	// One item: its 4 KiB columns in order.  With PF the next column's loads
	// are issued before this column's product, so HBM requests stay in
	// flight across it.  Live state is kept small on purpose: the crc64
	// instantiations ran out of SGPRs.
	// PRE: this is the workgroup's first item, its first column already
	// requested into xa by the prologue
	auto walk = [&](uint32_t s, uint32_t it, auto pre) {
			constexpr bool PRE = decltype(pre)::value;
			uint32_t c, i, col1, khrow;
			T crc[RM];

			mmcs_item(Q, it, c, i, col1, khrow);
			const uint64_t c0 = (uint64_t)c * Q.chunk_bytes;
			// reflected: this wave's item factor as W bit-products, lane b
			// holding e_b * f(item row, wave) (ecg_csum.c fused_kh); loaded
			// now, used after the walk -- its latency hides behind the walk
			T kbv = 0;
			if constexpr (REFL) {
				const uint32_t lane = threadIdx.x & 63u;
				const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

				if (lane < (uint32_t)W)
					kbv = kh[((size_t)khrow * 4u + wv) * 64u + lane];
			}
#pragma unroll
			for (int r = 0; r < RM; r++)
				crc[r] = 0;
			// Pipelined pairs of full columns, the prefetch buffers swapping
			// roles (a register copy xa = xb would wait for the prefetched loads
			// and serialise the walk); then the rest -- an odd full column, the
			// partial column of a cell that is not a multiple of 4 KiB -- one at
			// a time without prefetch, outside the pipelined loop so that loop
			// has a single path (a path that skips loads or stores makes the
			// compiler wait for everything at the loop head).  (Walking an
			// item's columns rotated, so concurrently running items stream
			// different address residues, measured no better:
			// profiles/r02/fused_libs/rotation.json.)
			const uint64_t nfull = (C - c0) / CHUNK_BYTES;
			const uint32_t ifull = nfull < col1 ? (uint32_t)nfull : col1;
			// DEFER: each column's fold runs one column late (mmcs_pend);
			// the zero state folds to nothing on the zero register
			mmcs_pend<RM> pd;
			constexpr int D1 = DEFER ? 1 : 0;	// steady state
			constexpr int D2 = DEFER ? 2 : 0;	// a walk's first column
#pragma unroll
			for (int r = 0; r < RM; r++)
				pd.v[r] = (u32x4){0, 0, 0, 0};
			pd.have = pd.first = pd.gshift = false;
			pd.pos = 0;
			const uint32_t iend = ifull > i ? i + ((ifull - i) & ~1u) : i;
			if (PF && i < iend) {
				u32x4 xb[PF ? KM : 1];
				u32x4 *xc = PF ? xb : xa;

				if constexpr (!PRE)
					mm_load_any<KM>(P, k, s, c0 + (uint64_t)i * CHUNK_BYTES, lo, xa);
				if constexpr (DEFER) {
					// the first trip peeled: nothing pending at its first column
					const uint64_t cb = c0 + (uint64_t)i * CHUNK_BYTES;
					mmcs_col<KM, RM, W, REFL, TB, true, CHUNK_BYTES, true, UF, D2>(
						P, s_tbl, s_sl, s_sh, k, rows, s, cb, cb + CHUNK_BYTES, lo, true,
						i == 0 && threadIdx.x == 0, Q.init, (col1 - 1 - i) % UF, true, xa, xc, crc, &pd);
					mmcs_col<KM, RM, W, REFL, TB, true, CHUNK_BYTES, true, UF, D1>(
						P, s_tbl, s_sl, s_sh, k, rows, s, cb + CHUNK_BYTES, cb + 2 * CHUNK_BYTES, lo,
						i + 2 < iend, false, Q.init, (col1 - 2 - i) % UF, true, xc, xa, crc, &pd);
					i += 2;
				}
				for (; i < iend; i += 2) {
					const uint64_t cb = c0 + (uint64_t)i * CHUNK_BYTES;
					mmcs_col<KM, RM, W, REFL, TB, true, CHUNK_BYTES, true, UF, D1>(
						P, s_tbl, s_sl, s_sh, k, rows, s, cb, cb + CHUNK_BYTES, lo, true,
						i == 0 && threadIdx.x == 0, Q.init, (col1 - 1 - i) % UF, true, xa, xc, crc, &pd);
					mmcs_col<KM, RM, W, REFL, TB, true, CHUNK_BYTES, true, UF, D1>(
						P, s_tbl, s_sl, s_sh, k, rows, s, cb + CHUNK_BYTES, cb + 2 * CHUNK_BYTES, lo,
						i + 2 < iend, false, Q.init, (col1 - 2 - i) % UF, true, xc, xa, crc, &pd);
				}
			}
			for (; i < col1; i++)
				mmcs_col<KM, RM, W, REFL, TB, false, CHUNK_BYTES, false, UF, D1>(
					P, s_tbl, s_sl, s_sh, k, rows, s, c0 + (uint64_t)i * CHUNK_BYTES, 0, lo, false,
					i == 0 && threadIdx.x == 0, Q.init, (col1 - 1 - i) % UF, true, xa, xa, crc, &pd);
			if constexpr (DEFER) {
				mmcs_fold<RM, W, REFL, TB, UF>(s_sl, s_sh, rows, pd.v, pd.have, pd.first, Q.init, pd.pos,
							       pd.gshift, crc);
			}
			// each wave XORs its partial into the (zeroed) output: no
			// workgroup barrier, other waves keep streaming.  Reflected CRCs:
			// every lane's value is multiplied by its lane factor
			// x^(8*16*(63-l)) from the LDS nibble tables (W/4 steps), the wave
			// XOR-reduces, and the wave's sum is multiplied by the item factor
			// bit-parallel -- lane b keeps e_b * f if bit b of the sum is set,
			// one more XOR reduction.  No table read in the tail depends on
			// HBM: the r03 per-(row, wave) nibble tables in HBM cost crc64 up
			// to 30 % at 4-column items (serialised L2 round trips under the
			// streaming load, an experimental build without the tail,
			// profiles/r03/fused_tail/).  crc16: a W-step multiply per thread.
			// The rows are finished side by side (one basic block: their
			// lookup chains and reductions interleave), reduced with DPP into
			// wave-uniform values, then lane 0 XORs them into the output.
			T v[RM];
			const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
			for (int r = 0; r < RM; r++) {
				if constexpr (REFL) {
					v[r] = ecg_crc::lane_mul_nib<W>(crc[r], s_nibl, s_r4, lane);
				} else {
					v[r] = ecg_crc::mulmod<W, REFL>(kh[khrow * 256 + threadIdx.x], crc[r], poly);
				}
			}
#pragma unroll
			for (int r = 0; r < RM; r++)
				v[r] = ecg_crc::wave_xor_uniform(v[r]);
			if constexpr (REFL) {
#pragma unroll
				for (int r = 0; r < RM; r++)
					v[r] = ecg_crc::wave_xor_uniform(((v[r] >> (lane & (uint32_t)(W - 1))) & 1u) ? kbv : (T)0);
			}
			if (lane == 0) {
#pragma unroll
				for (int r = 0; r < RM; r++) {
					if (r < rows) {
						T x = v[r];
						if (threadIdx.x == 0 && khrow == (c + 1 == Q.nch ? Q.nh : 0))
							x ^= (T)Q.xorout;	// once per chunk
						const uint64_t slot = ((uint64_t)Q.row_slot[r] * P.nstripes + s) * Q.nch + c;
						if constexpr (W == 16)
							atomicXor((uint32_t *)Q.out + slot / 2, (uint32_t)x << (16 * (slot & 1)));
						else
							atomicXor((T *)Q.out + slot, x);
					}
				}
			}
	};
	// The workgroup's work: items blockIdx.x, blockIdx.x + gridDim.x, ... of
	// stripe blockIdx.y (+ gridDim.y ...) -- the grid never exceeds the item
	// and stripe counts, so the first is always there
	walk(blockIdx.y, blockIdx.x, ecg_bool<true>{});
	for (uint32_t s = blockIdx.y; s < P.nstripes; s += gridDim.y)
		for (uint32_t it = s == blockIdx.y ? blockIdx.x + gridDim.x : blockIdx.x; it < Q.nitems; it += gridDim.x)
			walk(s, it, ecg_bool<false>{});
}

typedef void (*mmcs_fn_t)(const ecg_mm_params_t, const ecg_mmcs_params_t);

struct csentry {
	int k, r, type;
	mmcs_fn_t fn;
	const char *name;
	int b8;		/* CRC table kind TB of the instantiation */
};

/* The table kind TB of each instantiation is the one measured fastest for
 * its shape (tools/fused_tables_ab.py, profiles/r02/fused_tables_ab/,
 * profiles/r03/fused_tb3/, fused_tb4/): the byte tables (TB 1) for crc64 and
 * for crc32 at EC_8P2, the conflict-free 5-bit tables (TB 0) everywhere else. */
#define CS_TB(K_, R_, W_) ((W_) == 64 || ((W_) == 32 && (K_) == 8 && (R_) == 2) ? 1 : 0)
#define CSE(K_, R_, T_, W_, RF_, N_) \
	{K_, R_, T_, ecg_mm_csum_kernel<K_, R_, W_, RF_, CS_TB(K_, R_, W_)>, \
	 "ecg_mm_csum_kernel<" #K_ "," #R_ "," N_ ">", CS_TB(K_, R_, W_)}
#define CSE3(K_, R_) CSE(K_, R_, 1, 16, false, "crc16"), CSE(K_, R_, 2, 32, true, "crc32"), \
		     CSE(K_, R_, 3, 64, true, "crc64")

static const csentry g_cskernels[] = {
	CSE3(2, 1), CSE3(2, 2), CSE3(2, 3), CSE3(4, 1), CSE3(4, 2), CSE3(4, 3),
	CSE3(8, 1), CSE3(8, 2), CSE3(8, 3), CSE3(16, 1), CSE3(16, 2), CSE3(16, 3),
	CSE3(0, 0),
};
#define N_CSKERNELS ((uint32_t)(sizeof(g_cskernels) / sizeof(g_cskernels[0])))
#define KID_FUSED ECG_KID_FUSED	/* fused kernel ids: KID_FUSED + index */

extern "C" const char *ecg_k_fused_kernel_name(uint32_t id)
{
	if (id >= KID_FUSED && id < KID_FUSED + N_CSKERNELS)
		return g_cskernels[id - KID_FUSED].name;
	return "?";
}

extern "C" int ecg_k_launch_matmul_csum(const ecg_mm_params_t *p, const ecg_mmcs_params_t *q,
				       const ecg_launch_cfg_t *cfg, void *stream, uint32_t *kernel_id)
{
	uint32_t id = N_CSKERNELS;

	if (p->nstripes == 0 || p->cell_bytes == 0 || p->rows == 0)
		return (int)hipSuccess;
	if (!aligned16(p) || p->accumulate || p->diff || (p->cell_bytes & 15u) ||
	    (q->chunk_bytes % CHUNK_BYTES) || q->chunk_bytes == 0)
		return 1;
	for (uint32_t i = 0; i < N_CSKERNELS; i++)
		if (g_cskernels[i].type == (int)q->type && g_cskernels[i].k == (int)p->k &&
		    g_cskernels[i].r == (int)p->rows) {
			id = i;
			break;
		}
	if (id == N_CSKERNELS)
		for (uint32_t i = 0; i < N_CSKERNELS; i++)
			if (g_cskernels[i].type == (int)q->type && g_cskernels[i].k == 0) {
				id = i;
				break;
			}
	if (id == N_CSKERNELS)			// no instantiation (not 1: that means "two-pass")
		return (int)hipErrorInvalidDeviceFunction;
	if (q->nitems == 0 || q->ncols == 0 || q->kh == nullptr)
		return (int)hipErrorInvalidDeviceFunction;
	// default: ~16 KiB of columns per workgroup (tools/tune8.py,
	// profiles/r01/tune8_fused_chunks.json: walking more columns per
	// workgroup loses HBM parallelism, fewer pays a reduction per column);
	// one-column items (4 KiB chunks) 8 per workgroup, two-column items 2,
	// longer items one per workgroup
	const uint64_t ipb = q->ncols == 1 ? 8 : q->ncols == 2 ? 2 : 1;
	uint32_t gx = cfg && cfg->grid_x ? cfg->grid_x : (uint32_t)((q->nitems + ipb - 1) / ipb);
	uint32_t gy = cfg && cfg->grid_y ? cfg->grid_y : (p->nstripes < 65535 ? p->nstripes : 65535);
	if (gx > 65535)
		gx = 65535;
	hipLaunchKernelGGL(g_cskernels[id].fn, dim3(gx, gy), dim3(BLOCK), 0, (hipStream_t)stream, *p, *q);
	if (kernel_id)
		*kernel_id = KID_FUSED + id;
	return (int)hipGetLastError();
}
