// ecg_ptr_kernels.hip -- the pointer-table product: ISA-L's data[] / coding[]
// convention (ec_encode_data(len, k, rows, tbls, data, coding)) batched over
// stripes, for callers whose cells lie wherever their buffers put them -- the
// client's full-stripe encode over a user sgl uses each cell in place when it
// lies inside one iov (obj_ec_stripe_encode, ref:src/object/cli_ec.c:476-546),
// so cell addresses carry no alignment.
//
// cells[s*(k+rows) + j] is the device address of input cell j (j < k) or output
// cell j-k of stripe s.  Same columns, tables and arithmetic as ecg_mm_kernel
// (ecg_mm_dev.h); a stripe's k+rows addresses are wave-uniform (scalar loads).
// The lane access G follows the cells' alignment exactly as the offset kernel:
// 16 (every address and the cell size 16-byte aligned), 4 (every input
// dword-aligned), 1 (an input at any byte: each input dword funnel-shifted out
// of aligned loads, ld_src<1>), 2 (k = 8 with an input off a 16-byte boundary:
// 16-byte lanes funnel-shifted, ld_src16); outputs at any byte take
// misaligned stores (the hardware's unaligned access mode, ecg_mm_dev.h
// mm_dword).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../ecg_kabi.h"
#include "ecg_mm_dev.h"

template <int KM, int RM, int G>
__device__ __forceinline__ void mm_ptr_item(const ecg_mm_params_t &P, const u32x4 *tb, int k, int rows,
					    uint32_t s, uint64_t cbase, uint32_t lo, const uint64_t *a)
{
	// phased loads as the offset kernel's (ECG_MM_PHASE): the first PH cells
	// now, the rest as the fold reaches them
	constexpr int PH = (ECG_MM_PHASE(KM, G) > 0 && ECG_MM_PHASE(KM, G) < KM && KM % ECG_MM_PHASE(KM, G) == 0)
				   ? ECG_MM_PHASE(KM, G) : 0;
	u32x4 x[KM], outv[RM];

#pragma unroll
	for (int j = 0; j < (PH ? PH : KM); j++)
		if (j < k)
			x[j] = ld_src<G>(reinterpret_cast<const uint8_t *>(a[j]), lo);
	mm_compute<KM, RM, false, true, false, G, PH, false, true>(P, tb, k, rows, s, cbase, lo, x, outv, a);
#pragma unroll
	for (int r = 0; r < RM; r++)
		if (r < rows)
			st_g<G>(reinterpret_cast<uint8_t *>(a[KM + r]) + lo, outv[r]);
}

// The partial last column of the G = 4 / 1 kernels, at column offset `off`
// of every cell: one dword (nb = 4; misaligned cells read and written as they
// are) or the nb < 4 bytes after the cell's last whole dword.  The cell
// addresses come from the stripe's table row `pt` (scalar loads), up to 8
// cells' loads in flight.
template <int KM, int RM>
__device__ __forceinline__ void mm_ptr_bytes(const u32x4 *tb, int k, int rows, const uint64_t *pt, uint64_t off,
					     int nb)
{
	constexpr int T2V = (RM + 3) / 4;
	constexpr int PER_J = RM + T2V;
	constexpr int JB = KM < 4 ? KM : 4;
	const bool dw = nb == 4;

	for (int b = 0; b < (dw ? 1 : nb); b++) {
		uint32_t o[RM];
#pragma unroll
		for (int r = 0; r < RM; r++)
			o[r] = 0;
#pragma nounroll
		for (int j0 = 0; j0 < k; j0 += JB) {
			uint32_t x[JB];

#pragma unroll
			for (int i = 0; i < JB; i++) {
				if (j0 + i < k) {
					const uint8_t *c = reinterpret_cast<const uint8_t *>(pt[j0 + i]) + off;
					x[i] = dw ? *reinterpret_cast<const uint32_t *>(c) : (uint32_t)c[b];
				}
			}
#pragma unroll
			for (int i = 0; i < JB; i++) {
				const int j = j0 + i;

				if (j >= k)
					continue;
				const uint32_t v = x[i];
				const uint32_t s0 = v & 0x07070707u, s1 = (v >> 3) & 0x07070707u, s2 = (v >> 6) & 0x03030303u;
#pragma unroll
				for (int r = 0; r < RM; r++) {
					if (r < rows) {
						const u32x4 t = tb[j * PER_J + r];
						const uint32_t t2 = reinterpret_cast<const uint32_t *>(&tb[j * PER_J + RM])[r];
						o[r] ^= __builtin_amdgcn_perm(t[1], t[0], s0) ^
							__builtin_amdgcn_perm(t[3], t[2], s1) ^ __builtin_amdgcn_perm(t2, t2, s2);
					}
				}
			}
		}
#pragma unroll
		for (int r = 0; r < RM; r++) {
			if (r < rows) {
				uint8_t *d = reinterpret_cast<uint8_t *>(pt[k + r]) + off;
				if (dw)
					*reinterpret_cast<uint32_t *>(d) = o[r];
				else
					d[b] = (uint8_t)o[r];
			}
		}
	}
}

template <int K, int R, int G>
__global__ void __launch_bounds__(BLOCK, ECG_MM_WPE(K, R, G) ? ECG_MM_WPE(K, R, G) : 1)
ecg_mm_ptr_kernel(const ecg_mm_params_t P, const uint64_t *__restrict__ cells)
{
	constexpr int KM = K ? K : ECG_KMAX_K;
	constexpr int RM = R ? R : ECG_KMAX_R;
	constexpr int T2V = (RM + 3) / 4;
	constexpr int PER_J = RM + T2V;
	__shared__ u32x4 s_tbl[KM * PER_J];
	const int k = K ? K : (int)P.k;
	const int rows = R ? R : (int)P.rows;
	const uint64_t C = P.cell_bytes;
	const uint32_t nchunk = (uint32_t)((C + CHUNK_BYTES - 1) / CHUNK_BYTES);
	const uint32_t lo = lane_off<G>();

	for (int i = threadIdx.x; i < KM * RM; i += BLOCK) {
		const int j = i / RM, r = i % RM;
		if (j < k && r < rows) {
			const ecg_ptbl_t &t = P.tbl[r][j];
			s_tbl[j * PER_J + r] = (u32x4){t.t0lo, t.t0hi, t.t1lo, t.t1hi};
			reinterpret_cast<uint32_t *>(&s_tbl[j * PER_J + RM])[r] = t.t2;
		}
	}
	__syncthreads();

	for (uint32_t s = blockIdx.y; s < P.nstripes; s += gridDim.y) {
		const uint64_t *pt = cells + (uint64_t)s * (uint32_t)(k + rows);
		uint64_t base[KM + RM];

		// the stripe's addresses: one dependent (scalar) load per stripe, not
		// per column -- the workgroup then walks several columns
#pragma unroll
		for (int j = 0; j < KM + RM; j++)
			if (j < k || (j >= KM && j - KM < rows))
				base[j] = pt[j < KM ? j : k + (j - KM)];
		for (uint32_t ch = blockIdx.x; ch < nchunk; ch += gridDim.x) {
			const uint64_t cbase = (uint64_t)ch * CHUNK_BYTES;
			uint64_t a[KM + RM];
			uint32_t z = 0;

#pragma unroll
			for (int j = 0; j < KM + RM; j++) {
				if (j < k || (j >= KM && j - KM < rows)) {
					a[j] = base[j] + cbase;
					asm volatile("" : "+s"(a[j]));
				}
			}
			asm volatile("" : "+v"(z));
			const u32x4 *tb = s_tbl + z;
			if (cbase + CHUNK_BYTES <= C) {
				mm_ptr_item<KM, RM, G>(P, tb, k, rows, s, cbase, lo, a);
			} else if constexpr (G == 16) {
				if (cbase + lo + 16 <= C)	// C % 16 == 0 on this path
					mm_ptr_item<KM, RM, G>(P, tb, k, rows, s, cbase, lo, a);
			} else {
				// the partial last column, dword by dword of the lane
				// (once per cell; a loop, not four inlined copies)
#pragma nounroll
				for (int i = 0; i < 4; i++) {
					const uint64_t off = cbase + lo + elem_off<G>(i);

					if (off < C)
						mm_ptr_bytes<KM, RM>(tb, k, rows, pt, off, (int)(C - off < 4 ? C - off : 4));
				}
			}
		}
	}
}

// Pointer-table product, any alignment and length: one byte per lane (launch
// variant 2 only: a second implementation for tests and A/B runs).
__global__ void __launch_bounds__(BLOCK)
ecg_mm_ptr_byte_kernel(const ecg_mm_params_t P, const uint64_t *cells)
{
	const uint64_t C = P.cell_bytes;
	const uint64_t total = C * P.nstripes;
	const int k = (int)P.k, rows = (int)P.rows;

	for (uint64_t e = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; e < total;
	     e += (uint64_t)gridDim.x * BLOCK) {
		const uint64_t s = e / C, i = e % C;
		const uint64_t *pt = cells + s * (uint64_t)(k + rows);
		uint8_t o[ECG_KMAX_R];

		for (int r = 0; r < ECG_KMAX_R; r++)
			o[r] = 0;
		for (int j = 0; j < k; j++) {
			const uint32_t v = reinterpret_cast<const uint8_t *>(pt[j])[i];
			for (int r = 0; r < rows; r++)
				o[r] ^= gf_mul1(P.tbl[r][j], v);
		}
		for (int r = 0; r < rows; r++)
			reinterpret_cast<uint8_t *>(pt[k + r])[i] = o[r];
	}
}

// ---------------------------------------------------------------------------
// Per-request delta updates (ecg_kabi.h ECG_UPD_REC): the batching queue's
// device-cell aggregation updates, agg_update_parity's xor_gen +
// ec_encode_data_update per updated cell (ref:src/object/srv_ec_aggregate.c:
// 1086-1102), batched over requests whose cells lie anywhere.  Item = one set
// of parity cells and up to ECG_UPD_MU (old, new, column) pairs folded into it
// (the host folds requests naming the same parity cells), so the parity is
// read and written once per item however many cells of its stripe changed:
// per pair 2 C read, per item 2 p C of parity traffic.  The tables of every
// (row, column) pair are staged in LDS once per block; a pair's column picks
// its table base (wave-uniform).
// ---------------------------------------------------------------------------

// acc[r] ^= tbl[r] * x for the 4 dwords of x (one pair's delta)
template <int RM>
__device__ __forceinline__ void upd_fold(const u32x4 *tb, int rows, const u32x4 x, u32x4 *acc)
{
	constexpr int T2V = (RM + 3) / 4;
	u32x4 sel0, sel1, sel2, t2v[T2V];

#pragma unroll
	for (int w = 0; w < 4; w++) {
		sel0[w] = x[w] & 0x07070707u;
		sel1[w] = (x[w] >> 3) & 0x07070707u;
		sel2[w] = (x[w] >> 6) & 0x03030303u;
	}
#pragma unroll
	for (int q = 0; q < T2V; q++)
		t2v[q] = tb[RM + q];
#pragma unroll
	for (int r = 0; r < RM; r++) {
		if (r < rows) {
			const u32x4 t = tb[r];
			const uint32_t t2 = t2v[r / 4][r % 4];
#pragma unroll
			for (int w = 0; w < 4; w++)
				acc[r][w] = xor3(acc[r][w], __builtin_amdgcn_perm(t[1], t[0], sel0[w]),
						 xor3(__builtin_amdgcn_perm(t[3], t[2], sel1[w]),
						      __builtin_amdgcn_perm(t2, t2, sel2[w]), 0u));
		}
	}
}

// One whole 4 KiB column of item `it` at column offset `off` (= cbase + lane
// offset): parity loads first, then the pairs two at a time (four cell loads
// in flight), one store per parity row.
template <int RM, int G>
__device__ __forceinline__ void upd_col(const u32x4 *s_tbl, const uint64_t *it, int rows, uint32_t n,
					uint64_t cols, uint32_t ncols, uint64_t off)
{
	constexpr int PER_J = RM + (RM + 3) / 4;
	u32x4 acc[RM];

#pragma unroll
	for (int r = 0; r < RM; r++)
		if (r < rows)
			acc[r] = ld_g<G>(reinterpret_cast<const uint8_t *>(it[r]) + off);
	for (uint32_t m = 0; m < n; m += 2) {
		const uint64_t *pr = it + rows + 2 * m;
		const bool two = m + 1 < n;
		const u32x4 x0 = ld_g<G>(reinterpret_cast<const uint8_t *>(pr[0]) + off) ^
				 ld_g<G>(reinterpret_cast<const uint8_t *>(pr[1]) + off);
		u32x4 x1 = (u32x4){0u, 0u, 0u, 0u};
		if (two)
			x1 = ld_g<G>(reinterpret_cast<const uint8_t *>(pr[2]) + off) ^
			     ld_g<G>(reinterpret_cast<const uint8_t *>(pr[3]) + off);
		const uint32_t j0 = (uint32_t)(cols >> (8 * m)) & 0xffu;
		if (j0 < ncols)
			upd_fold<RM>(s_tbl + j0 * PER_J, rows, x0, acc);
		if (two) {
			const uint32_t j1 = (uint32_t)(cols >> (8 * (m + 1))) & 0xffu;
			if (j1 < ncols)
				upd_fold<RM>(s_tbl + j1 * PER_J, rows, x1, acc);
		}
	}
#pragma unroll
	for (int r = 0; r < RM; r++)
		if (r < rows)
			st_g<G>(reinterpret_cast<uint8_t *>(it[r]) + off, acc[r]);
}

// One dword of every parity row at byte offset `off` (partial last column;
// C % 4 == 0 on the lane kernels, so the lanes' dwords cover the cell).
template <int RM>
__device__ __forceinline__ void upd_dword(const u32x4 *s_tbl, const uint64_t *it, int rows, uint32_t n,
					  uint64_t cols, uint32_t ncols, uint64_t off)
{
	constexpr int PER_J = RM + (RM + 3) / 4;
	uint32_t a[RM];

#pragma unroll
	for (int r = 0; r < RM; r++)
		if (r < rows)
			a[r] = *reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(it[r]) + off);
	for (uint32_t m = 0; m < n; m++) {
		const uint64_t *pr = it + rows + 2 * m;
		const uint32_t j = (uint32_t)(cols >> (8 * m)) & 0xffu;
		const uint32_t v = *reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(pr[0]) + off) ^
				   *reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(pr[1]) + off);
		const uint32_t s0 = v & 0x07070707u, s1 = (v >> 3) & 0x07070707u, s2 = (v >> 6) & 0x03030303u;

		if (j >= ncols)
			continue;
		const u32x4 *tb = s_tbl + j * PER_J;
#pragma unroll
		for (int r = 0; r < RM; r++) {
			if (r < rows) {
				const u32x4 t = tb[r];
				const uint32_t t2 = reinterpret_cast<const uint32_t *>(&tb[RM])[r];
				a[r] ^= __builtin_amdgcn_perm(t[1], t[0], s0) ^ __builtin_amdgcn_perm(t[3], t[2], s1) ^
					__builtin_amdgcn_perm(t2, t2, s2);
			}
		}
	}
#pragma unroll
	for (int r = 0; r < RM; r++)
		if (r < rows)
			*reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(it[r]) + off) = a[r];
}

template <int R, int G>
__global__ void __launch_bounds__(BLOCK)
ecg_upd_ptr_kernel(const ecg_mm_params_t P, const uint64_t *__restrict__ items, uint32_t ncols)
{
	constexpr int RM = R ? R : ECG_KMAX_R;
	constexpr int PER_J = RM + (RM + 3) / 4;
	__shared__ u32x4 s_tbl[ECG_KMAX_K * PER_J];
	const int rows = R ? R : (int)P.rows;
	const uint32_t rec = (uint32_t)ECG_UPD_REC(rows);
	const uint64_t C = P.cell_bytes;
	const uint32_t nchunk = (uint32_t)((C + CHUNK_BYTES - 1) / CHUNK_BYTES);
	const uint32_t lo = lane_off<G>();

	for (int i = threadIdx.x; i < ECG_KMAX_K * RM; i += BLOCK) {
		const int j = i / RM, r = i % RM;
		if (j < (int)ncols && r < rows) {
			const ecg_ptbl_t &t = P.tbl[r][j];
			s_tbl[j * PER_J + r] = (u32x4){t.t0lo, t.t0hi, t.t1lo, t.t1hi};
			reinterpret_cast<uint32_t *>(&s_tbl[j * PER_J + RM])[r] = t.t2;
		}
	}
	__syncthreads();

	for (uint32_t s = blockIdx.y; s < P.nstripes; s += gridDim.y) {
		const uint64_t *it = items + (uint64_t)s * rec;
		const uint64_t cols = it[rows + 2 * ECG_UPD_MU];
		uint32_t n = (uint32_t)it[rows + 2 * ECG_UPD_MU + 1];

		if (n > ECG_UPD_MU)	/* host-validated; never read past the record */
			n = ECG_UPD_MU;
		for (uint32_t ch = blockIdx.x; ch < nchunk; ch += gridDim.x) {
			const uint64_t cbase = (uint64_t)ch * CHUNK_BYTES;

			if (cbase + CHUNK_BYTES <= C) {
				upd_col<RM, G>(s_tbl, it, rows, n, cols, ncols, cbase + lo);
			} else {
#pragma nounroll
				for (int i = 0; i < 4; i++) {
					const uint64_t off = cbase + lo + elem_off<G>(i);

					if (off + 4 <= C)
						upd_dword<RM>(s_tbl, it, rows, n, cols, ncols, off);
				}
			}
		}
	}
}

// Any alignment and length: one byte per lane (cells whose size is not a
// multiple of 4, or misaligned cells on a device without unaligned access).
__global__ void __launch_bounds__(BLOCK)
ecg_upd_ptr_byte_kernel(const ecg_mm_params_t P, const uint64_t *items, uint32_t ncols)
{
	const uint64_t C = P.cell_bytes;
	const uint64_t total = C * P.nstripes;
	const int rows = (int)P.rows;
	const uint32_t rec = (uint32_t)ECG_UPD_REC(rows);

	for (uint64_t e = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; e < total; e += (uint64_t)gridDim.x * BLOCK) {
		const uint64_t s = e / C, i = e % C;
		const uint64_t *it = items + s * rec;
		const uint64_t cols = it[rows + 2 * ECG_UPD_MU];
		const uint32_t n = (uint32_t)it[rows + 2 * ECG_UPD_MU + 1];
		uint8_t o[ECG_KMAX_R];

		for (int r = 0; r < ECG_KMAX_R; r++)
			o[r] = 0;
		for (uint32_t m = 0; m < n && m < ECG_UPD_MU; m++) {
			const uint32_t j = (uint32_t)(cols >> (8 * m)) & 0xffu;
			const uint32_t v = reinterpret_cast<const uint8_t *>(it[rows + 2 * m])[i] ^
					   reinterpret_cast<const uint8_t *>(it[rows + 2 * m + 1])[i];

			if (j >= ncols)
				continue;
			for (int r = 0; r < rows; r++)
				o[r] ^= gf_mul1(P.tbl[r][j], v);
		}
		for (int r = 0; r < rows; r++)
			reinterpret_cast<uint8_t *>(it[r])[i] ^= o[r];
	}
}

typedef void (*updptr_fn_t)(const ecg_mm_params_t, const uint64_t *, uint32_t);

struct uentry {
	int r, g;
	updptr_fn_t fn;
	const char *name;
};

#define UE(R_, G_) {R_, G_, ecg_upd_ptr_kernel<R_, G_>, "ecg_upd_ptr_kernel<" #R_ ",g" #G_ ">"}

// the DAOS classes' p = 1..3 specialised, 4..8 parity rows runtime-shaped
static const uentry g_ukernels[] = {
	UE(1, 16), UE(2, 16), UE(3, 16), UE(0, 16), UE(1, 4), UE(2, 4), UE(3, 4), UE(0, 4),
};
#define N_UKERNELS ((uint32_t)(sizeof(g_ukernels) / sizeof(g_ukernels[0])))
#define KID_UPD (ECG_KID_PTR + 60u)		/* below the byte kernels' ids */
#define KID_UPD_BYTE (KID_UPD + N_UKERNELS)

extern "C" int ecg_k_launch_update_ptrs(const ecg_mm_params_t *p, const uint64_t *items_dev, uint32_t ncols,
				       int granule, void *stream, uint32_t *kernel_id)
{
	hipStream_t st = (hipStream_t)stream;
	const uint64_t C = p->cell_bytes;
	const uint64_t nchunk = (C + CHUNK_BYTES - 1) / CHUNK_BYTES;
	uint32_t id = N_UKERNELS;

	if (p->nstripes == 0 || C == 0)
		return (int)hipSuccess;
	if (p->rows < 1 || p->rows > ECG_KMAX_R || ncols < 1 || ncols > ECG_KMAX_K)
		return (int)hipErrorInvalidValue;
	if ((granule == 16 && (C & 15u)) || (granule == 4 && (C & 3u)))
		granule = 0;
	if (granule == 0) {
		uint64_t blocks = (C * p->nstripes + BLOCK - 1) / BLOCK;
		if (blocks > 8192)
			blocks = 8192;
		hipLaunchKernelGGL(ecg_upd_ptr_byte_kernel, dim3((uint32_t)blocks), dim3(BLOCK), 0, st, *p, items_dev,
				   ncols);
		if (kernel_id)
			*kernel_id = KID_UPD_BYTE;
		return (int)hipGetLastError();
	}
	if (granule != 16 && granule != 4)
		return (int)hipErrorInvalidValue;
	for (uint32_t i = 0; i < N_UKERNELS && id == N_UKERNELS; i++)
		if (g_ukernels[i].g == granule && (g_ukernels[i].r == (int)p->rows || g_ukernels[i].r == 0))
			id = i;
	const uint32_t gx = (uint32_t)(nchunk < 65535 ? nchunk : 65535);
	const uint32_t gy = p->nstripes < 65535 ? p->nstripes : 65535;
	hipLaunchKernelGGL(g_ukernels[id].fn, dim3(gx, gy), dim3(BLOCK), 0, st, *p, items_dev, ncols);
	if (kernel_id)
		*kernel_id = KID_UPD + id;
	return (int)hipGetLastError();
}

typedef void (*mmptr_fn_t)(const ecg_mm_params_t, const uint64_t *);

struct pentry {
	int k, r, g;
	mmptr_fn_t fn;
	const char *name;
};

#define PE(K_, R_) {K_, R_, 16, ecg_mm_ptr_kernel<K_, R_, 16>, "ecg_mm_ptr_kernel<" #K_ "," #R_ ">"}
#define PEG(K_, R_, G_) {K_, R_, G_, ecg_mm_ptr_kernel<K_, R_, G_>, "ecg_mm_ptr_kernel<" #K_ "," #R_ ",g" #G_ ">"}
#define PEG_SET(G_) \
	PEG(2, 1, G_), PEG(2, 2, G_), PEG(2, 3, G_), PEG(4, 1, G_), PEG(4, 2, G_), PEG(4, 3, G_), \
	PEG(8, 1, G_), PEG(8, 2, G_), PEG(8, 3, G_), PEG(16, 1, G_), PEG(16, 2, G_), PEG(16, 3, G_), PEG(0, 0, G_)

static const pentry g_pkernels[] = {
	PE(2, 1), PE(2, 2), PE(2, 3), PE(4, 1), PE(4, 2), PE(4, 3),
	PE(8, 1), PE(8, 2), PE(8, 3), PE(16, 1), PE(16, 2), PE(16, 3), PE(0, 0),
	PEG_SET(4), PEG_SET(1),
	PEG(8, 1, 2), PEG(8, 2, 2), PEG(8, 3, 2),	/* k = 8 inputs off 16 B (ecg_ptrs.c ptr_granule) */
};
#define N_PKERNELS ((uint32_t)(sizeof(g_pkernels) / sizeof(g_pkernels[0])))
#define KID_PTR ECG_KID_PTR		/* pointer-table kernel ids: KID_PTR + index */
#define KID_PTR_BYTE (KID_PTR + N_PKERNELS)

extern "C" const char *ecg_k_ptr_kernel_name(uint32_t id)
{
	if (id >= KID_PTR && id < KID_PTR + N_PKERNELS)
		return g_pkernels[id - KID_PTR].name;
	if (id == KID_PTR_BYTE)
		return "ecg_mm_ptr_byte_kernel";
	if (id >= KID_UPD && id < KID_UPD + N_UKERNELS)
		return g_ukernels[id - KID_UPD].name;
	if (id == KID_UPD_BYTE)
		return "ecg_upd_ptr_byte_kernel";
	return "?";
}

extern "C" int ecg_k_launch_matmul_ptrs(const ecg_mm_params_t *p, const uint64_t *cells_dev, int granule,
				       const ecg_launch_cfg_t *cfg, void *stream, uint32_t *kernel_id)
{
	hipStream_t st = (hipStream_t)stream;
	const uint64_t nchunk = (p->cell_bytes + CHUNK_BYTES - 1) / CHUNK_BYTES;
	int g = granule;
	uint32_t id = N_PKERNELS;

	if (p->nstripes == 0 || p->cell_bytes == 0 || p->rows == 0)
		return (int)hipSuccess;
	if (g == 16 && (p->cell_bytes & 15u))	// the 16-byte lanes need whole 16-byte pieces
		g = 4;
	if (g == 0 || (cfg && cfg->variant == 2)) {	/* 0: the host found operands the
							 * device cannot serve as dwords */
		uint64_t blocks = (p->cell_bytes * p->nstripes + BLOCK - 1) / BLOCK;
		if (blocks > 8192)
			blocks = 8192;
		hipLaunchKernelGGL(ecg_mm_ptr_byte_kernel, dim3((uint32_t)blocks), dim3(BLOCK), 0, st, *p,
				   cells_dev);
		if (kernel_id)
			*kernel_id = KID_PTR_BYTE;
		return (int)hipGetLastError();
	}
	if (g != 16 && g != 4 && g != 2 && g != 1)
		return (int)hipErrorInvalidValue;
	for (uint32_t i = 0; i < N_PKERNELS && (!cfg || cfg->variant != 1); i++)
		if (g_pkernels[i].g == g && g_pkernels[i].k == (int)p->k && g_pkernels[i].r == (int)p->rows) {
			id = i;
			break;
		}
	// g = 2 exists only for k = 8's own shapes: with no such entry (variant
	// 1 skips them) the funnel-shifted dword lanes of g = 1 take the launch,
	// which have a runtime-shaped kernel
	if (id == N_PKERNELS && g == 2)
		g = 1;
	for (uint32_t i = 0; i < N_PKERNELS && id == N_PKERNELS; i++)
		if (g_pkernels[i].g == g && g_pkernels[i].k == 0)	/* runtime-shaped */
			id = i;
	if (id == N_PKERNELS)
		return (int)hipErrorInvalidDeviceFunction;
	uint32_t gx = cfg && cfg->grid_x ? cfg->grid_x : (uint32_t)(nchunk < 65535 ? nchunk : 65535);
	uint32_t gy = cfg && cfg->grid_y ? cfg->grid_y : (p->nstripes < 65535 ? p->nstripes : 65535);
	// blocks per CU as the offset kernel's (ecg_set_wg_per_cu): unused dynamic LDS
	const size_t lds = mm_dyn_lds(mm_wg_cap(p, cfg, (uint64_t)gx * gy), g_pkernels[id].k, g_pkernels[id].r);
	hipLaunchKernelGGL(g_pkernels[id].fn, dim3(gx, gy), dim3(BLOCK), lds, st, *p, cells_dev);
	if (kernel_id)
		*kernel_id = KID_PTR + id;
	return (int)hipGetLastError();
}
