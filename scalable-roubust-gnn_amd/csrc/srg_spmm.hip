// srg_spmm.hip -- CSR x dense-panel propagation kernels for MI355X (gfx950, CDNA4).
//
// The hot path of the reference is FloatCSRMulDenseOMP (SSRG/operators/csrc/matmul.c:23-40): per
// output row, for every stored nonzero in CSR order, answer[i,:] = fma(a_ij, X[j,:], answer[i,:]).
// It is HBM-bound (~0.48 flop/B at d = 128): the work is gathering 4*d-byte rows of X, one per
// nonzero.  The design here:
//
//  * One wavefront (64 lanes) owns one output row and a 64*VEC-column tile of it; each lane owns
//    VEC consecutive columns and keeps their running sums in registers.  Every output element is
//    therefore one sequential fp32 fma chain in CSR order -- bit-identical to the reference.
//  * The row's (column id, value) stream is wave-uniform, so it is read with scalar loads into
//    SGPRs (s_load_dwordx*), and each X row address is a scalar base + the lane's column offset:
//    one vector instruction (global_load_dwordx{1,2,4}) per nonzero gathers the whole 4*d-byte row.
//  * U nonzeros are processed per step: U independent gathers are issued back to back (U rows in
//    flight per wave, ~U*512 B at d = 128), then consumed in order by the fma chain.  The chain is
//    4 cycles per link; the gathers are what the wave waits on.
//  * Rows are scheduled through an optional permutation (host plan: decreasing length), so the
//    long power-law hub rows start first and overlap the bulk instead of forming the tail.
//  * No atomics, no inter-workgroup communication, no LDS: each row is owned by exactly one wave.
//
// The Chebyshev (wavelet) kernels reuse the same row-wave gather and add a fused epilogue that
// forms the next Chebyshev term and accumulates every scale's filter output in the same pass.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "srgnn_hip.h"
#include "srg_plan_internal.h"

#ifndef SRG_GIT_REV
#define SRG_GIT_REV "dev"
#endif

namespace {

// ------------------------------------------------------------------------------------------------
// error handling
// ------------------------------------------------------------------------------------------------
thread_local char g_err_msg[512] = "";
thread_local int g_err_code = SRG_OK;

int fail(int code, const char* fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err_msg, sizeof(g_err_msg), fmt, ap);
    va_end(ap);
    g_err_code = code;
    return code;
}

int ok()
{
    g_err_code = SRG_OK;
    g_err_msg[0] = '\0';
    return SRG_OK;
}

#define SRG_HIP_CHECK(expr)                                                                     \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return fail(SRG_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));            \
    } while (0)

// ------------------------------------------------------------------------------------------------
// vector helpers
// ------------------------------------------------------------------------------------------------
template <typename T, int VEC> struct Vec;
template <> struct Vec<float, 1> { typedef float type; };
template <> struct Vec<float, 2> { typedef float type __attribute__((ext_vector_type(2))); };
template <> struct Vec<float, 4> { typedef float type __attribute__((ext_vector_type(4))); };
template <> struct Vec<double, 1> { typedef double type; };
template <> struct Vec<double, 2> { typedef double type __attribute__((ext_vector_type(2))); };

// element i of a scalar-or-vector value
template <typename T> __device__ __forceinline__ T& elem(T& v, int) { return v; }
template <typename T> __device__ __forceinline__ const T& elem(const T& v, int) { return v; }
template <typename T, int N>
__device__ __forceinline__ T& elem(T __attribute__((ext_vector_type(N)))& v, int i) { return reinterpret_cast<T*>(&v)[i]; }
template <typename T, int N>
__device__ __forceinline__ const T& elem(const T __attribute__((ext_vector_type(N)))& v, int i) { return reinterpret_cast<const T*>(&v)[i]; }

template <typename T, int VEC>
__device__ __forceinline__ typename Vec<T, VEC>::type vload(const T* p)
{
    return *reinterpret_cast<const typename Vec<T, VEC>::type*>(p);
}
// Gather of one X row piece (plain loads: the gathered rows are re-read from L2 / Infinity Cache;
// non-temporal gathers measured 35 % slower on the products-shaped graph).
template <typename T, int VEC>
__device__ __forceinline__ typename Vec<T, VEC>::type gload(const T* p)
{
    return *reinterpret_cast<const typename Vec<T, VEC>::type*>(p);
}

template <typename T, int VEC>
__device__ __forceinline__ void vstore(T* p, typename Vec<T, VEC>::type v, bool nt)
{
    typedef typename Vec<T, VEC>::type V;
    if (nt)
        __builtin_nontemporal_store(v, reinterpret_cast<V*>(p));
    else
        *reinterpret_cast<V*>(p) = v;
}

// One link of the reference chain: acc = fma(a, x, acc) per component (fp32), or acc + a*x without
// contraction (fp64: scipy's csr_matvecs order, see srg_oracle.c).
__device__ __forceinline__ float link(float a, float x, float acc) { return __builtin_fmaf(a, x, acc); }
__device__ __forceinline__ double link(double a, double x, double acc)
{
    return __dadd_rn(acc, __dmul_rn(a, x));
}

// Epilogue arithmetic: fp64 follows numpy/scipy rounding exactly (no contraction into fma);
// fp32 leaves the compiler free (the fp32 Chebyshev path is tolerance-checked).
__device__ __forceinline__ double e_mul(double a, double b) { return __dmul_rn(a, b); }
__device__ __forceinline__ double e_add(double a, double b) { return __dadd_rn(a, b); }
__device__ __forceinline__ double e_sub(double a, double b) { return __dsub_rn(a, b); }
__device__ __forceinline__ double e_div(double a, double b) { return __ddiv_rn(a, b); }
__device__ __forceinline__ float e_mul(float a, float b) { return a * b; }
__device__ __forceinline__ float e_add(float a, float b) { return a + b; }
__device__ __forceinline__ float e_sub(float a, float b) { return a - b; }
__device__ __forceinline__ float e_div(float a, float b) { return a / b; }

template <typename T, int VEC>
__device__ __forceinline__ void chain(typename Vec<T, VEC>::type& acc, T a,
                                      const typename Vec<T, VEC>::type& x)
{
    if constexpr (VEC == 1) {
        acc = link(a, x, acc);
    } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc[i] = link(a, x[i], acc[i]);
    }
}

template <typename T, int VEC> __device__ __forceinline__ typename Vec<T, VEC>::type vzero()
{
    typename Vec<T, VEC>::type z;
    if constexpr (VEC == 1) {
        z = T(0);
    } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) z[i] = T(0);
    }
    return z;
}

constexpr int kWavesPerBlock = 4;   // 256-thread workgroups
constexpr int kBlock = 64 * kWavesPerBlock;

// ------------------------------------------------------------------------------------------------
// the row-wave gather: acc (+)= A[row, :] * X[:, col .. col+VEC)
//
// The row's (column id, value) stream is read 64 entries at a time with one coalesced vector load
// (lane l holds entry jb + l), prefetched one block ahead, and broadcast to the whole wave with
// v_readlane (the lane index is wave-uniform).  Each entry's X row address is then a scalar base
// plus the lane's column offset.  U gathers are issued back to back, then consumed in CSR order.
// Entries past the end of the row repeat its last entry and are skipped by a wave-uniform predicate
// (never folded in as 0*x: that would flip -0.0 sums and turn inf/nan inputs into nan).
// FULL: every lane of the wave owns columns (d is a multiple of 64*VEC), so no lane predicates.
// ------------------------------------------------------------------------------------------------
// SPAN: the row's entries end at row_end[row] instead of indptr[row + 1] (kEpiSpan below).
template <typename T, int VEC, int U, bool FULL, typename IP, bool SPAN = false>
__device__ __forceinline__ void row_gather(typename Vec<T, VEC>::type& acc,
                                           const IP* __restrict__ indptr,
                                           const int32_t* __restrict__ indices,
                                           const T* __restrict__ vals, int row,
                                           const T* __restrict__ X, int64_t ldx, int col, bool act,
                                           const int64_t* __restrict__ row_end = nullptr)
{
    typedef typename Vec<T, VEC>::type V;
    const int lane = threadIdx.x & 63;
    const int64_t beg = indptr[row];
    int64_t end;
    if constexpr (SPAN)
        end = row_end[row];
    else
        end = indptr[row + 1];
    if (beg >= end) return;
    // entries past the row end are clamped to its last entry (always a valid id; skipped below)
    int64_t j0 = beg + lane;
    j0 = j0 < end ? j0 : end - 1;
    int c_nxt = indices[j0];
    T a_nxt = vals[j0];
    for (int64_t jb = beg; jb < end; jb += 64) {
        const int c_blk = c_nxt;
        const T a_blk = a_nxt;
        int64_t jn = jb + 64 + lane;   // prefetch the next block of the stream
        jn = jn < end ? jn : end - 1;
        c_nxt = indices[jn];
        a_nxt = vals[jn];
        const int nblk = (end - jb) < 64 ? (int)(end - jb) : 64;   // wave-uniform
        for (int s0 = 0; s0 < nblk; s0 += U) {
            V x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int c = __builtin_amdgcn_readlane(c_blk, s0 + u);
                const T* p = X + (int64_t)c * ldx + col;
                if (FULL || act)
                    x[u] = gload<T, VEC>(p);
                else
                    x[u] = vzero<T, VEC>();
            }
            const int n = (nblk - s0) < U ? (nblk - s0) : U;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                T a;
                if constexpr (sizeof(T) == 8) {   // v_readlane is 32-bit: broadcast both halves
                    const unsigned long long bits = __builtin_bit_cast(unsigned long long, a_blk);
                    const unsigned lo = __builtin_amdgcn_readlane((unsigned)bits, s0 + u);
                    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(bits >> 32), s0 + u);
                    a = __builtin_bit_cast(T, ((unsigned long long)hi << 32) | lo);
                } else {
                    a = __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, a_blk), s0 + u));
                }
                if (u < n) chain<T, VEC>(acc, a, x[u]);
            }
        }
    }
}

__device__ __forceinline__ int wave_slot(int block_base)
{
    // wave-uniform by construction; readfirstlane makes that provable to the compiler so that the
    // row's index stream goes through the scalar path.
    return __builtin_amdgcn_readfirstlane((int)((block_base + (int)blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6)));
}

// A dispatch holds < 2^32 work-items per dimension: launches of more rows than that (111 M rows
// of the papers100M-shaped graph = 7.1e9 lanes) go out in chunks of kMaxLaunchBlocks blocks, the
// kernel adding the chunk's block_base to blockIdx.x.
constexpr int64_t kMaxLaunchBlocks = int64_t(1) << 23;

// ------------------------------------------------------------------------------------------------
// SpMM: Y = A * X  (or Y += A * X)
//
// One launch, two wave roles (wave-uniform, decided by blockIdx):
//  * blocks [0, nb_heavy): "slice" waves.  The first n_heavy rows of `order` are long rows; each is
//    cut into 32-column slices (128 B of every X row = one cache line) and every (row, slice) pair
//    is one wave.  Lane l gathers the 16-byte chunk (l & 7) of nonzero (l >> 3): one
//    global_load_dwordx4 instruction brings 8 nonzeros' slices (1 KiB); UH such instructions are in
//    flight per wave.  The 8x32 tile is transposed through a wave-private LDS slot so that lane c
//    (c < 32) runs the sequential fma chain of column c over the nonzeros in CSR order.  A row of
//    degree D is worked on by d/32 waves at once with UH*1 KiB in flight each, which keeps
//    power-law hubs (D > 10^5 on the products-shaped graph) off the critical path.
//  * blocks [nb_heavy, ...): "row" waves, one per remaining row (row_gather above).
// Both roles produce bit-identical results (one fma chain per output element, CSR order).
// ------------------------------------------------------------------------------------------------
constexpr int kSliceCols = 32;
// LDS tiles per slice wave (8 nonzeros x 32 columns, 1 KB each).  One suffices: a wave's LDS
// operations complete in issue order, so the next group's write cannot overtake this group's reads.
// Two (the round-1 layout) cost 8 KB per k_spmm block, which beside the hub group's 72 KB workgroups
// (halo exchange) left room for only two row blocks per CU.
constexpr int kSliceLdsBufs = 1;
// The slice waves' (column id, value) loads for the next group of entries are issued right after the
// current group's gathers, so their latency overlaps the gathers and the fma links instead of
// preceding the next gathers.  Products (one box, profiles/r04u_prefetch_ab.txt): none 6.02 ms per
// hop, slice waves 5.82.  It costs 2 UH registers (73 instead of 54-70: 6 waves per SIMD).  Same
// entries in the same order: same bits.  (The packed light rows stage their ids across their lanes
// instead, packed_rows; their round-4 per-group prefetch and LDS-staged entries measured slower,
// profiles/r04h_stage_entries_negative.txt.)
constexpr bool kPrefetchSliceIds = true;

// Epilogues of the SpMM kernels (every output element y a kernel stores may also go to):
//  * fused hop aggregation (srgnn.aggregate): with agg != nullptr it is folded into the accumulator
//    panel, agg = (init ? 0 : agg) + w*y, with separate multiply and add -- the same arithmetic as a
//    following srg_hop_accumulate_f32 step, without re-reading Y;
//  * fused Chebyshev step (srgnn.wavelet, srg_spmm_cheby_f32): y = A*T_k becomes T_{k+1} before it
//    is stored and every scale's output is updated, with k_cheby_epilogue's arithmetic --
//      INIT: T1 = (y - a2*T0) / a1,  R_s = (c0_s/2)*T0 + c1_s*T1   (T0 = X, the gathered panel)
//      STEP: T_{k+1} = y - T_{k-1},  R_s += ck_s*T_{k+1}
//    T0 / T_{k-1} is read before the chain (its latency hides under the gathers).  Y may alias
//    T_{k-1}: every element is read and then written by its one owner, and no wave gathers it, so
//    a step needs two work panels instead of three and one panel pass less than the split path.
template <typename T> struct ChebyCoef {
    T prev[8];   // c0_s / 2 (INIT, STEP_FIRST)
    T cur[8];    // c1_s (INIT) or ck_s (STEP, STEP_FIRST)
    T mid[8];    // c1_s (STEP_FIRST only)
};

struct Epi {
    float* agg;
    int64_t lda;
    float w;
    int init;
    // fused Chebyshev step (EX == kEpiCheby only)
    const float* cto;     // T_{k-1} (STEP)
    int64_t ldo;
    float* R;             // R_s = R + s * r_stride, rows ldr apart
    int64_t ldr, r_stride;
    int cmode, ns;
    float a1, a2;
    ChebyCoef<float> cf;
    // row spans (EX == kEpiSpan only): row r's entries are [indptr[r], row_end[r]) instead of
    // [indptr[r], indptr[r + 1]) -- a column block of a CSR whose rows hold sorted column ids is a
    // span of each row, so the block needs no copy of the ids and values (srg_spmm_span_f32)
    const int64_t* row_end;
    // kEpiSpan, optional: the spans by schedule slot (slot_beg[s] / slot_end[s] = the span of the row
    // in slot s of this launch's light-row schedule), read by the packed light rows instead of the
    // row-indexed arrays: consecutive slots, consecutive addresses (srg_propagate_plan_f32)
    const int64_t* slot_beg;
    const int64_t* slot_end;
};

// Epilogue kinds (template parameter EX of the SpMM kernels).  Every call site sits under
// `if constexpr`: a runtime branch cost the plain kernels ~20 %, and even an empty inlined call
// (the reference-bound acc) changed the gather loop's schedule (+10 % per hop on products);
// guarded, the kEpiPlain kernels are instruction-for-instruction the plain ones.  kEpiSpan is the
// plain epilogue (aggregation included) over row spans.
// (round 5 removed the fused halo pack, kEpiSend, and the per-row accumulation of the medium-span
// probe, kEpiSpanRA: both measured slower)
constexpr int kEpiPlain = 0, kEpiCheby = 2, kEpiSpan = 3;
template <int EX> constexpr bool kIsSpan = EX == kEpiSpan;

// End of row `row`'s entries: the next row's start, or the span's end.
template <int EX, typename IP>
__device__ __forceinline__ int64_t row_stop(const IP* __restrict__ indptr, const Epi& e, int row)
{
    if constexpr (kIsSpan<EX>)
        return e.row_end[row];
    else
        return (int64_t)indptr[row + 1];
}


// Operands of the Chebyshev epilogue at (row, col), loaded before the chain so that their latency
// hides under the gathers (loaded after it, the R round trips were the end of every light row:
// +40 % per order on products): T0 = X (INIT) or T_{k-1} (STEP), and in a step the current
// outputs of the first kChebyPre scales (further scales are read after the chain).
constexpr int kChebyPre = 2;
template <int VEC> struct ChebyOps {
    typename Vec<float, VEC>::type pre, r[kChebyPre];
};

template <int VEC>
__device__ __forceinline__ void cheby_load(const Epi& e, int row, int col, const float* __restrict__ X, int64_t ldx,
                                           ChebyOps<VEC>& o)
{
    if (e.cmode == SRG_CHEBY_INIT) {
        o.pre = vload<float, VEC>(X + (int64_t)row * ldx + col);
    } else {
        o.pre = vload<float, VEC>(e.cto + (int64_t)row * e.ldo + col);
        const float* rr = e.R + (int64_t)row * e.ldr + col;
#pragma unroll
        for (int s = 0; s < kChebyPre; ++s)
            if (s < e.ns) o.r[s] = vload<float, VEC>(rr + s * e.r_stride);
    }
}

// acc = A*T_k at (row, col) becomes T_{k+1}; R_s updated (k_cheby_epilogue's operations, in order).
template <int VEC>
__device__ __forceinline__ void cheby_epi(const Epi& e, int row, int col, typename Vec<float, VEC>::type& acc,
                                          const ChebyOps<VEC>& o)
{
    typedef typename Vec<float, VEC>::type V;
    V t;
    float* rr = e.R + (int64_t)row * e.ldr + col;
    if (e.cmode == SRG_CHEBY_INIT) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) elem(t, i) = e_div(e_sub(elem(acc, i), e_mul(e.a2, elem(o.pre, i))), e.a1);
        for (int s = 0; s < e.ns; ++s) {
            V r;
#pragma unroll
            for (int i = 0; i < VEC; ++i)
                elem(r, i) = e_add(e_mul(e.cf.prev[s], elem(o.pre, i)), e_mul(e.cf.cur[s], elem(t, i)));
            vstore<float, VEC>(rr + s * e.r_stride, r, false);
        }
    } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) elem(t, i) = e_sub(elem(acc, i), elem(o.pre, i));
#pragma unroll
        for (int s = 0; s < kChebyPre; ++s) {
            if (s < e.ns) {
                V r = o.r[s];
#pragma unroll
                for (int i = 0; i < VEC; ++i) elem(r, i) = e_add(elem(r, i), e_mul(e.cf.cur[s], elem(t, i)));
                vstore<float, VEC>(rr + s * e.r_stride, r, false);
            }
        }
        for (int s = kChebyPre; s < e.ns; ++s) {
            V r = vload<float, VEC>(rr + s * e.r_stride);
#pragma unroll
            for (int i = 0; i < VEC; ++i) elem(r, i) = e_add(elem(r, i), e_mul(e.cf.cur[s], elem(t, i)));
            vstore<float, VEC>(rr + s * e.r_stride, r, false);
        }
    }
    acc = t;
}

template <int UH, bool SFULL, typename IP, int EX>
__device__ __forceinline__ void slice_wave(const IP* __restrict__ indptr,
                                           const int32_t* __restrict__ indices,
                                           const float* __restrict__ vals, int row, int slice,
                                           const float* __restrict__ X, int64_t ldx,
                                           float* __restrict__ Y, int64_t ldy, int d, int accumulate,
                                           int nt, float* __restrict__ lds, const Epi& epi)
{
    typedef typename Vec<float, 4>::type V4;
    const int lane = threadIdx.x & 63;
    const int g = lane >> 3;                 // nonzero within a group of 8
    const int qcol = slice * kSliceCols + (lane & 7) * 4;   // gather columns of this lane
    const bool gact = SFULL || qcol < d;
    const int ccol = slice * kSliceCols + lane;             // chain column of this lane
    const bool cact = lane < kSliceCols && (SFULL || ccol < d);
    float* __restrict__ yrow = Y + (int64_t)row * ldy;
    float acc = 0.0f;
    const int64_t beg = indptr[row];
    if (accumulate && cact) acc = yrow[ccol];
    const float aprev = (epi.agg && !epi.init && cact) ? epi.agg[(int64_t)row * epi.lda + ccol] : 0.0f;
    [[maybe_unused]] ChebyOps<1> cop;
    if constexpr (EX == kEpiCheby)
        if (cact) cheby_load<1>(epi, row, ccol, X, ldx, cop);
    const int64_t end = row_stop<EX>(indptr, epi, row);
    float av[UH];
    int cv[UH];
    auto load_ids = [&](int64_t j0, int* c, float* a) {   // clamped: no branches
#pragma unroll
        for (int b = 0; b < UH; ++b) {
            int64_t jj = j0 + b * 8 + g;
            jj = jj < end ? jj : end - 1;
            c[b] = indices[jj];
            a[b] = vals[jj];
        }
    };
    if (kPrefetchSliceIds && beg < end) load_ids(beg, cv, av);
    for (int64_t j = beg; j < end; j += 8 * UH) {
        V4 x[UH];
        if constexpr (!kPrefetchSliceIds) load_ids(j, cv, av);   // all index/value loads first ...
        __builtin_amdgcn_sched_barrier(0);   // keep every index load ahead of the first gather
#pragma unroll
        for (int b = 0; b < UH; ++b)     // ... then UH dependent gathers in flight
            x[b] = gact ? gload<float, 4>(X + (int64_t)cv[b] * ldx + qcol) : vzero<float, 4>();
        [[maybe_unused]] int ncv[UH];
        [[maybe_unused]] float nav[UH];
        if constexpr (kPrefetchSliceIds) {    // the next group's ids behind the gathers
            if (j + 8 * UH < end) load_ids(j + 8 * UH, ncv, nav);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int b = 0; b < UH; ++b) {
            const int64_t jb = j + b * 8;
            if (jb >= end) break;                               // wave-uniform
            const int nb = (end - jb) < 8 ? (int)(end - jb) : 8;
            float* slot = lds + (kSliceLdsBufs == 2 ? (b & 1) * 256 : 0);
            *reinterpret_cast<V4*>(slot + lane * 4) = x[b];     // tile [g][32 cols]
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            float t[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) t[q] = slot[q * kSliceCols + (lane & 31)];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const float a = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, av[b]), q * 8));
                if (q < nb && cact) acc = __builtin_fmaf(a, t[q], acc);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if constexpr (kPrefetchSliceIds) {
#pragma unroll
            for (int b = 0; b < UH; ++b) {
                cv[b] = ncv[b];
                av[b] = nav[b];
            }
        }
    }
    if (cact) {
        if constexpr (EX == kEpiCheby) cheby_epi<1>(epi, row, ccol, acc, cop);
        if (nt)
            __builtin_nontemporal_store(acc, yrow + ccol);
        else
            yrow[ccol] = acc;
        if (epi.agg) epi.agg[(int64_t)row * epi.lda + ccol] = __fadd_rn(aprev, __fmul_rn(epi.w, acc));
    }
}

// Narrow panels (d <= 32): a row wave would leave 64 - d lanes idle, so here one wave runs
// R = 64 / S rows at once, S = the power of two >= d lanes per row (lane = sub-row g, column c).
// Each lane loads its own row's (column id, value) stream -- the S lanes of a row read the same
// address, one instruction for the whole wave -- then U gathers in flight, then U fma links.
// Rows come from the degree-sorted schedule, so the R rows of a wave have similar lengths.
// Still one sequential fma chain per output element, in CSR order.
template <int S, int U, typename IP, int EX>
__device__ __forceinline__ void narrow_rows(const IP* __restrict__ indptr, const int32_t* __restrict__ indices,
                                            const float* __restrict__ vals, const int32_t* __restrict__ order,
                                            int n_rows, int first, const float* __restrict__ X, int64_t ldx,
                                            float* __restrict__ Y, int64_t ldy, int d, int accumulate, int nt,
                                            const Epi& epi)
{
    const int lane = threadIdx.x & 63;
    const int g = lane / S, c = lane % S;
    const int slot = first + g;
    const bool rv = slot < n_rows;
    const int row = rv ? (order ? order[slot] : slot) : 0;
    const bool act = rv && c < d;
    const int64_t beg = rv ? (int64_t)indptr[row] : 0;
    const int len = rv ? (int)(row_stop<EX>(indptr, epi, row) - beg) : 0;
    int maxlen = len;
#pragma unroll
    for (int off = S; off < 64; off <<= 1) {
        const int o = __shfl_xor(maxlen, off);
        maxlen = o > maxlen ? o : maxlen;
    }
    maxlen = __builtin_amdgcn_readfirstlane(maxlen);
    float* __restrict__ yrow = Y + (int64_t)row * ldy;
    float acc = (accumulate && act) ? yrow[c] : 0.0f;
    const float aprev = (epi.agg && !epi.init && act) ? epi.agg[(int64_t)row * epi.lda + c] : 0.0f;
    [[maybe_unused]] ChebyOps<1> cop;
    if constexpr (EX == kEpiCheby)
        if (act) cheby_load<1>(epi, row, c, X, ldx, cop);
    for (int j = 0; j < maxlen; j += U) {
        int cv[U];
        float av[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool ok = j + u < len;
            const int64_t p = beg + (ok ? j + u : 0);
            cv[u] = ok ? indices[p] : 0;
            av[u] = ok ? vals[p] : 0.0f;
        }
        __builtin_amdgcn_sched_barrier(0);   // every id load ahead of the first gather
        float x[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            x[u] = (act && j + u < len) ? X[(int64_t)cv[u] * ldx + c] : 0.0f;
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (act && j + u < len) acc = __builtin_fmaf(av[u], x[u], acc);
    }
    if (act) {
        if constexpr (EX == kEpiCheby) cheby_epi<1>(epi, row, c, acc, cop);
        if (nt)
            __builtin_nontemporal_store(acc, yrow + c);
        else
            yrow[c] = acc;
        if (epi.agg) epi.agg[(int64_t)row * epi.lda + c] = __fadd_rn(aprev, __fmul_rn(epi.w, acc));
    }
}

// Light rows of wide panels (d = LQ * 4 * S, S = 64 / LR): one wave runs LR rows at once, S lanes
// per row, each lane LQ 16-byte column chunks (chunk q of lane l: columns q*4S + 4l .. +3, so the S
// lanes of a row read 16*S contiguous bytes per gather).  A one-row wave walks its row's short
// stream through a chain of dependent loads (schedule slot -> row pointers -> column ids -> X) and
// the phase is bound by how many rows are in flight, not by bytes; LR rows per wave multiply that.
// The S lanes of a row load S consecutive (column id, value) entries of it at once and hand them
// out by ds_bpermute, U gathers per row in flight, then the fma links in CSR order.  Entries past a
// row's end are skipped (never folded in as 0*x).  Still one sequential fma chain per output element.
template <int LR, int LQ, int U, typename IP, int EX>
__device__ __forceinline__ void packed_rows(const IP* __restrict__ indptr, const int32_t* __restrict__ indices,
                                            const float* __restrict__ vals, const int32_t* __restrict__ order,
                                            int n_rows, int first, const float* __restrict__ X, int64_t ldx,
                                            float* __restrict__ Y, int64_t ldy, int accumulate, int nt,
                                            const Epi& epi)
{
    typedef typename Vec<float, 4>::type V4;
    constexpr int S = 64 / LR;
    static_assert(S % U == 0, "a row's id chunk holds whole groups of U entries");
    const int lane = threadIdx.x & 63;
    const int g = lane / S, l = lane % S;
    const int slot = first + g;
    const bool rv = slot < n_rows;
    const int row = rv ? (order ? order[slot] : slot) : 0;
    int64_t beg = 0;
    int len = 0;
    if (rv) {
        if constexpr (kIsSpan<EX>) {
            if (epi.slot_beg) {
                beg = epi.slot_beg[slot];
                len = (int)(epi.slot_end[slot] - beg);
            } else {
                beg = indptr[row];
                len = (int)(epi.row_end[row] - beg);
            }
        } else {
            beg = indptr[row];
            len = (int)(row_stop<EX>(indptr, epi, row) - beg);
        }
    }
    int maxlen = len;
#pragma unroll
    for (int off = S; off < 64; off <<= 1) {
        const int o = __shfl_xor(maxlen, off);
        maxlen = o > maxlen ? o : maxlen;
    }
    maxlen = __builtin_amdgcn_readfirstlane(maxlen);
    float* __restrict__ yrow = Y + (int64_t)row * ldy;
    // the Chebyshev epilogue never aggregates nor accumulates (its entry rejects both): dropping
    // them statically keeps its registers (the prefetched operands) within 5 waves per SIMD
    float* __restrict__ arow = (EX != kEpiCheby && epi.agg) ? epi.agg + (int64_t)row * epi.lda : nullptr;
    V4 acc[LQ], aprev[LQ];
    [[maybe_unused]] ChebyOps<4> cop[LQ];
#pragma unroll
    for (int q = 0; q < LQ; ++q) {
        const int col = q * 4 * S + 4 * l;
        acc[q] = (EX != kEpiCheby && accumulate && rv) ? vload<float, 4>(yrow + col) : vzero<float, 4>();
        aprev[q] = (arow && !epi.init && rv) ? vload<float, 4>(arow + col) : vzero<float, 4>();
        if constexpr (EX == kEpiCheby)
            if (rv) cheby_load<4>(epi, row, col, X, ldx, cop[q]);
    }
    // The row's entries S at a time: lane l of the row loads the (column id, value) of entry j0 + l, and
    // each group of U gathers takes its ids from the row's S lanes by ds_bpermute, so the dependent
    // chain per U entries is the gather alone (one id load per S entries instead of one per U); the
    // next S entries' ids load behind the current chunk's gathers.  Products 5.52 -> 5.33 ms per hop,
    // arxiv 0.157 -> 0.154 (round 5, profiles/r05ab_shfl_ids_ab.txt; before, every U entries began
    // with their id loads).  Entries past a row's end load nothing and are skipped.
    const int base = g * S;
    auto load_ids = [&](int j0, int& c, float& a) {
        const bool ok = j0 + l < len;
        const int64_t p = beg + (ok ? j0 + l : 0);
        c = ok ? indices[p] : 0;
        a = ok ? vals[p] : 0.0f;
    };
    if constexpr (U <= 2) {
    // U = 2 (the column blocks' launches): two chunks of ids (A: entries [ca, ca + S), B: the next S)
    // and two gather buffers, so step j + U's gathers are issued before step j's fma links -- 2U
    // gathers in flight across the steps.  Products 5.33 -> 5.27 ms per hop; with U = 4 (the one-launch
    // hop) the same pipeline costs arxiv 6 % (0.154 -> 0.163 ms: 8 gathers in flight per row, like
    // U = 8), so that keeps one U-group in flight (profiles/r05af_pipe_gathers_ab.txt)
    int ida = 0, idb = 0;
    float vaa = 0.0f, vab = 0.0f;
    int ca = 0;
    if (maxlen > 0) load_ids(0, ida, vaa);
    if (S < maxlen) load_ids(S, idb, vab);
    auto issue = [&](int j, V4 (&x)[U][LQ], float (&av)[U]) {
        const bool in_a = j < ca + S;            // wave-uniform
        const int off = base + (j & (S - 1));
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = __shfl(in_a ? ida : idb, off + u);
            av[u] = __shfl(in_a ? vaa : vab, off + u);
#pragma unroll
            for (int q = 0; q < LQ; ++q)
                x[u][q] = (j + u < len) ? gload<float, 4>(X + (int64_t)c * ldx + q * 4 * S + 4 * l) : vzero<float, 4>();
        }
    };
    auto links = [&](int j, const V4 (&x)[U][LQ], const float (&av)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (j + u < len)
#pragma unroll
                for (int q = 0; q < LQ; ++q) chain<float, 4>(acc[q], av[u], x[u][q]);
        if (j + U == ca + S) {                   // chunk A done: B becomes A, B loads the next S
            ida = idb;
            vaa = vab;
            ca += S;
            if (ca + S < maxlen) load_ids(ca + S, idb, vab);
        }
    };
    V4 xa[U][LQ], xb[U][LQ];
    float fa[U], fb[U];
    if (maxlen > 0) issue(0, xa, fa);
    for (int j = 0; j < maxlen; j += 2 * U) {
        if (j + U < maxlen) issue(j + U, xb, fb);
        links(j, xa, fa);
        if (j + U >= maxlen) break;
        if (j + 2 * U < maxlen) issue(j + 2 * U, xa, fa);
        links(j + U, xb, fb);
    }
    } else {
    int nid = 0;
    float nva = 0.0f;
    if (maxlen > 0) load_ids(0, nid, nva);
    for (int j0 = 0; j0 < maxlen; j0 += S) {
        const int cid = nid;
        const float cva = nva;
        if (j0 + S < maxlen) load_ids(j0 + S, nid, nva);
        const int nstep = (maxlen - j0) < S ? (maxlen - j0) : S;   // wave-uniform; S is a multiple of U
        for (int jj = 0; jj < nstep; jj += U) {
            int cv[U];
            float av[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                cv[u] = __shfl(cid, base + jj + u);
                av[u] = __shfl(cva, base + jj + u);
            }
            const int j = j0 + jj;
            V4 x[U][LQ];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int q = 0; q < LQ; ++q)
                    x[u][q] = (j + u < len) ? gload<float, 4>(X + (int64_t)cv[u] * ldx + q * 4 * S + 4 * l)
                                            : vzero<float, 4>();
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (j + u < len)
#pragma unroll
                    for (int q = 0; q < LQ; ++q) chain<float, 4>(acc[q], av[u], x[u][q]);
        }
    }
    }
    if (!rv) return;
#pragma unroll
    for (int q = 0; q < LQ; ++q) {
        const int col = q * 4 * S + 4 * l;
        if constexpr (EX == kEpiCheby) cheby_epi<4>(epi, row, col, acc[q], cop[q]);
        vstore<float, 4>(yrow + col, acc[q], nt != 0);
        if (arow) {
#pragma unroll
            for (int i = 0; i < 4; ++i) aprev[q][i] = __fadd_rn(aprev[q][i], __fmul_rn(epi.w, acc[q][i]));
            vstore<float, 4>(arow + col, aprev[q], false);
        }
    }
}

template <int VEC, int U, int UH, bool FULL, bool SFULL, typename IP, int NS = 0, int EX = kEpiPlain, int LR = 0, int LQ = 1,
          bool XH = false>
__global__ void __launch_bounds__(kBlock)
k_spmm(const IP* __restrict__ indptr, const int32_t* __restrict__ indices,
       const float* __restrict__ vals, const int32_t* __restrict__ order, int n_rows, int n_heavy,
       int n_slices, int nb_heavy, const float* __restrict__ X, int64_t ldx, float* __restrict__ Y,
       int64_t ldy, int d, int accumulate, int nt, int block_base, Epi epi)
{
    typedef typename Vec<float, VEC>::type V;
    const int bid = block_base + (int)blockIdx.x;
    // dynamic: at least kSpmmLdsBytes, more when the launch caps its blocks per CU (spmm_lds_bytes)
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int lane = threadIdx.x & 63;
    const int wib = threadIdx.x >> 6;
    if (bid < nb_heavy) {
        if constexpr (XH) {
            // XCD-aware slice waves: blocks are dealt round-robin over the 8 XCDs (b and b + 8 share
            // one), so block b takes slice (b % 8) % n_slices of 4 rows: an XCD's L2 then holds one
            // slice of the X rows these waves gather.  Groups of 8 blocks cover 8 / n_slices row
            // groups x every slice.
            const int per = 8 / n_slices, x = bid & 7;
            const int item = __builtin_amdgcn_readfirstlane(((bid >> 3) * per + x / n_slices) * kWavesPerBlock + wib);
            if (item >= n_heavy) return;
            slice_wave<UH, SFULL, IP, EX>(indptr, indices, vals, order[item], x % n_slices, X, ldx, Y, ldy, d,
                                            accumulate, nt, lds + wib * kSliceLdsBufs * 256, epi);
            return;
        }
        const int item = __builtin_amdgcn_readfirstlane(bid * kWavesPerBlock + wib);
        if (item >= n_heavy * n_slices) return;
        const int row = order[item / n_slices];
        slice_wave<UH, SFULL, IP, EX>(indptr, indices, vals, row, item % n_slices, X, ldx, Y, ldy, d,
                           accumulate, nt, lds + wib * kSliceLdsBufs * 256, epi);
        return;
    }
    if constexpr (LR > 0) {   // wide panel: LR light rows per wave
        const int first = __builtin_amdgcn_readfirstlane((bid - nb_heavy) * kWavesPerBlock + wib) * LR + n_heavy;
        if (first >= n_rows) return;
        packed_rows<LR, LQ, U, IP, EX>(indptr, indices, vals, order, n_rows, first, X, ldx, Y, ldy, accumulate, nt, epi);
        return;
    }
    if constexpr (NS > 0) {   // narrow panel: 64 / NS light rows per wave
        const int first = __builtin_amdgcn_readfirstlane((bid - nb_heavy) * kWavesPerBlock + wib) * (64 / NS) + n_heavy;
        if (first >= n_rows) return;
        narrow_rows<NS, U, IP, EX>(indptr, indices, vals, order, n_rows, first, X, ldx, Y, ldy, d, accumulate, nt, epi);
        return;
    }
    const int w = __builtin_amdgcn_readfirstlane((bid - nb_heavy) * kWavesPerBlock + wib) + n_heavy;
    if (w >= n_rows) return;
    const int row = order ? order[w] : w;
    float* __restrict__ yrow = Y + (int64_t)row * ldy;
    for (int c0 = 0; c0 < d; c0 += 64 * VEC) {
        const int col = c0 + lane * VEC;
        const bool act = col < d;
        V acc = vzero<float, VEC>();
        if (EX != kEpiCheby && accumulate && (FULL || act)) acc = vload<float, VEC>(yrow + col);
        // the accumulator row is loaded before the chain, so its latency hides under the gathers
        V aprev = vzero<float, VEC>();
        float* arow = (EX != kEpiCheby && epi.agg) ? epi.agg + (int64_t)row * epi.lda : nullptr;
        if (arow && !epi.init && (FULL || act)) aprev = vload<float, VEC>(arow + col);
        [[maybe_unused]] ChebyOps<VEC> cop;
        if constexpr (EX == kEpiCheby)
            if (FULL || act) cheby_load<VEC>(epi, row, col, X, ldx, cop);
        row_gather<float, VEC, U, FULL, IP, kIsSpan<EX>>(acc, indptr, indices, vals, row, X, ldx, col, act,
                                                            epi.row_end);
        if (FULL || act) {
            if constexpr (EX == kEpiCheby) cheby_epi<VEC>(epi, row, col, acc, cop);
            vstore<float, VEC>(yrow + col, acc, nt != 0);
            if (arow) {
#pragma unroll
                for (int i = 0; i < VEC; ++i) elem(aprev, i) = __fadd_rn(elem(aprev, i), __fmul_rn(epi.w, elem(acc, i)));
                vstore<float, VEC>(arow + col, aprev, false);
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------
// hub rows: one workgroup per (row, 32-column slice), producer/consumer through LDS
//
// A slice wave keeps 8 KiB of gathers in flight, so a row of degree D costs ~D/64 load latencies
// (~6 ms for the 155,868-entry hub of the products-shaped graph): hidden at 1 GPU, the whole hop
// at 8.  Here the row's chain is fed from LDS by 8 producer waves:
//   * windows of kHubW = 512 nonzeros, double-buffered tiles: while the consumer runs window h
//     from one tile, the producers write window h+1 into the other (one barrier per window);
//   * each producer lane gathers W / 64 = 8 dwordx4 (8 nonzeros' 128-byte slices per wave
//     instruction) per window into one of two register sets, so a window's gathers are issued
//     two windows before they are written (~2 us of latency cover); the column ids / values of
//     the next window are loaded one window ahead;
//   * the tile is transposed, [32 columns][W + 16] with the 4-nonzero group index XOR-swizzled
//     per column group (conflict-free ds_write_b32 and ds_read_b128, see HubGeom);
//   * the consumer wave (lanes 0..31, one column each) runs the 32 chains, 4 links per
//     ds_read_b128, with a ring of three 16-link register sets so every LDS read is issued two
//     sets (~32 links) before its fmas.
// Still exactly one fma chain per output element, in CSR order.
// ------------------------------------------------------------------------------------------------
constexpr int kHubProducers = 8;
constexpr int kHubW = 512;                                   // nonzeros per window (the default)
constexpr int kHubThreads = 64 * (kHubProducers + 1);
// Window geometry for W nonzeros per window.  W = 512 (139 KB of LDS, one workgroup per CU) is the
// lowest-latency chain, for a few hub rows beside a big launch (one GPU).  W = 256 (72 KB) lets two
// workgroups share a CU, for launches with more hub workgroups than CUs (the halo exchange's hub
// group: hundreds of rows per rank), where the CUs' LDS, not one chain's latency, sets the time.
// Floats per tile column: W + 16 == 16 (mod 64).  With the 4-link group index XOR-ed by (c >> 2) & 7,
// both the producers' transposed ds_write_b32 (lanes: 4 nonzeros x 8 column chunks) and the
// consumer's ds_read_b128 (lanes: 32 columns, 16-lane groups) are bank-conflict-free (exhaustive
// check over all window offsets; the 4 (mod 64) stride of the first version made the reads 2-way)
template <int W, int NP = kHubProducers>
struct HubGeom {
    static constexpr int UW = W / (NP * 8);                  // gathers per producer lane per window
    static constexpr int LD = W + 16;
    static constexpr int TILE = kSliceCols * LD;             // floats per tile
    static constexpr size_t LDS_BYTES = (size_t)(2 * TILE + 2 * W) * sizeof(float);
};
constexpr int kHubWideLaunch = 256;   // more hub workgroups than this (the CU count) -> W = kHubWideW
constexpr int kHubWideW = 256;
__device__ __forceinline__ int hub_swz(int c) { return (c >> 2) & 7; }
// Full windows take their link values by DPP quad broadcast (hub_links16; the value-read-per-4-links
// loop it replaced in round 3 was removed in round 5)
constexpr int kHubDppL = 3;   // 16-link sets in flight (4 tile reads + 1 value read each)

// 16 links of one column chain: link 4i + j multiplies x = t[i][j] by the value that quad lane i
// holds in a[j] (quad_perm broadcast), acc = fma(value, x, acc) -- v_fmac_f32 with a DPP first
// operand, one instruction per link.  One asm block: the compiler's hazard pass would otherwise pad
// every link with an s_nop (it treats the chained accumulator like a DPP source; 0.95 vs 0.86 ms on
// the products hub row).  The DPP'd operands a[] normally come straight from LDS reads, but nothing
// stops the register allocator from producing one with a VALU copy (v_mov / v_accvgpr_read) right
// before the block, and gfx9 needs 2 wait states between a VALU write of a VGPR and a DPP read of
// it: the hazard pass cannot see inside the asm, so the block opens with its own `s_nop 1`.  This
// guard must stay (2 cycles per 16 links).
__device__ __forceinline__ void hub_links16(float& acc, const typename Vec<float, 4>::type& a,
                                            const typename Vec<float, 4>::type (&t)[4])
{
#define SRG_QP(I) " quad_perm:[" #I "," #I "," #I "," #I "] row_mask:0xf bank_mask:0xf\n"
    asm volatile(
        "s_nop 1\n"
        "v_fmac_f32_dpp %0, %1, %5" SRG_QP(0) "v_fmac_f32_dpp %0, %2, %6" SRG_QP(0)
        "v_fmac_f32_dpp %0, %3, %7" SRG_QP(0) "v_fmac_f32_dpp %0, %4, %8" SRG_QP(0)
        "v_fmac_f32_dpp %0, %1, %9" SRG_QP(1) "v_fmac_f32_dpp %0, %2, %10" SRG_QP(1)
        "v_fmac_f32_dpp %0, %3, %11" SRG_QP(1) "v_fmac_f32_dpp %0, %4, %12" SRG_QP(1)
        "v_fmac_f32_dpp %0, %1, %13" SRG_QP(2) "v_fmac_f32_dpp %0, %2, %14" SRG_QP(2)
        "v_fmac_f32_dpp %0, %3, %15" SRG_QP(2) "v_fmac_f32_dpp %0, %4, %16" SRG_QP(2)
        "v_fmac_f32_dpp %0, %1, %17" SRG_QP(3) "v_fmac_f32_dpp %0, %2, %18" SRG_QP(3)
        "v_fmac_f32_dpp %0, %3, %19" SRG_QP(3) "v_fmac_f32_dpp %0, %4, %20" SRG_QP(3)
        : "+v"(acc)
        : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]),
          "v"(t[0][0]), "v"(t[0][1]), "v"(t[0][2]), "v"(t[0][3]), "v"(t[1][0]), "v"(t[1][1]), "v"(t[1][2]), "v"(t[1][3]),
          "v"(t[2][0]), "v"(t[2][1]), "v"(t[2][2]), "v"(t[2][3]), "v"(t[3][0]), "v"(t[3][1]), "v"(t[3][2]), "v"(t[3][3]));
#undef SRG_QP
}

// kHubProducers producer waves + the consumer (the round-1 ablations and the round-4 4-producer
// "lite" workgroup were removed in round 5: DESIGN.md §5.1, §7)
template <bool SFULL, typename IP, int EX = kEpiPlain, int W = kHubW>
__global__ void __launch_bounds__(kHubThreads)
k_spmm_hub(const IP* __restrict__ indptr, const int32_t* __restrict__ indices,
           const float* __restrict__ vals, const int32_t* __restrict__ hub_rows, int n_slices,
           const float* __restrict__ X, int64_t ldx, float* __restrict__ Y, int64_t ldy, int d,
           int accumulate, int nt, Epi epi)
{
    typedef typename Vec<float, 4>::type V4;
    extern __shared__ __attribute__((aligned(16))) float hub_lds[];
    // [2 tiles][32 columns][HubGeom<W>::LD] then [2][W] values
    float* aval_base = hub_lds + 2 * HubGeom<W>::TILE;
    const int item = blockIdx.x;
    const int row = hub_rows[item / n_slices];
    const int slice = item % n_slices;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const int64_t beg = indptr[row];
    const int64_t end = row_stop<EX>(indptr, epi, row);
    const int n_win = (int)((end - beg + W - 1) / W);

    if (wave == 0) {   // ---------------- consumer: 32 column chains ----------------
        const int c = lane & 31;
        const int ccol = slice * kSliceCols + c;
        const bool cact = lane < kSliceCols && (SFULL || ccol < d);
        float* __restrict__ yrow = Y + (int64_t)row * ldy;
        float acc = 0.0f;
        if (accumulate && cact) acc = yrow[ccol];
        const float aprev = (epi.agg && !epi.init && cact) ? epi.agg[(int64_t)row * epi.lda + ccol] : 0.0f;
        [[maybe_unused]] ChebyOps<1> cop;
        if constexpr (EX == kEpiCheby)
            if (cact) cheby_load<1>(epi, row, ccol, X, ldx, cop);
        const int sw = hub_swz(c);
        constexpr int G = 2;                      // groups of 4 links per register set (8 links)
        V4 tA[G], aA[G], tB[G], aB[G], tC[G], aC[G], tD[G], aD[G];
        for (int h = 0; h < n_win; ++h) {
            __syncthreads();                      // window h is in tile h & 1
            if (lane < kSliceCols) {
                const float* tcol = hub_lds + (h & 1) * HubGeom<W>::TILE + c * HubGeom<W>::LD;
                const float* av = aval_base + (h & 1) * W;
                const int64_t sb = beg + (int64_t)h * W;
                const int nb = (end - sb) < W ? (int)(end - sb) : W;
                const int nc = nb / (4 * G);      // full 8-link sets
                auto ld = [&](int set, V4 (&t)[G], V4 (&a)[G]) {
#pragma unroll
                    for (int i = 0; i < G; ++i) {
                        const int grp = set * G + i;
                        t[i] = *reinterpret_cast<const V4*>(tcol + ((grp ^ sw) << 2));
                        a[i] = *reinterpret_cast<const V4*>(av + (grp << 2));   // broadcast
                    }
                };
                auto run = [&](const V4 (&t)[G], const V4 (&a)[G]) {
#pragma unroll
                    for (int i = 0; i < G; ++i) {
                        acc = __builtin_fmaf(a[i][0], t[i][0], acc);
                        acc = __builtin_fmaf(a[i][1], t[i][1], acc);
                        acc = __builtin_fmaf(a[i][2], t[i][2], acc);
                        acc = __builtin_fmaf(a[i][3], t[i][3], acc);
                    }
                };
                if (nb == W) {
                    // full window, values by DPP: per 16 links one ds_read_b128 of values (lane l
                    // reads values 16k + 4 (l & 3) .. +3, so register j of quad lane i holds value
                    // 16k + 4i + j) and four tile reads (4 links each); link 4i + j is
                    //   v_fmac_f32_dpp acc, a[j], t_i[j] quad_perm:[i,i,i,i]
                    // (the quad broadcast of lane i's a[j] as the fma's first operand: the same
                    // fused multiply-add as v_fma_f32, so the chain keeps its bits).  The value
                    // reads drop from one per 4 links to one per 16.  Ring: kHubDppL 16-link sets
                    // in flight (5 LDS reads each, 5 * kHubDppL <= 15 = lgkmcnt's range).
                    constexpr int NK = W / 16;
                    const float* tb[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) tb[k] = hub_lds + (h & 1) * HubGeom<W>::TILE + c * HubGeom<W>::LD + ((k ^ sw) << 2);
                    const float* avl = av + 4 * (lane & 3);
                    auto rt = [&](int grp) { return *reinterpret_cast<const V4*>(tb[grp & 7] + (grp >> 3) * 32); };
                    auto rv = [&](int k) { return *reinterpret_cast<const V4*>(avl + 16 * k); };
                    V4 t[kHubDppL][4], a[kHubDppL];
#pragma unroll
                    for (int r = 0; r < kHubDppL; ++r) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) t[r][i] = rt(4 * r + i);
                        a[r] = rv(r);
                    }
#pragma unroll
                    for (int k0 = 0; k0 < NK; k0 += kHubDppL) {
#pragma unroll
                        for (int r = 0; r < kHubDppL; ++r) {
                            const int k = k0 + r;
                            if (k < NK) {
                                hub_links16(acc, a[r], t[r]);
                                if (k + kHubDppL < NK) {
#pragma unroll
                                    for (int i = 0; i < 4; ++i) t[r][i] = rt(4 * (k + kHubDppL) + i);
                                    a[r] = rv(k + kHubDppL);
                                }
                                __builtin_amdgcn_sched_barrier(0);
                            }
                        }
                    }
                    continue;
                }
                // unconditional: sets past nc read stale tile / value words, never used (and the
                // waitcnt pass then sees one issue order on every path into the loop)
                ld(0, tA, aA);
                __builtin_amdgcn_sched_barrier(0);
                ld(1, tB, aB);
                __builtin_amdgcn_sched_barrier(0);
                ld(2, tC, aC);
                __builtin_amdgcn_sched_barrier(0);
                int k = 0;
                // ring of four 8-link sets: every read is issued three sets (24 links) before its
                // fmas, with at most 12 LDS reads outstanding (lgkmcnt counts 15).  The loop's
                // loads are unconditional (k + 6 < nc) and the scheduling barriers keep the ring's
                // order; the last <= 6 sets run after it.
                for (; k + 7 <= nc; k += 4) {
                    ld(k + 3, tD, aD);
                    __builtin_amdgcn_sched_barrier(0);
                    run(tA, aA);
                    __builtin_amdgcn_sched_barrier(0);
                    ld(k + 4, tA, aA);
                    __builtin_amdgcn_sched_barrier(0);
                    run(tB, aB);
                    __builtin_amdgcn_sched_barrier(0);
                    ld(k + 5, tB, aB);
                    __builtin_amdgcn_sched_barrier(0);
                    run(tC, aC);
                    __builtin_amdgcn_sched_barrier(0);
                    ld(k + 6, tC, aC);
                    __builtin_amdgcn_sched_barrier(0);
                    run(tD, aD);
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (k < nc) run(tA, aA);
                if (k + 1 < nc) run(tB, aB);
                if (k + 2 < nc) run(tC, aC);
                for (int j = k + 3; j < nc; ++j) {
                    ld(j, tD, aD);
                    run(tD, aD);
                }
                for (int q = nc * 4 * G; q < nb; ++q)
                    acc = __builtin_fmaf(av[q], tcol[(((q >> 2) ^ sw) << 2) + (q & 3)], acc);
            }
        }
        if (cact) {
            if constexpr (EX == kEpiCheby) cheby_epi<1>(epi, row, ccol, acc, cop);
            if (nt)
                __builtin_nontemporal_store(acc, yrow + ccol);
            else
                yrow[ccol] = acc;
            if (epi.agg) epi.agg[(int64_t)row * epi.lda + ccol] = __fadd_rn(aprev, __fmul_rn(epi.w, acc));
            }
        return;
    }

    // ---------------- producers ----------------
    const int p = wave - 1;
    const int g = lane >> 3;          // nonzero within a gather's group of 8
    const int qq = lane & 7;          // 16-byte chunk = columns qq*4 .. qq*4+3 of the slice
    const int qcol = slice * kSliceCols + qq * 4;
    const bool gact = SFULL || qcol < d;
    V4 x0[HubGeom<W>::UW], x1[HubGeom<W>::UW];        // gathered windows, two register sets (even / odd windows)
    float a0[HubGeom<W>::UW], a1[HubGeom<W>::UW];
    int cn[HubGeom<W>::UW];                   // column ids / values of the next window to gather
    float an[HubGeom<W>::UW];
    auto load_ids = [&](int w) {
        const int64_t sb = beg + (int64_t)w * W;
#pragma unroll
        for (int b = 0; b < HubGeom<W>::UW; ++b) {
            int64_t jj = sb + (p * HubGeom<W>::UW + b) * 8 + g;
            jj = jj < end ? jj : end - 1;
            cn[b] = indices[jj];
            an[b] = vals[jj];
        }
    };
    auto gather = [&](V4 (&x)[HubGeom<W>::UW], float (&a)[HubGeom<W>::UW]) {
#pragma unroll
        for (int b = 0; b < HubGeom<W>::UW; ++b) {
            x[b] = gact ? gload<float, 4>(X + (int64_t)cn[b] * ldx + qcol) : vzero<float, 4>();
            a[b] = an[b];
        }
    };
    auto put = [&](int w, const V4 (&x)[HubGeom<W>::UW], const float (&a)[HubGeom<W>::UW]) {
        float* tile = hub_lds + (w & 1) * HubGeom<W>::TILE;
        float* av = aval_base + (w & 1) * W;
#pragma unroll
        for (int b = 0; b < HubGeom<W>::UW; ++b) {
            const int nl = (p * HubGeom<W>::UW + b) * 8 + g;   // nonzero within the window
#pragma unroll
            for (int i = 0; i < 4; ++i) {             // transposed, swizzled: conflict-free
                const int cc = qq * 4 + i;
                tile[cc * HubGeom<W>::LD + ((((nl >> 2) ^ hub_swz(cc)) << 2) | (nl & 3))] = x[b][i];
            }
            if (qq == 0) av[nl] = a[b];
        }
    };
    // prologue: windows 0 and 1 in flight, window 0 published, window 2 in flight
    if (n_win > 0) {
        load_ids(0);
        __builtin_amdgcn_sched_barrier(0);
        gather(x0, a0);
        if (n_win > 1) { load_ids(1); gather(x1, a1); }
        if (n_win > 2) load_ids(2);
        put(0, x0, a0);
        if (n_win > 2) { gather(x0, a0); if (n_win > 3) load_ids(3); }
    }
    __syncthreads();                              // window 0 published
    for (int h = 0; h + 1 < n_win; h += 2) {
        // window h+1 (odd, set 1) -> tile 1 while the consumer runs window h; then gather h+3
        put(h + 1, x1, a1);
        if (h + 3 < n_win) { gather(x1, a1); if (h + 4 < n_win) load_ids(h + 4); }
        __syncthreads();
        if (h + 2 >= n_win) break;
        // window h+2 (even, set 0) -> tile 0 while the consumer runs window h+1; then gather h+4
        put(h + 2, x0, a0);
        if (h + 4 < n_win) { gather(x0, a0); if (h + 5 < n_win) load_ids(h + 5); }
        __syncthreads();
    }
    // barrier count: 1 (prologue) + (n_win - 1) in the loop == the consumer's n_win
}

constexpr size_t kHubLdsBytes = HubGeom<kHubW>::LDS_BYTES;

// ------------------------------------------------------------------------------------------------
// Chebyshev step with fused epilogue (wavelet basis)
// ------------------------------------------------------------------------------------------------
// The fused step's epilogue at VEC consecutive elements of row-offset `off`: acc = (A Tc) there becomes
// T_{k+1}, every scale's output updated -- k_cheby_epilogue's modes and operations:
//   INIT:       Tn = (acc - a2 Tc) / a1;  R_s = (c0_s/2) Tc + c1_s Tn
//   INIT_T:     Tn = (acc - a2 Tc) / a1   (R formed by the first step)
//   STEP_FIRST: Tn = acc - To (To = T0, Tc = T1);  R_s = ((c0_s/2) T0 + c1_s T1) + c2_s Tn
//   STEP:       Tn = acc - To;  R_s += ck_s Tn
// with SRG_CHEBY_NO_T leaving Tn unstored (the last order).  The lean sequence INIT_T, STEP_FIRST, ...,
// STEP | NO_T forms every R with the same operations in the same order as INIT, STEP, ..., STEP: the
// same bits with four panel passes less per order-3 filter.
template <typename T, int VEC>
__device__ __forceinline__ void cheby_epi_at(int mode, const typename Vec<T, VEC>::type& acc, const T* __restrict__ Tc,
                                             const T* __restrict__ To, T* __restrict__ Tn, T* __restrict__ R,
                                             int64_t off, int64_t r_stride, T a1, T a2, const ChebyCoef<T>& cf,
                                             int n_scales)
{
    typedef typename Vec<T, VEC>::type V;
    const int m = mode & 0xf;
    V tn;
    if (m == SRG_CHEBY_INIT || m == SRG_CHEBY_INIT_T) {
        const V tc = vload<T, VEC>(Tc + off);
#pragma unroll
        for (int i = 0; i < VEC; ++i) elem(tn, i) = e_div(e_sub(elem(acc, i), e_mul(a2, elem(tc, i))), a1);
        if (m == SRG_CHEBY_INIT)
            for (int s = 0; s < n_scales; ++s) {
                V r;
#pragma unroll
                for (int i = 0; i < VEC; ++i)
                    elem(r, i) = e_add(e_mul(cf.prev[s], elem(tc, i)), e_mul(cf.cur[s], elem(tn, i)));
                vstore<T, VEC>(R + s * r_stride + off, r, false);
            }
    } else if (m == SRG_CHEBY_STEP_FIRST) {
        const V t0 = vload<T, VEC>(To + off), t1 = vload<T, VEC>(Tc + off);
#pragma unroll
        for (int i = 0; i < VEC; ++i) elem(tn, i) = e_sub(elem(acc, i), elem(t0, i));
        for (int s = 0; s < n_scales; ++s) {
            V r;
#pragma unroll
            for (int i = 0; i < VEC; ++i)
                elem(r, i) = e_add(e_add(e_mul(cf.prev[s], elem(t0, i)), e_mul(cf.mid[s], elem(t1, i))),
                                   e_mul(cf.cur[s], elem(tn, i)));
            vstore<T, VEC>(R + s * r_stride + off, r, false);
        }
    } else {
        const V to = vload<T, VEC>(To + off);
#pragma unroll
        for (int i = 0; i < VEC; ++i) elem(tn, i) = e_sub(elem(acc, i), elem(to, i));
        for (int s = 0; s < n_scales; ++s) {
            T* rp = R + s * r_stride + off;
            V r = vload<T, VEC>(rp);
#pragma unroll
            for (int i = 0; i < VEC; ++i) elem(r, i) = e_add(elem(r, i), e_mul(cf.cur[s], elem(tn, i)));
            vstore<T, VEC>(rp, r, false);
        }
    }
    if (!(mode & SRG_CHEBY_NO_T)) vstore<T, VEC>(Tn + off, tn, false);
}

template <typename T, int VEC, int U>
__global__ void __launch_bounds__(kBlock)
k_cheby(const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
        const T* __restrict__ vals, const int32_t* __restrict__ order, int n_rows,
        const T* __restrict__ Tc, const T* __restrict__ To, T* __restrict__ Tn, int64_t ld, int d,
        int mode, T a1, T a2, ChebyCoef<T> cf, int n_scales, T* __restrict__ R, int64_t r_stride,
        int block_base)
{
    typedef typename Vec<T, VEC>::type V;
    const int w = wave_slot(block_base);
    if (w >= n_rows) return;
    const int row = order ? order[w] : w;
    const int lane = threadIdx.x & 63;
    const int64_t roff = (int64_t)row * ld;
    for (int c0 = 0; c0 < d; c0 += 64 * VEC) {
        const int col = c0 + lane * VEC;
        const bool act = col < d;
        V acc = vzero<T, VEC>();
        row_gather<T, VEC, U, false, int64_t>(acc, indptr, indices, vals, row, Tc, ld, col, act);
        if (!act) continue;
        cheby_epi_at<T, VEC>(mode, acc, Tc, To, Tn, R, roff + col, r_stride, a1, a2, cf, n_scales);
    }
}

// ------------------------------------------------------------------------------------------------
// fp64 Chebyshev step, hub rows: one workgroup per (hub row, 16-column slice)
//
// A row wave keeps U gathers of its row in flight, so a row of degree D costs ~D/U load latencies:
// in fp64 the products top row (155,868 entries) is one wave's chain beside the whole step.  As in
// k_spmm_hub, kHub64Producers waves gather windows of W entries into LDS (two tiles, one
// barrier per window; each window's gathers are issued two windows ahead) and one consumer wave
// runs the slice's 16 column chains out of LDS: link k of column c is acc = acc + a_k * x_k[c], the
// product and the sum rounded separately (scipy's csr_matvecs order, as row_gather), then k_cheby's
// epilogue for the row's 16 columns -- the same operations, so the same bits.
//   * producer lane (g, q) gathers the 16-byte chunk q (columns 2q, 2q + 1 of the slice) of entry g
//     of a group of 8: one dwordx4 instruction brings 8 entries' 128-byte slices;
//   * the tile is column-major, [16 columns][W + 4]: the consumer's lane c reads links k, k + 1
//     of its column with one ds_read_b128, their values with one broadcast ds_read_b128;
//   * the consumer keeps three 8-link register sets in flight (reads issued ~16 links ahead).
// ------------------------------------------------------------------------------------------------
constexpr int kHub64Cols = 16;
constexpr int kHub64Producers = 8;
constexpr int kHub64Threads = 64 * (kHub64Producers + 1);
constexpr int kHub64Slack = 32;                               // the ring's reads past the last window
// W entries per window: 512 (141 KB of LDS, one workgroup per CU) for a few hub rows beside the row waves,
// 256 (72 KB, two per CU) once a launch has more hub workgroups than CUs (as k_spmm_hub's kHubWideW)
template <int W>
struct Hub64Geom {
    static constexpr int UW = W / (kHub64Producers * 8);      // gathers per producer lane per window
    static constexpr int LD = W + 4;                          // doubles per tile column (16-byte rows)
    static constexpr int TILE = kHub64Cols * LD;
    static constexpr size_t LDS_BYTES = (size_t)(2 * TILE + 2 * W + kHub64Slack) * sizeof(double);
    static_assert(LDS_BYTES <= 160 * 1024, "k_cheby_hub64's LDS");
};

template <int W>
__global__ void __launch_bounds__(kHub64Threads)
k_cheby_hub64(const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
              const double* __restrict__ vals, const int32_t* __restrict__ hub_rows, int n_slices,
              const double* __restrict__ Tc, const double* __restrict__ To, double* __restrict__ Tn, int64_t ld,
              int d, int mode, double a1, double a2, ChebyCoef<double> cf, int n_scales, double* __restrict__ R,
              int64_t r_stride)
{
    typedef typename Vec<double, 2>::type V2;
    constexpr int UW = Hub64Geom<W>::UW, LD = Hub64Geom<W>::LD, TILE = Hub64Geom<W>::TILE;
    extern __shared__ __attribute__((aligned(16))) double h64_lds[];
    double* aval_base = h64_lds + 2 * TILE;
    const int row = hub_rows[blockIdx.x / n_slices];
    const int slice = blockIdx.x % n_slices;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const int64_t beg = indptr[row];
    const int64_t end = indptr[row + 1];
    const int n_win = (int)((end - beg + W - 1) / W);

    if (wave == 0) {   // ---------------- consumer: 16 column chains ----------------
        const int c = lane & (kHub64Cols - 1);
        const int col = slice * kHub64Cols + c;
        const bool act = lane < kHub64Cols && col < d;
        double acc = 0.0;
        for (int h = 0; h < n_win; ++h) {
            __syncthreads();                      // window h is in tile h & 1
            if (lane < kHub64Cols) {
                const double* tcol = h64_lds + (h & 1) * TILE + c * LD;
                const double* av = aval_base + (h & 1) * W;
                const int64_t sb = beg + (int64_t)h * W;
                const int nb = (end - sb) < W ? (int)(end - sb) : W;
                const int nc = nb / 8;            // full 8-link sets
                V2 tA[4], aA[4], tB[4], aB[4], tC[4], aC[4];
                // set k: links 8k .. 8k + 7 (reads past nb stay inside the LDS block: kHub64Slack)
                auto ld = [&](int k, V2 (&t)[4], V2 (&a)[4]) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        t[i] = *reinterpret_cast<const V2*>(tcol + 8 * k + 2 * i);
                        a[i] = *reinterpret_cast<const V2*>(av + 8 * k + 2 * i);   // broadcast
                    }
                };
                auto run = [&](const V2 (&t)[4], const V2 (&a)[4]) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        acc = link(a[i][0], t[i][0], acc);
                        acc = link(a[i][1], t[i][1], acc);
                    }
                };
                ld(0, tA, aA);
                __builtin_amdgcn_sched_barrier(0);
                ld(1, tB, aB);
                __builtin_amdgcn_sched_barrier(0);
                int k = 0;
                for (; k + 3 <= nc; k += 3) {
                    ld(k + 2, tC, aC);
                    __builtin_amdgcn_sched_barrier(0);
                    run(tA, aA);
                    __builtin_amdgcn_sched_barrier(0);
                    ld(k + 3, tA, aA);
                    __builtin_amdgcn_sched_barrier(0);
                    run(tB, aB);
                    __builtin_amdgcn_sched_barrier(0);
                    ld(k + 4, tB, aB);
                    __builtin_amdgcn_sched_barrier(0);
                    run(tC, aC);
                    __builtin_amdgcn_sched_barrier(0);
                }
                // the loop leaves at most two full sets, k and k + 1 (already read), then < 8 links
                if (k < nc) run(tA, aA);
                if (k + 1 < nc) run(tB, aB);
                for (int q = nc * 8; q < nb; ++q) acc = link(av[q], tcol[q], acc);
            }
        }
        if (act) cheby_epi_at<double, 1>(mode, acc, Tc, To, Tn, R, (int64_t)row * ld + col, r_stride, a1, a2, cf, n_scales);
        return;
    }

    // ---------------- producers ----------------
    const int p = wave - 1;
    const int g = lane >> 3;          // entry within a gather's group of 8
    const int qq = lane & 7;          // 16-byte chunk: columns 2qq, 2qq + 1 of the slice
    const int qcol = slice * kHub64Cols + qq * 2;
    const bool gact = qcol < d;       // d even (the launch's condition): both columns or neither
    V2 x0[UW], x1[UW];
    double a0[UW], a1v[UW];
    int cn[UW];
    double an[UW];
    auto load_ids = [&](int w) {
        const int64_t sb = beg + (int64_t)w * W;
#pragma unroll
        for (int b = 0; b < UW; ++b) {
            int64_t jj = sb + (p * UW + b) * 8 + g;
            jj = jj < end ? jj : end - 1;
            cn[b] = indices[jj];
            an[b] = vals[jj];
        }
    };
    auto gather = [&](V2 (&x)[UW], double (&a)[UW]) {
#pragma unroll
        for (int b = 0; b < UW; ++b) {
            x[b] = gact ? gload<double, 2>(Tc + (int64_t)cn[b] * ld + qcol) : vzero<double, 2>();
            a[b] = an[b];
        }
    };
    auto put = [&](int w, const V2 (&x)[UW], const double (&a)[UW]) {
        double* tile = h64_lds + (w & 1) * TILE;
        double* av = aval_base + (w & 1) * W;
#pragma unroll
        for (int b = 0; b < UW; ++b) {
            const int nl = (p * UW + b) * 8 + g;   // entry within the window
            tile[(2 * qq) * LD + nl] = x[b][0];
            tile[(2 * qq + 1) * LD + nl] = x[b][1];
            if (qq == 0) av[nl] = a[b];
        }
    };
    // prologue: windows 0 and 1 in flight, window 0 published, window 2 in flight
    if (n_win > 0) {
        load_ids(0);
        __builtin_amdgcn_sched_barrier(0);
        gather(x0, a0);
        if (n_win > 1) { load_ids(1); gather(x1, a1v); }
        if (n_win > 2) load_ids(2);
        put(0, x0, a0);
        if (n_win > 2) { gather(x0, a0); if (n_win > 3) load_ids(3); }
    }
    __syncthreads();                              // window 0 published
    for (int h = 0; h + 1 < n_win; h += 2) {
        put(h + 1, x1, a1v);
        if (h + 3 < n_win) { gather(x1, a1v); if (h + 4 < n_win) load_ids(h + 4); }
        __syncthreads();
        if (h + 2 >= n_win) break;
        put(h + 2, x0, a0);
        if (h + 4 < n_win) { gather(x0, a0); if (h + 5 < n_win) load_ids(h + 5); }
        __syncthreads();
    }
    // barrier count: 1 (prologue) + (n_win - 1) in the loop == the consumer's n_win
}

// the hub workgroups of n_items (row, slice) pairs on `s` (the window size by the launch's width)
void launch_hub64(int64_t n_items, hipStream_t s, const int64_t* indptr, const int32_t* indices, const double* vals,
                  const int32_t* rows, int n_slices, const double* Tc, const double* To, double* Tn, int64_t ld, int d,
                  int mode, double a1, double a2, const ChebyCoef<double>& cf, int n_scales, double* R, int64_t r_stride)
{
    if (n_items > kHubWideLaunch)
        hipLaunchKernelGGL(k_cheby_hub64<256>, dim3((unsigned)n_items), dim3(kHub64Threads), Hub64Geom<256>::LDS_BYTES, s,
                           indptr, indices, vals, rows, n_slices, Tc, To, Tn, ld, d, mode, a1, a2, cf, n_scales, R, r_stride);
    else
        hipLaunchKernelGGL(k_cheby_hub64<512>, dim3((unsigned)n_items), dim3(kHub64Threads), Hub64Geom<512>::LDS_BYTES, s,
                           indptr, indices, vals, rows, n_slices, Tc, To, Tn, ld, d, mode, a1, a2, cf, n_scales, R, r_stride);
}

// ------------------------------------------------------------------------------------------------
// fp64 Chebyshev step over a column-blocked plan (srg_plan_cheby_step_f64): one launch per block of
// the plan, the row waves of k_cheby over the launch's schedule, row w's entries the span
// [slot_beg[w], slot_end[w]) of the caller's arrays.  A row's chain starts at 0 in block 0 (FIRST),
// continues from the fp64 partial sum the block before stored in Tn (exact: the stored value is the
// chain's value), and ends -- k_cheby's epilogue, the same operations -- in block 0 for the whole rows
// and in the last block for the cut rows (LAST).  So bitwise srg_cheby_step_f64, with each launch
// gathering from one column block of Tc (1/B of the panel: the L2 / Infinity Cache keep it).
// ------------------------------------------------------------------------------------------------
template <int VEC, int U, bool FIRST, bool LAST>
__global__ void __launch_bounds__(kBlock)
k_cheby_blk64(const int64_t* __restrict__ slot_beg, const int64_t* __restrict__ slot_end,
              const int32_t* __restrict__ order, int n_rows, const int32_t* __restrict__ indices,
              const double* __restrict__ vals, const double* __restrict__ Tc, const double* __restrict__ To,
              double* __restrict__ Tn, int64_t ld, int d, int mode, double a1, double a2, ChebyCoef<double> cf,
              int n_scales, double* __restrict__ R, int64_t r_stride, int block_base)
{
    typedef typename Vec<double, VEC>::type V;
    const int w = wave_slot(block_base);
    if (w >= n_rows) return;
    if constexpr (!FIRST && !LAST) {
        if (slot_beg[w] >= slot_end[w]) return;   // nothing in this block: the partial sum stays
    }
    const int row = order[w];
    const int lane = threadIdx.x & 63;
    const int64_t roff = (int64_t)row * ld;
    for (int c0 = 0; c0 < d; c0 += 64 * VEC) {
        const int col = c0 + lane * VEC;
        const bool act = col < d;
        V acc = vzero<double, VEC>();
        if constexpr (!FIRST) {
            if (act) acc = vload<double, VEC>(Tn + roff + col);
        }
        row_gather<double, VEC, U, false, int64_t, true>(acc, slot_beg, indices, vals, w, Tc, ld, col, act, slot_end);
        if (!act) continue;
        if constexpr (!LAST)
            vstore<double, VEC>(Tn + roff + col, acc, false);
        else
            cheby_epi_at<double, VEC>(mode, acc, Tc, To, Tn, R, roff + col, r_stride, a1, a2, cf, n_scales);
    }
}

// Chebyshev epilogue after a load-balanced SpMM (fp32, large graphs): Tn holds acc = A*Tc (the
// same fma chain k_cheby forms, so results are bit-identical to the fused kernel) and becomes
// Tn; every panel has its own leading dimension, so column blocks of S and R need no copies.
// INIT_T / STEP_FIRST defer the INIT's scale outputs to the first step, which forms them from T0,
// T1 and T2 with the same operations in the same order (R = ((c0/2) T0 + c1 T1) + c2 T2), and
// SRG_CHEBY_NO_T leaves T_{k+1} unstored in the last order: 4 panel passes less per order-3 block.
__global__ void __launch_bounds__(256)
k_cheby_epilogue(float* __restrict__ Tn, int64_t ldn, const float* __restrict__ Tc, int64_t ldc,
                 const float* __restrict__ To, int64_t ldo, int64_t n_rows, int d, int mode, float a1,
                 float a2, ChebyCoef<float> cf, int n_scales, float* __restrict__ R, int64_t ldr,
                 int64_t r_stride)
{
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
    const bool store_t = !(mode & SRG_CHEBY_NO_T);
    const int m = mode & 0xf;
    for (int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < n_rows; r += waves) {
        float* tn = Tn + r * ldn;
        float* rr = R + r * ldr;
        for (int c = lane; c < d; c += 64) {
            const float acc = tn[c];
            float t;
            if (m == SRG_CHEBY_INIT || m == SRG_CHEBY_INIT_T) {
                const float tc = Tc[r * ldc + c];
                t = e_div(e_sub(acc, e_mul(a2, tc)), a1);
                if (m == SRG_CHEBY_INIT)
                    for (int s = 0; s < n_scales; ++s)
                        rr[s * r_stride + c] = e_add(e_mul(cf.prev[s], tc), e_mul(cf.cur[s], t));
            } else if (m == SRG_CHEBY_STEP_FIRST) {
                const float t0 = To[r * ldo + c], t1 = Tc[r * ldc + c];
                t = e_sub(acc, t0);
                for (int s = 0; s < n_scales; ++s)
                    rr[s * r_stride + c] = e_add(e_add(e_mul(cf.prev[s], t0), e_mul(cf.mid[s], t1)), e_mul(cf.cur[s], t));
            } else {
                t = e_sub(acc, To[r * ldo + c]);
                for (int s = 0; s < n_scales; ++s)
                    rr[s * r_stride + c] = e_add(rr[s * r_stride + c], e_mul(cf.cur[s], t));
            }
            if (store_t) tn[c] = t;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// hop aggregation (fused SGC / SSGC / GBP precompute: MessageOp.combine without the K+1 panels)
//
// The reference combines the hop list on the host (SSRG/operators/message_operator/{sum,mean,
// simple_weighted}_message_op.py, operators/utils.py:426-437).  Python's sum() is a left-to-right
// accumulation from +0; one_dim_weighted_add is torch's CPU dim-0 sum of rounded products, whose
// order (ATen cascade_sum) the host plans as a sequence of the element-wise steps below:
//   INIT: agg = 0 + w*y      ADD: agg = agg + w*y      DIV: agg = agg / w
// with separate multiply / add / correctly rounded divide (no contraction).  The last < 32 flat
// elements of a weighted sum take torch's scalar row_sum order instead (k_tail_*).
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
k_hop_accumulate(float* __restrict__ agg, int64_t lda, const float* __restrict__ y, int64_t ldy,
                 int64_t n_rows, int d, float w, int mode)
{
    // one wave per row (grid-stride over rows), lanes stride the columns: no index division
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < n_rows; r += waves) {
        float* a = agg + r * lda;
        const float* yr = y + r * ldy;
        for (int c = lane; c < d; c += 64) {
            if (mode == SRG_ACC_DIV) {
                a[c] = __fdiv_rn(a[c], w);
            } else {
                const float p = __fmul_rn(w, yr[c]);
                a[c] = __fadd_rn(mode == SRG_ACC_INIT ? 0.0f : a[c], p);
            }
        }
    }
}

// Row gather (the send-side pack of the halo exchange, srgnn.dist): dst[i, :] = src[idx[i], :].
// S lanes per row (the power of two >= the row's VEC-chunks, at most 64), 64 / S rows per wave
// step and U = 4 steps in flight: 16-byte loads at d = 128 are 2 rows per wave-instruction, 8 rows
// per wave in flight.  Indices outside [0, n_src) leave their dst row unwritten (never a fault).
template <int VEC, int S>
__global__ void __launch_bounds__(256)
k_gather_rows(const float* __restrict__ src, int64_t lds, int64_t n_src, const int64_t* __restrict__ idx,
              int64_t n_idx, float* __restrict__ dst, int64_t ldd, int cpr)
{
    typedef typename Vec<float, VEC>::type V;
    constexpr int R = 64 / S, U = 4;
    const int lane = threadIdx.x & 63;
    const int g = lane / S, c0 = lane % S;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t base = wave * (R * U); base < n_idx; base += waves * (R * U)) {
        int64_t sr[U], dr[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            dr[u] = base + u * R + g;
            sr[u] = dr[u] < n_idx ? idx[dr[u]] : -1;
            if (sr[u] >= n_src) sr[u] = -1;
        }
        for (int c = c0; c < cpr; c += S) {
            V v[U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (sr[u] >= 0) v[u] = vload<float, VEC>(src + sr[u] * lds + (int64_t)c * VEC);
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (sr[u] >= 0) vstore<float, VEC>(dst + dr[u] * ldd + (int64_t)c * VEC, v[u], false);
        }
    }
}

// torch's multi_row_sum (ATen/native/cpu/SumKernel.cpp) for one element over `count` rows of the
// tail history, rows start, start + stride, ...: 16-row blocks folded into 4 levels.
__device__ float torch_multi_row_sum(const float* hist, int start, int stride, int count, int e)
{
    int clog2 = 1;
    if (count > 2) clog2 = 32 - __clz(count - 1);
    const int lp = clog2 / 4 > 4 ? clog2 / 4 : 4;
    const int step = 1 << lp, mask = step - 1;
    float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    int i = 0;
    while (i + step <= count) {
        for (int j = 0; j < step; ++j, ++i)
            acc[0] = __fadd_rn(acc[0], hist[(int64_t)(start + i * stride) * SRG_TAIL_MAX + e]);
        for (int j = 1; j < 4; ++j) {
            acc[j] = __fadd_rn(acc[j], acc[j - 1]);
            acc[j - 1] = 0.0f;
            if ((i & (mask << (j * lp))) != 0) break;
        }
    }
    for (; i < count; ++i) acc[0] = __fadd_rn(acc[0], hist[(int64_t)(start + i * stride) * SRG_TAIL_MAX + e]);
    for (int j = 1; j < 4; ++j) acc[0] = __fadd_rn(acc[0], acc[j]);
    return acc[0];
}

// hist[term][e] = w * y[flat_start + e] (the rounded products of one hop's tail elements)
__global__ void k_tail_record(float* __restrict__ hist, const float* __restrict__ y, int64_t ldy, int d,
                              int64_t flat_start, int len, float w)
{
    const int e = threadIdx.x;
    if (e >= len) return;
    const int64_t f = flat_start + e;
    hist[e] = __fmul_rn(w, y[(f / d) * ldy + f % d]);
}

// torch's row_sum (4 interleaved partial sums, remainder into the first, then folded) over the
// recorded terms, stored as out = 0 + sum
__global__ void k_tail_rowsum(float* __restrict__ agg, int64_t lda, int d, int64_t flat_start, int len,
                              const float* __restrict__ hist, int n_terms)
{
    const int e = threadIdx.x;
    if (e >= len) return;
    const int n4 = n_terms / 4;
    float p[4];
    for (int c = 0; c < 4; ++c) p[c] = torch_multi_row_sum(hist, c, 4, n4, e);
    for (int i = 4 * n4; i < n_terms; ++i) p[0] = __fadd_rn(p[0], hist[(int64_t)i * SRG_TAIL_MAX + e]);
    for (int c = 1; c < 4; ++c) p[0] = __fadd_rn(p[0], p[c]);
    const int64_t f = flat_start + e;
    agg[(f / d) * lda + f % d] = __fadd_rn(0.0f, p[0]);
}

// ------------------------------------------------------------------------------------------------
// construct_adj on the device: sequential fp64 segment sums (duplicate merging and row degrees in
// storage order, starting from +0 -- scipy's csr_binop / csr_matvec accumulation order)
// ------------------------------------------------------------------------------------------------
// One wave per 64 consecutive segments.  A segment of at most kSegShort entries is summed by its
// own lane; a longer one (the degree of a hub row: 155,868 entries on the products-shaped graph,
// 30 ms as a one-lane loop of dependent loads) by the whole wave: the values are read 64 at a time
// with one coalesced load, the next block prefetched, and the sequential sum runs over them
// through v_readlane -- the same adds in the same order.
constexpr int64_t kSegShort = 64;

template <typename T>
__device__ __forceinline__ T bcast_lane(T v, int q)
{
    if constexpr (sizeof(T) == 8) {
        const unsigned long long bits = __builtin_bit_cast(unsigned long long, v);
        const unsigned lo = __builtin_amdgcn_readlane((unsigned)bits, q);
        const unsigned hi = __builtin_amdgcn_readlane((unsigned)(bits >> 32), q);
        return __builtin_bit_cast(T, ((unsigned long long)hi << 32) | lo);
    } else {
        return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), q));
    }
}

template <typename T>
__global__ void __launch_bounds__(256)
k_segment_sum(const int64_t* __restrict__ seg_ptr, const T* __restrict__ vals, int64_t n_seg,
              T* __restrict__ out)
{
    const int lane = threadIdx.x & 63;
    const int64_t wave_stride = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); w * 64 < n_seg;
         w += wave_stride) {
        const int64_t s = w * 64 + lane;
        const bool valid = s < n_seg;
        const int64_t beg = valid ? seg_ptr[s] : 0;
        const int64_t end = valid ? seg_ptr[s + 1] : 0;
        const bool wide = end - beg > kSegShort;
        if (valid && !wide) {
            T acc = T(0);
            for (int64_t j = beg; j < end; ++j) acc = e_add(acc, vals[j]);
            out[s] = acc;
        }
        unsigned long long todo = __ballot(wide);   // wave-uniform
        while (todo) {
            const int l = __builtin_ctzll(todo);
            todo &= todo - 1;
            const int64_t b = bcast_lane(beg, l), e = bcast_lane(end, l);
            T acc = T(0);
            int64_t j0 = b + lane;
            T v_nxt = j0 < e ? vals[j0] : T(0);
            for (int64_t jb = b; jb < e; jb += 64) {
                const T v = v_nxt;
                const int64_t jn = jb + 64 + lane;
                v_nxt = jn < e ? vals[jn] : T(0);
                const int nb = (e - jb) < 64 ? (int)(e - jb) : 64;   // wave-uniform
                for (int q = 0; q < nb; ++q) acc = e_add(acc, bcast_lane(v, q));
            }
            if (lane == 0) out[w * 64 + l] = acc;
        }
    }
}

// fp64 product Y = A * X in scipy's csr_matvec(s) order (sparsetools csr.h): each element starts
// from 0 and adds the separately rounded product of every stored entry, in storage order.  One
// thread per output element (row-major, so neighbouring threads share a row's entries); used by
// the construct_adj power iterations (srgnn/directed.py), not by the hop loop.
__global__ void __launch_bounds__(256)
k_spmm_f64(const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
           const double* __restrict__ vals, int64_t n_rows, const double* __restrict__ X, int64_t ldx,
           double* __restrict__ Y, int64_t ldy, int d)
{
    const int64_t total = n_rows * (int64_t)d;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
        const int64_t row = e / d;
        const int c = (int)(e - row * d);
        double acc = 0.0;
        for (int64_t j = indptr[row]; j < indptr[row + 1]; ++j)
            acc = __dadd_rn(acc, __dmul_rn(vals[j], X[(int64_t)indices[j] * ldx + c]));
        Y[row * ldy + c] = acc;
    }
}

// ------------------------------------------------------------------------------------------------
// validation kernel
// ------------------------------------------------------------------------------------------------
__global__ void k_validate(const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
                           int64_t n_rows, int64_t nnz, int64_t n_cols, unsigned int* __restrict__ bad)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    unsigned int b = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nnz; i += stride) {
        const int32_t c = indices[i];
        if (c < 0 || (int64_t)c >= n_cols) b |= 1u;
    }
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_rows; i += stride) {
        if (indptr[i + 1] < indptr[i]) b |= 2u;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (indptr[0] != 0) b |= 4u;
        if (indptr[n_rows] != nnz) b |= 8u;
    }
    if (b) atomicOr(bad, b);
}

// Column-block split points: splits[(b-1) * n_rows + r] = the first entry of row r whose column id
// is >= ceil(b * n_cols / B) (a lower bound over the row's sorted ids), b = 1 .. B-1.  One thread per
// (row, boundary).  For a row whose ids are not sorted the result is still a position in
// [indptr[r], indptr[r+1]] and the split points of a row never decrease with b, so the spans still
// partition the row in CSR order: the hop stays exact, only the blocks' locality is lost.
__global__ void __launch_bounds__(256)
k_col_splits(const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices, int64_t n_rows,
             int64_t n_cols, int n_blocks, int64_t* __restrict__ splits)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_rows * (n_blocks - 1)) return;
    const int b = (int)(t / n_rows) + 1;
    const int64_t r = t % n_rows;
    const int64_t bound = (b * n_cols + n_blocks - 1) / n_blocks;
    int64_t lo = indptr[r], hi = indptr[r + 1];
    while (lo < hi) {
        const int64_t mid = lo + (hi - lo) / 2;
        if ((int64_t)indices[mid] < bound)
            lo = mid + 1;
        else
            hi = mid;
    }
    splits[t] = lo;
}

// Span copy (DeviceCSR compact copies: the entries of a launch laid out in the order it takes its
// rows): row order[i]'s span [beg, end) of (indices, values) goes to [pos[i], pos[i] + len) of the
// output arrays, and out_beg / out_end of that row get the new span.  16 lanes per row, each lane
// copying every 16th entry (coalesced runs of the row); 4 rows per wave, a grid stride over rows.
__global__ void __launch_bounds__(256)
k_copy_spans(const int32_t* __restrict__ order, int64_t n, const int64_t* __restrict__ beg,
             const int64_t* __restrict__ end, const int32_t* __restrict__ ix, const float* __restrict__ v,
             const int64_t* __restrict__ pos, int32_t* __restrict__ oix, float* __restrict__ ov,
             int64_t* __restrict__ obeg, int64_t* __restrict__ oend)
{
    const int l = threadIdx.x & 15;
    const int64_t stride = (int64_t)gridDim.x * (blockDim.x / 16);
    for (int64_t i = (int64_t)blockIdx.x * (blockDim.x / 16) + (threadIdx.x >> 4); i < n; i += stride) {
        const int r = order[i];
        const int64_t b = beg[r], len = end[r] - b, p = pos[i];
        for (int64_t e = l; e < len; e += 16) {
            oix[p + e] = ix[b + e];
            ov[p + e] = v[b + e];
        }
        if (l == 0) {
            obeg[r] = p;
            oend[r] = p + len;
        }
    }
}

// Mirror positions of a CSR with sorted rows: mirror[e] = the position of entry (c, r) in row c for
// entry e = (r, c), or -1 when row c holds no column r (one binary search per entry).  All entries
// found <=> the structure is symmetric, and then the transpose of the matrix is the same structure
// with values[mirror] -- construct_adj's (A+I)^T without a sort (srgnn/construct.py).
__global__ void __launch_bounds__(256)
k_csr_mirror(const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
             const int64_t* __restrict__ rows, int64_t nnz, int64_t* __restrict__ mirror)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nnz; e += stride) {
        const int64_t r = rows[e];
        const int32_t c = indices[e];
        int64_t lo = indptr[c], hi = indptr[c + 1];
        while (lo < hi) {
            const int64_t mid = lo + (hi - lo) / 2;
            if ((int64_t)indices[mid] < r)
                lo = mid + 1;
            else
                hi = mid;
        }
        mirror[e] = (lo < indptr[c + 1] && (int64_t)indices[lo] == r) ? lo : -1;
    }
}

// ------------------------------------------------------------------------------------------------
// launch helpers
// ------------------------------------------------------------------------------------------------
constexpr int kUnroll = 8;

bool aligned(const void* p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

int pick_vec(int d, int64_t ldx, int64_t ldy, const void* X, const void* Y, size_t elem)
{
    // widest per-lane access whose tiles line up with every row of X and Y
    if (elem == 4 && d >= 256 && d % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && aligned(X, 16) &&
        aligned(Y, 16))
        return 4;
    if (d >= 128 && d % 2 == 0 && ldx % 2 == 0 && ldy % 2 == 0 && aligned(X, 2 * elem) &&
        aligned(Y, 2 * elem))
        return 2;
    return 1;
}

// slice-wave groups of 8 entries in flight.  Round 5, with the packed rows' id staging: for the
// 128- / 256-column packed launches 4 groups take the products hop from 5.26 to 5.22 ms (8 and 6
// measure the same, 2 is 4 % slower, 12 and 16 do not unroll: 9.9 / 11.7 ms; arxiv flat), but the
// RMAT-26 filter bank's 64-column blocks lose 3 % with 4 (1.243 against 1.202 s per step), so the
// 64-column packed launches and the other row paths keep 8 (profiles/r05bf_slice_unroll_ab.txt)
#ifndef SRG_UNROLL_HEAVY
#define SRG_UNROLL_HEAVY 8
#endif
constexpr int kUnrollHeavy = SRG_UNROLL_HEAVY;
constexpr int kUnrollHeavyWide = 4;           // the packed launches with 4 or 2 rows per wave (d = 128 / 256)

// One wave that sleeps ~`us` microseconds (s_memrealtime ticks at 100 MHz).  Enqueued on the main
// stream right after the hub workgroups are forked onto the side stream, so they are dispatched
// onto free CUs before the main launch's blocks fill every CU (a hub workgroup needs 9 waves and
// ~136 KB of LDS on one CU; behind a full-chip launch it could start milliseconds late and become
// the hop's tail).
__global__ void k_dispatch_delay(int us)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long ticks = 100ull * (unsigned long long)us;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(16);
}

// Light rows per wave for wide panels (packed_rows): 512 / d rows, so that every lane holds two
// 16-byte column chunks (d = 64: 8 rows of 8 lanes, d = 128: 4 rows of 16 lanes, d = 256: 2 rows of 32
// lanes; measured best, profiles/r02_ab_d256.txt: 4 rows at d = 256 are 2 % slower than one row per
// wave; d = 32 packed measured even with the narrow path, profiles/r02_ab_d32.txt), 4 gathers per row in
// flight (2 with SRG_SPMM_PACKED_U2; 8 measured slower).  Results are identical for every setting.
constexpr int kPackedU = 4;
constexpr int packed_rows_for(int d) { return d == 64 ? 8 : d == 128 ? 4 : d == 256 ? 2 : 0; }
// LDS a k_spmm block needs (its waves' slice tiles), and what a launch reserves with
// SRG_SPMM_CAP_WAVES: ~160 KiB / (5 + 0.5) per 4-wave block, so at most 5 blocks -- 5 waves per SIMD --
// share a CU (gfx950's 160 KiB LDS; below the 64 KiB default dynamic-LDS limit).  Fewer waves gather
// from fewer rows at once and the L2 re-serves more of their lines: products 6.08 -> 5.96 ms per hop
// and 35.4 -> 31.3 GB of traffic at 5 waves without the slice waves' id prefetch, 5.84 -> 5.81 ms with
// it (whose registers already hold the kernel at 6 waves); 4 and 3 waves lose; arxiv (an 87 MB panel)
// is 3 % faster uncapped, the halo chunks flat (profiles/r04v_*, r04w_*, r04x_*).
constexpr int kSpmmLdsBytes = kWavesPerBlock * kSliceLdsBufs * 256 * (int)sizeof(float);
constexpr int kSpmmCapLdsBytes = (int)((160.0 * 1024.0) / 5.5) / 512 * 512;
static_assert(kSpmmCapLdsBytes > kSpmmLdsBytes && kSpmmCapLdsBytes <= 65536, "k_spmm's capped LDS reservation");
constexpr int spmm_lds_bytes(uint32_t flags) { return (flags & SRG_SPMM_CAP_WAVES) ? kSpmmCapLdsBytes : kSpmmLdsBytes; }
// the single-wave delay after a hub fork (10 us: 0 and 5 stay bimodal, 20 is 1-3 % slower,
// profiles/r01_dispatch_delay_sweep.txt)
constexpr int kHubDelayUs = 10;

// Hub side streams.  One per (device, caller stream), created on first use, each with its own
// fork / join events: callers on different streams never share events.  The whole fork sequence
// of a launch (record fork, side-stream wait, hub launch, record join, main launch, join wait)
// runs under g_side_mu, so host threads sharing one caller stream cannot interleave their records
// either.  SRG_SPMM_HUB_NOJOIN leaves the join to srg_hub_join(stream), which waits on the same
// (device, stream) entry's join event.  At most kMaxSideStreams entries live per device: a caller
// that makes a new stream per call evicts the least recently used entry without an outstanding
// NOJOIN fork (its stream is destroyed asynchronously: queued hub work still completes).
struct SideStream {
    hipStream_t stream = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    uint64_t last_use = 0;
    bool pending = false;      // a NOJOIN fork not yet joined by srg_hub_join
};
constexpr int kMaxSideStreams = 8;
std::mutex g_side_mu;
std::map<std::pair<int, hipStream_t>, SideStream> g_side;   // guarded by g_side_mu
uint64_t g_side_tick = 0;                                     // guarded by g_side_mu
bool g_side_attr[64] = {};                                     // per-device kernel attributes set

// Sets the hub kernels' dynamic-LDS limit on the current device (attributes are per device).
template <typename IP>
int hub_attrs()
{
    for (const void* fn : {(const void*)k_spmm_hub<true, IP>, (const void*)k_spmm_hub<false, IP>,
                           (const void*)k_spmm_hub<true, IP, kEpiCheby>, (const void*)k_spmm_hub<false, IP, kEpiCheby>,
                           (const void*)k_spmm_hub<true, IP, kEpiSpan>, (const void*)k_spmm_hub<false, IP, kEpiSpan>})
        SRG_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kHubLdsBytes));
    for (const void* fn : {(const void*)k_spmm_hub<true, IP, kEpiPlain, kHubWideW>, (const void*)k_spmm_hub<false, IP, kEpiPlain, kHubWideW>,
                           (const void*)k_spmm_hub<true, IP, kEpiCheby, kHubWideW>, (const void*)k_spmm_hub<false, IP, kEpiCheby, kHubWideW>,
                           (const void*)k_spmm_hub<true, IP, kEpiSpan, kHubWideW>, (const void*)k_spmm_hub<false, IP, kEpiSpan, kHubWideW>})
        SRG_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)HubGeom<kHubWideW>::LDS_BYTES));
    return SRG_OK;
}

// The side stream of (current device, caller); the caller holds g_side_mu.
int side_stream_locked(hipStream_t caller, SideStream** out)
{
    int dev = 0;
    SRG_HIP_CHECK(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return fail(SRG_ERR_HIP, "device id %d", dev);
    if (!g_side_attr[dev]) {
        int rc = hub_attrs<int>();
        if (!rc) rc = hub_attrs<int64_t>();
        if (rc) return rc;
        SRG_HIP_CHECK(hipFuncSetAttribute((const void*)k_cheby_hub64<512>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)Hub64Geom<512>::LDS_BYTES));
        SRG_HIP_CHECK(hipFuncSetAttribute((const void*)k_cheby_hub64<256>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)Hub64Geom<256>::LDS_BYTES));
        g_side_attr[dev] = true;
    }
    const auto key = std::make_pair(dev, caller);
    if (g_side.find(key) == g_side.end()) {
        int live = 0;
        auto lru = g_side.end();
        for (auto it = g_side.begin(); it != g_side.end(); ++it) {
            if (it->first.first != dev) continue;
            ++live;
            if (!it->second.pending && (lru == g_side.end() || it->second.last_use < lru->second.last_use)) lru = it;
        }
        if (live >= kMaxSideStreams && lru != g_side.end()) {
            (void)hipEventDestroy(lru->second.fork);
            (void)hipEventDestroy(lru->second.join);
            (void)hipStreamDestroy(lru->second.stream);
            g_side.erase(lru);
        }
    }
    SideStream& ss = g_side[key];
    ss.last_use = ++g_side_tick;
    if (!ss.stream) {
        // highest queue priority: the hub workgroups (9 waves, ~136 KB LDS each) must get CUs
        // before the main launch's many small blocks occupy them all (normal priority measured the
        // same or slower: DESIGN.md §7, round 4)
        int least = 0, greatest = 0;
        SRG_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
        SRG_HIP_CHECK(hipStreamCreateWithPriority(&ss.stream, hipStreamNonBlocking, greatest));
        SRG_HIP_CHECK(hipEventCreateWithFlags(&ss.fork, hipEventDisableTiming));
        SRG_HIP_CHECK(hipEventCreateWithFlags(&ss.join, hipEventDisableTiming));
    }
    *out = &ss;
    return SRG_OK;
}

// Makes the device of `s` current for the lifetime of the guard (the null stream means the
// current device), so every launch, event and side stream of an entry point belongs to the
// device the caller's stream lives on.
struct DeviceGuard {
    int prev = -1, dev = -1, rc = SRG_OK;
    explicit DeviceGuard(hipStream_t s)
    {
        // no usable device: leave it to the entry point (argument checks and empty problems
        // need none; its first HIP call reports the error)
        hipError_t e = hipGetDevice(&prev);
        if (e != hipSuccess) { (void)hipGetLastError(); prev = -1; return; }
        dev = prev;
        if (s) {
            hipDevice_t d = 0;
            e = hipStreamGetDevice(s, &d);
            if (e != hipSuccess) { rc = fail(SRG_ERR_HIP, "hipStreamGetDevice failed: %s", hipGetErrorString(e)); return; }
            dev = (int)d;
        }
        if (dev != prev) {
            e = hipSetDevice(dev);
            if (e != hipSuccess) { rc = fail(SRG_ERR_HIP, "hipSetDevice(%d) failed: %s", dev, hipGetErrorString(e)); dev = prev; }
        }
    }
    ~DeviceGuard()
    {
        if (prev >= 0 && dev != prev) (void)hipSetDevice(prev);
    }
};

#define SRG_DEVICE_GUARD(stream)                                   \
    DeviceGuard guard_(static_cast<hipStream_t>(stream));          \
    if (guard_.rc) return guard_.rc

// ------------------------------------------------------------------------------------------------
// SRG_SPMM_FAST: the hub rows as kFastSegs segments each.  Segment s of hub row h (row order[h]) is
// entries [b + len*s/S, b + len*(s+1)/S) of the row -- a row span -- computed as an exact fma
// chain by the slice waves of the span kernel into a scratch panel; the S partial sums of a row are
// then added in segment order.  Tolerance mode (the reference's single chain is re-associated into
// S pieces, deterministically); the longest row's latency drops ~S-fold.
// ------------------------------------------------------------------------------------------------
constexpr int kFastSegs = 64;

template <typename IP, bool SPAN>
__global__ __launch_bounds__(256) void k_fast_segments(const IP* __restrict__ indptr, const int64_t* __restrict__ row_end,
                                                       const int32_t* __restrict__ order, int64_t n_hub,
                                                       int64_t* __restrict__ seg_beg, int64_t* __restrict__ seg_end,
                                                       int32_t* __restrict__ seg_order)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_hub * kFastSegs) return;
    const int64_t h = i / kFastSegs, sg = i % kFastSegs;
    const int r = order[h];
    const int64_t b = (int64_t)indptr[r];
    const int64_t e = SPAN ? row_end[r] : (int64_t)indptr[r + 1];
    const int64_t len = e - b;
    seg_beg[i] = b + len * sg / kFastSegs;
    seg_end[i] = b + len * (sg + 1) / kFastSegs;
    seg_order[i] = (int32_t)i;
}

__global__ __launch_bounds__(256) void k_fast_reduce(const int32_t* __restrict__ order, int64_t n_hub,
                                                     const float* __restrict__ part, int64_t ldp,
                                                     float* __restrict__ Y, int64_t ldy, int d, int acc)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t h = i / d;
    const int c = (int)(i % d);
    if (h >= n_hub) return;
    float* y = Y + (int64_t)order[h] * ldy + c;
    float v = acc ? *y : 0.0f;
    const float* p = part + h * kFastSegs * ldp + c;
    for (int sg = 0; sg < kFastSegs; ++sg) v = __fadd_rn(v, p[sg * ldp]);
    *y = v;
}

template <typename IP, int EX = kEpiPlain>
int launch_spmm(const IP* indptr, const int32_t* indices, const float* vals, int64_t n_rows,
                const int32_t* order, int64_t n_hub, int64_t n_heavy, const float* X, int64_t ldx,
                float* Y, int64_t ldy, int d, uint32_t flags, hipStream_t s,
                Epi epi = Epi{})
{
    if (n_rows <= 0 || d <= 0) return SRG_OK;
    if (n_hub < 0 || n_heavy < 0 || n_hub + n_heavy > n_rows || ((n_hub + n_heavy) > 0 && !order))
        return fail(SRG_ERR_INVALID, "n_hub=%lld n_heavy=%lld need a row_order and <= n_rows",
                    (long long)n_hub, (long long)n_heavy);
    // slice waves and hub blocks gather 16-byte chunks: they need d % 4 == 0 and aligned rows;
    // otherwise every row takes the row-wave path (same results)
    const bool slice_ok = d % 4 == 0 && ldx % 4 == 0 && aligned(X, 16);
    if (!slice_ok) {
        n_heavy = 0;
        n_hub = 0;
    }
    const int n_slices = (d + kSliceCols - 1) / kSliceCols;
    if ((n_hub + n_heavy) * (int64_t)n_slices > INT32_MAX - 64)
        return fail(SRG_ERR_INVALID, "too many heavy slices");
    const int acc = (flags & SRG_SPMM_ACCUMULATE) ? 1 : 0;
    const int nt = (flags & SRG_SPMM_NT_STORE) ? 1 : 0;
    const bool sfull = d % kSliceCols == 0;

    SideStream* ss = nullptr;
    std::unique_lock<std::mutex> side_lock(g_side_mu, std::defer_lock);
    const bool fast = (flags & SRG_SPMM_FAST) && (EX == kEpiPlain || EX == kEpiSpan) && !epi.agg;
    if (n_hub > 0 && fast) {   // fork: the hub rows' segments, then their sums, beside the main launch
        side_lock.lock();
        int rc = side_stream_locked(s, &ss);
        if (rc) return rc;
        SRG_HIP_CHECK(hipEventRecord(ss->fork, s));
        SRG_HIP_CHECK(hipStreamWaitEvent(ss->stream, ss->fork, 0));
        const int64_t T = n_hub * kFastSegs;
        const int64_t ldp = (d + 3) & ~3;
        const size_t idx_bytes = ((size_t)T * (2 * sizeof(int64_t) + sizeof(int32_t)) + 255) & ~(size_t)255;
        void* buf = nullptr;
        SRG_HIP_CHECK(hipMallocAsync(&buf, idx_bytes + (size_t)T * ldp * sizeof(float), ss->stream));
        int64_t* seg_beg = static_cast<int64_t*>(buf);
        int64_t* seg_end = seg_beg + T;
        int32_t* seg_order = reinterpret_cast<int32_t*>(seg_end + T);
        float* part = reinterpret_cast<float*>(static_cast<char*>(buf) + idx_bytes);
        const unsigned gs = (unsigned)((T + 255) / 256);
        if (EX == kEpiSpan)
            hipLaunchKernelGGL((k_fast_segments<IP, true>), dim3(gs), dim3(256), 0, ss->stream, indptr, epi.row_end,
                               order, n_hub, seg_beg, seg_end, seg_order);
        else
            hipLaunchKernelGGL((k_fast_segments<IP, false>), dim3(gs), dim3(256), 0, ss->stream, indptr, nullptr,
                               order, n_hub, seg_beg, seg_end, seg_order);
        SRG_HIP_CHECK(hipGetLastError());
        Epi se{};
        se.row_end = seg_end;
        // every segment a slice-wave row (exact chain over its span), no hubs, no accumulation
        rc = launch_spmm<int64_t, kEpiSpan>(seg_beg, indices, vals, T, seg_order, 0, T, X, ldx, part, ldp, d,
                                            flags & SRG_SPMM_PACKED_U2, ss->stream, se);
        if (rc) return rc;
        const unsigned gr = (unsigned)((n_hub * d + 255) / 256);
        hipLaunchKernelGGL(k_fast_reduce, dim3(gr), dim3(256), 0, ss->stream, order, n_hub, part, ldp, Y, ldy, d, acc);
        SRG_HIP_CHECK(hipGetLastError());
        SRG_HIP_CHECK(hipFreeAsync(buf, ss->stream));
        SRG_HIP_CHECK(hipEventRecord(ss->join, ss->stream));
        ss->pending = (flags & SRG_SPMM_HUB_NOJOIN) != 0;
    } else if (n_hub > 0) {   // fork: hub blocks run beside the main launch
        side_lock.lock();
        int rc = side_stream_locked(s, &ss);
        if (rc) return rc;
        // CONTINUE after an unjoined fork: the hub rows are appended to the side stream, which is
        // already ordered after everything they read (the caller's guarantee), with no new fork
        // and no dispatch delay on the caller's stream
        const bool cont = (flags & SRG_SPMM_HUB_CONTINUE) && ss->pending;
        if (!cont) {
            SRG_HIP_CHECK(hipEventRecord(ss->fork, s));
            SRG_HIP_CHECK(hipStreamWaitEvent(ss->stream, ss->fork, 0));
        }
        const dim3 hgrid((unsigned)(n_hub * n_slices));
        // 256-nonzero windows (two workgroups per CU) once a launch has more hub workgroups than CUs
        const bool w256 = n_hub * n_slices > kHubWideLaunch || (flags & SRG_SPMM_HUB_W256);
#define SRG_LAUNCH_HUB(SF, WW)                                                                                      \
    hipLaunchKernelGGL((k_spmm_hub<SF, IP, EX, WW>), hgrid, dim3(kHubThreads), (HubGeom<WW>::LDS_BYTES), ss->stream, \
                       indptr, indices, vals, order, n_slices, X, ldx, Y, ldy, d, acc, nt, epi)
        if (sfull) {
            if (w256) SRG_LAUNCH_HUB(true, kHubWideW);
            else SRG_LAUNCH_HUB(true, 512);
        } else {
            if (w256) SRG_LAUNCH_HUB(false, kHubWideW);
            else SRG_LAUNCH_HUB(false, 512);
        }
#undef SRG_LAUNCH_HUB
        SRG_HIP_CHECK(hipGetLastError());
        SRG_HIP_CHECK(hipEventRecord(ss->join, ss->stream));
        ss->pending = (flags & SRG_SPMM_HUB_NOJOIN) != 0;
        if (!cont) {
            hipLaunchKernelGGL(k_dispatch_delay, dim3(1), dim3(64), 0, s, kHubDelayUs);
            SRG_HIP_CHECK(hipGetLastError());
        }
    }

    const int32_t* morder = order ? order + n_hub : nullptr;
    const int64_t m_rows = n_rows - n_hub;
    const int nb_heavy = (int)((n_heavy * n_slices + kWavesPerBlock - 1) / kWavesPerBlock);
    const int64_t n_light = m_rows - n_heavy;
    // light rows: LR rows per wave (packed_rows) when the column tiles line up; else, for d <= 32,
    // 64 / S rows per wave (narrow_rows); else one row per wave
    int lr = 0;
    if (!(flags & SRG_SPMM_WIDE_ROWS)) {
        const int cand = packed_rows_for(d);
        const int S = cand ? 64 / cand : 0;
        const int q = cand ? d / (4 * S) : 0;
        const bool ok = cand && d % (4 * S) == 0 && q == 2 && ldx % 4 == 0 &&
                        ldy % 4 == 0 && aligned(X, 16) && aligned(Y, 16) &&
                        (!epi.agg || (epi.lda % 4 == 0 && aligned(epi.agg, 16))) &&
                        (EX != kEpiCheby || (epi.ldo % 4 == 0 && aligned(epi.cto, 16) && epi.ldr % 4 == 0 &&
                                             epi.r_stride % 4 == 0 && aligned(epi.R, 16)));
        if (ok) lr = cand;
    }
    const int ns = (!lr && d <= 32 && !(flags & SRG_SPMM_WIDE_ROWS)) ? (d <= 1 ? 1 : d <= 2 ? 2 : d <= 4 ? 4 : d <= 8 ? 8 : d <= 16 ? 16 : 32) : 0;
    const int64_t rows_per_block = (int64_t)kWavesPerBlock * (ns ? 64 / ns : lr ? lr : 1);
    // XCD-aware slice waves (k_spmm<..., XH>) with packed light rows, 2 / 4 / 8 slices
    const bool xh = lr && (n_slices == 2 || n_slices == 4 || n_slices == 8);
    int nb_heavy_launch = nb_heavy;
    if (xh) {
        const int64_t per = 8 / n_slices;
        const int64_t bh = ((n_heavy + kWavesPerBlock - 1) / kWavesPerBlock + per - 1) / per * 8;
        if (bh > INT32_MAX) return fail(SRG_ERR_INVALID, "grid too large");
        nb_heavy_launch = (int)bh;
    }
    const int64_t blocks = nb_heavy_launch + (n_light + rows_per_block - 1) / rows_per_block;
    if (blocks > INT32_MAX) return fail(SRG_ERR_INVALID, "grid too large");
    int vec = pick_vec(d, ldx, ldy, X, Y, sizeof(float));
    if (epi.agg) vec = std::min(vec, pick_vec(d, epi.lda, epi.lda, epi.agg, epi.agg, sizeof(float)));
    if (EX == kEpiCheby) {
        vec = std::min(vec, pick_vec(d, epi.ldo, epi.ldr, epi.cto, epi.R, sizeof(float)));
        while (vec > 1 && epi.r_stride % vec) vec /= 2;
    }
    const int nr = (int)m_rows, nh = (int)n_heavy;
    const int pu = (flags & SRG_SPMM_PACKED_U2) ? 2 : kPackedU;
    const unsigned shm = (unsigned)spmm_lds_bytes(flags);
    for (int64_t b0 = 0; b0 < blocks; b0 += kMaxLaunchBlocks) {
        const dim3 grid((unsigned)std::min<int64_t>(kMaxLaunchBlocks, blocks - b0));
        const int bb = (int)b0;
#define SRG_LAUNCH_SPMM(V, F, SF)                                                               \
    hipLaunchKernelGGL((k_spmm<V, kUnroll, kUnrollHeavy, F, SF, IP, 0, EX>), grid, dim3(kBlock), shm, s,   \
                       indptr, indices, vals, morder, nr, nh, n_slices, nb_heavy, X, ldx, Y, ldy, \
                       d, acc, nt, bb, epi)
        const bool full = d % (64 * vec) == 0;        // implies d % 32 == 0
#define SRG_LAUNCH_NARROW(NSV, SF)                                                                 \
    hipLaunchKernelGGL((k_spmm<1, kUnroll, kUnrollHeavy, false, SF, IP, NSV, EX>), grid, dim3(kBlock), shm, s, \
                       indptr, indices, vals, morder, nr, nh, n_slices, nb_heavy, X, ldx, Y, ldy,     \
                       d, acc, nt, bb, epi)
#define SRG_LAUNCH_PACKED(LRV, LQV, UV)                                                              \
    do {                                                                                              \
        if (xh)                                                                                       \
            hipLaunchKernelGGL((k_spmm<1, UV, (LRV < 8 ? kUnrollHeavyWide : kUnrollHeavy), false, true, IP, 0, EX, LRV, LQV, true>), grid, dim3(kBlock), \
                               shm, s, indptr, indices, vals, morder, nr, nh, n_slices, nb_heavy_launch, X, ldx, Y, ldy, \
                               d, acc, nt, bb, epi);                                                  \
        else                                                                                          \
            hipLaunchKernelGGL((k_spmm<1, UV, (LRV < 8 ? kUnrollHeavyWide : kUnrollHeavy), false, true, IP, 0, EX, LRV, LQV>), grid, dim3(kBlock), shm, s, \
                               indptr, indices, vals, morder, nr, nh, n_slices, nb_heavy, X, ldx, Y, ldy, \
                               d, acc, nt, bb, epi);                                                  \
    } while (0)
#define SRG_LAUNCH_PACKED_U(LRV, LQV)                                                                 \
    do {                                                                                              \
        if (pu == 2) SRG_LAUNCH_PACKED(LRV, LQV, 2);                                                  \
        else SRG_LAUNCH_PACKED(LRV, LQV, 4);                                                          \
    } while (0)
        // packed_rows_for gives two 16-byte chunks per lane (LQ = 2) at d = 64 / 128 / 256
        if (lr == 2) {
            SRG_LAUNCH_PACKED_U(2, 2);
        } else if (lr == 4) {
            SRG_LAUNCH_PACKED_U(4, 2);
        } else if (lr == 8) {
            SRG_LAUNCH_PACKED_U(8, 2);
        } else if (ns == 32) {
            if (sfull) SRG_LAUNCH_NARROW(32, true);
            else SRG_LAUNCH_NARROW(32, false);
        } else if (ns == 16) {
            SRG_LAUNCH_NARROW(16, false);
        } else if (ns == 8) {
            SRG_LAUNCH_NARROW(8, false);
        } else if (ns == 4) {
            SRG_LAUNCH_NARROW(4, false);
        } else if (ns == 2) {
            SRG_LAUNCH_NARROW(2, false);
        } else if (ns == 1) {
            SRG_LAUNCH_NARROW(1, false);
        } else if (vec == 4) {
            if (full) SRG_LAUNCH_SPMM(4, true, true);
            else if (sfull) SRG_LAUNCH_SPMM(4, false, true);
            else SRG_LAUNCH_SPMM(4, false, false);
        } else if (vec == 2) {
            if (full) SRG_LAUNCH_SPMM(2, true, true);
            else if (sfull) SRG_LAUNCH_SPMM(2, false, true);
            else SRG_LAUNCH_SPMM(2, false, false);
        } else {
            if (full) SRG_LAUNCH_SPMM(1, true, true);
            else if (sfull) SRG_LAUNCH_SPMM(1, false, true);
            else SRG_LAUNCH_SPMM(1, false, false);
        }
#undef SRG_LAUNCH_SPMM
#undef SRG_LAUNCH_NARROW
#undef SRG_LAUNCH_PACKED
#undef SRG_LAUNCH_PACKED_U
        SRG_HIP_CHECK(hipGetLastError());
    }
    if (ss && !(flags & SRG_SPMM_HUB_NOJOIN)) SRG_HIP_CHECK(hipStreamWaitEvent(s, ss->join, 0));   // join
    return SRG_OK;
}

int check_spmm_args(const void* indptr, const void* indices, const void* vals, int64_t n_rows,
                    const void* X, int64_t ldx, const void* Y, int64_t ldy, int d)
{
    if (n_rows < 0 || n_rows > INT32_MAX - 64)
        return fail(SRG_ERR_INVALID, "n_rows=%lld out of range [0, 2^31-64)", (long long)n_rows);
    if (d < 0) return fail(SRG_ERR_INVALID, "d=%d < 0", d);
    if (ldx < d || ldy < d)
        return fail(SRG_ERR_INVALID, "leading dimensions (ldx=%lld, ldy=%lld) < d=%d",
                    (long long)ldx, (long long)ldy, d);
    if (n_rows > 0 && d > 0 && (!indptr || !Y))
        return fail(SRG_ERR_INVALID, "null indptr or Y");
    (void)indices; (void)vals; (void)X;
    return SRG_OK;
}

// The fused step's mode and coefficients (cheby_epi_at): coef_prev holds c0 per scale (INIT) or c0 then c1
// per scale (STEP_FIRST), coef c1 (INIT) or ck (STEP, STEP_FIRST); INIT_T takes neither; | SRG_CHEBY_NO_T.
template <typename T>
int cheby_setup(int mode, const T* coef_prev, const T* coef, int n_scales, const void* To, ChebyCoef<T>& cf)
{
    const int m = mode & ~SRG_CHEBY_NO_T;
    if (m != SRG_CHEBY_INIT && m != SRG_CHEBY_STEP && m != SRG_CHEBY_INIT_T && m != SRG_CHEBY_STEP_FIRST)
        return fail(SRG_ERR_INVALID, "cheby mode %d", mode);
    if (n_scales < 1 || n_scales > 8) return fail(SRG_ERR_INVALID, "n_scales=%d not in [1,8]", n_scales);
    const bool needs_r = m != SRG_CHEBY_INIT_T;
    if ((needs_r && !coef) || ((m == SRG_CHEBY_INIT || m == SRG_CHEBY_STEP_FIRST) && !coef_prev))
        return fail(SRG_ERR_INVALID, "null coefficient array");
    if ((m == SRG_CHEBY_STEP || m == SRG_CHEBY_STEP_FIRST) && !To) return fail(SRG_ERR_INVALID, "null To for a step");
    for (int i = 0; i < 8; ++i) {
        const bool on = i < n_scales;
        cf.prev[i] = ((m == SRG_CHEBY_INIT || m == SRG_CHEBY_STEP_FIRST) && on) ? T(0.5) * coef_prev[i] : T(0);
        cf.mid[i] = (m == SRG_CHEBY_STEP_FIRST && on) ? coef_prev[n_scales + i] : T(0);
        cf.cur[i] = (needs_r && on) ? coef[i] : T(0);
    }
    return SRG_OK;
}

// n_hub (fp64 only): the first n_hub rows of `order` run as k_cheby_hub64 workgroups on the hub side
// stream beside the row waves of the others (joined before the call returns to the stream's order;
// with SRG_CHEBY_HUB_NOJOIN in mode, left running for srg_hub_join: later launches on the stream run
// beside them)
template <typename T>
int launch_cheby(const int64_t* indptr, const int32_t* indices, const T* vals, int64_t n_rows,
                 const int32_t* order, const T* Tc, const T* To, T* Tn, int64_t ld, int d, int mode,
                 T a1, T a2, const T* coef_prev, const T* coef, int n_scales, T* R, int64_t r_stride,
                 hipStream_t s, int64_t n_hub = 0)
{
    bool nojoin = false;
    if constexpr (sizeof(T) == 8) {
        nojoin = (mode & SRG_CHEBY_HUB_NOJOIN) != 0;
        mode &= ~SRG_CHEBY_HUB_NOJOIN;
    }
    ChebyCoef<T> cf;
    int rc = cheby_setup<T>(mode, coef_prev, coef, n_scales, To, cf);
    if (rc) return rc;
    rc = check_spmm_args(indptr, indices, vals, n_rows, Tc, ld, Tn, ld, d);
    if (rc) return rc;
    if (r_stride < n_rows * ld && n_scales > 1)
        return fail(SRG_ERR_INVALID, "r_stride too small for stacked scale panels");
    if (n_hub < 0 || n_hub > n_rows || (n_hub > 0 && !order))
        return fail(SRG_ERR_INVALID, "n_hub=%lld needs a row_order and <= n_rows", (long long)n_hub);
    if (n_rows == 0 || d == 0) return ok();
    // hub workgroups gather 16-byte pieces (two columns) of Tc's rows
    if (sizeof(T) != 8 || d % 2 || ld % 2 || !aligned(Tc, 16)) n_hub = 0;
    const int n_slices = (d + kHub64Cols - 1) / kHub64Cols;
    if (n_hub * n_slices > INT32_MAX - 64) return fail(SRG_ERR_INVALID, "too many hub slices");
    SideStream* ss = nullptr;
    std::unique_lock<std::mutex> side_lock(g_side_mu, std::defer_lock);
    if constexpr (sizeof(T) == 8) {
        if (n_hub > 0) {   // fork: the hub rows' workgroups beside the row waves
            side_lock.lock();
            int rc = side_stream_locked(s, &ss);
            if (rc) return rc;
            SRG_HIP_CHECK(hipEventRecord(ss->fork, s));
            SRG_HIP_CHECK(hipStreamWaitEvent(ss->stream, ss->fork, 0));
            launch_hub64(n_hub * n_slices, ss->stream, indptr, indices, vals, order, n_slices, Tc, To, Tn, ld, d, mode,
                         a1, a2, cf, n_scales, R, r_stride);
            SRG_HIP_CHECK(hipGetLastError());
            SRG_HIP_CHECK(hipEventRecord(ss->join, ss->stream));
            ss->pending = nojoin;
            hipLaunchKernelGGL(k_dispatch_delay, dim3(1), dim3(64), 0, s, kHubDelayUs);
            SRG_HIP_CHECK(hipGetLastError());
        }
    }
    order = order ? order + n_hub : nullptr;
    n_rows -= n_hub;
    const int64_t blocks = (n_rows + kWavesPerBlock - 1) / kWavesPerBlock;
    const int vec = pick_vec(d, ld, ld, Tc, Tn, sizeof(T)) >= 2 && aligned(R, 2 * sizeof(T)) &&
                            (r_stride % 2 == 0) && (To == nullptr || aligned(To, 2 * sizeof(T)))
                        ? 2
                        : 1;
    const int nr = (int)n_rows;
    for (int64_t b0 = 0; b0 < blocks; b0 += kMaxLaunchBlocks) {
        const dim3 grid((unsigned)std::min<int64_t>(kMaxLaunchBlocks, blocks - b0));
        if (vec == 2)
            hipLaunchKernelGGL((k_cheby<T, 2, kUnroll>), grid, dim3(kBlock), 0, s, indptr, indices,
                               vals, order, nr, Tc, To, Tn, ld, d, mode, a1, a2, cf, n_scales, R,
                               r_stride, (int)b0);
        else
            hipLaunchKernelGGL((k_cheby<T, 1, kUnroll>), grid, dim3(kBlock), 0, s, indptr, indices,
                               vals, order, nr, Tc, To, Tn, ld, d, mode, a1, a2, cf, n_scales, R,
                               r_stride, (int)b0);
        SRG_HIP_CHECK(hipGetLastError());
    }
    SRG_HIP_CHECK(hipGetLastError());
    if (ss && !nojoin) SRG_HIP_CHECK(hipStreamWaitEvent(s, ss->join, 0));   // join
    return ok();
}

// ------------------------------------------------------------------------------------------------
// host-compat staging: grow-only device buffers reused across calls (the reference calls the
// product once per hop from Python, utils.py:45)
// ------------------------------------------------------------------------------------------------
struct Staging {
    std::mutex mu;
    void* buf[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    size_t cap[5] = {0, 0, 0, 0, 0};
    int device[5] = {-1, -1, -1, -1, -1};
    hipStream_t stream = nullptr;
    int stream_device = -1;
};
Staging g_stage;

int stage_reserve(int slot, size_t bytes, int dev)
{
    if (g_stage.cap[slot] >= bytes && g_stage.device[slot] == dev) return SRG_OK;
    if (g_stage.buf[slot]) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(g_stage.device[slot]);
        (void)hipFree(g_stage.buf[slot]);
        (void)hipSetDevice(cur);
        g_stage.buf[slot] = nullptr;
        g_stage.cap[slot] = 0;
    }
    size_t want = std::max<size_t>(bytes, 256);
    if (hipMalloc(&g_stage.buf[slot], want) != hipSuccess) {
        g_stage.buf[slot] = nullptr;
        (void)hipGetLastError();
        return fail(SRG_ERR_ALLOC, "hipMalloc(%zu) failed", want);
    }
    g_stage.cap[slot] = want;
    g_stage.device[slot] = dev;
    return SRG_OK;
}

// answer (+)= A * mat on the GPU with host buffers.  overwrite: cuSPARSE beta = 0 semantics.
int host_compat_spmm(float* answer, const float* data, const int* indices, const int* indptr,
                     const float* mat, int mat_row, int mat_col, bool overwrite, int64_t nnz_hint)
{
    if (mat_row < 0 || mat_col < 0)
        return fail(SRG_ERR_INVALID, "mat_row=%d mat_col=%d", mat_row, mat_col);
    if (mat_row == 0 || mat_col == 0) return ok();
    if (!answer || !indptr || !mat) return fail(SRG_ERR_INVALID, "null host pointer");
    const int64_t nnz = indptr[mat_row];
    if (indptr[0] != 0 || nnz < 0) return fail(SRG_ERR_INVALID, "indptr[0]=%d indptr[n]=%lld", indptr[0], (long long)nnz);
    if (nnz_hint >= 0 && nnz_hint != nnz)
        return fail(SRG_ERR_INVALID, "data_nnz=%lld != indptr[mat_row]=%lld", (long long)nnz_hint, (long long)nnz);
    for (int i = 0; i < mat_row; ++i)
        if (indptr[i + 1] < indptr[i]) return fail(SRG_ERR_INVALID, "indptr decreases at row %d", i);
    if (nnz > 0 && (!indices || !data)) return fail(SRG_ERR_INVALID, "null indices/data");
    for (int64_t j = 0; j < nnz; ++j)
        if (indices[j] < 0 || indices[j] >= mat_row)
            return fail(SRG_ERR_INVALID, "column id %d at %lld outside [0, %d)", indices[j], (long long)j, mat_row);

    std::lock_guard<std::mutex> lock(g_stage.mu);
    int dev = 0;
    SRG_HIP_CHECK(hipGetDevice(&dev));
    if (!g_stage.stream || g_stage.stream_device != dev) {
        SRG_HIP_CHECK(hipStreamCreateWithFlags(&g_stage.stream, hipStreamNonBlocking));
        g_stage.stream_device = dev;
    }
    hipStream_t s = g_stage.stream;
    const size_t panel = (size_t)mat_row * (size_t)mat_col * sizeof(float);
    int rc;
    if ((rc = stage_reserve(0, (size_t)(mat_row + 1) * sizeof(int), dev))) return rc;
    if ((rc = stage_reserve(1, (size_t)nnz * sizeof(int), dev))) return rc;
    if ((rc = stage_reserve(2, (size_t)nnz * sizeof(float), dev))) return rc;
    if ((rc = stage_reserve(3, panel, dev))) return rc;
    if ((rc = stage_reserve(4, panel, dev))) return rc;
    int* d_ptr = static_cast<int*>(g_stage.buf[0]);
    int* d_idx = static_cast<int*>(g_stage.buf[1]);
    float* d_val = static_cast<float*>(g_stage.buf[2]);
    float* d_x = static_cast<float*>(g_stage.buf[3]);
    float* d_y = static_cast<float*>(g_stage.buf[4]);
    SRG_HIP_CHECK(hipMemcpyAsync(d_ptr, indptr, (size_t)(mat_row + 1) * sizeof(int), hipMemcpyHostToDevice, s));
    if (nnz > 0) {
        SRG_HIP_CHECK(hipMemcpyAsync(d_idx, indices, (size_t)nnz * sizeof(int), hipMemcpyHostToDevice, s));
        SRG_HIP_CHECK(hipMemcpyAsync(d_val, data, (size_t)nnz * sizeof(float), hipMemcpyHostToDevice, s));
    }
    SRG_HIP_CHECK(hipMemcpyAsync(d_x, mat, panel, hipMemcpyHostToDevice, s));
    uint32_t flags = 0;
    if (!overwrite) {
        SRG_HIP_CHECK(hipMemcpyAsync(d_y, answer, panel, hipMemcpyHostToDevice, s));
        flags |= SRG_SPMM_ACCUMULATE;
    }
    rc = launch_spmm<int>(d_ptr, d_idx, d_val, mat_row, nullptr, 0, 0, d_x, mat_col, d_y, mat_col, mat_col, flags, s);
    if (rc) return rc;
    SRG_HIP_CHECK(hipMemcpyAsync(answer, d_y, panel, hipMemcpyDeviceToHost, s));
    SRG_HIP_CHECK(hipStreamSynchronize(s));
    return ok();
}

}  // namespace

// ================================================================================================
// C ABI
// ================================================================================================
extern "C" {

void FloatCSRMulDenseOMP(float answer[], float data[], int indices[], int indptr[], float mat[],
                         int mat_row, int mat_col)
{
    (void)host_compat_spmm(answer, data, indices, indptr, mat, mat_row, mat_col, false, -1);
}

int FloatCSRMulDense(float answer[], int data_nnz, float data[], int indices[], int indptr[],
                     float mat[], int mat_row, int mat_col)
{
    return host_compat_spmm(answer, data, indices, indptr, mat, mat_row, mat_col, true, data_nnz) == SRG_OK ? 0 : 1;
}

int srg_spmm_csr_f32(const int64_t* indptr, const int32_t* indices, const float* values,
                     int64_t n_rows, const int32_t* row_order, int64_t n_hub, int64_t n_heavy,
                     const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t d, uint32_t flags,
                     void* stream)
{
    SRG_DEVICE_GUARD(stream);
    int rc = check_spmm_args(indptr, indices, values, n_rows, X, ldx, Y, ldy, d);
    if (rc) return rc;
    rc = launch_spmm<int64_t>(indptr, indices, values, n_rows, row_order, n_hub, n_heavy, X, ldx, Y, ldy, d, flags,
                              static_cast<hipStream_t>(stream));
    return rc ? rc : ok();
}

int srg_spmm_agg_f32(const int64_t* indptr, const int32_t* indices, const float* values,
                     int64_t n_rows, const int32_t* row_order, int64_t n_hub, int64_t n_heavy,
                     const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t d, uint32_t flags,
                     float* agg, int64_t lda, float w, int agg_init, void* stream)
{
    SRG_DEVICE_GUARD(stream);
    int rc = check_spmm_args(indptr, indices, values, n_rows, X, ldx, Y, ldy, d);
    if (rc) return rc;
    if (n_rows > 0 && d > 0 && (!agg || lda < d))
        return fail(SRG_ERR_INVALID, "aggregation panel: agg=%p lda=%lld < d=%d", (void*)agg, (long long)lda, d);
    if (agg && agg == Y) return fail(SRG_ERR_INVALID, "agg must not alias Y");
    rc = launch_spmm<int64_t>(indptr, indices, values, n_rows, row_order, n_hub, n_heavy, X, ldx, Y, ldy, d, flags,
                              static_cast<hipStream_t>(stream), Epi{agg, lda, w, agg_init ? 1 : 0});
    return rc ? rc : ok();
}

int srg_spmm_span_f32(const int64_t* row_beg, const int64_t* row_end, const int32_t* indices,
                      const float* values, int64_t n_rows, const int32_t* row_order, int64_t n_hub,
                      int64_t n_heavy, const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t d,
                      uint32_t flags, float* agg, int64_t lda, float w, int agg_init, void* stream)
{
    SRG_DEVICE_GUARD(stream);
    int rc = check_spmm_args(row_beg, indices, values, n_rows, X, ldx, Y, ldy, d);
    if (rc) return rc;
    if (n_rows > 0 && d > 0 && !row_end) return fail(SRG_ERR_INVALID, "null row_end");
    if (agg && (lda < d || agg == Y))
        return fail(SRG_ERR_INVALID, "aggregation panel: lda=%lld < d=%d or agg aliases Y", (long long)lda, d);
    Epi e{};
    e.agg = agg;
    e.lda = lda;
    e.w = w;
    e.init = agg_init ? 1 : 0;
    e.row_end = row_end;
    rc = launch_spmm<int64_t, kEpiSpan>(row_beg, indices, values, n_rows, row_order, n_hub, n_heavy, X, ldx, Y, ldy,
                                        d, flags, static_cast<hipStream_t>(stream), e);
    return rc ? rc : ok();
}

int srg_spmm_cheby_f32(const int64_t* indptr, const int32_t* indices, const float* values,
                       int64_t n_rows, const int32_t* row_order, int64_t n_hub, int64_t n_heavy,
                       const float* Tc, int64_t ldc, float* Tn, int64_t ldn, int32_t d, uint32_t flags,
                       int mode, float a1, float a2, const float* To, int64_t ldo, const float* coef_prev,
                       const float* coef, int32_t n_scales, float* R, int64_t ldr, int64_t r_stride,
                       void* stream)
{
    SRG_DEVICE_GUARD(stream);
    int rc = check_spmm_args(indptr, indices, values, n_rows, Tc, ldc, Tn, ldn, d);
    if (rc) return rc;
    if (mode != SRG_CHEBY_INIT && mode != SRG_CHEBY_STEP) return fail(SRG_ERR_INVALID, "cheby mode %d", mode);
    if (n_scales < 1 || n_scales > 8) return fail(SRG_ERR_INVALID, "n_scales=%d not in [1,8]", n_scales);
    if (!coef || (mode == SRG_CHEBY_INIT && !coef_prev)) return fail(SRG_ERR_INVALID, "null coefficient array");
    if (flags & SRG_SPMM_ACCUMULATE) return fail(SRG_ERR_INVALID, "the Chebyshev epilogue starts every chain from 0");
    if (n_rows == 0 || d == 0) return ok();
    if (!R || ldr < d) return fail(SRG_ERR_INVALID, "R=%p ldr=%lld < d=%d", (void*)R, (long long)ldr, d);
    if (n_scales > 1 && r_stride < n_rows * ldr && r_stride > -n_rows * ldr)
        return fail(SRG_ERR_INVALID, "r_stride overlaps the scale panels");
    if (mode == SRG_CHEBY_STEP && (!To || ldo < d))
        return fail(SRG_ERR_INVALID, "step needs To with ldo >= d (To=%p ldo=%lld)", (const void*)To, (long long)ldo);
    if (Tn == Tc) return fail(SRG_ERR_INVALID, "Tn must not alias Tc (its rows are gathered)");
    if (mode == SRG_CHEBY_STEP && To == Tn && ldo != ldn)
        return fail(SRG_ERR_INVALID, "Tn may alias To only with the same leading dimension");
    if (R == Tn || R == Tc || (mode == SRG_CHEBY_STEP && R == To)) return fail(SRG_ERR_INVALID, "R must not alias a T panel");
    Epi e{};
    e.cto = mode == SRG_CHEBY_STEP ? To : nullptr;
    e.ldo = mode == SRG_CHEBY_STEP ? ldo : 0;
    e.R = R;
    e.ldr = ldr;
    e.r_stride = r_stride;
    e.cmode = mode;
    e.ns = n_scales;
    e.a1 = a1;
    e.a2 = a2;
    for (int i = 0; i < 8; ++i) {
        e.cf.prev[i] = (mode == SRG_CHEBY_INIT && i < n_scales) ? 0.5f * coef_prev[i] : 0.0f;
        e.cf.cur[i] = i < n_scales ? coef[i] : 0.0f;
    }
    rc = launch_spmm<int64_t, kEpiCheby>(indptr, indices, values, n_rows, row_order, n_hub, n_heavy, Tc, ldc, Tn, ldn,
                                         d, flags, static_cast<hipStream_t>(stream), e);
    return rc ? rc : ok();
}

int srg_propagate_khop_f32(const int64_t* indptr, const int32_t* indices, const float* values,
                           int64_t n_rows, const int32_t* row_order, int64_t n_hub,
                           int64_t n_heavy, float* const* panels,
                           int64_t ld, int32_t d, int32_t K, uint32_t flags, void* stream)
{
    SRG_DEVICE_GUARD(stream);
    if (K < 0) return fail(SRG_ERR_INVALID, "K=%d < 0", K);
    if (K > 0 && !panels) return fail(SRG_ERR_INVALID, "null panels");
    for (int k = 0; k <= K; ++k)
        if (!panels[k] && n_rows > 0 && d > 0) return fail(SRG_ERR_INVALID, "panels[%d] is null", k);
    int rc = check_spmm_args(indptr, indices, values, n_rows, panels ? panels[0] : nullptr, ld,
                             panels ? panels[0] : nullptr, ld, d);
    if (rc) return rc;
    const uint32_t f = flags & ~SRG_SPMM_ACCUMULATE;
    if (!row_order && n_hub == 0 && n_heavy == 0 && K > 0 && n_rows > 0 && d > 0 &&
        !(f & ~(SRG_SPMM_NT_STORE | SRG_SPMM_FAST))) {
        // no schedule: the hops run through a plan made for them (srg_plan.hip), freed after them.  Without
        // a schedule there were never hub rows here, so FAST (which only re-associates hub rows) changed
        // nothing: the implicit plan then has no hub rows either, and the bits stay exact
        srg_plan* P = nullptr;
        const int64_t hub_t = (f & SRG_SPMM_FAST) ? SRG_PLAN_NONE : SRG_PLAN_AUTO;
        rc = srg_plan_build(indptr, indices, values, n_rows, d, K, 0, hub_t, SRG_PLAN_AUTO, 0, stream, &P);
        if (rc) return rc;
        rc = srg_plan_propagate_f32(P, panels, ld, d, K, f, stream);
        const int rc2 = srg_plan_destroy(P, stream);
        return rc ? rc : rc2;
    }
    for (int k = 1; k <= K; ++k) {
        rc = launch_spmm<int64_t>(indptr, indices, values, n_rows, row_order, n_hub, n_heavy, panels[k - 1], ld,
                                  panels[k], ld, d, f, static_cast<hipStream_t>(stream));
        if (rc) return rc;
    }
    return ok();
}

// one hop of a launch list: X (ldx) -> Y (ldy); launch i carries the aggregation epilogue (agg = (init ?
// 0 : agg) + w * Y, at the end of each of its rows' chains) when agg && agg_on[i]; with join_hub the
// hub side stream is joined into `s` after the hop
static int run_hop_launches(const srg_hop_launch* launches, int32_t n_launch, bool join_hub, const float* X,
                            int64_t ldx, float* Y, int64_t ldy, int32_t d, const uint8_t* agg_on, float* agg,
                            int64_t lda, float w, int agg_init, hipStream_t s, int dev)
{
    for (int i = 0; i < n_launch; ++i) {
        const srg_hop_launch& L = launches[i];
        Epi e{};
        if (agg && agg_on && agg_on[i]) {
            e.agg = agg;
            e.lda = lda;
            e.w = w;
            e.init = agg_init ? 1 : 0;
        }
        int rc;
        if (L.row_end) {
            e.row_end = L.row_end;
            // the light rows' slots count from the first non-hub row of the schedule
            e.slot_beg = L.slot_beg ? L.slot_beg + L.n_hub : nullptr;
            e.slot_end = L.slot_beg ? L.slot_end + L.n_hub : nullptr;
            rc = launch_spmm<int64_t, kEpiSpan>(L.row_beg, L.indices, L.values, L.n_rows, L.row_order, L.n_hub,
                                                L.n_heavy, X, ldx, Y, ldy, d, L.flags, s, e);
        } else {
            rc = launch_spmm<int64_t>(L.row_beg, L.indices, L.values, L.n_rows, L.row_order, L.n_hub, L.n_heavy,
                                      X, ldx, Y, ldy, d, L.flags, s, e);
        }
        if (rc) return rc;
    }
    if (join_hub) {
        std::lock_guard<std::mutex> lock(g_side_mu);
        auto it = g_side.find(std::make_pair(dev, s));
        if (it != g_side.end() && it->second.pending) {
            SRG_HIP_CHECK(hipStreamWaitEvent(s, it->second.join, 0));
            it->second.pending = false;
        }
    }
    return SRG_OK;
}

static int check_launches(const srg_hop_launch* launches, int32_t n_launch, const float* X, int64_t ldx,
                          const float* Y, int64_t ldy, int32_t d)
{
    for (int i = 0; i < n_launch; ++i) {
        const srg_hop_launch& L = launches[i];
        int rc = check_spmm_args(L.row_beg, L.indices, L.values, L.n_rows, X, ldx, Y, ldy, d);
        if (rc) return rc;
        if (L.n_rows > 0 && L.n_hub + L.n_heavy > 0 && !L.row_order)
            return fail(SRG_ERR_INVALID, "launch %d: hub / heavy rows need a row_order", i);
        if ((L.slot_beg != nullptr) != (L.slot_end != nullptr) || (L.slot_beg && !L.row_end))
            return fail(SRG_ERR_INVALID, "launch %d: slot_beg / slot_end come together, with row_end", i);
    }
    return SRG_OK;
}

int srg_propagate_plan_f32(const srg_hop_launch* launches, int32_t n_launch, int32_t join_hub,
                           float* const* panels, int64_t ld, int32_t d, int32_t K, void* stream)
{
    SRG_DEVICE_GUARD(stream);
    if (K < 0 || n_launch < 0) return fail(SRG_ERR_INVALID, "K=%d / n_launch=%d < 0", K, n_launch);
    if (K == 0 || n_launch == 0) return ok();
    if (!launches || !panels) return fail(SRG_ERR_INVALID, "null launches or panels");
    for (int k = 0; k <= K; ++k)
        if (!panels[k] && d > 0) return fail(SRG_ERR_INVALID, "panels[%d] is null", k);
    int rc = check_launches(launches, n_launch, panels[0], ld, panels[0], ld, d);
    if (rc) return rc;
    for (int i = 0; i < n_launch; ++i) {
        // without the per-hop join, hop k's hub rows would still run on the side stream while hop
        // k+1's launches on `stream` read panels[k]: a data race
        const srg_hop_launch& L = launches[i];
        if (!join_hub && K > 1 && L.n_hub > 0 && (L.flags & SRG_SPMM_HUB_NOJOIN))
            return fail(SRG_ERR_INVALID, "launch %d: HUB_NOJOIN hub rows over K=%d hops need join_hub", i, K);
    }
    const hipStream_t s = static_cast<hipStream_t>(stream);
    for (int k = 1; k <= K; ++k) {
        rc = run_hop_launches(launches, n_launch, join_hub != 0, panels[k - 1], ld, panels[k], ld, d, nullptr, nullptr,
                              0, 0.0f, 0, s, guard_.dev);
        if (rc) return rc;
    }
    return ok();
}

// srg_plan.hip's single hop (srg_plan_hop_f32): the launches of one hop between panels of their own
// leading dimensions, the aggregation epilogue on the launches agg_on names (checked here)
__attribute__((visibility("hidden"))) int srg_run_plan_hop(const srg_hop_launch* launches, int32_t n_launch,
                                                           int32_t join_hub, const float* X, int64_t ldx, float* Y,
                                                           int64_t ldy, int32_t d, const uint8_t* agg_on, float* agg,
                                                           int64_t lda, float w, int32_t agg_init, void* stream)
{
    SRG_DEVICE_GUARD(stream);
    if (n_launch <= 0) return ok();
    int rc = check_launches(launches, n_launch, X, ldx, Y, ldy, d);
    if (rc) return rc;
    if (X == Y) return fail(SRG_ERR_INVALID, "Y must not alias X (its rows are gathered)");
    if (agg && (lda < d || agg == Y || agg == X))
        return fail(SRG_ERR_INVALID, "aggregation panel: lda=%lld < d=%d or agg aliases X / Y", (long long)lda, d);
    rc = run_hop_launches(launches, n_launch, join_hub != 0, X, ldx, Y, ldy, d, agg_on, agg, lda, w, agg_init,
                          static_cast<hipStream_t>(stream), guard_.dev);
    return rc ? rc : ok();
}

int srg_cheby_step_f64(const int64_t* indptr, const int32_t* indices, const double* values,
                       int64_t n_rows, const int32_t* row_order, const double* Tc,
                       const double* To, double* Tn, int64_t ld, int32_t d, int mode, double a1,
                       double a2, const double* coef_prev, const double* coef, int32_t n_scales,
                       double* R, int64_t r_stride, void* stream)
{
    if (mode & SRG_CHEBY_HUB_NOJOIN) return fail(SRG_ERR_INVALID, "cheby mode %d: HUB_NOJOIN needs the hub entry", mode);
    SRG_DEVICE_GUARD(stream);
    return launch_cheby<double>(indptr, indices, values, n_rows, row_order, Tc, To, Tn, ld, d, mode,
                                a1, a2, coef_prev, coef, n_scales, R, r_stride,
                                static_cast<hipStream_t>(stream));
}

int srg_cheby_step_hub_f64(const int64_t* indptr, const int32_t* indices, const double* values,
                           int64_t n_rows, const int32_t* row_order, int64_t n_hub, const double* Tc,
                           const double* To, double* Tn, int64_t ld, int32_t d, int mode, double a1,
                           double a2, const double* coef_prev, const double* coef, int32_t n_scales,
                           double* R, int64_t r_stride, void* stream)
{
    SRG_DEVICE_GUARD(stream);
    return launch_cheby<double>(indptr, indices, values, n_rows, row_order, Tc, To, Tn, ld, d, mode,
                                a1, a2, coef_prev, coef, n_scales, R, r_stride,
                                static_cast<hipStream_t>(stream), n_hub);
}

// Library-internal (srg_plan.hip's srg_plan_cheby_step_f64): one fp64 Chebyshev step over a plan's
// launches.  roles[i]: SRG_CHEBY64_FIRST / _LAST bits (the block where launch i's rows' chains start /
// end), or SRG_CHEBY64_HUBS (the whole hub rows: k_cheby_hub64 on the hub side stream, joined at the
// end of the step).  A launch without spans by slot is the one-launch plan's CSR launch: srg_cheby_
// step_hub_f64 over its schedule.  `values` are the fp64 values at the plan's entry positions.
__attribute__((visibility("hidden"))) int srg_run_plan_cheby_f64(const srg_hop_launch* launches, const uint8_t* roles, int32_t n_launch, const int64_t* indptr,
                           const int32_t* indices, const double* values, const double* Tc, const double* To,
                           double* Tn, int64_t ld, int32_t d, int mode, double a1, double a2, const double* coef_prev,
                           const double* coef, int32_t n_scales, double* R, int64_t r_stride, void* stream)
{
    SRG_DEVICE_GUARD(stream);
    const hipStream_t s = static_cast<hipStream_t>(stream);
    ChebyCoef<double> cf;
    int rc0 = cheby_setup<double>(mode, coef_prev, coef, n_scales, To, cf);
    if (rc0) return rc0;
    if (d < 0 || ld < d) return fail(SRG_ERR_INVALID, "d=%d, ld=%lld", d, (long long)ld);
    if (n_launch == 1 && !launches[0].slot_beg) {
        const srg_hop_launch& L = launches[0];
        return launch_cheby<double>(indptr, indices, values, L.n_rows, L.row_order, Tc, To, Tn, ld, d, mode, a1, a2,
                                    coef_prev, coef, n_scales, R, r_stride, s, L.n_hub);
    }
    int64_t n_total = 0;
    for (int i = 0; i < n_launch; ++i) {
        const srg_hop_launch& L = launches[i];
        if (!L.slot_beg || !L.slot_end || (L.n_rows > 0 && !L.row_order))
            return fail(SRG_ERR_INVALID, "launch %d: a blocked fp64 step reads spans by slot", i);
        if (roles[i] & (SRG_CHEBY64_LAST | SRG_CHEBY64_HUBS)) n_total += L.n_rows;
    }
    if (d == 0 || n_total == 0) return ok();
    if (!Tc || !Tn || !R || !indices || !values) return fail(SRG_ERR_INVALID, "null panel or entry array");
    if (r_stride < n_total * ld && n_scales > 1) return fail(SRG_ERR_INVALID, "r_stride too small for stacked scale panels");
    const bool v2 = d % 2 == 0 && ld % 2 == 0 && aligned(Tc, 16) && aligned(Tn, 16) && aligned(R, 16) &&
                    r_stride % 2 == 0 && (To == nullptr || aligned(To, 16));
    const int n_slices = (d + kHub64Cols - 1) / kHub64Cols;
    SideStream* ss = nullptr;
    std::unique_lock<std::mutex> side_lock(g_side_mu, std::defer_lock);
    for (int i = 0; i < n_launch; ++i) {
        const srg_hop_launch& L = launches[i];
        if (L.n_rows <= 0) continue;
        int role = roles[i];
        if (role == SRG_CHEBY64_HUBS) {
            if (v2 && L.n_rows * n_slices <= INT32_MAX - 64) {   // fork: the hub workgroups beside the blocks
                side_lock.lock();
                int rc = side_stream_locked(s, &ss);
                if (rc) return rc;
                SRG_HIP_CHECK(hipEventRecord(ss->fork, s));
                SRG_HIP_CHECK(hipStreamWaitEvent(ss->stream, ss->fork, 0));
                launch_hub64(L.n_rows * n_slices, ss->stream, indptr, indices, values, L.row_order, n_slices, Tc, To,
                             Tn, ld, d, mode, a1, a2, cf, n_scales, R, r_stride);
                SRG_HIP_CHECK(hipGetLastError());
                SRG_HIP_CHECK(hipEventRecord(ss->join, ss->stream));
                hipLaunchKernelGGL(k_dispatch_delay, dim3(1), dim3(64), 0, s, kHubDelayUs);
                SRG_HIP_CHECK(hipGetLastError());
                continue;
            }
            role = SRG_CHEBY64_FIRST | SRG_CHEBY64_LAST;   // row waves over their whole spans
        }
        const int64_t blocks = (L.n_rows + kWavesPerBlock - 1) / kWavesPerBlock;
        const int nr = (int)L.n_rows;
        // (uncapped: 4 or 6 waves per SIMD measured 0.5-3 % slower, profiles/r06i_cheby64_plan_sweep.txt)
        for (int64_t b0 = 0; b0 < blocks; b0 += kMaxLaunchBlocks) {
            const dim3 grid((unsigned)std::min<int64_t>(kMaxLaunchBlocks, blocks - b0));
#define SRG_LAUNCH_BLK64(V, F, LA)                                                                                \
    hipLaunchKernelGGL((k_cheby_blk64<V, kUnroll, F, LA>), grid, dim3(kBlock), 0, s, L.slot_beg, L.slot_end,     \
                       L.row_order, nr, indices, values, Tc, To, Tn, ld, d, mode, a1, a2, cf, n_scales, R, r_stride, \
                       (int)b0)
#define SRG_LAUNCH_BLK64_V(F, LA)                  \
    do {                                           \
        if (v2) SRG_LAUNCH_BLK64(2, F, LA);        \
        else SRG_LAUNCH_BLK64(1, F, LA);           \
    } while (0)
            switch (role & (SRG_CHEBY64_FIRST | SRG_CHEBY64_LAST)) {
            case SRG_CHEBY64_FIRST | SRG_CHEBY64_LAST: SRG_LAUNCH_BLK64_V(true, true); break;
            case SRG_CHEBY64_FIRST: SRG_LAUNCH_BLK64_V(true, false); break;
            case SRG_CHEBY64_LAST: SRG_LAUNCH_BLK64_V(false, true); break;
            default: SRG_LAUNCH_BLK64_V(false, false); break;
            }
#undef SRG_LAUNCH_BLK64_V
#undef SRG_LAUNCH_BLK64
            SRG_HIP_CHECK(hipGetLastError());
        }
    }
    if (ss) SRG_HIP_CHECK(hipStreamWaitEvent(s, ss->join, 0));   // join
    return ok();
}

int srg_cheby_step_f32(const int64_t* indptr, const int32_t* indices, const float* values,
                       int64_t n_rows, const int32_t* row_order, const float* Tc, const float* To,
                       float* Tn, int64_t ld, int32_t d, int mode, float a1, float a2,
                       const float* coef_prev, const float* coef, int32_t n_scales, float* R,
                       int64_t r_stride, void* stream)
{
    SRG_DEVICE_GUARD(stream);
    return launch_cheby<float>(indptr, indices, values, n_rows, row_order, Tc, To, Tn, ld, d, mode,
                               a1, a2, coef_prev, coef, n_scales, R, r_stride,
                               static_cast<hipStream_t>(stream));
}

int srg_cheby_epilogue_f32(float* Tn, int64_t ldn, const float* Tc, int64_t ldc, const float* To,
                           int64_t ldo, int64_t n_rows, int32_t d, int mode, float a1, float a2,
                           const float* coef_prev, const float* coef, int32_t n_scales, float* R,
                           int64_t ldr, int64_t r_stride, void* stream)
{
    SRG_DEVICE_GUARD(stream);
    const int m = mode & ~SRG_CHEBY_NO_T;
    if (m != SRG_CHEBY_INIT && m != SRG_CHEBY_STEP && m != SRG_CHEBY_INIT_T && m != SRG_CHEBY_STEP_FIRST)
        return fail(SRG_ERR_INVALID, "cheby mode %d", mode);
    const bool init = m == SRG_CHEBY_INIT || m == SRG_CHEBY_INIT_T;
    const bool needs_r = m != SRG_CHEBY_INIT_T;
    if (n_scales < 1 || n_scales > 8) return fail(SRG_ERR_INVALID, "n_scales=%d not in [1,8]", n_scales);
    if ((needs_r && !coef) || ((m == SRG_CHEBY_INIT || m == SRG_CHEBY_STEP_FIRST) && !coef_prev))
        return fail(SRG_ERR_INVALID, "null coefficient array");
    if (n_rows < 0 || d < 0 || ldn < d || (needs_r && ldr < d) || (init ? ldc < d : ldo < d) ||
        (m == SRG_CHEBY_STEP_FIRST && ldc < d))
        return fail(SRG_ERR_INVALID, "bad shape n_rows=%lld d=%d", (long long)n_rows, d);
    if (needs_r && n_scales > 1 && r_stride < n_rows * ldr && r_stride > -n_rows * ldr)
        return fail(SRG_ERR_INVALID, "r_stride overlaps the scale panels");
    if (n_rows == 0 || d == 0) return ok();
    if (!Tn || (needs_r && !R) || (init ? !Tc : !To) || (m == SRG_CHEBY_STEP_FIRST && !Tc))
        return fail(SRG_ERR_INVALID, "null panel");
    ChebyCoef<float> cf;
    for (int i = 0; i < 8; ++i) {
        const bool on = i < n_scales;
        cf.prev[i] = ((m == SRG_CHEBY_INIT || m == SRG_CHEBY_STEP_FIRST) && on) ? 0.5f * coef_prev[i] : 0.0f;
        cf.mid[i] = (m == SRG_CHEBY_STEP_FIRST && on) ? coef_prev[n_scales + i] : 0.0f;
        cf.cur[i] = (needs_r && on) ? coef[i] : 0.0f;
    }
    const unsigned blocks = (unsigned)std::min<int64_t>((n_rows + 3) / 4, 256 * 16);
    hipLaunchKernelGGL(k_cheby_epilogue, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                       Tn, ldn, Tc, ldc, To, ldo, n_rows, d, mode, a1, a2, cf, n_scales, R, ldr, r_stride);
    SRG_HIP_CHECK(hipGetLastError());
    return ok();
}

int srg_hop_accumulate_f32(float* agg, int64_t lda, const float* y, int64_t ldy, int64_t n_rows,
                           int32_t d, float w, int mode, void* stream)
{
    SRG_DEVICE_GUARD(stream);
    if (mode != SRG_ACC_INIT && mode != SRG_ACC_ADD && mode != SRG_ACC_DIV)
        return fail(SRG_ERR_INVALID, "accumulate mode %d", mode);
    if (n_rows < 0 || d < 0 || lda < d || (mode != SRG_ACC_DIV && ldy < d))
        return fail(SRG_ERR_INVALID, "bad shape n_rows=%lld d=%d lda=%lld ldy=%lld", (long long)n_rows, d,
                    (long long)lda, (long long)ldy);
    if (n_rows == 0 || d == 0) return ok();
    if (!agg || (mode != SRG_ACC_DIV && !y)) return fail(SRG_ERR_INVALID, "null pointer");
    const unsigned blocks = (unsigned)std::min<int64_t>((n_rows + 3) / 4, 256 * 16);
    hipLaunchKernelGGL(k_hop_accumulate, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                       agg, lda, y, ldy, n_rows, d, w, mode);
    SRG_HIP_CHECK(hipGetLastError());
    return ok();
}

int srg_tail_record_f32(float* hist, const float* y, int64_t ldy, int32_t d, int64_t flat_start,
                        int32_t len, float w, void* stream)
{
    SRG_DEVICE_GUARD(stream);
    if (d <= 0 || ldy < d || flat_start < 0 || len < 0 || len > SRG_TAIL_MAX)
        return fail(SRG_ERR_INVALID, "bad tail d=%d ldy=%lld flat_start=%lld len=%d", d, (long long)ldy,
                    (long long)flat_start, len);
    if (len == 0) return ok();
    if (!hist || !y) return fail(SRG_ERR_INVALID, "null pointer");
    hipLaunchKernelGGL(k_tail_record, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream),
                       hist, y, ldy, d, flat_start, len, w);
    SRG_HIP_CHECK(hipGetLastError());
    return ok();
}

int srg_tail_rowsum_f32(float* agg, int64_t lda, int32_t d, int64_t flat_start, int32_t len,
                        const float* hist, int32_t n_terms, void* stream)
{
    SRG_DEVICE_GUARD(stream);
    if (d <= 0 || lda < d || flat_start < 0 || len < 0 || len > SRG_TAIL_MAX || n_terms < 0)
        return fail(SRG_ERR_INVALID, "bad tail d=%d lda=%lld flat_start=%lld len=%d n_terms=%d", d,
                    (long long)lda, (long long)flat_start, len, n_terms);
    if (len == 0) return ok();
    if (!agg || (n_terms > 0 && !hist)) return fail(SRG_ERR_INVALID, "null pointer");
    hipLaunchKernelGGL(k_tail_rowsum, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream),
                       agg, lda, d, flat_start, len, hist, n_terms);
    SRG_HIP_CHECK(hipGetLastError());
    return ok();
}

int srg_gather_rows_f32(const float* src, int64_t lds, int64_t n_src, const int64_t* idx, int64_t n_idx,
                        float* dst, int64_t ldd, int32_t d, void* stream)
{
    SRG_DEVICE_GUARD(stream);
    if (n_idx < 0 || n_src < 0 || d < 0 || (d > 0 && (lds < d || ldd < d)))
        return fail(SRG_ERR_INVALID, "bad gather shape n_idx=%lld n_src=%lld d=%d lds=%lld ldd=%lld",
                    (long long)n_idx, (long long)n_src, d, (long long)lds, (long long)ldd);
    if (n_idx == 0 || d == 0) return ok();
    if (!src || !idx || !dst) return fail(SRG_ERR_INVALID, "null pointer");
    const int vec = pick_vec(d, lds, ldd, src, dst, sizeof(float));
    const int cpr = d / vec;
    const int S = cpr >= 64 ? 64 : cpr > 16 ? 32 : cpr > 8 ? 16 : cpr > 4 ? 8 : 4;
    const int64_t rows_per_block = (int64_t)(256 / 64) * (64 / S) * 4;
    const unsigned blocks = (unsigned)std::min<int64_t>((n_idx + rows_per_block - 1) / rows_per_block, 256 * 64);
    hipStream_t st = static_cast<hipStream_t>(stream);
#define SRG_GATHER(V, SS) hipLaunchKernelGGL((k_gather_rows<V, SS>), dim3(blocks), dim3(256), 0, st, src, lds, n_src, \
                                             idx, n_idx, dst, ldd, cpr)
#define SRG_GATHER_S(V)                          \
    if (S == 64) SRG_GATHER(V, 64);              \
    else if (S == 32) SRG_GATHER(V, 32);         \
    else if (S == 16) SRG_GATHER(V, 16);         \
    else if (S == 8) SRG_GATHER(V, 8);           \
    else SRG_GATHER(V, 4);
    if (vec == 4) {
        SRG_GATHER_S(4)
    } else if (vec == 2) {
        SRG_GATHER_S(2)
    } else {
        SRG_GATHER_S(1)
    }
#undef SRG_GATHER_S
#undef SRG_GATHER
    SRG_HIP_CHECK(hipGetLastError());
    return ok();
}

int srg_hub_side_streams(void)
{
    std::lock_guard<std::mutex> lock(g_side_mu);
    return (int)g_side.size();
}

int srg_hub_join(void* stream)
{
    SRG_DEVICE_GUARD(stream);
    std::lock_guard<std::mutex> lock(g_side_mu);
    auto it = g_side.find(std::make_pair(guard_.dev, static_cast<hipStream_t>(stream)));
    if (it != g_side.end() && it->second.join) {
        SRG_HIP_CHECK(hipStreamWaitEvent(static_cast<hipStream_t>(stream), it->second.join, 0));
        it->second.pending = false;
    }
    return ok();
}

}  // extern "C"

namespace {
template <typename T>
int launch_segment_sum(const int64_t* seg_ptr, const T* vals, int64_t n_seg, T* out, void* stream)
{
    SRG_DEVICE_GUARD(stream);
    if (n_seg < 0) return fail(SRG_ERR_INVALID, "n_seg=%lld < 0", (long long)n_seg);
    if (n_seg == 0) return ok();
    if (!seg_ptr || !out) return fail(SRG_ERR_INVALID, "null pointer");
    const unsigned blocks = (unsigned)std::min<int64_t>((n_seg + 255) / 256, 1 << 16);   // 64 segments per wave
    hipLaunchKernelGGL(k_segment_sum<T>, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                       seg_ptr, vals, n_seg, out);
    SRG_HIP_CHECK(hipGetLastError());
    return ok();
}
}  // namespace

extern "C" {

int srg_segment_sum_f64(const int64_t* seg_ptr, const double* vals, int64_t n_seg, double* out, void* stream)
{
    return launch_segment_sum<double>(seg_ptr, vals, n_seg, out, stream);
}

int srg_segment_sum_f32(const int64_t* seg_ptr, const float* vals, int64_t n_seg, float* out, void* stream)
{
    return launch_segment_sum<float>(seg_ptr, vals, n_seg, out, stream);
}

int srg_spmm_csr_f64(const int64_t* indptr, const int32_t* indices, const double* values, int64_t n_rows,
                     const double* X, int64_t ldx, double* Y, int64_t ldy, int32_t d, void* stream)
{
    SRG_DEVICE_GUARD(stream);
    int rc = check_spmm_args(indptr, indices, values, n_rows, X, ldx, Y, ldy, d);
    if (rc) return rc;
    if (n_rows == 0 || d == 0) return ok();
    const int64_t total = n_rows * (int64_t)d;
    const unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 1 << 20);
    hipLaunchKernelGGL(k_spmm_f64, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                       indptr, indices, values, n_rows, X, ldx, Y, ldy, d);
    SRG_HIP_CHECK(hipGetLastError());
    return ok();
}

int srg_csr_validate(const int64_t* indptr, const int32_t* indices, int64_t n_rows, int64_t nnz,
                     int64_t n_cols, void* stream)
{
    SRG_DEVICE_GUARD(stream);
    if (n_rows < 0 || nnz < 0 || n_cols < 0) return fail(SRG_ERR_INVALID, "negative size");
    if (!indptr) return fail(SRG_ERR_INVALID, "null indptr");
    if (nnz > 0 && !indices) return fail(SRG_ERR_INVALID, "null indices");
    hipStream_t s = static_cast<hipStream_t>(stream);
    unsigned int* d_bad = nullptr;
    SRG_HIP_CHECK(hipMallocAsync(reinterpret_cast<void**>(&d_bad), sizeof(unsigned int), s));
    SRG_HIP_CHECK(hipMemsetAsync(d_bad, 0, sizeof(unsigned int), s));
    const int64_t work = std::max(nnz, n_rows);
    const unsigned blocks = (unsigned)std::min<int64_t>(std::max<int64_t>((work + 255) / 256, 1), 8192);
    hipLaunchKernelGGL(k_validate, dim3(blocks), dim3(256), 0, s, indptr, indices, n_rows, nnz, n_cols, d_bad);
    SRG_HIP_CHECK(hipGetLastError());
    unsigned int bad = 0;
    SRG_HIP_CHECK(hipMemcpyAsync(&bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost, s));
    SRG_HIP_CHECK(hipFreeAsync(d_bad, s));
    SRG_HIP_CHECK(hipStreamSynchronize(s));
    if (bad & 1u) return fail(SRG_ERR_INVALID, "column id outside [0, %lld)", (long long)n_cols);
    if (bad & 2u) return fail(SRG_ERR_INVALID, "indptr decreases");
    if (bad & 4u) return fail(SRG_ERR_INVALID, "indptr[0] != 0");
    if (bad & 8u) return fail(SRG_ERR_INVALID, "indptr[n_rows] != nnz=%lld", (long long)nnz);
    return ok();
}

int srg_csr_col_splits(const int64_t* indptr, const int32_t* indices, int64_t n_rows, int64_t n_cols,
                       int32_t n_blocks, int64_t* splits, void* stream)
{
    SRG_DEVICE_GUARD(stream);
    if (n_rows < 0 || n_cols < 0) return fail(SRG_ERR_INVALID, "negative size");
    if (n_blocks < 2 || n_blocks > 64) return fail(SRG_ERR_INVALID, "n_blocks=%d not in [2, 64]", n_blocks);
    const int64_t work = n_rows * (n_blocks - 1);
    if (work == 0) return ok();
    if (!indptr || !splits) return fail(SRG_ERR_INVALID, "null indptr or splits");
    if ((work + 255) / 256 > INT32_MAX) return fail(SRG_ERR_INVALID, "grid too large");
    hipLaunchKernelGGL(k_col_splits, dim3((unsigned)((work + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), indptr, indices, n_rows, n_cols, (int)n_blocks, splits);
    SRG_HIP_CHECK(hipGetLastError());
    return ok();
}

int srg_csr_copy_spans(const int32_t* order, int64_t n_order, const int64_t* beg, const int64_t* end,
                       const int32_t* indices, const float* values, const int64_t* pos, int32_t* out_indices,
                       float* out_values, int64_t* out_beg, int64_t* out_end, void* stream)
{
    SRG_DEVICE_GUARD(stream);
    if (n_order < 0) return fail(SRG_ERR_INVALID, "n_order=%lld < 0", (long long)n_order);
    if (n_order == 0) return ok();
    if (!order || !beg || !end || !pos || !out_beg || !out_end)
        return fail(SRG_ERR_INVALID, "null order / span / position array");
    const int64_t rows_per_block = 256 / 16;
    const unsigned blocks = (unsigned)std::min<int64_t>((n_order + rows_per_block - 1) / rows_per_block, 1 << 20);
    hipLaunchKernelGGL(k_copy_spans, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream), order, n_order,
                       beg, end, indices, values, pos, out_indices, out_values, out_beg, out_end);
    SRG_HIP_CHECK(hipGetLastError());
    return ok();
}

int srg_csr_mirror(const int64_t* indptr, const int32_t* indices, const int64_t* rows, int64_t n_rows,
                   int64_t nnz, int64_t* mirror, void* stream)
{
    SRG_DEVICE_GUARD(stream);
    if (n_rows < 0 || nnz < 0) return fail(SRG_ERR_INVALID, "negative size");
    if (nnz == 0) return ok();
    if (!indptr || !indices || !rows || !mirror) return fail(SRG_ERR_INVALID, "null pointer");
    const unsigned blocks = (unsigned)std::min<int64_t>((nnz + 255) / 256, 1 << 20);
    hipLaunchKernelGGL(k_csr_mirror, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream), indptr, indices,
                       rows, nnz, mirror);
    SRG_HIP_CHECK(hipGetLastError());
    return ok();
}

const char* srg_last_error(void) { return g_err_msg; }
int srg_last_error_code(void) { return g_err_code; }
// the communicator entries (srg_comm.hip) report through the same thread-local status
__attribute__((visibility("hidden"))) void srg_set_error(int code, const char* msg)
{
    (void)fail(code, "%s", msg);
}
void srg_clear_error(void) { (void)ok(); }
const char* srg_version(void) { return "srgnn_hip " SRG_GIT_REV " gfx950"; }

}  // extern "C"
