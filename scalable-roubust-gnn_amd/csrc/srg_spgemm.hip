// srg_spgemm.hip -- the sparse products of the wavelet model's preprocessing on MI355X (gfx950).
//
// SpectralModel.preprocess (SSRG/models/base_scalable/base_model.py:208-219) forms the product of
// the two sparsified wavelet matrices with torch_sparse.spspmm and multiplies it into the feature
// matrix with torch_sparse.spmm.  Both are CPU kernels in torch_sparse 0.6.x (spspmm_sum's CPU
// kernel; spmm = index_select, mul, scatter_add) with the arithmetic of scipy's csr_matmat:
//
//   C[i, j] = ((0 + A[i,k1]*B[k1,j]) + A[i,k2]*B[k2,j]) + ...   over row i of A in stored order,
//   every product rounded before it is added (no fma); entries that sum to 0 are dropped; the
//   columns of a row come out ascending.
//   Y[i, :] = ((0 + v1*X[c1, :]) + v2*X[c2, :]) + ...           (spmm: scatter_add in index order)
//
// SpGEMM design (Gustavson, one wave per output row, two passes: count, then fill):
//  * The row's running sums live in a dense accumulator over B's columns -- in LDS when B has at
//    most kLdsCols columns (the wavelet bases of the graphs the reference runs this on), else in a
//    per-workgroup slice of a caller-provided scratch buffer.  A bitmap marks the touched columns.
//  * A's entries are walked in stored order; the wave's 64 lanes take 64 entries of B's row at a
//    time (distinct columns, so no two lanes update one sum), and a barrier separates A's entries,
//    so every sum sees its products in A's order -- the CPU kernels' exact arithmetic.
//  * The touched words of the bitmap are scanned 64 at a time in ascending order; a wave prefix
//    sum over the lanes' nonzero counts places each kept entry, so the columns come out sorted.
//    The scan also resets what it read, leaving the accumulator zero for the workgroup's next row.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "srgnn_hip.h"

extern "C" void srg_set_error(int code, const char* msg);   // srg_spmm.hip: thread-local srg_last_error
extern "C" void srg_clear_error(void);

namespace {

int sg_fail(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    srg_set_error(code, buf);
    return code;
}

int sg_ok()
{
    srg_clear_error();
    return SRG_OK;
}

#define SG_HIP(expr)                                                                            \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return sg_fail(SRG_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));         \
    } while (0)

struct DeviceOf {          // the device of `s` current for the call (the null stream: the current one)
    int prev = -1, rc = SRG_OK;
    explicit DeviceOf(hipStream_t s)
    {
        if (hipGetDevice(&prev) != hipSuccess) { (void)hipGetLastError(); prev = -1; return; }
        if (!s) return;
        hipDevice_t d = 0;
        if (hipStreamGetDevice(s, &d) != hipSuccess) { rc = sg_fail(SRG_ERR_HIP, "hipStreamGetDevice failed"); return; }
        if ((int)d != prev && hipSetDevice((int)d) != hipSuccess) rc = sg_fail(SRG_ERR_HIP, "hipSetDevice failed");
        else if ((int)d == prev) prev = -1;
    }
    ~DeviceOf() { if (prev >= 0) (void)hipSetDevice(prev); }
};

// dense accumulator in LDS up to this many columns: 64 KiB of sums + 2 KiB of bitmap = 66 KiB, which
// fits only because gfx950 gives a workgroup up to 160 KiB of LDS (the 64 KiB of earlier CDNA parts
// would not hold it).  Cost model of the output scan below: it walks every bitmap word between the
// row's smallest and largest touched column, 64 words (2048 columns) per iteration, so a row costs
// O((hi - lo) / 2048) iterations however few entries it has -- on the scratch path (n_cols > 16384) a
// row touching columns 0 and n - 1 of an n = 2.4 M basis takes ~1.2 K iterations.  The wavelet bases
// the reference builds are dense-ish rows over N of a few thousand to ~10^5 columns (it is O(N^2) in
// memory), where the scan is a small part of the row; DESIGN.md §5.7.
constexpr int kLdsCols = 16384;
constexpr int kMaxGlobalSlots = 2048;    // workgroups of the scratch-accumulator path
constexpr int kWave = 64;

__device__ inline int64_t wave_excl_scan(int64_t v, int64_t* total)
{
    const int lane = threadIdx.x;
    int64_t x = v;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const int64_t y = __shfl_up(x, o, kWave);
        if (lane >= o) x += y;
    }
    *total = __shfl(x, kWave - 1, kWave);
    return x - v;
}

// phase 0: cnt[r] = kept entries of C's row r;  phase 1: fills C's row r at cptr[r].
template <bool LDS>
__global__ __launch_bounds__(64) void k_spgemm(const int64_t* __restrict__ ap, const int32_t* __restrict__ ai,
                                               const float* __restrict__ av, int64_t m,
                                               const int64_t* __restrict__ bp, const int32_t* __restrict__ bi,
                                               const float* __restrict__ bv, int64_t ncols, int phase,
                                               int64_t* __restrict__ cnt, const int64_t* __restrict__ cptr,
                                               int32_t* __restrict__ ci, float* __restrict__ cv,
                                               float* __restrict__ g_acc, uint32_t* __restrict__ g_bits,
                                               int serial_b)
{
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ int s_lo, s_hi;
    const int lane = threadIdx.x;
    const int64_t nwords = (ncols + 31) >> 5;
    float* acc;
    uint32_t* bits;
    if (LDS) {
        acc = reinterpret_cast<float*>(smem);
        bits = reinterpret_cast<uint32_t*>(smem + 4 * ((ncols + 3) & ~int64_t(3)));
        for (int64_t i = lane; i < ncols; i += kWave) acc[i] = 0.0f;
        for (int64_t w = lane; w < nwords; w += kWave) bits[w] = 0u;
    } else {
        acc = g_acc + (int64_t)blockIdx.x * ncols;          // zero on entry (host memset), left zero
        bits = g_bits + (int64_t)blockIdx.x * nwords;
    }
    if (lane == 0) { s_lo = INT_MAX; s_hi = -1; }
    __syncthreads();
    for (int64_t r = blockIdx.x; r < m; r += gridDim.x) {
        const int64_t e1 = ap[r + 1];
        for (int64_t e = ap[r]; e < e1; ++e) {              // A's entries in stored order
            const int32_t k = ai[e];
            const float a = av[e];
            const int64_t b0 = bp[k], b1 = bp[k + 1];
            for (int64_t q = b0 + (serial_b ? 0 : lane); q < b1; q += (serial_b ? 1 : kWave)) {
                if (serial_b && lane != 0) break;           // repeated columns in a B row: one lane
                const int32_t j = bi[q];
                acc[j] = __fadd_rn(acc[j], __fmul_rn(a, bv[q]));
                const uint32_t bit = 1u << (j & 31);
                const uint32_t old = atomicOr(&bits[j >> 5], bit);
                if (!(old & bit)) {
                    atomicMin(&s_lo, j >> 5);
                    atomicMax(&s_hi, j >> 5);
                }
            }
            __syncthreads();                                // every sum sees its products in A's order
        }
        const int lo = s_lo, hi = s_hi;
        int64_t run = 0;
        const int64_t base = phase ? cptr[r] : 0;
        if (hi >= 0) {
            for (int64_t w0 = lo; w0 <= hi; w0 += kWave) {
                const int64_t w = w0 + lane;
                const uint32_t word = (w <= hi) ? bits[w] : 0u;
                uint32_t keep = 0;
                for (uint32_t t = word; t; t &= t - 1) {
                    const int b = __ffs(t) - 1;
                    if (acc[w * 32 + b] != 0.0f) keep |= 1u << b;
                }
                int64_t total = 0;
                int64_t pos = base + run + wave_excl_scan(__popc(keep), &total);
                for (uint32_t t = word; t; t &= t - 1) {
                    const int b = __ffs(t) - 1;
                    const int64_t j = w * 32 + b;
                    if (phase && ((keep >> b) & 1u)) {
                        ci[pos] = (int32_t)j;
                        cv[pos] = acc[j];
                        ++pos;
                    }
                    acc[j] = 0.0f;
                }
                if (word) bits[w] = 0u;
                run += total;
            }
        }
        if (!phase && lane == 0) cnt[r] = run;
        __syncthreads();
        if (lane == 0) { s_lo = INT_MAX; s_hi = -1; }
        __syncthreads();
    }
}

// Y[r, :] = sum over row r's entries, in stored order, of (v * X[c, :]) -- each product rounded,
// then added, from +0: torch_sparse.spmm's index_select / mul / scatter_add arithmetic.
__global__ __launch_bounds__(256) void k_spmm_muladd(const int64_t* __restrict__ ip, const int32_t* __restrict__ ix,
                                                     const float* __restrict__ vv, int64_t n_rows,
                                                     const float* __restrict__ X, int64_t ldx,
                                                     float* __restrict__ Y, int64_t ldy, int d)
{
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n_rows) return;
    const int64_t e0 = ip[r], e1 = ip[r + 1];
    for (int c0 = 0; c0 < d; c0 += kWave) {
        const int c = c0 + lane;
        float s = 0.0f;
        if (c < d)
            for (int64_t e = e0; e < e1; ++e) s = __fadd_rn(s, __fmul_rn(vv[e], X[(int64_t)ix[e] * ldx + c]));
        if (c < d) Y[r * ldy + c] = s;
    }
}

}  // namespace

extern "C" {

int srg_spgemm_scratch_bytes(int64_t m, int64_t n_cols, int64_t* bytes)
{
    if (!bytes || m < 0 || n_cols < 0) return sg_fail(SRG_ERR_INVALID, "bad arguments");
    if (n_cols <= kLdsCols) {
        *bytes = 0;
        return sg_ok();
    }
    const int64_t per = 4 * n_cols + 4 * ((n_cols + 31) >> 5);
    const int64_t slots = m < kMaxGlobalSlots ? (m > 0 ? m : 1) : kMaxGlobalSlots;
    *bytes = slots * per;
    return sg_ok();
}

int srg_spgemm_f32(int phase, const int64_t* a_ptr, const int32_t* a_idx, const float* a_val, int64_t m,
                   const int64_t* b_ptr, const int32_t* b_idx, const float* b_val, int64_t n_cols,
                   int64_t* c_cnt, const int64_t* c_ptr, int32_t* c_idx, float* c_val, void* scratch,
                   int64_t scratch_bytes, uint32_t flags, void* stream)
{
    if (phase != 0 && phase != 1) return sg_fail(SRG_ERR_INVALID, "phase %d", phase);
    if (m < 0 || n_cols < 0 || n_cols > INT32_MAX) return sg_fail(SRG_ERR_INVALID, "bad shape m=%lld n=%lld",
                                                                   (long long)m, (long long)n_cols);
    if (m == 0) return sg_ok();
    if (!a_ptr || !b_ptr || (phase == 0 && !c_cnt) || (phase == 1 && !c_ptr))
        return sg_fail(SRG_ERR_INVALID, "null pointer");
    DeviceOf dev(static_cast<hipStream_t>(stream));
    if (dev.rc) return dev.rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int serial = (flags & SRG_SPGEMM_SERIAL_B) ? 1 : 0;
    if (n_cols <= kLdsCols) {
        const size_t lds = 4 * (size_t)((n_cols + 3) & ~int64_t(3)) + 4 * (size_t)((n_cols + 31) >> 5);
        if (lds > 48 * 1024)
            SG_HIP(hipFuncSetAttribute((const void*)k_spgemm<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds));
        const int64_t grid = m < 16384 ? m : 16384;
        hipLaunchKernelGGL(k_spgemm<true>, dim3((unsigned)grid), dim3(kWave), lds, s, a_ptr, a_idx, a_val, m,
                           b_ptr, b_idx, b_val, n_cols, phase, c_cnt, c_ptr, c_idx, c_val, (float*)nullptr,
                           (uint32_t*)nullptr, serial);
    } else {
        const int64_t per = 4 * n_cols + 4 * ((n_cols + 31) >> 5);
        const int64_t slots = scratch ? scratch_bytes / per : 0;
        if (slots < 1) return sg_fail(SRG_ERR_INVALID, "scratch of %lld bytes < one accumulator (%lld)",
                                      (long long)scratch_bytes, (long long)per);
        const int64_t grid = slots < m ? slots : m;
        float* acc = static_cast<float*>(scratch);
        uint32_t* bits = reinterpret_cast<uint32_t*>(acc + grid * n_cols);
        SG_HIP(hipMemsetAsync(scratch, 0, (size_t)(grid * per), s));
        hipLaunchKernelGGL(k_spgemm<false>, dim3((unsigned)grid), dim3(kWave), 0, s, a_ptr, a_idx, a_val, m,
                           b_ptr, b_idx, b_val, n_cols, phase, c_cnt, c_ptr, c_idx, c_val, acc, bits, serial);
    }
    SG_HIP(hipGetLastError());
    return sg_ok();
}

int srg_spmm_muladd_f32(const int64_t* indptr, const int32_t* indices, const float* values, int64_t n_rows,
                        const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t d, void* stream)
{
    if (n_rows < 0 || d < 0 || ldx < d || ldy < d) return sg_fail(SRG_ERR_INVALID, "bad shape");
    if (n_rows == 0 || d == 0) return sg_ok();
    if (!indptr || !Y) return sg_fail(SRG_ERR_INVALID, "null pointer");
    DeviceOf dev(static_cast<hipStream_t>(stream));
    if (dev.rc) return dev.rc;
    const int64_t blocks = (n_rows + 3) / 4;
    for (int64_t b0 = 0; b0 < blocks; b0 += (int64_t)1 << 23) {     // < 2^31 work-items per launch
        const int64_t nb = blocks - b0 < ((int64_t)1 << 23) ? blocks - b0 : ((int64_t)1 << 23);
        const int64_t r0 = b0 * 4;
        hipLaunchKernelGGL(k_spmm_muladd, dim3((unsigned)nb), dim3(256), 0, static_cast<hipStream_t>(stream),
                           indptr + r0, indices, values, n_rows - r0, X, ldx, Y + r0 * ldy, ldy, d);
    }
    SG_HIP(hipGetLastError());
    return sg_ok();
}

}  // extern "C"
