// srg_stream.hip -- the light rows of a hop as one LDS-DMA entry stream per wave (MI355X, gfx950).
//
// The packed light-row path of k_spmm (srg_spmm.hip) walks every row through a chain of dependent
// loads (schedule slot -> span -> column ids -> X rows) and keeps at most U gathers per row in flight,
// so on products' column-block launches it moves 5.2-5.4 TB/s of fabric traffic against the 6.85 TB/s
// of the whole-row launch and the 7.4-7.9 TB/s the MI355X guide measures for row gathers into LDS with
// ~72 KiB in flight per CU (MI355X_MICROARCH.md, "Indexed rows: gather into LDS").  Here a wave takes a
// run of consecutive light rows of the launch's schedule, whose entries a layout pass has copied into
// one contiguous stream, and treats the run as ONE entry stream, decoupled from the row structure:
//
//   * the stream is read in tiles of T entries = 8 KiB of X rows (T = 32 / 16 / 8 at d = 64 / 128 /
//     256); each tile's X rows are gathered straight into an LDS ring slot by 8 global_load_lds_dwordx4
//     (1 KiB each: 4 / 2 / 1 rows), NB = 4 slots, so 3 tiles (24 KiB) are in flight while one is
//     consumed;
//   * the tile's (column id, value) pairs travel the same way, 2 * NB - 2 tiles ahead of its gathers
//     (one global_load_lds_dword of 2 T lanes), so a gather's address never waits on a load issued in
//     the same iteration, and every wait is a counted s_waitcnt vmcnt(n) on loads issued in order;
//   * the consumer reads the tile from LDS (one ds_read_b64 per entry at d = 128) and runs the row's
//     fma chain in CSR order; at a row's end it stores the row and starts the next one;
//   * ACCUMULATE (the later column blocks) without a dependent Y load: the layout gives every row of
//     such a launch a leading pseudo entry (id -1 - row, value 1.0f) whose "gather" reads the row of Y
//     itself, and the chain starts from -0.0f, so its first link fma(1.0f, y, -0.0f) == y exactly and
//     the chain continues from the stored partial sum as the k_spmm ACCUMULATE path does.
//
// Every output element is still ONE sequential fp32 fma chain over its row's entries in stored order
// (the same entries in the same order as k_spmm's span launch): bit-identical results.  Rows longer
// than the launch's slice threshold and the hub rows stay on k_spmm / k_spmm_hub (a run of one such
// row would be one wave's latency); only the light part of a launch streams.
//
// Wave runs: row i of the stream ends at entry position e_i (inclusive prefix of the lengths); its
// cost metric is m_i = e_i + kStreamRowCost * (i + 1) (a row's store and bookkeeping count as a few
// entries), and row i belongs to wave (m_i - 1) / wave_entries.  A run therefore holds at most
// wave_entries / kStreamRowCost + 1 rows and about wave_entries entries (plus the first row's length).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "srgnn_hip.h"
#include "srg_stream_internal.h"

extern "C" void srg_set_error(int code, const char* msg);   // srg_spmm.hip: thread-local srg_last_error
extern "C" void srg_clear_error(void);

namespace {

int st_fail(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    srg_set_error(code, buf);
    return code;
}

#define ST_HIP(expr)                                                                            \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return st_fail(SRG_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));         \
    } while (0)

struct StreamDevice {      // the device of `s` current for the call (the null stream: the current one)
    int prev = -1, rc = SRG_OK;
    explicit StreamDevice(hipStream_t s)
    {
        if (hipGetDevice(&prev) != hipSuccess) { (void)hipGetLastError(); prev = -1; return; }
        if (!s) { prev = -1; return; }
        hipDevice_t d = 0;
        if (hipStreamGetDevice(s, &d) != hipSuccess) { rc = st_fail(SRG_ERR_HIP, "hipStreamGetDevice failed"); return; }
        if ((int)d != prev && hipSetDevice((int)d) != hipSuccess) rc = st_fail(SRG_ERR_HIP, "hipSetDevice failed");
        else if ((int)d == prev) prev = -1;
    }
    ~StreamDevice()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

constexpr int kTileBytes = 8192;    // one ring slot: 8 LDS-DMA instructions of 1 KiB
constexpr int kNBDefault = 4;       // ring slots (3 tiles in flight while one is consumed)

template <int D, int kNB = kNBDefault> struct SG {
    static constexpr int RB = D * 4;           // bytes of one X row
    static constexpr int EPI = 1024 / RB;      // entries per 1-KiB DMA instruction
    static constexpr int T = 8 * EPI;          // entries per tile
    static constexpr int LPE = 64 / EPI;       // lanes per entry in a DMA instruction
    static constexpr int VEC = D / 64;         // floats of a row per lane
    static constexpr int MS = 2 * kNB - 1;     // meta ring slots
};

template <int VEC> struct SV;
template <> struct SV<1> { typedef float type; };
template <> struct SV<2> { typedef float type __attribute__((ext_vector_type(2))); };
template <> struct SV<4> { typedef float type __attribute__((ext_vector_type(4))); };

template <int VEC> __device__ __forceinline__ typename SV<VEC>::type splat(float v)
{
    typename SV<VEC>::type r;
    if constexpr (VEC == 1) {
        r = v;
    } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) r[i] = v;
    }
    return r;
}

template <int VEC>
__device__ __forceinline__ void link(typename SV<VEC>::type& acc, float a, const typename SV<VEC>::type& x)
{
    if constexpr (VEC == 1) {
        acc = __builtin_fmaf(a, x, acc);
    } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc[i] = __builtin_fmaf(a, x[i], acc[i]);
    }
}

__device__ __forceinline__ uint32_t lds_off(const void* p)
{
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// One LDS-DMA instruction: every active lane copies 16 (or 4) bytes from its own global address to
// LDS at M0 + 16 * lane (4 * lane).  Inline asm, so the compiler's wait-count pass does not drain the
// ring at every LDS read: the kernel waits for the tiles itself (vm_wait).
__device__ __forceinline__ void dma16(const void* g, uint32_t l)
{
    int keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(l) : "memory");
}
__device__ __forceinline__ void dma4(const void* g, uint32_t l)
{
    int keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(l) : "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform n (the immediate is a constant: one case per value; larger
// counts wait for more, which is always safe).  Loads retire in issue order, so "at most n of the
// wave's vector-memory operations outstanding", with n = the DMA loads issued after a tile's last one,
// means that tile has landed (stores issued in between only make the wait longer).
#define ST_VMW(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
__device__ __forceinline__ void vm_wait(int n)
{
    switch (n) {
        ST_VMW(0) ST_VMW(1) ST_VMW(2) ST_VMW(3) ST_VMW(4) ST_VMW(5) ST_VMW(6) ST_VMW(7) ST_VMW(8) ST_VMW(9)
        ST_VMW(10) ST_VMW(11) ST_VMW(12) ST_VMW(13) ST_VMW(14) ST_VMW(15) ST_VMW(16) ST_VMW(17) ST_VMW(18)
        ST_VMW(19) ST_VMW(20) ST_VMW(21) ST_VMW(22) ST_VMW(23) ST_VMW(24) ST_VMW(25) ST_VMW(26) ST_VMW(27)
        ST_VMW(28) ST_VMW(29) ST_VMW(30) ST_VMW(31) ST_VMW(32) ST_VMW(33) ST_VMW(34) ST_VMW(35) ST_VMW(36)
        ST_VMW(37) ST_VMW(38) ST_VMW(39) ST_VMW(40) ST_VMW(41) ST_VMW(42) ST_VMW(43) ST_VMW(44) ST_VMW(45)
        ST_VMW(46) ST_VMW(47) ST_VMW(48) ST_VMW(49) ST_VMW(50) ST_VMW(51) ST_VMW(52) ST_VMW(53) ST_VMW(54)
        ST_VMW(55) ST_VMW(56) ST_VMW(57) ST_VMW(58) ST_VMW(59) ST_VMW(60) ST_VMW(61) ST_VMW(62)
        default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
    }
}
#undef ST_VMW

__device__ __forceinline__ int rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int64_t rfl64(int64_t v)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// One wave per block: wave w streams rows [st_wave[w], st_wave[w+1]) of the layout.
//   ent:    int32 pairs (column id, value bits) [entries][2]; id < 0: pseudo entry -1 - row (Y's row)
//   st_end: int64 [n] end position of every row in the stream (inclusive prefix of the lengths)
//   st_row: int32 [n] the row of the output panel each stream row writes
template <int D, int kNB>
__global__ void __launch_bounds__(64)
k_stream(const int32_t* __restrict__ ent, const int64_t* __restrict__ st_end, const int32_t* __restrict__ st_row,
         const int32_t* __restrict__ st_wave, const float* __restrict__ X, int64_t ldx, float* __restrict__ Y,
         int64_t ldy, int acc, int nt)
{
    typedef SG<D, kNB> G;
    constexpr int T = G::T, MS = G::MS, VEC = G::VEC;
    typedef typename SV<VEC>::type V;
    extern __shared__ __attribute__((aligned(16))) char lds[];
    char* xr = lds;                                                     // kNB tiles of X rows
    int* meta = reinterpret_cast<int*>(lds + kNB * kTileBytes);         // MS tiles of (id, value)
    int* rinfo = meta + MS * T * 2;                                     // the run's rows: (end, row)
    const int lane = threadIdx.x;
    const int w = blockIdx.x;
    const int r0 = rfl(st_wave[w]), r1 = rfl(st_wave[w + 1]);
    if (r0 >= r1) return;
    const int64_t E0 = r0 ? rfl64(st_end[r0 - 1]) : 0;
    const int64_t E1 = rfl64(st_end[r1 - 1]);
    const int nent = (int)(E1 - E0);
    const int ntiles = (nent + T - 1) / T;
    const int R = r1 - r0;
    const int32_t* eb = ent + 2 * E0;

    // (id, value) pairs of tile u into meta slot u % MS: lane l copies dword l of the tile (entries
    // past the run's end repeat its last entry, a valid id: the X issue below may read them)
    auto issue_meta = [&](int u) {
        if (lane < 2 * T) {
            int q = 2 * u * T + lane;
            if (q >= 2 * nent) q = 2 * nent - 2 + (lane & 1);
            dma4(eb + q, lds_off(meta + (u % MS) * T * 2));
        }
    };
    // X rows of tile u into ring slot u % kNB: instruction i, lane l gathers the 16-byte chunk
    // l % LPE of entry i * EPI + l / LPE (a pseudo entry reads the row of Y)
    auto issue_x = [&](int u) {
        const int* ms = meta + (u % MS) * T * 2;
        const uint32_t dst = lds_off(xr + (u % kNB) * kTileBytes);
        const int sub = lane % G::LPE;
        int id[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) id[i] = ms[2 * (i * G::EPI + lane / G::LPE)];   // all ids first (the
#pragma unroll                                                                     // DMAs are barriers)
        for (int i = 0; i < 8; ++i) {
            const float* src = id[i] >= 0 ? X + (int64_t)id[i] * ldx : Y + (int64_t)(-1 - id[i]) * ldy;
            dma16(src + sub * 4, dst + i * 1024);
        }
    };

    const int npro = ntiles < 2 * kNB - 2 ? ntiles : 2 * kNB - 2;
    for (int u = 0; u < npro; ++u) issue_meta(u);
    for (int k = lane; k < R; k += 64) {
        rinfo[2 * k] = (int)(st_end[r0 + k] - E0);
        rinfo[2 * k + 1] = st_row[r0 + k];
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");    // metas of the first tiles, run rows
    const int nx0 = ntiles < kNB - 1 ? ntiles : kNB - 1;
    for (int u = 0; u < nx0; ++u) issue_x(u);

    const float init = acc ? -0.0f : 0.0f;
    int k = 0;
    int cur_end = rfl(rinfo[0]), cur_row = rfl(rinfo[1]);
    V a = splat<VEC>(init);
    auto finish = [&]() {
        float* yr = Y + (int64_t)cur_row * ldy + lane * VEC;
        if (nt)
            __builtin_nontemporal_store(a, reinterpret_cast<V*>(yr));
        else
            *reinterpret_cast<V*>(yr) = a;
        ++k;
        if (k < R) {
            cur_end = rfl(rinfo[2 * k]);
            cur_row = rfl(rinfo[2 * k + 1]);
        }
        a = splat<VEC>(init);
    };
    while (k < R && cur_end == 0) finish();      // rows without entries at the run's start

    for (int t = 0; t < ntiles; ++t) {
        // X(t) (and the metas of tiles up to t + kNB - 1) landed: n = DMA loads issued after X(t)
        const int last = (t + kNB - 2 < ntiles - 1) ? t + kNB - 2 : ntiles - 1;
        int n = 8 * (last - t);
        for (int j = (t - kNB + 2 > 0 ? t - kNB + 2 : 0); j < t; ++j) n += (j + 2 * kNB - 2 < ntiles) ? 1 : 0;
        vm_wait(n);
        if (t + 2 * kNB - 2 < ntiles) issue_meta(t + 2 * kNB - 2);
        if (t + kNB - 1 < ntiles) issue_x(t + kNB - 1);
        const char* xs = xr + (t % kNB) * kTileBytes;
        const int* ms = meta + (t % MS) * T * 2;
        const int base = t * T;
        const int jn = nent - base < T ? nent - base : T;
        V x[T];
        float v[T];
#pragma unroll
        for (int j = 0; j < T; ++j) {
            x[j] = *reinterpret_cast<const V*>(xs + j * G::RB + lane * VEC * 4);
            v[j] = __int_as_float(ms[2 * j + 1]);
        }
        if (cur_end > base + jn) {          // no row ends in this tile
#pragma unroll
            for (int j = 0; j < T; ++j)
                if (j < jn) link<VEC>(a, v[j], x[j]);
        } else {
#pragma unroll
            for (int j = 0; j < T; ++j) {
                if (j < jn) {
                    link<VEC>(a, v[j], x[j]);
                    if (base + j + 1 == cur_end) {
                        finish();
                        while (k < R && cur_end == base + j + 1) finish();   // empty rows
                    }
                }
            }
        }
    }
}

// layout pass: lengths (+1 for the pseudo entry of an accumulating launch)
__global__ void __launch_bounds__(256)
k_stream_len(const int32_t* __restrict__ order, int64_t n, const int64_t* __restrict__ beg,
             const int64_t* __restrict__ end, int acc, int64_t* __restrict__ len)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int r = order[i];
    len[i] = end[r] - beg[r] + acc;
}

// layout pass: row order[i]'s entries (after its pseudo entry) to [st_end[i] - len, st_end[i]); 16 lanes
// per row, as k_copy_spans
__global__ void __launch_bounds__(256)
k_stream_fill(const int32_t* __restrict__ order, int64_t n, const int64_t* __restrict__ beg,
              const int64_t* __restrict__ end, const int32_t* __restrict__ ix, const float* __restrict__ v, int acc,
              const int64_t* __restrict__ st_end, int32_t* __restrict__ ent, int32_t* __restrict__ st_row)
{
    const int l = threadIdx.x & 15;
    const int64_t stride = (int64_t)gridDim.x * (blockDim.x / 16);
    for (int64_t i = (int64_t)blockIdx.x * (blockDim.x / 16) + (threadIdx.x >> 4); i < n; i += stride) {
        const int r = order[i];
        const int64_t b = beg[r], len = end[r] - b;
        int64_t p = st_end[i] - len;
        if (l == 0) {
            st_row[i] = r;
            if (acc) {
                ent[2 * (p - 1)] = -1 - r;
                ent[2 * (p - 1) + 1] = __float_as_int(1.0f);
            }
        }
        for (int64_t e = l; e < len; e += 16) {
            ent[2 * (p + e)] = ix[b + e];
            ent[2 * (p + e) + 1] = __float_as_int(v[b + e]);
        }
    }
}

// layout pass: st_wave[w] = the first row whose metric falls in wave w (see the file comment)
__global__ void __launch_bounds__(256)
k_stream_waves(const int64_t* __restrict__ st_end, int64_t n, int64_t wave_entries, int64_t waves,
               int32_t* __restrict__ st_wave)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t wi = (st_end[i] + kStreamRowCost * (i + 1) - 1) / wave_entries;
    const int64_t wp = i ? (st_end[i - 1] + kStreamRowCost * i - 1) / wave_entries : -1;
    for (int64_t w = wp + 1; w <= wi && w < waves; ++w) st_wave[w] = (int32_t)i;
    if (i == n - 1) st_wave[waves] = (int32_t)n;
}

template <int D, int NB>
size_t stream_lds_bytes(int64_t wave_entries)
{
    return (size_t)NB * kTileBytes + (size_t)SG<D, NB>::MS * SG<D, NB>::T * 8 +
           (size_t)(wave_entries / kStreamRowCost + 1) * 8;
}

// ring slots (probe knob SRGNN_STREAM_NB: 3, 4, 6 or 8)
int stream_nb()
{
    static const int v = [] {
        const char* e = getenv("SRGNN_STREAM_NB");
        const int x = e ? atoi(e) : kNBDefault;
        return (x == 2 || x == 3 || x == 4 || x == 6 || x == 8) ? x : kNBDefault;
    }();
    return v;
}

}  // namespace

// Launches the stream kernel of one launch's light rows on `s` (the caller has checked the layout).
__attribute__((visibility("hidden"))) int srg_stream_launch(const SrgStreamRun& r, const float* X, int64_t ldx, float* Y,
                                                            int64_t ldy, int d, int acc, int nt, hipStream_t s)
{
    if (r.waves <= 0) return SRG_OK;
    if (r.waves > INT32_MAX) return st_fail(SRG_ERR_INVALID, "stream: %lld waves", (long long)r.waves);
    const dim3 grid((unsigned)r.waves), block(64);
#define ST_LAUNCH(DD, NB)                                                                                         \
    hipLaunchKernelGGL((k_stream<DD, NB>), grid, block, (stream_lds_bytes<DD, NB>(r.wave_entries)), s, r.ent, r.end,   \
                       r.row, r.wave, X, ldx, Y, ldy, acc, nt)
#define ST_LAUNCH_D(NB)                                                                  \
    do {                                                                                  \
        if (d == 128) ST_LAUNCH(128, NB);                                                 \
        else if (d == 64) ST_LAUNCH(64, NB);                                              \
        else if (d == 256) ST_LAUNCH(256, NB);                                            \
        else return st_fail(SRG_ERR_INVALID, "stream: d=%d not in {64, 128, 256}", d);    \
    } while (0)
    const int nb = stream_nb();
    if (nb == 2) ST_LAUNCH_D(2);
    else if (nb == 3) ST_LAUNCH_D(3);
    else if (nb == 6) ST_LAUNCH_D(6);
    else if (nb == 8) ST_LAUNCH_D(8);
    else ST_LAUNCH_D(4);
#undef ST_LAUNCH_D
#undef ST_LAUNCH
    ST_HIP(hipGetLastError());
    return SRG_OK;
}

__attribute__((visibility("hidden"))) bool srg_stream_fits(const SrgStreamRun& r, const float* X, int64_t ldx,
                                                           const float* Y, int64_t ldy, int d)
{
    return r.ent && (d == 64 || d == 128 || d == 256) && ldx % 4 == 0 && ldy % 4 == 0 &&
           reinterpret_cast<uintptr_t>(X) % 16 == 0 && reinterpret_cast<uintptr_t>(Y) % 16 == 0 &&
           r.wave_entries >= kStreamRowCost && r.wave_entries <= kStreamMaxWaveEntries;
}

extern "C" {

int srg_stream_layout_size(const int32_t* order, int64_t n, const int64_t* beg, const int64_t* end,
                           int32_t accumulate, int64_t wave_entries, int64_t* entries, int64_t* waves, void* stream)
{
    StreamDevice g(static_cast<hipStream_t>(stream));
    if (g.rc) return g.rc;
    if (!entries || !waves) return st_fail(SRG_ERR_INVALID, "stream layout: null entries / waves");
    if (n < 0 || n > INT32_MAX - 1) return st_fail(SRG_ERR_INVALID, "stream layout: n=%lld", (long long)n);
    if (wave_entries < kStreamRowCost || wave_entries > kStreamMaxWaveEntries)
        return st_fail(SRG_ERR_INVALID, "stream layout: wave_entries=%lld not in [%d, %d]", (long long)wave_entries,
                       kStreamRowCost, kStreamMaxWaveEntries);
    *entries = 0;
    *waves = 0;
    if (n == 0) { srg_clear_error(); return SRG_OK; }
    if (!order || !beg || !end) return st_fail(SRG_ERR_INVALID, "stream layout: null order / spans");
    const hipStream_t s = static_cast<hipStream_t>(stream);
    int64_t* len = nullptr;        // [n] lengths, then the sum
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    ST_HIP(hipcub::DeviceReduce::Sum(nullptr, tmp_bytes, len, len, (int)n, s));
    ST_HIP(hipMallocAsync(reinterpret_cast<void**>(&len), (size_t)(n + 1) * 8, s));
    ST_HIP(hipMallocAsync(&tmp, tmp_bytes + 256, s));       // its own allocation: aligned for hipcub
    int64_t* sum = len + n;
    hipLaunchKernelGGL(k_stream_len, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, order, n, beg, end,
                       accumulate ? 1 : 0, len);
    ST_HIP(hipGetLastError());
    ST_HIP(hipcub::DeviceReduce::Sum(tmp, tmp_bytes, len, sum, (int)n, s));
    int64_t total = 0;
    ST_HIP(hipMemcpyAsync(&total, sum, 8, hipMemcpyDeviceToHost, s));
    ST_HIP(hipFreeAsync(len, s));
    ST_HIP(hipFreeAsync(tmp, s));
    ST_HIP(hipStreamSynchronize(s));
    if (total < 0 || total > (int64_t)INT32_MAX * 64) return st_fail(SRG_ERR_INVALID, "stream layout: %lld entries", (long long)total);
    *entries = total;
    *waves = (total + kStreamRowCost * n - 1) / wave_entries + 1;
    srg_clear_error();
    return SRG_OK;
}

int srg_stream_layout_build(const int32_t* order, int64_t n, const int64_t* beg, const int64_t* end,
                            const int32_t* indices, const float* values, int32_t accumulate, int64_t wave_entries,
                            int64_t entries, int64_t waves, int32_t* ent, int64_t* st_end, int32_t* st_row,
                            int32_t* st_wave, void* stream)
{
    StreamDevice g(static_cast<hipStream_t>(stream));
    if (g.rc) return g.rc;
    if (n < 0 || n > INT32_MAX - 1 || entries < 0 || waves < 0)
        return st_fail(SRG_ERR_INVALID, "stream layout: negative size");
    if (wave_entries < kStreamRowCost || wave_entries > kStreamMaxWaveEntries)
        return st_fail(SRG_ERR_INVALID, "stream layout: wave_entries=%lld", (long long)wave_entries);
    if (n == 0) { srg_clear_error(); return SRG_OK; }
    if (!order || !beg || !end || !st_end || !st_row || !st_wave || (entries > 0 && (!indices || !values || !ent)))
        return st_fail(SRG_ERR_INVALID, "stream layout: null pointer");
    if (waves != (entries + kStreamRowCost * n - 1) / wave_entries + 1)
        return st_fail(SRG_ERR_INVALID, "stream layout: waves=%lld does not match entries=%lld (srg_stream_layout_size)",
                       (long long)waves, (long long)entries);
    const hipStream_t s = static_cast<hipStream_t>(stream);
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    int64_t* len = nullptr;
    ST_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tmp_bytes, len, st_end, (int)n, s));
    ST_HIP(hipMallocAsync(reinterpret_cast<void**>(&len), (size_t)n * 8, s));
    ST_HIP(hipMallocAsync(&tmp, tmp_bytes + 256, s));       // its own allocation: aligned for hipcub
    const unsigned gb = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(k_stream_len, dim3(gb), dim3(256), 0, s, order, n, beg, end, accumulate ? 1 : 0, len);
    ST_HIP(hipGetLastError());
    ST_HIP(hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, len, st_end, (int)n, s));
    ST_HIP(hipFreeAsync(len, s));
    ST_HIP(hipFreeAsync(tmp, s));
    const unsigned gf = (unsigned)std::min<int64_t>((n + 15) / 16, 1 << 20);
    hipLaunchKernelGGL(k_stream_fill, dim3(gf), dim3(256), 0, s, order, n, beg, end, indices, values,
                       accumulate ? 1 : 0, st_end, ent, st_row);
    ST_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_stream_waves, dim3(gb), dim3(256), 0, s, st_end, n, wave_entries, waves, st_wave);
    ST_HIP(hipGetLastError());
    srg_clear_error();
    return SRG_OK;
}

int srg_spmm_stream_f32(const int32_t* ent, const int64_t* st_end, const int32_t* st_row, const int32_t* st_wave,
                        int64_t waves, int64_t wave_entries, const float* X, int64_t ldx, float* Y, int64_t ldy,
                        int32_t d, uint32_t flags, void* stream)
{
    StreamDevice g(static_cast<hipStream_t>(stream));
    if (g.rc) return g.rc;
    if (waves < 0) return st_fail(SRG_ERR_INVALID, "stream: waves=%lld < 0", (long long)waves);
    if (waves == 0) { srg_clear_error(); return SRG_OK; }
    SrgStreamRun r{ent, st_end, st_row, st_wave, waves, wave_entries};
    if (!ent || !st_end || !st_row || !st_wave || !X || !Y) return st_fail(SRG_ERR_INVALID, "stream: null pointer");
    if (!srg_stream_fits(r, X, ldx, Y, ldy, d))
        return st_fail(SRG_ERR_INVALID, "stream: needs d in {64, 128, 256}, 16-byte aligned panels with ld %% 4 == 0 "
                                        "and wave_entries in [%d, %d]", kStreamRowCost, kStreamMaxWaveEntries);
    const int rc = srg_stream_launch(r, X, ldx, Y, ldy, d, (flags & SRG_SPMM_ACCUMULATE) ? 1 : 0,
                                     (flags & SRG_SPMM_NT_STORE) ? 1 : 0, static_cast<hipStream_t>(stream));
    if (rc) return rc;
    srg_clear_error();
    return SRG_OK;
}

}  // extern "C"
