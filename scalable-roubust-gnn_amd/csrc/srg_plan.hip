// srg_plan.hip -- the one-GPU propagate planner (srg_plan_build / srg_plan_propagate_f32): the layout a
// long-lived operator gets for a run of K hops, built on the device in one pass, for C / C++ hosts and
// for srgnn.spmm (the boundary the reference's GraphOp.propagate hop loop,
// SSRG/operators/base_operator.py:32-35, is replaced behind).
//
// The layout:
//   * column blocks: block b of row r is the span of its entries whose column ids lie in
//     [ceil(b n / B), ceil((b+1) n / B)) (one binary search per row and boundary); rows of <= 48 entries
//     run whole in block 0; B from the panel size (12..16 for panels of 512 MiB .. 16 GiB at d >= 64, 4 above);
//   * launches: block 0 as its cut rows' first spans and its whole rows (panels < 16 GiB), then blocks
//     1..B-1 with ACCUMULATE -- every output element is the one-launch fma chain, continued;
//   * schedules: each launch's rows by decreasing span length (stable: ties in row order), the first
//     n_hub hub rows (> max(2048, nnz_L / 1024) entries), then n_heavy slice-wave rows
//     (> max(96, nnz_L / 30000); the one-launch hop: nnz / 100000);
//   * compact copies (long runs): the ids and values copied once more, launch after launch, each
//     launch's rows in its schedule order, so no cache line of the streams is read by two launches;
//   * spans by schedule slot (the packed light rows read consecutive slots);
//   * hub spans chained on the side stream when every launch over cut rows has the same hub rows.
// The package's only layout code (round 6: srgnn.spmm / srgnn.plan call this; the torch formulation that
// used to be built beside it is a test restatement now, tests/plan_layout_ref.py): one radix sort of
// (launch, span length) keys over every launch's rows, one scan of the lengths (the copy positions and
// each launch's nnz) and one copy pass; two host synchronisations (the degree statistics; the per-launch
// counts, checked before any span is derived).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <new>
#include <vector>

#include "srgnn_hip.h"

#include "srg_plan_internal.h"

struct srg_plan {
    struct Launch {
        int block = 0;
        const int64_t* row_beg = nullptr;
        const int64_t* row_end = nullptr;    // nullptr: a CSR launch (row_beg has n + 1 pointers)
        const int32_t* indices = nullptr;
        const float* values = nullptr;
        const int32_t* order = nullptr;
        int64_t n_rows = 0, n_hub = 0, n_heavy = 0, n_narrow = 0, nnz = 0;
        const int64_t* slot_beg = nullptr;
        const int64_t* slot_end = nullptr;
        int64_t item0 = 0;                   // the launch's first item (slot 0) among all the plan's items
        bool whole_rows = false;             // block 0's whole rows (not in the hub chain)
        bool hub_whole = false;              // the whole hub rows' launch (hub workgroups only)
    };
    int device = 0;
    int64_t n = 0, nnz = 0, n_items = 0;
    int32_t d = 0, B = 1;
    bool split0 = false, compact = false, same_hubs = false;
    bool block_hubs = false;                 // some launch over cut rows has hub rows
    bool no_values = false;                  // built without fp32 values (SRG_PLAN_SPANS): fp64 steps only
    int64_t n_hub_whole = 0;                 // rows in the whole hub rows' launch
    // compact plans: whether the row-indexed spans hold every scheduled row (the light-row paths of
    // panels other than 64 / 128 / 256 columns read them) or only the hub and slice-wave rows (the
    // packed light rows read the spans by slot); completed on first need (complete_rows)
    bool rows_full = true;
    int64_t* blk_beg = nullptr;
    int64_t* blk_end = nullptr;
    std::vector<Launch> launches;
    void* owned = nullptr;                   // one device allocation holds every array of the plan
    bool owns = true;                        // false: the caller's memory (srg_plan_build_in)
    int64_t bytes = 0;
    // Every stream that work reading the plan's memory was enqueued on, with an event recorded after
    // that work (the hub side stream already joined into it): srg_plan_destroy joins them all into
    // its stream and drains that before the memory goes
    struct Use {
        hipStream_t stream = nullptr;
        hipEvent_t done = nullptr;
    };
    std::vector<Use> uses;
    // the K-hop loop captured as a HIP graph, replayed while the caller repeats a call (SRG_PLAN_GRAPHS)
    struct Graph {
        std::vector<float*> panels;
        int64_t ld = 0;
        int32_t d = 0, K = 0;
        uint32_t flags = 0;
        void* stream = nullptr;
        int calls = 0;                       // eager calls with this key so far
        bool off = false;                    // capture failed once: eager from then on
        hipGraphExec_t exec = nullptr;
        hipEvent_t done = nullptr;           // recorded after the exec's last launch
    } graph;
    // executable graphs of earlier keys, destroyed once their last launch has completed (never while
    // a launch of theirs may still run)
    struct Retired {
        hipGraphExec_t exec = nullptr;
        hipEvent_t done = nullptr;
    };
    std::vector<Retired> retired;
};

namespace {

int pfail(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    srg_set_error(code, buf);
    return code;
}

#define SRG_PLAN_HIP(expr)                                                                       \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            return pfail(SRG_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));            \
    } while (0)

// The layout's constants (DESIGN.md §5.1 has the measurements behind each; srgnn.csr keeps kWholeMax and
// the narrow threshold for the halo planner's chunks and the one-launch schedule of a DeviceCSR)
constexpr int64_t kWholeMax = 48;              // rows this short run whole in block 0
constexpr int64_t kBlockHeavyPer = 30000;      // a column block's slice-wave rows: > nnz_b / this entries
constexpr int64_t kNarrowHeavy = 32;           // slice-wave rows of narrow panels (d <= 32)
constexpr int64_t kSplitBlock0MaxPanel = 16ll << 30;   // block 0 as two launches below this panel size
constexpr int64_t kCapWavesMinPanel = 512ll << 20;     // the row kernel's occupancy cap from this panel size
constexpr int kMaxBlocks = 64;
// automatic blocks for panels of 512 MiB .. 16 GiB at d >= 64: one per ~100 MiB, 12 to 16.
// Round 5, with the packed rows' id staging and gather pipeline (profiles/r05bn_col_blocks_final_kernels.txt):
// products d = 64 (0.63 GB) 3.37 / 3.13 / 3.08 ms per hop at 4 / 8 / 12 blocks, d = 128 (1.25 GB)
// 5.23 / 5.16 / 5.15 / 5.19 / 5.25 at 8 / 10 / 12 / 14 / 16, d = 256 (2.5 GB) 11.73 / 11.18 / 11.00 / 11.20
// at 8 / 12 / 16 / 20 (round 4: 4..8 blocks, one per ~150 MiB)
constexpr int64_t kAutoBlocksMin = 12, kAutoBlocksMax = 16;
constexpr int kMaxLaunch = kMaxBlocks + 1;
constexpr int kHubPrefix = 256;                // hub rows compared for the chain (more: no chain)
constexpr int64_t kCopyChunk = 4096;           // entries of the copy per wave task

// rows of a launch: every row, block 0's cut rows / whole rows, the whole hub rows (round 6)
enum RowSet { kAll = 0, kCut = 1, kWhole = 2, kHubWhole = 3 };

// Whole hub rows (round 6).  In a column-blocked hop a row longer than the one-launch
// hop's hub threshold, max(2048, nnz / 1024) entries, used to be a hub row of every block: twelve chained
// k_spmm_hub launches on the side stream per products hop, each queued behind a full-chip block launch
// (4.5 ms of the 5.15 ms hop from the first fork to the last join).  Such a row is now cut nowhere: it is
// the hub workgroups of one launch of its own, first in the hop, forked onto the side stream and joined at
// the end of the hop -- its whole chain, in CSR order, in one k_spmm_hub launch (the chained spans
// continued the same fma chain from the fp32 value stored between blocks: the same bits).  Only for
// automatic hub thresholds and column-blocked plans.
constexpr int kMaxLaunchTotal = kMaxLaunch + 1;

struct LaunchTable {
    int n_launch;
    int lbits;                                 // launch id bits above the length bits
    int lenbits;
    int whole_rule;                            // 1: the one-launch hop's heavy threshold (nnz / 100000)
    int base;                                  // 1: launch 0 is the whole hub rows' launch
    int64_t hub_t, heavy_t;                    // row lengths, or SRG_PLAN_AUTO / SRG_PLAN_NONE
    int64_t hubw_t;                            // rows longer than this are whole hub rows (INT64_MAX: none)
    int64_t whole_max;                         // rows this short run whole in block 0 (kWholeMax or the opts')
    int64_t off[kMaxLaunchTotal + 1];          // item offsets of the launches
    int64_t rows_lim[kMaxLaunchTotal];         // compact: items of launch L below off[L] + rows_lim[L] get row-indexed spans
    int32_t blk[kMaxLaunchTotal];              // the column block each launch's spans belong to
};

// Bump allocation out of one device allocation (256-byte aligned pieces): a plan makes two
// hipMalloc calls, one for what it keeps and one for its build's scratch.
struct Arena {
    char* base = nullptr;
    size_t used = 0;
    template <typename T>
    T* take(size_t count)
    {
        used = (used + 255) & ~size_t(255);
        T* p = reinterpret_cast<T*>(base ? base + used : nullptr);
        used += std::max<size_t>(count, 1) * sizeof(T);
        return p;
    }
};

// stats[0] = the longest row, stats[1] = rows of <= whole_max entries; stats[2], [3] = indptr[0], indptr[n]
__global__ void __launch_bounds__(256) k_plan_stats(const int64_t* __restrict__ ip, int64_t n, int64_t whole_max,
                                                    unsigned long long* __restrict__ stats)
{
    __shared__ unsigned long long smx[4], swh[4];
    unsigned long long mx = 0, whole = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += stride) {
        const int64_t deg = ip[r + 1] - ip[r];
        mx = max(mx, (unsigned long long)max<int64_t>(deg, 0));
        whole += deg <= whole_max ? 1 : 0;
    }
    for (int o = 32; o > 0; o >>= 1) {
        mx = max(mx, (unsigned long long)__shfl_xor((long long)mx, o));
        whole += (unsigned long long)__shfl_xor((long long)whole, o);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { smx[w] = mx; swh[w] = whole; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < (int)(blockDim.x >> 6); ++i) { mx = max(mx, smx[i]); whole += swh[i]; }
        atomicMax(&stats[0], mx);
        atomicAdd(&stats[1], whole);
        if (blockIdx.x == 0) {
            stats[2] = (unsigned long long)ip[0];
            stats[3] = (unsigned long long)ip[n];
        }
    }
}

// rows longer than t (the whole hub rows: a handful)
__global__ void __launch_bounds__(256) k_plan_count_above(const int64_t* __restrict__ ip, int64_t n, int64_t t,
                                                          unsigned long long* __restrict__ count)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    unsigned long long c = 0;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += stride) c += ip[r + 1] - ip[r] > t ? 1 : 0;
    for (int o = 32; o > 0; o >>= 1) c += (unsigned long long)__shfl_xor((long long)c, o);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(count, c);
}

// split points of the column blocks (srg_csr_col_splits' lower bounds) for the cut rows; the whole rows
// end in block 0 (only block 0's end is ever read for them), and the cut-row flags
// (the whole hub rows too: their one launch reads block 0's end).  flag[r]: 1 for a cut row, 1 << 32 for a
// whole hub row, 0 for a whole row -- one exclusive scan then gives both positions (low / high words)
__global__ void __launch_bounds__(256) k_plan_splits(const int64_t* __restrict__ ip, const int32_t* __restrict__ ix,
                                                     int64_t n, int B, int64_t hubw_t, int64_t whole_max,
                                                     int64_t* __restrict__ splits, int64_t* __restrict__ flag)
{
    // grid-stride over the n (B - 1) (row, boundary) pairs: the grid is capped, so an operator of any
    // size (n (B - 1) past 2^32 work-items: 1.4e9 rows at B = 4) launches
    const int64_t total = n * (B - 1), stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
        const int b = (int)(t / n) + 1;
        const int64_t r = t % n;
        const int64_t beg = ip[r], end = ip[r + 1];
        const bool whole = end - beg <= whole_max;
        const bool hubw = end - beg > hubw_t;
        if (b == 1) flag[r] = hubw ? (int64_t(1) << 32) : whole ? 0 : 1;
        if (whole || hubw) {
            if (b == 1) splits[t] = end;
            continue;
        }
        const int64_t bound = ((int64_t)b * n + B - 1) / B;
        int64_t lo = beg, hi = end;
        while (lo < hi) {
            const int64_t mid = lo + (hi - lo) / 2;
            if ((int64_t)ix[mid] < bound) lo = mid + 1; else hi = mid;
        }
        splits[t] = lo;
    }
}

__device__ __forceinline__ int64_t bound_of(const int64_t* __restrict__ ip, const int64_t* __restrict__ splits,
                                            int64_t n, int B, int b, int64_t r)
{
    return b == 0 ? ip[r] : (b == B ? ip[r + 1] : splits[(int64_t)(b - 1) * n + r]);
}


// the sort items: one (launch, span length) key and the row id per (launch, row of it), the launch's
// rows in ascending order (the stable sort keeps that order among equal lengths, as torch.sort does)
__global__ void __launch_bounds__(256) k_plan_items(const int64_t* __restrict__ ip, const int64_t* __restrict__ splits,
                                                    const int64_t* __restrict__ pos, int64_t n, int B, int split0,
                                                    LaunchTable T, uint64_t* __restrict__ keys,
                                                    int32_t* __restrict__ vals)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const uint64_t lmask = (1ull << T.lenbits) - 1;
    const int L0 = T.base;                     // block 0's (first) launch
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += stride) {
        const int64_t deg = ip[r + 1] - ip[r];
        auto put = [&](int L, int64_t p, int64_t len) {
            const int64_t i = T.off[L] + p;
            keys[i] = ((uint64_t)L << T.lenbits) | (lmask - (uint64_t)len);
            vals[i] = (int32_t)r;
        };
        if (B == 1) {
            put(0, r, deg);
            continue;
        }
        // the cut rows before r, the whole hub rows before r
        const int64_t cp = pos[r] & 0xffffffffll, hp = pos[r] >> 32;
        if (deg > T.hubw_t) {
            put(0, hp, deg);                   // the whole hub rows' launch: the whole row
        } else if (deg > T.whole_max) {
            put(L0, split0 ? cp : r - hp, bound_of(ip, splits, n, B, 1, r) - ip[r]);
            for (int b = 1; b < B; ++b)
                put(L0 + (split0 ? b + 1 : b), cp,
                    bound_of(ip, splits, n, B, b + 1, r) - bound_of(ip, splits, n, B, b, r));
        } else {
            put(L0 + (split0 ? 1 : 0), split0 ? r - cp - hp : r - hp, deg);
        }
    }
}

// every sorted item lies in its launch's segment (an item the items kernel did not write keeps the
// all-ones fill and lands outside): a cheap guard before any span is derived from the keys
__global__ void __launch_bounds__(256) k_plan_check(const uint64_t* __restrict__ keys, int64_t n_items, LaunchTable T,
                                                    int32_t* __restrict__ bad)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int b = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_items; i += stride) {
        const uint64_t L = keys[i] >> T.lenbits;
        b |= (L >= (uint64_t)T.n_launch || i < T.off[L] || i >= T.off[L + 1]) ? 1 : 0;
    }
    if (b) atomicOr(bad, 1);
}

// ------------------------------------------------------------------------------------------------
// The planner's sort and scans, hand-written (round 6; VERDICT r5 "weak" 9): rocPRIM's generic radix sort
// instantiated ~1,100 kernels for the one call -- ~4 MB of kernel metadata in the library.  These are a
// handful, and the sort gives the same permutation (a stable LSD sort by the same key bits):
//   * radix_sort_pairs: 8-bit digits, per pass one digit count per (tile of 4,096 items, digit), one
//     exclusive scan of the counts digit-major, and a stable scatter -- each tile places its items in
//     index order, 256 at a time, ranking equal digits inside a wave with 8 ballots and across the
//     block's 4 waves with per-wave counts in LDS;
//   * scan_i64: reduce-then-scan over tiles of 4,096 (tile sums, one workgroup scanning them, each tile
//     scanning its items from its offset).
// ------------------------------------------------------------------------------------------------
constexpr int kSortThreads = 256;
constexpr int kSortChunks = 16;                          // chunks of 256 items per tile
constexpr int64_t kSortTile = (int64_t)kSortThreads * kSortChunks;
constexpr int kScanThreads = 256;
constexpr int kScanIpt = 16;                             // consecutive items per thread
constexpr int64_t kScanTile = (int64_t)kScanThreads * kScanIpt;

// scan inputs: an int64 array, or the span lengths of sorted (launch, ~length) keys
struct LoadI64 {
    const int64_t* p;
    __device__ int64_t operator()(int64_t i) const { return p[i]; }
};
struct KeyLen {
    const uint64_t* k;
    uint64_t lmask;
    __device__ int64_t operator()(int64_t i) const { return (int64_t)(lmask - (k[i] & lmask)); }
};

// exclusive scan of the 256 values of a block (one per thread) in LDS; returns the block total
__device__ __forceinline__ int64_t block_exclusive_scan(int64_t v, int64_t& total)
{
    __shared__ int64_t sh[kScanThreads];
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int o = 1; o < kScanThreads; o <<= 1) {
        const int64_t x = t >= o ? sh[t - o] : 0;
        __syncthreads();
        sh[t] += x;
        __syncthreads();
    }
    total = sh[kScanThreads - 1];
    const int64_t ex = sh[t] - v;
    __syncthreads();
    return ex;
}

template <typename In>
__global__ void __launch_bounds__(kScanThreads) k_scan_reduce(In in, int64_t n, int64_t* __restrict__ part)
{
    const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanIpt;
    int64_t sum = 0;
#pragma unroll
    for (int j = 0; j < kScanIpt; ++j)
        if (base + j < n) sum += in(base + j);
    int64_t total;
    (void)block_exclusive_scan(sum, total);
    if (threadIdx.x == 0) part[blockIdx.x] = total;
}

// one workgroup: the tile sums' exclusive scan, in place
__global__ void __launch_bounds__(kScanThreads) k_scan_parts(int64_t* __restrict__ part, int64_t m)
{
    int64_t carry = 0;
    for (int64_t b = 0; b < m; b += kScanThreads) {
        const int64_t i = b + threadIdx.x;
        const int64_t v = i < m ? part[i] : 0;
        int64_t total;
        const int64_t ex = block_exclusive_scan(v, total);
        if (i < m) part[i] = carry + ex;
        carry += total;
    }
}

// out[i] = sum of in(0 .. i) (inclusive) or in(0 .. i-1); out may be the input array (each thread reads
// its items before it writes them)
template <typename In>
__global__ void __launch_bounds__(kScanThreads) k_scan_apply(In in, int64_t n, const int64_t* __restrict__ part,
                                                             int64_t* out, int inclusive)
{
    const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanIpt;
    int64_t v[kScanIpt];
    int64_t sum = 0;
#pragma unroll
    for (int j = 0; j < kScanIpt; ++j) {
        v[j] = base + j < n ? in(base + j) : 0;
        sum += v[j];
    }
    int64_t total;
    int64_t run = part[blockIdx.x] + block_exclusive_scan(sum, total);
#pragma unroll
    for (int j = 0; j < kScanIpt; ++j) {
        if (base + j < n) out[base + j] = inclusive ? run + v[j] : run;
        run += v[j];
    }
}

// the digit counts of each tile, digit-major: hist[digit * n_tiles + tile]
__global__ void __launch_bounds__(kSortThreads) k_sort_hist(const uint64_t* __restrict__ keys, int64_t n, int shift,
                                                           uint64_t dmask, int64_t n_tiles, int64_t* __restrict__ hist)
{
    __shared__ unsigned int h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * kSortTile;
    for (int c = 0; c < kSortChunks; ++c) {
        const int64_t i = base + (int64_t)c * kSortThreads + threadIdx.x;
        if (i < n) atomicAdd(&h[(keys[i] >> shift) & dmask], 1u);
    }
    __syncthreads();
    hist[(int64_t)threadIdx.x * n_tiles + blockIdx.x] = h[threadIdx.x];
}

// stable scatter of one pass: offs = the exclusive scan of k_sort_hist's counts
__global__ void __launch_bounds__(kSortThreads) k_sort_scatter(const uint64_t* __restrict__ kin,
                                                              const int32_t* __restrict__ vin, uint64_t* __restrict__ kout,
                                                              int32_t* __restrict__ vout, int64_t n, int shift,
                                                              uint64_t dmask, int64_t n_tiles,
                                                              const int64_t* __restrict__ offs)
{
    constexpr int kWaves = kSortThreads / 64;
    __shared__ int64_t run[256];                   // where this tile's next item of each digit goes
    __shared__ unsigned int wcnt[kWaves][256];     // items of each digit per wave, this chunk
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    run[t] = offs[(int64_t)t * n_tiles + blockIdx.x];
    const int64_t base = (int64_t)blockIdx.x * kSortTile;
    for (int c = 0; c < kSortChunks; ++c) {
#pragma unroll
        for (int q = 0; q < kWaves; ++q) wcnt[q][t] = 0;
        __syncthreads();
        const int64_t i = base + (int64_t)c * kSortThreads + t;
        const bool act = i < n;
        const uint64_t k = act ? kin[i] : 0;
        const unsigned dg = (unsigned)((k >> shift) & dmask);
        // the lanes of this wave holding the same digit, and how many of them come before this one
        unsigned long long same = __ballot(act);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const unsigned long long m = __ballot((dg >> b) & 1u);
            same &= ((dg >> b) & 1u) ? m : ~m;
        }
        const unsigned long long below = same & ((1ull << lane) - 1ull);
        if (act && below == 0) wcnt[w][dg] = (unsigned)__popcll(same);     // the group's first lane
        __syncthreads();
        if (act) {
            int64_t p = run[dg] + __popcll(below);
            for (int q = 0; q < w; ++q) p += wcnt[q][dg];
            kout[p] = k;
            vout[p] = vin[i];
        }
        __syncthreads();
        int64_t add = 0;
#pragma unroll
        for (int q = 0; q < kWaves; ++q) add += wcnt[q][t];
        run[t] += add;
        __syncthreads();
    }
}

// per launch: nnz, hub / slice-wave / narrow slice-wave rows (the sorted lengths decrease inside a
// launch: a count of lengths above t is a binary search), the first hub rows
__global__ void k_plan_counts(const uint64_t* __restrict__ keys, const int32_t* __restrict__ vals,
                              const int64_t* __restrict__ pos, LaunchTable T, int64_t* __restrict__ counts,
                              int32_t* __restrict__ hubs)
{
    const int L = threadIdx.x;
    if (L >= T.n_launch) return;
    const uint64_t lmask = (1ull << T.lenbits) - 1;
    const int64_t o = T.off[L], m = T.off[L + 1] - o;
    const int64_t nnz = pos[o + m] - pos[o];
    auto above = [&](int64_t t) {
        int64_t lo = 0, hi = m;
        while (lo < hi) {
            const int64_t mid = lo + (hi - lo) / 2;
            if ((int64_t)(lmask - (keys[o + mid] & lmask)) > t) lo = mid + 1; else hi = mid;
        }
        return lo;
    };
    // automatic thresholds from the launch's nnz; a caller's thresholds hold for every launch (the
    // narrow panels' slice waves then follow the heavy threshold too: DeviceCSR.heavy)
    if (T.base && L == 0) {
        // the whole hub rows' launch: every row is a hub row (hub workgroups only, no main launch)
        counts[4 * L + 0] = nnz;
        counts[4 * L + 1] = m;
        counts[4 * L + 2] = 0;
        counts[4 * L + 3] = 0;
        for (int64_t j = 0; j < min<int64_t>(m, kHubPrefix); ++j) hubs[(int64_t)L * kHubPrefix + j] = vals[o + j];
        return;
    }
    const int64_t hub_t = T.hub_t == SRG_PLAN_AUTO ? max<int64_t>(2048, nnz / 1024) : T.hub_t;
    const int64_t heavy_t = T.heavy_t == SRG_PLAN_AUTO ? max<int64_t>(96, nnz / (T.whole_rule ? 100000 : kBlockHeavyPer))
                                                       : T.heavy_t;
    const int64_t n_hub = T.hub_t == SRG_PLAN_NONE ? 0 : above(hub_t);
    const int64_t n_heavy = max<int64_t>(0, (T.heavy_t == SRG_PLAN_NONE ? 0 : above(heavy_t)) - n_hub);
    counts[4 * L + 0] = nnz;
    counts[4 * L + 1] = n_hub;
    counts[4 * L + 2] = n_heavy;
    counts[4 * L + 3] = T.heavy_t == SRG_PLAN_AUTO ? max<int64_t>(0, above(kNarrowHeavy) - n_hub) : n_heavy;
    for (int64_t j = 0; j < min<int64_t>(n_hub, kHubPrefix); ++j) hubs[(int64_t)L * kHubPrefix + j] = vals[o + j];
}

// The spans by slot (and, compact, the row-indexed spans of the first rows_lim[L] rows of each launch):
// item i's span is [pos[i], pos[i+1]) of the copy (compact) or its span of the caller's arrays.
__global__ void __launch_bounds__(256) k_plan_spans(const int64_t* __restrict__ ip, const int64_t* __restrict__ splits,
                                                    int64_t n, int B, int split0, LaunchTable T, int compact,
                                                    const uint64_t* __restrict__ keys, const int32_t* __restrict__ vals,
                                                    const int64_t* __restrict__ pos, int64_t n_items,
                                                    int64_t* __restrict__ slot_beg, int64_t* __restrict__ slot_end,
                                                    int64_t* __restrict__ blk_beg, int64_t* __restrict__ blk_end)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_items; i += stride) {
        const int L = (int)(keys[i] >> T.lenbits);
        const int b = T.blk[L];
        const int64_t len = pos[i + 1] - pos[i];
        if (compact) {
            const int64_t p = pos[i];
            slot_beg[i] = p;
            slot_end[i] = p + len;
            if (i - T.off[L] < T.rows_lim[L]) {
                const int64_t r = vals[i];
                blk_beg[(int64_t)b * n + r] = p;
                blk_end[(int64_t)b * n + r] = p + len;
            }
        } else {
            const int64_t src = bound_of(ip, splits, n, B, b, vals[i]);
            slot_beg[i] = src;
            slot_end[i] = src + len;
        }
    }
}

// The compact copy: the entries of all items laid end to end (item i's at [pos[i], pos[i+1])).  Each
// wave task copies kCopyChunk consecutive entries of the copy: it finds the item holding its first
// entry (a binary search of pos), holds 64 items' (position, source) pairs in its lanes, and every
// lane takes consecutive entries, finding its item among the lanes' positions with 6 shuffles -- so
// the writes are whole contiguous runs and the reads contiguous within each span, whatever the span
// lengths (5 M spans of ~23 entries on products: one span per 16-lane group read and wrote 64-byte
// pieces and took 1.3 ms; tools/plan_probe).
__global__ void __launch_bounds__(256) k_plan_copy(const int64_t* __restrict__ ip, const int64_t* __restrict__ splits,
                                                   const int32_t* __restrict__ ix, const float* __restrict__ v,
                                                   int64_t n, int B, const LaunchTable T, int lenbits,
                                                   const uint64_t* __restrict__ keys, const int32_t* __restrict__ vals,
                                                   const int64_t* __restrict__ pos, int64_t n_items, int64_t nnz,
                                                   int32_t* __restrict__ oix, float* __restrict__ ov)
{
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t n_waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const int64_t n_tasks = (nnz + kCopyChunk - 1) / kCopyChunk;
    for (int64_t task = wave; task < n_tasks; task += n_waves) {
        const int64_t e0 = task * kCopyChunk, e1 = min(e0 + kCopyChunk, nnz);
        // the item holding entry e0: the last i with pos[i] <= e0 (pos[0] = 0)
        int64_t lo = 0, hi = n_items;          // invariant: pos[lo] <= e0, answer in [lo, hi)
        while (hi - lo > 1) {
            const int64_t mid = lo + (hi - lo) / 2;
            if (pos[mid] <= e0) lo = mid; else hi = mid;
        }
        int64_t ibase = lo;
        int64_t e = e0;                        // wave-uniform: the first entry not yet copied
        while (e < e1) {
            const int64_t i = ibase + lane;
            int64_t p = INT64_MAX, src = 0;
            if (i < n_items) {
                p = pos[i];
                const int L = (int)(keys[i] >> lenbits);
                src = bound_of(ip, splits, n, B, T.blk[L], vals[i]);
            }
            // the batch's items cover [pos[ibase], pos[ibase + 64])
            const int64_t pend = ibase + 64 < n_items ? pos[ibase + 64] : nnz;
            const int64_t stop = min(e1, pend);
            for (int64_t eb = e; eb < stop; eb += 64) {
                const int64_t me = eb + lane;
                // the last lane j with p_j <= me
                int j = 0;
#pragma unroll
                for (int step = 32; step > 0; step >>= 1) {
                    const int64_t pj = __shfl((long long)p, j + step);
                    if (pj <= me) j += step;
                }
                const int64_t pj = __shfl((long long)p, j), sj = __shfl((long long)src, j);
                if (me < stop) {
                    const int64_t from = sj + (me - pj);
                    oix[me] = ix[from];
                    ov[me] = v[from];
                }
            }
            e = stop;
            ibase += 64;
        }
    }
}

// The row-indexed spans of every scheduled row of a compact plan (the light-row paths that read them)
__global__ void __launch_bounds__(256) k_plan_rows(int64_t n, const int32_t* __restrict__ order,
                                                   const int64_t* __restrict__ item_launch_block, int n_launch,
                                                   const int64_t* __restrict__ slot_beg, const int64_t* __restrict__ slot_end,
                                                   int64_t n_items, int64_t* __restrict__ blk_beg, int64_t* __restrict__ blk_end)
{
    // item_launch_block: [n_launch + 1] item offsets, then [n_launch] blocks
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_items; i += stride) {
        int L = 0;
        while (L + 1 < n_launch && i >= item_launch_block[L + 1]) ++L;
        const int64_t b = item_launch_block[n_launch + 1 + L];
        const int64_t r = order[i];
        blk_beg[b * n + r] = slot_beg[i];
        blk_end[b * n + r] = slot_end[i];
    }
}

int bits_for(uint64_t v)
{
    int b = 1;
    while (b < 64 && (v >> b) != 0) ++b;
    return b;
}

unsigned grid_for(int64_t work, int per_block, unsigned cap)
{
    const int64_t g = (work + per_block - 1) / per_block;
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

struct DevGuard {
    int prev = -1, rc = SRG_OK;
    explicit DevGuard(hipStream_t s)
    {
        if (hipGetDevice(&prev) != hipSuccess) { (void)hipGetLastError(); prev = -1; return; }
        if (!s) return;
        hipDevice_t d = 0;
        if (hipStreamGetDevice(s, &d) != hipSuccess) { rc = pfail(SRG_ERR_HIP, "hipStreamGetDevice failed"); return; }
        if ((int)d != prev && hipSetDevice((int)d) != hipSuccess) rc = pfail(SRG_ERR_HIP, "hipSetDevice(%d) failed", (int)d);
    }
    ~DevGuard()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// build temporaries: released after the work enqueued on `s` so far
struct DevBuf {
    void* p = nullptr;
    hipStream_t s = nullptr;
    ~DevBuf() { reset(); }
    void reset()
    {
        if (!p) return;
        (void)hipStreamSynchronize(s);
        (void)hipFree(p);
        p = nullptr;
    }
};

bool capturing(hipStream_t s)
{
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess) { (void)hipGetLastError(); return false; }
    return st != hipStreamCaptureStatusNone;
}

constexpr size_t kMaxUses = 16;              // streams remembered per plan (older ones are drained)

// Work reading the plan's memory has been enqueued on `s` (hub side stream joined into it): remember
// it.  A stream the caller is capturing into its own graph is not recorded (an event recorded there
// would be a graph node); such a caller orders its graph's launches before srg_plan_destroy itself.
void note_use(srg_plan* P, hipStream_t s)
{
    if (capturing(s)) return;
    srg_plan::Use* u = nullptr;
    for (auto& x : P->uses)
        if (x.stream == s) u = &x;
    if (!u) {
        if (P->uses.size() >= kMaxUses) {
            (void)hipEventSynchronize(P->uses.front().done);
            (void)hipEventDestroy(P->uses.front().done);
            P->uses.erase(P->uses.begin());
        }
        srg_plan::Use nu;
        nu.stream = s;
        if (hipEventCreateWithFlags(&nu.done, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipStreamSynchronize(s);   // no event: make the work complete instead
            return;
        }
        P->uses.push_back(nu);
        u = &P->uses.back();
    }
    if (hipEventRecord(u->done, s) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipStreamSynchronize(s);
    }
}

// executable graphs of earlier keys whose last launch has completed
void reap_retired(srg_plan* P, bool wait)
{
    for (size_t i = 0; i < P->retired.size();) {
        srg_plan::Retired& r = P->retired[i];
        const hipError_t q = wait ? hipEventSynchronize(r.done) : hipEventQuery(r.done);
        if (q == hipErrorNotReady) { ++i; continue; }
        (void)hipGetLastError();
        (void)hipGraphExecDestroy(r.exec);
        (void)hipEventDestroy(r.done);
        P->retired.erase(P->retired.begin() + (long)i);
    }
}

// the current key's graph goes: retired until its last launch has completed
void drop_graph(srg_plan* P)
{
    srg_plan::Graph& G = P->graph;
    if (G.exec) P->retired.push_back({G.exec, G.done});
    else if (G.done) (void)hipEventDestroy(G.done);
    G.exec = nullptr;
    G.done = nullptr;
}

// Releases the plan's memory after every reader: each stream the plan's work went to is joined into
// `s` (its last recorded event), then `s` is drained -- so the hub side stream (joined into those
// streams by the hops), replayed graphs and complete_rows' kernels have all finished -- and only then
// are the executable graphs destroyed and the memory freed.  Before round 6 the graph exec was
// destroyed first and only `s` was drained: a graph launch or a hop on another stream could still be
// reading the plan (hipFree's implicit device synchronisation hid it).
void release(srg_plan* P, hipStream_t s)
{
    for (const auto& u : P->uses)
        if (u.done && hipStreamWaitEvent(s, u.done, 0) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipEventSynchronize(u.done);
        }
    (void)hipStreamSynchronize(s);
    for (const auto& u : P->uses) (void)hipEventSynchronize(u.done);   // already complete: cheap
    drop_graph(P);
    reap_retired(P, true);
    for (auto& u : P->uses) (void)hipEventDestroy(u.done);
    P->uses.clear();
    if (P->owned && P->owns) (void)hipFree(P->owned);
    P->owned = nullptr;
}

// compact plans built with row-indexed spans for the hub and slice-wave rows only: fill the rest
int complete_rows(srg_plan* P, hipStream_t s)
{
    if (P->rows_full || !P->compact) return SRG_OK;
    const int nl = (int)P->launches.size();
    std::vector<int64_t> tab((size_t)2 * nl + 1);
    for (int L = 0; L < nl; ++L) {
        tab[L] = P->launches[L].item0;
        tab[(size_t)nl + 1 + L] = P->launches[L].block;
    }
    tab[nl] = P->n_items;
    DevBuf t;
    t.s = s;
    SRG_PLAN_HIP(hipMalloc(&t.p, tab.size() * sizeof(int64_t)));
    SRG_PLAN_HIP(hipMemcpyAsync(t.p, tab.data(), tab.size() * sizeof(int64_t), hipMemcpyHostToDevice, s));
    const srg_plan::Launch& L0 = P->launches[0];
    hipLaunchKernelGGL(k_plan_rows, dim3(grid_for(P->n_items, 256, 1u << 20)), dim3(256), 0, s, P->n, L0.order, (const int64_t*)t.p, nl, L0.slot_beg, L0.slot_end, P->n_items, P->blk_beg, P->blk_end);
    SRG_PLAN_HIP(hipGetLastError());
    P->rows_full = true;
    note_use(P, s);
    return SRG_OK;
}

bool packed_width(int d) { return d == 64 || d == 128 || d == 256; }

// int64 elements of scan_i64's temp (its tile sums) and of radix_sort_pairs' (digit counts + their scan)
int64_t scan_tmp_elems(int64_t n) { return std::max<int64_t>(1, (n + kScanTile - 1) / kScanTile); }
int64_t sort_tmp_elems(int64_t n)
{
    const int64_t cells = 256 * std::max<int64_t>(1, (n + kSortTile - 1) / kSortTile);
    return cells + scan_tmp_elems(cells);
}

template <typename In>
int scan_i64(In in, int64_t n, int64_t* out, bool inclusive, int64_t* part, hipStream_t s)
{
    if (n <= 0) return SRG_OK;
    const int64_t tiles = (n + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(k_scan_reduce<In>, dim3((unsigned)tiles), dim3(kScanThreads), 0, s, in, n, part);
    hipLaunchKernelGGL(k_scan_parts, dim3(1), dim3(kScanThreads), 0, s, part, tiles);
    hipLaunchKernelGGL(k_scan_apply<In>, dim3((unsigned)tiles), dim3(kScanThreads), 0, s, in, n, (const int64_t*)part,
                       out, inclusive ? 1 : 0);
    SRG_PLAN_HIP(hipGetLastError());
    return SRG_OK;
}

// (keys, vals) sorted by key bits [0, bits), stably, into (skeys, svals); keys / vals are clobbered
int radix_sort_pairs(uint64_t* keys, int32_t* vals, uint64_t* skeys, int32_t* svals, int64_t n, int bits, int64_t* tmp,
                     hipStream_t s)
{
    if (n <= 0) return SRG_OK;
    const int64_t tiles = (n + kSortTile - 1) / kSortTile;
    int64_t* hist = tmp;
    int64_t* part = tmp + 256 * tiles;
    uint64_t *ki = keys, *ko = skeys;
    int32_t *vi = vals, *vo = svals;
    for (int shift = 0; shift < bits; shift += 8) {
        // the last pass's digits stop at `bits`: keys that differ only above it keep their order
        const uint64_t dmask = bits - shift >= 8 ? 255u : (1u << (bits - shift)) - 1u;
        hipLaunchKernelGGL(k_sort_hist, dim3((unsigned)tiles), dim3(kSortThreads), 0, s, ki, n, shift, dmask, tiles, hist);
        const int rc = scan_i64(LoadI64{hist}, 256 * tiles, hist, false, part, s);
        if (rc) return rc;
        hipLaunchKernelGGL(k_sort_scatter, dim3((unsigned)tiles), dim3(kSortThreads), 0, s, ki, vi, ko, vo, n, shift,
                           dmask, tiles, (const int64_t*)hist);
        SRG_PLAN_HIP(hipGetLastError());
        std::swap(ki, ko);
        std::swap(vi, vo);
    }
    if (ki != skeys) {
        SRG_PLAN_HIP(hipMemcpyAsync(skeys, ki, (size_t)n * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
        SRG_PLAN_HIP(hipMemcpyAsync(svals, vi, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
    }
    return SRG_OK;
}

}  // namespace

// Where a build's memory comes from: the library (hipMalloc: srg_plan_build), the caller
// (srg_plan_build_in: `keep` for the plan's lifetime, `scratch` for the call), or nowhere -- a size
// query (srg_plan_query: the sizes and the resolved choices are returned, nothing is built).
namespace {
struct BuildMem {
    void* keep = nullptr;
    size_t keep_bytes = 0;
    void* scratch = nullptr;
    size_t scratch_bytes = 0;
    size_t* q_keep = nullptr;                // non-null: query only
    size_t* q_scratch = nullptr;
    uint32_t* q_opts = nullptr;
    int32_t* q_blocks = nullptr;
    bool query() const { return q_keep != nullptr; }
    bool caller() const { return keep != nullptr; }
};
}  // namespace

static int build_impl(const int64_t* indptr, const int32_t* indices, const float* values, int64_t n_rows, int32_t d,
               int32_t hops, int32_t col_blocks, int64_t hub_threshold, int64_t heavy_threshold, uint32_t opts,
               void* stream, srg_plan** plan, const BuildMem& mem)
{
    if (!plan && !mem.query()) return pfail(SRG_ERR_INVALID, "null plan");
    if (plan) *plan = nullptr;
    if (!indptr) return pfail(SRG_ERR_INVALID, "null indptr");
    if (n_rows < 0 || n_rows >= (1ll << 31)) return pfail(SRG_ERR_INVALID, "n_rows=%lld outside [0, 2^31)", (long long)n_rows);
    if (d <= 0 || hops < 0 || col_blocks < 0 || col_blocks > kMaxBlocks)
        return pfail(SRG_ERR_INVALID, "d=%d, hops=%d, col_blocks=%d (0 = automatic, at most %d)", d, hops, col_blocks, kMaxBlocks);
    if (hub_threshold < SRG_PLAN_NONE || heavy_threshold < SRG_PLAN_NONE)
        return pfail(SRG_ERR_INVALID, "hub_threshold=%lld, heavy_threshold=%lld: a row length, SRG_PLAN_AUTO or SRG_PLAN_NONE",
                     (long long)hub_threshold, (long long)heavy_threshold);
    const uint32_t known = SRG_PLAN_COMPACT | SRG_PLAN_SPANS | SRG_PLAN_SPLIT_BLOCK0 | SRG_PLAN_WHOLE_BLOCK0 |
                           SRG_PLAN_WHOLE_HUBS | (0xffffu << SRG_PLAN_WHOLE_MAX_SHIFT);
    // block 0's whole rows: at most this many entries (SRG_PLAN_WHOLE_MAX(n); 0: kWholeMax)
    const int64_t whole_max = (opts >> SRG_PLAN_WHOLE_MAX_SHIFT) ? (int64_t)(opts >> SRG_PLAN_WHOLE_MAX_SHIFT) : kWholeMax;
    if ((opts & ~known) || ((opts & SRG_PLAN_COMPACT) && (opts & SRG_PLAN_SPANS)) ||
        ((opts & SRG_PLAN_SPLIT_BLOCK0) && (opts & SRG_PLAN_WHOLE_BLOCK0)))
        return pfail(SRG_ERR_INVALID, "opts=0x%x: unknown or conflicting options", opts);
    const hipStream_t s = static_cast<hipStream_t>(stream);
    DevGuard g(s);
    if (g.rc) return g.rc;
    srg_plan* P = new (std::nothrow) srg_plan();
    if (!P) return pfail(SRG_ERR_ALLOC, "plan: host memory");
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) { delete P; return pfail(SRG_ERR_HIP, "hipGetDevice failed"); }
    P->device = dev;
    P->n = n_rows;
    P->d = d;
    auto bail = [&](int rc) { release(P, s); delete P; return rc; };
    const int64_t n = n_rows;
    DevBuf scratch;                          // the library's scratch (srg_plan_build)
    scratch.s = s;
    char* scratch_base = nullptr;
    // ---- 1: degree statistics (host sync 1) ----
    unsigned long long hs[4] = {0, 0, 0, 0};
    {
        DevBuf st;
        st.s = s;
        if (hipMalloc(&st.p, 4 * sizeof(unsigned long long)) != hipSuccess) { (void)hipGetLastError(); return bail(pfail(SRG_ERR_ALLOC, "plan: statistics")); }
        unsigned long long* dstats = (unsigned long long*)st.p;
        if (hipMemsetAsync(dstats, 0, 4 * sizeof(unsigned long long), s) != hipSuccess) return bail(pfail(SRG_ERR_HIP, "memset"));
        hipLaunchKernelGGL(k_plan_stats, dim3(grid_for(std::max<int64_t>(n, 1), 256, 512)), dim3(256), 0, s, indptr, n, whole_max,
                           dstats);
        if (hipMemcpyAsync(hs, dstats, sizeof(hs), hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
            return bail(pfail(SRG_ERR_HIP, "plan: degree statistics: %s", hipGetErrorString(hipGetLastError())));
    }
    const int64_t max_deg = (int64_t)hs[0], n_whole_rows = (int64_t)hs[1];
    const int64_t nnz = (int64_t)hs[3] - (int64_t)hs[2];
    unsigned long long* dstat = nullptr;     // (reused below for the whole hub rows' count)
    if (nnz < 0) return bail(pfail(SRG_ERR_INVALID, "indptr[n] < indptr[0]"));
    // values may be NULL for a SPANS plan (fp64 Chebyshev steps bring their own values: srg_plan_cheby_step_f64)
    if (nnz > 0 && !mem.query() && (!indices || (!values && !(opts & SRG_PLAN_SPANS))))
        return bail(pfail(SRG_ERR_INVALID, "null indices / values"));
    P->nnz = nnz;
    P->no_values = nnz > 0 && !values;
    // ---- 2: the layout: blocks, launches, copies ----
    const int64_t panel = n * (int64_t)d * 4;
    int B = col_blocks;
    if (B == 0) {
        if (d < 64 || panel < (512ll << 20)) B = 1;
        else if (panel >= kSplitBlock0MaxPanel) B = 4;
        else B = (int)std::min<int64_t>(kAutoBlocksMax, std::max<int64_t>(kAutoBlocksMin, (int64_t)std::nearbyint((double)panel / (100 << 20))));
        if (hops < SRG_PLAN_MIN_HOPS_TO_CUT) B = 1;
    }
    if (n == 0 || nnz == 0) B = 1;
    P->B = B;
    P->split0 = B > 1 && ((opts & SRG_PLAN_SPLIT_BLOCK0) ? true : (opts & SRG_PLAN_WHOLE_BLOCK0) ? false : panel < kSplitBlock0MaxPanel);
    bool compact = false;
    if (opts & SRG_PLAN_COMPACT) compact = nnz > 0;
    else if (!(opts & SRG_PLAN_SPANS) && hops >= SRG_PLAN_MIN_HOPS_TO_COMPACT && nnz > 0) {
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) != hipSuccess) { (void)hipGetLastError(); fr = 0; }
        // the copies, and the build's keys / ids / positions (< 24 B per entry)
        compact = (uint64_t)nnz * 8 + (uint64_t)nnz * 24 <= (uint64_t)fr / 4;
    }
    P->compact = compact;
    const bool split0 = P->split0;
    // whole hub rows (column-blocked plans with automatic hub rows): longer than the one-launch hop's hub
    // threshold; counted only when the longest row is (one more host sync)
    int64_t hubw_t = INT64_MAX, n_hubw = 0;
    // (SRG_PLAN_WHOLE_HUBS: longer than an explicit hub threshold -- and than a whole row, which is cut nowhere
    // already)
    const bool whole_hubs = (opts & SRG_PLAN_WHOLE_HUBS) && hub_threshold >= 0;
    const int64_t hubw_rule = hub_threshold == SRG_PLAN_AUTO ? std::max<int64_t>(2048, nnz / 1024)
                              : whole_hubs ? std::max<int64_t>(hub_threshold, whole_max) : INT64_MAX;
    if (B > 1 && hubw_rule != INT64_MAX && max_deg > hubw_rule) {
        hubw_t = hubw_rule;
        DevBuf st;
        st.s = s;
        unsigned long long hc = 0;
        if (hipMalloc(&st.p, sizeof(unsigned long long)) != hipSuccess) { (void)hipGetLastError(); return bail(pfail(SRG_ERR_ALLOC, "plan: statistics")); }
        dstat = (unsigned long long*)st.p;
        if (hipMemsetAsync(dstat, 0, sizeof(unsigned long long), s) != hipSuccess) return bail(pfail(SRG_ERR_HIP, "memset"));
        hipLaunchKernelGGL(k_plan_count_above, dim3(grid_for(n, 256, 512)), dim3(256), 0, s, indptr, n, hubw_t, dstat);
        if (hipMemcpyAsync(&hc, dstat, sizeof(hc), hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
            return bail(pfail(SRG_ERR_HIP, "plan: hub rows: %s", hipGetErrorString(hipGetLastError())));
        n_hubw = (int64_t)hc;
        if (!n_hubw) hubw_t = INT64_MAX;
    }
    const int64_t n_cut = B > 1 ? n - n_whole_rows - n_hubw : 0;
    std::vector<int> sets;     // row set per launch
    std::vector<int> blocks;
    if (B == 1) { sets = {kAll}; blocks = {0}; }
    else {
        if (n_hubw) { sets = {kHubWhole}; blocks = {0}; }
        if (split0) { sets.push_back(kCut); sets.push_back(kWhole); blocks.push_back(0); blocks.push_back(0); }
        else { sets.push_back(kAll); blocks.push_back(0); }
        for (int b = 1; b < B; ++b) { sets.push_back(kCut); blocks.push_back(b); }
    }
    LaunchTable T{};
    T.n_launch = (int)sets.size();
    T.whole_rule = B == 1 ? 1 : 0;
    T.base = n_hubw ? 1 : 0;
    // explicit whole hub rows: no launch over cut rows has hub rows of its own
    T.hub_t = B > 1 && whole_hubs ? SRG_PLAN_NONE : hub_threshold;
    T.heavy_t = heavy_threshold;
    T.hubw_t = hubw_t;
    T.whole_max = whole_max;
    T.lenbits = bits_for((uint64_t)max_deg);
    T.lbits = bits_for((uint64_t)std::max(0, T.n_launch - 1));
    T.off[0] = 0;
    for (int L = 0; L < T.n_launch; ++L) {
        T.blk[L] = blocks[L];
        T.off[L + 1] = T.off[L] + (sets[L] == kAll ? n - n_hubw : sets[L] == kCut ? n_cut
                                   : sets[L] == kWhole ? n_whole_rows : n_hubw);
    }
    const int64_t n_items = T.off[T.n_launch];
    P->n_items = n_items;
    if (T.lenbits + T.lbits > 64) return bail(pfail(SRG_ERR_INVALID, "row lengths too long to plan"));
    if (mem.query()) {
        *mem.q_opts = (compact ? SRG_PLAN_COMPACT : SRG_PLAN_SPANS) | (split0 ? SRG_PLAN_SPLIT_BLOCK0 : SRG_PLAN_WHOLE_BLOCK0) |
                      (opts & (SRG_PLAN_WHOLE_HUBS | (0xffffu << SRG_PLAN_WHOLE_MAX_SHIFT)));
        *mem.q_blocks = B;
        if (n == 0) {
            *mem.q_keep = 0;
            *mem.q_scratch = 0;
            delete P;
            srg_clear_error();
            return SRG_OK;
        }
    }
    if (n == 0) {
        *plan = P;
        srg_clear_error();
        return SRG_OK;
    }
    // the two allocations: what the plan keeps, the build's scratch (sizes first, then carved)
    const bool slots = B > 1 || compact;   // a one-launch CSR hop reads no slot spans
    // the scans' and the sort's temp (int64 elements)
    const int64_t tmp_elems = std::max({B > 1 ? scan_tmp_elems(n) : 1, sort_tmp_elems(n_items), scan_tmp_elems(n_items)});
    int64_t *splits = nullptr, *slot_beg = nullptr, *slot_end = nullptr, *pos = nullptr, *dcounts = nullptr;
    int64_t *cut = nullptr, *cutpos = nullptr;
    int32_t *vals = nullptr, *order = nullptr, *dhubs = nullptr, *oix = nullptr;
    uint64_t *keys = nullptr, *skeys = nullptr;
    float* ov = nullptr;
    int64_t* ptmp = nullptr;
    for (int pass = 0; pass < 2; ++pass) {
        Arena keep, tmp;
        if (pass == 1) {
            keep.base = (char*)P->owned;
            tmp.base = scratch_base;
        }
        order = keep.take<int32_t>((size_t)n_items);
        if (slots) {
            slot_beg = keep.take<int64_t>((size_t)n_items);
            slot_end = keep.take<int64_t>((size_t)n_items);
        }
        if (B > 1) splits = (compact ? tmp : keep).take<int64_t>((size_t)(B - 1) * n);
        if (compact) {
            oix = keep.take<int32_t>((size_t)nnz);
            ov = keep.take<float>((size_t)nnz);
            P->blk_beg = keep.take<int64_t>((size_t)B * n);
            P->blk_end = keep.take<int64_t>((size_t)B * n);
        }
        if (B > 1) {
            cut = tmp.take<int64_t>((size_t)n);
            cutpos = tmp.take<int64_t>((size_t)n);
        }
        keys = tmp.take<uint64_t>((size_t)n_items);
        skeys = tmp.take<uint64_t>((size_t)n_items);
        vals = tmp.take<int32_t>((size_t)n_items);
        pos = tmp.take<int64_t>((size_t)n_items + 1);
        dcounts = tmp.take<int64_t>((size_t)4 * T.n_launch + 1);
        dhubs = tmp.take<int32_t>((size_t)kHubPrefix * T.n_launch);
        ptmp = tmp.take<int64_t>((size_t)tmp_elems);
        if (pass == 0) {
            if (mem.query()) {
                *mem.q_keep = keep.used;
                *mem.q_scratch = tmp.used;
                delete P;
                srg_clear_error();
                return SRG_OK;
            }
            P->bytes = (int64_t)keep.used;
            if (mem.caller()) {
                // the caller's memory: 256-byte aligned (the arena's pieces are), large enough
                if (((uintptr_t)mem.keep & 255) || ((uintptr_t)mem.scratch & 255) || !mem.scratch ||
                    mem.keep_bytes < keep.used || mem.scratch_bytes < tmp.used)
                    return bail(pfail(SRG_ERR_INVALID, "plan: caller memory keep %zu of %zu bytes, scratch %zu of %zu "
                                      "(srg_plan_query's sizes, 256-byte aligned)", mem.keep_bytes, keep.used,
                                      mem.scratch_bytes, tmp.used));
                P->owned = mem.keep;
                P->owns = false;
                scratch_base = (char*)mem.scratch;
                continue;
            }
            if (hipMalloc(&P->owned, keep.used) != hipSuccess) {
                (void)hipGetLastError();
                P->owned = nullptr;
                return bail(pfail(SRG_ERR_ALLOC, "plan: %zu bytes of device memory", keep.used));
            }
            if (hipMalloc(&scratch.p, tmp.used) != hipSuccess) {
                (void)hipGetLastError();
                scratch.p = nullptr;
                return bail(pfail(SRG_ERR_ALLOC, "plan: %zu bytes of build scratch", tmp.used));
            }
            scratch_base = (char*)scratch.p;
        }
    }
    // split points and the cut rows' positions
    if (B > 1) {
        hipLaunchKernelGGL(k_plan_splits, dim3(grid_for(n * (B - 1), 256, 1u << 20)), dim3(256), 0, s, indptr, indices,
                           n, B, T.hubw_t, T.whole_max, splits, cut);
        const int rc = scan_i64(LoadI64{cut}, n, cutpos, false, ptmp, s);
        if (rc) return bail(rc);
    }
    // the sort items, sorted by (launch, decreasing span length)
    SRG_PLAN_HIP(hipMemsetAsync(keys, 0xff, (size_t)n_items * sizeof(uint64_t), s));
    hipLaunchKernelGGL(k_plan_items, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, indptr, splits, cutpos, n, B,
                       split0 ? 1 : 0, T, keys, vals);
    {
        const int rc = radix_sort_pairs(keys, vals, skeys, order, n_items, T.lenbits + T.lbits, ptmp, s);
        if (rc) return bail(rc);
    }
    {
        // pos[i] = the entries of the items before i (launch-major): copy positions and launch nnz
        SRG_PLAN_HIP(hipMemsetAsync(pos, 0, sizeof(int64_t), s));
        const int rc = scan_i64(KeyLen{skeys, (1ull << T.lenbits) - 1}, n_items, pos + 1, true, ptmp, s);
        if (rc) return bail(rc);
    }
    // ---- 3: per-launch counts and the guard (host sync 2) ----
    SRG_PLAN_HIP(hipMemsetAsync(dcounts + 4 * T.n_launch, 0, sizeof(int64_t), s));
    hipLaunchKernelGGL(k_plan_check, dim3(grid_for(n_items, 256, 4096)), dim3(256), 0, s, skeys, n_items, T,
                       (int32_t*)(dcounts + 4 * T.n_launch));
    hipLaunchKernelGGL(k_plan_counts, dim3(1), dim3(128), 0, s, skeys, order, pos, T, dcounts, dhubs);
    std::vector<int64_t> counts((size_t)4 * T.n_launch + 1);
    std::vector<int32_t> hubs((size_t)kHubPrefix * T.n_launch);
    SRG_PLAN_HIP(hipMemcpyAsync(counts.data(), dcounts, counts.size() * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    SRG_PLAN_HIP(hipMemcpyAsync(hubs.data(), dhubs, hubs.size() * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    {
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return bail(pfail(SRG_ERR_HIP, "plan build: %s", hipGetErrorString(e)));
        int64_t total = 0;
        for (int L = 0; L < T.n_launch; ++L) total += counts[4 * L];
        if (counts[4 * T.n_launch] != 0 || total != nnz)
            return bail(pfail(SRG_ERR_INVALID, "plan build: inconsistent layout (%lld of %lld entries placed%s)",
                              (long long)total, (long long)nnz, counts[4 * T.n_launch] ? ", items outside their launch" : ""));
    }
    // ---- 4: the spans the launches read ----
    // compact: row-indexed spans for the rows the packed-row width reads them for (hub and slice-wave
    // rows), or every row for the other widths
    P->rows_full = !compact || !packed_width(d);
    for (int L = 0; L < T.n_launch; ++L)
        T.rows_lim[L] = P->rows_full ? T.off[L + 1] - T.off[L] : counts[4 * L + 1] + counts[4 * L + 2];
    if (slots)
        hipLaunchKernelGGL(k_plan_spans, dim3(grid_for(n_items, 256, 1u << 20)), dim3(256), 0, s, indptr, splits, n, B,
                           split0 ? 1 : 0, T, compact ? 1 : 0, skeys, order, pos, n_items, slot_beg, slot_end,
                           P->blk_beg, P->blk_end);
    if (compact)
        hipLaunchKernelGGL(k_plan_copy, dim3(grid_for((nnz + kCopyChunk - 1) / kCopyChunk, 4, 1u << 16)), dim3(256), 0, s,
                           indptr, splits, indices, values, n, B, T, T.lenbits, skeys, order, pos, n_items,
                           nnz, oix, ov);
    {
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return bail(pfail(SRG_ERR_HIP, "plan build: %s", hipGetErrorString(e)));
    }
    // ---- 5: the launch descriptors ----
    for (int L = 0; L < T.n_launch; ++L) {
        srg_plan::Launch D;
        const int b = blocks[L];
        D.block = b;
        D.item0 = T.off[L];
        D.order = order + T.off[L];
        D.n_rows = T.off[L + 1] - T.off[L];
        D.nnz = counts[4 * L + 0];
        D.n_hub = counts[4 * L + 1];
        D.n_heavy = counts[4 * L + 2];
        D.n_narrow = counts[4 * L + 3];
        D.whole_rows = sets[L] == kWhole;
        D.hub_whole = sets[L] == kHubWhole;
        if (compact) {
            D.row_beg = P->blk_beg + (int64_t)b * n;
            D.row_end = P->blk_end + (int64_t)b * n;
            D.indices = oix;
            D.values = ov;
        } else {
            D.row_beg = b == 0 ? indptr : splits + (int64_t)(b - 1) * n;
            D.row_end = B == 1 ? nullptr : (b == B - 1 ? indptr + 1 : splits + (int64_t)b * n);
            D.indices = indices;
            D.values = values;
        }
        if (slots) {
            D.slot_beg = slot_beg + T.off[L];
            D.slot_end = slot_end + T.off[L];
        }
        P->launches.push_back(D);
    }
    // hub spans chain on the side stream when every launch over cut rows has the same hub rows
    if (B > 1) {
        bool same = true;
        std::vector<int32_t> ref;
        bool first = true;
        for (int L = 0; L < T.n_launch && same; ++L) {
            if (sets[L] == kWhole || sets[L] == kHubWhole) continue;
            const int64_t h = counts[4 * L + 1];
            if (h > kHubPrefix) { same = false; break; }
            std::vector<int32_t> set(hubs.begin() + (size_t)L * kHubPrefix, hubs.begin() + (size_t)L * kHubPrefix + h);
            std::sort(set.begin(), set.end());
            if (first) { ref = set; first = false; }
            else same = set == ref;
        }
        P->same_hubs = same;
        for (int L = 0; L < T.n_launch; ++L)
            if (sets[L] == kCut || sets[L] == kAll) P->block_hubs |= counts[4 * L + 1] > 0;
        P->n_hub_whole = n_hubw;
    }
    // after the build's kernels (one more wait on the stream: the copy); the caller's scratch may go
    // once the call returns
    scratch.reset();
    if (mem.caller()) {
        const hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) return bail(pfail(SRG_ERR_HIP, "plan build: %s", hipGetErrorString(e)));
    }
    note_use(P, s);
    *plan = P;
    srg_clear_error();
    return SRG_OK;
}

extern "C" {

int srg_plan_build(const int64_t* indptr, const int32_t* indices, const float* values, int64_t n_rows, int32_t d,
                   int32_t hops, int32_t col_blocks, int64_t hub_threshold, int64_t heavy_threshold, uint32_t opts,
                   void* stream, srg_plan** plan)
{
    return build_impl(indptr, indices, values, n_rows, d, hops, col_blocks, hub_threshold, heavy_threshold, opts,
                      stream, plan, BuildMem{});
}

int srg_plan_query(const int64_t* indptr, int64_t n_rows, int32_t d, int32_t hops, int32_t col_blocks,
                   int64_t hub_threshold, int64_t heavy_threshold, uint32_t opts, void* stream, size_t* keep_bytes,
                   size_t* scratch_bytes, uint32_t* resolved_opts, int32_t* resolved_col_blocks)
{
    if (!keep_bytes || !scratch_bytes || !resolved_opts || !resolved_col_blocks)
        return pfail(SRG_ERR_INVALID, "null output");
    BuildMem m;
    m.q_keep = keep_bytes;
    m.q_scratch = scratch_bytes;
    m.q_opts = resolved_opts;
    m.q_blocks = resolved_col_blocks;
    // the sizes do not depend on the ids / values, only on indptr (lengths and split counts) and the hub
    // threshold (automatic hub rows may be whole hub rows: one item each instead of one per block)
    return build_impl(indptr, nullptr, nullptr, n_rows, d, hops, col_blocks, hub_threshold, heavy_threshold, opts,
                      stream, nullptr, m);
}

int srg_plan_build_in(const int64_t* indptr, const int32_t* indices, const float* values, int64_t n_rows, int32_t d,
                      int32_t hops, int32_t col_blocks, int64_t hub_threshold, int64_t heavy_threshold, uint32_t opts,
                      void* keep, size_t keep_bytes, void* scratch, size_t scratch_bytes, void* stream,
                      srg_plan** plan)
{
    if (!keep) return pfail(SRG_ERR_INVALID, "null keep memory (srg_plan_build allocates its own)");
    BuildMem m;
    m.keep = keep;
    m.keep_bytes = keep_bytes;
    m.scratch = scratch;
    m.scratch_bytes = scratch_bytes;
    return build_impl(indptr, indices, values, n_rows, d, hops, col_blocks, hub_threshold, heavy_threshold, opts,
                      stream, plan, m);
}

int srg_plan_destroy(srg_plan* plan, void* stream)
{
    if (!plan) return SRG_OK;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    DevGuard g(s);
    if (!s) (void)hipSetDevice(plan->device);
    // hub rows a caller driving the launches itself (srg_plan_launch) left on the side stream of `s`
    (void)srg_hub_join(stream);
    release(plan, s);
    delete plan;
    return SRG_OK;
}

int srg_plan_describe(const srg_plan* plan, srg_plan_desc* desc)
{
    if (!plan || !desc) return pfail(SRG_ERR_INVALID, "null plan / desc");
    desc->n_rows = plan->n;
    desc->nnz = plan->nnz;
    desc->device_bytes = plan->bytes;
    desc->d = plan->d;
    desc->col_blocks = plan->B;
    desc->n_launch = (int32_t)plan->launches.size();
    desc->compact = plan->compact ? 1 : 0;
    desc->split_block0 = plan->split0 ? 1 : 0;
    desc->hub_chain = (plan->B > 1 && plan->same_hubs && plan->block_hubs) ? 1 : 0;
    desc->hub_rows_whole = (int32_t)plan->n_hub_whole;
    desc->device = plan->device;
    srg_clear_error();
    return SRG_OK;
}

// A caller that repeats a propagate (the same panels, widths, hops, flags and stream) gets the K hops as
// one HIP graph from the second call on: hipGraphLaunch instead of ~5 API calls per launch.  Products
// and arxiv hops measure the same either way (GPU-bound, profiles/r05n_*); a 4,000-row operator's 10-hop
// call costs the host 0.12 instead of 0.21 ms to enqueue.  -DSRG_PLAN_GRAPHS=0 builds without it.
#ifndef SRG_PLAN_GRAPHS
#define SRG_PLAN_GRAPHS 1
#endif

// the launches of one hop over a d-column panel with their flags; returns whether the hub side
// stream must be joined at the end of each hop
static int plan_launches(const srg_plan* P, int32_t d, uint32_t flags, std::vector<srg_hop_launch>& out)
{
    const bool fast = (flags & SRG_SPMM_FAST) != 0;
    const bool blocked = P->B > 1;
    uint32_t base = flags & SRG_SPMM_NT_STORE;
    if (blocked) {
        base |= (d >= 128 ? SRG_SPMM_PACKED_U2 : 0u) |
                (P->n * (int64_t)d * 4 >= kCapWavesMinPanel ? SRG_SPMM_CAP_WAVES : 0u);
    }
    const bool chain = blocked && !fast && P->same_hubs;
    bool forked = false;
    out.clear();
    for (const srg_plan::Launch& D : P->launches) {
        srg_hop_launch L{};
        L.row_beg = D.row_beg;
        L.row_end = D.row_end;
        L.indices = D.indices;
        L.values = D.values;
        L.row_order = D.n_rows ? D.order : nullptr;
        L.n_rows = D.n_rows;
        L.n_hub = D.n_hub;
        L.n_heavy = d <= 32 ? D.n_narrow : D.n_heavy;
        L.slot_beg = D.slot_beg;
        L.slot_end = D.slot_end;
        uint32_t f = base | (D.block > 0 ? SRG_SPMM_ACCUMULATE : 0u);
        if (D.hub_whole) {
            // the whole hub rows: forked first, joined at the end of the hop (FAST: their segments)
            f |= SRG_SPMM_HUB_NOJOIN | (fast ? SRG_SPMM_FAST : 0u);
            forked = true;
        } else if (chain && D.n_hub > 0) {
            f |= SRG_SPMM_HUB_NOJOIN | (forked ? SRG_SPMM_HUB_CONTINUE : 0u);
            forked = true;
        } else if (fast) {
            f |= SRG_SPMM_FAST;
        }
        L.flags = f;
        out.push_back(L);
    }
    return forked ? 1 : 0;
}

int srg_plan_launch(const srg_plan* plan, int32_t i, int32_t d, srg_hop_launch* launch, int32_t* join_hub, void* stream)
{
    if (!plan || !launch) return pfail(SRG_ERR_INVALID, "null plan / launch");
    if (i < 0 || i >= (int32_t)plan->launches.size() || d <= 0)
        return pfail(SRG_ERR_INVALID, "launch %d of %zu, d=%d", i, plan->launches.size(), d);
    if (!plan->rows_full) {
        // a caller driving the launches may run any width: every row-indexed span, on `stream`
        DevGuard g(static_cast<hipStream_t>(stream));
        if (g.rc) return g.rc;
        const int rc = complete_rows(const_cast<srg_plan*>(plan), static_cast<hipStream_t>(stream));
        if (rc) return rc;
    }
    std::vector<srg_hop_launch> L;
    const int join = plan_launches(plan, d, 0, L);
    *launch = L[(size_t)i];
    if (join_hub) *join_hub = join;
    srg_clear_error();
    return SRG_OK;
}

int srg_plan_propagate_f32(const srg_plan* plan, float* const* panels, int64_t ld, int32_t d, int32_t K, uint32_t flags,
                           void* stream)
{
    if (!plan) return pfail(SRG_ERR_INVALID, "null plan");
    if (flags & ~(SRG_SPMM_NT_STORE | SRG_SPMM_FAST))
        return pfail(SRG_ERR_INVALID, "flags=0x%x: a plan's hops take NT_STORE and FAST only", flags);
    if (plan->no_values)
        return pfail(SRG_ERR_INVALID, "the plan was built without fp32 values (SRG_PLAN_SPANS, values NULL): it serves "
                     "srg_plan_cheby_step_f64 only");
    if (d <= 0 || K < 0) return pfail(SRG_ERR_INVALID, "d=%d, K=%d", d, K);
    if (K == 0 || plan->launches.empty()) { srg_clear_error(); return SRG_OK; }
    DevGuard g(static_cast<hipStream_t>(stream));
    if (g.rc) return g.rc;
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev != plan->device)
        return pfail(SRG_ERR_INVALID, "the plan lives on device %d, the stream on %d", plan->device, dev);
    if (!plan->rows_full) {
        // the packed light rows (spans by slot) run only at 64 / 128 / 256 columns on 16-byte rows
        bool packed = packed_width(d) && ld % 4 == 0;
        for (int k = 0; packed && panels && k <= K; ++k) packed = panels[k] && ((uintptr_t)panels[k] % 16) == 0;
        if (!packed) {
            const int rc = complete_rows(const_cast<srg_plan*>(plan), static_cast<hipStream_t>(stream));
            if (rc) return rc;
        }
    }
    std::vector<srg_hop_launch> L;
    const int join = plan_launches(plan, d, flags, L);
    srg_plan* P = const_cast<srg_plan*>(plan);
    const hipStream_t s = static_cast<hipStream_t>(stream);
    reap_retired(P, false);
#if SRG_PLAN_GRAPHS
    // A repeated call (same panels, widths, hops, flags and stream) replays the K hops as one HIP graph,
    // captured from the second call on: the same launches with the same arguments, so the same bits.
    // Not for FAST (its scratch is stream-ordered allocation) nor the null stream (not capturable).
    // A graph of an earlier key is retired, not destroyed: its last launch may still be running.
    srg_plan::Graph& G = P->graph;
    if (stream && !(flags & SRG_SPMM_FAST) && panels && !capturing(s)) {
        const std::vector<float*> key(panels, panels + K + 1);
        if (G.panels != key || G.ld != ld || G.d != d || G.K != K || G.flags != flags || G.stream != stream) {
            drop_graph(P);
            G.panels = key;
            G.ld = ld; G.d = d; G.K = K; G.flags = flags; G.stream = stream;
            G.calls = 0;
            G.off = false;
        }
        auto replay = [&]() {
            SRG_PLAN_HIP(hipGraphLaunch(G.exec, s));
            SRG_PLAN_HIP(hipEventRecord(G.done, s));
            note_use(P, s);
            srg_clear_error();
            return SRG_OK;
        };
        if (G.exec) return replay();
        if (G.calls >= 1 && !G.off) {
            if (hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed) == hipSuccess) {
                const int rc = srg_propagate_plan_f32(L.data(), (int32_t)L.size(), join, panels, ld, d, K, stream);
                hipGraph_t gr = nullptr;
                const hipError_t e = hipStreamEndCapture(s, &gr);
                hipGraphExec_t x = nullptr;
                hipEvent_t done = nullptr;
                if (!rc && e == hipSuccess && gr && hipGraphInstantiate(&x, gr, nullptr, nullptr, 0) == hipSuccess &&
                    hipEventCreateWithFlags(&done, hipEventDisableTiming) == hipSuccess) {
                    (void)hipGraphDestroy(gr);
                    G.exec = x;
                    G.done = done;
                    return replay();
                }
                if (x) (void)hipGraphExecDestroy(x);
                if (gr) (void)hipGraphDestroy(gr);
            }
            (void)hipGetLastError();
            G.off = true;                    // nothing ran: the eager loop below does the hops
        }
        ++G.calls;
    }
#endif
    const int rc = srg_propagate_plan_f32(L.data(), (int32_t)L.size(), join, panels, ld, d, K, stream);
    if (!rc) note_use(P, s);
    return rc;
}

int srg_plan_hop_f32(const srg_plan* plan, const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t d,
                     uint32_t flags, float* agg, int64_t lda, float w, int32_t agg_init, void* stream)
{
    if (!plan) return pfail(SRG_ERR_INVALID, "null plan");
    if (flags & ~(SRG_SPMM_NT_STORE | SRG_SPMM_FAST))
        return pfail(SRG_ERR_INVALID, "flags=0x%x: a plan's hops take NT_STORE and FAST only", flags);
    if (plan->no_values)
        return pfail(SRG_ERR_INVALID, "the plan was built without fp32 values (SRG_PLAN_SPANS, values NULL): it serves "
                     "srg_plan_cheby_step_f64 only");
    if ((flags & SRG_SPMM_FAST) && agg)
        return pfail(SRG_ERR_INVALID, "FAST takes no aggregation epilogue");
    if (d <= 0 || ldx < d || ldy < d) return pfail(SRG_ERR_INVALID, "d=%d, ldx=%lld, ldy=%lld", d, (long long)ldx, (long long)ldy);
    if (plan->launches.empty()) {
        // no rows: nothing to write
        srg_clear_error();
        return SRG_OK;
    }
    if (!X || !Y) return pfail(SRG_ERR_INVALID, "null X / Y");
    if (agg && lda < d) return pfail(SRG_ERR_INVALID, "lda=%lld < d=%d", (long long)lda, d);
    DevGuard g(static_cast<hipStream_t>(stream));
    if (g.rc) return g.rc;
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev != plan->device)
        return pfail(SRG_ERR_INVALID, "the plan lives on device %d, the stream on %d", plan->device, dev);
    if (!plan->rows_full) {
        // the packed light rows run only at 64 / 128 / 256 columns on 16-byte rows (agg's too)
        const bool packed = packed_width(d) && ldx % 4 == 0 && ldy % 4 == 0 && (uintptr_t)X % 16 == 0 &&
                            (uintptr_t)Y % 16 == 0 && (!agg || (lda % 4 == 0 && (uintptr_t)agg % 16 == 0));
        if (!packed) {
            const int rc = complete_rows(const_cast<srg_plan*>(plan), static_cast<hipStream_t>(stream));
            if (rc) return rc;
        }
    }
    std::vector<srg_hop_launch> L;
    const int join = plan_launches(plan, d, flags, L);
    // the epilogue runs where the rows' chains end: the one launch; with block 0 split, its whole rows'
    // launch and the last block's (every cut row is in it).  Block 0 as one launch ends some chains
    // (its whole rows) and continues others: the hop runs plain, then one accumulation pass over Y
    // (the same two roundings, srg_hop_accumulate_f32)
    std::vector<uint8_t> on(L.size(), 0);
    bool fused = agg != nullptr;
    if (agg) {
        if (plan->B == 1) on[0] = 1;
        else if (plan->split0) {
            for (size_t i = 0; i < L.size(); ++i) on[i] = (plan->launches[i].whole_rows || plan->launches[i].hub_whole) ? 1 : 0;
            on.back() = 1;
        } else fused = false;
    }
    int rc = srg_run_plan_hop(L.data(), (int32_t)L.size(), join, X, ldx, Y, ldy, d, fused ? on.data() : nullptr,
                              fused ? agg : nullptr, lda, w, agg_init, stream);
    if (rc) return rc;
    note_use(const_cast<srg_plan*>(plan), static_cast<hipStream_t>(stream));
    if (agg && !fused) {
        rc = srg_hop_accumulate_f32(agg, lda, Y, ldy, plan->n, d, w, agg_init ? SRG_ACC_INIT : SRG_ACC_ADD, stream);
        if (rc) return rc;
    }
    srg_clear_error();
    return SRG_OK;
}

int srg_plan_cheby_step_f64(const srg_plan* plan, const double* values, const double* Tc, const double* To, double* Tn,
                            int64_t ld, int32_t d, int mode, double a1, double a2, const double* coef_prev,
                            const double* coef, int32_t n_scales, double* R, int64_t r_stride, void* stream)
{
    if (!plan) return pfail(SRG_ERR_INVALID, "null plan");
    if (plan->compact)
        return pfail(SRG_ERR_INVALID, "an fp64 step reads spans of the caller's arrays: build the plan with SRG_PLAN_SPANS");
    if (plan->B > 1 && !plan->split0)
        return pfail(SRG_ERR_INVALID, "an fp64 step needs block 0 as two launches: build the plan with SRG_PLAN_SPLIT_BLOCK0");
    if (plan->launches.empty()) { srg_clear_error(); return SRG_OK; }
    if (!values && plan->nnz > 0) return pfail(SRG_ERR_INVALID, "null values");
    DevGuard g(static_cast<hipStream_t>(stream));
    if (g.rc) return g.rc;
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev != plan->device)
        return pfail(SRG_ERR_INVALID, "the plan lives on device %d, the stream on %d", plan->device, dev);
    std::vector<srg_hop_launch> L;
    (void)plan_launches(plan, d, 0, L);
    std::vector<uint8_t> roles(L.size(), 0);
    for (size_t i = 0; i < L.size(); ++i) {
        const srg_plan::Launch& D = plan->launches[i];
        if (D.hub_whole) roles[i] = SRG_CHEBY64_HUBS;
        else roles[i] = (D.block == 0 ? SRG_CHEBY64_FIRST : 0) |
                        (D.whole_rows || plan->B == 1 || D.block == plan->B - 1 ? SRG_CHEBY64_LAST : 0);
    }
    const int64_t* indptr = plan->launches[0].row_beg;   // block 0 of a spans plan: the caller's indptr
    const int32_t* indices = plan->launches[0].indices;
    const int rc = srg_run_plan_cheby_f64(L.data(), roles.data(), (int32_t)L.size(), indptr, indices, values, Tc, To, Tn,
                                          ld, d, mode, a1, a2, coef_prev, coef, n_scales, R, r_stride, stream);
    if (rc) return rc;
    note_use(const_cast<srg_plan*>(plan), static_cast<hipStream_t>(stream));
    srg_clear_error();
    return SRG_OK;
}

}  // extern "C"
